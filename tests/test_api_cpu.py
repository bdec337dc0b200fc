"""REST API shape (cake-core/src/cake/api) against a tiny CPU model."""
import json

import pytest
import torch

from cake_amd.cli import build_parser
from cake_amd.context import Context
from cake_amd.master import Master
from cake_amd.utils.synth import tiny_config, write_checkpoint


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    from fastapi.testclient import TestClient
    from cake_amd.api.server import create_app
    d = tmp_path_factory.mktemp("tinyapi")
    write_checkpoint(d, tiny_config(), torch.float32)
    (d / "topo.yml").write_text("{}\n")
    args = build_parser().parse_args(["--model", str(d), "--topology", str(d / "topo.yml"),
                                      "--cpu", "--temperature", "0", "-n", "8"])
    return TestClient(create_app(Master(Context.from_args(args))))


def test_chat_completion_shape_and_determinism(client):
    req = {"messages": [{"role": "system", "content": "be brief"},
                        {"role": "user", "content": "hello"}]}
    r = client.post("/api/v1/chat/completions", json=req)
    assert r.status_code == 200
    j = r.json()
    assert j["object"] == "chat.completion" and j["model"] == "llama3"
    assert len(j["id"]) == 36 and isinstance(j["created"], int)
    assert j["choices"][0]["index"] == 0 and j["choices"][0]["message"]["role"] == "assistant"
    # second identical request gives the same text (state reset between requests)
    r2 = client.post("/api/v1/chat/completions", json=req)
    assert r2.json()["choices"][0]["message"]["content"] == j["choices"][0]["message"]["content"]
    # capitalised roles accepted on input (chat.rs aliases)
    r3 = client.post("/api/v1/chat/completions",
                     json={"messages": [{"role": "User", "content": "hello"}], "max_tokens": 3})
    assert r3.status_code == 200 and r3.json()["usage"]["completion_tokens"] <= 3


def test_streaming_and_404(client):
    r = client.post("/api/v1/chat/completions",
                    json={"messages": [{"role": "user", "content": "x"}], "stream": True,
                          "max_tokens": 4})
    lines = [l for l in r.text.splitlines() if l.startswith("data: ")]
    assert lines[-1] == "data: [DONE]"
    assert all(json.loads(l[6:])["object"] == "chat.completion.chunk" for l in lines[:-1])
    r = client.get("/anything")
    assert r.status_code == 404 and r.text == "nope"
    r = client.post("/api/v1/image", json={"image_args": {}})
    assert r.status_code == 400
