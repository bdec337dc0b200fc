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


def test_per_request_sampling(client):
    """temperature / top_p / top_k / seed per request (SURVEY Appendix E Q5 superset):
    a seeded sampled request is reproducible, invalid values are rejected, and a
    request without them returns to the server's (greedy) configuration."""
    msgs = [{"role": "user", "content": "hello"}]
    greedy = client.post("/api/v1/chat/completions", json={"messages": msgs}).json()
    req = {"messages": msgs, "temperature": 1.5, "top_k": 50, "top_p": 0.95, "seed": 7}
    a = client.post("/api/v1/chat/completions", json=req)
    b = client.post("/api/v1/chat/completions", json=req)
    assert a.status_code == 200
    assert a.json()["choices"][0]["message"]["content"] == b.json()["choices"][0]["message"]["content"]
    outs = {client.post("/api/v1/chat/completions", json=dict(req, seed=s)).json()
            ["choices"][0]["message"]["content"] for s in range(6)}
    assert len(outs) > 1  # the draw depends on the seed
    back = client.post("/api/v1/chat/completions", json={"messages": msgs}).json()
    assert back["choices"][0]["message"]["content"] == greedy["choices"][0]["message"]["content"]
    for bad in ({"temperature": -1}, {"top_p": 0}, {"top_p": 1.5}, {"top_k": -3}, {"top_k": 1.5},
                {"seed": "x"}):
        r = client.post("/api/v1/chat/completions", json=dict(messages=msgs, **bad))
        assert r.status_code == 400, bad


def test_request_sampling_merge():
    from cake_amd.api.server import request_sampling
    from cake_amd.models.sampling import SamplingConfig
    d = SamplingConfig(temperature=0.0, top_k=None, top_p=None, seed=1)
    s = request_sampling({"temperature": 0.7, "top_p": 1.0, "top_k": 0}, d)
    assert s.temperature == 0.7 and s.top_p is None and s.top_k is None and s.seed == 1
    assert request_sampling({}, d) == d


def test_max_tokens_beyond_max_seq_is_clamped(tmp_path):
    """A request for more tokens than the KV cache holds stops at the cache end instead
    of writing past it (all-local generator; the TP and pipeline engines clamp the same
    way: tests/test_tp_cpu.py, tests/test_pipeline_cpu.py)."""
    from fastapi.testclient import TestClient
    from cake_amd.api.server import create_app
    write_checkpoint(tmp_path, tiny_config(), torch.float32)
    (tmp_path / "topo.yml").write_text("{}\n")
    args = build_parser().parse_args(["--model", str(tmp_path), "--topology",
                                      str(tmp_path / "topo.yml"), "--cpu", "--temperature", "0",
                                      "--max-seq-len", "48"])
    master = Master(Context.from_args(args))
    c = TestClient(create_app(master))
    r = c.post("/api/v1/chat/completions",
               json={"messages": [{"role": "user", "content": "hello"}], "max_tokens": 500})
    assert r.status_code == 200
    n_prompt = len(master.llm.tokens) - r.json()["usage"]["completion_tokens"]
    assert 0 < r.json()["usage"]["completion_tokens"] <= 48 - n_prompt
    assert len(master.llm.tokens) == 48   # generated up to the last cache row, no further
