"""Layer-sharded SERVING on the device transport (``cake-cli --transport rccl``, PP2):
the master's REST API answers two sequential chat requests through a rank pipeline
whose decode hops are device-side IPC stores captured in every rank's graph, with
every request announced to the worker on the host control channel.  The completions
must equal the all-local (single-rank) server's, token for token (f32 hops).

Both ranks share cuda:0 on the 1-GPU pool (CAKE_DIST_BACKEND=gloo: RCCL refuses two
ranks on one device; the decode hops do not use the process group)."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _post(port: int, body: dict, timeout: float = 60.0) -> dict:
    req = urllib.request.Request(f"http://127.0.0.1:{port}/api/v1/chat/completions",
                                 data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read())


REQS = [{"messages": [{"role": "system", "content": "be brief"},
                      {"role": "user", "content": "hello there"}], "max_tokens": 24},
        {"messages": [{"role": "user", "content": "why is the sky blue?"}], "max_tokens": 40}]


def test_rccl_pp2_api_serving_matches_local(cuda, tmp_path):
    from fastapi.testclient import TestClient
    from cake_amd.api.server import create_app
    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import Master
    from cake_amd.utils.synth import tiny_config, write_checkpoint

    d = tmp_path / "m"
    write_checkpoint(d, tiny_config(num_hidden_layers=4), torch.bfloat16)
    (tmp_path / "empty.yml").write_text("{}\n")
    topo = tmp_path / "t.yml"
    topo.write_text("w1:\n  host: 'rank1'\n  layers: ['model.layers.2-3']\n")
    common = ["--model", str(d), "--dtype", "bf16", "--temperature", "0", "--max-seq-len", "512"]

    # all-local reference server (in this process)
    args = build_parser().parse_args(common + ["--topology", str(tmp_path / "empty.yml")])
    local = TestClient(create_app(Master(Context.from_args(args))))
    want = [local.post("/api/v1/chat/completions", json=r).json() for r in REQS]
    assert all(w["choices"][0]["message"]["content"] for w in want)

    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0",
               CAKE_DIST_BACKEND="gloo", CAKE_HOP_TIMEOUT="30")
    env.pop("WORLD_SIZE", None)
    log = open(tmp_path / "serve.log", "w")
    p = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node=2", "--master-addr=127.0.0.1",
                          f"--master-port={_free_port()}", "-m", "cake_amd.cli",
                          "--transport", "rccl", "--hop", "ipc", "--hop-dtype", "f32",
                          "--topology", str(topo), "--api", f"127.0.0.1:{port}", *common],
                         cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT,
                         start_new_session=True)
    try:
        deadline = time.time() + 150
        while True:
            assert p.poll() is None, (tmp_path / "serve.log").read_text()[-3000:]
            try:
                with socket.create_connection(("127.0.0.1", port), timeout=1):
                    break
            except OSError:
                assert time.time() < deadline, (tmp_path / "serve.log").read_text()[-3000:]
                time.sleep(1.0)
        try:
            got = [_post(port, r) for r in REQS]
            # a third request equal to the first: per-request state is reset
            again = _post(port, REQS[0])
        except Exception as e:  # noqa: BLE001  (show what the server said)
            time.sleep(2)
            raise AssertionError(f"{e!r}\n" + (tmp_path / "serve.log").read_text()[-4000:])
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(timeout=30)
        log.close()
    text = (tmp_path / "serve.log").read_text()
    assert "hops: ipc" in text, text[-3000:]
    for w, g in zip(want, got):
        assert g["choices"][0]["message"]["content"] == w["choices"][0]["message"]["content"]
        assert g["usage"]["completion_tokens"] == w["usage"]["completion_tokens"]
    assert again["choices"][0]["message"]["content"] == want[0]["choices"][0]["message"]["content"]
