"""Native entry points on CPU: the cake-cli executable (native flag parsing + topology,
compute runtime embedded in-process) and the C ABI cake_start_worker (worker hosted in the
calling process), checked against the Python entry on a tiny synthetic checkpoint."""
import ctypes  # noqa: F401  (used in the worker host snippet)
import os
import socket
import subprocess
import sys
import time

import pytest
import torch

from cake_amd.utils.synth import tiny_config, write_checkpoint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "cake_amd", "lib", "cake-cli")
RTLIB = os.path.join(ROOT, "cake_amd", "lib", "libcake_runtime.so")
pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="cake-cli not built")


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = tmp_path_factory.mktemp("tiny3")
    write_checkpoint(d, tiny_config(num_hidden_layers=3), torch.float32)
    return d


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


GEN = ["--cpu", "--temperature", "0", "-n", "6", "--prompt", "hello there"]


def _run(cmd, timeout=180):
    env = dict(os.environ, CAKE_LOG="warning")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def test_cli_flag_validation():
    for bad in (["--bogus"], ["--temperature", "x"], ["--mode", "boss"], ["--cpu=1"],
                ["--mode", "worker", "--topology", "/nonexistent.yml"]):
        r = _run([CLI, *bad])
        assert r.returncode == 2, (bad, r.stderr)
    r = _run([CLI, "--help"])
    assert r.returncode == 0 and "--sd-img2img-strength" in r.stdout


def test_native_cli_matches_python_entry(ckpt, tmp_path):
    args = ["--model", str(ckpt), "--topology", str(tmp_path / "none.yml"), *GEN]
    nat = _run([CLI, *args])
    py = _run([sys.executable, "-m", "cake_amd.cli", *args])
    assert nat.returncode == 0, nat.stderr[-2000:]
    assert py.returncode == 0, py.stderr[-2000:]
    assert nat.stdout.strip() and nat.stdout == py.stdout


def _wait_port(port, proc, timeout=120):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise AssertionError(f"worker exited: {proc.stderr.read()[-2000:]}")
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return
        except OSError:
            time.sleep(0.2)
    raise AssertionError("worker did not listen")


@pytest.mark.parametrize("host", ["cli", "capi"])
def test_native_worker_serves_master(ckpt, tmp_path, host):
    """A worker hosted natively (cake-cli --mode worker, or cake_start_worker from a host
    process) serves layers 1-2 to a cake-cli master: same tokens as all-local."""
    port = _port()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{port}'\n  layers:\n    - 'model.layers.1-2'\n")
    local = _run([CLI, "--model", str(ckpt), "--topology", str(tmp_path / "none.yml"), *GEN])
    assert local.returncode == 0, local.stderr[-2000:]
    env = dict(os.environ, CAKE_LOG="warning")
    if host == "cli":
        cmd = [CLI, "--mode", "worker", "--name", "w1", "--model", str(ckpt), "--topology",
               str(topo), "--address", f"127.0.0.1:{port}", "--cpu"]
    else:  # C ABI from a host process (here: a Python host; the worker runs inside it)
        snippet = (f"import ctypes,sys; lib=ctypes.CDLL({RTLIB!r}); "
                   f"sys.exit(lib.cake_start_worker(b'w1', {str(ckpt).encode()!r}, "
                   f"{str(topo).encode()!r}, b'text', b'127.0.0.1:{port}'))")
        cmd = [sys.executable, "-c", snippet]
    w = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.PIPE, text=True)
    try:
        _wait_port(port, w)
        dist = _run([CLI, "--model", str(ckpt), "--topology", str(topo), *GEN])
        assert dist.returncode == 0, dist.stderr[-2000:]
        assert dist.stdout == local.stdout
    finally:
        w.kill()
        w.wait()


def test_native_bridge_tokenizer_matches_generator(ckpt):
    """The tokenizer half of the native text path (cake_amd/native_bridge.py, called by
    cake-cli through the embedded interpreter): the prompt ids and per-token text equal
    what the Python generator uses."""
    import json
    from cake_amd import native_bridge as B
    from cake_amd.models.chat import Message
    from cake_amd.models.llama3.config import LlamaConfig
    from cake_amd.models.llama3.generator import LLamaGenerator, load_tokenizer
    r = json.loads(B.encode_chat(json.dumps({"model": str(ckpt), "system": "sys",
                                             "prompt": "hello there"})))
    cfg = LlamaConfig.from_path(ckpt)
    tok, eos = load_tokenizer(ckpt, cfg.eos_token_id)
    gen = LLamaGenerator.__new__(LLamaGenerator)
    gen.tokenizer, gen.eos_ids = tok, eos
    from cake_amd.models.chat import History
    gen.history = History()
    gen.add_message(Message.system("sys"))
    gen.add_message(Message.user("hello there"))
    ids = tok.encode(gen.history.encode_dialog_to_prompt(), add_special_tokens=False).ids
    assert r["ids"] == list(ids) and r["eos"] == sorted(eos)
    for t in (5, 72, 300, 259):
        assert B.decode_token(json.dumps({"model": str(ckpt), "id": t})) == (gen._decode(t) or "")
