"""Native Llama engine (libcake_engine.so) vs the Python DeviceDecoder on the same
checkpoint: same kernels in the same order, so prefill logits agree to rounding and the
generated tokens are identical — greedy (fused head), greedy with a penalty window past
the fused head's bound, several steps per replay, sampled (top-k / top-p / seed), a
dtype conversion on load (bf16 checkpoint -> f16 engine), and a generation that crosses
the attention split-cap buckets."""
import pytest
import torch

from cake_amd.models.llama3.config import preset
from cake_amd.utils.synth import write_checkpoint

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = tmp_path_factory.mktemp("native_ckpt")
    cfg = preset("llama3-8b", num_hidden_layers=3, vocab_size=2048, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=8, num_key_value_heads=2,
                 bos_token_id=1, eos_token_id=2)
    write_checkpoint(d, cfg, torch.bfloat16, seed=3, single_file=True)
    return d


def _python(ckpt, dtype, max_seq, prompt, n, sampling=None, penalty=1.1, last_n=16, k=1):
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.factory import load_model
    from cake_amd.models.llama3.model import DeviceDecoder
    model = load_model(ckpt, "cuda:0", dtype, max_seq=max_seq)
    dec = DeviceDecoder(model, repeat_penalty=penalty, repeat_last_n=last_n, greedy=True,
                        steps_per_graph=k, sampling=sampling)
    first = dec.start(prompt)
    dec.capture()
    toks = [first] + run_decode(dec, n - 1).tokens
    logits = model.forward(prompt, 0).float().cpu()
    del dec, model
    torch.cuda.empty_cache()
    return toks, logits


def test_native_engine_matches_python_decoder(cuda, ckpt):
    from cake_amd.engine import NativeLlama
    from cake_amd.models.sampling import SamplingConfig
    prompt = [1, 17, 300, 5, 99, 1024, 7, 8]
    n = 24
    eng = NativeLlama(ckpt, max_seq=256, dtype="bf16")
    assert (eng.num_layers, eng.num_kv_heads, eng.head_dim) == (3, 2, 64)
    ref, ref_logits = _python(ckpt, torch.bfloat16, 256, prompt, n)
    logits = torch.from_numpy(eng.prefill_logits(prompt))
    torch.testing.assert_close(logits, ref_logits.reshape(-1)[-logits.numel():], atol=2e-2,
                               rtol=2e-2)
    got = eng.generate(prompt, n, repeat_penalty=1.1, repeat_last_n=16)
    assert got.tokens == ref
    assert got.n_prompt == len(prompt) and got.p50_ms > 0 and got.tokens_per_s > 0
    # the same engine again (graphs reused, state reset by the prefill)
    assert eng.generate(prompt, n, repeat_penalty=1.1, repeat_last_n=16).tokens == ref
    # penalty window beyond the fused head's bound: embed + lm_head + penalty + argmax tail
    ref2, _ = _python(ckpt, torch.bfloat16, 256, prompt, n, last_n=300)
    assert eng.generate(prompt, n, repeat_penalty=1.1, repeat_last_n=300).tokens == ref2
    # sampled: threshold + Gumbel-max draws keyed by (seed, step)
    s = SamplingConfig(temperature=0.8, top_k=20, top_p=0.9, seed=5)
    ref3, _ = _python(ckpt, torch.bfloat16, 256, prompt, n, sampling=s)
    got3 = eng.generate(prompt, n, temperature=0.8, top_k=20, top_p=0.9, seed=5,
                        repeat_penalty=1.1, repeat_last_n=16)
    assert got3.tokens == ref3
    # EOS stops the generation (inclusive) and the callback sees every token
    seen = []
    stop_at = ref[5]
    got4 = eng.generate(prompt, n, repeat_penalty=1.1, repeat_last_n=16, eos_ids=[stop_at],
                        on_token=lambda t: seen.append(t))
    assert got4.tokens == ref[:ref.index(stop_at) + 1] == seen
    eng.close()


def test_native_engine_f16_multistep_and_buckets(cuda, ckpt):
    """bf16 checkpoint converted to f16 on load, 4 steps per replay, and a live length
    crossing the one-split (320 keys) and 512-key bucket edges."""
    from cake_amd.engine import NativeLlama
    g = torch.Generator().manual_seed(2)
    prompt = torch.randint(3, 2048, (500,), generator=g).tolist()
    n = 20
    ref, _ = _python(ckpt, torch.float16, 1024, prompt, n, k=4)
    eng = NativeLlama(ckpt, max_seq=1024, dtype="f16", steps_per_graph=4)
    assert eng.generate(prompt, n, repeat_penalty=1.1, repeat_last_n=16).tokens == ref
    short = prompt[:300]
    ref2, _ = _python(ckpt, torch.float16, 1024, short, 40, k=4)
    assert eng.generate(short, 40, repeat_penalty=1.1, repeat_last_n=16).tokens == ref2
    eng.close()


def test_cake_cli_native_text_matches_python_cli(cuda, ckpt, tmp_path):
    """cake-cli on an all-local text model runs the native engine (the embedded
    interpreter only tokenizes); its streamed text equals the Python CLI's
    (CAKE_NATIVE=0) on the same flags."""
    import os
    import subprocess
    import sys
    from cake_amd.utils.synth import write_tokenizer  # noqa: F401  (ckpt has tokenizer.json)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    args = ["--model", str(ckpt), "--topology", str(tmp_path / "none.yml"), "--temperature", "0",
            "-n", "16", "--dtype", "bf16", "--prompt", "hello there", "--max-seq-len", "256"]
    env = dict(os.environ, CAKE_LOG="warning")
    nat = subprocess.run([cli, *args], capture_output=True, text=True, timeout=300, env=env,
                         cwd=root)
    assert nat.returncode == 0, nat.stderr[-3000:]
    assert "native engine" in nat.stderr and "token/s" in nat.stderr
    py = subprocess.run([sys.executable, "-m", "cake_amd.cli", *args], capture_output=True,
                        text=True, timeout=300, env=dict(env, CAKE_NATIVE="0"), cwd=root)
    assert py.returncode == 0, py.stderr[-3000:]
    assert nat.stdout.strip() and nat.stdout == py.stdout


def test_native_pipeline_two_ranks_share_one_gpu(cuda, ckpt, tmp_path):
    """Layer-sharded native pipeline: two rank processes on the same GPU (device hops
    through IPC-mapped inboxes, prefill rows through IPC-mapped buffers, TCP control
    plane).  f32 hops are exact, so tokens equal the single-rank engine — greedy, sampled,
    an EOS stop in the middle of an announced chunk, and a generation after it.  Both
    ranks are children of this process (siblings, as under torchrun: an IPC import reads
    the exporter's dmabuf through its pid)."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from cake_amd.engine import NativeLlama
    prompt = [1, 17, 300, 5, 99, 1024, 7, 8]
    single = NativeLlama(ckpt, max_seq=256, dtype="bf16")
    ref = single.generate(prompt, 30, repeat_penalty=1.1, repeat_last_n=16).tokens
    ref_s = single.generate(prompt, 30, temperature=0.7, top_k=40, seed=11,
                            repeat_penalty=1.1, repeat_last_n=16).tokens
    single.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    addr = f"127.0.0.1:{port}"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stop = ref[12]
    rank0 = ("import sys, json; sys.path.insert(0, %r)\n"
             "from cake_amd.engine import NativeLlama\n"
             "e = NativeLlama(%r, max_seq=256, dtype='bf16', rank=0, world=2, master_addr=%r)\n"
             "p = %r\n"
             "out = {'layers': [e.first_layer, e.end_layer]}\n"
             "out['greedy'] = e.generate(p, 30, repeat_penalty=1.1, repeat_last_n=16).tokens\n"
             "out['sampled'] = e.generate(p, 30, temperature=0.7, top_k=40, seed=11,\n"
             "                            repeat_penalty=1.1, repeat_last_n=16).tokens\n"
             "out['eos'] = e.generate(p, 30, repeat_penalty=1.1, repeat_last_n=16,\n"
             "                        eos_ids=[%d]).tokens\n"
             "out['again'] = e.generate(p, 30, repeat_penalty=1.1, repeat_last_n=16).tokens\n"
             "e.close()\n"
             "print(json.dumps(out), flush=True)\n") % (root, str(ckpt), addr, prompt, stop)
    rank1 = ("import sys; sys.path.insert(0, %r)\n"
             "from cake_amd.engine import NativeLlama\n"
             "e = NativeLlama(%r, max_seq=256, dtype='bf16', rank=1, world=2, master_addr=%r)\n"
             "e.serve()\n"
             "e.close()\n") % (root, str(ckpt), addr)
    logs = [tmp_path / "rank0.log", tmp_path / "rank1.log"]
    procs = [subprocess.Popen([sys.executable, "-c", c], stdout=subprocess.PIPE,
                              stderr=open(lg, "w"), text=True)
             for c, lg in ((rank0, logs[0]), (rank1, logs[1]))]
    try:
        out0, _ = procs[0].communicate(timeout=240)
        procs[1].wait(timeout=60)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    msg = "\n".join(f"---- {lg.name} ----\n" + lg.read_text()[-3000:] for lg in logs)
    assert procs[0].returncode == 0 and procs[1].returncode == 0, msg
    got = json.loads(out0.strip().splitlines()[-1])
    assert got["layers"][0] == 0 and got["layers"][1] < 3
    assert got["greedy"] == ref, msg
    assert got["sampled"] == ref_s
    assert got["eos"] == ref[:ref.index(stop) + 1]
    assert got["again"] == ref


@pytest.mark.parametrize("par", ["pp", "tp"])
def test_cake_cli_native_pipeline_torchrun(cuda, ckpt, tmp_path, par):
    """cake-cli --transport rccl --parallel pp|tp under torchrun (2 ranks sharing the GPU):
    the native pipeline prints the same text as the single-process native CLI (tensor
    parallel: the same first tokens — partial sums change the rounding only)."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    common = ["--model", str(ckpt), "--temperature", "0", "-n", "16", "--dtype", "bf16",
              "--prompt", "hello there", "--max-seq-len", "256", "--topology",
              str(tmp_path / "none.yml")]
    env = dict(os.environ, CAKE_LOG="warning")
    single = subprocess.run([cli, *common], capture_output=True, text=True, timeout=300, env=env,
                            cwd=root)
    assert single.returncode == 0, single.stderr[-3000:]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    pp = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
                         "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                         str(port), "--no-python", cli, *common, "--transport", "rccl",
                         "--parallel", par, "--hop", "ipc", "--hop-dtype", "f32"],
                        capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert pp.returncode == 0, pp.stderr[-3000:]
    if par == "pp":
        assert single.stdout.strip() and pp.stdout == single.stdout
    else:
        assert pp.stdout.strip() and pp.stdout[:8] == single.stdout[:8]


def test_cake_cli_native_tcp_worker(cuda, ckpt, tmp_path):
    """cake-cli --mode worker on the GPU serves its topology layers with the native engine
    (no interpreter in the worker: KV cache per master connection); a master using it
    prints the same text as the all-local native CLI."""
    import os
    import socket
    import subprocess
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{port}'\n  layers:\n    - 'model.layers.1-2'\n")
    gen = ["--temperature", "0", "-n", "12", "--dtype", "bf16", "--prompt", "hello there",
           "--max-seq-len", "256"]
    env = dict(os.environ, CAKE_LOG="warning")
    local = subprocess.run([cli, "--model", str(ckpt), "--topology", str(tmp_path / "none.yml"),
                            *gen], capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert local.returncode == 0, local.stderr[-3000:]
    w = subprocess.Popen([cli, "--mode", "worker", "--name", "w1", "--model", str(ckpt),
                          "--topology", str(topo), "--address", f"127.0.0.1:{port}", "--dtype",
                          "bf16", "--max-seq-len", "256"], cwd=root, env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        t0 = time.time()
        while True:
            if w.poll() is not None:
                raise AssertionError(f"worker exited: {w.stderr.read()[-3000:]}")
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
                break
            except OSError:
                assert time.time() - t0 < 180, "worker did not listen"
                time.sleep(0.3)
        dist = subprocess.run([cli, "--model", str(ckpt), "--topology", str(topo), *gen],
                              capture_output=True, text=True, timeout=300, env=env, cwd=root)
        assert dist.returncode == 0, dist.stderr[-3000:]
        assert local.stdout.strip() and dist.stdout == local.stdout
    finally:
        w.kill()
        err = w.communicate()[1]
    assert "native worker" in err


def test_native_tensor_parallel_two_ranks(cuda, ckpt, tmp_path):
    """Native tensor parallelism: two rank processes on the shared GPU, each 1/2 of every
    layer's heads and MLP rows and of the vocabulary; device all-reduces (IPC inboxes) in
    the captured step, prefill sums through IPC slabs.  The partial sums change rounding
    only: the first token and a long prefix of the greedy tokens equal the single-rank
    engine's; EOS truncation and a second generation work in lock step."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from cake_amd.engine import NativeLlama
    prompt = [1, 17, 300, 5, 99, 1024, 7, 8]
    single = NativeLlama(ckpt, max_seq=256, dtype="bf16")
    ref = single.generate(prompt, 24, repeat_penalty=1.1, repeat_last_n=16).tokens
    single.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    addr = f"127.0.0.1:{port}"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rank0 = ("import sys, json; sys.path.insert(0, %r)\n"
             "from cake_amd.engine import NativeLlama\n"
             "e = NativeLlama(%r, max_seq=256, dtype='bf16', rank=0, world=2, master_addr=%r, tp=True)\n"
             "p = %r\n"
             "out = {'greedy': e.generate(p, 24, repeat_penalty=1.1, repeat_last_n=16).tokens}\n"
             "out['sampled'] = e.generate(p, 16, temperature=0.8, top_k=20, seed=3,\n"
             "                            repeat_penalty=1.1, repeat_last_n=16).tokens\n"
             "g = out['greedy']\n"
             "out['eos'] = e.generate(p, 24, repeat_penalty=1.1, repeat_last_n=16,\n"
             "                        eos_ids=[g[6]]).tokens\n"
             "out['again'] = e.generate(p, 24, repeat_penalty=1.1, repeat_last_n=16).tokens\n"
             "e.close()\n"
             "print(json.dumps(out), flush=True)\n") % (root, str(ckpt), addr, prompt)
    rank1 = ("import sys; sys.path.insert(0, %r)\n"
             "from cake_amd.engine import NativeLlama\n"
             "e = NativeLlama(%r, max_seq=256, dtype='bf16', rank=1, world=2, master_addr=%r, tp=True)\n"
             "e.serve()\n"
             "e.close()\n") % (root, str(ckpt), addr)
    logs = [tmp_path / "tp0.log", tmp_path / "tp1.log"]
    procs = [subprocess.Popen([sys.executable, "-c", c], stdout=subprocess.PIPE,
                              stderr=open(lg, "w"), text=True)
             for c, lg in ((rank0, logs[0]), (rank1, logs[1]))]
    try:
        out0, _ = procs[0].communicate(timeout=240)
        procs[1].wait(timeout=60)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    msg = "\n".join(f"---- {lg.name} ----\n" + lg.read_text()[-3000:] for lg in logs)
    assert procs[0].returncode == 0 and procs[1].returncode == 0, msg
    got = json.loads(out0.strip().splitlines()[-1])
    g = got["greedy"]
    assert len(g) == 24 and g[0] == ref[0], (g, ref)
    same = next((i for i, (a, b) in enumerate(zip(g, ref)) if a != b), len(ref))
    assert same >= 8, f"TP diverged from single-GPU at token {same}: {g} vs {ref}"
    assert got["again"] == g and len(got["sampled"]) == 16
    assert got["eos"] == g[:g.index(g[6]) + 1]
