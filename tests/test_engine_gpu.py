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


@pytest.mark.parametrize("fused", ["0", "1"])
def test_native_engine_f16_multistep_and_buckets(cuda, ckpt, fused, monkeypatch):
    """bf16 checkpoint converted to f16 on load, 4 steps per replay, and a live length
    crossing the one-split (320 keys) and 512-key bucket edges; with and without the
    opt-in fused attention + o_proj bucket (CAKE_ATTN_OPROJ=1, engine and Python alike)."""
    from cake_amd.engine import NativeLlama
    monkeypatch.setenv("CAKE_ATTN_OPROJ", fused)
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


@pytest.mark.parametrize("par", ["pp", "tp", "pp-topology"])
def test_cake_cli_native_pipeline_torchrun(cuda, ckpt, tmp_path, par):
    """cake-cli --transport rccl --parallel pp|tp under torchrun (2 ranks sharing the GPU):
    the native pipeline prints the same text as the single-process native CLI (tensor
    parallel: the same first tokens — partial sums change the rounding only).  pp-topology:
    topology.yml places layer 1 on the worker (node 1 -> rank 1): master 0, worker 1,
    master 2, as the reference's placement loop."""
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
    extra = []
    if par == "pp-topology":
        topo = tmp_path / "t.yml"
        topo.write_text("w1:\n  host: 'rank1'\n  layers:\n    - 'model.layers.1'\n")
        extra = ["--topology", str(topo)]
    pp = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
                         "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                         str(port), "--no-python", cli, *common, *extra, "--transport", "rccl",
                         "--parallel", par.split("-")[0], "--hop", "ipc", "--hop-dtype", "f32"],
                        capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert pp.returncode == 0, pp.stderr[-3000:]
    if par.startswith("pp"):
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
        # the master ran natively too (the engine's TCP client, no interpreter compute)
        assert "native master over TCP workers" in dist.stderr, dist.stderr[-3000:]
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


# ---------------------------------------------------------------------------------------
# multi-rank native groups: N rank processes (siblings, sharing the GPU on the 1-GPU pool)
# ---------------------------------------------------------------------------------------
def _port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _group(tmp_path, ckpt, world, rank0_body, kw="", timeout=240, tag="g"):
    """Run rank 0 (``rank0_body`` with ``e`` the engine, printing ``out`` as JSON) and
    world - 1 serving ranks; ``kw`` = extra NativeLlama keyword text.  Returns rank 0's
    dict; on failure every rank's log is in the assertion message."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    addr = f"127.0.0.1:{_port()}"
    head = ("import sys, json; sys.path.insert(0, %r)\n"
            "from cake_amd.engine import NativeLlama\n"
            "e = NativeLlama(%r, max_seq=1024, dtype='bf16', rank=%%d, world=%d, master_addr=%r, "
            "hop_timeout_s=30.0%s)\n") % (root, str(ckpt), world, addr, kw)
    r0 = head % 0 + "out = {'walk': e.walk()}\n" + rank0_body + \
        "e.close()\nprint(json.dumps(out), flush=True)\n"
    rw = head + "e.serve()\ne.close()\n"
    logs = [tmp_path / f"{tag}{r}.log" for r in range(world)]
    procs = [subprocess.Popen([sys.executable, "-c", r0 if r == 0 else rw % r],
                              stdout=subprocess.PIPE, stderr=open(logs[r], "w"), text=True)
             for r in range(world)]
    try:
        out0, _ = procs[0].communicate(timeout=timeout)
        for p in procs[1:]:
            p.wait(timeout=60)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    msg = "\n".join(f"---- {lg.name} ----\n" + lg.read_text()[-3000:] for lg in logs)
    assert all(p.returncode == 0 for p in procs), msg
    return json.loads(out0.strip().splitlines()[-1]), msg


PROMPT = [1, 17, 300, 5, 99, 1024, 7, 8]


@pytest.mark.parametrize("world,owners,walk", [
    (2, [0, 1, 0], "0:0-0,1:1-1,0:2-2"),   # master, worker, master (llama.rs:95-114)
    (2, [1, 0, 1], "1:0-0,0:1-1,1:2-2"),   # a worker visited twice per token
    (3, [2, 1, 0], "2:0-0,1:1-1,0:2-2"),   # reversed ranks: edges 0->2->1->0
    (3, [0, 0, 2], "0:0-1,2:2-2"),         # rank 1 idle (a topology node with no layers)
])
def test_native_pipeline_topology_placement(cuda, ckpt, tmp_path, world, owners, walk):
    """cake_engine_open_pp with an owner map (topology.yml: node i -> rank i + 1): the walk
    has one stop per maximal run and f32 hops are exact, so greedy and sampled tokens equal
    the single-rank engine, and continue() extends a generation as one longer one."""
    from cake_amd.engine import NativeLlama
    single = NativeLlama(ckpt, max_seq=1024, dtype="bf16")
    ref = single.generate(PROMPT, 30, repeat_penalty=1.1, repeat_last_n=16).tokens
    ref_s = single.generate(PROMPT, 20, temperature=0.7, top_k=40, seed=11,
                            repeat_penalty=1.1, repeat_last_n=16).tokens
    single.close()
    body = ("g = e.generate(%r, 18, repeat_penalty=1.1, repeat_last_n=16).tokens\n"
            "out['greedy'] = g + e.continue_(12).tokens\n"
            "out['sampled'] = e.generate(%r, 20, temperature=0.7, top_k=40, seed=11,\n"
            "                            repeat_penalty=1.1, repeat_last_n=16).tokens\n"
            ) % (PROMPT, PROMPT)
    got, msg = _group(tmp_path, ckpt, world, body, kw=", owners=%r" % (owners,))
    assert got["walk"] == walk, msg
    assert got["greedy"] == ref, msg
    assert got["sampled"] == ref_s, msg


def _forced_ref(ckpt, n):
    """Single-rank engine: its greedy tokens and the teacher-forced logits along them."""
    from cake_amd.engine import NativeLlama
    single = NativeLlama(ckpt, max_seq=1024, dtype="bf16")
    toks = single.generate(PROMPT, n + 1, repeat_penalty=1.0).tokens
    ref = single.forced_logits(PROMPT, toks[:n])
    single.close()
    return toks[:n], ref


def _assert_forced_close(got, ref, rel, what):
    """Every step's logits within rel x max|logit| of the single-rank engine's, and the
    argmax equal wherever the single-rank top-2 margin exceeds that bound."""
    import numpy as np
    got, ref = np.asarray(got, dtype=np.float32), np.asarray(ref, dtype=np.float32)
    assert got.shape == ref.shape
    tol = rel * float(np.abs(ref).max())
    err = float(np.abs(got - ref).max())
    assert err <= tol, f"{what}: max |dlogit| {err:.4g} > {tol:.4g}"
    top2 = np.sort(ref, axis=1)[:, -2:]
    sure = (top2[:, 1] - top2[:, 0]) > 2 * tol
    assert (got.argmax(1)[sure] == ref.argmax(1)[sure]).all(), f"{what}: argmax differs"


def test_native_pipeline_bf16_hops_world3_teacher_forced(cuda, ckpt, tmp_path):
    """bf16 hop payloads (half the bytes; the reference ships the model dtype) over a
    3-rank walk: teacher-forced over 32 decode steps, every step's logits within 2 % of
    the logit range of the single-rank engine's (f32 hops are exact; bf16 rounds the
    residual stream at each of the 3 edges)."""
    import numpy as np
    forced, ref = _forced_ref(ckpt, 32)
    body = "import numpy as np\nout['logits'] = e.forced_logits(%r, %r).tolist()\n" % (PROMPT, forced)
    got, msg = _group(tmp_path, ckpt, 3, body, kw=", hop_bf16=True")
    assert got["walk"] == "0:0-0,1:1-1,2:2-2", msg
    _assert_forced_close(np.array(got["logits"]), ref, 0.02, "pp3 bf16 hops")
    # f32 hops: exact
    got2, msg = _group(tmp_path, ckpt, 3, body, tag="f")
    assert np.array_equal(np.array(got2["logits"], dtype=np.float32), ref), msg


@pytest.fixture(scope="module")
def ckpt3(tmp_path_factory):
    """3 KV heads (6 query heads, head_dim 64): tensor parallelism of degree 3."""
    d = tmp_path_factory.mktemp("native_ckpt3")
    cfg = preset("llama3-8b", num_hidden_layers=3, vocab_size=2048, intermediate_size=768,
                 hidden_size=384, num_attention_heads=6, num_key_value_heads=3,
                 bos_token_id=1, eos_token_id=2)
    write_checkpoint(d, cfg, torch.bfloat16, seed=4, single_file=True)
    return d


@pytest.mark.parametrize("world", [2, 3])
def test_native_tensor_parallel_teacher_forced(cuda, ckpt, ckpt3, tmp_path, world):
    """Native tensor parallelism teacher-forced over 32 decode steps (the decode kernels and
    device all-reduces of the captured step, launched eagerly): every step's logits within
    1 % of the logit range of the single-rank engine's (partial sums reorder f32 adds and
    round each rank's bf16 attention / MLP activations), argmax equal wherever the margin
    is larger; then greedy generate + continue in lock step."""
    import numpy as np
    ck = ckpt if world == 2 else ckpt3
    forced, ref = _forced_ref(ck, 32)
    body = ("out['logits'] = e.forced_logits(%r, %r).tolist()\n"
            "g = e.generate(%r, 10, repeat_penalty=1.0).tokens\n"
            "out['gen'] = g + e.continue_(6).tokens\n"
            "out['eos'] = e.generate(%r, 16, repeat_penalty=1.0, eos_ids=[g[4]]).tokens\n"
            ) % (PROMPT, forced, PROMPT, PROMPT)
    got, msg = _group(tmp_path, ck, world, body, kw=", tp=True", tag=f"tp{world}_")
    _assert_forced_close(np.array(got["logits"]), ref, 0.01, f"tp{world}")
    g = got["gen"]
    assert len(g) == 16 and g[0] == forced[0], msg
    assert got["eos"] == g[:g.index(g[4]) + 1], msg


def test_native_engine_attention_error_word(cuda, ckpt):
    """A split-K attention merge that gives up waiting (test hook: the other splits never
    publish) sets tickets[2 nkv]; the engine raises after the generation instead of
    returning its tokens, clears the word, and the next generation is correct."""
    from cake_amd.engine import NativeLlama
    from cake_amd.ops import hip as K
    g = torch.Generator().manual_seed(5)
    prompt = torch.randint(3, 2048, (400,), generator=g).tolist()  # > 320 keys: split merge
    eng = NativeLlama(ckpt, max_seq=1024, dtype="bf16")
    ref = eng.generate(prompt, 4, repeat_penalty=1.0).tokens
    # the hook is a launch argument: a new sampling mode recaptures the graphs with it
    K.attn_debug_drop_partials(True)
    try:
        with pytest.raises(RuntimeError, match="split merge timed out"):
            eng.generate(prompt, 3, repeat_penalty=1.05)
    finally:
        K.attn_debug_drop_partials(False)
    assert eng.generate(prompt, 4, repeat_penalty=1.0).tokens == ref  # recaptured, clean
    eng.close()


def test_native_continue_equals_one_generation(cuda, ckpt):
    from cake_amd.engine import NativeLlama
    eng = NativeLlama(ckpt, max_seq=1024, dtype="bf16")
    ref = eng.generate(PROMPT, 40, repeat_penalty=1.1, repeat_last_n=16).tokens
    a = eng.generate(PROMPT, 15, repeat_penalty=1.1, repeat_last_n=16).tokens
    b = eng.continue_(10).tokens
    c = eng.continue_(15).tokens
    assert a + b + c == ref
    # random init: config.json only, seeded device draws (benchmarks); deterministic
    from cake_amd.engine import write_config
    from cake_amd.models.llama3.config import LlamaConfig
    import tempfile
    d = write_config(tempfile.mkdtemp(), LlamaConfig.from_path(ckpt))
    r1 = NativeLlama(d, max_seq=256, dtype="bf16", random_init=True, seed=7)
    t1 = r1.generate(PROMPT, 12, repeat_penalty=1.0).tokens
    r1.close()
    r2 = NativeLlama(d, max_seq=256, dtype="bf16", random_init=True, seed=7)
    assert r2.generate(PROMPT, 12, repeat_penalty=1.0).tokens == t1
    r2.close()
    eng.close()


def _wait_listen(proc, port, what, t_max=180):
    import socket
    import time
    t0 = time.time()
    while True:
        if proc.poll() is not None:
            raise AssertionError(f"{what} exited: {proc.stderr.read()[-3000:]}")
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return
        except OSError:
            assert time.time() - t0 < t_max, f"{what} did not listen"
            time.sleep(0.3)


def test_native_master_two_tcp_workers_interleaved(cuda, ckpt, tmp_path):
    """A topology with two native TCP workers, one of them visited twice per token
    (w1: layers 0 and 2, w2: layer 1): the native master's walk is w0 -> w1 -> w0, each a
    Batch round trip; the text equals the all-local engine's.  w2 is started through the
    embeddable C ABI (cake_start_worker in libcake_runtime.so), which serves text natively."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    p1, p2 = _port(), _port()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{p1}'\n  layers:\n    - 'model.layers.0'\n"
                    f"    - 'model.layers.2'\n"
                    f"w2:\n  host: '127.0.0.1:{p2}'\n  layers:\n    - 'model.layers.1'\n")
    gen = ["--temperature", "0", "-n", "14", "--prompt", "hello there", "--max-seq-len", "256"]
    env = dict(os.environ, CAKE_LOG="warning")
    local = subprocess.run([cli, "--model", str(ckpt), "--topology", str(tmp_path / "none.yml"),
                            *gen], capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert local.returncode == 0, local.stderr[-3000:]
    w1 = subprocess.Popen([cli, "--mode", "worker", "--name", "w1", "--model", str(ckpt),
                           "--topology", str(topo), "--address", f"127.0.0.1:{p1}",
                           "--max-seq-len", "256"], cwd=root, env=env,
                          stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    capi = ("import ctypes, sys\n"
            "L = ctypes.CDLL(%r)\n"
            "L.cake_start_worker.argtypes = [ctypes.c_char_p] * 5\n"
            "sys.exit(L.cake_start_worker(b'w2', %r, %r, b'text', b'127.0.0.1:%d'))\n") % (
        os.path.join(root, "cake_amd", "lib", "libcake_runtime.so"), str(ckpt).encode(),
        str(topo).encode(), p2)
    w2 = subprocess.Popen([sys.executable, "-c", capi], cwd=root, env=env,
                          stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        _wait_listen(w1, p1, "worker w1")
        _wait_listen(w2, p2, "worker w2 (cake_start_worker)")
        dist = subprocess.run([cli, "--model", str(ckpt), "--topology", str(topo), *gen],
                              capture_output=True, text=True, timeout=300,
                              env=dict(env, CAKE_ENGINE_TRACE="1"), cwd=root)
        assert dist.returncode == 0, dist.stderr[-3000:]
        assert "native master over TCP workers" in dist.stderr, dist.stderr[-3000:]
        assert local.stdout.strip() and dist.stdout == local.stdout, (dist.stdout, local.stdout)
    finally:
        for w in (w1, w2):
            w.kill()
        e1, e2 = w1.communicate()[1], w2.communicate()[1]
    assert "native worker w1" in e1
    assert "[cake_start_worker] native worker w2" in e2, e2[-2000:]


def test_native_api_serving_over_tcp_workers(cuda, ckpt, tmp_path):
    """--api on the native engine with a TCP worker in the topology: the REST answer
    equals the all-local native server's (greedy), and the master's text path is the
    engine (NativeLLM over cake_engine_open_remote)."""
    import os
    import subprocess
    from fastapi.testclient import TestClient
    from cake_amd.api.server import create_app
    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import Master
    from cake_amd.models.llama3.native_generator import NativeLLM
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    port = _port()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{port}'\n  layers:\n    - 'model.layers.1-2'\n")
    (tmp_path / "empty.yml").write_text("{}\n")
    common = ["--model", str(ckpt), "--dtype", "bf16", "--temperature", "0", "--max-seq-len",
              "256"]
    req = {"messages": [{"role": "user", "content": "hello there"}], "max_tokens": 16}
    m0 = Master(Context.from_args(build_parser().parse_args(
        common + ["--topology", str(tmp_path / "empty.yml")])))
    assert isinstance(m0.llm, NativeLLM)
    want = TestClient(create_app(m0)).post("/api/v1/chat/completions", json=req).json()
    m0.llm.eng.close()
    w = subprocess.Popen([cli, "--mode", "worker", "--name", "w1", "--model", str(ckpt),
                          "--topology", str(topo), "--address", f"127.0.0.1:{port}", "--dtype",
                          "bf16", "--max-seq-len", "256"], cwd=root,
                         env=dict(os.environ, CAKE_LOG="warning"), stdout=subprocess.DEVNULL,
                         stderr=subprocess.PIPE, text=True)
    try:
        _wait_listen(w, port, "worker")
        m1 = Master(Context.from_args(build_parser().parse_args(common + ["--topology", str(topo)])))
        assert isinstance(m1.llm, NativeLLM) and m1.llm.eng.walk() == "0:0-0,w0:1-2"
        got = TestClient(create_app(m1)).post("/api/v1/chat/completions", json=req).json()
        m1.llm.eng.close()
    finally:
        w.kill()
        w.communicate()
    assert want["choices"][0]["message"]["content"]
    assert got["choices"][0]["message"]["content"] == want["choices"][0]["message"]["content"]


def test_native_master_fails_loudly_when_a_worker_dies(cuda, ckpt, tmp_path):
    """Failure detection on the native master's TCP client: a generation through a live
    worker succeeds; after the worker is killed the next generation raises (connection
    error or the remote timeout) instead of hanging or emitting tokens."""
    import os
    import subprocess
    import time

    from cake_amd.engine import NativeLlama
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    port = _port()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{port}'\n  layers:\n    - 'model.layers.1'\n")
    env = dict(os.environ, CAKE_LOG="warning")
    w = subprocess.Popen([cli, "--mode", "worker", "--name", "w1", "--model", str(ckpt),
                          "--topology", str(topo), "--address", f"127.0.0.1:{port}",
                          "--max-seq-len", "256"], cwd=root, env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    eng = None
    try:
        _wait_listen(w, port, "worker w1")
        eng = NativeLlama(ckpt, max_seq=256, dtype="bf16", workers=[f"127.0.0.1:{port}"],
                          worker_of=[-1, 0, -1], remote_timeout_s=10.0)
        ok = eng.generate(PROMPT, 6, repeat_penalty=1.0).tokens
        assert len(ok) == 6
        w.kill()
        w.wait(timeout=30)
        t0 = time.time()
        with pytest.raises(RuntimeError):
            eng.generate(PROMPT, 6, repeat_penalty=1.0)
        assert time.time() - t0 < 60
    finally:
        if eng is not None:
            eng.close()
        if w.poll() is None:
            w.kill()
        w.communicate()
