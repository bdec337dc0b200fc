"""Whole-model golden tests on the GPU: HIP kernel path vs the PyTorch reference path."""
import pytest
import torch

from cake_amd.models.llama3.config import preset
from cake_amd.models.llama3.factory import random_model

pytestmark = pytest.mark.gpu


def _pair(cfg, dt, seed=0, max_seq=512):
    hip = random_model(cfg, "cuda:0", dt, max_seq=max_seq, backend="hip", seed=seed)
    ref = random_model(cfg, "cuda:0", dt, max_seq=max_seq, backend="torch", seed=seed)
    return hip, ref


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("name", ["tiny", "mid"])
def test_prefill_and_decode_logits_match_reference(cuda, dt, name):
    cfg = preset("tiny") if name == "tiny" else preset(
        "llama3-8b", num_hidden_layers=2, vocab_size=4096, intermediate_size=2048)
    hip, ref = _pair(cfg, dt)
    prompt = list(range(3, 40))
    lh = hip.forward(prompt, 0)
    lr = ref.forward(prompt, 0)
    torch.testing.assert_close(lh, lr, atol=5e-2, rtol=5e-2)
    # decode 8 tokens one at a time, greedy, teacher-forced on the reference argmax
    pos = len(prompt)
    tok = int(torch.argmax(lr))
    for _ in range(8):
        lh = hip.forward([tok], pos)
        lr = ref.forward([tok], pos)
        torch.testing.assert_close(lh, lr, atol=5e-2, rtol=5e-2)
        tok = int(torch.argmax(lr))
        pos += 1


@pytest.mark.parametrize("use_graph", [False, True])
@pytest.mark.parametrize("k", [1, 4])
def test_device_decoder_matches_host_loop(cuda, use_graph, k):
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.ops import reference as R

    cfg = preset("llama3-8b", num_hidden_layers=3, vocab_size=2048, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=4, num_key_value_heads=1)
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=256, seed=3)
    prompt = [5, 6, 7, 8, 9, 10, 11]
    # host loop (generic path + host penalty/argmax)
    toks = list(prompt)
    logits = model.forward(prompt, 0)
    host = []
    for i in range(12):
        lp = R.apply_repeat_penalty(logits, 1.1, toks[-16:])
        t = int(torch.argmax(lp))
        host.append(t)
        toks.append(t)
        logits = model.forward([t], len(toks) - 1)
    dec = DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16, greedy=True,
                        use_graph=use_graph, steps_per_graph=k)
    first = dec.start(prompt)
    dec.capture()
    st = run_decode(dec, 11)  # 11 is not a multiple of k: the last launch overshoots
    assert [first] + st.tokens == host
    assert len(st.step_ms) == 11 and all(x > 0 for x in st.step_ms)


@pytest.mark.parametrize("k", [1, 3])
def test_native_decode_loop_eos_and_callback(cuda, k):
    """The C++ decode driver (graph_loop.cpp): tokens equal the eager loop's, it stops at
    the first EOS (inclusive) and when the per-token callback asks, and the host position
    mirror advances by whole replays."""
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.model import DeviceDecoder

    cfg = preset("llama3-8b", num_hidden_layers=2, vocab_size=2048, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=4, num_key_value_heads=1)
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=256, seed=7)
    prompt = [3, 1, 4, 1, 5, 9, 2, 6]

    def fresh(use_graph):
        dec = DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16, greedy=True,
                            use_graph=use_graph, steps_per_graph=k)
        first = dec.start(prompt)
        dec.capture()
        return dec, first

    dec, first = fresh(False)
    ref = [first] + run_decode(dec, 14).tokens            # eager Python loop
    dec, first = fresh(True)
    pos0 = dec.host_pos
    st = run_decode(dec, 14)                              # native loop
    assert [first] + st.tokens == ref
    assert dec.host_pos == pos0 + -(-14 // k) * k
    assert len(st.step_ms) == 14 and all(x > 0 for x in st.step_ms)
    eos = ref[6]
    dec, first = fresh(True)
    got = run_decode(dec, 14, eos_ids={eos}).tokens
    assert got == ref[1:ref.index(eos, 1) + 1]
    seen = []
    dec, first = fresh(True)
    got = run_decode(dec, 14, on_token=lambda t: (seen.append(t), len(seen) >= 4)[1]).tokens
    assert got == seen == ref[1:5]


def test_device_decoder_crosses_split_buckets(cuda):
    """Graphs captured per attention split cap: a generation whose live length crosses
    the 512-key bucket edge (cap 8 -> 16) matches the host loop token for token."""
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.ops import hip as K
    from cake_amd.ops import reference as R

    cfg = preset("llama3-8b", num_hidden_layers=2, vocab_size=2048, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=8, num_key_value_heads=2)
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=4096, seed=4)
    g = torch.Generator().manual_seed(9)
    prompt = torch.randint(0, 2048, (503,), generator=g).tolist()
    toks = list(prompt)
    logits = model.forward(prompt, 0)
    host = []
    for _ in range(16):
        t = int(torch.argmax(R.apply_repeat_penalty(logits, 1.1, toks[-16:])))
        host.append(t)
        toks.append(t)
        logits = model.forward([t], len(toks) - 1)
    dec = DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16, greedy=True)
    first = dec.start(prompt)
    dec.capture()
    # caps up to the first covering every live length (core 2 at 16 splits: 8 and 16),
    # below them the one-split bucket of fused attention + o_proj launches (key 1)
    assert sorted(dec.graphs) == ([1] if model.stack.attn_oproj_ok() else []) + \
        K.attn_split_caps(4096)
    assert [c for c in sorted(dec.graphs) if c > 1][:2] == [8, 16]
    assert dec._graph_for(500) is dec.graphs[8] and dec._graph_for(600) is dec.graphs[16]
    assert K.attn_splits(4096) == (32 if K._ATTN_IMPL[0] == 1 else 16)
    st = run_decode(dec, 15)
    assert [first] + st.tokens == host


@pytest.mark.parametrize("k", [1, 4])
def test_device_decoder_crosses_one_split_edge(cuda, k, monkeypatch):
    """Live lengths crossing the one-split edge (320 keys): the one-split graph of fused
    attention + o_proj launches (opt-in, CAKE_ATTN_OPROJ=1) up to it, the split-K graph
    (cap 8) after it — tokens equal the host loop."""
    monkeypatch.setenv("CAKE_ATTN_OPROJ", "1")
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.ops import hip as K
    from cake_amd.ops import reference as R
    if not hasattr(K.kernels(), "cake_attn_oproj"):
        pytest.skip("fused attention + o_proj not built (csrc/experimental: "
                    "CAKE_BUILD_EXPERIMENTAL=1)")

    cfg = preset("llama3-8b", num_hidden_layers=2, vocab_size=2048, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=8, num_key_value_heads=2)
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=1024, seed=6)
    g = torch.Generator().manual_seed(3)
    prompt = torch.randint(0, 2048, (310,), generator=g).tolist()
    toks = list(prompt)
    logits = model.forward(prompt, 0)
    host = []
    for _ in range(20):
        t = int(torch.argmax(R.apply_repeat_penalty(logits, 1.1, toks[-16:])))
        host.append(t)
        toks.append(t)
        logits = model.forward([t], len(toks) - 1)
    dec = DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16, greedy=True,
                        steps_per_graph=k)
    first = dec.start(prompt)
    dec.capture()
    assert 1 in dec.graphs
    assert dec._graph_for(320) is dec.graphs[1] and dec._graph_for(321) is dec.graphs[8]
    st = run_decode(dec, 19)
    assert [first] + st.tokens == host


def test_pipeline_engine_single_rank_streams(cuda):
    """The RCCL pipeline's graph bodies (world=1, 2 streams) == DeviceDecoder per stream."""
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.factory import random_head, random_stack
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.parallel.pipeline import PipelineEngine

    cfg = preset("llama3-8b", num_hidden_layers=3, vocab_size=2048, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=4, num_key_value_heads=1)
    prompts = [[5, 6, 7, 8, 9], [100, 3, 3, 12]]
    expect = []
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=256, seed=3)
    for p in prompts:
        dec = DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16, greedy=True)
        first = dec.start(p)
        dec.capture()
        expect.append(p + [first] + run_decode(dec, 9).tokens)
    stack = random_stack(cfg, list(range(3)), "cuda:0", torch.bfloat16, max_seq=256, seed=3)
    eng = PipelineEngine(cfg, stack, [0, 0, 0], 0, 1, streams=2,
                         head=random_head(cfg, "cuda:0", torch.bfloat16, seed=3),
                         repeat_penalty=1.1, repeat_last_n=16)
    for s, p in enumerate(prompts):
        eng.prefill(s, p)
    eng.capture()
    eng.decode(9)
    torch.cuda.synchronize()
    assert [eng.tokens(0), eng.tokens(1)] == expect


def test_profile_layers_per_layer_ms(cuda):
    """Per-layer decode kernel ms for the --metrics sink (one small graph per layer)."""
    from cake_amd.models.llama3.config import preset
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.factory import random_model
    from cake_amd.models.llama3.model import DeviceDecoder
    cfg = preset("llama3-8b", num_hidden_layers=3, vocab_size=4096, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=4, num_key_value_heads=1)
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=128, seed=1)
    dec = DeviceDecoder(model)
    first = dec.start([1, 2, 3])
    dec.capture()
    toks = [first] + run_decode(dec, 6).tokens
    ms = dec.profile_layers()
    assert len(ms) == 3 and all(0 < x < 5 for x in ms)
    # decoding again from the same prompt is unaffected by the profiling replays
    first = dec.start([1, 2, 3])
    assert [first] + run_decode(dec, 6).tokens == toks


def test_worker_step_graphs_match_eager(cuda):
    """Worker serving path: T = 1 forward() over a layer run replays one captured graph
    per (session, run); outputs equal the eager launches, sessions stay independent,
    and evicting a session drops its graphs."""
    cfg = preset("llama3-8b", num_hidden_layers=4, vocab_size=512, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=4, num_key_value_heads=1)
    m = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=64, seed=3)
    st = m.stack
    torch.manual_seed(0)
    xs = [torch.randn(1, 512, device=cuda) for _ in range(6)]

    def run(graphs):
        st.step_graphs = graphs
        st.reset()
        outs = []
        for sess in (0, 1):
            for p, x in enumerate(xs[:3] if sess == 0 else xs[3:]):
                h = x.clone()
                st.forward(h, [1, 2], p, session=sess)
                outs.append(h)
        return torch.stack(outs)
    ref = run(False)
    got = run(True)
    torch.testing.assert_close(got, ref, atol=1e-3, rtol=1e-3)
    assert {k[0] for k in st._step_graph_cache} == {0, 1}
    st.drop(1)
    assert {k[0] for k in st._step_graph_cache} == {0}
    st.step_graphs = False
