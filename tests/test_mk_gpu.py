"""Persistent decode (csrc/experimental/decode_mk.hip) against the five-launch layer path.

Experimental: measured slower than the launch path (profiles/r4_mk_summary.md), so it is
not in the default build; build with CAKE_BUILD_EXPERIMENTAL=1 to run these.

Both paths run the same decode step (RMSNorm, QKV + RoPE + KV write, GQA attention
over the cache, o_proj + residual, RMSNorm + SwiGLU, down_proj + residual) from the
same state; the per-launch path is itself pinned to the f32 PyTorch reference math by
test_kernels_gpu.py / test_model_gpu.py.  Positions cover the single-split attention
(<= 320 keys), the multi-split merge (> 320 keys) and the split count's growth.
"""
import pytest
import torch

from cake_amd.models.llama3.config import preset
from cake_amd.models.llama3.factory import random_stack

pytestmark = pytest.mark.gpu


def _stack(cfg, max_seq, seed=0):
    st = random_stack(cfg, list(range(cfg.num_hidden_layers)), "cuda:0", torch.bfloat16,
                      max_seq=max_seq, seed=seed)
    st.use_mk = True
    from cake_amd.ops import hip as K
    if not K.mk_available():
        pytest.skip("persistent decode engine not built (CAKE_BUILD_EXPERIMENTAL=1)")
    if not st.mk_enabled():
        pytest.skip("persistent decode not supported here")
    return st


def _torch_step(st, layers, resid0, pos):
    """The f32 PyTorch reference math of the step (LayerStack._block_torch: model-dtype
    normalised rows, f32 attention) on a copy of the cache."""
    kv = st.cache(0)
    kc, vc = kv.k.clone(), kv.v.clone()
    h = resid0.clone()[None]
    for li in layers:
        s = st.slot_of[li]
        st._block_torch(h, st.weights[li], kc[s], vc[s], pos)
    return h[0]


def _step(st, bufs, layers, resid0, pos, use_mk):
    st.use_mk = use_mk
    bufs.resid.copy_(resid0)
    bufs.pos.fill_(pos)
    st.decode_step(bufs, layers)
    torch.cuda.synchronize()
    return bufs.resid.clone()


CFGS = {
    # GQA 4:1 (8B-like heads), small widths
    "small": dict(hidden_size=1024, intermediate_size=2560, num_attention_heads=8,
                  num_key_value_heads=2, num_hidden_layers=3, vocab_size=512),
    # the 8B layer itself (2 layers)
    "8b": dict(num_hidden_layers=2, vocab_size=512),
    # GQA 8:1 (70B-like heads), small widths
    "gqa8": dict(hidden_size=2048, intermediate_size=3072, num_attention_heads=16,
                 num_key_value_heads=2, num_hidden_layers=2, vocab_size=512),
}


@pytest.mark.parametrize("name", list(CFGS))
def test_mk_step_matches_launches(cuda, name):
    cfg = preset("llama3-8b", **CFGS[name])
    max_seq = 2048
    st = _stack(cfg, max_seq)
    layers = list(range(cfg.num_hidden_layers))
    bufs = st.decode_buffers()
    kv = st.cache(0)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    # a populated cache (keys/values of earlier positions)
    kv.k.normal_(0.0, 1.0, generator=g)
    kv.v.normal_(0.0, 1.0, generator=g)
    for pos in (0, 7, 200, 319, 320, 333, 700, 1500, max_seq - 1):
        resid0 = torch.randn(cfg.hidden_size, device="cuda:0", generator=g)
        gold = _torch_step(st, layers, resid0, pos)
        ref = _step(st, bufs, layers, resid0, pos, False)
        kref = kv.k[:, :, pos].clone()
        vref = kv.v[:, :, pos].clone()
        kv.k[:, :, pos] = 0
        kv.v[:, :, pos] = 0
        out = _step(st, bufs, layers, resid0, pos, True)
        st.mk_check(bufs)
        # both paths against the f32 reference math: the persistent path rounds the
        # normalised rows to the model dtype (as the reference's Linear sees them), the
        # per-launch path keeps them f32, so their errors differ in the last bits only
        err = float((out - gold).norm() / gold.norm())
        err_l = float((ref - gold).norm() / gold.norm())
        assert err < 2e-2 and err <= 2 * err_l + 1e-3, \
            f"{name} pos {pos}: relative error {err:.3e} (per-launch path {err_l:.3e})"
        # the K/V rows of this position (written by the QKV epilogue, bf16)
        torch.testing.assert_close(kv.k[:, :, pos].float(), kref.float(), atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(kv.v[:, :, pos].float(), vref.float(), atol=3e-2, rtol=2e-2)


def test_mk_graph_replays_and_epochs(cuda):
    """Graph-captured persistent steps replayed back to back: the launch epoch advances
    per replay, every replay's output matches an eager per-launch step."""
    cfg = preset("llama3-8b", **CFGS["small"])
    st = _stack(cfg, 512, seed=2)
    layers = list(range(cfg.num_hidden_layers))
    bufs = st.decode_buffers()
    g = torch.Generator(device="cuda:0").manual_seed(5)
    resid0 = torch.randn(cfg.hidden_size, device="cuda:0", generator=g)
    # eager reference trajectory over 6 positions (per-launch path)
    refs = []
    x = resid0.clone()
    for pos in range(6):
        x = _step(st, bufs, layers, x, pos, False)
        refs.append(x)
    st.reset()
    st.use_mk = True
    bufs.resid.copy_(resid0)
    bufs.pos.fill_(0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        st.decode_step(bufs, layers)  # warm (position 0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    torch.testing.assert_close(bufs.resid, refs[0], atol=1e-2, rtol=1e-2)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        st.decode_step(bufs, layers)
    epoch0 = int(bufs.mk_ctl[0])
    for pos in range(1, 6):
        bufs.pos.fill_(pos)
        graph.replay()
        torch.cuda.synchronize()
        err = (bufs.resid - refs[pos]).norm() / refs[pos].norm()
        assert err < 1e-2, f"replay at {pos}: {err:.3e}"
    st.mk_check(bufs)
    assert int(bufs.mk_ctl[0]) == epoch0 + 5
