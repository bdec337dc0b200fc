"""Numerics of the gfx950 HIP kernels vs the plain-PyTorch f32 reference."""
import math

import pytest
import torch

from cake_amd.ops import reference as R

pytestmark = pytest.mark.gpu

DTYPES = [torch.bfloat16, torch.float16]


def _tol(dt):
    return dict(atol=3e-2, rtol=3e-2) if dt == torch.bfloat16 else dict(atol=1e-2, rtol=1e-2)


def _rand(*shape, dt=torch.float32, std=1.0, dev="cuda"):
    return (torch.randn(*shape, device=dev) * std).to(dt)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("K,N", [(4096, 4096), (256, 6), (1024, 14336 // 4), (14336, 512)])
def test_gemv_accumulate(cuda, dt, K, N):
    from cake_amd.ops import hip as K_
    torch.manual_seed(0)
    x = _rand(K, dt=dt)
    w = _rand(N, K, dt=dt, std=0.02)
    out = torch.randn(N, device=cuda)
    ref = out + (w.float() @ x.float())
    K_.gemv(x, w, out, accumulate=True)
    torch.testing.assert_close(out, ref, atol=2e-3 * math.sqrt(K / 256), rtol=1e-3)
    out2 = torch.empty(N, device=cuda)
    K_.gemv(x, w, out2, accumulate=False)
    torch.testing.assert_close(out2, w.float() @ x.float(), atol=2e-3 * math.sqrt(K / 256), rtol=1e-3)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("K,N", [(4096, 128256), (256, 512), (512, 7)])
def test_norm_gemv_f32(cuda, dt, K, N):
    from cake_amd.ops import hip as K_
    torch.manual_seed(1)
    resid = torch.randn(K, device=cuda) * 3
    nw = (1 + 0.1 * torch.randn(K, device=cuda)).to(dt)
    w = _rand(N, K, dt=dt, std=0.02)
    out = torch.empty(N, device=cuda)
    K_.norm_gemv_f32(resid, nw, 1e-5, w, out)
    ref = w.float() @ R.rms_norm(resid, nw, 1e-5)
    torch.testing.assert_close(out, ref, atol=3e-3, rtol=1e-3)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("K,I", [(4096, 14336), (256, 512)])
def test_swiglu(cuda, dt, K, I):
    from cake_amd.ops import hip as K_
    torch.manual_seed(2)
    resid = torch.randn(K, device=cuda)
    nw = (1 + 0.1 * torch.randn(K, device=cuda)).to(dt)
    wg = _rand(I, K, dt=dt, std=0.05)
    wu = _rand(I, K, dt=dt, std=0.05)
    act = torch.empty(I, device=cuda, dtype=dt)
    K_.swiglu(resid, nw, 1e-5, wg, wu, act)
    x = R.rms_norm(resid, nw, 1e-5)
    ref = R.silu_mul(wg.float() @ x, wu.float() @ x)
    torch.testing.assert_close(act.float(), ref, **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("H,nh,nkv,hd,pos", [(4096, 32, 8, 128, 0), (4096, 32, 8, 128, 777),
                                             (256, 4, 1, 64, 5), (1024, 8, 8, 128, 4095)])
def test_qkv_rope(cuda, dt, H, nh, nkv, hd, pos):
    from cake_amd.ops import hip as K_
    torch.manual_seed(3)
    S = 4096
    resid = torch.randn(H, device=cuda)
    nw = (1 + 0.1 * torch.randn(H, device=cuda)).to(dt)
    wq, wk, wv = (_rand(n * hd, H, dt=dt, std=0.05) for n in (nh, nkv, nkv))
    invf = R.inv_freq(hd, 500000.0).to(cuda)
    kc = torch.zeros(nkv, S, hd, device=cuda, dtype=dt)
    vc = torch.zeros_like(kc)
    q = torch.empty(nh * hd, device=cuda)
    p = torch.tensor([pos], dtype=torch.int32, device=cuda)
    K_.qkv_rope(resid, nw, 1e-5, wq, wk, wv, invf, p, q, kc, vc)
    x = R.rms_norm(resid, nw, 1e-5)
    posv = torch.tensor([pos], device=cuda)
    qr = R.rope((wq.float() @ x).view(1, nh, hd), posv, invf).view(-1)
    kr = R.rope((wk.float() @ x).view(1, nkv, hd), posv, invf).view(nkv, hd)
    vr = (wv.float() @ x).view(nkv, hd)
    torch.testing.assert_close(q, qr, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(kc[:, pos].float(), kr, **_tol(dt))
    torch.testing.assert_close(vc[:, pos].float(), vr, **_tol(dt))
    assert kc[:, :pos].abs().sum() == 0 and kc[:, pos + 1:].abs().sum() == 0


@pytest.fixture(params=[(1, 320), (2, 320), (2, 0)], ids=["core1", "core2", "core2-split"])
def attn_impl(request, cuda):
    """Both decode-attention cores (attn_core.h chunks / attn_core2.h wave-stream MFMA);
    core 2 also with its one-split range off, so short contexts take the split + merge
    path too."""
    from cake_amd.ops import hip as K_
    impl, single = request.param
    prev, prev_single = K_._ATTN_IMPL[0], K_._ATTN_SINGLE[0]
    K_.attn_set_impl(impl)
    K_.attn_set_single_max(single)
    yield impl
    K_.attn_set_impl(prev)
    K_.attn_set_single_max(prev_single)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("nh,nkv,hd,pos,S", [(32, 8, 128, 0, 2048), (32, 8, 128, 63, 2048),
                                             (32, 8, 128, 64, 2048), (32, 8, 128, 1000, 2048),
                                             (32, 8, 128, 2047, 2048), (64, 8, 128, 300, 2048),
                                             (4, 1, 64, 17, 2048), (8, 8, 64, 200, 2048),
                                             (16, 4, 128, 70, 100), (32, 8, 128, 8190, 8192)])
@pytest.mark.parametrize("min_keys", [64, 256])
def test_attn_decode(cuda, attn_impl, dt, nh, nkv, hd, pos, S, min_keys):
    """Split-K decode attention (split count derived on device from pos) vs f32 attention;
    S not a multiple of 64, more than 64 splits' worth of keys (S = 8192: 128-key splits)."""
    from cake_amd.ops import hip as K_
    torch.manual_seed(4)
    kc = _rand(nkv, S, hd, dt=dt)
    vc = _rand(nkv, S, hd, dt=dt)
    q = torch.randn(nh * hd, device=cuda)
    p = torch.tensor([pos], dtype=torch.int32, device=cuda)
    part = torch.zeros(K_.attn_workspace_numel(nh, hd, S), device=cuda)
    out = torch.empty(nh * hd, device=cuda, dtype=dt)
    tickets = torch.zeros(2 * nkv + 2, dtype=torch.int32, device=cuda)
    K_.attn_set_min_keys(min_keys)
    try:
        # the first call (another q) leaves its partials behind: the second must not
        # merge them (core 1: tickets re-armed; core 2: epoch-tagged granules)
        for it in range(2):
            out.zero_()
            K_.attn_decode(q if it else torch.randn_like(q), kc, vc, p, 1 / math.sqrt(hd), part,
                           tickets, out)
            assert int(tickets[:nkv].abs().sum()) == 0
    finally:
        K_.attn_set_min_keys(64)
    Tk = pos + 1
    ref = R.attention(q.view(1, nh, hd), kc[:, :Tk].transpose(0, 1), vc[:, :Tk].transpose(0, 1),
                      pos).reshape(-1)
    torch.testing.assert_close(out.float(), ref, **_tol(dt))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nh,nkv,hd", [(32, 8, 128), (16, 16, 64), (8, 1, 128)])
@pytest.mark.parametrize("pos", [0, 15, 16, 70, 127, 600])
@pytest.mark.parametrize("waves,prefetch", [(1, 2), (2, 2), (4, 2), (8, 2), (16, 2), (4, 4),
                                            (16, 4)])
def test_attn_decode_heads(cuda, dt, nh, nkv, hd, pos, waves, prefetch):
    """Head-parallel short-context attention (one workgroup per query head, one split)
    vs f32 attention: block edges (16 / 17 keys), a ragged tail, and a long context it is
    still correct for (601 keys walked by one workgroup)."""
    from cake_amd.ops import hip as K_
    torch.manual_seed(5)
    S = 1000
    kc = _rand(nkv, S, hd, dt=dt)
    vc = _rand(nkv, S, hd, dt=dt)
    q = torch.randn(nh * hd, device=cuda)
    p = torch.tensor([pos], dtype=torch.int32, device=cuda)
    out = torch.full((nh * hd,), float("nan"), device=cuda, dtype=dt)
    K_.attn_decode_heads(q, kc, vc, p, 1 / math.sqrt(hd), out, waves=waves, prefetch=prefetch)
    Tk = pos + 1
    ref = R.attention(q.view(1, nh, hd), kc[:, :Tk].transpose(0, 1), vc[:, :Tk].transpose(0, 1),
                      pos).reshape(-1)
    torch.testing.assert_close(out.float(), ref, **_tol(dt))


def test_attn_decode_merge_timeout_raises(cuda):
    """Core 2's split 0 spins on the other splits' partials: if they never arrive, the
    bounded poll must end the launch and raise the error word (not merge stale partials
    silently)."""
    from cake_amd.ops import hip as K_
    nh, nkv, hd, S, pos = 32, 8, 128, 2048, 1500  # > 320 keys: several splits
    kc = _rand(nkv, S, hd, dt=torch.bfloat16)
    vc = _rand(nkv, S, hd, dt=torch.bfloat16)
    q = torch.randn(nh * hd, device=cuda)
    p = torch.tensor([pos], dtype=torch.int32, device=cuda)
    part = torch.zeros(K_.attn_workspace_numel(nh, hd, S), device=cuda)
    out = torch.empty(nh * hd, device=cuda, dtype=torch.bfloat16)
    tickets = torch.zeros(2 * nkv + 2, dtype=torch.int32, device=cuda)
    K_.attn_set_impl(2)
    K_.attn_decode(q, kc, vc, p, 1 / math.sqrt(hd), part, tickets, out)
    assert not K_.attn_error(tickets)
    K_.attn_debug_drop_partials(True)
    try:
        K_.attn_decode(q, kc, vc, p, 1 / math.sqrt(hd), part, tickets, out)
        torch.cuda.synchronize()
    finally:
        K_.attn_debug_drop_partials(False)
    assert K_.attn_error(tickets)


def test_wave_reductions(cuda):
    """DPP / permlane-swap wave reductions (common.h) against torch, every lane."""
    from cake_amd.ops._lib import check, kernels
    torch.manual_seed(8)
    x = torch.randn(64, device=cuda)
    out = torch.empty(320, device=cuda)
    check(kernels().cake_wave_reduce_probe(x.data_ptr(), out.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream), "probe")
    torch.cuda.synchronize()
    idx = torch.arange(64, device=cuda)
    torch.testing.assert_close(out[:64], x.sum().expand(64), atol=1e-5, rtol=1e-5)
    assert torch.equal(out[64:128], x.max().expand(64))
    assert out[:64].unique().numel() == 1  # identical bits in every lane
    for k, off in enumerate((8, 16, 32)):
        torch.testing.assert_close(out[128 + 64 * k:192 + 64 * k], x + x[idx ^ off])


@pytest.mark.parametrize("pos", [0, 5, 63, 64, 130])
def test_attn_decode_dead_rows_nan(cuda, attn_impl, pos):
    """Cache rows past the live length hold NaN: split 0 loads its first chunk before
    the length is known, so those rows must never reach the output."""
    from cake_amd.ops import hip as K_
    torch.manual_seed(5)
    nh, nkv, hd, S = 32, 8, 128, 512
    kc = _rand(nkv, S, hd, dt=torch.bfloat16)
    vc = _rand(nkv, S, hd, dt=torch.bfloat16)
    kc[:, pos + 1:] = float("nan")
    vc[:, pos + 1:] = float("nan")
    q = torch.randn(nh * hd, device=cuda)
    p = torch.tensor([pos], dtype=torch.int32, device=cuda)
    part = torch.zeros(K_.attn_workspace_numel(nh, hd, S), device=cuda)
    out = torch.empty(nh * hd, device=cuda, dtype=torch.bfloat16)
    tickets = torch.zeros(2 * nkv + 2, dtype=torch.int32, device=cuda)
    K_.attn_decode(q, kc, vc, p, 1 / math.sqrt(hd), part, tickets, out)
    Tk = pos + 1
    ref = R.attention(q.view(1, nh, hd), kc[:, :Tk].transpose(0, 1), vc[:, :Tk].transpose(0, 1),
                      pos).reshape(-1)
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.float(), ref, **_tol(torch.bfloat16))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("T,pos0,nh,nkv,hd", [(7, 0, 32, 8, 128), (70, 0, 4, 1, 64),
                                              (33, 100, 32, 8, 128), (1, 5, 8, 8, 64)])
def test_rope_kv_and_prefill_attention(cuda, dt, T, pos0, nh, nkv, hd):
    from cake_amd.ops import hip as K_
    torch.manual_seed(5)
    S = 512
    kc = _rand(nkv, S, hd, dt=dt)
    vc = _rand(nkv, S, hd, dt=dt)
    q = _rand(T, nh * hd, dt=dt)
    k = _rand(T, nkv * hd, dt=dt)
    v = _rand(T, nkv * hd, dt=dt)
    invf = R.inv_freq(hd, 500000.0).to(cuda)
    positions = torch.arange(pos0, pos0 + T, device=cuda)
    qr = R.rope(q.view(T, nh, hd), positions, invf)
    kr = R.rope(k.view(T, nkv, hd), positions, invf)
    q_in = q.clone()
    K_.rope_kv(q_in, k, v, invf, pos0, kc, vc)
    torch.testing.assert_close(q_in.float().view(T, nh, hd), qr, **_tol(dt))
    torch.testing.assert_close(kc[:, pos0:pos0 + T].float().transpose(0, 1), kr, **_tol(dt))
    torch.testing.assert_close(vc[:, pos0:pos0 + T].transpose(0, 1).reshape(T, -1), v)
    out = torch.empty_like(q_in)
    Tk = pos0 + T
    K_.flash_attn(q_in.view(1, T, nh, hd).transpose(1, 2), kc[None, :, :Tk], vc[None, :, :Tk],
                  out.view(1, T, nh, hd).transpose(1, 2), 1 / math.sqrt(hd), causal=True, pos0=pos0)
    ref = R.attention(q_in.view(T, nh, hd), kc[:, :Tk].transpose(0, 1), vc[:, :Tk].transpose(0, 1),
                      pos0)
    torch.testing.assert_close(out.float().view(T, nh, hd), ref, **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
def test_embed_rmsnorm_silu_add(cuda, dt):
    from cake_amd.ops import hip as K_
    torch.manual_seed(6)
    V, H, T = 1000, 4096, 5
    table = _rand(V, H, dt=dt)
    tok = torch.tensor([3, 999, 0, 17, 3], dtype=torch.int32, device=cuda)
    out = torch.empty(T, H, device=cuda)
    K_.embed(table, tok, out)
    torch.testing.assert_close(out, table[tok.long()].float())
    w = (1 + 0.1 * torch.randn(H, device=cuda)).to(dt)
    xn = torch.empty(T, H, device=cuda, dtype=dt)
    K_.rmsnorm(out, w, 1e-5, xn)
    torch.testing.assert_close(xn.float(), R.rms_norm(out, w, 1e-5), **_tol(dt))
    g, u = _rand(T, 300, dt=dt), _rand(T, 300, dt=dt)
    act = torch.empty_like(g)
    K_.silu_mul(g, u, act)
    torch.testing.assert_close(act.float(), R.silu_mul(g, u), **_tol(dt))
    resid = torch.randn(T, 300, device=cuda)
    ref = resid + act.float()
    K_.add_resid(resid, act)
    torch.testing.assert_close(resid, ref)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("H", [64, 1004, 2048, 3072, 4096, 5120, 8192, 12288])
@pytest.mark.parametrize("reg", [1, 0])
def test_rmsnorm_widths(cuda, dt, H, reg):
    """Prefill RMSNorm: the register-resident row kernel (H <= 8192, partial last
    vector group) and the two-pass loop kernel, against the f32 reference."""
    from cake_amd.ops import _lib
    from cake_amd.ops import hip as K_
    torch.manual_seed(H)
    T = 37
    x = torch.randn(T, H, device=cuda) * 3
    w = (1 + 0.1 * torch.randn(H, device=cuda)).to(dt)
    out = torch.empty(T, H, device=cuda, dtype=dt)
    lib = _lib.kernels()
    lib.cake_rmsnorm_set_reg(reg)
    try:
        K_.rmsnorm(x, w, 1e-5, out)
    finally:
        lib.cake_rmsnorm_set_reg(1)
    torch.testing.assert_close(out.float(), R.rms_norm(x, w, 1e-5), **_tol(dt))


def test_penalty_argmax_finalize(cuda):
    from cake_amd.ops import hip as K_
    torch.manual_seed(7)
    V = 128256
    logits = torch.randn(V, device=cuda)
    hist_list = [5, 9, 5, 100, 7, 9, 120000]
    hist = torch.zeros(64, dtype=torch.int32, device=cuda)
    hist[:len(hist_list)] = torch.tensor(hist_list, dtype=torch.int32)
    hist_len = torch.tensor([len(hist_list)], dtype=torch.int32, device=cuda)
    logits[9] = 50.0
    logits[5] = -3.0
    ref = R.apply_repeat_penalty(logits, 1.3, hist_list[-4:])
    K_.repeat_penalty(logits, hist, hist_len, 4, 1.3)
    torch.testing.assert_close(logits, ref)
    slot = torch.zeros(1, dtype=torch.int64, device=cuda)
    K_.argmax(logits, slot)
    tok = torch.zeros(1, dtype=torch.int32, device=cuda)
    pos = torch.tensor([10], dtype=torch.int32, device=cuda)
    K_.finalize_token(slot, tok, hist, hist_len, pos)
    expect = int(torch.argmax(ref))
    assert int(tok) == expect
    assert int(hist_len) == len(hist_list) + 1 and int(hist[len(hist_list)]) == expect
    assert int(pos) == 11 and int(slot) == 0
    # ties resolve to the smallest index
    logits.fill_(1.0)
    K_.argmax(logits, slot)
    K_.finalize_token(slot, tok, hist, hist_len, pos)
    assert int(tok) == 0


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("K,N,last_n,penalty", [(4096, 128256, 128, 1.1), (256, 1001, 256, 1.3),
                                                (512, 7, 0, 1.0), (512, 4097, 3, 2.0)])
def test_head_select_matches_four_launches(cuda, dt, K, N, last_n, penalty):
    """Fused lm_head + penalty + argmax + finalize (+ the next step's embedding row) in one
    launch vs norm_gemv_f32 + repeat_penalty + argmax + finalize_token + embed on the same
    inputs; three steps in a row (slot / ticket re-armed by the kernel; the history grows,
    so from step 2 on the previous choice is itself penalised; each step's input is the
    previous step's embedded token)."""
    from cake_amd.ops import hip as K_
    torch.manual_seed(11)
    resid0 = torch.randn(K, device=cuda) * 3
    nw = (1 + 0.1 * torch.randn(K, device=cuda)).to(dt)
    w = _rand(N, K, dt=dt, std=0.02)
    table = _rand(N, K, dt=dt, std=2.0)
    hist0 = torch.randint(0, N, (300,), dtype=torch.int32)
    hist0[:20] = hist0[0]  # repeated tokens: penalised once
    state = []
    for _ in range(2):
        hist = torch.zeros(400, dtype=torch.int32, device=cuda)
        hist[:300] = hist0.to(cuda)
        state.append(dict(hist=hist, hist_len=torch.tensor([300], dtype=torch.int32, device=cuda),
                          tok=torch.zeros(1, dtype=torch.int32, device=cuda),
                          pos=torch.tensor([299], dtype=torch.int32, device=cuda),
                          slot=torch.zeros(1, dtype=torch.int64, device=cuda),
                          ticket=torch.zeros(1, dtype=torch.int32, device=cuda),
                          logits=torch.empty(N, device=cuda), resid=resid0.clone()))
    a, b = state
    ref = w.float() @ R.rms_norm(resid0, nw, 1e-5)
    for step in range(3):
        K_.head_select(a["resid"], nw, 1e-5, w, a["logits"], a["hist"], a["hist_len"], last_n,
                       penalty, a["slot"], a["ticket"], a["tok"], a["pos"],
                       embed=table if step < 2 else None)
        K_.norm_gemv_f32(b["resid"], nw, 1e-5, w, b["logits"])
        if penalty != 1.0:
            K_.repeat_penalty(b["logits"], b["hist"], b["hist_len"], last_n, penalty)
        K_.argmax(b["logits"], b["slot"])
        K_.finalize_token(b["slot"], b["tok"], b["hist"], b["hist_len"], b["pos"])
        if step < 2:
            K_.embed(table, b["tok"], b["resid"])
        torch.cuda.synchronize()
        torch.testing.assert_close(a["logits"], b["logits"])
        for k in ("tok", "pos", "hist_len", "hist", "resid"):
            assert torch.equal(a[k], b[k]), (step, k)
        assert int(a["slot"]) == 0 and int(a["ticket"]) == 0
        if step == 0:  # the first choice against f32 torch math
            if penalty != 1.0 and last_n:
                ref = R.apply_repeat_penalty(ref, penalty, hist0[300 - last_n:].tolist())
            assert abs(float(ref[int(a["tok"])]) - float(ref.max())) <= \
                3e-3 * max(1.0, float(ref.abs().max()))
    # without embed the input row is left alone
    assert torch.equal(a["resid"], b["resid"])


@pytest.mark.parametrize("dt", DTYPES)
def test_rope_kv_fused_qkv_and_silu_mul_rows(cuda, dt):
    """Prefill layouts: q/k/v as column slices of one fused projection; gate|up fused."""
    from cake_amd.ops import hip as K_
    torch.manual_seed(9)
    T, nh, nkv, hd, S, pos0 = 37, 32, 8, 128, 256, 11
    qkv = _rand(T, (nh + 2 * nkv) * hd, dt=dt)
    nq, nk = nh * hd, nkv * hd
    q, k, v = qkv[:, :nq], qkv[:, nq:nq + nk], qkv[:, nq + nk:]
    kc = torch.zeros(nkv, S, hd, device=cuda, dtype=dt)
    vc = torch.zeros_like(kc)
    invf = R.inv_freq(hd, 500000.0).to(cuda)
    positions = torch.arange(pos0, pos0 + T, device=cuda)
    qr = R.rope(q.reshape(T, nh, hd), positions, invf)
    kr = R.rope(k.reshape(T, nkv, hd), positions, invf)
    v_ref = v.clone()
    K_.rope_kv(q, k, v, invf, pos0, kc, vc)
    torch.testing.assert_close(q.float().reshape(T, nh, hd), qr, **_tol(dt))
    torch.testing.assert_close(kc[:, pos0:pos0 + T].float().transpose(0, 1), kr, **_tol(dt))
    torch.testing.assert_close(vc[:, pos0:pos0 + T].transpose(0, 1).reshape(T, -1), v_ref)
    I = 1024
    gu = _rand(T, 2 * I, dt=dt)
    act = torch.empty(T, I, device=cuda, dtype=dt)
    K_.silu_mul_rows(gu, act)
    ref = torch.nn.functional.silu(gu[:, :I].float()) * gu[:, I:].float()
    torch.testing.assert_close(act.float(), ref, **_tol(dt))

GEMV_DEFAULTS = {"qkv": (2, 4, 1024), "swiglu": (2, 4, 512), "x16": (4, 4, 1024),
                 "norm_f32": (4, 4, 256), "x16s": (4, 4, 1024)}


@pytest.fixture
def gemv_tuning():
    from cake_amd.ops import hip as K_
    yield K_
    for kind, (u, pf, mb) in GEMV_DEFAULTS.items():
        K_.set_gemv_tuning(kind, U=u, prefetch=pf, max_blocks=mb)


@pytest.mark.parametrize("U,pf", [(2, 4), (4, 4), (8, 8), (4, 8)])
@pytest.mark.parametrize("mb", [3, 1024])
def test_gemv_split_prologue(cuda, gemv_tuning, U, pf, mb):
    """Weight prefetch with the split x prologue (x loads, then weights, then the norm /
    staging): the model K values (4096 RMSNorm rows; 4096 / 14336 16-bit rows), idle
    waves (N < waves) and many pairs per wave (grid cap 3)."""
    K_ = gemv_tuning
    for kind in GEMV_DEFAULTS:
        K_.set_gemv_tuning(kind, U=U, prefetch=pf, max_blocks=mb)
    torch.manual_seed(8)
    dt = torch.bfloat16
    # TP shard K values too: 3584 / 2048 take guarded split prologues, 1792 the plain one
    for Kd, N in [(4096, 4096), (14336, 1030), (4096, 6), (3584, 257), (2048, 100), (1792, 64)]:
        x = _rand(Kd, dt=dt)
        w = _rand(N, Kd, dt=dt, std=0.02)
        out = torch.randn(N, device=cuda)
        ref = out + (w.float() @ x.float())
        K_.gemv(x, w, out, accumulate=True)
        torch.testing.assert_close(out, ref, atol=2e-3 * math.sqrt(Kd / 256), rtol=1e-3)
    r3 = torch.randn(3072, device=cuda)
    n3 = (1 + 0.1 * torch.randn(3072, device=cuda)).to(dt)
    w3 = _rand(999, 3072, dt=dt, std=0.02)
    o3 = torch.empty(999, device=cuda)
    K_.norm_gemv_f32(r3, n3, 1e-5, w3, o3)
    torch.testing.assert_close(o3, w3.float() @ R.rms_norm(r3, n3, 1e-5), atol=3e-3, rtol=1e-3)
    resid = torch.randn(4096, device=cuda)
    nw = (1 + 0.1 * torch.randn(4096, device=cuda)).to(dt)
    xn = R.rms_norm(resid, nw, 1e-5)
    w = _rand(3001, 4096, dt=dt, std=0.02)
    out = torch.empty(3001, device=cuda)
    K_.norm_gemv_f32(resid, nw, 1e-5, w, out)
    torch.testing.assert_close(out, w.float() @ xn, atol=3e-3, rtol=1e-3)
    wg, wu = _rand(1000, 4096, dt=dt, std=0.05), _rand(1000, 4096, dt=dt, std=0.05)
    act = torch.empty(1000, device=cuda, dtype=dt)
    K_.swiglu(resid, nw, 1e-5, wg, wu, act)
    torch.testing.assert_close(act.float(), R.silu_mul(wg.float() @ xn, wu.float() @ xn), **_tol(dt))
    nh, nkv, hd, pos = 32, 8, 128, 77
    wq, wk, wv = (_rand(n * hd, 4096, dt=dt, std=0.05) for n in (nh, nkv, nkv))
    invf = R.inv_freq(hd, 500000.0).to(cuda)
    kc = torch.zeros(nkv, 128, hd, device=cuda, dtype=dt)
    vc = torch.zeros_like(kc)
    q = torch.empty(nh * hd, device=cuda)
    K_.qkv_rope(resid, nw, 1e-5, wq, wk, wv, invf, torch.tensor([pos], dtype=torch.int32,
                device=cuda), q, kc, vc)
    posv = torch.tensor([pos], device=cuda)
    torch.testing.assert_close(q, R.rope((wq.float() @ xn).view(1, nh, hd), posv, invf).view(-1),
                               atol=2e-3, rtol=2e-3)
    kr = R.rope((wk.float() @ xn).view(1, nkv, hd), posv, invf).view(nkv, hd)
    torch.testing.assert_close(kc[:, pos].float(), kr, **_tol(dt))
    torch.testing.assert_close(vc[:, pos].float(), (wv.float() @ xn).view(nkv, hd), **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("H,nh,nkv,hd", [(4096, 32, 8, 128), (8192, 64, 8, 128), (512, 8, 2, 64),
                                         (256, 4, 2, 64), (1024, 8, 8, 128), (512, 4, 1, 128)])
def test_attn_oproj_fused(cuda, dt, H, nh, nkv, hd):
    """Decode attention + o_proj as one launch (attn_oproj.hip) vs the two launches it
    replaces (attn_decode, then the o_proj GEMV) and vs the f32 reference, over the
    one-split lengths it serves, accumulating into the residual and plain (tensor-parallel
    partial); back to back, so the row-block tickets must re-arm."""
    from cake_amd.ops import hip as K_
    if not hasattr(K_.kernels(), "cake_attn_oproj"):
        pytest.skip("fused attention + o_proj not built (csrc/experimental: "
                    "CAKE_BUILD_EXPERIMENTAL=1)")
    assert K_.attn_oproj_supported(nh, nkv, hd, H)
    torch.manual_seed(11)
    S = 512
    kc = _rand(nkv, S, hd, dt=dt)
    vc = _rand(nkv, S, hd, dt=dt)
    wo = _rand(H, nh * hd, dt=dt, std=(nh * hd) ** -0.5)
    q = _rand(nh * hd)
    nws, ntk = K_.attn_oproj_ws_sizes(nkv, H)
    ws = torch.zeros(nws, device=cuda)
    tk = torch.zeros(ntk, dtype=torch.int32, device=cuda)
    part = torch.zeros(K_.attn_workspace_numel(nh, hd, S), device=cuda)
    tickets = torch.zeros(2 * nkv + 2, dtype=torch.int32, device=cuda)
    attn = torch.empty(nh * hd, device=cuda, dtype=dt)
    scale = 1 / math.sqrt(hd)
    for pos in (0, 1, 15, 16, 63, 200, 318):
        p = torch.tensor([pos], dtype=torch.int32, device=cuda)
        base = torch.randn(H, device=cuda)
        # two launches
        K_.attn_decode(q, kc, vc, p, scale, part, tickets, attn)
        want = base.clone()
        K_.gemv(attn, wo, want, accumulate=True)
        # fused, accumulating
        got = base.clone()
        K_.attn_oproj(q, kc, vc, p, scale, wo, got, True, ws, tk)
        # fused, plain (out = W_o . attn)
        plain = torch.full((H,), float("nan"), device=cuda)
        K_.attn_oproj(q, kc, vc, p, scale, wo, plain, False, ws, tk)
        torch.cuda.synchronize()
        rb = 32 if nh // nkv == 8 else 64  # row block (attn_oproj.hip ao_rows)
        assert int(tk[:H // rb].abs().sum()) == 0, "row-block tickets not re-armed"
        torch.testing.assert_close(got, want, atol=2e-3, rtol=2e-3)
        torch.testing.assert_close(plain, want - base, atol=2e-3, rtol=2e-3)
        # f32 reference (16-bit attention output, as both paths round it)
        Tk = pos + 1
        ref = R.attention(q.view(1, nh, hd), kc[:, :Tk].transpose(0, 1).float(),
                          vc[:, :Tk].transpose(0, 1).float(), pos).reshape(-1)
        ref_out = base + wo.float() @ ref.to(dt).float()
        err = (got - ref_out).abs().max().item()
        assert err <= 2e-2 * max(1.0, ref_out.abs().max().item()), err
