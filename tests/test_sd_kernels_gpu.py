"""MFMA flash attention + SD normalisation kernels vs PyTorch f32 references."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DTYPES = [torch.bfloat16, torch.float16]


def _tol(dt):
    return dict(atol=2e-2, rtol=2e-2) if dt == torch.bfloat16 else dict(atol=5e-3, rtol=5e-3)


def _ref_attn(q, k, v, scale, causal, pos0):
    B, H, N, D = q.shape
    Hkv, M = k.shape[1], k.shape[2]
    kk = k.float().repeat_interleave(H // Hkv, dim=1)
    vv = v.float().repeat_interleave(H // Hkv, dim=1)
    s = (q.float() @ kk.transpose(-1, -2)) * scale
    if causal:
        qi = torch.arange(N, device=q.device)[:, None] + pos0
        kj = torch.arange(M, device=q.device)[None, :]
        s = s.masked_fill(kj > qi, float("-inf"))
    return torch.softmax(s, -1) @ vv


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,H,Hkv,N,M,D,causal,pos0", [
    (2, 8, 8, 4096 // 4, 1024, 40, False, 0),    # SD1.5 self-attn (smaller N)
    (2, 8, 8, 1024, 77, 40, False, 0),           # SD cross-attn, 77 context tokens
    (2, 10, 10, 300, 300, 64, False, 0),         # SDXL head_dim 64, ragged N
    (1, 5, 5, 200, 77, 80, False, 0),            # head_dim 80 (padded to 96)
    (1, 2, 2, 100, 100, 160, False, 0),          # head_dim 160
    (1, 32, 8, 77, 77, 128, True, 0),            # Llama prefill, GQA 4:1
    (1, 32, 8, 50, 150, 128, True, 100),         # chunked prefill (offset causal)
    (1, 12, 12, 77, 77, 64, True, 0),            # CLIP causal
    (2, 16, 16, 4096, 256, 64, False, 0),        # large grid: 4-wave workgroups, DP 64
    (1, 32, 8, 2048, 2048, 128, True, 0),        # large grid: 4-wave workgroups, DP 128
])
@pytest.mark.parametrize("impl", [1, 2])
def test_flash_attn(cuda, dt, B, H, Hkv, N, M, D, causal, pos0, impl):
    from cake_amd.ops import hip as K
    torch.manual_seed(0)
    # projection-style layouts: [B, rows, heads, D] viewed as [B, heads, rows, D]
    q = torch.randn(B, N, H, D, device=cuda).to(dt).transpose(1, 2)
    k = torch.randn(B, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    v = torch.randn(B, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    out = torch.empty(B, N, H, D, device=cuda, dtype=dt).transpose(1, 2)
    scale = 1 / math.sqrt(D)
    K.flash_set_impl(impl)
    try:
        K.flash_attn(q, k, v, out, scale, causal, pos0)
    finally:
        K.flash_set_impl(2)
    torch.testing.assert_close(out.float(), _ref_attn(q, k, v, scale, causal, pos0), **_tol(dt))


@pytest.mark.parametrize("N,pos0,D", [(1400, 0, 128), (2048, 0, 64), (300, 37, 128),
                                       (128, 0, 128)])
@pytest.mark.parametrize("pair_min", [1, 0])
def test_flash_causal_pairing(cuda, N, pos0, D, pair_min):
    """Causal q-tile pairing (workgroup x runs tiles x and n-1-x; odd tile counts leave
    one unpaired middle tile) forced on / off gives the reference result."""
    from cake_amd.ops import hip as K
    torch.manual_seed(1)
    dt, H, Hkv = torch.bfloat16, 8, 2
    M = N + pos0
    q = torch.randn(1, N, H, D, device=cuda).to(dt).transpose(1, 2)
    k = torch.randn(1, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    v = torch.randn(1, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    out = torch.full((1, N, H, D), float("nan"), device=cuda, dtype=dt).transpose(1, 2)
    K.flash_set_pair_min(pair_min)
    try:
        K.flash_attn(q, k, v, out, 1 / math.sqrt(D), True, pos0)
    finally:
        K.flash_set_pair_min(512)
    torch.testing.assert_close(out.float(), _ref_attn(q, k, v, 1 / math.sqrt(D), True, pos0),
                               **_tol(dt))


@pytest.mark.parametrize("ksplit", [0, 2, 4])
@pytest.mark.parametrize("B,H,N,M,D", [(2, 20, 1024, 1024, 64), (1, 3, 200, 1000, 64),
                                       (2, 4, 77, 600, 128), (1, 2, 64, 513, 40)])
def test_flash_key_split(cuda, ksplit, B, H, N, M, D):
    """Non-causal key split (f32 partial rows per split + the merge launch), forced to 2 / 4
    splits and automatic (SDXL's 1024-token self-attention splits by itself), including
    ragged key counts whose last split is short; a spike in the second half makes the
    splits' maxima differ."""
    from cake_amd.ops import hip as K
    torch.manual_seed(5)
    dt = torch.bfloat16
    q = torch.randn(B, N, H, D, device=cuda).to(dt).transpose(1, 2)
    k = torch.randn(B, M, H, D, device=cuda)
    k[:, M - 3, :, :] = q[:, :, 1, :].float() * 3  # row 1: its mass sits in the last split
    k = k.to(dt).transpose(1, 2)
    v = torch.randn(B, M, H, D, device=cuda).to(dt).transpose(1, 2)
    out = torch.full((B, N, H, D), float("nan"), device=cuda, dtype=dt).transpose(1, 2)
    K.flash_set_ksplit(ksplit)
    try:
        K.flash_attn(q, k, v, out, 1 / math.sqrt(D))
    finally:
        K.flash_set_ksplit(0)
    torch.testing.assert_close(out.float(), _ref_attn(q, k, v, 1 / math.sqrt(D), False, 0),
                               **_tol(dt))


@pytest.mark.parametrize("ksplit", [2, 4])
@pytest.mark.parametrize("pair_min", [1, 0])
@pytest.mark.parametrize("N,pos0", [(700, 0), (300, 90)])
def test_flash_causal_forced_key_split(cuda, ksplit, pair_min, N, pos0):
    """The forced causal key split (measured slower, kept opt-in): splits wholly past a
    row's position write empty partials the merge skips; paired and unpaired tiles."""
    import ctypes

    from cake_amd.ops import hip as K
    torch.manual_seed(9)
    dt, H, Hkv, D = torch.bfloat16, 8, 2, 128
    M = N + pos0
    q = torch.randn(1, N, H, D, device=cuda).to(dt).transpose(1, 2)
    k = torch.randn(1, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    v = torch.randn(1, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    out = torch.full((1, N, H, D), float("nan"), device=cuda, dtype=dt).transpose(1, 2)
    ws = torch.empty(4 * H * N * (D + 1), device=cuda)
    st = [x for t in (q, k, v, out) for x in t.stride()[:3]]
    arr = (ctypes.c_longlong * 12)(*st)
    lib = K.kernels()
    K.flash_set_pair_min(pair_min)
    lib.cake_flash_set_ksplit(ksplit)
    try:
        K.check(lib.cake_flash_attn_ws(0, K._p(q), K._p(k), K._p(v), K._p(out), 1, H, Hkv, N, M,
                                       D, ctypes.cast(arr, ctypes.c_void_p), 1 / math.sqrt(D), 1,
                                       pos0, K._p(ws), ws.numel() * 4, K._stream()), "flash")
        torch.cuda.synchronize()
    finally:
        K.flash_set_pair_min(512)
        lib.cake_flash_set_ksplit(0)
    torch.testing.assert_close(out.float(), _ref_attn(q, k, v, 1 / math.sqrt(D), True, pos0),
                               **_tol(dt))


@pytest.mark.parametrize("impl", [1, 2])
def test_flash_attn_softmax_rescale_branch(cuda, impl):
    """A late key tile with a much larger score forces the online-softmax rescale."""
    from cake_amd.ops import hip as K
    K.flash_set_impl(impl)
    dt = torch.bfloat16
    q = torch.randn(1, 1, 64, 64, device=cuda).to(dt)
    k = torch.randn(1, 1, 256, 64, device=cuda)
    k[0, 0, 200] = q[0, 0, 5].float() * 4  # spike for row 5 in tile 3
    k = k.to(dt)
    v = torch.randn(1, 1, 256, 64, device=cuda).to(dt)
    out = torch.empty_like(q)
    K.flash_attn(q, k, v, out, 0.125)
    K.flash_set_impl(2)
    torch.testing.assert_close(out.float(), _ref_attn(q, k, v, 0.125, False, 0), **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("shape,G,silu", [((2, 320, 64, 64), 32, True), ((1, 512, 32, 32), 32, False),
                                          ((2, 1280, 8, 8), 32, True), ((1, 96, 5, 7), 32, False)])
def test_group_norm(cuda, dt, shape, G, silu):
    from cake_amd.ops import hip as K
    torch.manual_seed(1)
    x = (torch.randn(shape, device=cuda) * 3 + 1).to(dt)
    g = (1 + 0.1 * torch.randn(shape[1], device=cuda)).to(dt)
    b = (0.1 * torch.randn(shape[1], device=cuda)).to(dt)
    y = torch.empty_like(x)
    K.group_norm(x, g, b, G, 1e-5, silu, y)
    ref = torch.nn.functional.group_norm(x.float(), G, g.float(), b.float(), 1e-5)
    if silu:
        ref = torch.nn.functional.silu(ref)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("C", [768, 320, 1280, 2048, 100])  # wave kernel (1/2/4 chunks), fallback
def test_layer_norm_and_geglu(cuda, dt, C):
    from cake_amd.ops import hip as K
    torch.manual_seed(2)
    x = (torch.randn(2, 77, C, device=cuda) * 2 + 3).to(dt)
    g = (1 + 0.1 * torch.randn(C, device=cuda)).to(dt)
    b = (0.1 * torch.randn(C, device=cuda)).to(dt)
    y = torch.empty_like(x)
    K.layer_norm(x, g, b, 1e-5, y)
    ref = torch.nn.functional.layer_norm(x.float(), (C,), g.float(), b.float(), 1e-5)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))
    h = torch.randn(2, 50, 2 * C, device=cuda).to(dt)
    o = torch.empty(2, 50, C, device=cuda, dtype=dt)
    K.geglu(h, o)
    a, gate = h.float().chunk(2, -1)
    torch.testing.assert_close(o.float(), a * torch.nn.functional.gelu(gate, approximate="tanh"),
                               **_tol(dt))


def _ref_conv(x, w, b, stride, pad, up, bias2=None, resid=None):
    """x NHWC, w [OC,IC,KH,KW] -> NHWC, f32."""
    xc = x.float().permute(0, 3, 1, 2)
    if up:
        xc = torch.nn.functional.interpolate(xc, scale_factor=2.0, mode="nearest")
    y = torch.nn.functional.conv2d(xc, w.float(), None if b is None else b.float(), stride=stride,
                                   padding=pad).permute(0, 2, 3, 1)
    if bias2 is not None:
        y = y + bias2[:, None, None, :]
    if resid is not None:
        y = y + resid.float()
    return y


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,H,W,IC,OC,k,stride,up", [
    (2, 16, 16, 64, 128, 3, 1, False),
    (2, 9, 7, 128, 320, 3, 1, False),    # ragged pixels, OC not a tile multiple
    (1, 16, 16, 64, 64, 3, 2, False),    # downsampler (stride 2)
    (1, 15, 17, 64, 64, 3, 2, False),    # stride 2, odd sizes
    (2, 8, 8, 64, 128, 3, 1, True),      # upsampler (nearest 2x fused)
    (2, 12, 12, 192, 64, 1, 1, False),   # 1x1 shortcut
    (1, 8, 8, 320, 4, 3, 1, False),      # conv_out-like OC=4
])
@pytest.mark.parametrize("cfg,splits", [(None, None), (0, 1), (3, 1), (1, 3), (2, 2),
                                        (4, 1), (5, 2), (6, 1), (7, 3),
                                        (8, 1), (9, 1), (10, 1), (11, 1), (12, 1), (13, 1)])
def test_conv2d_nhwc(cuda, dt, N, H, W, IC, OC, k, stride, up, cfg, splits):
    from cake_amd.ops import hip as K
    if cfg is not None and cfg >= 8 and stride != 1:
        pytest.skip("halo kernels are stride-1 only")
    torch.manual_seed(5)
    x = torch.randn(N, H, W, IC, device=cuda).to(dt)
    w = (torch.randn(OC, IC, k, k, device=cuda) / math.sqrt(IC * k * k)).to(dt)
    b = torch.randn(OC, device=cuda).to(dt)
    pad = k // 2
    wp = w.permute(0, 2, 3, 1).contiguous()
    y = K.conv2d_nhwc(x, wp, b, stride=stride, pad=pad, up=up, cfg=cfg, splits=splits)
    ref = _ref_conv(x, w, b, stride, pad, up)
    assert y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref, **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("cfg", [0, 6, 8, 11, 12])
def test_conv2d_nhwc_fused_epilogue(cuda, dt, splits, cfg):
    """bias + per-sample f32 bias (time embedding) + residual, as ResnetBlock2D uses them."""
    from cake_amd.ops import hip as K
    torch.manual_seed(6)
    N, H, W, IC, OC = 2, 10, 12, 128, 192
    x = torch.randn(N, H, W, IC, device=cuda).to(dt)
    w = (torch.randn(OC, IC, 3, 3, device=cuda) / math.sqrt(IC * 9)).to(dt)
    b = torch.randn(OC, device=cuda).to(dt)
    b2 = torch.randn(N, OC, device=cuda)
    r = torch.randn(N, H, W, OC, device=cuda).to(dt)
    y = K.conv2d_nhwc(x, w.permute(0, 2, 3, 1).contiguous(), b, bias2=b2, resid=r,
                      cfg=cfg, splits=splits)
    torch.testing.assert_close(y.float(), _ref_conv(x, w, b, 1, 1, False, b2, r), **_tol(dt))


@pytest.mark.parametrize("cfg,tile", [(8, (8, 16)), (8, (16, 8)), (8, (10, 12)), (8, (12, 10)),
                                      (12, (16, 16)), (12, (8, 32)), (13, (32, 8))])
def test_conv2d_halo_tiles(cuda, cfg, tile):
    """Every spatial tile shape of the halo kernel, with partial edge tiles."""
    from cake_amd.ops import hip as K
    torch.manual_seed(7)
    dt = torch.bfloat16
    x = torch.randn(2, 21, 19, 128, device=cuda).to(dt)
    w = (torch.randn(192, 128, 3, 3, device=cuda) / math.sqrt(128 * 9)).to(dt)
    b = torch.randn(192, device=cuda).to(dt)
    y = K.conv2d_nhwc(x, w.permute(0, 2, 3, 1).contiguous(), b, cfg=cfg, tile=tile)
    torch.testing.assert_close(y.float(), _ref_conv(x, w, b, 1, 1, False), **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,H,W,C,G", [
    (2, 16, 16, 320, 32),    # Cg = 10: 8-channel vectors straddle groups
    (2, 8, 8, 2560, 32),     # concat width (Cg = 80), > 256 channel vectors
    (1, 32, 24, 128, 32),    # VAE (Cg = 4)
    (2, 5, 7, 640, 32),      # ragged spatial size
    (1, 64, 64, 256, 32),    # Cg = 8, many pixels
])
@pytest.mark.parametrize("silu", [False, True])
def test_group_norm_nhwc(cuda, dt, N, H, W, C, G, silu):
    from cake_amd.ops import hip as K
    torch.manual_seed(11)
    x = (torch.randn(N, H, W, C, device=cuda) * 3 + 2).to(dt)
    g = (1 + 0.1 * torch.randn(C, device=cuda)).to(dt)
    b = (0.1 * torch.randn(C, device=cuda)).to(dt)
    y = torch.empty_like(x)
    for _ in range(2):  # second call checks the re-armed tickets
        K.group_norm_nhwc(x, g, b, G, 1e-5, silu, y)
    ref = torch.nn.functional.group_norm(x.float().permute(0, 3, 1, 2), G, g.float(), b.float(),
                                         1e-5)
    if silu:
        ref = torch.nn.functional.silu(ref)
    torch.testing.assert_close(y.float(), ref.permute(0, 2, 3, 1), **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,H,W,Cx,Cs,G", [
    (2, 16, 16, 1280, 640, 32),   # SDXL up path: x ++ skip with different widths
    (2, 8, 8, 320, 320, 32),      # Cg = 20 straddles the x / skip boundary
    (1, 5, 7, 640, 1280, 32),     # ragged spatial size
])
@pytest.mark.parametrize("want_cat", [False, True])
def test_group_norm_nhwc_two_source(cuda, dt, N, H, W, Cx, Cs, G, want_cat):
    """GroupNorm of the skip concatenation read in place (and the raw concat written)."""
    from cake_amd.ops import hip as K
    torch.manual_seed(12)
    x = (torch.randn(N, H, W, Cx, device=cuda) * 2 + 1).to(dt)
    s = (torch.randn(N, H, W, Cs, device=cuda) * 0.5 - 1).to(dt)
    C = Cx + Cs
    g = (1 + 0.1 * torch.randn(C, device=cuda)).to(dt)
    b = (0.1 * torch.randn(C, device=cuda)).to(dt)
    y = torch.empty(N, H, W, C, device=cuda, dtype=dt)
    cat = torch.empty_like(y) if want_cat else None
    for _ in range(2):
        K.group_norm_nhwc(x, g, b, G, 1e-5, True, y, skip=s, cat_out=cat)
    xc = torch.cat([x, s], -1)
    ref = torch.nn.functional.group_norm(xc.float().permute(0, 3, 1, 2), G, g.float(), b.float(),
                                         1e-5)
    ref = torch.nn.functional.silu(ref)
    torch.testing.assert_close(y.float(), ref.permute(0, 2, 3, 1), **_tol(dt))
    if want_cat:
        assert torch.equal(cat, xc)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,H,W,IC,OC,stride", [
    (2, 32, 32, 4, 320, 1),     # UNet conv_in (SD1.5 / SDXL latents)
    (1, 17, 13, 4, 512, 1),     # VAE decoder conv_in, ragged
    (1, 16, 16, 3, 128, 1),     # VAE encoder RGB input
    (1, 15, 16, 3, 64, 2),      # strided, odd size
])
@pytest.mark.parametrize("fused", [False, True])
def test_conv2d_small_ic(cuda, dt, N, H, W, IC, OC, stride, fused):
    """Direct 3x3 kernel for IC 3 / 4 (conv_in) vs the f32 reference, with fused epilogue."""
    from cake_amd.ops import hip as K
    torch.manual_seed(8)
    x = torch.randn(N, H, W, IC, device=cuda).to(dt)
    w = (torch.randn(OC, IC, 3, 3, device=cuda) / math.sqrt(IC * 9)).to(dt)
    b = torch.randn(OC, device=cuda).to(dt)
    OH, OW = (H + 2 - 3) // stride + 1, (W + 2 - 3) // stride + 1
    b2 = torch.randn(N, OC, device=cuda) if fused else None
    r = torch.randn(N, OH, OW, OC, device=cuda).to(dt) if fused else None
    y = K.conv2d_nhwc(x, w.permute(0, 2, 3, 1).contiguous(), b, stride=stride, bias2=b2, resid=r)
    ref = _ref_conv(x, w, b, stride, 1, False, b2, r)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))
    if not fused:  # planar input and output (UNet conv_in from / conv_out to NCHW)
        y2 = K.conv2d_nhwc(x.permute(0, 3, 1, 2).contiguous(), w.permute(0, 2, 3, 1).contiguous(),
                           b, stride=stride, in_nchw=True, out_nchw=True)
        assert y2.shape == (N, OC, OH, OW)
        torch.testing.assert_close(y2.float(), ref.permute(0, 3, 1, 2), **_tol(dt))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,H,W,IC,OC", [(1, 128, 128, 4, 4), (2, 17, 9, 8, 8), (1, 5, 7, 3, 16),
                                         (3, 8, 8, 16, 1)])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_conv1x1_small(cuda, dt, N, H, W, IC, OC, layout):
    """Few-channel 1x1 conv (VAE quant / post_quant) in every input / output layout vs
    the f32 reference."""
    from cake_amd.ops import hip as K
    torch.manual_seed(11)
    x = torch.randn(N, H, W, IC, device=cuda).to(dt)
    w = (torch.randn(OC, IC, device=cuda) / math.sqrt(IC)).to(dt)
    b = torch.randn(OC, device=cuda).to(dt)
    ref = (x.float() @ w.float().t() + b.float())            # [N, H, W, OC]
    in_nchw, out_nchw = bool(layout & 1), bool(layout & 2)
    xi = x.permute(0, 3, 1, 2).contiguous() if in_nchw else x
    y = K.conv1x1_small(xi, w, b, in_nchw=in_nchw, out_nchw=out_nchw)
    torch.testing.assert_close(y.float(), ref.permute(0, 3, 1, 2) if out_nchw else ref, **_tol(dt))


@pytest.mark.parametrize("cfg,splits", [(0, 1), (4, 2), (8, 1)])
def test_conv2d_out_nchw(cuda, cfg, splits):
    """conv_out-like (IC 320 -> OC 4) written straight into NCHW planes, incl. split-K."""
    from cake_amd.ops import hip as K
    torch.manual_seed(9)
    dt = torch.float16
    x = torch.randn(2, 12, 10, 320, device=cuda).to(dt)
    w = (torch.randn(4, 320, 3, 3, device=cuda) / math.sqrt(320 * 9)).to(dt)
    b = torch.randn(4, device=cuda).to(dt)
    y = K.conv2d_nhwc(x, w.permute(0, 2, 3, 1).contiguous(), b, cfg=cfg, splits=splits,
                      out_nchw=True)
    torch.testing.assert_close(y.float(), _ref_conv(x, w, b, 1, 1, False).permute(0, 3, 1, 2),
                               **_tol(dt))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,N,M", [(1, 4096, 4096), (2, 1000, 777), (1, 16384, 16384), (1, 70, 33)])
def test_attn512_vs_fp32(cuda, dt, B, N, M):
    """Head-dim-512 flash attention (VAE mid-block) vs the f32 softmax reference."""
    import math
    from cake_amd.ops import hip as K
    torch.manual_seed(N + M)
    q = (torch.randn(B, N, 512, device=cuda) * 0.5).to(dt)
    k = (torch.randn(B, M, 512, device=cuda) * 0.5).to(dt)
    v = torch.randn(B, M, 512, device=cuda).to(dt)
    out = torch.empty(B, N, 512, device=cuda, dtype=dt)
    scale = 1 / math.sqrt(512)
    K.attn512(q, k, v, out, scale)
    ref = torch.empty(B, N, 512, device=cuda)
    for b in range(B):
        for s0 in range(0, N, 4096):  # bounded f32 score slabs
            sc = (q[b, s0:s0 + 4096].float() @ k[b].float().t()) * scale
            ref[b, s0:s0 + 4096] = torch.softmax(sc, -1) @ v[b].float()
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("dim,flip,shift", [(320, True, 0.0), (256, False, 1.0)])
def test_timestep_embed_vs_torch(cuda, dt, dim, flip, shift):
    """sd_small.hip timestep_embed (device table + device step) vs the torch embedding."""
    from cake_amd.models.sd.unet import timestep_embedding
    from cake_amd.ops import hip as K
    table = torch.tensor([999.0, 761.0, 21.0], device=cuda)
    step = torch.tensor([1], device=cuda, dtype=torch.int32)
    out = torch.empty(2, dim, device=cuda, dtype=dt)
    K.timestep_embed(table, step, 2, dim, flip, shift, out)
    ref = timestep_embedding(torch.tensor([761.0, 761.0]), dim, flip, shift)
    tol = dict(atol=1e-3, rtol=1e-3) if dt == torch.float32 else _tol(dt)
    torch.testing.assert_close(out.float().cpu(), ref, **tol)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cfg", [True, False])
def test_sched_step_deterministic_vs_torch(cuda, dt, cfg):
    """CFG combine + DDIM-style update (N = 0) + next input == the torch expression."""
    from cake_amd.ops import hip as K
    n = 4 * 32 * 32
    x = torch.randn(n, device=cuda)
    pred = torch.randn((2 if cfg else 1) * n, device=cuda).to(dt)
    coef = torch.tensor([[0.9, -0.3, 0.0, 0.5], [1.1, 0.2, 0.0, 2.0]], device=cuda)
    step = torch.tensor([1], device=cuda, dtype=torch.int32)
    seed = torch.tensor([7], device=cuda, dtype=torch.int64)
    nxt = torch.empty_like(pred)
    x0 = x.clone()
    K.sched_step(x, pred, cfg, 7.5, coef, step, seed, next_in=nxt)
    e = pred.float()
    if cfg:
        u, c = e[:n], e[n:]
        e = u + 7.5 * (c - u)
    ref = 1.1 * x0 + 0.2 * e
    torch.testing.assert_close(x, ref, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(nxt[:n].float(), (2.0 * ref).to(dt).float(), atol=0, rtol=0)
    if cfg:
        assert torch.equal(nxt[:n], nxt[n:])
    K.step_advance(step)
    assert int(step.item()) == 2


def test_sched_step_noise_is_standard_normal(cuda):
    """Euler-ancestral noise term: N(0, 1) per element, fresh per step, keyed by the seed."""
    from cake_amd.ops import hip as K
    n = 1 << 20
    pred = torch.zeros(n, device=cuda, dtype=torch.bfloat16)
    coef = torch.tensor([[0.0, 0.0, 1.0, 1.0]] * 2, device=cuda)
    seed = torch.tensor([12345], device=cuda, dtype=torch.int64)
    draws = []
    for s in (0, 1, 0):
        x = torch.zeros(n, device=cuda)
        K.sched_step(x, pred, False, 1.0, coef, torch.tensor([s], device=cuda, dtype=torch.int32),
                     seed)
        draws.append(x)
    z = draws[0]
    assert abs(float(z.mean())) < 5e-3 and abs(float(z.std()) - 1.0) < 5e-3
    assert abs(float(((z > 1.96).float().mean())) - 0.025) < 2e-3
    assert torch.equal(draws[0], draws[2])  # same (seed, step) -> same noise
    assert abs(float((draws[0] * draws[1]).mean())) < 5e-3  # steps independent
    seed.fill_(54321)
    x = torch.zeros(n, device=cuda)
    K.sched_step(x, pred, False, 1.0, coef, torch.tensor([0], device=cuda, dtype=torch.int32), seed)
    assert abs(float((x * z).mean())) < 5e-3


@pytest.mark.parametrize("nhwc", [False, True])
def test_to_rgb8_vs_torch(cuda, nhwc):
    from cake_amd.ops import hip as K
    img = (torch.rand(2, 3, 40, 24, device=cuda) * 2.4 - 1.2).half()
    src = img.permute(0, 2, 3, 1).contiguous() if nhwc else img
    got = K.to_rgb8(src, nhwc=nhwc)
    ref = ((img.float() / 2 + 0.5).clamp(0, 1) * 255).to(torch.uint8).permute(0, 2, 3, 1)
    assert torch.equal(got, ref)
