"""Shape fuzzing (hypothesis) of the hand-written kernels against PyTorch f32
references: implicit-GEMM conv (every tile/staging variant), flash attention v2,
channels-last GroupNorm and the decode GEMV."""
import math

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu
FUZZ = settings(max_examples=25, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture])


@FUZZ
@given(n=st.integers(1, 2), h=st.integers(1, 19), w=st.integers(1, 19),
       ic=st.sampled_from([64, 128, 192]), oc=st.integers(1, 48).map(lambda v: 4 * v),
       k=st.sampled_from([1, 3]), stride=st.sampled_from([1, 2]), up=st.booleans(),
       cfg=st.integers(0, 13), splits=st.sampled_from([1, 2, 3]),
       resid=st.booleans())
def test_fuzz_conv2d(cuda, n, h, w, ic, oc, k, stride, up, cfg, splits, resid):
    from cake_amd.ops import hip as K
    if up and stride != 1:
        stride = 1
    if cfg >= 8 and (stride != 1 or k == 1):
        cfg = cfg - 8
    pad = k // 2
    g = torch.Generator(device="cpu").manual_seed(n * 1000 + h * 37 + w)
    x = torch.randn(n, h, w, ic, generator=g).to(cuda, torch.bfloat16)
    wt = (torch.randn(oc, ic, k, k, generator=g) / math.sqrt(ic * k * k)).to(cuda, torch.bfloat16)
    b = torch.randn(oc, generator=g).to(cuda, torch.bfloat16)
    xc = x.float().permute(0, 3, 1, 2)
    if up:
        xc = torch.nn.functional.interpolate(xc, scale_factor=2.0, mode="nearest")
    ref = torch.nn.functional.conv2d(xc, wt.float(), b.float(), stride=stride, padding=pad)
    ref = ref.permute(0, 2, 3, 1)
    r = torch.randn(ref.shape, generator=g).to(cuda, torch.bfloat16) if resid else None
    if r is not None:
        ref = ref + r.float()
    y = K.conv2d_nhwc(x, wt.permute(0, 2, 3, 1).contiguous(), b, stride=stride, pad=pad, up=up,
                      resid=r, cfg=cfg, splits=splits)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@FUZZ
@given(b=st.integers(1, 2), hkv=st.integers(1, 3), rep=st.sampled_from([1, 2, 4]),
       n=st.integers(1, 300), m=st.integers(1, 300), d=st.integers(1, 16).map(lambda v: 8 * v),
       causal=st.booleans(), pos0=st.integers(0, 64))
def test_fuzz_flash_attn(cuda, b, hkv, rep, n, m, d, causal, pos0):
    from cake_amd.ops import hip as K
    h = hkv * rep
    if causal:
        m = max(m, n + pos0)  # every query row sees at least key 0 .. pos0 + row
    else:
        pos0 = 0
    g = torch.Generator(device="cpu").manual_seed(n * 7 + m * 13 + d)
    q = torch.randn(b, n, h, d, generator=g).to(cuda, torch.bfloat16).transpose(1, 2)
    k = torch.randn(b, m, hkv, d, generator=g).to(cuda, torch.bfloat16).transpose(1, 2)
    v = torch.randn(b, m, hkv, d, generator=g).to(cuda, torch.bfloat16).transpose(1, 2)
    o = torch.empty(b, n, h, d, device=cuda, dtype=torch.bfloat16).transpose(1, 2)
    scale = 1 / math.sqrt(d)
    K.flash_attn(q, k, v, o, scale, causal, pos0)
    kk = k.float().repeat_interleave(rep, 1)
    vv = v.float().repeat_interleave(rep, 1)
    s = (q.float() @ kk.transpose(-1, -2)) * scale
    if causal:
        qi = torch.arange(n, device=cuda)[:, None] + pos0
        s = s.masked_fill(torch.arange(m, device=cuda)[None] > qi, float("-inf"))
    torch.testing.assert_close(o.float(), torch.softmax(s, -1) @ vv, atol=2e-2, rtol=2e-2)


@FUZZ
@given(n=st.integers(1, 3), hw=st.integers(1, 300), groups=st.sampled_from([8, 16, 32]),
       cg=st.sampled_from([4, 8, 10, 12, 20, 40]), silu=st.booleans())
def test_fuzz_group_norm_nhwc(cuda, n, hw, groups, cg, silu):
    from cake_amd.ops import hip as K
    c = groups * cg
    if c % 8:
        return
    g = torch.Generator(device="cpu").manual_seed(hw * 3 + c)
    x = (torch.randn(n, hw, c, generator=g) * 2 + 1).to(cuda, torch.bfloat16)
    gm = (1 + 0.1 * torch.randn(c, generator=g)).to(cuda, torch.bfloat16)
    bt = (0.1 * torch.randn(c, generator=g)).to(cuda, torch.bfloat16)
    y = torch.empty_like(x)
    K.group_norm_nhwc(x, gm, bt, groups, 1e-5, silu, y)
    ref = torch.nn.functional.group_norm(x.float().permute(0, 2, 1), groups, gm.float(),
                                         bt.float(), 1e-5).permute(0, 2, 1)
    if silu:
        ref = torch.nn.functional.silu(ref)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@FUZZ
@given(rows=st.integers(1, 700), k=st.integers(1, 800).map(lambda v: 8 * v),
       acc=st.booleans())
def test_fuzz_gemv(cuda, rows, k, acc):
    from cake_amd.ops import hip as K
    g = torch.Generator(device="cpu").manual_seed(rows * 5 + k)
    x = torch.randn(k, generator=g).to(cuda, torch.bfloat16)
    w = (torch.randn(rows, k, generator=g) / math.sqrt(k)).to(cuda, torch.bfloat16)
    out = torch.randn(rows, generator=g).to(cuda)
    ref = (w.float() @ x.float()) + (out if acc else 0)
    K.gemv(x, w, out, accumulate=acc)
    torch.testing.assert_close(out, ref, atol=2e-2, rtol=2e-2)
