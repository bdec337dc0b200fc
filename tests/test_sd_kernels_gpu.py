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
])
def test_flash_attn(cuda, dt, B, H, Hkv, N, M, D, causal, pos0):
    from cake_amd.ops import hip as K
    torch.manual_seed(0)
    # projection-style layouts: [B, rows, heads, D] viewed as [B, heads, rows, D]
    q = torch.randn(B, N, H, D, device=cuda).to(dt).transpose(1, 2)
    k = torch.randn(B, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    v = torch.randn(B, M, Hkv, D, device=cuda).to(dt).transpose(1, 2)
    out = torch.empty(B, N, H, D, device=cuda, dtype=dt).transpose(1, 2)
    scale = 1 / math.sqrt(D)
    K.flash_attn(q, k, v, out, scale, causal, pos0)
    torch.testing.assert_close(out.float(), _ref_attn(q, k, v, scale, causal, pos0), **_tol(dt))


def test_flash_attn_softmax_rescale_branch(cuda):
    """A late key tile with a much larger score forces the online-softmax rescale."""
    from cake_amd.ops import hip as K
    dt = torch.bfloat16
    q = torch.randn(1, 1, 64, 64, device=cuda).to(dt)
    k = torch.randn(1, 1, 256, 64, device=cuda)
    k[0, 0, 200] = q[0, 0, 5].float() * 4  # spike for row 5 in tile 3
    k = k.to(dt)
    v = torch.randn(1, 1, 256, 64, device=cuda).to(dt)
    out = torch.empty_like(q)
    K.flash_attn(q, k, v, out, 0.125)
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
def test_layer_norm_and_geglu(cuda, dt):
    from cake_amd.ops import hip as K
    torch.manual_seed(2)
    x = torch.randn(2, 77, 768, device=cuda).to(dt)
    g = (1 + 0.1 * torch.randn(768, device=cuda)).to(dt)
    b = (0.1 * torch.randn(768, device=cuda)).to(dt)
    y = torch.empty_like(x)
    K.layer_norm(x, g, b, 1e-5, y)
    ref = torch.nn.functional.layer_norm(x.float(), (768,), g.float(), b.float(), 1e-5)
    torch.testing.assert_close(y.float(), ref, **_tol(dt))
    h = torch.randn(2, 50, 2 * 1280, device=cuda).to(dt)
    o = torch.empty(2, 50, 1280, device=cuda, dtype=dt)
    K.geglu(h, o)
    a, gate = h.float().chunk(2, -1)
    torch.testing.assert_close(o.float(), a * torch.nn.functional.gelu(gate, approximate="tanh"),
                               **_tol(dt))
