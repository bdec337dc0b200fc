"""SD op dispatch: gfx950 HIP kernels on the device path, PyTorch on CPU / f32.

GroupNorm(+SiLU), LayerNorm, multi-head attention (MFMA flash attention) and
GEGLU run as our kernels; convolutions go to MIOpen and the
plain linears to hipBLASLt (library GEMMs) through torch.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _hip(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype in (torch.float16, torch.bfloat16)


def group_norm(x, w, b, groups: int, eps: float, silu: bool = False):
    if _hip(x):
        from ...ops import hip as K
        x = x.contiguous()
        y = torch.empty_like(x)
        K.group_norm(x, w, b, groups, eps, silu, y)
        return y
    y = F.group_norm(x.float(), groups, w.float(), b.float(), eps)
    return (F.silu(y) if silu else y).to(x.dtype)


def layer_norm(x, w, b, eps: float):
    if _hip(x):
        from ...ops import hip as K
        x = x.contiguous()
        y = torch.empty_like(x)
        K.layer_norm(x, w, b, eps, y)
        return y
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def attention(q, k, v, heads: int, causal: bool = False, sliced: int | None = None):
    """q [B, N, C], k/v [B, M, C] -> [B, N, C] (softmax in f32)."""
    B, N, C = q.shape
    M = k.shape[1]
    D = C // heads
    scale = 1.0 / math.sqrt(D)
    if _hip(q) and D <= 256:
        from ...ops import hip as K
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out = torch.empty_like(q)
        K.flash_attn(q.view(B, N, heads, D).transpose(1, 2), k.view(B, M, heads, D).transpose(1, 2),
                     v.view(B, M, heads, D).transpose(1, 2), out.view(B, N, heads, D).transpose(1, 2),
                     scale, causal)
        return out
    qh = q.view(B, N, heads, D).transpose(1, 2).float()
    kh = k.view(B, M, heads, D).transpose(1, 2).float()
    vh = v.view(B, M, heads, D).transpose(1, 2).float()
    step = sliced or N  # sliced attention (--sd-sliced-attention-size) bounds score memory
    outs = []
    for s0 in range(0, N, step):
        sc = (qh[:, :, s0:s0 + step] @ kh.transpose(-1, -2)) * scale
        if causal:
            qi = torch.arange(s0, min(N, s0 + step), device=q.device)[:, None]
            sc = sc.masked_fill(torch.arange(M, device=q.device)[None] > qi, float("-inf"))
        outs.append(torch.softmax(sc, -1) @ vh)
    return torch.cat(outs, 2).transpose(1, 2).reshape(B, N, C).to(q.dtype)


def geglu(h):
    if _hip(h):
        from ...ops import hip as K
        h = h.contiguous()
        out = torch.empty(*h.shape[:-1], h.shape[-1] // 2, device=h.device, dtype=h.dtype)
        K.geglu(h, out)
        return out
    a, g = h.float().chunk(2, -1)
    return (a * F.gelu(g, approximate="tanh")).to(h.dtype)


def linear(x, w, b=None):
    return F.linear(x, w, b)


def conv2d(x, w, b=None, stride: int = 1, padding: int = 1):
    return F.conv2d(x, w, b, stride=stride, padding=padding)
