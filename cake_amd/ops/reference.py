"""Plain-PyTorch implementation of the Llama-3 math.

Used (a) as the CPU / f32 execution backend — the reference's ``--cpu`` mode —
and (b) as the numerical oracle for every HIP kernel test.  It mirrors:

* RMSNorm           cake-core/src/models/llama3/transformer.rs:60,68 (candle RmsNorm)
* RoPE (half-split) cake-core/src/models/llama3/attention.rs:25-35, cache.rs:23-61
* GQA attention     cake-core/src/models/llama3/attention.rs:38-123 (f32 softmax)
* SwiGLU            cake-core/src/models/llama3/mlp.rs:15-18
* repeat penalty    cake-core/src/models/llama3/llama.rs:311-320

All math is f32 internally; inputs/outputs keep the caller's dtype except the
residual stream, which is f32.
"""
from __future__ import annotations

import math

import torch


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return xf * r * w.float()


def inv_freq(head_dim: int, theta: float, rope_scaling: dict | None = None) -> torch.Tensor:
    """θ_i = 1/θ^(2i/d) (cache.rs:29-32), with optional Llama-3.1 'llama3' scaling."""
    f = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if rope_scaling and rope_scaling.get("rope_type", rope_scaling.get("type")) == "llama3":
        factor = rope_scaling["factor"]
        lo = rope_scaling.get("low_freq_factor", 1.0)
        hi = rope_scaling.get("high_freq_factor", 4.0)
        old = rope_scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / f
        out = torch.where(wl > lo_wl, f / factor, f)
        smooth = (old / wl - lo) / (hi - lo)
        mid = (1 - smooth) * out / factor + smooth * out
        is_mid = (wl >= hi_wl) & (wl <= lo_wl)
        f = torch.where(is_mid, mid, out)
    return f.float()


def rope(x: torch.Tensor, positions: torch.Tensor, inv_f: torch.Tensor) -> torch.Tensor:
    """x [T, nheads, hd] -> rotated (f32). Non-interleaved: pairs (i, i + hd/2)."""
    ang = positions.float()[:, None] * inv_f.to(x.device)[None, :]  # [T, hd/2]
    c, s = torch.cos(ang)[:, None, :], torch.sin(ang)[:, None, :]
    xf = x.float()
    h = xf.shape[-1] // 2
    a, b = xf[..., :h], xf[..., h:]
    return torch.cat([a * c - b * s, a * s + b * c], dim=-1)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, pos0: int) -> torch.Tensor:
    """q [T, nh, hd]; k, v [Tk, nkv, hd] (Tk = pos0 + T).  Causal with offset. f32 out."""
    T, nh, hd = q.shape
    Tk, nkv, _ = k.shape
    rep = nh // nkv
    qf = q.float().transpose(0, 1)                                      # [nh, T, hd]
    kf = k.float().transpose(0, 1).repeat_interleave(rep, dim=0)        # [nh, Tk, hd]
    vf = v.float().transpose(0, 1).repeat_interleave(rep, dim=0)
    att = (qf @ kf.transpose(1, 2)) / math.sqrt(hd)                     # [nh, T, Tk]
    if T > 1 or pos0 + T < Tk:
        qi = torch.arange(T, device=q.device)[:, None] + pos0
        kj = torch.arange(Tk, device=q.device)[None, :]
        att = att.masked_fill(kj > qi, float("-inf"))
    att = torch.softmax(att, dim=-1)
    return (att @ vf).transpose(0, 1)                                   # [T, nh, hd]


def silu_mul(g: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    gf = g.float()
    return gf * torch.sigmoid(gf) * u.float()


def apply_repeat_penalty(logits: torch.Tensor, penalty: float, context: list[int]) -> torch.Tensor:
    """candle_transformers::utils::apply_repeat_penalty semantics (unique tokens)."""
    out = logits.clone()
    for t in sorted(set(int(x) for x in context)):
        if 0 <= t < out.shape[-1]:
            s = out[..., t]
            out[..., t] = torch.where(s >= 0, s / penalty, s * penalty)
    return out
