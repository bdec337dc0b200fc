"""SD op dispatch: gfx950 HIP kernels on the device path, PyTorch on CPU / f32.

On the device path the UNet and VAE run channels-last (NHWC): convolutions are
our MFMA implicit-GEMM kernels (conv2d.hip, per-shape autotuned, time-embedding
bias and residual fused into the epilogue, nearest-2x upsample fused into the
operand addressing), GroupNorm(+SiLU) is the channels-last kernel, and the
SpatialTransformer consumes [B, HW, C] views with no permutes.  LayerNorm,
multi-head attention (MFMA flash attention) and GEGLU are our kernels too
(SURVEY K31-K36); every linear is the MFMA GEMM (gemm.hip) with bias, block
residual and GEGLU fused in its epilogue.  The CPU / f32 path is plain NCHW
PyTorch.
"""
from __future__ import annotations

import math
import os
import threading
from contextlib import contextmanager

import torch
import torch.nn.functional as F

_state = threading.local()


def nhwc() -> bool:
    """True while a channels-last forward is running on this thread."""
    return getattr(_state, "nhwc", False)


@contextmanager
def layout_nhwc(on: bool):
    prev = nhwc()
    _state.nhwc = on
    try:
        yield
    finally:
        _state.nhwc = prev


def want_nhwc(x: torch.Tensor) -> bool:
    return _hip(x) and os.environ.get("CAKE_SD_NHWC", "1") != "0"


def cdim() -> int:
    return -1 if nhwc() else 1


def to_internal(x: torch.Tensor) -> torch.Tensor:
    """NCHW module input -> the active layout."""
    return x.permute(0, 2, 3, 1).contiguous() if nhwc() else x


def to_external(x: torch.Tensor) -> torch.Tensor:
    """Active layout -> NCHW module output."""
    return x.permute(0, 3, 1, 2).contiguous() if nhwc() else x


def pad_hw_end(x: torch.Tensor) -> torch.Tensor:
    """Zero-pad one row at the bottom and one column at the right."""
    return F.pad(x, (0, 0, 0, 1, 0, 1)) if nhwc() else F.pad(x, (0, 1, 0, 1))


def tokens(x: torch.Tensor) -> torch.Tensor:
    """Feature map -> [B, HW, C] tokens."""
    if nhwc():
        B, H, W, C = x.shape
        return x.reshape(B, H * W, C)
    B, C, H, W = x.shape
    return x.permute(0, 2, 3, 1).reshape(B, H * W, C)


def untokens(t: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    """[B, HW, C] tokens -> feature map shaped like `like`."""
    if nhwc():
        return t.reshape(like.shape)
    B, C, H, W = like.shape
    return t.reshape(B, H, W, C).permute(0, 3, 1, 2).contiguous()


def _hip(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype in (torch.float16, torch.bfloat16)


def group_norm(x, w, b, groups: int, eps: float, silu: bool = False):
    if nhwc():
        from ...ops import hip as K
        if _hip(x) and K.group_norm_nhwc_supported(x.shape[-1], groups):
            x = x.contiguous()
            y = torch.empty_like(x)
            K.group_norm_nhwc(x, w, b, groups, eps, silu, y)
            return y
        y = F.group_norm(x.float().permute(0, 3, 1, 2), groups, w.float(), b.float(), eps)
        y = F.silu(y) if silu else y
        return y.permute(0, 2, 3, 1).to(x.dtype).contiguous()
    if _hip(x):
        from ...ops import hip as K
        x = x.contiguous()
        y = torch.empty_like(x)
        K.group_norm(x, w, b, groups, eps, silu, y)
        return y
    y = F.group_norm(x.float(), groups, w.float(), b.float(), eps)
    return (F.silu(y) if silu else y).to(x.dtype)


def group_norm_cat(x, skip, w, b, groups: int, eps: float, silu: bool = False,
                   want_cat: bool = True):
    """GroupNorm of the channel concatenation [x, skip] -> (normalised, raw concat or None).

    Channels-last on the device: one two-source GroupNorm pass reads x and skip in
    place and (want_cat) writes the raw concatenation alongside the normalised
    output, so the UNet up path's skip concat is not a separate copy kernel."""
    if nhwc():
        from ...ops import hip as K
        C = x.shape[-1] + skip.shape[-1]
        if _hip(x) and K.group_norm_nhwc_supported(C, groups) and x.shape[-1] % 8 == 0:
            x, skip = x.contiguous(), skip.contiguous()
            shape = (*x.shape[:-1], C)
            y = torch.empty(shape, device=x.device, dtype=x.dtype)
            cat = torch.empty(shape, device=x.device, dtype=x.dtype) if want_cat else None
            K.group_norm_nhwc(x, w, b, groups, eps, silu, y, skip=skip, cat_out=cat)
            return y, cat
    xc = torch.cat([x, skip], cdim())
    return group_norm(xc, w, b, groups, eps, silu), xc


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

        def heads4(t, rows):  # [B, rows, C] (any row stride, unit channel stride) -> [B, h, rows, D]
            if t.stride(-1) != 1 or t.data_ptr() % 16 or any(st % 8 for st in t.stride()[:2]):
                t = t.contiguous()
            return t.view(B, rows, heads, D).transpose(1, 2)

        out = torch.empty(B, N, C, device=q.device, dtype=q.dtype)
        K.flash_attn(heads4(q, N), heads4(k, M), heads4(v, M),
                     out.view(B, N, heads, D).transpose(1, 2), scale, causal)
        return out
    if _hip(q) and D == 512 and heads == 1:  # VAE mid-block: flash kernel for head dim 512
        from ...ops import hip as K

        def rows(t):
            return t if (t.stride(-1) == 1 and t.data_ptr() % 16 == 0 and t.stride(1) % 8 == 0) \
                else t.contiguous()
        out = torch.empty(B, N, C, device=q.device, dtype=q.dtype)
        K.attn512(rows(q), rows(k), rows(v), out, scale)
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


def _gemm_ok(x, w) -> bool:
    return _hip(x) and w.dtype == x.dtype and x.shape[-1] % 8 == 0 and w.stride(-1) == 1 \
        and w.stride(0) % 8 == 0


def linear(x, w, b=None, resid=None, gated: str | None = None, act: str | None = None):
    """y = x w^T (+ b) on the MFMA GEMM (gemm.hip), with fused epilogues:
    resid -> y + resid (block residual); gated="geglu" -> GEGLU over the two halves
    of w's rows (diffusers FeedForward proj, bias included); act="quick_gelu" /
    "gelu" -> the activation applied to y (+ b) (CLIP MLP)."""
    if act is not None and (gated is not None or resid is not None):
        raise ValueError("act combines with neither gated nor resid")
    if _gemm_ok(x, w):
        from ...ops import gemm as G
        if gated is not None:
            return G.linear(x, w, b, epi=gated)
        if resid is not None:
            return G.linear(x, w, b, epi="add16", resid=resid.contiguous())
        if act is not None:
            return G.linear(x, w, b, epi=act)
        return G.linear(x, w, b)
    y = F.linear(x, w, b)
    if act == "quick_gelu":
        return y * torch.sigmoid(1.702 * y)
    if act == "gelu":
        return F.gelu(y)
    if act is not None:
        raise ValueError(act)
    if gated == "geglu":
        a, g = y.float().chunk(2, -1)
        y = (a * F.gelu(g, approximate="tanh")).to(x.dtype)
    elif gated is not None:
        raise ValueError(gated)
    if resid is not None:
        y = y + resid
    return y


def conv2d(x, w, b=None, stride: int = 1, padding: int = 1):
    return F.conv2d(x, w, b, stride=stride, padding=padding)


def conv(W, name: str, x, stride: int = 1, padding: int = 1, up: bool = False, bias2=None,
         resid=None, in_nchw: bool = False, out_nchw: bool = False):
    """Convolution `name` of W on x in the active layout.

    up: nearest-2x upsample x first; bias2 [B, OC]: per-sample additive bias
    (ResnetBlock2D time embedding); resid: added to the output (block residual).
    in_nchw / out_nchw (channels-last layout only): x arrives in / the output leaves in
    the external NCHW layout — the UNet's conv_in / conv_out, so the layout change is
    part of those kernels instead of two copy kernels per step.
    """
    w, b = W[f"{name}.weight"], W.get(f"{name}.bias")
    if not nhwc():
        in_nchw = out_nchw = False  # NCHW throughout
    if nhwc():
        from ...ops import hip as K
        OC, IC = w.shape[:2]
        if (_hip(x) and w.shape[2] == w.shape[3] == 1 and IC <= 16 and OC <= 16 and stride == 1
                and padding == 0 and not up and bias2 is None and resid is None):
            # few-channel 1x1 (VAE quant_conv / post_quant_conv): per-pixel kernel that
            # reads / writes either layout itself
            key = f"{name}.weight@1x1"
            wp = W.get(key)
            if wp is None or wp.dtype != x.dtype:
                wp = W[key] = w.to(x.dtype).reshape(OC, IC).contiguous()
            bb = None if b is None else b.to(x.dtype)
            return K.conv1x1_small(x.contiguous(), wp, bb, in_nchw=in_nchw, out_nchw=out_nchw)
        if (_hip(x) and OC < 4 and w.shape[2] == w.shape[3] and bias2 is None and resid is None
                and K.conv_supported(IC, 4, stride, up, w.shape[2])):
            # OC < 4 (VAE decoder.conv_out 128 -> 3): the MFMA conv on 4 output channels,
            # the padded ones with zero filters, sliced off
            from ...ops import conv as C
            key = f"{name}.weight@nhwc4"
            wp = W.get(key)
            if wp is None or wp.dtype != x.dtype:
                w4 = torch.zeros((4,) + tuple(w.shape[1:]), device=w.device, dtype=x.dtype)
                w4[:OC] = w.to(x.dtype)
                wp = W[key] = w4.permute(0, 2, 3, 1).contiguous()
                b4 = torch.zeros(4, device=w.device, dtype=x.dtype)
                if b is not None:
                    b4[:OC] = b.to(x.dtype)
                W[key + ".bias"] = b4
            if in_nchw:
                x = to_internal(x)
            y = C.conv2d(x.contiguous(), wp, W[key + ".bias"], stride=stride, pad=padding, up=up,
                         out_nchw=out_nchw)
            y = y[:, :OC] if out_nchw else y[..., :OC]
            return y if (out_nchw and y.shape[0] == 1) else y.contiguous()
        if _hip(x) and w.shape[2] == w.shape[3] and K.conv_supported(IC, OC, stride, up, w.shape[2]):
            from ...ops import conv as C
            key = f"{name}.weight@nhwc"
            wp = W.get(key)
            if wp is None or wp.dtype != x.dtype:
                wp = W[key] = w.to(x.dtype).permute(0, 2, 3, 1).contiguous()
            if in_nchw and IC % 64 == 0:  # only the direct small-IC kernel reads planes
                x, in_nchw = to_internal(x), False
            if out_nchw and resid is not None:
                y = conv(W, name, x, stride, padding, up, bias2, resid, in_nchw=in_nchw)
                return to_external(y)
            return C.conv2d(x.contiguous(), wp, b, stride=stride, pad=padding, up=up,
                            bias2=None if bias2 is None else
                            (bias2 if bias2.dtype == torch.float32 else bias2.float()),
                            resid=None if resid is None else resid.contiguous(),
                            in_nchw=in_nchw, out_nchw=out_nchw)
        if in_nchw:
            x = to_internal(x)
        if out_nchw:
            return to_external(conv(W, name, x, stride, padding, up, bias2, resid))
        xn = x.permute(0, 3, 1, 2)  # channels_last view: MIOpen's NHWC kernels
        if up:
            xn = F.interpolate(xn, scale_factor=2.0, mode="nearest")
        y = F.conv2d(xn, w, b, stride=stride, padding=padding).permute(0, 2, 3, 1)
        if bias2 is not None:
            y = y + bias2[:, None, None, :].to(y.dtype)
        if resid is not None:
            y = y + resid
        return y.contiguous()
    if up:
        x = F.interpolate(x, scale_factor=2.0, mode="nearest")
    y = conv2d(x, w, b, stride, padding)
    if bias2 is not None:
        y = y + bias2[:, :, None, None].to(y.dtype)
    if resid is not None:
        y = y + resid
    return y
