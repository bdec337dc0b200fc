"""Torch-tensor wrappers around the gfx950 HIP kernels.

Every wrapper validates shapes / dtypes / contiguity / device on the host
*before* launching (a bad pointer or shape on the GPU can take down the box),
then launches on torch's current stream.  No wrapper falls back to PyTorch: if
the kernel library is missing, :func:`cake_amd.ops._lib.kernels` raises.
"""
from __future__ import annotations

import torch

from ._lib import check, kernels

_DT = {torch.bfloat16: 0, torch.float16: 1}


def _dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"HIP kernels take bf16/f16 weights, got {t.dtype}") from None


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _req(t: torch.Tensor, name: str, *, dtype=None, numel=None, shape=None) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected contiguous")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name}: expected >= {numel} elements, got {t.numel()}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")


# ---------------------------------------------------------------------------
# decode (batch 1) fused projections
# ---------------------------------------------------------------------------

def qkv_rope(resid, norm_w, eps, wq, wk, wv, inv_freq, pos, q_out, kcache, vcache, rearm=None):
    """rmsnorm(resid) -> q/k/v GEMV -> RoPE(pos) -> q_out f32, k/v into cache[:, pos].

    kcache/vcache: [nkv, S, hd] (one layer). pos: int32 device scalar.
    """
    K = resid.numel()
    nkv, S, hd = kcache.shape
    nh = wq.shape[0] // hd
    dt = wq.dtype
    _req(resid, "resid", dtype=torch.float32)
    _req(norm_w, "norm_w", dtype=dt, shape=(K,))
    _req(wq, "wq", dtype=dt, shape=(nh * hd, K))
    _req(wk, "wk", dtype=dt, shape=(nkv * hd, K))
    _req(wv, "wv", dtype=dt, shape=(nkv * hd, K))
    _req(inv_freq, "inv_freq", dtype=torch.float32, shape=(hd // 2,))
    _req(pos, "pos", dtype=torch.int32, numel=1)
    _req(q_out, "q_out", dtype=torch.float32, numel=nh * hd)
    _req(kcache, "kcache", dtype=dt)
    _req(vcache, "vcache", dtype=dt, shape=kcache.shape)
    if K % 8:
        raise ValueError("hidden size must be a multiple of 8")
    check(kernels().cake_qkv_rope(_dt(wq), _p(resid), _p(norm_w), float(eps), _p(wq), _p(wk),
                                  _p(wv), K, nh, nkv, hd, _p(inv_freq), _p(pos), _p(q_out),
                                  _p(kcache), _p(vcache), S,
                                  None if rearm is None else rearm[1:].data_ptr(), _stream()),
          "qkv_rope")


def swiglu(resid, norm_w, eps, wg, wu, act):
    """act = silu(rmsnorm(resid) @ wg.T) * (rmsnorm(resid) @ wu.T)   (batch 1)."""
    K = resid.numel()
    I = wg.shape[0]
    dt = wg.dtype
    _req(resid, "resid", dtype=torch.float32)
    _req(norm_w, "norm_w", dtype=dt, shape=(K,))
    _req(wg, "wg", dtype=dt, shape=(I, K))
    _req(wu, "wu", dtype=dt, shape=(I, K))
    _req(act, "act", dtype=dt, numel=I)
    check(kernels().cake_swiglu(_dt(wg), _p(resid), _p(norm_w), float(eps), _p(wg), _p(wu), K,
                                I, _p(act), _stream()), "swiglu")


def gemv(x, w, out, accumulate: bool):
    """out (f32) [+]= w @ x with a 16-bit x (batch 1)."""
    N, K = w.shape
    _req(w, "w")
    _req(x, "x", dtype=w.dtype, numel=K)
    _req(out, "out", dtype=torch.float32, numel=N)
    if K % 8:
        raise ValueError("K must be a multiple of 8")
    check(kernels().cake_gemv_x16(_dt(w), _p(x), _p(w), K, N, _p(out), int(accumulate),
                                  _stream()), "gemv_x16")


def norm_gemv_f32(resid, norm_w, eps, w, out):
    """out (f32) = w @ rmsnorm(resid)  — the lm_head (batch 1)."""
    N, K = w.shape
    _req(resid, "resid", dtype=torch.float32, numel=K)
    _req(norm_w, "norm_w", dtype=w.dtype, shape=(K,))
    _req(w, "w")
    _req(out, "out", dtype=torch.float32, numel=N)
    check(kernels().cake_gemv_norm_f32(_dt(w), _p(resid), _p(norm_w), float(eps), _p(w), K, N,
                                       _p(out), _stream()), "gemv_norm_f32")


def attn_decode(q, kcache, vcache, pos, scale, part, tickets, out):
    """Split-K GQA decode attention for the token at device position `pos`.

    part: f32 workspace (:func:`attn_workspace_numel`); tickets: int32 [nkv],
    zero-initialised once and re-armed by the kernel itself.
    """
    nkv, S, hd = kcache.shape
    nh = q.numel() // hd
    nsplit = (S + 63) // 64
    _req(q, "q", dtype=torch.float32)
    _req(kcache, "kcache")
    _req(vcache, "vcache", dtype=kcache.dtype, shape=kcache.shape)
    _req(pos, "pos", dtype=torch.int32, numel=1)
    _req(part, "part", dtype=torch.float32, numel=nh * nsplit * (hd + 2))
    _req(out, "out", dtype=kcache.dtype, numel=nh * hd)
    _req(tickets, "tickets", dtype=torch.int32, numel=nkv)
    if hd not in (64, 128) or nh % nkv or (nh // nkv) not in (1, 2, 4, 8):
        raise ValueError(f"unsupported attention shape nh={nh} nkv={nkv} hd={hd}")
    check(kernels().cake_attn_decode(_dt(kcache), _p(q), _p(kcache), _p(vcache), _p(pos), S, nh,
                                     nkv, hd, float(scale), _p(part), _p(tickets), _p(out),
                                     _stream()),
          "attn_decode")


def attn_workspace_numel(nh: int, hd: int, S: int) -> int:
    return nh * ((S + 63) // 64) * (hd + 2)


# ---------------------------------------------------------------------------
# prefill / generic
# ---------------------------------------------------------------------------

def embed(table, tok, out):
    V, H = table.shape
    T = tok.numel()
    _req(table, "table")
    _req(tok, "tok", dtype=torch.int32)
    _req(out, "out", dtype=torch.float32, numel=T * H)
    check(kernels().cake_embed(_dt(table), _p(table), _p(tok), T, H, _p(out), _stream()), "embed")


def rmsnorm(x, w, eps, out):
    T, H = x.shape
    _req(x, "x", dtype=torch.float32)
    _req(w, "w", shape=(H,))
    _req(out, "out", dtype=w.dtype, shape=(T, H))
    check(kernels().cake_rmsnorm(_dt(w), _p(x), _p(w), float(eps), T, H, _p(out), _stream()),
          "rmsnorm")


def rope_kv(q, k, v, inv_freq, pos0: int, kcache, vcache):
    """q [T, nh*hd] roped in place; k roped / v copied into cache rows pos0..pos0+T-1."""
    nkv, S, hd = kcache.shape
    T = q.shape[0]
    nh = q.shape[1] // hd
    if pos0 < 0 or pos0 + T > S:
        raise ValueError(f"positions {pos0}..{pos0 + T} exceed cache length {S}")
    _req(q, "q", dtype=kcache.dtype)
    _req(k, "k", dtype=kcache.dtype, shape=(T, nkv * hd))
    _req(v, "v", dtype=kcache.dtype, shape=(T, nkv * hd))
    _req(inv_freq, "inv_freq", dtype=torch.float32, shape=(hd // 2,))
    _req(kcache, "kcache")
    _req(vcache, "vcache", shape=kcache.shape)
    check(kernels().cake_rope_kv(_dt(q), _p(q), _p(k), _p(v), T, nh, nkv, hd, _p(inv_freq),
                                 int(pos0), S, _p(kcache), _p(vcache), _stream()), "rope_kv")


def attn_prefill(q, kcache, vcache, pos0: int, scale: float, out):
    nkv, S, hd = kcache.shape
    T = q.shape[0]
    nh = q.shape[1] // hd
    if pos0 < 0 or pos0 + T > S:
        raise ValueError("positions exceed cache length")
    if hd not in (64, 128) or nh % nkv:
        raise ValueError(f"unsupported attention shape nh={nh} nkv={nkv} hd={hd}")
    _req(q, "q", dtype=kcache.dtype)
    _req(out, "out", dtype=kcache.dtype, shape=q.shape)
    check(kernels().cake_attn_prefill(_dt(q), _p(q), _p(kcache), _p(vcache), int(pos0), T, S,
                                      nh, nkv, hd, float(scale), _p(out), _stream()),
          "attn_prefill")


def silu_mul(g, u, out):
    _req(g, "g")
    _req(u, "u", dtype=g.dtype, shape=g.shape)
    _req(out, "out", dtype=g.dtype, shape=g.shape)
    check(kernels().cake_silu_mul(_dt(g), _p(g), _p(u), g.numel(), _p(out), _stream()),
          "silu_mul")


def add_resid(resid, y):
    _req(resid, "resid", dtype=torch.float32)
    _req(y, "y", numel=resid.numel())
    check(kernels().cake_add_resid(_dt(y), _p(resid), _p(y), resid.numel(), _stream()),
          "add_resid")


# ---------------------------------------------------------------------------
# token selection
# ---------------------------------------------------------------------------

def repeat_penalty(logits, hist, hist_len, last_n: int, penalty: float):
    _req(logits, "logits", dtype=torch.float32)
    _req(hist, "hist", dtype=torch.int32)
    _req(hist_len, "hist_len", dtype=torch.int32, numel=1)
    check(kernels().cake_repeat_penalty(_p(logits), _p(hist), _p(hist_len), int(last_n),
                                        float(penalty), _stream()), "repeat_penalty")


def argmax(logits, slot):
    _req(logits, "logits", dtype=torch.float32)
    _req(slot, "slot", dtype=torch.int64, numel=1)
    check(kernels().cake_argmax(_p(logits), logits.numel(), _p(slot), _stream()), "argmax")


def finalize_token(slot, tok, hist, hist_len, pos):
    for t, n in ((tok, "tok"), (hist, "hist"), (hist_len, "hist_len"), (pos, "pos")):
        _req(t, n, dtype=torch.int32)
    check(kernels().cake_finalize_token(_p(slot), _p(tok), _p(hist), _p(hist_len), _p(pos),
                                        hist.numel(), _stream()), "finalize_token")


def push_token(src, tok, hist, hist_len, pos):
    for t, n in ((src, "src"), (tok, "tok"), (hist, "hist"), (hist_len, "hist_len"),
                 (pos, "pos")):
        _req(t, n, dtype=torch.int32)
    check(kernels().cake_push_token(_p(src), _p(tok), _p(hist), _p(hist_len), _p(pos),
                                    hist.numel(), _stream()), "push_token")


GEMV_KINDS = {"qkv": 0, "swiglu": 1, "x16": 2, "norm_f32": 3}


def set_gemv_tuning(kind: str, U: int = 4, prefetch: int = 0, max_blocks: int = 1024) -> None:
    """Select the decode-GEMV launch geometry for one kernel kind (see gemv.hip)."""
    check(kernels().cake_gemv_set_tuning(GEMV_KINDS[kind], int(U), int(prefetch), int(max_blocks)),
          "gemv_set_tuning")


# ---------------------------------------------------------------------------
# MFMA flash attention + SD normalisation kernels
# ---------------------------------------------------------------------------

def flash_attn(q, k, v, out, scale: float, causal: bool = False, pos0: int = 0):
    """out = softmax(q kᵀ * scale [+causal mask]) v on MFMA.

    All four are 4-D *views* [B, H|Hkv, rows, D] with unit stride on D (any
    batch/head/row strides — e.g. [B, N, H, D] projections viewed as
    .transpose(1, 2), or a KV cache [Hkv, S, D][None]).  GQA when
    Hkv < H.  Causal: query row i sits at absolute position pos0 + i.
    """
    import ctypes
    B, H, N, D = q.shape
    Bk, Hkv, M, Dk = k.shape
    if v.shape != k.shape or Dk != D or Bk != B or tuple(out.shape) != (B, H, N, D):
        raise ValueError(f"flash_attn shapes q{tuple(q.shape)} k{tuple(k.shape)} "
                         f"v{tuple(v.shape)} o{tuple(out.shape)}")
    if H % Hkv or D > 256:
        raise ValueError("flash_attn: H % Hkv != 0 or D > 256")
    for t, n in ((q, "q"), (k, "k"), (v, "v"), (out, "out")):
        if not t.is_cuda or t.dtype != q.dtype or t.stride(3) != 1:
            raise ValueError(f"flash_attn: {n} must be a unit-stride-D device tensor of {q.dtype}")
        if (t.data_ptr() % 16) or (D % 8 == 0 and any(s % 8 for s in t.stride()[:3])):
            raise ValueError(f"flash_attn: {n} not 16-byte aligned for vector loads")
    st = [s for t in (q, k, v, out) for s in t.stride()[:3]]
    arr = (ctypes.c_longlong * 12)(*st)
    check(kernels().cake_flash_attn(_dt(q), _p(q), _p(k), _p(v), _p(out), B, H, Hkv, N, M, D,
                                    ctypes.cast(arr, ctypes.c_void_p), float(scale), int(causal),
                                    int(pos0), _stream()), "flash_attn")


def group_norm(x, gamma, beta, groups: int, eps: float, silu: bool, out):
    """GroupNorm over NCHW (contiguous) [+ fused SiLU]."""
    B, C = x.shape[:2]
    HW = x.numel() // (B * C)
    _req(x, "x")
    _req(gamma, "gamma", dtype=x.dtype, shape=(C,))
    _req(beta, "beta", dtype=x.dtype, shape=(C,))
    _req(out, "out", dtype=x.dtype, shape=x.shape)
    if C % groups:
        raise ValueError("C % groups != 0")
    part = torch.empty(B * groups * 16 * 3, device=x.device, dtype=torch.float32)
    check(kernels().cake_groupnorm(_dt(x), _p(x), _p(gamma), _p(beta), B, C, HW, groups,
                                   float(eps), int(silu), _p(part), _p(out), _stream()),
          "groupnorm")


def layer_norm(x, gamma, beta, eps: float, out):
    C = x.shape[-1]
    _req(x, "x")
    _req(gamma, "gamma", dtype=x.dtype, shape=(C,))
    _req(beta, "beta", dtype=x.dtype, shape=(C,))
    _req(out, "out", dtype=x.dtype, shape=x.shape)
    check(kernels().cake_layernorm(_dt(x), _p(x), _p(gamma), _p(beta), x.numel() // C, C,
                                   float(eps), _p(out), _stream()), "layernorm")


def geglu(h, out):
    F = h.shape[-1] // 2
    _req(h, "h")
    _req(out, "out", dtype=h.dtype, numel=h.numel() // 2)
    check(kernels().cake_geglu(_dt(h), _p(h), h.numel() // (2 * F), F, _p(out), _stream()),
          "geglu")


def attn_oproj_supported(nh: int, nkv: int, hd: int, H: int) -> bool:
    return hd == 128 and nh % nkv == 0 and nh // nkv in (4, 8) and 4096 <= nh * hd <= 8192


def attn_oproj(q, kcache, vcache, pos, scale, part, tickets, ctl, attn_out, wo, resid, err,
               prefetch: bool = True, grid: int | None = None, sleep: int = 1):
    """Fused decode attention + o_proj + residual (decode_fused.hip).

    ctl: int32[3] (ctl[1] must be 0 at launch: qkv_rope(rearm=ctl) zeroes it); err: int32[1].
    """
    nkv, S, hd = kcache.shape
    nh = q.numel() // hd
    N, K = wo.shape
    if not attn_oproj_supported(nh, nkv, hd, N) or K != nh * hd:
        raise ValueError(f"attn_oproj: unsupported shape nh={nh} nkv={nkv} hd={hd} wo={tuple(wo.shape)}")
    _req(q, "q", dtype=torch.float32)
    _req(kcache, "kcache")
    _req(vcache, "vcache", dtype=kcache.dtype, shape=kcache.shape)
    _req(pos, "pos", dtype=torch.int32, numel=1)
    _req(part, "part", dtype=torch.float32, numel=nh * ((S + 63) // 64) * (hd + 2))
    _req(tickets, "tickets", dtype=torch.int32, numel=nkv)
    _req(ctl, "ctl", dtype=torch.int32, numel=3)
    _req(attn_out, "attn_out", dtype=kcache.dtype, numel=nh * hd)
    _req(wo, "wo", dtype=kcache.dtype)
    _req(resid, "resid", dtype=torch.float32, numel=N)
    _req(err, "err", dtype=torch.int32, numel=1)
    if grid is None:
        grid = max(1, ((N + 1) // 2 + 3) // 4)
    check(kernels().cake_attn_oproj(_dt(kcache), _p(q), _p(kcache), _p(vcache), _p(pos), S, nh,
                                    nkv, hd, float(scale), _p(part), _p(tickets), _p(ctl),
                                    _p(attn_out), _p(wo), N, _p(resid), _p(err), int(grid),
                                    int(prefetch), int(sleep), _stream()),
          "attn_oproj")
