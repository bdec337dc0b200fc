"""Torch-tensor wrappers around the gfx950 HIP kernels.

Every wrapper validates shapes / dtypes / contiguity / device on the host
*before* launching (a bad pointer or shape on the GPU can take down the box),
then launches on torch's current stream.  No wrapper falls back to PyTorch: if
the kernel library is missing, :func:`cake_amd.ops._lib.kernels` raises.
"""
from __future__ import annotations

import ctypes as C

import os
import threading

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

def qkv_rope(resid, norm_w, eps, wq, wk, wv, inv_freq, pos, q_out, kcache, vcache):
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
                                  _p(kcache), _p(vcache), S, _stream()),
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


HEAD_SELECT_MAX_LAST_N = 256


def head_select(resid, norm_w, eps, w, logits, hist, hist_len, last_n: int, penalty: float,
                slot, ticket, tok, pos, embed=None) -> None:
    """Greedy decode tail in ONE launch (gemv.hip cake_head_select): logits = lm_head(
    rmsnorm(resid)), repeat penalty over the last `last_n` (<= 256) history tokens, argmax
    (ties -> smallest id), then tok / history / pos advanced as finalize_token does.
    With `embed` (the [V, H] table) the launch also writes the next step's input,
    resid = embed[tok] (f32), as :func:`embed` would.  slot (int64[1]) and ticket
    (int32[1]) start at zero; the kernel re-arms them."""
    N, K = w.shape
    _req(resid, "resid", dtype=torch.float32, numel=K)
    _req(norm_w, "norm_w", dtype=w.dtype, shape=(K,))
    _req(w, "w")
    _req(logits, "logits", dtype=torch.float32, numel=N)
    _req(slot, "slot", dtype=torch.int64, numel=1)
    _req(ticket, "ticket", dtype=torch.int32, numel=1)
    for t, n in ((tok, "tok"), (hist, "hist"), (hist_len, "hist_len"), (pos, "pos")):
        _req(t, n, dtype=torch.int32)
    if not 0 <= int(last_n) <= HEAD_SELECT_MAX_LAST_N:
        raise ValueError(f"head_select: last_n {last_n} > {HEAD_SELECT_MAX_LAST_N}")
    if embed is not None:
        _req(embed, "embed", dtype=w.dtype)
        if embed.dim() != 2 or embed.shape[1] != K:
            raise ValueError(f"head_select: embed {tuple(embed.shape)} does not match H={K}")
    check(kernels().cake_head_select(_dt(w), _p(resid), _p(norm_w), float(eps), _p(w), K, N,
                                     _p(logits), _p(hist), _p(hist_len), int(last_n),
                                     float(penalty), _p(slot), _p(ticket), _p(tok), _p(pos),
                                     hist.numel(), None if embed is None else _p(embed),
                                     None if embed is None else _p(resid), _stream()),
          "head_select")


def attn_oproj_supported(nh: int, nkv: int, hd: int, H: int) -> bool:
    """Shapes of the fused decode attention + o_proj launch (csrc/experimental/attn_oproj.hip,
    built with CAKE_BUILD_EXPERIMENTAL=1; False when the library was built without it)."""
    L = kernels()
    if not hasattr(L, "cake_attn_oproj_supported"):
        return False
    return bool(L.cake_attn_oproj_supported(int(nh), int(nkv), int(hd), int(H)))


def attn_oproj_ws_sizes(nkv: int, H: int) -> tuple[int, int]:
    """(f32 words of the {partial, tag} granules, int32 ticket / epoch words) of its
    workspace."""
    return 2 * nkv * H, 2 * (H // 32) + 2 * nkv + 2


def attn_oproj(q, kcache, vcache, pos, scale, wo, out, accumulate: bool, ws, tickets,
               err_tickets=None):
    """Decode attention + o_proj in ONE launch (short contexts: the attention runs as one
    split): out (+)= W_o . attention(q, K, V).  wo [H, nh*hd] (this rank's columns);
    ws f32, tickets int32 (:func:`attn_oproj_ws_sizes`, zeroed once); err_tickets: the
    attention tickets whose error word [2 nkv] a partial poll that gave up sets."""
    nkv, S, hd = kcache.shape
    nh = q.numel() // hd
    H = wo.shape[0]
    _req(q, "q", dtype=torch.float32)
    _req(kcache, "kcache")
    _req(vcache, "vcache", dtype=kcache.dtype, shape=kcache.shape)
    _req(pos, "pos", dtype=torch.int32, numel=1)
    _req(wo, "wo", dtype=kcache.dtype, shape=(H, nh * hd))
    _req(out, "out", dtype=torch.float32, numel=H)
    nws, ntk = attn_oproj_ws_sizes(nkv, H)
    _req(ws, "ws", dtype=torch.float32, numel=nws)
    _req(tickets, "tickets", dtype=torch.int32, numel=ntk)
    if not attn_oproj_supported(nh, nkv, hd, H):
        raise ValueError(f"attn_oproj: unsupported shape nh={nh} nkv={nkv} hd={hd} H={H}")
    check(kernels().cake_attn_oproj(_dt(kcache), _p(q), _p(kcache), _p(vcache), _p(pos), S, nh,
                                    nkv, hd, float(scale), _p(wo), nh * hd, H, _p(out),
                                    int(bool(accumulate)), _p(ws), _p(tickets),
                                    None if err_tickets is None else
                                    err_tickets.data_ptr() + 4 * 2 * nkv, _stream()),
          "attn_oproj")


_AO_FUSED = threading.local()


class attn_oproj_fused:
    """Context: decode steps recorded / run inside use the fused attention + o_proj
    launch (the short-context graph bucket; eager steps at a short live length)."""

    def __init__(self, on: bool = True):
        self.on = bool(on)

    def __enter__(self):
        self.prev = getattr(_AO_FUSED, "on", False)
        _AO_FUSED.on = self.on
        return self

    def __exit__(self, *exc):
        _AO_FUSED.on = self.prev
        return False


def attn_oproj_active() -> bool:
    return getattr(_AO_FUSED, "on", False)


def attn_oproj_short(pos: int) -> bool:
    """An eager step at device position `pos` takes the fused launch exactly when a
    one-step graph replay there would (its bucket: one attention split at pos + 2)."""
    return attn_splits(int(pos) + 2) == 1


def attn_decode(q, kcache, vcache, pos, scale, part, tickets, out):
    """Split-K GQA decode attention for the token at device position `pos`.

    The split count is derived on the device from the live length, so one
    captured launch serves every position.  part: f32 workspace
    (:func:`attn_workspace_numel`) and tickets: int32 [2 nkv + 2], both zero-initialised
    once, together, and maintained by the kernel itself (core 1: arrival tickets,
    re-armed; core 2: per-kv-head epochs that tag the published partials; word 2 nkv is
    the error word a timed-out merge sets — :func:`attn_error`).
    """
    nkv, S, hd = kcache.shape
    nh = q.numel() // hd
    _req(q, "q", dtype=torch.float32)
    _req(kcache, "kcache")
    _req(vcache, "vcache", dtype=kcache.dtype, shape=kcache.shape)
    _req(pos, "pos", dtype=torch.int32, numel=1)
    _req(part, "part", dtype=torch.float32, numel=attn_workspace_numel(nh, hd, S))
    _req(out, "out", dtype=kcache.dtype, numel=nh * hd)
    _req(tickets, "tickets", dtype=torch.int32, numel=2 * nkv + 2)
    if hd not in (64, 128) or nh % nkv or (nh // nkv) not in (1, 2, 4, 8):
        raise ValueError(f"unsupported attention shape nh={nh} nkv={nkv} hd={hd}")
    if not _ATTN_IMPL_SET[0]:  # CAKE_ATTN_IMPL / CAKE_ATTN_TARGET, applied once
        attn_set_impl(_ATTN_IMPL[0])
        if os.environ.get("CAKE_ATTN_TARGET"):
            attn_set_target_splits(int(os.environ["CAKE_ATTN_TARGET"]))
        if os.environ.get("CAKE_ATTN_SINGLE"):
            attn_set_single_max(int(os.environ["CAKE_ATTN_SINGLE"]))
        if os.environ.get("CAKE_ATTN_PREFETCH"):
            attn_set_prefetch(int(os.environ["CAKE_ATTN_PREFETCH"]))
    check(kernels().cake_attn_decode(_dt(kcache), _p(q), _p(kcache), _p(vcache), _p(pos), S,
                                     nh, nkv, hd, float(scale), _p(part), _p(tickets),
                                     _p(out), _stream()),
          "attn_decode")


def attn_decode_heads(q, kcache, vcache, pos, scale, out, waves: int = 2, prefetch: int = 2):
    """Head-parallel short-context decode attention (attention.hip attn_head_kernel): one
    workgroup per query head, the whole live length as one split; no workspace."""
    nkv, S, hd = kcache.shape
    nh = q.numel() // hd
    _req(q, "q", dtype=torch.float32)
    _req(kcache, "kcache")
    _req(vcache, "vcache", dtype=kcache.dtype, shape=kcache.shape)
    _req(pos, "pos", dtype=torch.int32, numel=1)
    _req(out, "out", dtype=kcache.dtype, numel=nh * hd)
    if hd not in (64, 128) or nh % nkv:
        raise ValueError(f"unsupported attention shape nh={nh} nkv={nkv} hd={hd}")
    L = kernels()
    prev = int(L.cake_attn_heads_max())
    check(L.cake_attn_set_heads(max(prev, 1), int(waves)), "attn_set_heads")
    check(L.cake_attn_set_head_prefetch(int(prefetch)), "attn_set_head_prefetch")
    check(L.cake_attn_decode_heads(_dt(kcache), _p(q), _p(kcache), _p(vcache), _p(pos), S, nh,
                                   nkv, hd, float(scale), _p(out), _stream()),
          "attn_decode_heads")
    check(L.cake_attn_set_heads(prev, 2), "attn_set_heads")
    check(L.cake_attn_set_head_prefetch(2), "attn_set_head_prefetch")


# ---------------------------------------------------------------------------
# persistent decode (decode_mk.hip): every layer of one token in one launch
# ---------------------------------------------------------------------------

MK_LAYER_PTRS = 8  # ln1, wqkv, wo, ln2, wgu, wd, kc, vc
MK_CTL_WORDS = 4   # epoch, exit ticket, error flag, error site


def mk_available() -> bool:
    """The persistent decode engine was built (csrc/experimental, CAKE_BUILD_EXPERIMENTAL=1)."""
    return hasattr(kernels(), "cake_mk_decode")


def mk_supported(H: int, I: int, nh: int, nkv: int, hd: int) -> bool:
    """Shapes the persistent decode kernel handles on this device (H, I, nh*hd
    multiples of 512; head_dim 128; GQA group 4 or 8); False when it is not built."""
    if not mk_available():
        return False
    return kernels().cake_mk_supported(int(H), int(I), int(nh), int(nkv), int(hd)) == 0


def mk_gstride(H: int, I: int, nh: int, nkv: int, hd: int) -> int:
    """Granule words (8 bytes) per layer of the persistent-decode workspace."""
    return int(kernels().cake_mk_gstride(int(H), int(I), int(nh), int(nkv), int(hd)))


def mk_decode(dtype, table, n_layers: int, H: int, I: int, nh: int, nkv: int, hd: int, S: int,
              eps: float, scale: float, inv_freq, pos, resid, gran, ctl,
              timeout_s: float = 2.0) -> None:
    """One decode token through `n_layers` layers in ONE launch (decode_mk.hip).

    table: int64 [n_layers, 8] device pointers (ln1, wqkv, wo, ln2, wgu, wd, kc, vc);
    resid: f32 [H] — the layer-0 input, overwritten with the last layer's output;
    gran: int64 [n_layers * mk_gstride(...)] and ctl: int32 [4], both zeroed once
    (the kernel keeps them consistent across launches; a bounded spin that gives up
    sets ctl[2] — see :func:`mk_error`)."""
    _req(table, "table", dtype=torch.int64, shape=(n_layers, MK_LAYER_PTRS))
    _req(inv_freq, "inv_freq", dtype=torch.float32, shape=(hd // 2,))
    _req(pos, "pos", dtype=torch.int32, numel=1)
    _req(resid, "resid", dtype=torch.float32, numel=H)
    _req(gran, "gran", dtype=torch.int64, numel=n_layers * mk_gstride(H, I, nh, nkv, hd))
    _req(ctl, "ctl", dtype=torch.int32, numel=MK_CTL_WORDS)
    if not mk_supported(H, I, nh, nkv, hd):
        raise ValueError(f"persistent decode does not support H={H} I={I} nh={nh} "
                         f"nkv={nkv} hd={hd}")
    check(kernels().cake_mk_decode(_DT[dtype], _p(table), int(n_layers), int(H), int(I), int(nh),
                                   int(nkv), int(hd), int(S), float(eps), float(scale),
                                   _p(inv_freq), _p(pos), _p(resid), _p(gran), _p(ctl),
                                   float(timeout_s), _stream()),
          "mk_decode")


def mk_error(ctl) -> int:
    """Nonzero site code when a persistent-decode spin gave up (host sync)."""
    c = ctl.cpu()
    return int(c[3]) if int(c[2]) != 0 else 0


def attn_error(tickets) -> bool:
    """True when a split-K merge of :func:`attn_decode` gave up waiting for the
    partials of its other splits (the error word after the 2 nkv tickets; host sync)."""
    return int(tickets[-2].item()) != 0


def attn_clear_error(tickets) -> None:
    """Re-arm the error word after it was reported (the kernels never clear it)."""
    tickets[-2].zero_()


def attn_debug_drop_partials(on: bool) -> None:
    """Test hook: core 2's splits >= 1 stop publishing, so the merges time out."""
    check(kernels().cake_attn_debug_drop_partials(int(bool(on))), "attn_debug_drop_partials")


def attn_workspace_numel(nh: int, hd: int, S: int) -> int:
    """f32 elements of the partials of at most 64 splits per head (attention.hip
    kMaxSplit): core 2 stores each value as an 8-byte {value, tag} granule."""
    del S
    return 2 * nh * 64 * (hd + 2)


_ATTN_MIN_KEYS = [64]


def attn_set_min_keys(n: int) -> None:
    """Minimum keys per decode-attention split (multiple of 64; default 64)."""
    check(kernels().cake_attn_set_min_keys(int(n)), "attn_set_min_keys")
    _ATTN_MIN_KEYS[0] = int(n)


def attn_max_split(S: int) -> int:
    """Splits per kv head of a max_seq = S launch (attention.hip attn_max_split)."""
    return min((S + 63) // 64, 64)


def attn_splits(Tk: int) -> int:
    """Splits the decode-attention kernel uses at live length Tk with no cap (the
    device-side policy of attn_core.h, mirrored for choosing a capped graph)."""
    Tk = max(int(Tk), 1)
    if _ATTN_IMPL[0] == 2:  # attn_core2.h attn2_splits
        if Tk <= _ATTN_SINGLE[0]:
            return 1
        keys = max(_ATTN_MIN_KEYS[0], -(-(-(-Tk // _ATTN_TARGET[0])) // 16) * 16)
        ns = min(-(-Tk // keys), 64)
        kps = -(-(-(-Tk // ns)) // 16) * 16
        return -(-Tk // kps)
    keys = max(_ATTN_MIN_KEYS[0], 128 if Tk > 1024 else 64, -(-Tk // 64))
    return -(-Tk // keys)


_ATTN_TARGET = [16]
_ATTN_SINGLE = [320]


def attn_set_single_max(keys: int) -> None:
    """Core 2: live lengths up to `keys` run as one split per kv head (no merge)."""
    check(kernels().cake_attn_set_single_max(int(keys)), "attn_set_single_max")
    _ATTN_SINGLE[0] = int(keys)


def attn_set_prefetch(depth: int) -> None:
    """Core 2: key blocks per wave in flight (1 or 2; 0 = by split cap, the default)."""
    check(kernels().cake_attn_set_prefetch(int(depth)), "attn_set_prefetch")


def attn_set_target_splits(n: int) -> None:
    """Core 2: splits per kv head aimed at (keys per split = ceil(Tk / n), >= min_keys)."""
    check(kernels().cake_attn_set_target_splits(int(n)), "attn_set_target_splits")
    _ATTN_TARGET[0] = int(n)


_ATTN_IMPL = [int(os.environ.get("CAKE_ATTN_IMPL", "2"))]
_ATTN_IMPL_SET = [False]


def attn_set_impl(impl: int) -> None:
    """Decode-attention core: 1 = LDS-staged chunks (attn_core.h), 2 = wave-stream MFMA
    (attn_core2.h).  Graphs captured before a change keep the core they recorded."""
    check(kernels().cake_attn_set_impl(int(impl)), "attn_set_impl")
    _ATTN_IMPL[0] = int(impl)
    _ATTN_IMPL_SET[0] = True


def attn_split_caps(max_seq: int) -> list[int]:
    """Position-bucket split caps a decode graph set needs for live lengths up to max_seq:
    the 8/16/32/64 caps (clamped to the max_seq grid) up to the first that covers every
    live length's split count under the current policy (core 2 at a 16-split target
    needs 8 and 16 only)."""
    full = attn_max_split(max_seq)
    need = max(attn_splits(t) for t in range(1, max_seq + 1))
    caps = []
    for c in (8, 16, 32, 64):
        caps.append(min(c, full))
        if c >= need:
            break
    return sorted(set(caps))


class attn_split_cap:
    """Context manager: decode-attention launches (and graph captures) inside it use at
    most `cap` splits per kv head (correct at any live length; fastest where
    attn_splits(Tk) <= cap)."""

    def __init__(self, cap: int):
        self.cap = int(cap)

    def __enter__(self):
        check(kernels().cake_attn_set_split_cap(self.cap), "attn_set_split_cap")
        return self

    def __exit__(self, *exc):
        check(kernels().cake_attn_set_split_cap(0), "attn_set_split_cap")
        return False


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


def _rows(t: torch.Tensor, name: str, cols: int, T: int, dtype) -> int:
    """Validate a [T, cols] row-strided view (unit column stride); return its row stride."""
    if not t.is_cuda or t.dtype != dtype or t.dim() != 2 or tuple(t.shape) != (T, cols) \
            or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a [{T}, {cols}] {dtype} device view with unit "
                         f"column stride, got {tuple(t.shape)} {t.dtype} strides {t.stride()}")
    return t.stride(0)


def rope_kv(q, k, v, inv_freq, pos0: int, kcache, vcache):
    """q [T, nh*hd] roped in place; k roped / v copied into cache rows pos0..pos0+T-1.

    q, k, v may be column slices of one fused [T, (nh + 2 nkv) hd] projection
    or separate contiguous tensors (k and v share a row stride)."""
    nkv, S, hd = kcache.shape
    T = q.shape[0]
    nh = q.shape[1] // hd
    if pos0 < 0 or pos0 + T > S:
        raise ValueError(f"positions {pos0}..{pos0 + T} exceed cache length {S}")
    ldq = _rows(q, "q", nh * hd, T, kcache.dtype)
    ld = _rows(k, "k", nkv * hd, T, kcache.dtype)
    if _rows(v, "v", nkv * hd, T, kcache.dtype) != ld and T > 1:
        raise ValueError("rope_kv: k and v need the same row stride")
    _req(inv_freq, "inv_freq", dtype=torch.float32, shape=(hd // 2,))
    _req(kcache, "kcache")
    _req(vcache, "vcache", shape=kcache.shape)
    check(kernels().cake_rope_kv(_dt(q), _p(q), _p(k), _p(v), ldq, ld, T, nh, nkv, hd, _p(inv_freq),
                                 int(pos0), S, _p(kcache), _p(vcache), _stream()), "rope_kv")


def silu_mul(g, u, out):
    _req(g, "g")
    _req(u, "u", dtype=g.dtype, shape=g.shape)
    _req(out, "out", dtype=g.dtype, shape=g.shape)
    check(kernels().cake_silu_mul(_dt(g), _p(g), _p(u), g.numel(), _p(out), _stream()),
          "silu_mul")


def silu_mul_rows(gu, out):
    """out [T, I] = silu(gu[:, :I]) * gu[:, I:]  (fused gate|up projection output)."""
    T, I2 = gu.shape
    _req(gu, "gu")
    _req(out, "out", dtype=gu.dtype, shape=(T, I2 // 2))
    check(kernels().cake_silu_mul_rows(_dt(gu), _p(gu), T, I2 // 2, _p(out), _stream()),
          "silu_mul_rows")


def add_resid(resid, y):
    _req(resid, "resid", dtype=torch.float32)
    _req(y, "y", numel=resid.numel())
    check(kernels().cake_add_resid(_dt(y), _p(resid), _p(y), resid.numel(), _stream()),
          "add_resid")


def stream_read(buf, blocks, sink, nbytes=None):
    """Bandwidth probe: read ``nbytes`` (default all) of ``buf`` and nothing else."""
    _req(buf, "buf")
    _req(sink, "sink", dtype=torch.int32)
    n = buf.numel() * buf.element_size() if nbytes is None else int(nbytes)
    check(kernels().cake_stream_read(_p(buf), n, int(blocks), _p(sink), _stream()),
          "stream_read")


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


def sample_threshold(logits, temperature: float, top_k: int | None, top_p: float | None, thr):
    """thr (int32[1]) <- order key of the least logit in the top-k / top-p set."""
    _req(logits, "logits", dtype=torch.float32)
    _req(thr, "thr", dtype=torch.int32, numel=1)
    check(kernels().cake_sample_threshold(_p(logits), logits.numel(), float(temperature),
                                          int(top_k or 0), float(top_p or 0.0), _p(thr),
                                          _stream()), "sample_threshold")


def gumbel_argmax(logits, temperature: float, seed: int, step, slot, thr=None):
    """slot <- argmax_i(logits_i / T + Gumbel_i) over logits keys >= thr: one draw from
    softmax(logits / T) restricted to the set (Philox(seed; i, *step) variates)."""
    _req(logits, "logits", dtype=torch.float32)
    _req(step, "step", dtype=torch.int32, numel=1)
    _req(slot, "slot", dtype=torch.int64, numel=1)
    if thr is not None:
        _req(thr, "thr", dtype=torch.int32, numel=1)
    check(kernels().cake_gumbel_argmax(_p(logits), logits.numel(), float(temperature),
                                       int(seed) & 0xFFFFFFFFFFFFFFFF, _p(step), _p(thr),
                                       _p(slot), _stream()), "gumbel_argmax")


SAMPLE_PARAMS_WORDS = 8


def sample_params_tensor(sampling, device) -> torch.Tensor:
    """Pack a SamplingConfig (None = greedy) into the 32-byte device SampleParams."""
    return pack_sample_params(sampling).to(device)


def pack_sample_params(sampling) -> torch.Tensor:
    import struct
    if sampling is None or sampling.greedy:
        t, k, p, seed = 0.0, 0, 0.0, 0
    else:
        t = float(sampling.temperature)
        k = int(sampling.top_k) if sampling.top_k else 0
        p = float(sampling.top_p) if sampling.top_p is not None else 0.0
        seed = int(sampling.seed) & 0xFFFFFFFFFFFFFFFF
    raw = struct.pack("<fif2I3I", t, k, p, seed & 0xFFFFFFFF, seed >> 32, 0, 0, 0)
    return torch.frombuffer(bytearray(raw), dtype=torch.int32).clone()


def select_token(logits, slot, hist, hist_len, tok, pos, sampling=None, thr=None, params=None):
    """Device token selection of one decode step: argmax (greedy) or a seeded draw
    (temperature / top-k / top-p), then the step finalizer (tok, history, pos).
    params (int32[8] device SampleParams): the sampling configuration is read on the
    device instead (temperature <= 0 = greedy), so it can change between graph replays."""
    if params is not None:
        _req(params, "params", dtype=torch.int32, numel=SAMPLE_PARAMS_WORDS)
        _req(thr, "thr", numel=1)
        _req(hist_len, "hist_len", dtype=torch.int32)
        check(kernels().cake_select_dev(_p(logits), logits.numel(), _p(params), _p(hist_len),
                                        _p(thr), _p(slot), _stream()), "select_dev")
    elif sampling is None or sampling.greedy:
        argmax(logits, slot)
    else:
        restrict = (sampling.top_k is not None and sampling.top_k > 0) or \
            (sampling.top_p is not None and 0.0 < sampling.top_p < 1.0)
        if restrict:
            sample_threshold(logits, sampling.temperature, sampling.top_k, sampling.top_p, thr)
        gumbel_argmax(logits, sampling.temperature, sampling.seed, hist_len, slot,
                      thr if restrict else None)
    finalize_token(slot, tok, hist, hist_len, pos)


def select_shard(logits, off: int, hist, hist_len, last_n: int, penalty: float,
                 temperature: float, seed: int, slot):
    """Tensor-parallel vocab shard (global ids [off, off + len(logits))): repeat penalty
    on the shard, then its argmax / Gumbel-max key into slot (all-reduce max next)."""
    _req(logits, "logits", dtype=torch.float32)
    _req(slot, "slot", dtype=torch.int64, numel=1)
    check(kernels().cake_select_shard(_p(logits), logits.numel(), int(off), _p(hist),
                                      _p(hist_len), int(last_n), float(penalty),
                                      float(temperature or 0.0),
                                      int(seed) & 0xFFFFFFFFFFFFFFFF, _p(slot), _stream()),
          "select_shard")


def ar_sum(partial, out, accumulate: bool, peers, inbox: int, seq, err, rank: int, world: int,
           timeout_s: float):
    """out (+)= all-reduce-sum of the f32 vector partial over the TP ranks (allreduce.hip).
    peers: ctypes array of the peers' inbox pointers; inbox: this rank's inbox."""
    _req(partial, "partial", dtype=torch.float32)
    _req(out, "out", dtype=torch.float32, numel=partial.numel())
    check(kernels().cake_ar_sum(_p(partial), _p(out), partial.numel(), int(bool(accumulate)),
                                peers, C.c_void_p(inbox), _p(seq), _p(err), int(rank),
                                int(world), float(timeout_s), _stream()), "ar_sum")


def ar_max_key(slot, peers, inbox: int, seq, err, rank: int, world: int, timeout_s: float):
    """slot (u64 argmax key) <- max over the TP ranks."""
    _req(slot, "slot", dtype=torch.int64, numel=1)
    check(kernels().cake_ar_max_key(_p(slot), peers, C.c_void_p(inbox), _p(seq), _p(err),
                                    int(rank), int(world), float(timeout_s), _stream()),
          "ar_max_key")


def ar_gather(shard, off: int, full, peers, inbox: int, seq, err, rank: int, world: int,
              timeout_s: float):
    """full (f32[V], every rank) <- the TP ranks' contiguous vocabulary shards; this
    rank's shard covers full[off:off + shard.numel()]."""
    _req(shard, "shard", dtype=torch.float32)
    _req(full, "full", dtype=torch.float32)
    if off < 0 or off + shard.numel() > full.numel():
        raise ValueError("shard outside the gathered vector")
    check(kernels().cake_ar_gather(_p(shard), int(off), shard.numel(), _p(full), full.numel(),
                                   peers, C.c_void_p(inbox), _p(seq), _p(err), int(rank),
                                   int(world), float(timeout_s), _stream()), "ar_gather")


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


GEMV_KINDS = {"qkv": 0, "swiglu": 1, "x16": 2, "norm_f32": 3, "x16s": 4}  # x16s: K <= 8192


def set_gemv_tuning(kind: str, U: int = 4, prefetch: int = 0, max_blocks: int = 1024) -> None:
    """Select the decode-GEMV launch geometry for one kernel kind (see gemv.hip)."""
    check(kernels().cake_gemv_set_tuning(GEMV_KINDS[kind], int(U), int(prefetch), int(max_blocks)),
          "gemv_set_tuning")



# ---------------------------------------------------------------------------
# MFMA flash attention + SD normalisation kernels
# ---------------------------------------------------------------------------

def flash_set_impl(v: int) -> None:
    """1 = 16-row 16x16x32 kernel, 2 = 32x32x16 swapped-QKᵀ kernel (default where shapes allow)."""
    kernels().cake_flash_set_impl(int(v))


def flash_set_pair_min(n: int) -> None:
    """Causal flash (v2): pair q tiles x / n-1-x per workgroup once the unpaired grid has
    at least n workgroups (default 512; <= 0 never pairs)."""
    kernels().cake_flash_set_pair_min(int(n))


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
    ws, nbytes = None, 0
    if not causal:  # room for up to 4 key splits (the kernel picks; flash_attn.hip)
        ws = _flash_ws(q.device, 4 * B * H * N * (D + 1))
        nbytes = ws.numel() * 4
    check(kernels().cake_flash_attn_ws(_dt(q), _p(q), _p(k), _p(v), _p(out), B, H, Hkv, N, M, D,
                                       ctypes.cast(arr, ctypes.c_void_p), float(scale),
                                       int(causal), int(pos0), _p(ws), nbytes, _stream()),
          "flash_attn")


_flash_wsd: dict = {}
_flash_ws_keep: list = []


def _flash_ws(dev, numel: int) -> torch.Tensor:
    """f32 partial rows of the key-split flash path, one buffer per (device, stream): the
    launches of one stream are serialized, so they may share it; work on another stream
    (a graph captured on torch's capture stream, a side stream) gets its own.  A graph
    replayed later must be replayed on the stream order it was captured in (the usual
    single-stream replay).  Superseded buffers stay alive: a captured hipGraph may still
    point at them."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    w = _flash_wsd.get(key)
    if w is None or w.numel() < numel:
        if w is not None:
            _flash_ws_keep.append(w)
        w = _flash_wsd[key] = torch.empty(numel, dtype=torch.float32, device=dev)
    return w


def flash_set_ksplit(k: int) -> None:
    """Key splits of non-causal flash attention: 0 auto, 1 off, 2 / 4 forced (tests / A-B)."""
    kernels().cake_flash_set_ksplit(int(k))


_zero16: dict = {}


def attn512(q, k, v, out, scale: float):
    """Single-head attention with head dim 512 (VAE mid-block): q/out [B, N, 512],
    k/v [B, M, 512] 16-bit views with unit column stride (attn512.hip)."""
    B, N, D = q.shape
    Bk, M, Dk = k.shape
    if D != 512 or Dk != 512 or Bk != B or v.shape != k.shape or tuple(out.shape) != (B, N, D):
        raise ValueError(f"attn512 shapes q{tuple(q.shape)} k{tuple(k.shape)} v{tuple(v.shape)}")
    for t, n in ((q, "q"), (k, "k"), (v, "v"), (out, "out")):
        if not t.is_cuda or t.dtype != q.dtype or t.stride(2) != 1 or t.data_ptr() % 16 or \
                t.stride(1) % 8:
            raise ValueError(f"attn512: {n} must be a 16-byte aligned unit-stride {q.dtype} view")
    z = _zero16.get(q.device)
    if z is None:
        z = _zero16[q.device] = torch.zeros(64, dtype=torch.int32, device=q.device)
    check(kernels().cake_attn512(_dt(q), _p(q), _p(k), _p(v), _p(out), B, N, M, q.stride(1),
                                 k.stride(1), v.stride(1), out.stride(1), q.stride(0),
                                 k.stride(0), v.stride(0), out.stride(0), float(scale), _p(z),
                                 _stream()), "attn512")


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


_gn_tickets: dict = {}


def group_norm_nhwc_supported(C: int, groups: int) -> bool:
    cg = C // groups
    return C % groups == 0 and C % 8 == 0 and C <= 4096 and cg >= 4 and (cg >= 8 or 8 % cg == 0)


def group_norm_nhwc(x, gamma, beta, groups: int, eps: float, silu: bool, out, skip=None,
                    cat_out=None):
    """GroupNorm over channels-last x [N, ..., C] (contiguous) [+ fused SiLU].

    skip [N, ..., Cs]: normalise the channel concatenation x ++ skip without
    materialising it first (the UNet up path); cat_out [N, ..., C + Cs] then
    optionally receives the raw concatenation (written by the same pass)."""
    N, Cx = x.shape[0], x.shape[-1]
    HW = x.numel() // (N * Cx)
    _req(x, "x")
    C = Cx
    if skip is not None:
        _req(skip, "skip", dtype=x.dtype)
        if skip.shape[:-1] != x.shape[:-1]:
            raise ValueError(f"group_norm_nhwc: skip {tuple(skip.shape)} vs x {tuple(x.shape)}")
        C = Cx + skip.shape[-1]
    oshape = (*x.shape[:-1], C)
    _req(gamma, "gamma", dtype=x.dtype, shape=(C,))
    _req(beta, "beta", dtype=x.dtype, shape=(C,))
    _req(out, "out", dtype=x.dtype, shape=oshape)
    if cat_out is not None:
        if skip is None:
            raise ValueError("group_norm_nhwc: cat_out needs a skip source")
        _req(cat_out, "cat_out", dtype=x.dtype, shape=oshape)
    if not group_norm_nhwc_supported(C, groups) or Cx % 8:
        raise ValueError(f"group_norm_nhwc: unsupported C={C} (x {Cx}) groups={groups}")
    S = kernels().cake_groupnorm_nhwc_splits(HW)
    t = _gn_tickets.get(x.device)
    if t is None or t.numel() < N:
        t = _gn_tickets[x.device] = torch.zeros(max(N, 64), device=x.device, dtype=torch.int32)
    part = torch.empty(N * S * groups * 2, device=x.device, dtype=torch.float64)
    stats = torch.empty(N * groups * 2, device=x.device, dtype=torch.float32)
    check(kernels().cake_groupnorm_nhwc2(_dt(x), _p(x), None if skip is None else _p(skip), Cx,
                                         None if cat_out is None else _p(cat_out), _p(gamma),
                                         _p(beta), N, HW, C, groups, float(eps), int(silu),
                                         _p(part), _p(t), _p(stats), _p(out), _stream()),
          "groupnorm_nhwc")


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


# ---------------------------------------------------------------------------
# implicit-GEMM convolution (conv2d.hip), NHWC activations
# ---------------------------------------------------------------------------

# cfg ids 0-3: register-staged LDS tiles; 4-7: the same tiles staged by LDS-DMA
_CONV_TILES = ((128, 128), (64, 128), (128, 64), (64, 64)) * 2  # (oc, pixel) tile per cfg
_CONV_SLOTS = (2, 3, 3, 5) * 2        # resident workgroups per CU (VGPR/LDS bound)
_CONV_EFF = (1.0, 0.8, 0.8, 0.6) * 2  # relative MFMA efficiency of the tile shapes
_CONV_CFGS = (0, 1, 2, 3)             # planner candidates
_NUM_CUS = 256
_zero_lines: dict = {}


def _zeros16(dev) -> torch.Tensor:
    z = _zero_lines.get(dev)
    if z is None:
        z = _zero_lines[dev] = torch.zeros(64, dtype=torch.int32, device=dev)
    return z


def conv_supported(IC: int, OC: int, stride: int = 1, up: bool = False, k: int = 3) -> bool:
    if IC in (3, 4):  # direct small-IC kernel (conv_in)
        return k == 3 and OC % 8 == 0 and 9 * IC * OC <= 18432 and not up
    return IC % 64 == 0 and OC % 4 == 0 and not (up and stride != 1)


def conv1x1_small(x, w, bias=None, out=None, *, in_nchw: bool = False, out_nchw: bool = False):
    """1x1 convolution with IC, OC <= 16 (conv2d.hip conv1x1_small_kernel): x [N,H,W,IC]
    (or [N,IC,H,W] with in_nchw), w [OC, IC] (or [OC, IC, 1, 1]) -> [N,H,W,OC] (or
    [N,OC,H,W] with out_nchw)."""
    if in_nchw:
        N, IC, H, W = x.shape
    else:
        N, H, W, IC = x.shape
    OC = w.shape[0]
    if w.numel() != OC * IC or not (1 <= IC <= 16 and 1 <= OC <= 16):
        raise ValueError(f"conv1x1_small: unsupported IC={IC} OC={OC} w={tuple(w.shape)}")
    _req(x, "x")
    _req(w, "w", dtype=x.dtype)
    if bias is not None:
        _req(bias, "bias", dtype=x.dtype, numel=OC)
    oshape = (N, OC, H, W) if out_nchw else (N, H, W, OC)
    if out is None:
        out = torch.empty(*oshape, device=x.device, dtype=x.dtype)
    _req(out, "out", dtype=x.dtype, shape=oshape)
    check(kernels().cake_conv1x1_small(_dt(x), _p(x), _p(w), None if bias is None else _p(bias),
                                       _p(out), N, H * W, IC, OC,
                                       int(in_nchw) | (int(out_nchw) << 1), _stream()),
          "conv1x1_small")
    return out


_HALO_TILES = {256: ((16, 16), (8, 32), (32, 8)),
               128: ((8, 16), (16, 8), (10, 12), (12, 10)), 64: ((8, 8), (4, 16), (16, 4))}


def halo_tile(OH: int, OW: int, bn: int) -> tuple[int, int]:
    """Spatial output tile (th, tw), th*tw <= bn, with the least padded area."""
    return min(_HALO_TILES[bn], key=lambda t: (-(-OH // t[0]) * t[0] * -(-OW // t[1]) * t[1],
                                                -t[1]))


def conv_plan(P: int, OC: int, ksteps: int) -> tuple[int, int]:
    """(tile cfg, split-K) minimising a waves-of-tiles cost model."""
    best = None
    for cfg in _CONV_CFGS:
        bm, bn = _CONV_TILES[cfg]
        tiles = -(-OC // bm) * -(-P // bn)
        for splits in (1, 2, 4, 8):
            if splits > 1 and (ksteps // splits < 4 or tiles * splits > 2 * _NUM_CUS * _CONV_SLOTS[cfg]):
                continue
            waves = -(-tiles * splits // (_NUM_CUS * _CONV_SLOTS[cfg]))
            cost = waves * _CONV_SLOTS[cfg] * bm * bn * (-(-ksteps // splits)) / _CONV_EFF[cfg]
            cost += (splits > 1) * P * OC * splits * 0.05  # slab round trip + finalize launch
            if best is None or cost < best[0]:
                best = (cost, cfg, splits)
    return best[1], best[2]


def conv2d_nhwc(x, w, bias=None, *, stride: int = 1, pad: int = 1, up: bool = False,
                bias2=None, resid=None, out=None, cfg: int | None = None,
                splits: int | None = None, tile: tuple[int, int] | None = None,
                in_nchw: bool = False, out_nchw: bool = False):
    """NHWC conv: x [N,H,W,IC], w packed [OC,KH,KW,IC] -> [N,OH,OW,OC].

    bias [OC]; bias2 [N,OC] f32 (per-sample additive, e.g. time embedding);
    resid [N,OH,OW,OC] added in the epilogue; up = nearest-2x upsample of x first.
    in_nchw: x is [N,IC,H,W] (the direct small-IC kernel only: UNet conv_in reads the
    external layout); out_nchw: the output is written [N,OC,OH,OW] (no resid: conv_out).
    """
    if in_nchw:
        N, IC, H, W = x.shape
    else:
        N, H, W, IC = x.shape
    OC, KH, KW, IC2 = w.shape
    if IC2 != IC or KH != KW or not conv_supported(IC, OC, stride, up, KH):
        raise ValueError(f"conv2d_nhwc: unsupported IC={IC} OC={OC} w={tuple(w.shape)}")
    VH, VW = H << int(up), W << int(up)
    OH, OW = (VH + 2 * pad - KH) // stride + 1, (VW + 2 * pad - KW) // stride + 1
    _req(x, "x")
    _req(w, "w", dtype=x.dtype)
    if bias is not None:
        _req(bias, "bias", dtype=x.dtype, numel=OC)
    bias2_ld = 0
    if bias2 is not None:  # [N, OC] f32, rows may be strided (one slice of a batched projection)
        if not (bias2.is_cuda and bias2.dtype == torch.float32 and tuple(bias2.shape) == (N, OC)
                and bias2.stride(1) == 1 and bias2.stride(0) % 4 == 0 and bias2.data_ptr() % 16 == 0):
            raise ValueError(f"bias2: expected an f32 [{N}, {OC}] device view with unit column "
                             f"stride and 16-byte aligned rows")
        bias2_ld = bias2.stride(0) if N > 1 else OC
    if resid is not None:
        if out_nchw:
            raise ValueError("conv2d_nhwc: out_nchw takes no resid")
        _req(resid, "resid", dtype=x.dtype, shape=(N, OH, OW, OC))
    oshape = (N, OC, OH, OW) if out_nchw else (N, OH, OW, OC)
    if out is None:
        out = torch.empty(*oshape, device=x.device, dtype=x.dtype)
    _req(out, "out", dtype=x.dtype, shape=oshape)
    P, ksteps = N * OH * OW, KH * KW * IC // 64
    if IC % 64:  # small-IC direct kernel: one variant
        cfg, splits, ksteps = 14, 1, 1
    elif in_nchw:
        raise ValueError("conv2d_nhwc: in_nchw needs the small-IC kernel (IC 3 / 4)")
    if cfg is None or splits is None:
        c0, s0 = conv_plan(P, OC, ksteps)
        cfg = c0 if cfg is None else cfg
        splits = s0 if splits is None else splits
    th = tw = 0
    if 8 <= cfg < 14:  # halo kernels: stride 1, no split-K
        if stride != 1:
            raise ValueError("conv2d_nhwc: halo tiles need stride 1")
        splits = 1
        th, tw = tile or halo_tile(OH, OW, 256 if cfg >= 12 else 128 if cfg < 10 else 64)
    splits = max(1, min(splits, ksteps))
    kps = -(-ksteps // splits)
    splits = -(-ksteps // kps)
    ws = torch.empty(splits * P * OC, device=x.device, dtype=torch.float32) if splits > 1 else None
    check(kernels().cake_conv2d_nhwc2(_dt(x), _p(x), _p(w), None if bias is None else _p(bias),
                                      None if bias2 is None else _p(bias2),
                                      None if resid is None else _p(resid), _p(out),
                                      None if ws is None else _p(ws), _p(_zeros16(x.device)),
                                      N, H, W, IC, OC, KH, KW,
                                      stride, pad, int(up), int(cfg), int(splits), th, tw,
                                      int(bias2_ld), int(in_nchw) | (int(out_nchw) << 1),
                                      _stream()),
          "conv2d_nhwc")
    return out


# ---------------------------------------------------------------------------
# Stable Diffusion step glue (sd_small.hip)
# ---------------------------------------------------------------------------

def timestep_embed(t_table, step, B: int, dim: int, flip: bool, shift: float, out):
    """out [B, dim] (16-bit or f32) = sinusoidal embedding of t_table[*step] (step may be
    None: t_table[0]); both read on the device, so the launch replays across steps."""
    _req(t_table, "t_table", dtype=torch.float32)
    if step is not None:
        _req(step, "step", dtype=torch.int32, numel=1)
    _req(out, "out", numel=B * dim)
    out16 = out.dtype in _DT
    if not out16 and out.dtype != torch.float32:
        raise TypeError("timestep_embed: out must be 16-bit or f32")
    check(kernels().cake_timestep_embed(_DT.get(out.dtype, 0), _p(t_table), _p(step), B, dim,
                                        int(flip), float(shift), int(out16), _p(out), _stream()),
          "timestep_embed")


def sched_step(x, pred, cfg: bool, guidance: float, coef, step, seed, next_in=None):
    """x (f32 latents) <- A x + B eps + N z  with eps the CFG-combined UNet prediction
    and (A, B, N, S) = coef[*step]; next_in (16-bit) <- S * x (duplicated for CFG).
    seed: int64 device scalar keying the Philox noise (read on the device)."""
    n = x.numel()
    _req(x, "x", dtype=torch.float32)
    _req(pred, "pred", numel=n * (2 if cfg else 1))
    _req(coef, "coef", dtype=torch.float32)
    _req(step, "step", dtype=torch.int32, numel=1)
    if coef.dim() != 2 or coef.shape[1] != 4:
        raise ValueError("coef must be [steps, 4]")
    if next_in is not None:
        _req(next_in, "next_in", dtype=pred.dtype, numel=n * (2 if cfg else 1))
    _req(seed, "seed", dtype=torch.int64, numel=1)
    check(kernels().cake_sched_step(_dt(pred), _p(x), _p(pred), n, int(cfg), float(guidance),
                                    _p(coef), _p(step), _p(seed), _p(next_in), _stream()),
          "sched_step")


def step_advance(step):
    _req(step, "step", dtype=torch.int32, numel=1)
    check(kernels().cake_step_advance(_p(step), _stream()), "step_advance")


def scale_copy(x, scale: float, dup: bool, out):
    """out (16-bit) <- scale * x (f32), written twice back to back when dup (CFG batch)."""
    n = x.numel()
    _req(x, "x", dtype=torch.float32)
    _req(out, "out", numel=n * (2 if dup else 1))
    check(kernels().cake_scale_copy(_dt(out), _p(x), n, float(scale), int(dup), _p(out),
                                    _stream()), "scale_copy")


def to_rgb8(img, nhwc: bool = False) -> torch.Tensor:
    """Decoded image (16-bit, [B,3,H,W] or [B,H,W,3] when nhwc) -> u8 [B,H,W,3]."""
    _req(img, "img")
    if nhwc:
        B, H, W, C = img.shape
    else:
        B, C, H, W = img.shape
    if C != 3:
        raise ValueError("to_rgb8: 3 channels expected")
    out = torch.empty(B, H, W, 3, device=img.device, dtype=torch.uint8)
    check(kernels().cake_to_rgb8(_dt(img), _p(img), B, H, W, int(nhwc), _p(out), _stream()),
          "to_rgb8")
    return out
