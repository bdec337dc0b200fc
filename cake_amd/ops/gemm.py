"""Host side of the MFMA GEMM (csrc/kernels/gemm.hip): y = x W^T + fused epilogue.

Every T > 1 linear on the device path goes through :func:`linear`: Llama prefill
q|k|v, o (+residual), gate|up (+SwiGLU), down (+residual); every SD UNet / VAE /
CLIP projection (+bias, +residual, +GEGLU).  Shapes and strides are validated
on the host before launch; there is no library fallback.

Tile choice: a cost model over the kernel's tile configurations (waves of
tiles x per-tile work, split-K when the grid is smaller than the chip), with an
optional measured override table (:func:`set_plan`, filled by
scripts/tune_gemm.py on the GPU box).
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import check, kernels

EPI = {"store": 0, "resid32": 1, "add16": 2, "swiglu": 3, "geglu": 4, "store32": 6, "silu": 7,
       "quick_gelu": 8, "gelu": 9}
_DT = {torch.bfloat16: 0, torch.float16: 1}
# (BM, BN) of the kernel's tile configurations (gemm.hip CAKE_GEMM_CFGS)
CFG_TILES = {0: (128, 128), 1: (64, 128), 2: (256, 128), 3: (128, 256), 4: (64, 64),
             5: (256, 256), 6: (256, 128), 7: (128, 128), 8: (128, 128), 11: (256, 256),
             12: (64, 128), 13: (64, 64), 14: (64, 160), 15: (64, 160), 16: (128, 160),
             17: (128, 160), 18: (64, 160), 19: (128, 160), 20: (256, 256), 21: (256, 256),
             22: (256, 256), 23: (256, 192),
             24: (128, 256), 25: (256, 256), 26: (256, 192), 27: (128, 256)}
_SLOTS = {0: 2, 1: 2, 2: 1, 3: 1, 4: 4, 5: 1, 6: 1, 7: 1, 8: 2, 11: 1, 12: 2, 13: 2,
          14: 2, 15: 2, 16: 1, 17: 1, 18: 1, 19: 1, 20: 1, 21: 1, 22: 1, 23: 1, 24: 1, 25: 1, 26: 1, 27: 1}  # WGs/CU
# 80-column wave tiles (two waves across the 160 columns): no gated epilogue
NO_GATED = {14, 17, 18, 19}
# register-staged / four-wave 256x256 (gemm_rs.h, gemm_4w.h): whole 64-element k steps only
K64_ONLY = {21, 22, 23, 24, 25, 26, 27}
# relative per-tile throughput (measured per-config sweep,
# profiles/r2_gemm_sweep_agpr.jsonl): the AGPR-accumulator 128x128 tile (0) for most
# shapes, the 8-wave 256x256 tile (11) where its tiles fill the chip, 64-wide tiles
# (1, 4) for short M
_EFF = {0: 1.0, 1: 0.8, 2: 0.8, 3: 0.8, 4: 0.7, 5: 1.2, 6: 0.95, 7: 0.9, 8: 0.9, 11: 1.1,
        12: 0.8, 13: 0.7, 14: 0.8, 15: 0.7, 16: 0.9, 17: 0.9, 18: 0.8, 19: 0.9, 20: 1.2, 21: 1.3, 22: 1.3, 23: 1.3, 24: 1.2, 25: 1.3, 26: 1.3, 27: 1.2}
NUM_CUS = 256
# plan cfg of the library GEMM (hipBLASLt, csrc/driver/blaslt.cpp), kept as the A/B arm of
# scripts/bench_gemm_lib.py: off the default path (table entries naming it are read only
# under CAKE_GEMM_LIB=1, or when a caller passes cfg=LIB); epilogues it can carry: plain
# store, f32 store / accumulate (beta 1), and SwiGLU as library GEMM + silu_mul_rows
LIB = -1
LIB_EPIS = ("store", "resid32", "store32", "swiglu")
_LIB_WS_BYTES = 32 << 20
_bound = False
_plans: dict = {}
_ws: dict = {}
_zeros: dict = {}


def _lib():
    global _bound
    lib = kernels()
    if not _bound:
        P, I, L = C.c_void_p, C.c_int, C.c_longlong
        lib.cake_gemm.argtypes = [I, I, I, I, P, L, P, L, P, L, P, P, L, P, P, I, I, I, P]
        lib.cake_gemm.restype = I
        lib.cake_gemm_ws_floats.argtypes = [I, I, I, I, I, I]
        lib.cake_gemm_ws_floats.restype = L
        lib.cake_blaslt_gemm.argtypes = [I, I, P, L, P, L, P, L, I, I, I, P, C.c_size_t, P]
        lib.cake_blaslt_gemm.restype = I
        _bound = True
    return lib


def _zeros16(dev) -> torch.Tensor:
    z = _zeros.get(dev)
    if z is None:
        z = _zeros[dev] = torch.zeros(64, dtype=torch.int32, device=dev)
    return z


_ws_keep: list = []


def _workspace(dev, numel: int) -> torch.Tensor:
    """Split-K slabs.  Superseded buffers are kept alive: a captured hipGraph may
    still point at them."""
    w = _ws.get(dev)
    if w is None or w.numel() < numel:
        if w is not None:
            _ws_keep.append(w)
        w = _ws[dev] = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=dev)
    return w


def _load_tuned() -> list:
    """Measured best (cfg, split-K) per model shape (gemm_tuned.json, written by
    scripts/gemm_tune_table.py from a bench_gemm.py --sweep on an MI355X)."""
    import json
    import os
    p = os.environ.get("CAKE_GEMM_TABLE") or os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "gemm_tuned.json")
    lib_ok = os.environ.get("CAKE_GEMM_LIB") == "1"
    try:
        with open(p) as f:
            return [e for e in json.load(f)["entries"]
                    if e["cfg"] in CFG_TILES
                    or (lib_ok and e["cfg"] == LIB and e["epi"] in LIB_EPIS)]
    except (OSError, ValueError, KeyError):
        return []


_TUNED = _load_tuned()


def _near_splits(splits: int, m_near: int, M: int) -> int:
    """Split-K of a measured neighbour scaled to this M (the split fills the grid the
    neighbour's M left short: twice the rows, half the splits), a power of two >= 1."""
    s = splits * m_near // max(M, 1)
    p = 1
    while p * 2 <= s:
        p *= 2
    return p


def _tuned(M: int, Nv: int, K: int, epi: str, mfma_only: bool = False):
    """Exact measured shape, else the same (Nv, K, epilogue) measured at the nearest M
    within 2x (its tile config, split-K scaled to this M).  mfma_only skips the library
    GEMM's entries."""
    near = None
    for e in _TUNED:
        if e["Nv"] != Nv or e["K"] != K or e["epi"] != epi:
            continue
        if mfma_only and e["cfg"] == LIB:
            continue
        if e["M"] == M:
            return e["cfg"], e["splits"]
        r = max(M, e["M"]) / min(M, e["M"])
        if r <= 2 and (near is None or r < near[0]):
            near = (r, e)
    if near is None:
        return None
    e = near[1]
    return e["cfg"], (1 if e["cfg"] == LIB else _near_splits(e["splits"], e["M"], M))


def plan_mfma(M: int, Nv: int, K: int, epi: str = "store") -> tuple[int, int]:
    """The MFMA kernel's (cfg, splits) for a shape: its measured entries, else the cost
    model (the library GEMM's entries ignored)."""
    p = _tuned(M, Nv, K, epi, mfma_only=True)
    return p if p is not None else _cost_plan(M, Nv, K)


def set_plan(M: int, N: int, K: int, epi: str, cfg: int, splits: int) -> None:
    """Pin the tile configuration / split-K of one shape (measured tuning)."""
    _plans[(M, N, K, epi)] = (cfg, splits)


def plan(M: int, Nv: int, K: int, epi: str = "store") -> tuple[int, int]:
    """(cfg, splits) for an M x Nv x K problem (Nv = weight rows read)."""
    p = _plans.get((M, Nv, K, epi))
    if p is not None:
        return p
    p = _tuned(M, Nv, K, epi)
    if p is not None:
        _plans[(M, Nv, K, epi)] = p
        return p
    return _cost_plan(M, Nv, K)


def _cost_plan(M: int, Nv: int, K: int) -> tuple[int, int]:
    """The MFMA kernel's (cfg, splits) by the cost model."""
    best = None
    ksteps = -(-K // 64)
    cands = (1, 4, 0) if M <= 64 else (0, 1, 4, 5)
    # the four-wave 256x256 tile where it can run (whole 64-element k steps, operands under
    # 2 GB); unsplit (its split-2 form is the shape-specific remainder pair)
    four = M > 64 and K % 64 == 0 and M * K * 2 < 2 ** 31 and Nv * K * 2 < 2 ** 31
    if four:
        cands = cands + (22,)
    for cfg in cands:
        bm, bn = CFG_TILES[cfg]
        tiles = -(-M // bm) * -(-Nv // bn)
        for splits in (1, 2, 4, 8, 16):
            if splits > 1 and (cfg == 22 or ksteps // splits < 4 or
                               tiles * splits > 2 * NUM_CUS * _SLOTS[cfg]):
                continue
            waves = -(-tiles * splits // (NUM_CUS * _SLOTS[cfg]))
            cost = waves * _SLOTS[cfg] * bm * bn * (-(-ksteps // splits)) / _EFF[cfg]
            cost += (splits > 1) * M * Nv * splits * 0.1   # slab round trip + finalize
            if best is None or cost < best[0]:
                best = (cost, cfg, splits)
    return best[1], best[2]


def _rows_view(t: torch.Tensor, name: str) -> tuple[torch.Tensor, int]:
    """[..., C] tensor with unit column stride -> ([R, C] VIEW of it, row stride)."""
    if t.dim() < 2:
        t = t.view(1, -1)
    if t.stride(-1) != 1:
        raise ValueError(f"{name}: needs unit column stride")
    if t.dim() > 2:
        try:
            t2 = t.view(-1, t.shape[-1])   # never a copy: outputs are written through it
        except RuntimeError:
            raise ValueError(f"{name}: leading dims do not flatten to one row stride") from None
    else:
        t2 = t
    if t2.dim() == 2 and t2.shape[0] > 1 and t2.stride(0) < t2.shape[1]:
        raise ValueError(f"{name}: overlapping rows")
    return t2, (t2.stride(0) if t2.shape[0] > 1 else t2.shape[1])


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, *,
           epi: str = "store", out: torch.Tensor | None = None,
           resid: torch.Tensor | None = None, cfg: int | None = None,
           splits: int | None = None) -> torch.Tensor:
    """y = epilogue(x @ w.T) on MFMA.

    x [..., K] (16-bit, unit column stride, any row stride that is a multiple of
    8); w [N, K] ([2F, K] for the gated epilogues: rows [0, F) gate/h, [F, 2F)
    up/gate).  Epilogues:
      store   -> out [..., N] = y (+ bias)
      resid32 -> resid (f32 [..., N]) += y (+ bias); returns resid
      add16   -> out = y (+ bias) + resid (16-bit [..., N])
      swiglu  -> out [..., F] = silu(y_gate) * y_up
      geglu   -> out [..., F] = (y_h + b_h) * gelu_tanh(y_gate + b_gate)
      store32 -> resid (f32 [..., N], any row stride) = y (+ bias); returns resid
      silu    -> out = silu(y (+ bias))
      quick_gelu / gelu -> out = act(y (+ bias)) (CLIP MLP: x*sigmoid(1.702x) / erf GELU)
    """
    if epi not in EPI:
        raise ValueError(f"unknown epilogue {epi}")
    if not (x.is_cuda and w.is_cuda) or x.dtype not in _DT or w.dtype != x.dtype:
        raise TypeError("gemm.linear: 16-bit device tensors of one dtype expected")
    lead = x.shape[:-1]
    K = x.shape[-1]
    if x.dim() > 2 and x.stride(-1) == 1:
        try:
            x.view(-1, K)
        except RuntimeError:
            x = x.contiguous()
    x2, lda = _rows_view(x, "x")
    M = x2.shape[0]
    if w.dim() != 2 or w.shape[1] != K or w.stride(1) != 1:
        raise ValueError(f"gemm.linear: weight {tuple(w.shape)} does not match K={K}")
    ldb = w.stride(0)
    gated = epi in ("swiglu", "geglu")
    Nv = w.shape[0]
    if gated and Nv % 32:
        raise ValueError("gated epilogue needs 2F weight rows with F % 16 == 0")
    N = Nv // 2 if gated else Nv
    if K % 8 or lda % 8 or ldb % 8 or x2.data_ptr() % 16 or w.data_ptr() % 16:
        raise ValueError("gemm.linear: K, row strides must be multiples of 8 and bases 16-byte "
                         "aligned")
    if bias is not None:
        if not (bias.is_cuda and bias.dtype == x.dtype and bias.is_contiguous()
                and bias.numel() == Nv):
            raise ValueError(f"gemm.linear: bias must be a contiguous {x.dtype} [{Nv}] tensor")
    ldr = 0
    rptr = None
    if epi in ("resid32", "store32"):
        if resid is None or resid.dtype != torch.float32 or not resid.is_cuda:
            raise ValueError(f"{epi} needs an f32 device output/residual")
        r2, ldr = _rows_view(resid, "resid")
        if tuple(r2.shape) != (M, N):
            raise ValueError(f"resid shape {tuple(resid.shape)} != {(M, N)}")
        rptr = r2.data_ptr()
    elif epi == "add16":
        if resid is None or resid.dtype != x.dtype or not resid.is_cuda:
            raise ValueError("add16 needs a 16-bit device residual")
        r2, ldr = _rows_view(resid, "resid")
        if tuple(r2.shape) != (M, N):
            raise ValueError(f"resid shape {tuple(resid.shape)} != {(M, N)}")
        rptr = r2.data_ptr()
    if epi in ("resid32", "store32"):
        out2, ldc, cptr = None, 0, None
    else:
        if out is None:
            out = torch.empty(*lead, N, device=x.device, dtype=x.dtype)
        if out.dtype != x.dtype or not out.is_cuda:
            raise ValueError("out dtype/device mismatch")
        out2, ldc = _rows_view(out, "out")
        if tuple(out2.shape) != (M, N):
            raise ValueError(f"out shape {tuple(out.shape)} != {(M, N)}")
        cptr = out2.data_ptr()
    f32_out = epi in ("resid32", "store32")
    if M == 0:
        return resid if f32_out else out
    c0, s0 = plan(M, Nv, K, epi)
    cfg = c0 if cfg is None else cfg
    lib_ok = epi != "swiglu" or (ldc == N and N % 8 == 0 and out2.data_ptr() % 16 == 0)
    if cfg == LIB and bias is None and epi in LIB_EPIS and lib_ok:
        _lib_gemm(x2, lda, w, ldb, epi, out2, ldc, r2 if f32_out else None, ldr, M, N, K)
        return resid if f32_out else out
    if cfg == LIB:  # an epilogue / bias / strided output the library form does not carry
        cfg, s0 = plan_mfma(M, Nv, K, epi)
    splits = s0 if splits is None else max(1, int(splits))
    # the kernel library sizes it (an in-kernel pair needs its slabs only)
    ws = _workspace(x.device, int(_lib().cake_gemm_ws_floats(
        int(cfg), int(splits), M, N, K, 1 if Nv != N else 0))) if splits > 1 else None
    check(_lib().cake_gemm(_DT[x.dtype], EPI[epi], int(cfg), int(splits), x2.data_ptr(), lda,
                           w.data_ptr(), ldb, cptr, ldc,
                           None if bias is None else bias.data_ptr(), rptr, ldr,
                           None if ws is None else ws.data_ptr(), _zeros16(x.device).data_ptr(),
                           M, N, K, torch.cuda.current_stream().cuda_stream), "gemm")
    return resid if f32_out else out


def _lib_gemm(x2, lda, w, ldb, epi, out2, ldc, r2, ldr, M, N, K) -> None:
    """The library GEMM (hipBLASLt) for a plan that names it.  Its workspace is one buffer
    per (device, stream), so library GEMMs on two streams never share one."""
    dev = x2.device
    st = torch.cuda.current_stream().cuda_stream
    ws = _lib_ws.get((dev, st))
    if ws is None:
        ws = _lib_ws[(dev, st)] = torch.empty(_LIB_WS_BYTES, dtype=torch.uint8, device=dev)
    dt = _DT[x2.dtype]

    def run(mode, cptr, ld, n):
        check(_lib().cake_blaslt_gemm(dt, mode, x2.data_ptr(), lda, w.data_ptr(), ldb, cptr, ld,
                                      M, n, K, ws.data_ptr(), _LIB_WS_BYTES, st), "blaslt gemm")
    if epi == "store":
        run(0, out2.data_ptr(), ldc, N)
    elif epi in ("store32", "resid32"):
        run(1 if epi == "store32" else 2, r2.data_ptr(), ldr, N)
    else:  # swiglu: [M, 2N] library product (cached scratch), then silu(gate) * up
        gu = _lib_gu.get((dev, st, x2.dtype))
        if gu is None or gu.numel() < M * 2 * N:
            gu = _lib_gu[(dev, st, x2.dtype)] = torch.empty(M * 2 * N, device=dev,
                                                            dtype=x2.dtype)
        run(0, gu.data_ptr(), 2 * N, 2 * N)
        check(kernels().cake_silu_mul_rows(dt, gu.data_ptr(), M, N, out2.data_ptr(), st),
              "silu_mul_rows")


_lib_ws: dict = {}
_lib_gu: dict = {}
