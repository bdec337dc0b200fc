"""ctypes front of the native decode driver (csrc/driver/graph_loop.cpp).

The per-token host loop of every serving mode — replay the captured step graph of
the right position bucket, read the tokens back one replay behind, stop at EOS —
runs in C++ with the GIL released (ctypes drops it for the call; the optional
per-token / announce callbacks take it back only while they run).  Python builds
the spec once per generate call: graph exec handles (``raw_cuda_graph_exec``), a
live-length -> bucket table and the device token history.

Reference: the master token loop cake-core/src/cake/master.rs:80-124 and the
generator step cake-core/src/models/llama3/llama.rs:277-341.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Callable

import torch

from ._lib import check, kernels

TOKEN_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32)
ANNOUNCE_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.c_int32)


class LoopSpec(C.Structure):
    _fields_ = [
        ("execs", C.POINTER(C.c_void_p)), ("n_execs", C.c_int32),
        ("bucket_of", C.POINTER(C.c_int32)), ("n_len", C.c_int32),
        ("k", C.c_int32), ("hist", C.c_void_p), ("base", C.c_int32), ("pos", C.c_int32),
        ("n", C.c_int32), ("chunk", C.c_int32),
        ("eos", C.POINTER(C.c_int32)), ("n_eos", C.c_int32),
        ("on_token", TOKEN_CB), ("token_ctx", C.c_void_p),
        ("announce", ANNOUNCE_CB), ("announce_ctx", C.c_void_p),
        ("stream", C.c_void_p),
        ("out_tokens", C.POINTER(C.c_int32)), ("out_ms", C.POINTER(C.c_float)),
        ("out_cap", C.c_int32),
    ]


class LoopResult(C.Structure):
    _fields_ = [("n_tokens", C.c_int32), ("replays", C.c_int32), ("pos", C.c_int32),
                ("stopped", C.c_int32), ("wall_s", C.c_double)]


_bound = False


def _lib():
    global _bound
    lib = kernels()
    if not _bound:
        lib.cake_graph_decode.argtypes = [C.POINTER(LoopSpec), C.POINTER(LoopResult)]
        lib.cake_graph_decode.restype = C.c_int
        _bound = True
    return lib


@dataclass
class LoopOut:
    tokens: list[int] = field(default_factory=list)
    step_ms: list[float] = field(default_factory=list)
    replays: int = 0
    pos: int = 0
    stopped: bool = False
    wall_s: float = 0.0


class GraphSet:
    """Step graphs of one engine, one per position bucket, and the live-length ->
    bucket table the native loop indexes (the table is built once from `pick`)."""

    def __init__(self, graphs: list[torch.cuda.CUDAGraph], pick: Callable[[int], int],
                 max_len: int):
        self.graphs = list(graphs)   # keeps the graphs (and their memory pools) alive
        self._execs = (C.c_void_p * len(self.graphs))(
            *[int(g.raw_cuda_graph_exec()) for g in self.graphs])
        if any(not e for e in self._execs):
            raise RuntimeError("graph not instantiated")
        self.n_len = int(max_len) + 1
        self._table = (C.c_int32 * self.n_len)(*[int(pick(t)) for t in range(self.n_len)])


def run(gs: GraphSet, *, k: int, n: int, pos: int, hist: torch.Tensor | None = None,
        base: int = 0, eos_ids=None, on_token: Callable[[int], bool | None] | None = None,
        announce: Callable[[int, int], None] | None = None, chunk: int = 0,
        callback_stops: bool = True) -> LoopOut:
    """Replay `ceil(n / k)` step graphs on the current stream.

    hist: the device int32 token history the graphs append to (the master); None on a
    worker rank (no read-back).  base: history index of the first generated token.
    pos: host mirror of the device position.  on_token(tok) -> True stops the loop
    (after EOS the at most one replay already enqueued past it is discarded by the
    caller's next prefill).  announce(first, count) runs before each chunk of replays.
    callback_stops=False: on_token's return value and exceptions never stop the loop
    (exceptions are re-raised after it) — for lock-step ranks (tensor parallel) where
    only one rank has a callback and every rank must replay the same number of steps.
    """
    out = LoopOut(pos=pos)
    if n <= 0:
        return out
    if hist is not None:
        if not (hist.is_cuda and hist.dtype == torch.int32 and hist.is_contiguous()):
            raise ValueError("hist must be a contiguous int32 device tensor")
        if base + -(-n // k) * k > hist.numel():
            raise ValueError("generation overruns the token history")
    cap = n if hist is not None else 0
    toks = (C.c_int32 * max(cap, 1))()
    ms = (C.c_float * max(n, 1))()
    eos = list(eos_ids or [])
    eos_arr = (C.c_int32 * max(len(eos), 1))(*eos)
    errors: list[BaseException] = []

    def _tok(_ctx, t):
        try:
            stop = bool(on_token(int(t)))
            return 1 if stop and callback_stops else 0
        except BaseException as e:  # noqa: BLE001  (re-raised after the loop)
            errors.append(e)
            return 1 if callback_stops else 0

    def _ann(_ctx, first, count):
        try:
            announce(int(first), int(count))
            return 0
        except BaseException as e:  # noqa: BLE001
            errors.append(e)
            return 1

    tok_cb = TOKEN_CB(_tok) if on_token is not None else TOKEN_CB()
    ann_cb = ANNOUNCE_CB(_ann) if announce is not None else ANNOUNCE_CB()
    spec = LoopSpec(gs._execs, len(gs.graphs), gs._table, gs.n_len, int(k),
                    C.c_void_p(hist.data_ptr() if hist is not None else None), int(base),
                    int(pos), int(n), int(chunk), eos_arr, len(eos), tok_cb, None, ann_cb, None,
                    C.c_void_p(torch.cuda.current_stream().cuda_stream), toks, ms,
                    max(cap, n))
    res = LoopResult()
    rc = _lib().cake_graph_decode(C.byref(spec), C.byref(res))
    if errors:
        raise errors[0]
    check(rc, "graph_decode")
    out.tokens = [int(toks[i]) for i in range(res.n_tokens)] if hist is not None else []
    out.step_ms = [float(ms[i]) for i in range(res.n_tokens)]
    out.replays, out.pos, out.stopped, out.wall_s = (int(res.replays), int(res.pos),
                                                     bool(res.stopped), float(res.wall_s))
    return out
