"""Host side of the device decode loop (one step of host/GPU overlap).

The GPU graph for step k+1 only needs the token chosen by step k, which the
graph itself leaves in device memory — so the host enqueues step k+1 *before*
it reads token k back (4 bytes through a pinned ring).  EOS detection lags by
one step (the extra speculative step is discarded).  Per-token latency comes
from device events recorded after every step: the reference only logs an
aggregate rate (cake-core/src/cake/master.rs:93-121); BASELINE asks for p50.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable

import torch

from .model import DeviceDecoder


@dataclass
class DecodeStats:
    tokens: list[int] = field(default_factory=list)
    step_ms: list[float] = field(default_factory=list)   # device time per token
    wall_s: float = 0.0

    def percentile(self, q: float) -> float:
        if not self.step_ms:
            return float("nan")
        xs = sorted(self.step_ms)
        k = min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))
        return xs[k]


def run_decode(dec: DeviceDecoder, n_steps: int, eos_ids: set[int] | None = None,
               on_token: Callable[[int], None] | None = None,
               sampler: Callable[[torch.Tensor], int] | None = None) -> DecodeStats:
    """Run up to n_steps decode steps; stop at EOS (unless eos_ids is None)."""
    st = DecodeStats()
    if n_steps <= 0:
        return st
    dev = dec.bufs.tok.device
    if sampler is not None:
        # sampled mode: the host draws each token, so no lookahead is possible
        t0 = time.perf_counter()
        prev_ev = torch.cuda.Event(enable_timing=True)
        prev_ev.record()
        for _ in range(n_steps):
            dec.launch()
            tok = sampler(dec.logits())
            dec.push(tok)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            ev.synchronize()
            st.step_ms.append(prev_ev.elapsed_time(ev))
            prev_ev = ev
            st.tokens.append(tok)
            if on_token:
                on_token(tok)
            if eos_ids and tok in eos_ids:
                break
        st.wall_s = time.perf_counter() - t0
        return st

    if dec.graph is not None:
        st = _run_native(dec, n_steps, eos_ids, on_token)
        _check(dec)
        return st
    # eager (no graphs): every launch runs dec.k steps; their tokens are the next k
    # entries of the device history, copied to a pinned ring one launch behind
    k = dec.k
    base = int(dec.bufs.hist_len.item())
    ring = torch.empty(2 * k, dtype=torch.int32, pin_memory=True)
    start_ev = torch.cuda.Event(enable_timing=True)
    start_ev.record()
    prev_done = start_ev
    t0 = time.perf_counter()
    pending = None  # (slot, event, n_tokens)
    issued = 0
    stop = False
    while not stop:
        cur = None
        if issued < n_steps and base + issued + k <= dec.bufs.hist.numel():
            slot = (issued // k) & 1
            dec.launch()
            lo = base + issued
            ring[slot * k:slot * k + k].copy_(dec.bufs.hist[lo:lo + k], non_blocking=True)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            cur = (slot, ev, min(k, n_steps - issued))
            issued += k
        if pending is not None:
            slot, ev, n = pending
            ev.synchronize()
            dt = prev_done.elapsed_time(ev) / k  # device time per token of this launch
            prev_done = ev
            for i in range(n):
                tok = int(ring[slot * k + i].item())
                st.step_ms.append(dt)
                st.tokens.append(tok)
                if on_token:
                    on_token(tok)
                if eos_ids and tok in eos_ids:
                    stop = True
                    break
        pending = cur
        if pending is None:
            stop = True
    if pending is not None:
        pending[1].synchronize()
    st.wall_s = time.perf_counter() - t0
    del dev
    _check(dec)
    return st


def _check(dec: DeviceDecoder) -> None:
    """Raise (and re-arm) when a decode launch of this run gave up in a bounded spin:
    the split-K attention merge's error word (tickets[2 nkv]) or a persistent-decode
    hand-off — its tokens are invalid (one host read, after the loop's final sync)."""
    stack = getattr(dec.m, "stack", None)
    if stack is not None and getattr(stack, "backend", "hip") == "hip":
        stack.mk_check(dec.bufs)


def _run_native(dec: DeviceDecoder, n_steps: int, eos_ids, on_token) -> DecodeStats:
    """Greedy graph decode through the native driver (csrc/driver/graph_loop.cpp): the
    replay / one-behind read-back / EOS loop runs in C++ without the GIL."""
    from ...ops import graph_loop as GL
    st = DecodeStats()
    k = dec.k
    # the device history holds one token per position up to the current one: its
    # length is host_pos + 1 (no device read-back — a sync — inside the timed loop)
    base = dec.host_pos + 1
    room = min(dec.bufs.hist.numel() - base, dec.m.stack.max_seq - 1 - dec.host_pos)
    n = min(n_steps, room // k * k)
    if n <= 0:
        return st
    res = GL.run(dec.graph_set(), k=k, n=n, pos=dec.host_pos, hist=dec.bufs.hist, base=base,
                 eos_ids=eos_ids,
                 on_token=(lambda t: bool(on_token(t))) if on_token is not None else None)
    dec.host_pos = res.pos
    st.tokens, st.step_ms, st.wall_s = res.tokens, res.step_ms, res.wall_s
    return st
