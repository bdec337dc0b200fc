"""Chrome-trace JSON writer (+ roctx ranges on the GPU).

The reference installs ``tracing_chrome`` for one SD request when
``--sd-tracing`` is set (cake-core/src/models/sd/sd.rs:350-356) — a process-wide
subscriber that panics on a second traced request (Appendix E Q10).  Here a
trace is a per-request object writing ``[{name, ph: "X", ts, dur, pid, tid}]``
events; spans also push roctx ranges (torch.cuda.nvtx is roctx on ROCm) so
``rocprofv3 --marker-trace`` shows the same structure.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time


class ChromeTrace:
    def __init__(self):
        self.events: list[dict] = []
        self.t0 = time.perf_counter()
        self.pid = os.getpid()

    def add(self, name: str, start: float, end: float, **args) -> None:
        self.events.append({"name": name, "ph": "X", "ts": (start - self.t0) * 1e6,
                            "dur": (end - start) * 1e6, "pid": self.pid,
                            "tid": threading.get_ident() % 100000, "args": args})

    @staticmethod
    @contextlib.contextmanager
    def span(trace: "ChromeTrace | None", name: str, **args):
        nvtx = None
        try:
            import torch
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                nvtx = torch.cuda.nvtx
                nvtx.range_push(name)
        except Exception:  # noqa: BLE001
            nvtx = None
        start = time.perf_counter()
        try:
            yield
        finally:
            if trace is not None:
                trace.add(name, start, time.perf_counter(), **args)
            if nvtx is not None:
                nvtx.range_pop()

    def save(self, path) -> None:
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)
