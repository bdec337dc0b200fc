"""Worker role: serve placed layers / model components over the framed TCP protocol.

Reference: cake-core/src/cake/worker.rs.
* Resolve ``--name`` in the topology; an unknown name serves the FIRST node
  with a loud warning (worker.rs:90-104, Appendix E Q12).
* Load only the owned units (text: ``model.layers.N`` blocks into one
  :class:`LayerStack`; image: clip/clip2/vae/unet — worker.rs:110-125).
* Accept many masters; each connection gets its own KV session while weights
  are shared (worker.rs:52-72, 290-303).  Per connection: ``Hello`` →
  ``WorkerInfo`` (latency = ms spent reading Hello), then ``SingleOp``/``Batch``
  → run the ops in order → ``Tensor`` (worker.rs:177-287).
* Every 5 messages log ops/s and read/write bandwidth (worker.rs:18-19,271-282).
* Extensions: ``Reset`` clears the session KV, ``Ping``→``Pong``, failures
  are returned as ``Error`` instead of aborting the process (Appendix E Q6),
  and ``CAKE_FAULT_INJECT=drop_after=N`` drops a connection after N ops (tests).
"""
from __future__ import annotations

import logging
import os
import platform
import threading
import time
import warnings

import torch

from . import proto as P

log = logging.getLogger("cake.worker")
NUM_OPS_TO_STATS = 5


def _layer_index(name: str) -> int:
    prefix = "model.layers."
    if not name.startswith(prefix):
        raise ValueError(f"not a transformer block: {name}")
    return int(name[len(prefix):])


class Worker:
    def __init__(self, ctx):
        self.ctx = ctx
        topo = ctx.topology
        node = topo.get(ctx.name) if ctx.name else None
        if node is None:
            if not topo.nodes:
                raise ValueError("topology has no workers")
            node = topo.nodes[0]
            log.warning("worker name %r not found in topology, serving the FIRST node %r",
                        ctx.name, node.name)
        self.node = node
        self.text = ctx.model_type == "text-model"
        self.compute_lock = threading.Lock()
        self.stack = None
        self.units = {}
        if self.text:
            from ..models.llama3.config import LlamaConfig
            from ..models.llama3.factory import load_stack
            cfg = LlamaConfig.from_path(ctx.model_path)
            layers = sorted(_layer_index(l) for l in node.layers if l.startswith("model.layers."))
            self.stack = load_stack(ctx.model_path, cfg, layers, ctx.device, ctx.dtype,
                                    max_seq=ctx.max_seq_len)
            self.stack.max_sessions = 64
            # T = 1 requests replay one captured graph per (session, layer run)
            self.stack.step_graphs = os.environ.get("CAKE_WORKER_GRAPH", "1") != "0"
            log.info("loaded %d blocks on %s (%s)", len(layers), ctx.device, ctx.dtype)
        else:
            from ..models.sd.shardable import load_sd_units
            self.units = load_sd_units(ctx, node.layers)
        host, _, port = ctx.address.rpartition(":")
        from ..utils.native import runtime
        self.server = runtime().WorkerServer(host or "0.0.0.0", int(port), self.info(0), node.name)
        self.port = self.server.port
        fi = os.environ.get("CAKE_FAULT_INJECT", "")
        if fi.startswith("drop_after="):
            self.server.set_drop_after(int(fi.split("=")[1]))
        self.server.set_stats_every(NUM_OPS_TO_STATS)
        self.server.set_compute(self._compute)
        self.server.set_reset(self._reset)
        self.server.set_drop(self._drop_session)
        self.server.set_log(lambda m: log.info("%s", m))
        log.info("worker %s listening on %s:%d", node.name, host, self.port)

    # ------------------------------------------------------------------ info
    def info(self, latency_ms: int) -> dict:
        dev = self.ctx.device
        return {"version": P.PROTO_VERSION,
                "dtype": P.CANDLE_DTYPES.get(self.ctx.dtype, str(self.ctx.dtype)),
                "os": platform.system().lower(), "arch": platform.machine(),
                "device": "rocm" if dev.type == "cuda" else "cpu",
                "device_idx": int(dev.index or 0), "latency": int(latency_ms)}

    # ------------------------------------------------------------------ serving
    def run(self) -> None:
        """Blocking accept loop (native: csrc/runtime/server.cpp)."""
        self.server.serve()

    def serve_in_thread(self) -> threading.Thread:
        t = threading.Thread(target=self.run, daemon=True)
        t.start()
        return t

    def stop(self) -> None:
        self.server.stop()

    def stats(self) -> dict:
        return self.server.stats()

    def _compute(self, session: int, ops, dtype: str, shape, data) -> tuple:
        """Native-server callback: run `ops` on the payload, return (dtype, shape, data).

        The request tensor is a zero-copy view of the native server's receive buffer
        (copied once, straight to the device); the reply is one device-to-host copy
        whose buffer the native server copies into the frame."""
        with warnings.catch_warnings():  # the receive buffer is read-only; it is only read
            warnings.simplefilter("ignore", UserWarning)
            raw = torch.frombuffer(data, dtype=torch.uint8) if len(data) else \
                torch.empty(0, dtype=torch.uint8)
        x = raw.view(P.FROM_CANDLE[dtype]).reshape(list(shape))
        if x.device == self.ctx.device or self.ctx.device.type == "cpu":
            # a CPU worker would compute in place on the server's read-only receive
            # buffer (x.to(cpu) aliases it): take the one copy explicitly instead
            x = x.clone()
        y = self._run_ops(x, ops, session)
        name, shp, buf = P.tensor_payload(y)
        return name, shp, buf

    def _reset(self, session: int) -> None:
        if self.stack is not None:
            with self.compute_lock:
                self.stack.reset(session)

    def _drop_session(self, session: int) -> None:
        if self.stack is not None:
            with self.compute_lock:
                self.stack.drop(session)

    def _run_ops(self, x: torch.Tensor, ops, session: int) -> torch.Tensor:
        if self.text:
            shape = x.shape
            h = x.to(self.ctx.device).float().reshape(-1, shape[-1]).contiguous()
            i = 0
            with self.compute_lock:
                while i < len(ops):  # consecutive ops at one position -> one stack call
                    pos = int(ops[i][1])
                    j = i
                    layers = []
                    while j < len(ops) and int(ops[j][1]) == pos:
                        li = _layer_index(ops[j][0])
                        if li not in self.stack.weights:
                            raise ValueError(f"layer {ops[j][0]} is not served by {self.node.name}")
                        layers.append(li)
                        j += 1
                    self.stack.forward(h, layers, pos, session)
                    i = j
            return h.reshape(shape)
        with self.compute_lock:
            for name, _, _ in ops:
                unit = self.units.get(name)
                if unit is None:
                    raise ValueError(f"{name} is not served by {self.node.name}")
                x = unit.forward_packed(x)
            return x
