"""Loopback transport: the whole master/worker deployment in ONE process.

Every topology node gets an in-process worker (native WorkerServer on an
ephemeral 127.0.0.1 port, its own weights / KV sessions, exactly the code a
remote worker runs) and the topology hosts are rewritten to those ports, so the
master talks the real wire protocol ("loopback").  Used by
``--transport loopback`` and by tests; no network or extra processes needed.
"""
from __future__ import annotations

import dataclasses
import logging

from .worker import Worker

log = logging.getLogger("cake.loopback")


def start_loopback_workers(ctx) -> list[Worker]:
    workers = []
    for node in ctx.topology.nodes:
        wctx = dataclasses.replace(ctx, mode="worker", name=node.name, address="127.0.0.1:0")
        w = Worker(wctx)
        w.serve_in_thread()
        node.host = f"127.0.0.1:{w.port}"
        log.info("loopback worker %s on %s (%d layers)", node.name, node.host, len(node.layers))
        workers.append(w)
    return workers


def stop_loopback_workers(workers: list[Worker]) -> None:
    for w in workers:
        w.stop()
