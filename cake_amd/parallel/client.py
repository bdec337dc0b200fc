"""Master-side proxy for blocks served by a remote worker (cake-core/src/cake/client.rs).

Connect + ``Hello`` → ``WorkerInfo`` handshake (client.rs:23-47), then
``SingleOp`` (forward_mut, client.rs:99-113) or ``Batch`` (forward_batch,
client.rs:116-124) requests answered by a ``Tensor``.  ``ident()`` is the
worker address, which groups consecutive remote layers into one hop.

Differences from the reference: ONE connection per worker shared by all of
its layers (the reference opens one per layer and uses only the first of each
run); worker-side failures come back as ``Error``
messages raised here as :class:`RemoteError`; ``reset`` clears the worker's KV
for this connection (Q7); requests are serialised by a lock so API threads
can share a client.
"""
from __future__ import annotations

import logging
import threading

import torch

from . import proto as P
from .forwarder import Forwarder

log = logging.getLogger("cake.client")


class RemoteError(RuntimeError):
    pass


class Client(Forwarder):
    def __init__(self, device, address: str, layer_name: str = "", timeout: float = 30.0):
        self.device = torch.device(device)
        self.address = address
        self._layer_name = layer_name
        self._lock = threading.Lock()
        self.conn = P.Connection.connect(address, timeout)
        self.conn.set_timeout(max(timeout, 600.0))
        self.conn.send({"type": P.HELLO})
        msg, _ = self.conn.recv()
        if msg["type"] != P.WORKER_INFO:
            raise RemoteError(f"{address}: unexpected handshake reply {msg['type']}")
        self.info = msg["info"]

    def __str__(self) -> str:  # client.rs:70-84
        i = self.info
        return (f"{self._layer_name}@{self.address} [{i['os']} {i['arch']} {i['device']}:"
                f"{i['device_idx']} {i['dtype']}] latency={i['latency']}ms")

    def layer_name(self) -> str:
        return self._layer_name

    def ident(self) -> str:
        return self.address

    def _request(self, msg: dict, x: torch.Tensor | None) -> torch.Tensor | None:
        with self._lock:
            self.conn.send(msg, x)
            reply, body = self.conn.recv()
        if reply["type"] == P.ERROR:
            raise RemoteError(f"{self.address}: {reply['error']}")
        if reply["type"] == P.TENSOR:
            return P.tensor_from_payload(reply, body, self.device)
        if reply["type"] == P.PONG:
            return None
        raise RemoteError(f"{self.address}: unexpected reply type {reply['type']}")

    def forward(self, x, index_pos, block_idx, session=0):
        return self.forward_mut(x, index_pos, block_idx, session)

    def forward_mut(self, x, index_pos, block_idx, session=0):
        return self._request({"type": P.SINGLE_OP, "layer_name": self._layer_name,
                              "index_pos": int(index_pos), "block_idx": int(block_idx)}, x)

    def forward_named(self, layer_name: str, x: torch.Tensor, index_pos=0, block_idx=0):
        return self._request({"type": P.SINGLE_OP, "layer_name": layer_name,
                              "index_pos": int(index_pos), "block_idx": int(block_idx)}, x)

    def forward_batch(self, x, batch, session=0):
        return self._request({"type": P.BATCH, "batch": [(n, int(p), int(b)) for n, p, b in batch]},
                             x)

    def reset(self, session: int = 0) -> None:
        self._request({"type": P.RESET, "session": int(session)}, None)

    def ping(self) -> None:
        self._request({"type": P.PING}, None)

    def close(self) -> None:
        self.conn.close()


def connect_remote_layers(ctx) -> dict[int, Client]:
    """layer index -> Client for every text-model layer the topology places on a worker."""
    from ..models.llama3.config import LlamaConfig
    cfg = LlamaConfig.from_path(ctx.model_path)
    clients: dict[str, Client] = {}
    remote: dict[int, Client] = {}
    for i in range(cfg.num_hidden_layers):
        node = ctx.topology.get_node_for_layer(f"model.layers.{i}")
        if node is None:
            continue
        if node.name not in clients:
            clients[node.name] = Client(ctx.device, node.host, f"model.layers.{i}")
            log.info("connected %s", clients[node.name])
        remote[i] = clients[node.name]
    return remote
