"""The shardable-unit interface (cake-core/src/cake/mod.rs:103-146 ``trait Forwarder``).

``forward``/``forward_mut`` run one unit, ``forward_batch`` runs a contiguous
run of units in one hop, ``ident`` is "local" for in-process units and the
worker address for remote proxies (it drives contiguous-block batching).
"""
from __future__ import annotations

import torch


class Forwarder:
    def layer_name(self) -> str:
        raise NotImplementedError

    def ident(self) -> str:
        return "local"

    def forward(self, x: torch.Tensor, index_pos: int, block_idx: int, session: int = 0):
        raise NotImplementedError

    def forward_mut(self, x: torch.Tensor, index_pos: int, block_idx: int, session: int = 0):
        return self.forward(x, index_pos, block_idx, session)

    def forward_batch(self, x: torch.Tensor, batch: list[tuple[str, int, int]], session: int = 0):
        raise NotImplementedError("forward_batch")  # mod.rs: default unimplemented!

    def reset(self, session: int = 0) -> None:
        pass
