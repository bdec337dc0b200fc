"""Equivalence invariant: any placement gives the all-local token stream.

Multi-process gloo on CPU, torch backend, tiny random Llama."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cake_amd.models.llama3.config import preset
from cake_amd.models.llama3.factory import random_head, random_model, random_stack
from cake_amd.ops import reference as R
from cake_amd.parallel.pipeline import PipelineEngine, plan_from_owners, shard_layers

CFG = dict(num_hidden_layers=5)
PROMPTS = [[1, 5, 9, 33, 2, 7], [3, 3, 8, 100, 41]]
STEPS = 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reference_tokens(prompt, steps, penalty=1.1, last_n=16):
    cfg = preset("tiny", **CFG)
    m = random_model(cfg, "cpu", torch.float32, max_seq=64)
    toks = list(prompt)
    logits = m.forward(prompt, 0)
    for _ in range(steps + 1):
        t = int(torch.argmax(R.apply_repeat_penalty(logits, penalty, toks[-last_n:])))
        toks.append(t)
        logits = m.forward([t], len(toks) - 1)
    return toks


def _worker(rank, world, port, owners, streams, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = preset("tiny", **CFG)
        mine = [li for li, r in enumerate(owners) if r == rank]
        stack = random_stack(cfg, mine, "cpu", torch.float32, max_seq=64)
        head = random_head(cfg, "cpu", torch.float32) if rank == 0 else None
        eng = PipelineEngine(cfg, stack, owners, rank, world, streams=streams, head=head,
                             repeat_penalty=1.1, repeat_last_n=16)
        for s in range(streams):
            eng.prefill(s, PROMPTS[s] if rank == 0 else None)
        eng.decode(STEPS)
        eng.flush()
        if rank == 0:
            q.put([eng.tokens(s) for s in range(streams)])
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, owners, streams):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, owners, streams, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_plan_and_shards():
    for L, w, hc in ((32, 3, 0.0), (32, 8, 2.4), (80, 8, 1.2), (5, 5, 10.0), (7, 2, 0.0)):
        sh = shard_layers(L, w, hc)
        assert [li for s in sh for li in s] == list(range(L)) and all(sh)
        loads = [len(s) + (hc if r == 0 else 0) for r, s in enumerate(sh)]
        if L >= 2 * w and hc < L / w:
            assert max(loads) - min(loads) <= 1.5
    runs = plan_from_owners([0, 0, 1, 1, 1, 0, 2])
    assert [(r.owner, r.layers) for r in runs] == [(0, [0, 1]), (1, [2, 3, 4]), (0, [5]), (2, [6])]


@pytest.mark.parametrize("world,owners,streams", [
    (2, [0, 0, 1, 1, 1], 1),       # master owns first shard (bench layout)
    (2, [1, 1, 1, 1, 1], 1),       # master owns nothing (pure worker)
    (3, [0, 1, 2, 1, 0], 2),       # non-contiguous, master owns first+last, 2 streams
    (3, [1, 1, 2, 2, 2], 2),
])
def test_pipeline_matches_local(world, owners, streams):
    got = _run(world, owners, streams)
    for s in range(streams):
        assert got[s] == _reference_tokens(PROMPTS[s], STEPS)
