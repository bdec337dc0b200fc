"""Tensor-parallel decode (parallel/tensor_parallel.py): N ranks holding 1/N of every
layer produce the all-local token stream.  Multi-process gloo on CPU, torch backend."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cake_amd.models.llama3.config import preset
from cake_amd.models.llama3.factory import random_model
from cake_amd.ops import reference as R
from cake_amd.parallel.tensor_parallel import (AllReduce, TPEngine, check_tp, shard_block,
                                               shard_head, split_range)

CFG = dict(num_hidden_layers=3, num_attention_heads=4, num_key_value_heads=2,
           intermediate_size=520, vocab_size=509)


def _cfg(world):
    # TP needs nkv % world == 0: widen the GQA geometry for 4 and 8 ranks (n_rep 2 kept)
    if world > 2:
        return preset("tiny", **dict(CFG, num_attention_heads=2 * world,
                                     num_key_value_heads=world))
    return preset("tiny", **CFG)
PROMPT = [1, 5, 9, 33, 2, 7]
STEPS = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reference_tokens(world, penalty=1.1, last_n=16):
    cfg = _cfg(world)
    m = random_model(cfg, "cpu", torch.float32, max_seq=64, seed=3)
    toks = list(PROMPT)
    logits = m.forward(PROMPT, 0)
    for _ in range(STEPS + 1):
        t = int(torch.argmax(R.apply_repeat_penalty(logits, penalty, toks[-last_n:])))
        toks.append(t)
        logits = m.forward([t], len(toks) - 1)
    return toks


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _cfg(world)
        m = random_model(cfg, "cpu", torch.float32, max_seq=64, seed=3)
        blocks = {li: shard_block(w, cfg, rank, world) for li, w in m.stack.weights.items()}
        head = shard_head(m.head.embed, m.head.norm, m.head.lm_head, rank, world)
        comm = AllReduce(rank, world, "cpu", cfg.hidden_size)
        eng = TPEngine(cfg, blocks, head, rank, world, "cpu", torch.float32, 64, comm,
                       repeat_penalty=1.1, repeat_last_n=16)
        eng.prefill(PROMPT)
        eng.decode(STEPS)
        q.put((rank, eng.tokens))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_tp_matches_all_local(world):
    ref = _reference_tokens(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r] == ref, (r, got[r], ref)


def test_split_and_checks():
    assert [split_range(10, 3, r) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert [split_range(128256, 8, r)[1] - split_range(128256, 8, r)[0] for r in range(8)] == [16032] * 8
    check_tp(preset("llama3-8b"), 8)
    check_tp(preset("llama3-70b"), 8)
    with pytest.raises(ValueError):
        check_tp(preset("llama3-8b"), 3)


def _sample_worker(rank, world, port, q):
    from cake_amd.models.sampling import SamplingConfig
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _cfg(world)
        m = random_model(cfg, "cpu", torch.float32, max_seq=64, seed=3)
        blocks = {li: shard_block(w, cfg, rank, world) for li, w in m.stack.weights.items()}
        head = shard_head(m.head.embed, m.head.norm, m.head.lm_head, rank, world)
        comm = AllReduce(rank, world, "cpu", cfg.hidden_size, n_gather=cfg.vocab_size)
        eng = TPEngine(cfg, blocks, head, rank, world, "cpu", torch.float32, 64, comm,
                       repeat_penalty=1.1, repeat_last_n=16)
        out = []
        for seed in (11, 12):
            eng.set_sampling(SamplingConfig(temperature=0.9, top_k=40, top_p=0.9, seed=seed))
            eng.prefill(PROMPT)
            eng.decode(STEPS)
            out.append(list(eng.tokens))
        q.put((rank, out))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_tp_sampling_matches_all_local():
    """temperature / top-k / top-p under TP: the gathered full logits give every rank
    the reference's draw (host LogitsProcessor, same seed) -> the all-local stream."""
    from cake_amd.models.sampling import LogitsProcessor, SamplingConfig
    world = 2
    cfg = _cfg(world)
    m = random_model(cfg, "cpu", torch.float32, max_seq=64, seed=3)
    ref = []
    for seed in (11, 12):
        lp = LogitsProcessor(SamplingConfig(temperature=0.9, top_k=40, top_p=0.9, seed=seed))
        toks = list(PROMPT)
        logits = m.forward(PROMPT, 0)
        for _ in range(STEPS + 1):
            t = lp.sample(R.apply_repeat_penalty(logits, 1.1, toks[-16:]))
            toks.append(t)
            logits = m.forward([t], len(toks) - 1)
        ref.append(toks)
    assert ref[0] != ref[1]   # the seed matters
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sample_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1] == ref
