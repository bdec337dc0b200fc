"""bench.py's N>1 path: layer-sharded decode over RCCL (see parallel/pipeline.py)."""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

from ..models.llama3.config import preset
from ..models.llama3.factory import parse_dtype, random_head, random_stack
from .pipeline import PipelineEngine, head_cost_in_layers, init_process_group, shard_layers


def bench_pipeline(a, emit) -> None:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank))) % max(1, torch.cuda.device_count())
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = getattr(a, "dist_backend", "nccl")
    if backend == "nccl":
        init_process_group("nccl", rank, world, dev)
    else:  # gloo: host-staged hops (lets N ranks share one GPU in tests)
        init_process_group("gloo", rank, world)
    cfg = preset(a.model)
    dtype = parse_dtype(a.dtype)
    shards = shard_layers(cfg.num_hidden_layers, world, head_cost_in_layers(cfg))
    owners = [r for r, sh in enumerate(shards) for _ in sh]
    streams = a.streams if a.streams > 0 else world
    t0 = time.time()
    stack = random_stack(cfg, shards[rank], dev, dtype, a.max_seq, max_sessions=streams)
    head = random_head(cfg, dev, dtype) if rank == 0 else None
    eng = PipelineEngine(cfg, stack, owners, rank, world, streams=streams, head=head,
                         repeat_penalty=a.repeat_penalty, repeat_last_n=a.repeat_last_n,
                         use_graph=not a.no_graph)
    torch.cuda.synchronize()
    if rank == 0:
        print(f"[bench] {a.model} pp{world} streams={streams} layers/rank="
              f"{[len(s) for s in shards]} init {time.time() - t0:.1f}s", file=sys.stderr,
              flush=True)
    g = torch.Generator().manual_seed(1234)
    for s in range(streams):
        prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
        eng.prefill(s, prompt if rank == 0 else None)
    eng.capture()
    if a.warmup:
        eng.decode(a.warmup)
    eng.flush()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.decode(a.steps)
    eng.flush()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    hbm = torch.tensor([torch.cuda.max_memory_allocated(dev) / 2**20],
                       device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(hbm, op=dist.ReduceOp.MAX)
    if rank == 0 and getattr(a, "dump_tokens", None):
        import json
        with open(a.dump_tokens, "w") as f:
            json.dump([eng.tokens(s) for s in range(streams)], f)
    if rank == 0:
        ms_round = dt * 1e3 / a.steps
        emit(a, streams * a.steps / dt, ms_round, ms_round, ms_round, world,
             {"streams": streams, "per_stream_tokens_per_sec": round(a.steps / dt, 3),
              "note": "per-token latency = decode round time (one token per stream per round)",
              "hbm_peak_mib_max_rank": round(float(hbm.item()), 1),
              "scaling": "weak" if streams == world else "strong"})
    dist.barrier()
    dist.destroy_process_group()
