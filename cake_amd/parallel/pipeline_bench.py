"""bench.py's N>1 path: layer-sharded batch-1 decode, one rank per GPU.

The reference's only parallelism is layer sharding with one request in flight
(cake-core/src/models/llama3/llama.rs:95-114, client.rs:116-124): every token
walks master -> worker runs -> master.  Here the hops are device-side peer
stores over xGMI captured in each rank's decode graph (``--hop ipc``, default;
falls back to host-issued RCCL p2p if any link fails its self-test) or
host-issued torch.distributed p2p (``--hop dist``).  ``--streams S`` keeps S
independent sequences in flight (aggregate throughput, reported separately).

Timing: W untimed warm-up tokens, then exactly K tokens bracketed by a barrier
and a device synchronise on both sides; the MAX over ranks is reported.
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

from ..models.llama3.config import preset
from ..models.llama3.factory import parse_dtype, random_head, random_stack
from .pipeline import PipelineEngine, head_cost_in_layers, init_process_group, shard_layers


def _pct(xs: list[float], q: float) -> float:
    if not xs:
        return float("nan")
    xs = sorted(xs)
    return xs[min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))]


def bench_pipeline(a, emit) -> None:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    cpu = bool(getattr(a, "cpu", False))
    if cpu:  # plumbing check without a GPU: torch reference math, gloo
        dev = torch.device("cpu")
        backend = "gloo"
    else:
        local = int(os.environ.get("LOCAL_RANK", str(rank))) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        backend = getattr(a, "dist_backend", "nccl")

    def sync():
        if not cpu:
            torch.cuda.synchronize()
    if backend == "nccl":
        init_process_group("nccl", rank, world, dev)
    else:  # gloo: host-staged control/prefill hops (lets N ranks share one GPU in tests)
        init_process_group("gloo", rank, world)
    fail = os.environ.get("CAKE_BENCH_FAIL_RANK")
    if fail is not None and int(fail) == rank:  # fault injection (tests): this rank dies
        raise SystemExit(f"[bench] rank {rank}: injected failure")
    cfg = preset(a.model)
    dtype = torch.float32 if cpu else parse_dtype(a.dtype)
    shards = shard_layers(cfg.num_hidden_layers, world, head_cost_in_layers(cfg))
    owners = [r for r, sh in enumerate(shards) for _ in sh]
    streams = max(1, a.streams)
    t0 = time.time()
    stack = random_stack(cfg, shards[rank], dev, dtype, a.max_seq, max_sessions=streams)
    head = random_head(cfg, dev, dtype) if rank == 0 else None
    eng = PipelineEngine(cfg, stack, owners, rank, world, streams=streams, head=head,
                         repeat_penalty=a.repeat_penalty, repeat_last_n=a.repeat_last_n,
                         use_graph=not a.no_graph, hop=a.hop, hop_bf16=a.hop_dtype == "bf16",
                         steps_per_graph=a.steps_per_graph)
    sync()
    if rank == 0:
        print(f"[bench] {a.model} pp{world} streams={streams} hop={eng.hop} layers/rank="
              f"{[len(s) for s in shards]} init {time.time() - t0:.1f}s", file=sys.stderr,
              flush=True)
    hop_us = eng.measure_hop_us()
    g = torch.Generator().manual_seed(1234)
    for s in range(streams):
        prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
        eng.prefill(s, prompt if rank == 0 else None)
    eng.flush()
    eng.capture()
    if a.warmup:
        eng.decode(a.warmup)
    eng.flush()
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    eng.decode(a.steps)
    eng.flush()
    sync()
    dist.barrier()
    sync()
    dt_local = time.perf_counter() - t0
    eng.check_hops()
    step_ms = eng.step_times_ms() if rank == 0 else []
    red_dev = dev if backend == "nccl" else "cpu"
    dt = torch.tensor([dt_local], device=red_dev, dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    hbm = torch.tensor([0.0 if cpu else torch.cuda.max_memory_allocated(dev) / 2**20],
                       device=red_dev)
    dist.all_reduce(hbm, op=dist.ReduceOp.MAX)
    if rank == 0 and getattr(a, "dump_tokens", None):
        import json
        with open(a.dump_tokens, "w") as f:
            json.dump([eng.tokens(s) for s in range(streams)], f)
    if rank == 0:
        k = eng.k if (eng.hop == "ipc" and streams == 1) else 1
        per_tok = [x / k for x in step_ms] if step_ms else [dt * 1e3 / a.steps]
        emit(a, streams * a.steps / dt, dt * 1e3 / a.steps, _pct(per_tok, 50), _pct(per_tok, 99),
             world,
             {"parallel": "pp", "streams": streams,
              "per_stream_tokens_per_sec": round(a.steps / dt, 3),
              "hop": eng.hop + ("-bf16" if eng.hop == "ipc" and eng.hop_bf16 else ""),
              "hop_us": None if hop_us is None else round(hop_us, 2),
              "hops_per_token": sum(1 for k in range(1, len(eng.runs) + 2) if eng._recv_point(k)),
              "layers_per_rank": [len(s) for s in shards],
              "hbm_peak_mib_max_rank": round(float(hbm.item()), 1),
              "scaling": "weak" if streams == world else "strong"})
    dist.barrier()
    dist.destroy_process_group()
