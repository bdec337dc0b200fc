"""bench.py's tensor-parallel measurement (beyond-reference; reported beside the
layer-sharded headline), one rank per GPU.

Each rank holds 1/N of every layer (parallel/tensor_parallel.py), so one decode
stream gets N GPUs' HBM bandwidth — the MI355X-first alternative to the
reference's layer sharding (``--parallel pp``, parallel/pipeline_bench.py).  The
per-layer all-reduces are device-side one-shot kernels over xGMI inside each
rank's decode graph (``--allreduce ipc``, default; falls back to RCCL if the
self-test fails) or torch.distributed (``--allreduce dist``).

Timing: W untimed warm-up tokens, then exactly K tokens bracketed by a barrier
and a device synchronise on both sides; the MAX over ranks is reported.
"""
from __future__ import annotations

import sys
import time

import torch
import torch.distributed as dist

from ..models.llama3.config import preset
from ..models.llama3.factory import parse_dtype
from .pipeline_bench import DistEnv, _pct
from .tensor_parallel import AllReduce, TPEngine, check_tp, random_shards


def tp_supported(model: str, world: int) -> bool:
    try:
        check_tp(preset(model), world)
        return True
    except ValueError:
        return False


def measure_tp(a, env: DistEnv, model: str, steps: int, warmup: int,
               dump_tokens: str | None = None) -> dict | None:
    rank, world, dev = env.rank, env.world, env.dev
    cfg = preset(model)
    check_tp(cfg, world)
    dtype = torch.float32 if env.cpu else parse_dtype(a.dtype)
    t0 = time.time()
    blocks, head = random_shards(cfg, rank, world, dev, dtype, seed=1)
    comm = AllReduce(rank, world, dev, cfg.hidden_size, mode=a.allreduce)
    eng = TPEngine(cfg, blocks, head, rank, world, dev, dtype, a.max_seq, comm,
                   repeat_penalty=a.repeat_penalty, repeat_last_n=a.repeat_last_n,
                   use_graph=not a.no_graph)
    env.sync()
    if rank == 0:
        print(f"[bench] {model} tp{world} all-reduce={comm.mode} init {time.time() - t0:.1f}s",
              file=sys.stderr, flush=True)
    ar_us = comm.measure_us()
    g = torch.Generator().manual_seed(1234)
    prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
    eng.prefill(prompt)
    eng.capture()
    for _ in range(warmup):
        eng.launch()
    env.sync()
    eng.check()
    dist.barrier()
    env.sync()
    evs = []
    t0 = time.perf_counter()
    for _ in range(steps):
        if not env.cpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
        eng.launch()
    env.sync()
    dist.barrier()
    env.sync()
    dt_local = time.perf_counter() - t0
    eng.check()
    if evs:
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        end.synchronize()
        evs.append(end)
    step_ms = [x.elapsed_time(y) for x, y in zip(evs, evs[1:])]
    dt = env.max_over_ranks(dt_local)
    hbm = env.hbm_peak_mib()
    if rank == 0 and dump_tokens:
        import json
        toks = eng.b.hist[:int(eng.b.hist_len.item())].tolist() if eng.hip else eng.tokens
        with open(dump_tokens, "w") as f:
            json.dump([toks], f)
    out = None
    if rank == 0:
        per_tok = step_ms or [dt * 1e3 / steps]
        out = {"tokens_per_sec": round(steps / dt, 3), "ms_per_step": round(dt * 1e3 / steps, 4),
               "p50_token_latency_ms": round(_pct(per_tok, 50), 4),
               "p99_token_latency_ms": round(_pct(per_tok, 99), 4),
               "parallel": "tp", "streams": 1, "allreduce": comm.mode,
               "allreduce_us": None if ar_us is None else round(ar_us, 2),
               "allreduces_per_token": 2 * cfg.num_hidden_layers + 1,
               "hbm_peak_mib_max_rank": round(hbm, 1)}
    comm.close()
    del eng, blocks, head, comm
    env.release()
    return out


def bench_tp(a, emit) -> None:
    """Stand-alone tp measurement (one JSON line)."""
    env = DistEnv(a)
    try:
        r = measure_tp(a, env, a.model, a.steps, a.warmup, getattr(a, "dump_tokens", None))
        if r is not None:
            emit(a, r["tokens_per_sec"], r["ms_per_step"], r["p50_token_latency_ms"],
                 r["p99_token_latency_ms"], env.world,
                 {k: v for k, v in r.items() if k not in ("tokens_per_sec", "ms_per_step",
                                                           "p50_token_latency_ms",
                                                           "p99_token_latency_ms")})
        dist.barrier()
    finally:
        dist.destroy_process_group()
