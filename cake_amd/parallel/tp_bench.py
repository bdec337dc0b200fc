"""bench.py's N>1 default: tensor-parallel batch-1 decode, one rank per GPU.

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

import os
import sys
import time

import torch
import torch.distributed as dist

from ..models.llama3.config import preset
from ..models.llama3.factory import parse_dtype
from .pipeline import init_process_group
from .pipeline_bench import _pct
from .tensor_parallel import AllReduce, TPEngine, check_tp, random_shards


def bench_tp(a, emit) -> None:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    cpu = bool(getattr(a, "cpu", False))
    if cpu:
        dev, backend = torch.device("cpu"), "gloo"
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
    else:
        init_process_group("gloo", rank, world)
    fail = os.environ.get("CAKE_BENCH_FAIL_RANK")
    if fail is not None and int(fail) == rank:  # fault injection (tests)
        raise SystemExit(f"[bench] rank {rank}: injected failure")
    cfg = preset(a.model)
    check_tp(cfg, world)
    dtype = torch.float32 if cpu else parse_dtype(a.dtype)
    t0 = time.time()
    blocks, head = random_shards(cfg, rank, world, dev, dtype, seed=1)
    comm = AllReduce(rank, world, dev, cfg.hidden_size, mode=a.allreduce)
    eng = TPEngine(cfg, blocks, head, rank, world, dev, dtype, a.max_seq, comm,
                   repeat_penalty=a.repeat_penalty, repeat_last_n=a.repeat_last_n,
                   use_graph=not a.no_graph)
    sync()
    if rank == 0:
        print(f"[bench] {a.model} tp{world} all-reduce={comm.mode} init {time.time() - t0:.1f}s",
              file=sys.stderr, flush=True)
    ar_us = comm.measure_us()
    g = torch.Generator().manual_seed(1234)
    prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
    eng.prefill(prompt)
    eng.capture()
    for _ in range(a.warmup):
        eng.launch()
    sync()
    eng.check()
    dist.barrier()
    sync()
    evs = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if not cpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
        eng.launch()
    sync()
    dist.barrier()
    sync()
    dt_local = time.perf_counter() - t0
    eng.check()
    if evs:
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        end.synchronize()
        evs.append(end)
    step_ms = [x.elapsed_time(y) for x, y in zip(evs, evs[1:])]
    red_dev = dev if backend == "nccl" else "cpu"
    dt = torch.tensor([dt_local], device=red_dev, dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    hbm = torch.tensor([0.0 if cpu else torch.cuda.max_memory_allocated(dev) / 2**20],
                       device=red_dev)
    dist.all_reduce(hbm, op=dist.ReduceOp.MAX)
    if rank == 0 and getattr(a, "dump_tokens", None):
        import json
        toks = eng.b.hist[:int(eng.b.hist_len.item())].tolist() if eng.hip else eng.tokens
        with open(a.dump_tokens, "w") as f:
            json.dump([toks], f)
    if rank == 0:
        per_tok = step_ms or [dt * 1e3 / a.steps]
        emit(a, a.steps / dt, dt * 1e3 / a.steps, _pct(per_tok, 50), _pct(per_tok, 99), world,
             {"parallel": "tp", "streams": 1, "allreduce": comm.mode,
              "allreduce_us": None if ar_us is None else round(ar_us, 2),
              "allreduces_per_token": 2 * cfg.num_hidden_layers + 1,
              "hbm_peak_mib_max_rank": round(float(hbm.item()), 1)})
    comm.close()
    dist.barrier()
    dist.destroy_process_group()
