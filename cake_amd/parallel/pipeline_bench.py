"""bench.py's N>1 headline: layer-sharded batch-1 decode, one rank per GPU.

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

import gc
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


class DistEnv:
    """rank / world / device / backend of a bench rank; the process group is created
    once and shared by every measurement of the run (pp, tp, 8B, 70B)."""

    def __init__(self, a):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        self.cpu = bool(getattr(a, "cpu", False))
        if self.cpu:  # plumbing check without a GPU: torch reference math, gloo
            self.dev = torch.device("cpu")
            self.backend = "gloo"
        else:
            local = int(os.environ.get("LOCAL_RANK", str(self.rank))) % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            self.dev = torch.device("cuda", local)
            self.backend = getattr(a, "dist_backend", "nccl")
        if not dist.is_initialized():
            if self.backend == "nccl":
                init_process_group("nccl", self.rank, self.world, self.dev)
            else:  # gloo: host-staged control/prefill hops (N ranks may share one GPU in tests)
                init_process_group("gloo", self.rank, self.world)
        fail = os.environ.get("CAKE_BENCH_FAIL_RANK")
        if fail is not None and int(fail) == self.rank:  # fault injection (tests)
            raise SystemExit(f"[bench] rank {self.rank}: injected failure")

    def sync(self) -> None:
        if not self.cpu:
            torch.cuda.synchronize()

    @property
    def red_dev(self):
        return self.dev if self.backend == "nccl" else "cpu"

    def max_over_ranks(self, x: float) -> float:
        t = torch.tensor([x], device=self.red_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def hbm_peak_mib(self) -> float:
        return self.max_over_ranks(0.0 if self.cpu else torch.cuda.max_memory_allocated(self.dev) / 2**20)

    def release(self) -> None:
        """Free one measurement's model before the next one allocates."""
        gc.collect()
        if not self.cpu:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(self.dev)
        dist.barrier()


def measure_pipeline(a, env: DistEnv, model: str, steps: int, warmup: int,
                     dump_tokens: str | None = None) -> dict | None:
    """Layer-sharded decode of `model` over env.world ranks; rank 0 gets the result dict
    (tokens/s, ms/token, p50/p99, hop info), the other ranks None."""
    rank, world, dev = env.rank, env.world, env.dev
    cfg = preset(model)
    dtype = torch.float32 if env.cpu else parse_dtype(a.dtype)
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
    env.sync()
    if rank == 0:
        print(f"[bench] {model} pp{world} streams={streams} hop={eng.hop} layers/rank="
              f"{[len(s) for s in shards]} init {time.time() - t0:.1f}s", file=sys.stderr,
              flush=True)
    hop_us = eng.measure_hop_us()
    g = torch.Generator().manual_seed(1234)
    for s in range(streams):
        prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
        eng.prefill(s, prompt if rank == 0 else None)
    eng.flush()
    eng.capture()
    k = eng.k if (eng.hop == "ipc" and streams == 1) else 1
    if warmup:
        eng.decode(-(-warmup // k) * k)
    eng.flush()
    env.sync()
    dist.barrier()
    env.sync()
    t0 = time.perf_counter()
    eng.decode(steps)
    eng.flush()
    env.sync()
    dist.barrier()
    env.sync()
    dt_local = time.perf_counter() - t0
    eng.check_hops()
    step_ms = eng.step_times_ms() if rank == 0 else []
    dt = env.max_over_ranks(dt_local)
    hbm = env.hbm_peak_mib()
    if rank == 0 and dump_tokens:
        import json
        with open(dump_tokens, "w") as f:
            json.dump([eng.tokens(s) for s in range(streams)], f)
    out = None
    if rank == 0:
        per_tok = [x / k for x in step_ms] if step_ms else [dt * 1e3 / steps]
        out = {"tokens_per_sec": round(streams * steps / dt, 3),
               "ms_per_step": round(dt * 1e3 / steps, 4),
               "p50_token_latency_ms": round(_pct(per_tok, 50), 4),
               "p99_token_latency_ms": round(_pct(per_tok, 99), 4),
               "parallel": "pp", "streams": streams,
               "per_stream_tokens_per_sec": round(steps / dt, 3),
               "hop": eng.hop + ("-bf16" if eng.hop == "ipc" and eng.hop_bf16 else ""),
               "hop_us": None if hop_us is None else round(hop_us, 2),
               "hops_per_token": eng.hops_per_token(),
               "layers_per_rank": [len(s) for s in shards],
               "hbm_peak_mib_max_rank": round(hbm, 1)}
    eng.close()
    del eng, stack, head
    env.release()
    return out


def bench_pipeline(a, emit) -> None:
    """Stand-alone pp measurement (one JSON line; kept for --only-headline runs and tests)."""
    env = DistEnv(a)
    try:
        r = measure_pipeline(a, env, a.model, a.steps, a.warmup, getattr(a, "dump_tokens", None))
        if r is not None:
            emit(a, r["tokens_per_sec"], r["ms_per_step"], r["p50_token_latency_ms"],
                 r["p99_token_latency_ms"], env.world,
                 {k: v for k, v in r.items() if k not in ("tokens_per_sec", "ms_per_step",
                                                           "p50_token_latency_ms",
                                                           "p99_token_latency_ms")}
                 | {"scaling": "weak" if env.world > 1 and r["streams"] == env.world else "strong"})
        dist.barrier()
    finally:
        dist.destroy_process_group()
