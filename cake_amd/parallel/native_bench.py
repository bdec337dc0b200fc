"""bench.py on the native engine (libcake_engine.so): the product path that cake-cli,
the API and the torchrun roles run, measured by the driver.

* one GPU: :func:`measure_native_single` — the whole decode step (embedding, every
  layer, lm_head, repeat penalty, argmax, next-token bookkeeping) is one hipGraph
  replay driven by the engine's C++ token loop (csrc/driver/graph_loop.cpp);
* N ranks (one per GPU): :func:`measure_native_multi` — ``pp``: the reference's layer
  sharding (cake-core/src/models/llama3/llama.rs:95-114), contiguous shards as a
  topology would place them, hops as device-side peer stores inside every rank's
  graph; ``tp``: tensor parallel (beyond the reference), two device-side all-reduces
  per layer inside every rank's graph.

Weights are seeded random-normal draws of the named architecture made on the device
(``NativeLlama(random_init=True)``: only ``config.json`` is written), so a 70B rank
starts in seconds and nothing is read from disk.

Timing (the bench contract): a cold generation (module load, graph capture), then a
generation of W + 1 tokens (prefill + W untimed warm-up steps), then exactly K decode
steps with :meth:`NativeLlama.continue_`, bracketed on rank 0 by a device synchronise
on both sides.  In a multi-rank run every token walks all ranks (pp) or all-reduces
with every rank (tp) inside the replays rank 0 paces, so rank 0's wall clock is the
run's; the other ranks are inside :meth:`NativeLlama.serve` for the whole timed region
and report 0, so the MAX over ranks is rank 0's time.
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile
import time

import torch

from ..models.llama3.config import preset

_PORT_SEQ = [0]  # per-process measurement counter: every rank runs the same sequence


def _prompt(cfg, n: int) -> list[int]:
    g = torch.Generator().manual_seed(1234)
    return torch.randint(0, cfg.vocab_size, (n,), generator=g).tolist()


def _max_seq(a, steps: int, warmup: int) -> int:
    # the KV cache holds the prompt, the cold / warm-up / timed steps and the graph
    # look-ahead (a run longer than --max-seq would stop early)
    need = a.prompt_len + warmup + steps + 16 * max(1, a.steps_per_graph) + 8
    return max(a.max_seq, -(-need // 64) * 64)


def _config_dir(cfg) -> str:
    from ..engine import write_config
    d = tempfile.mkdtemp(prefix="cake_bench_cfg_")
    write_config(d, cfg)
    return d


def _hbm_used_mib() -> float:
    if not torch.cuda.is_available():
        return 0.0
    free, total = torch.cuda.mem_get_info()
    return (total - free) / 2**20


def _timed(eng, cfg, a, steps: int, warmup: int, dump_tokens=None) -> dict:
    """Rank 0 (or the only rank): cold run, warm-up, then exactly `steps` timed tokens."""
    prompt = _prompt(cfg, a.prompt_len)
    kw = dict(temperature=0.0, repeat_penalty=a.repeat_penalty, repeat_last_n=a.repeat_last_n,
              eos_ids=[])  # EOS ignored: exactly K tokens
    eng.generate(prompt, 2, **kw)               # cold: first launches + graph capture
    # TTFT: the best of three warm prefills (one sample swings by ~1 ms with the clock)
    pre = [eng.generate(prompt, 1, **kw).prefill_s for _ in range(2)]
    warm = eng.generate(prompt, 1 + warmup, **kw)  # prefill + first token + W warm-up steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = eng.continue_(steps, eos_ids=[])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if len(r.tokens) != steps:
        raise RuntimeError(f"timed {len(r.tokens)} decode steps, expected {steps}")
    if dump_tokens:
        import json
        with open(dump_tokens, "w") as f:
            json.dump([prompt + warm.tokens + r.tokens], f)
    return {"dt": dt, "ttft_ms_prefill": round(min(pre + [warm.prefill_s]) * 1e3, 3),
            "p50": r.p50_ms, "p99": r.p99_ms}


def measure_native_single(a, model: str, steps: int, warmup: int, dump_tokens=None) -> dict:
    """All layers on cuda:0 in the native engine."""
    from ..engine import NativeLlama
    cfg = preset(model)
    torch.cuda.set_device(0)
    d = _config_dir(cfg)
    t0 = time.time()
    eng = NativeLlama(d, max_seq=_max_seq(a, steps, warmup), dtype=a.dtype, device=0,
                      steps_per_graph=a.steps_per_graph, random_init=True, seed=1)
    print(f"[bench] native {model}: random-init in {time.time() - t0:.1f}s, "
          f"HBM used {_hbm_used_mib() / 1024:.1f} GiB", file=sys.stderr, flush=True)
    try:
        t = _timed(eng, cfg, a, steps, warmup, dump_tokens)
        hbm = _hbm_used_mib()
    finally:
        eng.close()
        shutil.rmtree(d, ignore_errors=True)
    dt = t["dt"]
    return {"tokens_per_sec": round(steps / dt, 3), "ms_per_step": round(dt * 1e3 / steps, 4),
            "p50_token_latency_ms": round(t["p50"], 4), "p99_token_latency_ms": round(t["p99"], 4),
            "ttft_ms_prefill": t["ttft_ms_prefill"], "graph": True,
            "steps_per_graph": max(1, a.steps_per_graph), "engine": "native",
            "hbm_used_mib": round(hbm, 1)}


def measure_native_multi(a, env, model: str, steps: int, warmup: int, mode: str = "pp",
                         dump_tokens=None) -> dict | None:
    """One rank per GPU (env: pipeline_bench.DistEnv) on the native engine; rank 0 gets
    the result dict, the others None."""
    from ..engine import NativeLlama
    rank, world = env.rank, env.world
    cfg = preset(model)
    _PORT_SEQ[0] += 1
    port = int(os.environ.get("MASTER_PORT", "29500")) + 100 + _PORT_SEQ[0]
    addr = f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{port}"
    d = _config_dir(cfg)
    t0 = time.time()
    out = None
    eng = None
    err = None
    try:
        eng = NativeLlama(d, max_seq=_max_seq(a, steps, warmup), dtype=a.dtype,
                          device=env.dev.index or 0, steps_per_graph=1, rank=rank, world=world,
                          master_addr=addr, hop_bf16=a.hop_dtype == "bf16", hop_timeout_s=60.0,
                          connect_timeout_s=300.0, tp=mode == "tp", random_init=True, seed=1)
    except RuntimeError as e:  # the start-up self-test (or the group's start) failed
        err = str(e)
    # every rank agrees: one failed start sends the whole group to the RCCL transport
    if env.max_over_ranks(1.0 if err is not None else 0.0) > 0:
        if eng is not None:
            eng.close()
        shutil.rmtree(d, ignore_errors=True)
        env.release()
        return _dist_fallback(a, env, model, steps, warmup, mode, dump_tokens, err)
    try:
        hbm = _hbm_used_mib()
        if rank == 0:
            print(f"[bench] native {model} {mode}{world}: ranks joined in {time.time() - t0:.1f}s"
                  + (f", walk {eng.walk()}" if mode == "pp" else ""), file=sys.stderr, flush=True)
            t = _timed(eng, cfg, a, steps, warmup, dump_tokens)
            walk = eng.walk() if mode == "pp" else None
            eng.close()  # tells the workers to leave serve()
            dt = t["dt"]
        else:
            eng.serve()
            eng.close()
            dt = 0.0
        eng = None
    finally:
        if eng is not None:
            eng.close()
        shutil.rmtree(d, ignore_errors=True)
    dt = env.max_over_ranks(dt)
    hbm_max = env.max_over_ranks(hbm)
    if rank == 0:
        out = {"tokens_per_sec": round(steps / dt, 3), "ms_per_step": round(dt * 1e3 / steps, 4),
               "p50_token_latency_ms": round(t["p50"], 4),
               "p99_token_latency_ms": round(t["p99"], 4),
               "ttft_ms_prefill": t["ttft_ms_prefill"], "parallel": mode, "streams": 1,
               "engine": "native", "hbm_used_mib_max_rank": round(hbm_max, 1)}
        if mode == "pp":
            out.update({"hop": "ipc" + ("-bf16" if a.hop_dtype == "bf16" else ""),
                        "walk": walk, "hops_per_token": _hops(walk),
                        "layers_per_rank": _layers_per_rank(walk, world)})
        else:
            out.update({"allreduce": "ipc", "allreduces_per_token": 2 * cfg.num_hidden_layers + 1})
    env.release()
    return out


def _dist_fallback(a, env, model, steps, warmup, mode, dump_tokens, err):
    """The record on the Python engines over torch.distributed (RCCL p2p hops / all-reduces)
    after the native group could not start on its device IPC transport; the JSON names
    the transport it ran on and the native start's error."""
    import copy
    from .pipeline_bench import measure_pipeline
    from .tp_bench import measure_tp
    if env.rank == 0:
        print(f"[bench] native {model} {mode}{env.world} did not start ({err}); "
              "falling back to the torch.distributed transport", file=sys.stderr, flush=True)
    a2 = copy.copy(a)
    a2.hop, a2.allreduce, a2.streams = "dist", "dist", 1
    fn = measure_tp if mode == "tp" else measure_pipeline
    r = fn(a2, env, model, steps, warmup, dump_tokens)
    if env.rank == 0 and r is not None:
        r = dict(r)
        r.update({"engine": "python", "native_fallback": (err or "a peer rank failed")[:300]})
        if mode == "pp":
            r["hop"] = "dist"
        else:
            r["allreduce"] = "dist"
    return r


def _hops(walk: str | None) -> int:
    """Edges of the token's walk: master -> run -> ... -> run -> master, one per change
    of rank (rank 0's own runs cost none)."""
    if not walk:
        return 0
    ranks = [0] + [int(r.split(":")[0]) for r in walk.split(",")] + [0]
    return sum(1 for x, y in zip(ranks, ranks[1:]) if x != y)


def _layers_per_rank(walk: str | None, world: int) -> list[int]:
    n = [0] * world
    for run in (walk.split(",") if walk else []):
        r, span = run.split(":")
        lo, hi = span.split("-")
        n[int(r)] += int(hi) - int(lo) + 1
    return n
