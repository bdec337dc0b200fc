#!/usr/bin/env python3
"""Headline benchmark: Llama-3 batch-1 decode tokens/s (+ p50/p99 per-token latency).

BASELINE.json metric: "decode tokens/sec + p50 per-token latency, Llama-3-8B
1-worker & 70B 8-worker".  The reference's formula (cake-core/src/cake/master.rs
:93-121) excludes the first (prefill) token; here the prefill happens before the
timed region and exactly K decode steps are timed.

* Engine: the native engine (libcake_engine.so, ``--engine native``, default) —
  the same C++ engine cake-cli, the REST API and the torchrun roles run; the
  torch-hosted decoders (``--engine python``) remain as test oracles.
* N = 1: all 32 layers local on one MI355X; the whole step (embedding, layers,
  lm_head, repeat penalty 1.1 over the last 128 tokens, argmax, next-token
  bookkeeping) is one hipGraph replay; the engine's C++ loop reads each token back
  one step behind the GPU.  ``llama3_70b.single`` is the same for Llama-3-70B
  (141 GB fits one 288 GB MI355X).
* N > 1 (one rank per GPU; launched by torchrun, or self-launched: with no
  WORLD_SIZE in the environment bench.py spawns the N ranks itself and only
  relays rank 0's JSON line): ``value`` is the reference's parallelism, layer
  sharding (``--parallel pp``, cake-core/src/models/llama3/llama.rs:95-114): the
  layers are sharded contiguously over the N ranks as a cake topology would
  place them (rank 0 = master with embedding/lm_head + the first shard); the
  hidden state hops rank->rank as device-side peer stores over xGMI (bf16
  payload, as the reference ships the model dtype) captured inside every rank's
  decode graph, the last shard returns it to the master.  Batch-1 layer sharding
  does not add throughput (one token walks the ranks in sequence): the curve is
  strong scaling of ONE decode stream.  Extra fields (``--no-extras`` skips them):
  ``tp`` = tensor parallelism (beyond the reference: every rank streams 1/N of
  every layer, device-side all-reduces over xGMI), ``pp_streams`` = the layer-
  sharded pipeline with N independent batch-1 sequences in flight (one per stage:
  the pipeline's aggregate serving throughput; Python pipeline) and
  ``llama3_70b`` = pp / tp for 70B — the BASELINE's "70B 8-worker" point is
  ``llama3_70b.pp`` at N = 8.
* Timing: W untimed warm-up steps, then exactly K decode steps bracketed by a
  device synchronise on both sides on rank 0 (parallel/native_bench.py: in a
  multi-rank run every token walks all ranks inside the replays rank 0 paces).

Weights are random-init of the named architecture (no network, no checkpoints);
EOS is ignored so exactly K tokens are generated.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--model", default="llama3-8b", choices=["llama3-8b", "llama3-70b", "tiny", "tiny-kv2"])
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--max-seq", type=int, default=4096)
    ap.add_argument("--repeat-penalty", type=float, default=1.1)
    ap.add_argument("--repeat-last-n", type=int, default=128)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--steps-per-graph", type=int, default=1,
                    help="greedy decode steps captured per graph launch (per-token latency "
                         "is then measured at that granularity)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 transport: nccl (= RCCL over xGMI) or host-staged gloo (tests)")
    ap.add_argument("--dump-tokens", default=None, help="write generated token ids (JSON)")
    ap.add_argument("--streams", type=int, default=1,
                    help="N>1: concurrent sequences in the pipeline (1 = cake's single-sequence "
                         "pipeline, the headline; S > 1 = aggregate throughput of S sequences)")
    ap.add_argument("--parallel", default="pp", choices=["tp", "pp"],
                    help="N > 1 headline: pp = the reference's layer sharding (default), "
                         "tp = tensor-parallel (every rank 1/N of every layer)")
    ap.add_argument("--no-sd", action="store_true",
                    help="skip the N=1 Stable Diffusion seconds/step sub-record")
    ap.add_argument("--no-extras", action="store_true",
                    help="headline only: skip the tp / llama3_70b sub-records")
    ap.add_argument("--extras", default="all",
                    help="comma list of the sub-records to run: tp (or pp: the other mode), "
                         "pp_streams, 70b_pp, 70b_tp, 70b_single, sd (default: all)")
    ap.add_argument("--tiny-extras", action="store_true",
                    help="run every sub-record (tp, pp_streams, 70B pp/tp, split SD) on the "
                         "tiny presets: the N-rank plumbing of the full default bench, cheap "
                         "enough for CPU (gloo) tests")
    ap.add_argument("--sd-steps", type=int, default=4,
                    help="N>1: timed diffusion steps of the split-UNet sd sub-record")
    ap.add_argument("--allreduce", default="ipc", choices=["ipc", "dist"],
                    help="tp all-reduce: device-side one-shot kernels over xGMI, or "
                         "torch.distributed")
    ap.add_argument("--hop", default="ipc", choices=["ipc", "dist"],
                    help="N>1 decode hop: device-side peer stores in the graph (ipc) or "
                         "host-issued torch.distributed p2p (dist)")
    ap.add_argument("--hop-dtype", default="bf16", choices=["bf16", "f32"],
                    help="hidden-state payload of an ipc hop (the reference ships the model dtype)")
    ap.add_argument("--cpu", action="store_true",
                    help="plumbing check without a GPU (torch reference math, f32, gloo)")
    ap.add_argument("--engine", default="native", choices=["native", "python"],
                    help="native = libcake_engine.so (the product path: cake-cli, the API, the "
                         "torchrun roles); python = the torch-hosted decoders (test oracles)")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launch (N>1 without torchrun): kill the ranks after this many s")
    return ap.parse_args(argv)


def _emit(a, value, ms, p50, p99, n, extra):
    baseline = None  # the reference publishes no number
    out = {
        "metric": "decode_tokens_per_sec",
        "value": round(value, 3),
        "unit": "tokens/s",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "p50_token_latency_ms": round(p50, 4),
        "p99_token_latency_ms": round(p99, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": baseline,
        "dtype": "f32" if getattr(a, "cpu", False) else a.dtype,
        "data": "synthetic (random-init weights, synthetic prompt ids, EOS ignored)",
        "config": {"model": {"llama3-8b": "Llama-3-8B", "llama3-70b": "Llama-3-70B",
                             "tiny": "tiny", "tiny-kv2": "tiny-kv2"}[a.model],
                   "global_batch": extra.get("streams", 1), "seq_len": a.prompt_len + a.warmup + a.steps,
                   "prompt_len": a.prompt_len,
                   "parallelism": "single" if "parallel" not in extra else
                   (f"tp{n} (tensor-parallel, {extra.get('allreduce')} all-reduce)"
                    if extra.get("parallel") == "tp" else
                    f"pp{n} (layer-sharded, {extra.get('hop', 'dist')} hops, "
                    f"{extra.get('streams', 1)} stream(s))"),
                   "decode": "greedy, repeat_penalty %.2f last_n %d" % (a.repeat_penalty,
                                                                        a.repeat_last_n)},
    }
    out.update(extra)
    print(json.dumps(out), flush=True)


def bench_cpu_single(a) -> None:
    """--cpu --gpus 1: the all-local host loop (reference math) — plumbing only."""
    from cake_amd.models.llama3.factory import random_model
    from cake_amd.ops import reference as R
    model = random_model(a.model, "cpu", torch.float32, max_seq=a.max_seq)
    g = torch.Generator().manual_seed(1234)
    prompt = torch.randint(0, model.cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
    toks = list(prompt)
    logits = model.forward(prompt, 0)

    def step():
        nonlocal logits
        t = int(torch.argmax(R.apply_repeat_penalty(logits, a.repeat_penalty,
                                                    toks[-a.repeat_last_n:])))
        toks.append(t)
        logits = model.forward([t], len(toks) - 1)
    for _ in range(a.warmup):
        step()
    times = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t1 = time.perf_counter()
        step()
        times.append((time.perf_counter() - t1) * 1e3)
    dt = time.perf_counter() - t0
    t = int(torch.argmax(R.apply_repeat_penalty(logits, a.repeat_penalty, toks[-a.repeat_last_n:])))
    toks.append(t)
    if a.dump_tokens:
        with open(a.dump_tokens, "w") as f:
            json.dump([toks], f)
    xs = sorted(times)
    _emit(a, a.steps / dt, dt * 1e3 / a.steps, xs[len(xs) // 2], xs[min(len(xs) - 1, int(0.99 * len(xs)))],
          1, {"device": "cpu"})


def measure_single(a, model_name: str, steps: int, warmup: int, dump_tokens=None) -> dict:
    """All layers local on cuda:0 (DeviceDecoder: one graph replay per token)."""
    import gc
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.factory import parse_dtype, random_model
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.context import hbm_mib

    torch.cuda.set_device(0)
    dtype = parse_dtype(a.dtype)
    t0 = time.time()
    # the KV cache holds the prompt and every warm-up / timed step (a longer run than
    # --max-seq allows would stop early and time fewer steps than it reports)
    need = a.prompt_len + warmup + steps + 16 * max(1, a.steps_per_graph)
    max_seq = max(a.max_seq, -(-need // 64) * 64)
    model = random_model(model_name, "cuda:0", dtype, max_seq=max_seq)
    torch.cuda.synchronize()
    load_s = time.time() - t0
    print(f"[bench] model {model_name} random-init in {load_s:.1f}s, "
          f"HBM {torch.cuda.memory_allocated() / 2**30:.1f} GiB", file=sys.stderr, flush=True)
    dec = DeviceDecoder(model, repeat_penalty=a.repeat_penalty, repeat_last_n=a.repeat_last_n,
                        greedy=True, use_graph=not a.no_graph, steps_per_graph=a.steps_per_graph)
    g = torch.Generator().manual_seed(1234)
    prompt = torch.randint(0, model.cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
    dec.start(prompt)  # cold: first-call library/module setup
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dec.start(prompt)  # warm TTFT (prefill + first token), reported separately from tok/s
    torch.cuda.synchronize()
    ttft = (time.perf_counter() - t0) * 1e3
    dec.capture()
    if warmup:
        run_decode(dec, warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = run_decode(dec, steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if len(st.tokens) != steps:
        raise RuntimeError(f"timed {len(st.tokens)} decode steps, expected {steps}")
    if dump_tokens:
        with open(dump_tokens, "w") as f:
            json.dump([dec.bufs.hist[:int(dec.bufs.hist_len.item())].tolist()], f)
    out = {"tokens_per_sec": round(steps / dt, 3), "ms_per_step": round(dt * 1e3 / steps, 4),
           "p50_token_latency_ms": round(st.percentile(50), 4),
           "p99_token_latency_ms": round(st.percentile(99), 4),
           "ttft_ms_prefill": round(ttft, 3), "graph": not a.no_graph,
           "steps_per_graph": dec.k, **hbm_mib()}
    del dec, model, st
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    return out


_MAIN_KEYS = ("tokens_per_sec", "ms_per_step", "p50_token_latency_ms", "p99_token_latency_ms")


def _summary(r: dict | None) -> dict | None:
    """Compact sub-record of one extra measurement."""
    if r is None:
        return None
    keep = _MAIN_KEYS + ("streams", "per_stream_tokens_per_sec", "hop", "hop_us",
                         "hops_per_token", "allreduce", "allreduce_us", "layers_per_rank",
                         "hbm_peak_mib_max_rank", "hbm_peak_mib", "ttft_ms_prefill", "engine",
                         "walk", "hbm_used_mib_max_rank", "hbm_used_mib", "native_fallback")
    return {k: r[k] for k in keep if k in r}


def _extras_on(a) -> bool:
    """Sub-records next to the headline: the full default bench (8B headline on the
    GPU), or the tiny presets with --tiny-extras (CPU plumbing)."""
    if a.no_extras:
        return False
    return bool(a.tiny_extras) or (not a.cpu and a.model == "llama3-8b")


def _extra_runs(a):
    """(key path, model, mode) of the sub-records next to the headline."""
    if not _extras_on(a):
        return []
    m8, m70 = ("tiny-kv2", "tiny") if a.tiny_extras else ("llama3-8b", "llama3-70b")
    other = "tp" if a.parallel == "pp" else "pp"
    # pp_streams: the same layer-sharded pipeline with one sequence in flight per stage
    # (N independent batch-1 requests; aggregate tok/s — the pipeline's serving throughput)
    # the Python pipeline (pp_streams) runs last: a speculative replay it leaves queued
    # on a rank must not share a hardware queue with a later engine's replays
    runs = [((other,), m8, other), (("llama3_70b", "pp"), m70, "pp"),
            (("llama3_70b", "tp"), m70, "tp"), (("pp_streams",), m8, "pp_streams")]
    return [r for r in runs if _want(a, "_".join(("70b",) + r[0][1:]) if r[0][0] == "llama3_70b"
                                     else r[0][0])]


def _want(a, name: str) -> bool:
    """--extras selection (default all)."""
    sel = {x.strip() for x in str(getattr(a, "extras", "all")).split(",") if x.strip()}
    return "all" in sel or name in sel


def _native(a) -> bool:
    # the native engine's hops / all-reduces are the in-graph device IPC ones: a run that
    # asks for the host-staged torch.distributed transports stays on the Python engines
    if getattr(a, "hop", "ipc") == "dist" or getattr(a, "allreduce", "ipc") == "dist":
        return False
    return a.engine == "native" and not a.cpu and not a.no_graph and a.dtype in ("bf16", "f16")


def bench_single(a) -> None:
    if _native(a):
        from cake_amd.parallel.native_bench import measure_native_single as measure
    else:
        measure = measure_single
    r = measure(a, a.model, a.steps, a.warmup, a.dump_tokens)
    extra = {k: v for k, v in r.items() if k not in _MAIN_KEYS}
    if not a.no_extras and a.model == "llama3-8b" and _want(a, "70b_single"):
        # the 70B point on one GPU (135 GB of bf16 weights in 288 GB of HBM)
        try:
            extra["llama3_70b"] = {"single": _summary(measure(a, "llama3-70b", a.steps,
                                                              a.warmup))}
        except Exception as e:  # noqa: BLE001  (the headline stands; the miss is reported)
            extra["llama3_70b"] = {"single": None, "error": f"{type(e).__name__}: {e}"[:300]}
        # the reference's second metric: SD seconds per diffusion step (SDXL 1024^2,
        # CFG batch 2, the UNet + scheduler step as one graph replay)
        if not a.no_sd and _want(a, "sd"):
            try:
                from cake_amd.models.sd.bench import measure_denoise, measure_native
                # native engine (the product path) unless --engine python
                extra["sd"] = {"sdxl_1024": measure_native("xl", 8) if _native(a)
                               else measure_denoise("xl", 8)}
            except Exception as e:  # noqa: BLE001
                extra["sd"] = {"sdxl_1024": None, "error": f"{type(e).__name__}: {e}"[:300]}
    _emit(a, r["tokens_per_sec"], r["ms_per_step"], r["p50_token_latency_ms"],
          r["p99_token_latency_ms"], 1, extra)


def bench_multi(a) -> None:
    """N ranks (torchrun or self-launched): the headline mode, then the extras."""
    import torch.distributed as dist
    from cake_amd.parallel.pipeline_bench import DistEnv, measure_pipeline
    from cake_amd.parallel.tp_bench import measure_tp, tp_supported
    env = DistEnv(a)
    try:
        def measure_streams(a_, env_, model, steps, warmup):
            import copy
            a2 = copy.copy(a_)
            a2.streams = env_.world
            return measure_pipeline(a2, env_, model, steps, warmup)
        measure = {"pp": measure_pipeline, "tp": measure_tp, "pp_streams": measure_streams}
        if _native(a):
            from cake_amd.parallel.native_bench import measure_native_multi

            def native_pp(a_, env_, model, steps, warmup, dump=None):
                return measure_native_multi(a_, env_, model, steps, warmup, "pp", dump)

            def native_tp(a_, env_, model, steps, warmup, dump=None):
                return measure_native_multi(a_, env_, model, steps, warmup, "tp", dump)
            # pp_streams (several sequences in flight) stays on the Python pipeline
            measure.update(pp=native_pp, tp=native_tp)
        head_fn = measure[a.parallel] if a.streams == 1 else measure_pipeline
        head = head_fn(a, env, a.model, a.steps, a.warmup, a.dump_tokens)
        extra = {}
        for path, model, mode in _extra_runs(a):
            if mode == "pp_streams" and (env.world == 1 or a.streams == env.world):
                continue
            if mode == "tp" and not tp_supported(model, env.world):
                r = {"skipped": f"tp{env.world} does not divide the KV heads"}
            else:
                r = _summary(measure[mode](a, env, model, a.steps, a.warmup))
            if env.rank == 0:
                d = extra
                for k in path[:-1]:
                    d = d.setdefault(k, {})
                d[path[-1]] = r
        if _extras_on(a) and not a.no_sd and _want(a, "sd"):
            # BASELINE config 5: SDXL 1024^2 (CFG) with the UNet's block groups split over
            # the N ranks; seconds per diffusion step of one image (parallel/sd_split.py)
            from cake_amd.parallel.sd_split import measure_sd_split
            key = "sdxl_tiny_split" if a.tiny_extras else "sdxl_1024_split"
            r, err = None, None
            if _native(a) and not a.tiny_extras:  # the native engine's split UNet
                from cake_amd.models.sd.bench import measure_native_split
                try:
                    r = measure_native_split(env, "xl", steps=a.sd_steps)
                except Exception as e:  # noqa: BLE001  (falls back below, on every rank)
                    err = f"{type(e).__name__}: {e}"[:300]
                if env.max_over_ranks(1.0 if err else 0.0) == 0:
                    err = None
                else:
                    r = None
                    err = err or "a peer rank failed"
            if r is None and (err is not None or not _native(a) or a.tiny_extras):
                try:
                    r = measure_sd_split(env, steps=a.sd_steps, warmup=2, tiny=a.tiny_extras)
                    if err and r is not None:
                        r = dict(r, native_fallback=err)
                except Exception as e:  # noqa: BLE001  (setup failures are symmetric: all ranks)
                    r = {"error": f"{type(e).__name__}: {e}"[:300]}
            if env.rank == 0:
                extra["sd"] = {key: r}
        if env.rank == 0:
            rest = {k: v for k, v in head.items() if k not in _MAIN_KEYS}
            if a.parallel == "pp":
                weak = env.world > 1 and head["streams"] == env.world
                rest["scaling"] = "weak" if weak else "strong"
            _emit(a, head["tokens_per_sec"], head["ms_per_step"], head["p50_token_latency_ms"],
                  head["p99_token_latency_ms"], env.world, {**rest, **extra})
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(a, argv) -> int:
    """Spawn the N ranks as child processes (before this process touches the GPU),
    relay rank 0's output, and fail fast: if any rank exits non-zero (or the launch
    exceeds --launch-timeout) every other rank is killed and the exit code is
    non-zero."""
    import subprocess
    n = a.gpus
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                      env=env, stdout=subprocess.PIPE if r == 0 else
                                      sys.stderr, text=True))
    deadline = time.time() + a.launch_timeout
    rc = 0
    out = ""
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                print(f"[bench] a rank exited with {rc}; stopping the others", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            if time.time() > deadline:
                rc = 124
                print("[bench] launch timeout; stopping the ranks", file=sys.stderr)
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
        if procs[0].stdout is not None:
            out = procs[0].stdout.read()
    sys.stdout.write(out)
    sys.stdout.flush()
    return rc


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = _args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(a, argv)
    # under torchrun (WORLD_SIZE set) the distributed path runs even at N = 1
    if world > 1 or a.gpus > 1 or "WORLD_SIZE" in os.environ:
        bench_multi(a)
    elif a.cpu:
        bench_cpu_single(a)
    else:
        bench_single(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
