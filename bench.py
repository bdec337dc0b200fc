#!/usr/bin/env python3
"""Headline benchmark: Llama-3 batch-1 greedy decode tokens/s (+ p50/p99 per-token latency).

BASELINE.json metric: "decode tokens/sec + p50 per-token latency, Llama-3-8B
1-worker & 70B 8-worker".  The reference's formula (cake-core/src/cake/master.rs
:93-121) excludes the first (prefill) token; here the prefill happens before the
timed region and exactly K decode steps are timed.

* N = 1: all 32 layers local on one MI355X; the whole step (embedding, layers,
  lm_head, repeat penalty 1.1 over the last 128 tokens, argmax, next-token
  bookkeeping) is one hipGraph replay; the host reads each token back one step
  behind the GPU.
* N > 1 (one rank per GPU; launched by torchrun, or self-launched: with no
  WORLD_SIZE in the environment bench.py spawns the N ranks itself and only
  relays rank 0's JSON line), default ``--parallel tp``: every rank holds 1/N
  of every layer (heads, MLP rows, vocabulary) and streams 1/N of the weights
  per token; the two per-layer all-reduces and the argmax max are device-side
  one-shot kernels over xGMI inside each rank's decode graph
  (parallel/tensor_parallel.py).  ``--parallel pp``: the reference's layer
  sharding — the layers are sharded contiguously over the N
  ranks as a cake topology would place them (rank 0 = master with
  embedding/lm_head + the first shard); the hidden state hops rank→rank as
  device-side peer stores over xGMI captured inside every rank's decode graph
  (cake's TCP hop; --hop dist = host-issued RCCL p2p), the last
  shard returns it to the master.  Batch-1 layer sharding does not add
  throughput (one token walks the ranks in sequence): the curve is strong
  scaling of ONE decode stream (--streams S > 1 keeps S sequences in flight and
  reports their aggregate instead).

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
    ap.add_argument("--parallel", default="tp", choices=["tp", "pp"],
                    help="N > 1: tp = tensor-parallel (every rank 1/N of every layer, default), "
                         "pp = the reference's layer sharding (pipeline)")
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


def bench_single(a) -> None:
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.factory import parse_dtype, random_model
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.context import hbm_mib

    torch.cuda.set_device(0)
    dtype = parse_dtype(a.dtype)
    t0 = time.time()
    model = random_model(a.model, "cuda:0", dtype, max_seq=a.max_seq)
    torch.cuda.synchronize()
    load_s = time.time() - t0
    print(f"[bench] model {a.model} random-init in {load_s:.1f}s, "
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
    if a.warmup:
        run_decode(dec, a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = run_decode(dec, a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if a.dump_tokens:
        with open(a.dump_tokens, "w") as f:
            json.dump([dec.bufs.hist[:int(dec.bufs.hist_len.item())].tolist()], f)
    _emit(a, a.steps / dt, dt * 1e3 / a.steps, st.percentile(50), st.percentile(99), 1,
          {"ttft_ms_prefill": round(ttft, 3), "graph": not a.no_graph,
           "steps_per_graph": dec.k, **hbm_mib()})


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
        if a.parallel == "tp":
            from cake_amd.parallel.tp_bench import bench_tp
            bench_tp(a, _emit)
        else:
            from cake_amd.parallel.pipeline_bench import bench_pipeline
            bench_pipeline(a, _emit)
    elif a.cpu:
        bench_cpu_single(a)
    else:
        bench_single(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
