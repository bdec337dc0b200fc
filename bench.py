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
* N > 1 (torchrun, one rank per GPU): the layers are sharded contiguously over
  the N ranks as a cake topology would place them (rank 0 = master with
  embedding/lm_head + the first shard); the hidden state hops rank→rank with
  RCCL point-to-point send/recv over xGMI (cake's TCP hop), the last
  shard returns it to the master.  Each rank replays a hipGraph of its shard.
  Batch-1 layer sharding does not add throughput (the work is sequential); the
  curve is reported as strong scaling of one decode stream.

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
    ap.add_argument("--model", default="llama3-8b", choices=["llama3-8b", "llama3-70b", "tiny"])
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
    ap.add_argument("--streams", type=int, default=0,
                    help="N>1: concurrent sequences in the pipeline (default = N; 1 = cake's "
                         "single-sequence pipeline)")
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
        "dtype": a.dtype,
        "data": "synthetic (random-init weights, synthetic prompt ids, EOS ignored)",
        "config": {"model": {"llama3-8b": "Llama-3-8B", "llama3-70b": "Llama-3-70B",
                             "tiny": "tiny"}[a.model],
                   "global_batch": extra.get("streams", 1), "seq_len": a.prompt_len + a.warmup + a.steps,
                   "prompt_len": a.prompt_len,
                   "parallelism": "single" if n == 1 else
                   f"pp{n} (layer-sharded, RCCL p2p, {extra.get('streams', 1)} streams)",
                   "decode": "greedy, repeat_penalty %.2f last_n %d" % (a.repeat_penalty,
                                                                        a.repeat_last_n)},
    }
    out.update(extra)
    print(json.dumps(out), flush=True)


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


def main(argv=None) -> int:
    a = _args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or a.gpus > 1:
        from cake_amd.parallel.pipeline_bench import bench_pipeline
        bench_pipeline(a, _emit)
    else:
        bench_single(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
