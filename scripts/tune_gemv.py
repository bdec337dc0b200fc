"""Sweep the decode-GEMV launch geometry (U, prefetch, grid cap) per kernel kind.

Each configuration is timed as a hipGraph of `reps` back-to-back launches over
rotating weight copies (> 512 MiB in total, so the 256 MiB Infinity Cache cannot
serve repeats — as in the real 15 GB/token stream).  Rounds are interleaved in
one process (cdna guide §5.4 rule 24); we report the median per launch and the
effective HBM bandwidth.
"""
import argparse
import itertools
import json
import statistics
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402


def make_case(kind, H, I, nh, nkv, hd, V, dt, dev):
    copies = []
    budget = 600 * 2**20
    f32 = torch.float32
    resid = torch.randn(H, device=dev)
    nw = torch.ones(H, device=dev, dtype=dt)
    if kind == "qkv":
        per = (nh + 2 * nkv) * hd * H * 2
        n = max(2, budget // per)
        for _ in range(n):
            copies.append(tuple(torch.randn(r * hd, H, device=dev).mul_(0.02).to(dt) for r in (nh, nkv, nkv)))
        invf = torch.ones(hd // 2, device=dev)
        pos = torch.zeros(1, dtype=torch.int32, device=dev)
        q = torch.empty(nh * hd, device=dev)
        kc = torch.zeros(nkv, 128, hd, device=dev, dtype=dt)
        vc = torch.zeros_like(kc)
        fn = lambda w: K.qkv_rope(resid, nw, 1e-5, w[0], w[1], w[2], invf, pos, q, kc, vc)
        return copies, fn, per
    if kind == "swiglu":
        per = 2 * I * H * 2
        n = max(2, budget // per)
        copies = [(torch.randn(I, H, device=dev).mul_(0.02).to(dt),
                   torch.randn(I, H, device=dev).mul_(0.02).to(dt)) for _ in range(n)]
        act = torch.empty(I, device=dev, dtype=dt)
        fn = lambda w: K.swiglu(resid, nw, 1e-5, w[0], w[1], act)
        return copies, fn, per
    if kind in ("o_proj", "down"):
        Kd = H if kind == "o_proj" else I
        per = H * Kd * 2
        n = max(2, budget // per)
        copies = [torch.randn(H, Kd, device=dev).mul_(0.02).to(dt) for _ in range(n)]
        x = torch.randn(Kd, device=dev).to(dt)
        out = torch.zeros(H, device=dev, dtype=f32)
        fn = lambda w: K.gemv(x, w, out, accumulate=True)
        return copies, fn, per
    if kind == "lm_head":
        per = V * H * 2
        n = max(2, budget // per)
        copies = [torch.randn(V, H, device=dev).mul_(0.02).to(dt) for _ in range(n)]
        out = torch.empty(V, device=dev, dtype=f32)
        fn = lambda w: K.norm_gemv_f32(resid, nw, 1e-5, w, out)
        return copies, fn, per
    raise ValueError(kind)


TUNE_KIND = {"qkv": "qkv", "swiglu": "swiglu", "o_proj": "x16", "down": "x16", "lm_head": "norm_f32"}


def time_config(copies, fn, reps):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(copies[0])
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(copies[i % len(copies)])
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps  # us per launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="8b", choices=["8b", "70b"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=64)
    ap.add_argument("--kinds", default="qkv,swiglu,o_proj,down,lm_head")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    if a.model == "8b":
        H, I, nh, nkv, hd, V = 4096, 14336, 32, 8, 128, 128256
    else:
        H, I, nh, nkv, hd, V = 8192, 28672, 64, 8, 128, 128256
    configs = list(itertools.product((2, 4, 8), (0, 4, 8), (256, 512, 1024, 2048)))
    results = {}
    for kind in a.kinds.split(","):
        copies, fn, per = make_case(kind, H, I, nh, nkv, hd, V, dt, dev)
        times = {c: [] for c in configs}
        for _ in range(a.rounds):
            for c in configs:
                K.set_gemv_tuning(TUNE_KIND[kind], U=c[0], prefetch=c[1], max_blocks=c[2])
                times[c].append(time_config(copies, fn, a.reps))
        K.set_gemv_tuning(TUNE_KIND[kind])
        rows = sorted(((statistics.median(v), min(v), c) for c, v in times.items()))
        print(f"== {kind} ({per / 2**20:.1f} MiB per launch)")
        for med, mn, c in rows[:8]:
            print(f"  U={c[0]} pf={int(c[1])} mb={c[2]:5d}  median {med:8.2f} us  min {mn:8.2f} us  "
                  f"{per / med / 1e6:6.2f} TB/s")
        base = statistics.median(times[(4, 0, 1024)])
        print(f"  default U=4 pf=0 mb=1024: {base:.2f} us  {per / base / 1e6:.2f} TB/s")
        results[kind] = [{"U": c[0], "pf": c[1], "mb": c[2], "median_us": med, "min_us": mn}
                         for med, mn, c in rows]
        del copies
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
