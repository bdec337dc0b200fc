"""Ping-pong 256x256 GEMM (cfg 20) against the interleaved 256x256 tile (cfg 5, or the
table's MFMA plan) and the library GEMM (hipBLASLt) on the Llama prefill projections and
8192^3, interleaved rounds in one process on random operands, each checked against an
f32 reference.  One JSON line per shape.

Usage: python scripts/bench_gemm_pp.py [--shapes 8b,70b,sq] [--ms 2048]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import gemm as G  # noqa: E402

MODELS = {"8b": (4096, 14336, 4096, 1024), "70b": (8192, 28672, 8192, 1024)}


def shapes(which, ms):
    out = []
    for w in which:
        if w == "sq":
            out.append(("sq8192", 8192, 8192, 8192, "store"))
            out.append(("sq4096", 4096, 4096, 4096, "store"))
            continue
        H, I, nq, nk = MODELS[w]
        for M in ms:
            out += [(f"{w}_qkv_t{M}", M, nq + 2 * nk, H, "store"),
                    (f"{w}_o_t{M}", M, H, nq, "resid32"),
                    (f"{w}_gateup_t{M}", M, 2 * I, H, "swiglu"),
                    (f"{w}_down_t{M}", M, H, I, "resid32")]
    return out


def timeit(fn, reps=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="sq,8b,70b")
    ap.add_argument("--ms", default="2048")
    ap.add_argument("--arms", default="mfma,rs,rs2,lib")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    torch.manual_seed(0)
    arms = a.arms.split(",")
    for name, M, Nv, K, epi in shapes(a.shapes.split(","), [int(m) for m in a.ms.split(",")]):
        w = (torch.rand(Nv, K, device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        N = Nv // 2 if epi == "swiglu" else Nv
        r0 = torch.randn(M, N, device="cuda") if epi == "resid32" else None
        out = None if epi == "resid32" else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        cfg5, s5 = G.plan_mfma(M, Nv, K, epi)
        plans = {"mfma": (cfg5, s5), "pp": (20, 1), "pp2": (20, 2), "rs": (21, 1), "rs2": (21, 2), "w4": (22, 1), "w42": (22, 2), "w3": (23, 1), "w32": (23, 2), "w1": (24, 1), "w12": (24, 2),
                 "b4": (25, 1), "b42": (25, 2), "b3": (26, 1), "b32": (26, 2), "b1": (27, 1), "b12": (27, 2),
                 "lib": (G.LIB, 1)}
        y = x.float() @ w.float().t()
        if epi == "swiglu":
            ref = torch.nn.functional.silu(y[:, :N]) * y[:, N:]
        elif epi == "resid32":
            ref = r0 + y
        else:
            ref = y
        scale = ref.abs().max().item()
        errs, fns = {}, {}
        for arm in arms:
            cfg, spl = plans[arm]
            rr = r0.clone() if r0 is not None else None
            o = G.linear(x, w, epi=epi, resid=rr, out=None if out is None else out.clone(),
                         cfg=cfg, splits=spl)
            errs[arm] = (o.float() - ref).abs().max().item() / scale
            rr2 = r0.clone() if r0 is not None else None

            def f(cfg=cfg, spl=spl, rr2=rr2):
                G.linear(x, w, epi=epi, resid=rr2, out=out, cfg=cfg, splits=spl)
            f()
            fns[arm] = f
        torch.cuda.synchronize()
        best = {arm: 1e9 for arm in arms}
        for _ in range(a.rounds):
            for arm in arms:
                best[arm] = min(best[arm], timeit(fns[arm]))
        fl = 2.0 * M * Nv * K
        rec = {"shape": name, "M": M, "Nv": Nv, "K": K, "epi": epi, "mfma_plan": [cfg5, s5]}
        for arm in arms:
            rec[f"{arm}_ms"] = round(best[arm], 4)
            rec[f"{arm}_tflops"] = round(fl / best[arm] / 1e9, 1)
            rec[f"{arm}_err"] = float(f"{errs[arm]:.3g}")
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
