"""MFMA GEMM (its tuned plan) vs the library GEMM path (ops/gemm.py LIB: hipBLASLt) on
the Llama prefill projections across prompt lengths, with the error of each against a
float32 reference.  Output: one JSON line per (shape, M), input of
scripts/gemm_lib_table.py.

Usage: python scripts/bench_gemm_lib.py [--models 8b,70b] [--ms 128,256,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import gemm as G  # noqa: E402

MODELS = {  # name -> (H, I, nq, nkv*hd)
    "8b": (4096, 14336, 4096, 1024),
    "70b": (8192, 28672, 8192, 1024),
}


def shapes(model, tp=1):
    """The prefill projections of one rank: all layers (tp 1: o / down accumulate into the
    residual) or a tensor-parallel rank's slices (o / down write f32 partials, store32)."""
    H, I, nq, nk = MODELS[model]
    if tp == 1:
        return [("qkv", nq + 2 * nk, H, "store"), ("o", H, nq, "resid32"),
                ("gate_up", 2 * I, H, "swiglu"), ("down", H, I, "resid32")]
    return [(f"tp{tp}_qkv", (nq + 2 * nk) // tp, H, "store"), (f"tp{tp}_o", H, nq // tp, "store32"),
            (f"tp{tp}_gate_up", 2 * I // tp, H, "swiglu"), (f"tp{tp}_down", H, I // tp, "store32")]


def timeit(fn, reps=15):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="8b,70b")
    ap.add_argument("--ms", default="128,256,384,512,768,1024,1536,2048,3072,4096")
    ap.add_argument("--tp", default="1", help="comma list of tensor-parallel degrees")
    ap.add_argument("--sweep-splits", action="store_true",
                    help="time the MFMA plan's tile at split-K 1/2/4/8 and keep the best")
    a = ap.parse_args()
    torch.manual_seed(0)
    for model, tp in [(m, int(t)) for m in a.models.split(",") for t in a.tp.split(",")]:
        for name, Nv, K, epi in shapes(model, tp):
            w = (torch.randn(Nv, K, device="cuda") * K ** -0.5).bfloat16()
            N = Nv // 2 if epi == "swiglu" else Nv
            for M in [int(m) for m in a.ms.split(",")]:
                x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
                r0 = torch.randn(M, N, device="cuda") if epi in ("resid32", "store32") else None
                cfg, spl = G.plan_mfma(M, Nv, K, epi)
                outs = {}

                def run(kind):
                    r = r0.clone() if r0 is not None else None
                    c = None if kind == "ours" else G.LIB
                    s = None if kind == "ours" else 1
                    return G.linear(x, w, epi=epi, resid=r, cfg=cfg if c is None else c,
                                    splits=spl if s is None else s)
                for kind in ("ours", "lib"):
                    outs[kind] = run(kind).float()
                y = x.float() @ w.float().t()
                if epi == "swiglu":
                    ref = torch.nn.functional.silu(y[:, :N]) * y[:, N:]
                elif epi == "resid32":
                    ref = r0 + y
                elif epi == "store32":
                    ref = y
                else:
                    ref = y
                scale = ref.abs().max().item()
                err = {k: (v - ref).abs().max().item() / scale for k, v in outs.items()}
                # timed forms write in place (resid32 accumulates: harmless for timing)
                rr = r0.clone() if r0 is not None else None
                out = None if epi in ("resid32", "store32") else torch.empty(
                    M, N, device="cuda", dtype=torch.bfloat16)

                def ours():
                    G.linear(x, w, epi=epi, resid=rr, out=out, cfg=cfg, splits=spl)

                def lib():
                    G.linear(x, w, epi=epi, resid=rr, out=out, cfg=G.LIB, splits=1)
                if a.sweep_splits:
                    best = None
                    for sp in (1, 2, 4, 8):
                        if sp > 1 and K // sp < 256:
                            continue
                        def f(sp=sp):
                            G.linear(x, w, epi=epi, resid=rr, out=out, cfg=cfg, splits=sp)
                        f()
                        t = min(timeit(f, 10) for _ in range(2))
                        if best is None or t < best[0]:
                            best = (t, sp)
                    spl = best[1]
                ours(), lib()
                torch.cuda.synchronize()
                to = tl = 1e9
                for _ in range(3):
                    to, tl = min(to, timeit(ours)), min(tl, timeit(lib))
                fl = 2.0 * M * Nv * K
                print(json.dumps({"model": model, "proj": name, "M": M, "Nv": Nv, "K": K,
                                  "epi": epi, "ours_cfg": cfg, "ours_splits": spl,
                                  "ours_ms": round(to, 4), "lib_ms": round(tl, 4),
                                  "ours_tflops": round(fl / to / 1e9, 1),
                                  "lib_tflops": round(fl / tl / 1e9, 1),
                                  "ours_rel_err": float(f"{err['ours']:.3g}"),
                                  "lib_rel_err": float(f"{err['lib']:.3g}")}), flush=True)


if __name__ == "__main__":
    main()
