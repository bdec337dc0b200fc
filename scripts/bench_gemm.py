"""MFMA GEMM (gemm.hip) vs torch.matmul (hipBLASLt) on the model shapes: TFLOP/s per shape.

Usage: python scripts/bench_gemm.py [--sweep] > profiles/...jsonl
--sweep also times every (cfg, splits) candidate and reports the best (tuning input).
Timing: interleaved rounds in one process, median of device-event times, random data.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import gemm as G  # noqa: E402

SHAPES = [  # name, M, N (output features), K, epi
    ("8b_qkv_t2048", 2048, 6144, 4096, "store"), ("8b_o_t2048", 2048, 4096, 4096, "resid32"),
    ("8b_gateup_t2048", 2048, 14336, 4096, "swiglu"), ("8b_down_t2048", 2048, 4096, 14336, "resid32"),
    ("8b_qkv_t512", 512, 6144, 4096, "store"), ("8b_gateup_t512", 512, 14336, 4096, "swiglu"),
    ("8b_down_t512", 512, 4096, 14336, "resid32"),
    ("8b_qkv_t128", 128, 6144, 4096, "store"), ("8b_down_t32", 32, 4096, 14336, "resid32"),
    ("70b_qkv_t2048", 2048, 10240, 8192, "store"), ("70b_gateup_t2048", 2048, 28672, 8192, "swiglu"),
    ("sdxl_qkv_4096tok", 8192, 1920, 640, "store"), ("sdxl_ff_in_4096tok", 8192, 2560, 640, "geglu"),
    ("sdxl_ff_out_4096tok", 8192, 640, 2560, "add16"), ("sdxl_qkv_1024tok", 2048, 3840, 1280, "store"),
    ("sdxl_ff_in_1024tok", 2048, 5120, 1280, "geglu"), ("sd15_qkv_4096tok", 8192, 960, 320, "store"),
    ("sdxl_attn_out_1024tok", 2048, 1280, 1280, "add16"), ("sdxl_ff_out_1024tok", 2048, 1280, 5120, "add16"),
    ("sdxl_attn_out_4096tok", 8192, 640, 640, "add16"), ("sdxl_q_1024tok", 2048, 1280, 1280, "store"),
    ("sd15_ff_in_4096tok", 8192, 1280, 320, "geglu"), ("sd15_ff_out_4096tok", 8192, 320, 1280, "add16"),
    ("square_4096", 4096, 4096, 4096, "store"), ("square_8192", 8192, 8192, 8192, "store"),
]


INNER = 1


def timeit(fn, reps=20):
    """Median over reps of (event time of INNER back-to-back calls) / INNER: INNER > 1
    amortises the event / launch overhead that dominates a single ~20 us kernel."""
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(INNER):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / INNER)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--only", default=None)
    ap.add_argument("--cfgs", default=None, help="comma list: time each cfg (splits 1)")
    ap.add_argument("--inner", type=int, default=1, help="back-to-back calls per timing")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    a = ap.parse_args()
    global INNER
    INNER = max(1, a.inner)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    for name, M, N, K, epi in SHAPES:
        if a.only and a.only not in name:
            continue
        gated = epi in ("swiglu", "geglu")
        Nw = 2 * N if gated else N
        x = (torch.randn(M, K, device="cuda") * 0.5).to(dt)
        w = (torch.randn(Nw, K, device="cuda") * K ** -0.5).to(dt)
        r32 = torch.randn(M, N, device="cuda") if epi == "resid32" else None
        r16 = torch.randn(M, N, device="cuda").to(dt) if epi == "add16" else None
        flops = 2.0 * M * Nw * K

        def ours(cfg=None, splits=None):
            return G.linear(x, w, epi=epi, resid=r32 if r32 is not None else r16, cfg=cfg,
                            splits=splits)

        def lib():  # the same math through torch (hipBLASLt GEMM + elementwise epilogue)
            y = torch.matmul(x, w.t())
            if epi == "resid32":
                r32.add_(y)
            elif epi == "add16":
                y.add_(r16)
            elif gated:
                y = torch.nn.functional.silu(y[:, :N]) * y[:, N:]
            return y

        def libmm():  # the bare library GEMM
            return torch.matmul(x, w.t())
        for f in (ours, lib, libmm):
            f()
        torch.cuda.synchronize()
        t_ours = t_lib = t_mm = None
        for _ in range(3):  # interleaved rounds
            to, tl, tm = timeit(ours), timeit(lib), timeit(libmm)
            t_ours = to if t_ours is None else min(t_ours, to)
            t_lib = tl if t_lib is None else min(t_lib, tl)
            t_mm = tm if t_mm is None else min(t_mm, tm)
        rec = {"shape": name, "M": M, "N": N, "K": K, "epi": epi, "plan": G.plan(M, Nw, K, epi),
               "ours_ms": round(t_ours, 4), "torch_fused_ms": round(t_lib, 4),
               "hipblaslt_gemm_ms": round(t_mm, 4),
               "ours_tflops": round(flops / t_ours / 1e9, 1),
               "hipblaslt_tflops": round(flops / t_mm / 1e9, 1)}
        if a.sweep:
            best = None
            for cfg in G.CFG_TILES:
                for splits in (1, 2, 4, 8):
                    try:
                        t = timeit(lambda: ours(cfg, splits), reps=10)
                    except Exception:  # noqa: BLE001
                        continue
                    if best is None or t < best[0]:
                        best = (t, cfg, splits)
            rec["best"] = {"cfg": best[1], "splits": best[2], "ms": round(best[0], 4),
                           "tflops": round(flops / best[0] / 1e9, 1)}
        if a.cfgs:
            per = {}
            for _ in range(3):
                for cfg in [int(c) for c in a.cfgs.split(",")]:
                    if gated and cfg in G.NO_GATED:
                        continue
                    t = timeit(lambda: ours(cfg, 1), reps=10)
                    per[cfg] = min(per.get(cfg, 1e9), t)
            rec["per_cfg_tflops"] = {c: round(flops / t / 1e9, 1) for c, t in per.items()}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
