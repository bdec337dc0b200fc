"""Measured GEMM plans for the exact linears of one UNet step (SDXL 1024^2 / SD 1.5 512^2, CFG
batch 2): record every (M, weight rows, K, epilogue) that gemm.linear plans during one eager
UNet forward, time every tile configuration (and split-K where the grid is small) on that
shape, and merge the winners into cake_amd/ops/gemm_tuned.json.

    python scripts/tune_sd_gemm.py [--versions xl,v1-5] [--write OUT.json] > profiles/...jsonl

Timing: INNER launches captured in one hipGraph, median replay time / INNER (GPU time only: host
launch overhead would otherwise hide the differences between tiles on ~15 us kernels).
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import gemm as G  # noqa: E402

INNER, REPS = 10, 10
# A/B forms measured slower everywhere (the non-interleaved 8 / 11, ping-pong 20,
# register-staged 21: profiles/r6_gemm_*): not timed unless --cfgs names them
SKIP = {8, 11, 20, 21}
TUNED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cake_amd",
                     "ops", "gemm_tuned.json")


def record_shapes(version, dt):
    from cake_amd.models.sd.config import get_config
    from cake_amd.models.sd.unet import UNet2DConditionModel
    from cake_amd.models.sd.weights import random_component
    cfg = get_config(version)
    dev = torch.device("cuda:0")
    w = random_component("unet", cfg, dev, dt)
    unet = UNet2DConditionModel(cfg.unet)
    x = torch.randn(2, 4, cfg.height // 8, cfg.width // 8, device=dev, dtype=dt)
    ctx = torch.randn(2, 77, cfg.unet.cross_attention_dim, device=dev, dtype=dt)
    tbuf = torch.full((), 999.0, device=dev)
    kv = {}
    with torch.no_grad():
        unet.forward(w, x, tbuf, ctx, kv)  # first call: cross-attention k/v cache filled
        torch.cuda.synchronize()
        seen = collections.Counter()
        orig = G.plan

        def spy(M, Nv, K, epi="store"):
            seen[(M, Nv, K, epi)] += 1
            return orig(M, Nv, K, epi)
        G.plan = spy
        try:
            unet.forward(w, x, tbuf, ctx, kv)
        finally:
            G.plan = orig
        torch.cuda.synchronize()
    del w, unet
    torch.cuda.empty_cache()
    return seen


def timeit(fn):
    """GPU time per call: INNER calls captured in one hipGraph, median replay / INNER (no
    host launch cost in the number, as inside the UNet step's graph)."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(INNER):
            fn()
    g.replay()
    ts = []
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / INNER)
    del g
    ts.sort()
    return ts[len(ts) // 2]


def tune(M, Nv, K, epi, dt, cfgs=None):
    gated = epi in ("swiglu", "geglu")
    N = Nv // 2 if gated else Nv
    x = (torch.randn(M, K, device="cuda") * 0.5).to(dt)
    w = (torch.randn(Nv, K, device="cuda") * K ** -0.5).to(dt)
    b = (torch.randn(Nv, device="cuda") * 0.1).to(dt)
    r = None
    if epi in ("resid32", "store32"):
        r = torch.zeros(M, N, device="cuda")
    elif epi == "add16":
        r = torch.randn(M, N, device="cuda").to(dt)

    def run(cfg, splits):
        return G.linear(x, w, b, epi=epi, resid=r, cfg=cfg, splits=splits)
    cur = G.plan(M, Nv, K, epi)
    res = {}
    for cfg, (bm, bn) in G.CFG_TILES.items():
        if gated and cfg in getattr(G, "NO_GATED", ()):
            continue
        if cfgs is not None and cfg not in cfgs:
            continue
        if cfgs is None and (cfg in SKIP or (M >= 1024 and bm <= 64)):
            continue
        if cfg in getattr(G, "K64_ONLY", ()) and K % 64:
            continue
        tiles = -(-M // bm) * -(-Nv // bn)
        for splits in (1, 2, 4):
            # four-wave tiles at splits 2 pair only the tiles past the last whole wave (the
            # in-kernel pair, gemm.hip), whatever the tile count
            pair = cfg in getattr(G, "K64_ONLY", ()) and cfg >= 22 and splits == 2
            if splits > 1 and not pair and (tiles * splits > 2 * G.NUM_CUS or K // splits < 256):
                continue
            try:
                run(cfg, splits)
                res[(cfg, splits)] = timeit(lambda: run(cfg, splits))
            except Exception:  # noqa: BLE001  (a config the shape cannot take)
                continue
    if cur not in res and cur[0] != G.LIB:
        run(*cur)
        res[cur] = timeit(lambda: run(*cur))
    best = min(res, key=res.get)
    return cur, res.get(cur, float("nan")), best, res[best]


LLAMA_LENS = {"8b": (32, 128, 512, 1024, 2048, 4096), "70b": (512, 2048)}


def llama_shapes(lens=None):
    """Prefill linears of Llama-3-8B / 70B (q|k|v, o + residual, gate|up + SwiGLU, down +
    residual) at the prompt lengths the engine and the bench run (``lens``: model ->
    prompt lengths, default LLAMA_LENS)."""
    lens = lens or LLAMA_LENS
    out = collections.Counter()
    for (H, I, nq, nkv), Ts in (((4096, 14336, 32, 8), lens.get("8b", ())),
                                ((8192, 28672, 64, 8), lens.get("70b", ()))):
        hd = H // nq
        for T in Ts:
            out[(T, (nq + 2 * nkv) * hd, H, "store")] += 1
            out[(T, H, H, "resid32")] += 1
            out[(T, 2 * I, H, "swiglu")] += 1
            out[(T, H, I, "resid32")] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--versions", default="xl,v1-5",
                    help="comma list of SD versions, and/or 'llama' for the prefill shapes")
    ap.add_argument("--llama-lens", default=None,
                    help="prompt lengths of the llama shapes, e.g. '8b:256,384;70b:1024'")
    ap.add_argument("--lib-shapes", action="store_true",
                    help="re-tune (MFMA only) every table entry that names the library GEMM")
    ap.add_argument("--cfgs", default=None, help="comma list of tile configs to time")
    ap.add_argument("--write", default=None,
                    help="write gemm_tuned.json with the winners merged in to this path")
    a = ap.parse_args()
    dt = torch.float16
    new = []
    cfgs = None if a.cfgs is None else {int(c) for c in a.cfgs.split(",")}
    if a.lib_shapes:  # the library GEMM's measured shapes (CAKE_GEMM_LIB A/B arm)
        with open(TUNED) as f:
            lib = [e for e in json.load(f)["entries"] if e["cfg"] == G.LIB]
        a.versions = ""
        for e in lib:
            M, Nv, K, epi = e["M"], e["Nv"], e["K"], e["epi"]
            cur, t_cur, best, t_best = tune(M, Nv, K, epi, torch.bfloat16, cfgs)
            fl = 2.0 * M * Nv * K
            rec = {"version": "llama_lib", "M": M, "Nv": Nv, "K": K, "epi": epi,
                   "lib_tflops": e.get("tflops"), "best": list(best),
                   "best_ms": round(t_best, 4), "best_tflops": round(fl / t_best / 1e9, 1)}
            print(json.dumps(rec), flush=True)
            new.append({"M": M, "Nv": Nv, "K": K, "epi": epi, "cfg": best[0], "splits": best[1],
                        "tflops": rec["best_tflops"], "shape": e.get("shape", "llama_prefill"),
                        "lib_tflops": e.get("tflops")})
    for version in [v for v in a.versions.split(",") if v]:
        dt = torch.bfloat16 if version == "llama" else torch.float16
        lens = None
        if a.llama_lens:
            lens = {k: tuple(int(x) for x in v.split(",")) for k, v in
                    (part.split(":") for part in a.llama_lens.split(";"))}
        shapes = llama_shapes(lens) if version == "llama" else record_shapes(version, dt)
        tot_cur = tot_best = 0.0
        for (M, Nv, K, epi), n in sorted(shapes.items(), key=lambda kv: -kv[1] * kv[0][0] * kv[0][1] * kv[0][2]):
            cur, t_cur, best, t_best = tune(M, Nv, K, epi, dt)
            fl = 2.0 * M * Nv * K
            tot_cur += n * t_cur
            tot_best += n * t_best
            rec = {"version": version, "M": M, "Nv": Nv, "K": K, "epi": epi, "calls": n,
                   "plan": list(cur), "plan_ms": round(t_cur, 4), "best": list(best),
                   "best_ms": round(t_best, 4), "best_tflops": round(fl / t_best / 1e9, 1)}
            print(json.dumps(rec), flush=True)
            new.append({"M": M, "Nv": Nv, "K": K, "epi": epi, "cfg": best[0], "splits": best[1],
                        "tflops": rec["best_tflops"],
                        "shape": "llama_prefill" if version == "llama" else f"sd_{version}_unet"})
        print(json.dumps({"version": version, "step_gemm_ms_plan": round(tot_cur, 3),
                          "step_gemm_ms_best": round(tot_best, 3)}), flush=True)
    if a.write:
        with open(TUNED) as f:
            table = json.load(f)
        uniq = {}
        for e in new:  # a shape shared by two versions (time embedding) keeps one plan
            uniq.setdefault((e["M"], e["Nv"], e["K"], e["epi"]), e)
        new = list(uniq.values())
        keys = set(uniq)
        old = [e for e in table["entries"] if (e["M"], e["Nv"], e["K"], e["epi"]) not in keys]
        if a.lib_shapes:  # the library arm stays, as its own entries (read under CAKE_GEMM_LIB=1)
            old += [dict(e, shape="lib_ab") for e in table["entries"]
                    if e["cfg"] == G.LIB and (e["M"], e["Nv"], e["K"], e["epi"]) in keys]
        table["entries"] = old + new
        table["sd_source"] = "scripts/tune_sd_gemm.py"
        with open(a.write, "w") as f:
            json.dump(table, f, indent=1)
        print(f"# {len(new)} SD entries merged into {a.write}", file=sys.stderr)


if __name__ == "__main__":
    main()
