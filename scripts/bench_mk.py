"""Layer-stack decode step: persistent launch (decode_mk.hip) vs five launches per layer.

Captures one hipGraph per path over every layer of a random-init model and times
back-to-back replays (device events).  Prints one JSON line per path.

    python scripts/bench_mk.py --model llama3-8b --pos 32 --reps 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cake_amd.models.llama3.config import preset  # noqa: E402
from cake_amd.models.llama3.factory import random_stack  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--pos", type=int, nargs="+", default=[32])
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--max-seq", type=int, default=4096)
    ap.add_argument("--thin", type=int, default=1)
    ap.add_argument("--ring", type=int, default=0)
    ap.add_argument("--fly", type=int, default=1)
    ap.add_argument("--o-all", type=int, default=1)
    a = ap.parse_args()
    from cake_amd.ops._lib import kernels as _k
    _k().cake_mk_set_tuning(a.thin, a.ring, a.fly, a.o_all)
    over = {"num_hidden_layers": a.layers} if a.layers else {}
    cfg = preset(a.model, **over)
    layers = list(range(cfg.num_hidden_layers))
    st = random_stack(cfg, layers, "cuda:0", torch.bfloat16, max_seq=a.max_seq)
    bufs = st.decode_buffers()
    kv = st.cache(0)
    kv.k.normal_(0, 1)
    kv.v.normal_(0, 1)
    resid0 = torch.randn(cfg.hidden_size, device="cuda:0")
    nbytes = len(layers) * cfg.layer_bytes()
    outs = {}
    for path in ("launches", "mk"):
        st.use_mk = path == "mk"
        bufs.resid.copy_(resid0)
        bufs.pos.fill_(a.pos[0])
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            st.decode_step(bufs, layers)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            st.decode_step(bufs, layers)
        for pos in a.pos:
            bufs.pos.fill_(pos)
            bufs.resid.copy_(resid0)
            g.replay()
            torch.cuda.synchronize()
            outs[(path, pos)] = bufs.resid.clone()
            for _ in range(3):
                g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            rec = {"path": path, "model": a.model, "layers": len(layers), "pos": pos,
                   "thin": a.thin, "ring": a.ring, "fly": a.fly, "o_all": a.o_all,
                   "us_per_step": round(us, 2), "us_per_layer": round(us / len(layers), 3),
                   "TBps": round(nbytes / us / 1e6, 3)}
            if path == "mk":
                st.mk_check(bufs)
                ref = outs[("launches", pos)]
                rec["rel_err_vs_launches"] = float((outs[(path, pos)] - ref).norm() / ref.norm())
            print(json.dumps(rec), flush=True)
        del g


if __name__ == "__main__":
    main()
