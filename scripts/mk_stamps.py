"""Phase timeline of one persistent decode step (decode_mk.hip stamps).

Every workgroup records s_memrealtime (100 MHz, one clock for all CUs) at ten
points per layer: QKV x ready / walk done / published, O x ready / walk done,
SwiGLU x ready / walk done, down x ready / walk done / published.  Prints, per
op, the median over workgroups and over the middle layers of: the walk time, the
wait for the input vector after the op's inputs were complete, and the per-layer
total — the numbers a persistent design lives or dies by.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cake_amd.models.llama3.config import preset  # noqa: E402
from cake_amd.models.llama3.factory import random_stack  # noqa: E402
from cake_amd.ops._lib import kernels  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--pos", type=int, default=32)
    ap.add_argument("--out", default="")
    ap.add_argument("--thin", type=int, default=1)
    ap.add_argument("--ring", type=int, default=0)
    ap.add_argument("--fly", type=int, default=1)
    ap.add_argument("--o-all", type=int, default=1)
    a = ap.parse_args()
    from cake_amd.ops._lib import kernels as _k
    _k().cake_mk_set_tuning(a.thin, a.ring, a.fly, a.o_all)
    cfg = preset(a.model, **({"num_hidden_layers": a.layers} if a.layers else {}))
    L = cfg.num_hidden_layers
    st = random_stack(cfg, list(range(L)), "cuda:0", torch.bfloat16, max_seq=4096)
    st.use_mk = True
    bufs = st.decode_buffers()
    bufs.pos.fill_(a.pos)
    G = int(kernels().cake_mk_grid())
    S = 14  # decode_mk.hip kStampsPerLayer
    stamps = torch.zeros(G * (L * S + 2), dtype=torch.int64, device="cuda:0")
    for _ in range(3):
        st.decode_step(bufs, list(range(L)))
    torch.cuda.synchronize()
    kernels().cake_mk_set_stamps(stamps.data_ptr())
    st.decode_step(bufs, list(range(L)))
    torch.cuda.synchronize()
    kernels().cake_mk_set_stamps(None)
    st.mk_check(bufs)
    t = stamps.view(G, L * S + 2).cpu().numpy().astype(np.float64)
    t0 = t[:, L * S].min()
    rel = (t - t0) * 0.01  # us
    rel[t == 0] = np.nan
    ph = rel[:, :L * S].reshape(G, L, S)
    mid = slice(1, L - 1) if L > 2 else slice(0, L)

    def med(x):
        return float(np.nanmedian(x))

    rows = {}
    # walk times (per WG)
    rows["qkv_walk"] = med(ph[:, mid, 1] - ph[:, mid, 0])
    rows["o_walk"] = med(ph[:, mid, 4] - ph[:, mid, 3])
    rows["swiglu_walk"] = med(ph[:, mid, 6] - ph[:, mid, 5])
    rows["down_walk"] = med(ph[:, mid, 8] - ph[:, mid, 7])
    # edges: consumer x-ready minus the LAST producer's publish/walk-done of that layer
    last_qkv_pub = np.nanmax(ph[:, :, 2], axis=0)
    last_o_done = np.nanmax(ph[:, :, 4], axis=0)
    last_swi_done = np.nanmax(ph[:, :, 6], axis=0)
    last_down_pub = np.nanmax(ph[:, :, 9], axis=0)
    rows["attn_chain(qkv_pub_last->o_xready_med)"] = med(ph[:, mid, 3] - last_qkv_pub[None, mid])
    rows["edge_mid(o_done_last->swi_xready_med)"] = med(ph[:, mid, 5] - last_o_done[None, mid])
    rows["edge_act(swi_done_last->down_xready_med)"] = med(ph[:, mid, 7] - last_swi_done[None, mid])
    nxt = ph[:, 1:, 0] - last_down_pub[None, :-1]
    rows["edge_res(down_pub_last->qkv_xready_med)"] = med(nxt)
    # skew: last minus median walk-done per op
    rows["skew_qkv_done"] = med(np.nanmax(ph[:, mid, 1], 0) - np.nanmedian(ph[:, mid, 1], 0))
    rows["skew_swi_done"] = med(np.nanmax(ph[:, mid, 6], 0) - np.nanmedian(ph[:, mid, 6], 0))
    rows["skew_down_done"] = med(np.nanmax(ph[:, mid, 8], 0) - np.nanmedian(ph[:, mid, 8], 0))
    lay = np.nanmedian(ph[:, 1:, 0], 0) - np.nanmedian(ph[:, :-1, 0], 0)
    rows["layer_us_median"] = float(np.median(lay))
    # loader 0: o_proj first / last slot issued, gate/up and down first slot issued,
    # relative to this layer's QKV x-ready of the same workgroup
    x0 = ph[:, mid, 0]
    for k, name in ((10, "ld_o_first"), (11, "ld_o_last"), (12, "ld_swi_first"), (13, "ld_down_first")):
        rows[name] = med(ph[:, mid, k] - x0)
    for k, name in ((1, "qkv_done"), (2, "qkv_pub"), (3, "o_xready"), (4, "o_done"), (5, "swi_xready"),
                    (6, "swi_done"), (7, "down_xready"), (8, "down_done")):
        rows["t_" + name] = med(ph[:, mid, k] - x0)
    rows["step_us"] = float(np.nanmax(rel[:, L * S + 1]))
    out = {"model": a.model, "layers": L, "pos": a.pos, "grid": G, "thin": a.thin, "ring": a.ring, "fly": a.fly, "o_all": a.o_all,
           **{k: round(v, 3) for k, v in rows.items()}}
    print(json.dumps(out))
    if a.out:
        np.save(a.out, rel)


if __name__ == "__main__":
    main()
