"""Per-phase timeline of one decode-megakernel launch (Llama-3 random init).

Every workgroup's control wave records s_memrealtime (100 MHz) per phase:
t0 = arrival (results stored), t1 = grid barrier passed, t2 = x staged,
t3 = compute waves done; attention units add t4 (gathered + roped),
t5 (scores), t6 (P.V), t7 (partials stored + ticket).
Prints, per phase kind, the mean segment durations in microseconds, the
arrival spread (max - min t0 over workgroups: imbalance) and the barrier
latency (min t1 - max t0).
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from cake_amd.models.llama3.factory import random_model  # noqa: E402
from cake_amd.models.llama3.model import DeviceDecoder  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--prompt-len", type=int, default=160)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import os
    os.environ["CAKE_MEGA"] = "1"
    model = random_model(a.model, "cuda:0", torch.bfloat16, max_seq=4096)
    dec = DeviceDecoder(model, repeat_penalty=1.1, greedy=True, use_graph=False)
    L = model.cfg.num_hidden_layers
    G = dec.mega.grid
    NP = 5 * L + 1
    dec.mega.trace = torch.zeros(NP * G * 8, dtype=torch.int64, device="cuda:0")
    dec.start(list(range(1, a.prompt_len + 1)))
    for _ in range(3):
        dec.launch()
    torch.cuda.synchronize()
    t = dec.mega.trace.view(NP, G, 8).cpu().double() / 100.0  # us
    names = ["qkv", "att", "o", "swi", "down"]
    agg = {}
    for p in range(NP):
        k = names[p % 5] if p < 5 * L else "head"
        d = agg.setdefault(k, dict(n=0, wait=0.0, stage=0.0, compute=0.0, spread=0.0, lat=0.0,
                                   total=0.0))
        d["n"] += 1
        tp = t[p]
        d["wait"] += float((tp[:, 1] - tp[:, 0]).mean())
        d["stage"] += float((tp[:, 2] - tp[:, 1]).mean())
        d["compute"] += float((tp[:, 3] - tp[:, 2]).mean())
        if p > 0:
            d["spread"] += float(tp[:, 0].max() - tp[:, 0].min())
            d["lat"] += float(tp[:, 1].min() - tp[:, 0].max())
        end = t[p + 1, :, 0].max() if p + 1 < NP else tp[:, 3].max()
        d["total"] += float(end - tp[:, 0].max()) if p > 0 else float(end - tp[:, 0].min())
        if k == "att":
            act = tp[:, 4] > 0
            if act.any():
                ta = tp[act]
                for key, i, j in (("a_gather", 2, 4), ("a_scores", 4, 5), ("a_pv", 5, 6),
                                  ("a_store_ticket", 6, 7)):
                    d[key] = d.get(key, 0.0) + float((ta[:, j] - ta[:, i]).clamp(min=0).mean())
                d["a_units"] = int(act.sum())
    rows = {k: {kk: (vv / v["n"] if isinstance(vv, float) else vv) for kk, vv in v.items()}
            for k, v in agg.items()}
    out = {"launch_us": float(t[-1, :, 3].max() - t[0, :, 0].min()), "grid": G, "phases": rows,
           "skew": skew_report(dec.mega.trace, L, G)}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f)



def skew_report(trace, L, G):
    """Per-workgroup compute time of the big phases: is the skew systematic?"""
    import numpy as np
    t = trace.view(5 * L + 1, G, 8).cpu().double().numpy() / 100.0
    out = {}
    for name, k in (("swi", 3), ("down", 4), ("qkv", 0)):
        d = np.stack([t[l * 5 + k, :, 3] - t[l * 5 + k, :, 2] for l in range(L)])  # [L, G]
        m = d.mean(0)
        # correlation of per-WG time between even and odd layers (1 = systematic)
        c = float(np.corrcoef(d[0::2].mean(0), d[1::2].mean(0))[0, 1])
        xcd = [float(m[x::8].mean()) for x in range(8)]
        out[name] = {"mean": float(m.mean()), "min": float(m.min()), "max": float(m.max()),
                     "even_odd_corr": c, "per_xcd_mean": [round(v, 2) for v in xcd],
                     "slowest_wg": [int(i) for i in np.argsort(-m)[:8]]}
    return out


if __name__ == "__main__":
    main()
