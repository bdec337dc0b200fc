"""Decode attention launch latency at short context: graph of back-to-back launches (warm
K/V) vs the same launches separated by a 64 MiB streaming read (cold K/V, as in decode)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402


def timed(g, n):
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    return best


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    nh, nkv, hd, S = 32, 8, 128, 4096
    kc = torch.randn(nkv, S, hd, device=dev).to(dt)
    vc = torch.randn(nkv, S, hd, device=dev).to(dt)
    q = torch.randn(nh * hd, device=dev)
    part = torch.zeros(K.attn_workspace_numel(nh, hd, S), device=dev)
    tickets = torch.zeros(2 * nkv + 2, dtype=torch.int32, device=dev)
    out = torch.empty(nh * hd, device=dev, dtype=dt)
    pos = torch.zeros(1, dtype=torch.int32, device=dev)
    big = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    sink = torch.empty(1, device=dev)
    for Tk in (33, 64, 176, 1024, 2048):
        pos.fill_(Tk - 1)
        rec = {"Tk": Tk}
        for cap in (8, 64):
            with K.attn_split_cap(cap):
                n = 50
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(n):
                        K.attn_decode(q, kc, vc, pos, 1 / math.sqrt(hd), part, tickets, out)
                rec[f"warm_cap{cap}_us"] = round(timed(g, n), 2)
                g2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g2):
                    for _ in range(n):
                        big.view(torch.int32)[: 8 << 20].sum()
                g3 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g3):
                    for _ in range(n):
                        big.view(torch.int32)[: 8 << 20].sum()
                        K.attn_decode(q, kc, vc, pos, 1 / math.sqrt(hd), part, tickets, out)
                rec[f"cold_cap{cap}_us"] = round(timed(g3, n) - timed(g2, n), 2)
        print(json.dumps(rec), flush=True)
    del sink


if __name__ == "__main__":
    main()
