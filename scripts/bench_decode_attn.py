"""Decode attention (attention.hip) alone: µs per launch and effective KV TB/s vs live
context, per min-keys-per-split setting (graph of back-to-back launches, Llama-3 8B heads)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    nh, nkv, hd = 32, 8, 128
    for S in (4096, 8192):
        kc = torch.randn(nkv, S, hd, device=dev).to(dt)
        vc = torch.randn(nkv, S, hd, device=dev).to(dt)
        q = torch.randn(nh * hd, device=dev)
        part = torch.zeros(K.attn_workspace_numel(nh, hd, S), device=dev)
        tickets = torch.zeros(2 * nkv + 2, dtype=torch.int32, device=dev)
        out = torch.empty(nh * hd, device=dev, dtype=dt)
        pos = torch.zeros(1, dtype=torch.int32, device=dev)
        for Tk in (55, 176, 512, 1024, 2048, 4096, 8192):
            if Tk > S or (S == 8192 and Tk < 4096):
                continue
            pos.fill_(Tk - 1)
            rec = {"S": S, "Tk": Tk}
            for mk in (64, 128, 256, 512):
                K.attn_set_min_keys(mk)
                K.attn_decode(q, kc, vc, pos, 1 / math.sqrt(hd), part, tickets, out)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(50):
                        K.attn_decode(q, kc, vc, pos, 1 / math.sqrt(hd), part, tickets, out)
                g.replay()
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(5):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    g.replay()
                    b.record()
                    b.synchronize()
                    best = min(best, a.elapsed_time(b) * 1e3 / 50)
                rec[f"mk{mk}_us"] = round(best, 2)
                rec[f"mk{mk}_TBps"] = round(2 * nkv * Tk * hd * 2 / best / 1e6, 3)
            print(json.dumps(rec), flush=True)
        K.attn_set_min_keys(64)


if __name__ == "__main__":
    main()
