"""Speed-of-light reference for 8B batch-1 decode on one MI355X.

Replays, in one hipGraph, kernels that ONLY stream the decode's weight bytes
(elementwise.hip stream_read_kernel: 16-byte non-temporal loads, 8 per lane in
flight, no math) with the decode graph's kernel structure — per layer QKV (48 MiB),
attention (KV bytes at a 64-token context), o_proj (32 MiB), gate|up (224 MiB),
down (112 MiB), then lm_head (1002 MiB) — from distinct buffers so nothing is
served from the Infinity Cache.  Compares against the same bytes read by one
kernel.  The ratio (decode tok/s) / (ceiling tok/s) is the fraction of the
achievable bound the real kernels reach.

    python scripts/decode_ceiling.py [--blocks 512,1024,2048] > out.jsonl
"""
from __future__ import annotations

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cake_amd.ops import hip as K  # noqa: E402

H, I, NH, NKV, HD, V, L = 4096, 14336, 32, 8, 128, 128256, 32
SIZES = {"qkv": (NH + 2 * NKV) * HD * H * 2, "attn": NKV * 64 * HD * 2 * 2,
         "o_proj": H * H * 2, "gate_up": 2 * I * H * 2, "down": H * I * 2}
HEAD = V * H * 2


def timed(fn, reps=10):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", default="512,1024,2048,4096")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    per_layer = sum(SIZES.values())
    total = L * per_layer + HEAD
    # one arena, sliced per layer/kernel (distinct bytes everywhere)
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    bufs, off = [], 0
    for li in range(L):
        row = {}
        for k, n in SIZES.items():
            row[k] = arena[off:off + n]
            off += n
        bufs.append(row)
    head = arena[off:off + HEAD]
    for blocks in [int(b) for b in a.blocks.split(",")]:
        ms_one = timed(lambda: K.stream_read(arena, blocks * 4, sink))

        def layered(kinds):
            def fn():
                for row in bufs:
                    for k in kinds:
                        K.stream_read(row[k], blocks if k != "attn" else 64, sink)
                K.stream_read(head, blocks, sink)
            return fn
        ms5 = timed(layered(list(SIZES)))
        ms4 = timed(layered([k for k in SIZES if k != "attn"]))
        rec = {"blocks": blocks, "bytes_per_token": total,
               "one_kernel_ms": round(ms_one, 4),
               "one_kernel_TBps": round(total / ms_one / 1e9, 3),
               "graph_5k_per_layer_ms": round(ms5, 4),
               "graph_5k_TBps": round(total / ms5 / 1e9, 3),
               "graph_5k_tok_s": round(1e3 / ms5, 1),
               "graph_4k_per_layer_ms": round(ms4, 4),
               "graph_4k_tok_s": round(1e3 / ms4, 1)}
        # per-kind isolated: L back-to-back launches of one kind (kernel + boundary cost)
        for k, n in SIZES.items():
            ms = timed(lambda k=k: [K.stream_read(row[k], blocks if k != "attn" else 64, sink)
                                    for row in bufs])
            rec[f"{k}_us"] = round(ms * 1e3 / L, 2)
            rec[f"{k}_TBps"] = round(n * L / ms / 1e9, 3)
        ms = timed(lambda: K.stream_read(head, blocks, sink))
        rec["lm_head_us"] = round(ms * 1e3, 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
