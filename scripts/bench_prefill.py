"""Prefill throughput (tokens/s) for one long prompt: MFMA flash attention + hipBLASLt GEMMs.

TTFT in the reference is the first next_token() call (prefill at position 0,
cake-core/src/models/llama3/llama.rs:285-298)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.models.llama3.factory import random_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--lens", default="128,512,2048,4096")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    m = random_model(a.model, "cuda:0", torch.bfloat16, max_seq=4096)
    out = []
    for T in map(int, a.lens.split(",")):
        toks = torch.randint(0, m.cfg.vocab_size, (T,)).tolist()
        m.reset()
        m.forward(toks, 0)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            m.reset()
            t0 = time.perf_counter()
            m.forward(toks, 0)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        out.append({"prompt_len": T, "ttft_ms": round(best * 1e3, 2),
                    "prefill_tokens_per_sec": round(T / best, 1)})
        print(json.dumps({"model": a.model, **out[-1]}), flush=True)


if __name__ == "__main__":
    main()
