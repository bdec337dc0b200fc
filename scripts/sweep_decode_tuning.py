"""In-graph decode tok/s (8B, batch 1) under different decode-GEMV launch tunings, interleaved
rounds in one process (a tuning is captured into a fresh graph each time)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.models.llama3.decode_loop import run_decode  # noqa: E402
from cake_amd.models.llama3.factory import random_model  # noqa: E402
from cake_amd.models.llama3.model import DeviceDecoder  # noqa: E402
from cake_amd.ops import hip as K  # noqa: E402

VARIANTS = {
    "default": {},
    "qkv_pf4": {"qkv": (8, 4, 1024)},
    "qkv_pf8": {"qkv": (8, 8, 1024)},
    "qkv_u4pf8": {"qkv": (4, 8, 1024)},
    "swiglu_pf4": {"swiglu": (2, 4, 512)},
    "x16_pf4": {"x16": (4, 4, 1024)},
    "all_pf4": {"qkv": (8, 4, 1024), "swiglu": (2, 4, 512), "x16": (4, 4, 1024)},
}
DEFAULTS = {"qkv": (8, 0, 1024), "swiglu": (2, 0, 512), "x16": (4, 0, 1024)}


def main():
    m = random_model("llama3-8b", "cuda:0", torch.bfloat16, max_seq=1024)
    prompt = list(range(100, 132))
    res = {k: [] for k in VARIANTS}
    for rnd in range(3):
        for name, tune in VARIANTS.items():
            for kind, (u, pf, mb) in {**DEFAULTS, **tune}.items():
                K.set_gemv_tuning(kind, U=u, prefetch=pf, max_blocks=mb)
            dec = DeviceDecoder(m, repeat_penalty=1.1, repeat_last_n=128)
            dec.start(prompt)
            dec.capture()
            run_decode(dec, 8)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run_decode(dec, 96)
            torch.cuda.synchronize()
            res[name].append(96 / (time.perf_counter() - t0))
            del dec
    for name, v in res.items():
        print(json.dumps({"variant": name, "tok_s": [round(x, 1) for x in v],
                          "best": round(max(v), 1)}), flush=True)


if __name__ == "__main__":
    main()
