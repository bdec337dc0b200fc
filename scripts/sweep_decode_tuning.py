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

# kind -> (U, prefetch, max_blocks); prefetch > 0 also selects the split x prologue
# (gemv.hip NormPre / Plain16Pre) for the model's K
DEFAULTS = {"qkv": (2, 4, 1024), "swiglu": (2, 4, 512), "x16": (4, 4, 1024),
            "norm_f32": (4, 4, 256), "x16s": (4, 4, 1024)}
BEST = {"qkv": (2, 4, 1024), "swiglu": (2, 4, 512), "x16": (4, 4, 1024)}
VARIANTS = {
    "default": {},
    # o_proj (x16s, K <= 8192) on its own
    "o_u2pf4": {"x16s": (2, 4, 1024)},
    "o_u2pf8": {"x16s": (2, 8, 1024)},
    "o_u4pf8": {"x16s": (4, 8, 1024)},
    "o_u8pf8": {"x16s": (8, 8, 1024)},
    "o_u4pf4_256": {"x16s": (4, 4, 256)},
    "o_u2pf8_256": {"x16s": (2, 8, 256)},
    "o_u4pf4_384": {"x16s": (4, 4, 384)},
    "best": BEST,
    "best_head_pf4": {**BEST, "norm_f32": (4, 4, 256)},
    "best_q2pf8": {**BEST, "qkv": (2, 8, 1024)},
    "best_q8pf8": {**BEST, "qkv": (8, 8, 1024)},
    "best_q4pf8_768": {**BEST, "qkv": (4, 8, 768)},
    "best_sw256": {**BEST, "swiglu": (2, 4, 256)},
    "best_sw1024": {**BEST, "swiglu": (2, 4, 1024)},
    "best_sw4_1024": {**BEST, "swiglu": (4, 4, 1024)},
    "best_x512": {**BEST, "x16": (4, 4, 512)},
    "best_x2048": {**BEST, "x16": (4, 4, 2048)},
    "best_x2pf4": {**BEST, "x16": (2, 4, 1024)},
    "best_x8pf4": {**BEST, "x16": (8, 4, 1024)},
    "best_sw2pf8": {**BEST, "swiglu": (2, 8, 512)},
    "best_sw4pf8": {**BEST, "swiglu": (4, 8, 512)},
    "best_sw2pf4_768": {**BEST, "swiglu": (2, 4, 768)},
    "best_sw2pf8_1024": {**BEST, "swiglu": (2, 8, 1024)},
    "best_x4pf8": {**BEST, "x16": (4, 8, 1024)},
    "best_x2pf8": {**BEST, "x16": (2, 8, 1024)},
    "best_q4pf4": {**BEST, "qkv": (4, 4, 1024)},
    "best_q2pf4": {**BEST, "qkv": (2, 4, 1024)},
    "best_sw2pf4_1024": {**BEST, "swiglu": (2, 4, 1024)},
    "best_x2pf4_512": {**BEST, "x16": (2, 4, 512)},
    "best_x4pf4_512": {**BEST, "x16": (4, 4, 512)},
    "best_x4pf0": {**BEST, "x16": (4, 0, 1024)},
    "best_head_u2": {**BEST, "norm_f32": (2, 4, 256)},
    "best_head_512": {**BEST, "norm_f32": (4, 4, 512)},
}
if os.environ.get("SWEEP_VARIANTS"):
    VARIANTS = {k: v for k, v in VARIANTS.items()
                if k in os.environ["SWEEP_VARIANTS"].split(",") or k == "default"}


def main():
    model = os.environ.get("SWEEP_MODEL", "llama3-8b")
    m = random_model(model, "cuda:0", torch.bfloat16, max_seq=1024)
    steps = int(os.environ.get("SWEEP_STEPS", "96"))
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
            run_decode(dec, steps)
            torch.cuda.synchronize()
            res[name].append(steps / (time.perf_counter() - t0))
            del dec
    for name, v in res.items():
        print(json.dumps({"variant": name, "tok_s": [round(x, 1) for x in v],
                          "best": round(max(v), 1)}), flush=True)


if __name__ == "__main__":
    main()
