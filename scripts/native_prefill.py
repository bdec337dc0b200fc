"""Native-engine prefill of one long prompt, repeated (for rocprofv3 --kernel-trace windows:
the last prefill is the trailing kernels).  Random-init weights of the named preset.

python scripts/native_prefill.py [--model llama3-8b] [--len 2048] [--reps 3]"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.engine import NativeLlama, write_config  # noqa: E402
from cake_amd.models.llama3.config import preset  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--len", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    d = write_config(tempfile.mkdtemp(prefix="cake_prefill_"), preset(a.model))
    eng = NativeLlama(d, max_seq=a.len + 16, dtype="bf16", random_init=True, seed=1)
    prompt = [(i * 7919) % 1000 + 10 for i in range(a.len)]
    for r in range(a.reps):
        t0 = time.perf_counter()
        eng.prefill_logits(prompt)
        print(f"prefill {a.len} rep {r}: {1e3 * (time.perf_counter() - t0):.2f} ms (host clock)",
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
