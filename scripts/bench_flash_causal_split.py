"""Causal flash attention (Llama prefill shapes) with a forced key split (f32 partial rows +
merge launch) vs the paired default: us per call (graph of back-to-back launches) and the
max difference to the default's output."""
import ctypes
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
    lib = K.kernels()
    for (H, Hkv, D, N) in [(32, 8, 128, 1024), (32, 8, 128, 2048), (32, 8, 128, 4096),
                           (64, 8, 128, 2048)]:
        q = torch.randn(1, N, H, D, device=dev).to(dt).transpose(1, 2)
        k = torch.randn(1, N, Hkv, D, device=dev).to(dt).transpose(1, 2)
        v = torch.randn(1, N, Hkv, D, device=dev).to(dt).transpose(1, 2)
        ws = torch.empty(4 * H * N * (D + 1), device=dev)
        st = [s for t in (q, k, v, q) for s in t.stride()[:3]]
        arr = (ctypes.c_longlong * 12)(*st)
        rec = {"H": H, "D": D, "N": N}
        outs = {}
        for name, pm, ks in (("paired", 512, 1), ("paired_ks2", 512, 2), ("unpaired_ks2", 0, 2),
                             ("paired_ks4", 512, 4), ("unpaired_ks4", 0, 4)):
            out = torch.empty(1, N, H, D, device=dev, dtype=dt).transpose(1, 2)
            st[9:12] = list(out.stride()[:3])
            arr = (ctypes.c_longlong * 12)(*st)

            def run():
                K.check(lib.cake_flash_attn_ws(0, K._p(q), K._p(k), K._p(v), K._p(out), 1, H, Hkv,
                                               N, N, D, ctypes.cast(arr, ctypes.c_void_p),
                                               1 / math.sqrt(D), 1, 0, K._p(ws), ws.numel() * 4,
                                               K._stream()), "flash")
            K.flash_set_pair_min(pm)
            lib.cake_flash_set_ksplit(ks)
            run()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    run()
            best = 1e9
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(); g.replay(); b.record(); b.synchronize()
                best = min(best, a.elapsed_time(b) / 10 * 1e3)
            outs[name] = out.float()
            rec[name + "_us"] = round(best, 2)
            rec[name + "_maxdiff"] = float((out.float() - outs["paired"]).abs().max())
        K.flash_set_pair_min(512)
        lib.cake_flash_set_ksplit(0)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
