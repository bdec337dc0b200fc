"""Decode attention latency breakdown from in-kernel phase clocks (s_memtime, thread 0 of
every workgroup; cake_attn_set_stamps).  Phases: 0 start, 1 position read issued,
2 first chunk in LDS, 3 chunk loop done, 4 key groups combined, 5 partial published /
direct write issued, 6 ticket known, 7 merge done (last workgroup only).

Each launch follows a 64 MiB streaming read, as in decode (K/V not L2-resident).
IMPLS=1,2 selects the decode-attention cores (attn_core.h / attn_core2.h); TARGETS the
core-2 split targets, MINKS the minimum keys per split."""
import ctypes as C
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cake_amd.ops import hip as K  # noqa: E402
from cake_amd.ops._lib import kernels  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    nh, nkv, hd, S = 32, 8, 128, 8192
    kc = torch.randn(nkv, S, hd, device=dev).to(dt)
    vc = torch.randn(nkv, S, hd, device=dev).to(dt)
    q = torch.randn(nh * hd, device=dev)
    part = torch.zeros(K.attn_workspace_numel(nh, hd, S), device=dev)
    tickets = torch.zeros(2 * nkv + 2, dtype=torch.int32, device=dev)
    out = torch.empty(nh * hd, device=dev, dtype=dt)
    pos = torch.zeros(1, dtype=torch.int32, device=dev)
    big = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    stamps = torch.zeros(nkv * 64 * 8, dtype=torch.int64, device=dev)
    lib = kernels()
    lib.cake_attn_set_stamps.argtypes = [C.c_void_p]
    lib.cake_attn_set_stamps.restype = C.c_int
    impls = [int(x) for x in os.environ.get("IMPLS", "1,2").split(",")]
    minks = [int(x) for x in os.environ.get("MINKS", "64").split(",")]
    targets = [int(x) for x in os.environ.get("TARGETS", "16").split(",")]
    K.attn_set_single_max(int(os.environ.get("SINGLE", "320")))
    cases = [(i, mk, tg, int(x)) for i in impls for mk in minks for tg in targets
             for x in os.environ.get("TKS", "57,176,512,1024,2048,4000").split(",")]
    for impl, mk, tg, Tk in cases:
        K.attn_set_impl(impl)
        K.attn_set_min_keys(mk)
        K.attn_set_target_splits(tg)
        pos.fill_(Tk - 1)
        need = K.attn_splits(Tk)
        cap = next(c for c in (8, 16, 32, 64) if c >= need) if need <= 64 else 64
        rec = {"impl": impl, "min_keys": mk, "target": tg, "Tk": Tk, "cap": cap, "splits": need}
        with K.attn_split_cap(cap):
            # plain timing: events around each launch after a streaming read
            ts = []
            for _ in range(20):
                big.view(torch.int32)[: 8 << 20].sum()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                K.attn_decode(q, kc, vc, pos, 1 / math.sqrt(hd), part, tickets, out)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            rec["event_us_median"] = round(sorted(ts)[len(ts) // 2], 2)
            lib.cake_attn_set_stamps(C.c_void_p(stamps.data_ptr()))
            rows = []
            for _ in range(10):
                stamps.zero_()
                big.view(torch.int32)[: 8 << 20].sum()
                K.attn_decode(q, kc, vc, pos, 1 / math.sqrt(hd), part, tickets, out)
                torch.cuda.synchronize()
                st = stamps.view(64, nkv, 8).cpu()
                rows.append(st)
            lib.cake_attn_set_stamps(C.c_void_p(0))
        ph = {}
        for st in rows:
            for s in range(64):
                for g in range(nkv):
                    r = st[s, g].tolist()
                    if r[0] == 0:
                        continue
                    for k in range(1, 8):
                        if r[k] != 0:
                            ph.setdefault(f"p{k}", []).append(r[k] - r[0])
        for k, v in sorted(ph.items()):
            v = sorted(v)
            rec[k + "_cyc_med"] = v[len(v) // 2]
            rec[k + "_cyc_max"] = v[-1]
            rec[k + "_n"] = len(v)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
