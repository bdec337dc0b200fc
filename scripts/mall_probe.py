"""Does a weight matrix read shortly before its GEMV (e.g. by idle CUs during the decode
attention) make the GEMV faster?  MI355X's 256 MB memory-side cache (MALL) keeps lines a
prior read brought in; this probe times the o_proj-shaped GEMV cold vs after a read of the
same matrix (MALL + L2 warm) vs after that read plus an L2-evicting read (MALL only).

All timings are hipGraph replays of 64 (reads, GEMV) groups over 64 distinct matrices
(2.1 GB, beyond the MALL), so every "cold" GEMV really comes from HBM.
Prints one JSON line per case."""
import argparse
import json

import torch

from cake_amd.ops import hip as K


def timed(fn, reps=5):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e3
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--mats", type=int, default=64)
    ap.add_argument("--blocks", type=int, default=1024)
    a = ap.parse_args()
    dev = "cuda:0"
    W = [torch.randn(a.n, a.k, device=dev, dtype=torch.bfloat16) for _ in range(a.mats)]
    E = torch.empty(48 << 20, device=dev, dtype=torch.uint8)  # > 32 MB of L2
    x = torch.randn(a.k, device=dev, dtype=torch.bfloat16)
    out = torch.empty(a.n, device=dev, dtype=torch.float32)
    sink = torch.zeros(64, device=dev, dtype=torch.int32)
    M = a.mats
    rd = lambda t: K.stream_read(t, a.blocks, sink)  # noqa: E731
    t_cold = timed(lambda: [K.gemv(x, w, out, False) for w in W])
    t_read = timed(lambda: [rd(w) for w in W])
    t_read_gemv = timed(lambda: [(rd(w), K.gemv(x, w, out, False)) for w in W])
    t_read_evict = timed(lambda: [(rd(w), rd(E)) for w in W])
    t_read_evict_gemv = timed(lambda: [(rd(w), rd(E), K.gemv(x, w, out, False)) for w in W])
    mb = a.n * a.k * 2 / 1e6
    rows = {
        "gemv_cold_us": t_cold / M,
        "read_us": t_read / M,
        "gemv_after_read_us": (t_read_gemv - t_read) / M,
        "gemv_after_read_and_l2_evict_us": (t_read_evict_gemv - t_read_evict) / M,
    }
    for k, v in rows.items():
        print(json.dumps({"case": k, "us": round(v, 3), "MB": round(mb, 2),
                          "TBps": round(mb / v, 3) if v > 0 else None}))


if __name__ == "__main__":
    main()
