"""Per-token timeline analysis of a rocprofv3 kernel trace: busy time vs inter-kernel gaps."""
import sqlite3
import sys
from collections import defaultdict


def main(db, marker="gemv_norm_f32"):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    # token boundaries = lm_head kernel (one per token)
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(idx) < 3:
        print("not enough tokens")
        return
    busy, wall, gaps = 0.0, 0.0, 0.0
    per_kernel = defaultdict(float)
    gap_after = defaultdict(float)
    ntok = 0
    for a, b in zip(idx[-12:-1], idx[-11:]):  # last ~10 decode tokens
        seg = rows[a + 1:b + 1]
        wall += (seg[-1][2] - rows[a][2]) / 1e3
        prev_end = rows[a][2]
        for n, s, e in seg:
            short = n.split("(")[0].replace("void ", "").replace("cake::", "")[:48]
            per_kernel[short] += (e - s) / 1e3
            busy += (e - s) / 1e3
            g = max(0, s - prev_end) / 1e3
            gaps += g
            gap_after[short] += g
            prev_end = e
        ntok += 1
    print(f"tokens analysed: {ntok}; per token: wall {wall/ntok:.1f} us, kernels {busy/ntok:.1f} us, "
          f"gaps {gaps/ntok:.1f} us")
    for k, v in sorted(per_kernel.items(), key=lambda kv: -kv[1]):
        print(f"  {k:<50} {v/ntok:9.1f} us/token   gap-before {gap_after[k]/ntok:7.1f} us/token")


if __name__ == "__main__":
    main(*sys.argv[1:])
