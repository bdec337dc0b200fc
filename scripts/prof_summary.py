"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a per-kernel table."""
import sqlite3
import sys


def main(db, top=25):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        d = (e - s) / 1e3
        a = agg.setdefault(n, [0, 0.0, 1e30, 0.0])
        a[0] += 1; a[1] += d; a[2] = min(a[2], d); a[3] = max(a[3], d)
    tot = sum(a[1] for a in agg.values())
    print(f"{'kernel':<80} {'calls':>7} {'total_us':>11} {'avg_us':>9} {'min_us':>8} {'%':>6}")
    for n, a in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        short = n if len(n) < 80 else n[:77] + "..."
        print(f"{short:<80} {a[0]:>7} {a[1]:>11.1f} {a[1]/a[0]:>9.2f} {a[2]:>8.2f} {100*a[1]/tot:>6.1f}")
    print(f"total kernel time {tot/1e3:.2f} ms over {sum(a[0] for a in agg.values())} dispatches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
