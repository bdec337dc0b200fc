"""Per-kernel summary of the LAST `window_ms` of a rocprofv3 kernel trace (steady state,
excluding library autotuning and warmup dispatches at the start of the run)."""
import sqlite3
import sys


def main(db, window_ms, top=25):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    t_end = rows[-1][2]
    rows = [r for r in rows if r[1] >= t_end - window_ms * 1e6]
    agg = {}
    for n, s, e in rows:
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    tot = sum(a[1] for a in agg.values())
    span = (rows[-1][2] - rows[0][1]) / 1e6
    print(f"window {window_ms} ms: {len(rows)} dispatches, kernel busy {tot/1e3:.2f} ms of {span:.2f} ms span")
    print(f"{'kernel':<80} {'calls':>6} {'total_us':>10} {'avg_us':>8} {'%':>6}")
    for n, a in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        short = n if len(n) < 80 else n[:77] + "..."
        print(f"{short:<80} {a[0]:>6} {a[1]:>10.1f} {a[1]/a[0]:>8.2f} {100*a[1]/tot:>6.1f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 25)
