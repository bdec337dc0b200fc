"""Per-kernel totals from a rocprofv3 --kernel-trace SQLite database (rocpd): calls, total
and mean time, share; optional --last-ms window (the tail of the run, e.g. the timed steps).

    python scripts/kernel_stats_db.py run_results.db [--top 30] [--per N] [--last-ms MS]
(--per N divides the totals by N: per step / per token tables)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--last-ms", type=float, default=0.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    if a.last_ms > 0 and rows:
        t_end = max(r[2] for r in rows)
        rows = [r for r in rows if r[1] >= t_end - a.last_ms * 1e6]
    agg: dict = {}
    for n, s, e in rows:
        t = agg.setdefault(n, [0, 0.0])
        t[0] += 1
        t[1] += (e - s)
    tot = sum(v[1] for v in agg.values())
    print(f"kernels: {len(rows)} dispatches, {tot / 1e6 / a.per:.3f} ms (per {a.per:g})")
    print(f"{'ms':>9} {'calls':>7} {'avg_us':>9} {'share':>6}  kernel")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / 1e6 / a.per:9.3f} {k / a.per:7.1f} {t / k / 1e3:9.2f} {100 * t / tot:5.1f}%  {n[:120]}")


if __name__ == "__main__":
    main()
