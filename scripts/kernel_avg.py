"""Average duration (us) of the kernels whose name contains each argument, from a
rocprofv3 kernel-trace database:  python scripts/kernel_avg.py run_results.db argmax ..."""
import sqlite3
import sys


def main(db, pats):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    nc = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {nc}, start, end from kernels").fetchall()
    for p in pats:
        v = [(e - s) / 1e3 for n, s, e in rows if p in n]
        print(f"{p}: {len(v)} calls, avg {sum(v) / max(1, len(v)):.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
