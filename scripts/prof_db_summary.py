"""Per-kernel table from a rocprofv3 SQLite output (run_results.db): calls, mean and total
device time, sorted by total.   python scripts/prof_db_summary.py DB [--top N]"""
import argparse
import sqlite3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, count(*), avg(end - start) / 1000.0, sum(end - start) / 1e6 "
                       "from kernels group by name order by sum(end - start) desc limit ?",
                       (a.top,)).fetchall()
    print(f"{'calls':>7} {'avg_us':>9} {'total_ms':>9}  kernel")
    for name, n, avg, tot in rows:
        print(f"{n:7d} {avg:9.2f} {tot:9.2f}  {name[:120]}")


if __name__ == "__main__":
    main()
