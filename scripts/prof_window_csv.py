"""Kernel table of the last `ms` milliseconds of a rocprofv3 kernel_trace.csv (the timed
window of a run), with a count of library (non-cake) kernels.
    python scripts/prof_window_csv.py TRACE.csv --ms 18.3 [--title ...]"""
import argparse
import collections
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--ms", type=float, required=True)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    lo = end - int(a.ms * 1e6)
    win = [r for r in rows if int(r["Start_Timestamp"]) >= lo]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]][0] += 1
        agg[r["Kernel_Name"]][1] += d
    busy = sum(v[1] for v in agg.values())
    span = end - min(int(r["Start_Timestamp"]) for r in win)
    if a.title:
        print(f"# {a.title}")
    print(f"window {a.ms} ms: {len(win)} dispatches, kernel busy {busy / 1e6:.2f} ms of "
          f"{span / 1e6:.2f} ms span")
    lib = [n for n in agg if "cake::" not in n]
    print(f"non-cake kernels in the window: {len(lib)}"
          + (f" ({', '.join(sorted(set(n.split('(')[0][:60] for n in lib)))})" if lib else ""))
    print(f"{'kernel':80s} {'calls':>6s} {'total_us':>10s} {'avg_us':>8s} {'%':>6s}")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n[:80]:80s} {c:6d} {t / 1e3:10.1f} {t / 1e3 / c:8.2f} {100 * t / busy:6.1f}")


if __name__ == "__main__":
    main()
