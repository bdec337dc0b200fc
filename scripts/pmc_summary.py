"""Summarise rocprofv3 --pmc CSV (counter_collection.csv): per kernel, the mean of each
counter over dispatches (counters summed over their dimensions within a dispatch)."""
import csv
import sys
from collections import defaultdict


def summarise(path, match=None):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    for r in csv.DictReader(open(path)):
        k = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if match and match not in k:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    out = {}
    for k, cs in agg.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["_dispatches"] = len(next(iter(cs.values())))
    return out


if __name__ == "__main__":
    for k, cs in summarise(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None).items():
        print(k[:100])
        for c, v in sorted(cs.items()):
            print(f"   {c:<28} {v:>16.0f}")
