"""Stall classes and LDS conflicts per kernel from one rocprofv3 --pmc pass:
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES (scripts/gpu_runs/gpu_sdpmc2.sh).

    python scripts/prof_pmc_stalls.py COUNTERS.csv --last N [--title ...]

Per kernel over the last N dispatches (the final steps): share of the kernels' wave-cycles,
then of its own wave-cycles parked at s_waitcnt / barriers (WAIT_ANY), stalled at issue
(WAIT_INST_ANY, of which LDS issue: WAIT_INST_LDS) and issuing (ACTIVE_INST_ANY) — these
three are disjoint and sum to about WAVE_CYCLES (MI355X_MICROARCH, PMC table) — the LDS bank
conflict cycles as a share of all LDS-array cycles, and MFMA busy per wave-cycle.
"""
import argparse
import collections
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("--last", type=int, required=True)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(a.pmc)):
        d = per[(int(r["Dispatch_Id"]), r["Kernel_Name"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for (_, name), d in sorted(per.items())[-a.last:]:
        g = agg[name]
        g["n"] += 1
        for k, v in d.items():
            g[k] += v
    tot = sum(g.get("SQ_WAVE_CYCLES", 0.0) for g in agg.values()) or 1.0
    if a.title:
        print(f"# {a.title}")
    print(f"{'kernel':58s} {'calls':>5s} {'wave%':>6s} {'wait%':>6s} {'stall%':>6s} "
          f"{'lds_st%':>7s} {'active%':>7s} {'ldsconf%':>8s} {'mfma/wc':>8s}")
    for name, g in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0.0)):
        wc = g.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0:
            continue
        lds = g.get("SQ_LDS_IDX_ACTIVE", 0.0)
        short = name.replace("void ", "").split("(")[0][:58]
        # WAVE/WAIT/ACTIVE count quad-cycles, MFMA busy counts cycles
        print(f"{short:58s} {g['n']:5.0f} {100 * wc / tot:6.1f} "
              f"{100 * g.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
              f"{100 * g.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
              f"{100 * g.get('SQ_WAIT_INST_LDS', 0) / wc:7.1f} "
              f"{100 * g.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.1f} "
              f"{(100 * g.get('SQ_LDS_BANK_CONFLICT', 0) / lds) if lds else 0.0:8.1f} "
              f"{g.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (4 * wc):8.3f}")


if __name__ == "__main__":
    main()
