"""Per-kernel MFMA roofline of one step from a rocprofv3 --pmc pass and a --kernel-trace run.

    python scripts/prof_pmc_roofline.py --pmc COUNTERS.csv --trace TRACE.csv --ms 148.5 \
        --steps 5 [--pmc-steps 2] [--title ...]

The PMC pass (GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES) gives, per
kernel name, averages per dispatch:
  * effective clock  = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall (MI355X_MICROARCH "DVFS");
  * MFMA work        = SQ_VALU_MFMA_BUSY_CYCLES x 1024 FLOP: the counter sums busy cycles over
    every SIMD, and one SIMD retires 1024 dense bf16/f16 FLOP per busy cycle (a 32x32x16
    MFMA = 32 cycles = 32768 FLOP), so this is the MFMA FLOP count the kernel executed,
    padding included, with no FLOP model;
  * MFMA utilisation = busy cycles / (1024 SIMDs x clock cycles of the dispatch).
The kernel-trace window (un-profiled clock) gives the dispatches and kernel time per step;
the table itself comes from the PMC run alone, TFLOP/s against the 2.5 PFLOP/s dense peak.
"""
import argparse
import collections
import csv

PEAK_TFLOPS = 2500.0
SIMDS = 256 * 4
FLOP_PER_BUSY_CYCLE = 1024


def pmc_by_kernel(path, last):
    """Counters summed per kernel name over the LAST `last` dispatches of the run (the
    final steps: earlier dispatches include tuning trials of other shapes)."""
    per_disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = per_disp[(int(r["Dispatch_Id"]), r["Kernel_Name"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["wall"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for (_, name), d in sorted(per_disp.items())[-last:]:
        a = agg[name]
        a["n"] += 1
        for k, v in d.items():
            a[k] += v
    return agg


def trace_window(path, ms):
    rows = list(csv.DictReader(open(path)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    lo = end - int(ms * 1e6)
    agg = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        if int(r["Start_Timestamp"]) >= lo:
            agg[r["Kernel_Name"]][0] += 1
            agg[r["Kernel_Name"]][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return agg


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--ms", type=float, required=True)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--pmc-steps", type=int, default=2,
                    help="steps at the end of the PMC run to take counters from")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    win = trace_window(a.trace, a.ms)
    per_step = round(sum(c for c, _ in win.values()) / a.steps)
    pmc = pmc_by_kernel(a.pmc, per_step * a.pmc_steps)
    if a.title:
        print(f"# {a.title}")
    kt_ms = sum(t for _, t in win.values()) / 1e6 / a.steps
    print(f"# un-profiled kernel-trace run: {kt_ms:.3f} ms of kernels per step, "
          f"{per_step} dispatches per step")
    print(f"# table: the last {a.pmc_steps} steps of the PMC run ALONE (the kernel variants the "
          f"tuner picks can differ run to run, so no cross-run join); ms = profiled dispatch "
          f"wall; FLOP = SQ_VALU_MFMA_BUSY_CYCLES x 1024 (executed MFMA work, padding "
          f"included); mfma% = busy / (1024 SIMDs x clock cycles)")
    print(f"{'kernel':64s} {'calls':>5s} {'ms/step':>8s} {'GFLOP/step':>10s} {'TFLOP/s':>8s} "
          f"{'%peak':>6s} {'mfma%':>6s} {'GHz':>5s} {'waves':>7s}")
    tot_t = tot_f = 0.0
    rows = []
    for name, p in pmc.items():
        n = p["n"]
        t_ms = p["wall"] / 1e6 / a.pmc_steps
        cyc = p.get("GRBM_GUI_ACTIVE", 0.0) / 8
        busy = p.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        gflop = busy * FLOP_PER_BUSY_CYCLE / 1e9 / a.pmc_steps
        ghz = cyc / p["wall"] if p["wall"] else 0.0
        util = 100 * busy / (SIMDS * cyc) if cyc else 0.0
        rows.append((t_ms, name, n / a.pmc_steps, gflop, util, ghz, p.get("SQ_WAVES", 0.0) / n))
        tot_t += t_ms
        tot_f += gflop
    for t_ms, name, calls_s, gflop, util, ghz, waves in sorted(rows, key=lambda r: -r[0]):
        tf = gflop / t_ms if t_ms else 0.0  # GFLOP / ms = TFLOP/s
        short = name.replace("void ", "").split("(")[0][:64]
        print(f"{short:64s} {calls_s:5.0f} {t_ms:8.3f} {gflop:10.1f} {tf:8.1f} "
              f"{100 * tf / PEAK_TFLOPS:6.1f} {util:6.1f} {ghz:5.2f} {waves:7.0f}")
    tf = tot_f / tot_t if tot_t else 0.0
    print(f"{'TOTAL (profiled)':64s} {'':5s} {tot_t:8.3f} {tot_f:10.1f} {tf:8.1f} "
          f"{100 * tf / PEAK_TFLOPS:6.1f}")
    print(f"{'TOTAL FLOP at the un-profiled step time':64s} {'':5s} {kt_ms:8.3f} {tot_f:10.1f} "
          f"{tot_f / kt_ms:8.1f} {100 * tot_f / kt_ms / PEAK_TFLOPS:6.1f}")


if __name__ == "__main__":
    main()
