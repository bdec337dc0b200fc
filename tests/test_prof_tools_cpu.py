"""The rocprofv3 summary tools whose tables are committed under profiles/ (PMC roofline, stall
classes, timed-window kernel table) on small synthetic CSVs in rocprofv3's column layout."""
import csv
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _write_pmc(path: Path, kernels: list[tuple[str, dict]]) -> None:
    cols = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id",
            "Grid_Size", "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size",
            "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Counter_Name",
            "Counter_Value", "Start_Timestamp", "End_Timestamp"]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        t = 1_000_000
        for i, (name, counters) in enumerate(kernels, start=1):
            for cn, cv in counters.items():
                w.writerow([i, i, "Agent 2", 1, 1, 1, 65536, 7, name, 256, 0, 0, 64, 0, 32, cn,
                            cv, t, t + 10_000])
            t += 20_000


def _write_trace(path: Path, kernels: list[str]) -> None:
    cols = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Thread_Id", "Dispatch_Id", "Kernel_Id",
            "Kernel_Name", "Correlation_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size_X"]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        t = 1_000_000
        for i, name in enumerate(kernels, start=1):
            w.writerow(["KERNEL_DISPATCH", 2, 1, 1, 1, i, 7, name, i, t, t + 10_000, 65536])
            t += 20_000


def _run(*args) -> str:
    r = subprocess.run([sys.executable, *map(str, args)], capture_output=True, text=True,
                       cwd=ROOT, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_roofline_and_stalls_tables(tmp_path):
    gemm = "void cake::gemm_kernel<1, 64, 160, 2, 2, 3, 2, 6>(cake::GemmArgs)"
    norm = "void cake::layernorm_wave_kernel<1, 4>(unsigned short const*)"
    # 10 us dispatches: 24000 GRBM cycles / 8 XCDs = 3000 cycles -> 0.3 GHz; MFMA busy
    # 1024 SIMDs x 3000 cycles x 25 % = 768000 -> 0.786 GFLOP per dispatch
    c = {"GRBM_GUI_ACTIVE": 24000, "SQ_BUSY_CYCLES": 1, "SQ_VALU_MFMA_BUSY_CYCLES": 768000,
         "SQ_WAVES": 2560, "SQ_WAVE_CYCLES": 1000, "SQ_WAIT_ANY": 400,
         "SQ_WAIT_INST_ANY": 200, "SQ_ACTIVE_INST_ANY": 400, "SQ_WAIT_INST_LDS": 10,
         "SQ_LDS_BANK_CONFLICT": 5, "SQ_LDS_IDX_ACTIVE": 50}
    n = {**c, "SQ_VALU_MFMA_BUSY_CYCLES": 0}
    pmc = tmp_path / "pmc.csv"
    _write_pmc(pmc, [(gemm, c), (norm, n)] * 3)
    trace = tmp_path / "kt.csv"
    _write_trace(trace, [gemm, norm] * 3)
    out = _run("scripts/prof_pmc_roofline.py", "--pmc", pmc, "--trace", trace, "--ms", 1,
               "--steps", 3, "--pmc-steps", 3)
    row = next(line for line in out.splitlines() if line.startswith("cake::gemm_kernel"))
    f = row.split()
    assert f[-3] == "25.0"        # MFMA utilisation
    assert float(f[-6]) == 0.8    # GFLOP per step (one dispatch per step)
    out = _run("scripts/prof_pmc_stalls.py", pmc, "--last", 6)
    row = next(line for line in out.splitlines() if line.startswith("cake::gemm_kernel"))
    f = row.split()
    assert f[-6:-1] == ["40.0", "20.0", "1.0", "40.0", "10.0"]


def test_window_table_counts_library_kernels(tmp_path):
    trace = tmp_path / "kt.csv"
    _write_trace(trace, ["void cake::swiglu_kernel<0, 2, 4, 4>(float const*)",
                         "__amd_rocclr_copyBuffer"] * 2)
    out = _run("scripts/prof_window_csv.py", trace, "--ms", 1)
    assert "non-cake kernels in the window: 1 (__amd_rocclr_copyBuffer)" in out
    assert "4 dispatches" in out
