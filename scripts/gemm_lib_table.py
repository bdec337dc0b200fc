"""Merge a bench_gemm_lib.py run into ops/gemm_tuned.json: per measured (M, Nv, K, epi)
the library GEMM (cfg -1) where it was >= 3% faster, else the MFMA kernel's plan.

Usage: python scripts/gemm_lib_table.py profiles/r5_gemm_lib.jsonl
"""
import json
import os
import sys

MARGIN = 0.97


def main(path):
    table = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "cake_amd", "ops", "gemm_tuned.json")
    with open(table) as f:
        t = json.load(f)
    rows = [json.loads(ln) for ln in open(path) if ln.strip().startswith("{")]
    keys = {(r["M"], r["Nv"], r["K"], r["epi"]) for r in rows}
    kept = [e for e in t["entries"] if (e["M"], e["Nv"], e["K"], e["epi"]) not in keys]
    lib = 0
    for r in rows:
        use_lib = r["lib_ms"] < MARGIN * r["ours_ms"]
        lib += use_lib
        kept.append({"M": r["M"], "Nv": r["Nv"], "K": r["K"], "epi": r["epi"],
                     "cfg": -1 if use_lib else r["ours_cfg"],
                     "splits": 1 if use_lib else r["ours_splits"],
                     "tflops": r["lib_tflops"] if use_lib else r["ours_tflops"],
                     "shape": f"llama{r['model']}_{r['proj']}"})
    t["entries"] = kept
    srcs = [x for x in t.get("lib_sources", []) if x != os.path.basename(path)]
    t["lib_sources"] = srcs + [os.path.basename(path)]  # cfg -1 = hipBLASLt where >= 3% faster
    t.pop("lib_source", None)
    with open(table, "w") as f:
        json.dump(t, f, indent=1)
    print(f"{len(rows)} shapes merged, {lib} on the library GEMM")


if __name__ == "__main__":
    main(sys.argv[1])
