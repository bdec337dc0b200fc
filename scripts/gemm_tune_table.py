"""Write cake_amd/ops/gemm_tuned.json from a bench_gemm.py --sweep JSONL: the measured
best (tile config, split-K) per (M, weight rows, K, epilogue)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, dst=os.path.join(ROOT, "cake_amd", "ops", "gemm_tuned.json")):
    table = []
    for line in open(src):
        r = json.loads(line)
        if "best" not in r:
            continue
        nv = 2 * r["N"] if r["epi"] in ("swiglu", "geglu") else r["N"]
        table.append({"M": r["M"], "Nv": nv, "K": r["K"], "epi": r["epi"],
                      "cfg": r["best"]["cfg"], "splits": r["best"]["splits"],
                      "tflops": r["best"]["tflops"], "shape": r["shape"]})
    with open(dst, "w") as f:
        json.dump({"source": os.path.basename(src), "entries": table}, f, indent=1)
    print(f"{len(table)} entries -> {dst}")


if __name__ == "__main__":
    main(*sys.argv[1:])
