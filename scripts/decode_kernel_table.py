"""Per-kernel bytes / TB/s table for 8B batch-1 decode from a rocprofv3 kernel-trace db.

Decode steps are the kernels between prefill and the end; gemv_x16 launches alternate
o_proj / down_proj within a layer.  The lm_head row is the fused greedy tail (lm_head +
repeat penalty + argmax + finalize + the next step's embedding row) in greedy decode.  Bytes are the weight (and KV) bytes each kernel
must stream; the speed-of-light column is scripts/decode_ceiling.py's pure-read probe
for the same bytes and kernel structure (profiles/r2_decode_ceiling.jsonl).

    python scripts/decode_kernel_table.py run_results.db --ctx 2064
"""
import argparse
import sqlite3

H, I, NH, NKV, HD, V = 4096, 14336, 32, 8, 128, 128256
BYTES = {"qkv_rope": (NH + 2 * NKV) * HD * H * 2, "o_proj": H * H * 2, "swiglu": 2 * I * H * 2,
         "down_proj": H * I * 2, "lm_head": V * H * 2}
PROBE_US = {"qkv_rope": 9.03, "attn_decode": 1.94, "o_proj": 6.59, "swiglu": 35.79,
            "down_proj": 18.92, "lm_head": 165.6}


def kind(name):
    if "attn_oproj" in name:  # fused attention + o_proj (one-split lengths)
        return "attn_oproj"
    if "attn2_decode" in name or "attn_head_kernel" in name:  # core 2 / head-parallel
        return "attn_decode"
    for k in ("qkv_rope", "swiglu", "attn_decode", "gemv_norm_f32", "gemv_x16"):
        if k in name:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--ctx", type=int, required=True, help="mean live context of the decode steps")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    agg, x16 = {}, 0
    fused = any(kind(n) == "attn_oproj" for n, _, _ in rows)
    for n, s, e in rows:
        k = kind(n)
        if k is None:
            continue
        if k == "gemv_x16":  # o_proj / down_proj alternate; only down_proj beside the fused
            k = "down_proj" if fused else ("o_proj" if x16 % 2 == 0 else "down_proj")
            x16 += 1
        if k == "gemv_norm_f32":
            k = "lm_head"
        agg.setdefault(k, []).append((e - s) / 1e3)
    BYTES["attn_decode"] = 2 * NKV * a.ctx * HD * 2
    BYTES["attn_oproj"] = BYTES["o_proj"] + BYTES["attn_decode"]
    PROBE_US["attn_oproj"] = PROBE_US["o_proj"]
    print(f"{'kernel':<12} {'calls':>6} {'avg_us':>8} {'MB':>9} {'TB/s':>6} {'probe_us':>9} {'of_probe':>8}")
    per_tok = 0.0
    for k in ("qkv_rope", "attn_decode", "o_proj", "attn_oproj", "swiglu", "down_proj", "lm_head"):
        if k not in agg:
            continue
        d = sorted(agg[k])
        avg = sum(d) / len(d)
        per_tok += avg * (1 if k == "lm_head" else 32)
        b = BYTES[k]
        print(f"{k:<12} {len(d):>6} {avg:>8.2f} {b / 1e6:>9.1f} {b / avg / 1e6:>6.2f} "
              f"{PROBE_US[k]:>9.2f} {PROBE_US[k] / avg:>8.0%}")
    print(f"sum of kernel time per token (32 layers + head): {per_tok / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
