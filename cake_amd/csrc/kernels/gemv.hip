// Batch-1 decode projections: bandwidth-bound GEMV with fused prologues/epilogues.
//
// Replaces the reference's per-layer chain of candle ops for one decode token
// (SURVEY §2.4.1 K02 rms_norm, K03 Linear, K04 head-major copy, K05 rope,
// K06 kv cat, K14 residual add, K15 silu*mul, K17 logits cast), i.e.
//   cake-core/src/models/llama3/transformer.rs:51-73 (block forward),
//   cake-core/src/models/llama3/attention.rs:49-83 (q/k/v proj + rope),
//   cake-core/src/models/llama3/mlp.rs:15-18 (SwiGLU),
//   cake-core/src/models/llama3/llama.rs:119-137 (ln_f + lm_head -> f32).
//
// Design (MI355X-first):
//   * Weights stay in HF [out, in] row-major layout; every weight byte is read
//     exactly once per token with 16-byte non-temporal loads.
//   * One wave64 computes a PAIR of output rows so that the pair needs no
//     cross-wave communication in its epilogue:
//       - QKV:    rows (i, i + d/2) of one head -> RoPE rotation in registers,
//                 q written f32, k/v written straight into the preallocated
//                 KV cache slot [kvh][pos][d] (no cat, no transpose kernel).
//       - SwiGLU: gate row j and up row j -> act[j] = silu(g) * u.
//       - Resid:  rows (2p, 2p+1) -> residual stream += W x (in place, f32).
//       - F32:    rows (2p, 2p+1) -> f32 output (lm_head logits).
//   * RMSNorm is a block prologue: the f32 residual row is normalised into LDS
//     once per workgroup (4 waves), so no separate norm launch exists.
//   * The token position is read from device memory so the launches replay
//     unchanged inside a hipGraph.
#include "gemv_kernel.h"

namespace cake {
GemvTune g_tune[kNumKinds] = {{2, 4, 1024}, {2, 4, 512}, {4, 4, 1024}, {4, 4, 256},
                                     {4, 4, 1024}};

}  // namespace cake

CAKE_API int cake_gemv_set_tuning(int kind, int U, int prefetch, int max_blocks) {
  if (kind < 0 || kind >= kNumKinds || (U != 2 && U != 4 && U != 8) || max_blocks < 1 ||
      (prefetch != 0 && prefetch != 4 && prefetch != 8))
    return (int)hipErrorInvalidValue;
  g_tune[kind] = GemvTune{U, prefetch, max_blocks};
  return 0;
}

CAKE_API int cake_qkv_rope(int dt, const float* resid, const void* norm_w, float eps,
                           const void* wq, const void* wk, const void* wv, int K, int nh,
                           int nkv, int hd, const float* inv_freq, const int* pos,
                           float* q_out, void* kcache, void* vcache, int S,
                           hipStream_t st) {
  if (K % 8 || hd % 2) return (int)hipErrorInvalidValue;
  QkvArgs a{resid, (const uint16_t*)norm_w, eps, (const uint16_t*)wq,
            (const uint16_t*)wk, (const uint16_t*)wv, K, nh, nkv, hd, inv_freq, pos,
            q_out, (uint16_t*)kcache, (uint16_t*)vcache, S};
  const int npairs = (nh + 2 * nkv) * (hd / 2);
  const size_t lds = (size_t)K * sizeof(float);
  const GemvTune t = g_tune[kQkv];
  DISPATCH_DT(dt, DISPATCH_TUNE(t, K, CAKE_NX_NORM(K, hipLaunchKernelGGL((qkv_rope_kernel<DT, U, PF, NX>),
                                                      dim3(grid_for(npairs, t.MB)),
                                                      dim3(kGemvThreads), lds, st, a))));
  return (int)hipGetLastError();
}


