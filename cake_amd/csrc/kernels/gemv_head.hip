// Decode GEMV launchers: the f32-output RMSNorm GEMV (lm_head) and the fused greedy
// tail (lm_head + repeat penalty + argmax + step finalize).  Kernels: gemv_kernel.h.
#include "gemv_kernel.h"

template <bool SEL>
static int launch_norm_f32(int dt, const float* resid, const void* norm_w, float eps,
                           const void* w, int K, int N, float* out, const HeadSel& hs,
                           hipStream_t st) {
  if (K % 8) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)K * sizeof(float);
  const GemvTune t = g_tune[kNormF32];
  DISPATCH_DT(dt, DISPATCH_TUNE(t, K, CAKE_NX_NORM(K, hipLaunchKernelGGL((gemv_norm_f32_kernel<DT, U, PF, NX, SEL>),
                                                      dim3(grid_for((N + 1) / 2, t.MB)),
                                                      dim3(kGemvThreads), lds, st, resid,
                                                      (const uint16_t*)norm_w, eps,
                                                      (const uint16_t*)w, K, N, out, hs))));
  return (int)hipGetLastError();
}

CAKE_API int cake_gemv_norm_f32(int dt, const float* resid, const void* norm_w, float eps,
                                const void* w, int K, int N, float* out, hipStream_t st) {
  return launch_norm_f32<false>(dt, resid, norm_w, eps, w, K, N, out, HeadSel{}, st);
}

// lm_head + repeat penalty + argmax + step finalizer in one launch (greedy decode);
// with `embed`, also the next step's input emb_out[K] = embed[tok] (f32).  slot (u64)
// and ticket (u32) must be zero before the first launch; the kernel re-arms them.
// last_n <= 256.
CAKE_API int cake_head_select(int dt, const float* resid, const void* norm_w, float eps,
                              const void* w, int K, int N, float* out, int* hist, int* hist_len,
                              int last_n, float penalty, unsigned long long* slot,
                              unsigned int* ticket, int* tok, int* pos, int max_hist,
                              const void* embed, float* emb_out, hipStream_t st) {
  if (last_n < 0 || last_n > 256 || !(penalty > 0.f) || slot == nullptr || ticket == nullptr ||
      (embed != nullptr && (emb_out == nullptr || K % 8)))
    return (int)hipErrorInvalidValue;
  const HeadSel hs{hist, hist_len, last_n, penalty, slot, ticket, tok, hist, hist_len, pos,
                   max_hist, (const uint16_t*)embed, emb_out, K};
  return launch_norm_f32<true>(dt, resid, norm_w, eps, w, K, N, out, hs, st);
}
