// Decode GEMV launchers: SwiGLU (gate|up with the RMSNorm prologue) and the 16-bit-input
// GEMV (o_proj / down_proj, optional residual accumulate).  Kernels: gemv_kernel.h.
#include "gemv_kernel.h"

CAKE_API int cake_swiglu(int dt, const float* resid, const void* norm_w, float eps,
                         const void* wg, const void* wu, int K, int I, void* act,
                         hipStream_t st) {
  if (K % 8) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)K * sizeof(float);
  const GemvTune t = g_tune[kSwiglu];
  // at least one block per 28 rows (7 row pairs per wave): 70B's I = 28672 runs 1024
  // blocks (+0.7 %, profiles/r2_decode_gemv_tuning_70b.jsonl), 8B's 14336 the tuned 512
  const int mb = t.MB > (I + 27) / 28 ? t.MB : (I + 27) / 28;
  DISPATCH_DT(dt, DISPATCH_TUNE(t, K, CAKE_NX_NORM(K, hipLaunchKernelGGL((swiglu_kernel<DT, U, PF, NX>),
                                                      dim3(grid_for(I, mb)), dim3(kGemvThreads),
                                                      lds, st, resid, (const uint16_t*)norm_w, eps,
                                                      (const uint16_t*)wg, (const uint16_t*)wu, K,
                                                      I, (uint16_t*)act))));
  return (int)hipGetLastError();
}

CAKE_API int cake_gemv_x16(int dt, const void* x, const void* w, int K, int N, float* out,
                           int accumulate, hipStream_t st) {
  if (K % 8) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)K * 2;
  const GemvTune t = g_tune[K <= 8192 ? kX16S : kX16];
  const int g = grid_for((N + 1) / 2, t.MB);
  if (accumulate) {
    DISPATCH_DT(dt, DISPATCH_TUNE(t, K, CAKE_NX_X16(K, hipLaunchKernelGGL((gemv_x16_kernel<DT, U, PF, NX, true>),
                                                        dim3(g), dim3(kGemvThreads), lds, st,
                                                        (const uint16_t*)x, (const uint16_t*)w, K,
                                                        N, out))));
  } else {
    DISPATCH_DT(dt, DISPATCH_TUNE(t, K, CAKE_NX_X16(K, hipLaunchKernelGGL((gemv_x16_kernel<DT, U, PF, NX, false>),
                                                        dim3(g), dim3(kGemvThreads), lds, st,
                                                        (const uint16_t*)x, (const uint16_t*)w, K,
                                                        N, out))));
  }
  return (int)hipGetLastError();
}

