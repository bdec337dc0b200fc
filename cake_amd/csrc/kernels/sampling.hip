// On-device token selection: repeat penalty, argmax, and the step finalizer.
//
// Reference: cake-core/src/models/llama3/llama.rs:311-327 — repeat penalty over
// the last `repeat_last_n` tokens (candle-transformers apply_repeat_penalty: for
// each *unique* recent token, s >= 0 ? s / p : s * p, done on the host after a
// D2H copy of the logits) followed by LogitsProcessor::sample (ArgMax when
// temperature <= 0).  Here both run on the device so the whole decode step
// (embedding -> layers -> lm_head -> penalty -> argmax -> next input token)
// is one hipGraph replay with a 4-byte readback.
#include "common.h"

namespace cake {

__global__ void repeat_penalty_kernel(float* __restrict__ logits, const int* __restrict__ hist,
                                      const int* __restrict__ hist_len, int last_n,
                                      float penalty) {
  const int len = *hist_len;
  const int n = min(last_n, len);
  const int start = len - n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int tok = hist[start + i];
    bool dup = false;
    for (int j = 0; j < i; ++j) dup |= (hist[start + j] == tok);
    if (!dup) {
      const float s = logits[tok];
      logits[tok] = s >= 0.f ? s / penalty : s * penalty;
    }
  }
}

__device__ __forceinline__ unsigned int ordered(float f) {
  const unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// slot holds max over (ordered(value) << 32 | ~index): ties -> smallest index.
__global__ __launch_bounds__(256) void argmax_kernel(const float* __restrict__ logits, int V,
                                                     unsigned long long* __restrict__ slot) {
  __shared__ unsigned long long red[4];
  unsigned long long best = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < V; i += gridDim.x * blockDim.x) {
    const unsigned long long key =
        ((unsigned long long)ordered(logits[i]) << 32) | (0xffffffffu - (unsigned int)i);
    best = key > best ? key : best;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(best, off, 64);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) best = red[w] > best ? red[w] : best;
    atomicMax(slot, best);
  }
}

// Publish the argmax as the next input token; advance position/history; reset slot.
__global__ void finalize_kernel(unsigned long long* __restrict__ slot, int* __restrict__ tok,
                                int* __restrict__ hist, int* __restrict__ hist_len,
                                int* __restrict__ pos, int max_hist) {
  const unsigned long long key = *slot;
  const int t = (int)(0xffffffffu - (unsigned int)(key & 0xffffffffu));
  *tok = t;
  const int len = *hist_len;
  if (len < max_hist) { hist[len] = t; *hist_len = len + 1; }
  *pos += 1;
  *slot = 0ull;
}

// Write an externally chosen token (host-side sampler path) into the same state.
__global__ void push_token_kernel(const int* __restrict__ src, int* __restrict__ tok,
                                  int* __restrict__ hist, int* __restrict__ hist_len,
                                  int* __restrict__ pos, int max_hist) {
  const int t = *src;
  *tok = t;
  const int len = *hist_len;
  if (len < max_hist) { hist[len] = t; *hist_len = len + 1; }
  *pos += 1;
}

}  // namespace cake

using namespace cake;

CAKE_API int cake_repeat_penalty(float* logits, const int* hist, const int* hist_len,
                                 int last_n, float penalty, hipStream_t st) {
  hipLaunchKernelGGL(repeat_penalty_kernel, dim3(1), dim3(256), 0, st, logits, hist, hist_len,
                     last_n, penalty);
  return (int)hipGetLastError();
}

CAKE_API int cake_argmax(const float* logits, int V, unsigned long long* slot,
                         hipStream_t st) {
  int g = (V + 255) / 256;
  if (g > 512) g = 512;
  hipLaunchKernelGGL(argmax_kernel, dim3(g), dim3(256), 0, st, logits, V, slot);
  return (int)hipGetLastError();
}

CAKE_API int cake_finalize_token(unsigned long long* slot, int* tok, int* hist, int* hist_len,
                                 int* pos, int max_hist, hipStream_t st) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(1), 0, st, slot, tok, hist, hist_len, pos,
                     max_hist);
  return (int)hipGetLastError();
}

CAKE_API int cake_push_token(const int* src, int* tok, int* hist, int* hist_len, int* pos,
                             int max_hist, hipStream_t st) {
  hipLaunchKernelGGL(push_token_kernel, dim3(1), dim3(1), 0, st, src, tok, hist, hist_len, pos,
                     max_hist);
  return (int)hipGetLastError();
}
