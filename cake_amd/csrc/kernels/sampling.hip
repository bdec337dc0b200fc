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

// logits holds vocab entries [off, off + V) (tensor-parallel shard; off = 0, V = all
// otherwise); history tokens outside the shard are skipped.
__global__ void repeat_penalty_kernel(float* __restrict__ logits, const int* __restrict__ hist,
                                      const int* __restrict__ hist_len, int last_n,
                                      float penalty, int off, int V) {
  const int len = *hist_len;
  const int n = min(last_n, len);
  const int start = len - n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int tok = hist[start + i];
    bool dup = false;
    for (int j = 0; j < i; ++j) dup |= (hist[start + j] == tok);
    const int t = tok - off;
    if (!dup && t >= 0 && t < V) {
      const float s = logits[t];
      logits[t] = s >= 0.f ? s / penalty : s * penalty;
    }
  }
}

__device__ __forceinline__ unsigned int ordered(float f) {
  const unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// slot holds max over (ordered(value) << 32 | ~index): ties -> smallest index.
// off: global vocab index of logits[0] (tensor-parallel shard)
__global__ __launch_bounds__(256) void argmax_kernel(const float* __restrict__ logits, int V,
                                                     unsigned long long* __restrict__ slot,
                                                     int off) {
  __shared__ unsigned long long red[4];
  unsigned long long best = 0;
#pragma unroll 8
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < V; i += gridDim.x * blockDim.x) {
    const unsigned long long key =
        ((unsigned long long)ordered(logits[i]) << 32) | (0xffffffffu - (unsigned int)(i + off));
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

// ---------------------------------------------------------------------------
// Sampled decoding on the device (temperature / top-k / top-p / multinomial).
//
// candle's LogitsProcessor (llama.rs:34-48, 323-326) draws from
// softmax(logits / T), optionally restricted to the top-k tokens and/or the
// smallest top-probability prefix whose mass reaches p, with a seeded host RNG.
// Here the draw is the Gumbel-max identity: argmax_i(l_i / T + G_i) with
// G_i = -log(-log(U_i)) is distributed exactly as softmax(l / T), and the same
// argmax restricted to a set S is the renormalised draw over S.  U_i comes from
// a counter-based Philox4x32-10 keyed by the 64-bit seed with counter
// (token index i, step = history length), so a replayed graph draws a fresh,
// reproducible variate every step with no RNG state.  top-k / top-p reduce to
// one threshold on the (order-preserving) logit key, found by radix select in
// one workgroup; the draw itself is the multi-workgroup argmax of the greedy
// path (same slot + finalize kernels).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t philox_u32(uint32_t c0, uint32_t c1, uint32_t k0,
                                               uint32_t k1) {
  uint32_t c2 = 0u, c3 = 0u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c1 = lo1;
    c3 = lo0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c0;
}

__device__ __forceinline__ float gumbel(uint32_t bits) {
  const float u = (float)(bits >> 8) * 5.9604644775390625e-08f + 2.98023223876953125e-08f;
  return -__logf(-__logf(u));  // u in (0, 1)
}

// Per-request sampling parameters read on the device (the API's temperature /
// top_k / top_p / seed change without recapturing the decode graph).
// temperature <= 0 selects greedy argmax.
struct SampleParams {
  float temperature;
  int top_k;
  float top_p;
  uint32_t seed_lo, seed_hi;
  uint32_t pad[3];
};

// params != nullptr overrides (inv_t, k0, k1); inv_t == 0 -> plain argmax (greedy)
__global__ __launch_bounds__(256) void gumbel_argmax_kernel(
    const float* __restrict__ logits, int V, float inv_t, uint32_t k0, uint32_t k1,
    const int* __restrict__ step_ptr, const unsigned int* __restrict__ thr,
    const SampleParams* __restrict__ params, unsigned long long* __restrict__ slot, int off) {
  __shared__ unsigned long long red[4];
  if (params != nullptr) {
    const float t = params->temperature;
    inv_t = t > 0.f ? 1.f / t : 0.f;
    k0 = params->seed_lo;
    k1 = params->seed_hi;
  }
  const bool greedy = !(inv_t > 0.f);
  const uint32_t step = (uint32_t)*step_ptr;
  const unsigned int lim = thr != nullptr ? *thr : 0u;
  unsigned long long best = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < V; i += gridDim.x * blockDim.x) {
    const float l = logits[i];
    if (ordered(l) < lim) continue;
    const uint32_t gi = (uint32_t)(i + off);  // global index: shard-independent draw
    const float v = greedy ? l : l * inv_t + gumbel(philox_u32(gi, step, k0, k1));
    const unsigned long long key = ((unsigned long long)ordered(v) << 32) | (0xffffffffu - gi);
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

constexpr int kSelThreads = 1024;

// Block-wide max / sum (1024 threads = 16 waves).
__device__ __forceinline__ float sel_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
  for (int w = 1; w < kSelThreads / 64; ++w) r = fmaxf(r, red[w]);
  return r;
}

// Threshold key: tokens with ordered(logit) >= *thr_out form the sampling set
// (top-k, then the top-p cutoff over those tokens' full-vocabulary probabilities).  One workgroup; each radix level is one pass
// over the logits (L2-resident right after the lm_head).
__global__ __launch_bounds__(kSelThreads) void sample_threshold_kernel(
    const float* __restrict__ logits, int V, float inv_t, int top_k, float top_p,
    const SampleParams* __restrict__ params, unsigned int* __restrict__ thr_out) {
  __shared__ unsigned int cnt[256];
  __shared__ float mass[256];
  __shared__ float red[kSelThreads / 64];
  __shared__ unsigned int sel[2];
  const int tid = threadIdx.x;
  if (params != nullptr) {
    const float t = params->temperature;
    if (!(t > 0.f)) {  // greedy: no restriction
      if (tid == 0) *thr_out = 0u;
      return;
    }
    inv_t = 1.f / t;
    top_k = params->top_k;
    top_p = params->top_p;
  }
  unsigned int kthr = 0u;
  if (top_k > 0 && top_k < V) {
    unsigned int prefix = 0u, pmask = 0u;
    int k = top_k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int b = tid; b < 256; b += kSelThreads) cnt[b] = 0u;
      __syncthreads();
      for (int i = tid; i < V; i += kSelThreads) {
        const unsigned int key = ordered(logits[i]);
        if ((key & pmask) == prefix) atomicAdd(&cnt[(key >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        int cum = 0, b = 255;
        for (; b > 0; --b) {
          if (cum + (int)cnt[b] >= k) break;
          cum += (int)cnt[b];
        }
        sel[0] = (unsigned int)b;
        sel[1] = (unsigned int)(k - cum);
      }
      __syncthreads();
      prefix |= sel[0] << shift;
      pmask |= 255u << shift;
      k = (int)sel[1];
      __syncthreads();
    }
    kthr = prefix;  // key of the k-th largest logit
  }
  unsigned int pthr = 0u;
  if (top_p > 0.f && top_p < 1.f) {
    // candle's TopKThenTopP / the host LogitsProcessor: the p cutoff applies to the
    // FULL-vocabulary probabilities of the top-k tokens (no renormalisation inside
    // top-k), so Z sums every token; when the top-k mass is below p all k are kept
    float m = -INFINITY;
    for (int i = tid; i < V; i += kSelThreads) m = fmaxf(m, logits[i]);
    m = sel_max(m, red);
    float z = 0.f;
    for (int i = tid; i < V; i += kSelThreads) z += __expf((logits[i] - m) * inv_t);
    z = wave_sum(z);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = z;
    __syncthreads();
    float Z = 0.f;
    for (int w = 0; w < kSelThreads / 64; ++w) Z += red[w];
    float target = top_p * Z, before = 0.f;
    unsigned int prefix = 0u, pmask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int b = tid; b < 256; b += kSelThreads) mass[b] = 0.f;
      __syncthreads();
      for (int i = tid; i < V; i += kSelThreads) {
        const float l = logits[i];
        const unsigned int key = ordered(l);
        if (key >= kthr && (key & pmask) == prefix)
          atomicAdd(&mass[(key >> shift) & 255u], __expf((l - m) * inv_t));
      }
      __syncthreads();
      if (tid == 0) {
        // descending bins: the first whose inclusive mass reaches the target holds
        // the last kept token (element J); rounding: fall back to the lowest non-empty bin
        int b = 255, last_nz = -1;
        float cum = before;
        for (; b >= 0; --b) {
          if (mass[b] > 0.f) last_nz = b;
          if (mass[b] > 0.f && cum + mass[b] >= target) break;
          cum += mass[b];
        }
        if (b < 0) { b = last_nz < 0 ? 0 : last_nz; cum -= (last_nz < 0 ? 0.f : mass[b]); }
        sel[0] = (unsigned int)b;
        red[0] = cum;
      }
      __syncthreads();
      prefix |= sel[0] << shift;
      pmask |= 255u << shift;
      before = red[0];
      __syncthreads();
    }
    pthr = prefix;
  }
  if (tid == 0) *thr_out = kthr > pthr ? kthr : pthr;
}

}  // namespace cake

using namespace cake;

// Blocks of an argmax launch: every block ends in ONE atomicMax on the shared slot,
// and those serialise (~11-13 ns each: 512 blocks were ~6 us of a 7 us kernel), so
// the grid stays at 64 blocks and each thread folds ~8 logits.
static inline int argmax_grid(int V) {
  int g = (V + 2047) / 2048;
  return g < 1 ? 1 : (g > 64 ? 64 : g);
}


CAKE_API int cake_sample_threshold(const float* logits, int V, float temperature, int top_k,
                                   float top_p, unsigned int* thr, hipStream_t st) {
  if (V <= 0 || !(temperature > 0.f)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_threshold_kernel, dim3(1), dim3(kSelThreads), 0, st, logits, V,
                     1.f / temperature, top_k, top_p, (const SampleParams*)nullptr, thr);
  return (int)hipGetLastError();
}

// Device-parameter selection (SampleParams in device memory): threshold (a no-op
// write of 0 when greedy / unrestricted) then the Gumbel (or plain) argmax.
CAKE_API int cake_select_dev(const float* logits, int V, const void* params, const int* step,
                             unsigned int* thr, unsigned long long* slot, hipStream_t st) {
  if (V <= 0 || params == nullptr || thr == nullptr) return (int)hipErrorInvalidValue;
  const SampleParams* p = (const SampleParams*)params;
  hipLaunchKernelGGL(sample_threshold_kernel, dim3(1), dim3(kSelThreads), 0, st, logits, V, 1.f,
                     0, 0.f, p, thr);
  const int g = argmax_grid(V);
  hipLaunchKernelGGL(gumbel_argmax_kernel, dim3(g), dim3(256), 0, st, logits, V, 1.f, 0u, 0u,
                     step, (const unsigned int*)thr, p, slot, 0);
  return (int)hipGetLastError();
}

CAKE_API int cake_gumbel_argmax(const float* logits, int V, float temperature,
                                unsigned long long seed, const int* step, const unsigned int* thr,
                                unsigned long long* slot, hipStream_t st) {
  if (V <= 0 || !(temperature > 0.f)) return (int)hipErrorInvalidValue;
  const int g = argmax_grid(V);
  hipLaunchKernelGGL(gumbel_argmax_kernel, dim3(g), dim3(256), 0, st, logits, V,
                     1.f / temperature, (uint32_t)(seed & 0xffffffffull), (uint32_t)(seed >> 32),
                     step, thr, (const SampleParams*)nullptr, slot, 0);
  return (int)hipGetLastError();
}

CAKE_API int cake_repeat_penalty(float* logits, const int* hist, const int* hist_len,
                                 int last_n, float penalty, hipStream_t st) {
  hipLaunchKernelGGL(repeat_penalty_kernel, dim3(1), dim3(256), 0, st, logits, hist, hist_len,
                     last_n, penalty, 0, 0x7fffffff);
  return (int)hipGetLastError();
}

CAKE_API int cake_argmax(const float* logits, int V, unsigned long long* slot,
                         hipStream_t st) {
  hipLaunchKernelGGL(argmax_kernel, dim3(argmax_grid(V)), dim3(256), 0, st, logits, V, slot, 0);
  return (int)hipGetLastError();
}

// Tensor-parallel vocab shard: logits = entries [off, off + V) of the vocabulary.
// Penalty over the shard, then the shard's argmax key (global index) or, with
// temperature > 0, its Gumbel-max key (Philox counter = global index, so the
// all-reduced max equals the single-GPU draw).
CAKE_API int cake_select_shard(float* logits, int V, int off, const int* hist, const int* hist_len,
                               int last_n, float penalty, float temperature,
                               unsigned long long seed, unsigned long long* slot, hipStream_t st) {
  if (V <= 0 || off < 0) return (int)hipErrorInvalidValue;
  if (penalty != 1.f)
    hipLaunchKernelGGL(repeat_penalty_kernel, dim3(1), dim3(256), 0, st, logits, hist, hist_len,
                       last_n, penalty, off, V);
  const int g = argmax_grid(V);
  if (temperature > 0.f)
    hipLaunchKernelGGL(gumbel_argmax_kernel, dim3(g), dim3(256), 0, st, logits, V,
                       1.f / temperature, (uint32_t)(seed & 0xffffffffull), (uint32_t)(seed >> 32),
                       hist_len, (const unsigned int*)nullptr, (const SampleParams*)nullptr, slot,
                       off);
  else
    hipLaunchKernelGGL(argmax_kernel, dim3(argmax_grid(V)), dim3(256), 0, st, logits, V, slot, off);
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
