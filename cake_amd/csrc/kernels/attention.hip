// KV-cached GQA attention (decode split-K + causal prefill).
//
// Replaces the reference's attention core:
//   cake-core/src/models/llama3/attention.rs:89-119  (repeat_kv, f32 upcast,
//   q·kᵀ/√d, causal mask, softmax, ·v, transpose back) and the KV growth of
//   cake-core/src/models/llama3/cache.rs:93-122 (Tensor::cat per step).
//
// MI355X design:
//   * KV lives in a preallocated per-layer cache [nkv][S][hd] (16-bit); the
//     QKV kernel writes the new row in place, so nothing is ever copied.
//   * GQA is handled by indexing: the n_rep query heads that share a kv head
//     are the waves of one workgroup and read the same K/V rows (L1/L2 hits);
//     repeat_kv is never materialised.
//   * Decode is flash-decoding: grid (nkv, S/64) — each workgroup owns 64 keys
//     (one per lane), computes a local softmax and P·V in f32, and writes
//     (max, sum, o[hd]) partials; a combine kernel merges the splits.  The
//     grid is sized for max_seq so the launch is hipGraph-replayable; blocks
//     past the live length exit immediately.
//   * Prefill: one wave per (query row, head) with an online softmax over
//     64-key tiles; the causal limit is offset-aware (pos0 + t), which fixes the
//     reference's index_pos==0-only mask and enables
//     chunked prefill.
#include "common.h"

namespace cake {

constexpr int kKeysPerSplit = 64;

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
template <int DT, int HD>
__global__ void attn_decode_kernel(const float* __restrict__ q,
                                   const uint16_t* __restrict__ kc,
                                   const uint16_t* __restrict__ vc,
                                   const int* __restrict__ pos_ptr, int S, int nkv,
                                   int n_rep, float scale, float* __restrict__ part,
                                   int nsplit) {
  constexpr int DPL = HD / 64;  // output dims per lane
  __shared__ float qs[8 * HD];  // n_rep <= 8
  const int g = blockIdx.x, s = blockIdx.y;
  const int Tk = *pos_ptr + 1;
  const int k0 = s * kKeysPerSplit;
  if (k0 >= Tk) return;
  const int kn = min(kKeysPerSplit, Tk - k0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = g * n_rep + wave;
  for (int i = threadIdx.x; i < n_rep * HD; i += blockDim.x) qs[i] = q[g * n_rep * HD + i];
  __syncthreads();

  const uint16_t* kbase = kc + ((size_t)g * S + k0) * HD;
  const uint16_t* vbase = vc + ((size_t)g * S + k0) * HD;
  const float* qh = qs + wave * HD;

  // scores: lane j <-> key k0 + j
  float sc = -INFINITY;
  if (lane < kn) {
    const uint4* kr = reinterpret_cast<const uint4*>(kbase + (size_t)lane * HD);
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) {
      float kf[8];
      unpack8<DT>(kr[c], kf);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(qh[c * 8 + e], kf[e], acc);
    }
    sc = acc * scale;
  }
  const float m = wave_max(sc);
  const float p = lane < kn ? __expf(sc - m) : 0.f;
  const float l = wave_sum(p);

  // o[d] = sum_j p_j v_j[d]; lane owns dims lane*DPL .. +DPL
  float o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  for (int j = 0; j < kn; ++j) {
    const float pj = __shfl(p, j, 64);
    const uint16_t* vr = vbase + (size_t)j * HD + lane * DPL;
    if constexpr (DPL == 2) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(vr);
      o[0] = fmaf(pj, to_f32<DT>((uint16_t)(w & 0xffff)), o[0]);
      o[1] = fmaf(pj, to_f32<DT>((uint16_t)(w >> 16)), o[1]);
    } else {
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[d] = fmaf(pj, to_f32<DT>(vr[d]), o[d]);
    }
  }
  float* dst = part + ((size_t)h * nsplit + s) * (HD + 2);
  if (lane == 0) { dst[0] = m; dst[1] = l; }
#pragma unroll
  for (int d = 0; d < DPL; ++d) dst[2 + lane * DPL + d] = o[d];
}

template <int DT, int HD>
__global__ void attn_combine_kernel(const float* __restrict__ part,
                                    const int* __restrict__ pos_ptr, int nsplit,
                                    uint16_t* __restrict__ out) {
  constexpr int DPL = HD / 64;
  const int h = blockIdx.x, lane = threadIdx.x;
  const int Tk = *pos_ptr + 1;
  const int ns = (Tk + kKeysPerSplit - 1) / kKeysPerSplit;
  const float* src = part + (size_t)h * nsplit * (HD + 2);
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, src[s * (HD + 2)]);
  float L = 0.f, o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  for (int s = 0; s < ns; ++s) {
    const float* ps = src + s * (HD + 2);
    const float w = __expf(ps[0] - M);
    L = fmaf(w, ps[1], L);
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[d] = fmaf(w, ps[2 + lane * DPL + d], o[d]);
  }
  const float inv = 1.f / L;
#pragma unroll
  for (int d = 0; d < DPL; ++d) out[(size_t)h * HD + lane * DPL + d] = from_f32<DT>(o[d] * inv);
}

// ---------------------------------------------------------------------------
// prefill (T query rows at positions pos0 .. pos0+T-1, causal)
// q: [T, nh, HD] (16-bit, roped); out: [T, nh, HD] (16-bit)
// ---------------------------------------------------------------------------
template <int DT, int HD>
__global__ __launch_bounds__(256) void attn_prefill_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, int pos0, int T, int S, int nh, int nkv,
    float scale, uint16_t* __restrict__ out) {
  constexpr int DPL = HD / 64;
  __shared__ float qs[4 * HD];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.x;
  const int t = blockIdx.y * 4 + wave;
  const int g = h / (nh / nkv);
  const bool active = t < T;
  if (active)
    for (int i = lane; i < HD; i += 64)
      qs[wave * HD + i] = to_f32<DT>(q[((size_t)t * nh + h) * HD + i]);
  __syncthreads();
  if (!active) return;
  const float* qh = qs + wave * HD;
  const int Tk = pos0 + t + 1;
  const uint16_t* kbase = kc + (size_t)g * S * HD;
  const uint16_t* vbase = vc + (size_t)g * S * HD;
  float m = -INFINITY, l = 0.f, o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  for (int k0 = 0; k0 < Tk; k0 += 64) {
    const int kn = min(64, Tk - k0);
    float sc = -INFINITY;
    if (lane < kn) {
      const uint4* kr = reinterpret_cast<const uint4*>(kbase + (size_t)(k0 + lane) * HD);
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < HD / 8; ++c) {
        float kf[8];
        unpack8<DT>(kr[c], kf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(qh[c * 8 + e], kf[e], acc);
      }
      sc = acc * scale;
    }
    const float mt = wave_max(sc);
    const float mn = fmaxf(m, mt);
    const float alpha = __expf(m - mn);  // m=-inf on the first tile -> 0
    const float p = lane < kn ? __expf(sc - mn) : 0.f;
    l = l * alpha + wave_sum(p);
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[d] *= alpha;
    for (int j = 0; j < kn; ++j) {
      const float pj = __shfl(p, j, 64);
      const uint16_t* vr = vbase + (size_t)(k0 + j) * HD + lane * DPL;
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[d] = fmaf(pj, to_f32<DT>(vr[d]), o[d]);
    }
    m = mn;
  }
  const float inv = 1.f / l;
#pragma unroll
  for (int d = 0; d < DPL; ++d)
    out[((size_t)t * nh + h) * HD + lane * DPL + d] = from_f32<DT>(o[d] * inv);
}

}  // namespace cake

using namespace cake;

#define DISPATCH_DT_HD(dt, hd, ...)                                              \
  do {                                                                           \
    if ((dt) == kBF16 && (hd) == 128) { constexpr int DT = kBF16, HD = 128; __VA_ARGS__; } \
    else if ((dt) == kBF16 && (hd) == 64) { constexpr int DT = kBF16, HD = 64; __VA_ARGS__; } \
    else if ((dt) == kF16 && (hd) == 128) { constexpr int DT = kF16, HD = 128; __VA_ARGS__; } \
    else if ((dt) == kF16 && (hd) == 64) { constexpr int DT = kF16, HD = 64; __VA_ARGS__; } \
    else return (int)hipErrorInvalidValue;                                        \
  } while (0)

// part: workspace [nh][nsplit][hd+2] f32, nsplit = ceil(S / 64)
CAKE_API int cake_attn_decode(int dt, const float* q, const void* kc, const void* vc,
                              const int* pos, int S, int nh, int nkv, int hd, float scale,
                              float* part, void* out, hipStream_t st) {
  const int n_rep = nh / nkv;
  if (nh % nkv || n_rep > 8) return (int)hipErrorInvalidValue;
  const int nsplit = (S + kKeysPerSplit - 1) / kKeysPerSplit;
  DISPATCH_DT_HD(dt, hd, {
    hipLaunchKernelGGL((attn_decode_kernel<DT, HD>), dim3(nkv, nsplit), dim3(64 * n_rep), 0,
                       st, q, (const uint16_t*)kc, (const uint16_t*)vc, pos, S, nkv, n_rep,
                       scale, part, nsplit);
    hipLaunchKernelGGL((attn_combine_kernel<DT, HD>), dim3(nh), dim3(64), 0, st, part, pos,
                       nsplit, (uint16_t*)out);
  });
  return (int)hipGetLastError();
}

CAKE_API int cake_attn_prefill(int dt, const void* q, const void* kc, const void* vc,
                               int pos0, int T, int S, int nh, int nkv, int hd, float scale,
                               void* out, hipStream_t st) {
  if (nh % nkv) return (int)hipErrorInvalidValue;
  DISPATCH_DT_HD(dt, hd,
                 hipLaunchKernelGGL((attn_prefill_kernel<DT, HD>), dim3(nh, (T + 3) / 4),
                                    dim3(256), 0, st, (const uint16_t*)q,
                                    (const uint16_t*)kc, (const uint16_t*)vc, pos0, T, S, nh,
                                    nkv, scale, (uint16_t*)out));
  return (int)hipGetLastError();
}
