// Flash attention for head_dim 512: the AutoencoderKL mid-block self-attention
// (one head over all C = 512 channels; candle-transformers VAE AttentionBlock,
// reached from cake-core/src/models/sd/vae.rs:55-61).
//
//   O = softmax(Q K^T * scale) V,   Q [B][N][512], K/V [B][M][512] (16-bit),
//   N = M = latent pixels (4096 at 512^2, 16384 at 1024^2).
//
// The f32 score matrix never exists (N x M x 4 B = 1 GiB at 1024^2): one pass
// over the keys with an online softmax, as in flash_attn.hip, but with a
// geometry for D = 512 on MFMA 16x16x32:
//   * workgroup = 64 query rows, 4 waves x 16 rows; each wave keeps its Q rows
//     as MFMA A-fragments in registers for the whole kernel (16 x 16 B / lane)
//     and owns a 16 x 512 f32 output accumulator (32 MFMA tiles, 128 VGPRs);
//   * per 32-key step: K tile [32][512] staged by LDS-DMA (16-byte slots XOR-
//     swizzled by key on the source address: conflict-free fragment reads),
//     V staged transposed [512][32] through registers (4 keys x 8 dims per
//     thread, 8-byte LDS writes, slot-swizzled), S = Q K^T (2 x 16 MFMAs per
//     wave), row max / sum by 16-lane shuffles, P -> bf16 through a padded LDS
//     tile into an A-fragment, O += P V (32 MFMAs).
#include "common.h"

namespace cake {

constexpr int kD512 = 512;
constexpr int kBQ = 64, kBK = 32;

template <int DT>
__device__ __forceinline__ uint16_t cvt16(float f) { return from_f32<DT>(f); }

template <int DT>
__global__ __launch_bounds__(256) void attn512_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
    const uint16_t* __restrict__ V, uint16_t* __restrict__ O, int N, int M, long long sq,
    long long sk, long long sv, long long so, long long bq, long long bk, long long bv,
    long long bo, float scale_log2, const uint16_t* __restrict__ zeros) {
  constexpr int D = kD512;
  constexpr int PROW = 40;  // P tile row stride (bf16): 80 B rows -> conflict-free A reads
  // one LDS array: K [32][512] | Vt [512][32] | P [4 waves][16][PROW]
  __shared__ __attribute__((aligned(16))) uint16_t smem[kBK * D + D * kBK + 4 * 16 * PROW];
  uint16_t* Ks = smem;
  uint16_t* Vt = smem + kBK * D;
  uint16_t* Ps = Vt + D * kBK;

  const int b = blockIdx.y;
  const int q0 = blockIdx.x * kBQ;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lh = lane >> 4;
  Q += (size_t)b * bq;
  K += (size_t)b * bk;
  V += (size_t)b * bv;
  O += (size_t)b * bo;

  // Q A-fragments: row q0 + 16 wave + lr, dims 32 ks + 8 lh .. +8
  uint4 qa[16];
  {
    const int row = q0 + wave * 16 + lr;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      qa[ks] = row < N ? *reinterpret_cast<const uint4*>(Q + (size_t)row * sq + ks * 32 + lh * 8)
                       : make_uint4(0u, 0u, 0u, 0u);
  }
  cf32x4 acc[32];
#pragma unroll
  for (int t = 0; t < 32; ++t) acc[t] = cf32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) { mrow[e] = -INFINITY; lrow[e] = 0.f; }

  for (int k0 = 0; k0 < M; k0 += kBK) {
    __syncthreads();  // previous step's K / Vt / P fully consumed
    // ---- K tile: one DMA wave-instruction per key row (1 KiB), 8 per wave ----
#pragma unroll
    for (int i = 0; i < kBK / 4; ++i) {
      const int r = wave * (kBK / 4) + i;
      const int key = k0 + r;
      const uint16_t* src = key < M ? K + (size_t)key * sk + ((lane ^ (r & 15)) * 8) : zeros;
      glds16(src, Ks + r * D);
    }
    // ---- V tile transposed: thread unit = 4 keys x 8 dims ----------------
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int unit = tid + u * 256;
      const int kg = unit >> 6, dc = unit & 63;  // key group (4 keys), 8-dim chunk
      uint4 rows[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = k0 + kg * 4 + j;
        rows[j] = key < M ? *reinterpret_cast<const uint4*>(V + (size_t)key * sv + dc * 8)
                          : make_uint4(0u, 0u, 0u, 0u);
      }
      const uint32_t* w0 = reinterpret_cast<const uint32_t*>(&rows[0]);
      const uint32_t* w1 = reinterpret_cast<const uint32_t*>(&rows[1]);
      const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&rows[2]);
      const uint32_t* w3 = reinterpret_cast<const uint32_t*>(&rows[3]);
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const int sh = (d & 1) * 16;
        const uint32_t a = ((w0[d >> 1] >> sh) & 0xffffu) | (((w1[d >> 1] >> sh) & 0xffffu) << 16);
        const uint32_t c = ((w2[d >> 1] >> sh) & 0xffffu) | (((w3[d >> 1] >> sh) & 0xffffu) << 16);
        const int n = dc * 8 + d;  // dim row of Vt (64 B = 4 slots of 8 keys)
        const int slot = (kg >> 1) ^ ((n >> 2) & 3);
        *reinterpret_cast<uint2*>(Vt + n * kBK + slot * 8 + (kg & 1) * 4) = make_uint2(a, c);
      }
    }
    __builtin_amdgcn_s_waitcnt(vm_wait(0));
    __syncthreads();

    // ---- S = Q K^T for this wave's 16 rows x 32 keys --------------------
    cf32x4 s[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      s[c] = cf32x4{0.f, 0.f, 0.f, 0.f};
      const int kr = c * 16 + lr;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        const int slot = (ks * 4 + lh) ^ (kr & 15);
        const uint4 kb = *reinterpret_cast<const uint4*>(Ks + kr * D + slot * 8);
        s[c] = cmfma<DT>(qa[ks], kb, s[c]);
      }
    }
    // ---- online softmax over the 32 keys (rows 4 lh + e, key column lr) --
    float p[2][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mx = -INFINITY;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float v = (k0 + c * 16 + lr < M) ? s[c][e] * scale_log2 : -INFINITY;
        p[c][e] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mn = fmaxf(mrow[e], mx);
      const float alpha = exp2f(mrow[e] - mn);
      float sum = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        p[c][e] = exp2f(p[c][e] - mn);
        sum += p[c][e];
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
      lrow[e] = lrow[e] * alpha + sum;
      mrow[e] = mn;
#pragma unroll
      for (int t = 0; t < 32; ++t) acc[t][e] *= alpha;
    }
    // ---- P (C layout) -> bf16 A-fragment through this wave's LDS tile ------
    uint16_t* pw = Ps + wave * 16 * PROW;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) pw[(lh * 4 + e) * PROW + c * 16 + lr] = cvt16<DT>(p[c][e]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const uint4 pa = *reinterpret_cast<const uint4*>(pw + lr * PROW + lh * 8);
    // ---- O += P V: B-fragment = Vt[dim 16 t + lr][keys 8 lh .. +8] ----------
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      const int n = t * 16 + lr;
      const int slot = lh ^ ((n >> 2) & 3);
      const uint4 vb = *reinterpret_cast<const uint4*>(Vt + n * kBK + slot * 8);
      acc[t] = cmfma<DT>(pa, vb, acc[t]);
    }
  }

  // ---- normalise and store: rows 4 lh + e, dims 16 t + lr ----------------
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = q0 + wave * 16 + lh * 4 + e;
    if (row >= N) continue;
    const float inv = 1.f / lrow[e];
    uint16_t* dst = O + (size_t)row * so;
#pragma unroll
    for (int t = 0; t < 32; ++t) dst[t * 16 + lr] = cvt16<DT>(acc[t][e] * inv);
  }
}

}  // namespace cake

using namespace cake;

// q/k/v/o: [B][rows][512] with row strides s* and batch strides b* (elements).
CAKE_API int cake_attn512(int dt, const void* q, const void* k, const void* v, void* o, int B,
                          int N, int M, long long sq, long long sk, long long sv, long long so,
                          long long bq, long long bk, long long bv, long long bo, float scale,
                          const void* zeros, hipStream_t st) {
  if (B <= 0 || N <= 0 || M <= 0 || (sq | sk | sv) % 8) return (int)hipErrorInvalidValue;
  const dim3 grid((N + kBQ - 1) / kBQ, B);
  const float sl2 = scale * 1.4426950408889634f;
  if (dt == kBF16)
    hipLaunchKernelGGL((attn512_kernel<kBF16>), grid, dim3(256), 0, st, (const uint16_t*)q,
                       (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, N, M, sq, sk, sv, so,
                       bq, bk, bv, bo, sl2, (const uint16_t*)zeros);
  else if (dt == kF16)
    hipLaunchKernelGGL((attn512_kernel<kF16>), grid, dim3(256), 0, st, (const uint16_t*)q,
                       (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, N, M, sq, sk, sv, so,
                       bq, bk, bv, bo, sl2, (const uint16_t*)zeros);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
