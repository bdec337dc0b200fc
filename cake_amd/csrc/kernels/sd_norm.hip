// Stable Diffusion normalisation / activation kernels (NCHW activations).
//
// Reference ops (candle-transformers stable_diffusion via cake's UNet/VAE/CLIP
// forwarders):
//   K31/K33 GroupNorm(32) [+ SiLU] in every ResnetBlock2D and the attention
//           blocks' group_norm,
//   K34     LayerNorm in the BasicTransformerBlock / CLIP encoder,
//   K36     GEGLU feed-forward gate (candle: x * gelu_tanh(gate)).
// GroupNorm is two launches so the reduction spreads over the whole chip even
// at batch 2 (B*32 groups would fill only a quarter of the 256 CUs):
//   1. stats:  grid (B*G, S) — each workgroup folds a slice of one group into a
//              Welford (count, mean, M2) partial;
//   2. apply:  grid over the tensor — each workgroup merges its group's S
//              partials (Chan's formula) once, then normalises + affine
//              (+ SiLU) with 16-byte accesses.
#include "common.h"

#include <algorithm>

namespace cake {

constexpr int kGnSplit = 16;

__device__ __forceinline__ void welford_merge(float& n, float& mean, float& m2, float nb,
                                              float meanb, float m2b) {
  if (nb == 0.f) return;
  const float nt = n + nb;
  const float d = meanb - mean;
  mean += d * (nb / nt);
  m2 += m2b + d * d * (n * nb / nt);
  n = nt;
}

template <int DT>
__global__ __launch_bounds__(256) void gn_stats_kernel(const uint16_t* __restrict__ x,
                                                       long long group_elems,
                                                       float* __restrict__ part) {
  const int bg = blockIdx.x, s = blockIdx.y;
  const long long per = (group_elems + kGnSplit - 1) / kGnSplit;
  const long long beg = s * per, end = min(group_elems, beg + per);
  const uint16_t* base = x + (long long)bg * group_elems;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  for (long long i = beg + threadIdx.x; i < end; i += blockDim.x) {
    const float v = to_f32<DT>(base[i]);
    n += 1.f;
    const float d = v - mean;
    mean += d / n;
    m2 += d * (v - mean);
  }
  // wave then block merge
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float nb = __shfl_xor(n, off, 64), mb = __shfl_xor(mean, off, 64),
                qb = __shfl_xor(m2, off, 64);
    welford_merge(n, mean, m2, nb, mb, qb);
  }
  __shared__ float red[4][3];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[w][0] = n; red[w][1] = mean; red[w][2] = m2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) welford_merge(n, mean, m2, red[i][0], red[i][1], red[i][2]);
    float* p = part + ((long long)bg * kGnSplit + s) * 3;
    p[0] = n; p[1] = mean; p[2] = m2;
  }
}

// x, y: [B, C, HW]; gamma/beta [C]
template <int DT, bool SILU>
__global__ __launch_bounds__(256) void gn_apply_kernel(const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ gamma,
                                                       const uint16_t* __restrict__ beta,
                                                       const float* __restrict__ part, int C,
                                                       int G, long long HW, float eps,
                                                       uint16_t* __restrict__ y) {
  // one workgroup covers a contiguous 8*256-element chunk inside ONE group
  const long long group_elems = (long long)(C / G) * HW;
  const long long chunks_per_group = (group_elems + 2047) / 2048;
  const long long bg = blockIdx.x / chunks_per_group;
  const long long chunk = blockIdx.x - bg * chunks_per_group;
  __shared__ float stat[2];
  if (threadIdx.x == 0) {
    float n = 0.f, mean = 0.f, m2 = 0.f;
    const float* p = part + bg * kGnSplit * 3;
    for (int s = 0; s < kGnSplit; ++s) welford_merge(n, mean, m2, p[3 * s], p[3 * s + 1], p[3 * s + 2]);
    stat[0] = mean;
    stat[1] = rsqrtf(m2 / n + eps);
  }
  __syncthreads();
  const float mean = stat[0], rstd = stat[1];
  const int g = (int)(bg % G);
  const long long base = bg * group_elems;
  const long long i0 = chunk * 2048 + threadIdx.x * 8;
  if (i0 >= group_elems) return;
  const bool vec = (HW % 8 == 0) && (i0 + 8 <= group_elems);
  if (vec) {
    float f[8];
    unpack8<DT>(*reinterpret_cast<const uint4*>(x + base + i0), f);
    const int c = g * (C / G) + (int)(i0 / HW);  // 8 elements never straddle a channel
    const float ga = to_f32<DT>(gamma[c]) * rstd, be = to_f32<DT>(beta[c]);
    uint16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = (f[e] - mean) * ga + be;
      if (SILU) v = silu(v);
      o[e] = from_f32<DT>(v);
    }
    *reinterpret_cast<uint4*>(y + base + i0) = *reinterpret_cast<uint4*>(o);
  } else {
    for (long long i = i0; i < min(i0 + 8, group_elems); ++i) {
      const int c = g * (C / G) + (int)(i / HW);
      float v = (to_f32<DT>(x[base + i]) - mean) * rstd * to_f32<DT>(gamma[c]) + to_f32<DT>(beta[c]);
      if (SILU) v = silu(v);
      y[base + i] = from_f32<DT>(v);
    }
  }
}

// LayerNorm over the last dim (rows of C)
template <int DT>
__global__ __launch_bounds__(256) void layernorm_kernel(const uint16_t* __restrict__ x,
                                                        const uint16_t* __restrict__ gamma,
                                                        const uint16_t* __restrict__ beta, int C,
                                                        float eps, uint16_t* __restrict__ y) {
  __shared__ float red[16];
  const uint16_t* xr = x + (long long)blockIdx.x * C;
  uint16_t* yr = y + (long long)blockIdx.x * C;
  float s = 0.f;
  for (int i = threadIdx.x; i < C; i += blockDim.x) s += to_f32<DT>(xr[i]);
  const float mean = block_sum(s, red) / (float)C;
  float q = 0.f;
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    const float d = to_f32<DT>(xr[i]) - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, red) / (float)C + eps);
  for (int i = threadIdx.x; i < C; i += blockDim.x)
    yr[i] = from_f32<DT>((to_f32<DT>(xr[i]) - mean) * rstd * to_f32<DT>(gamma[i]) +
                         to_f32<DT>(beta[i]));
}

// h [rows, 2F] -> out [rows, F] = h[:, :F] * gelu_tanh(h[:, F:])
template <int DT>
__global__ void geglu_kernel(const uint16_t* __restrict__ h, long long rows, int F,
                             uint16_t* __restrict__ out) {
  const long long n = rows * F;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / F;
    const int c = (int)(i - r * F);
    const float a = to_f32<DT>(h[r * 2 * F + c]), g = to_f32<DT>(h[r * 2 * F + F + c]);
    out[i] = from_f32<DT>(a * gelu_tanh(g));
  }
}

// LayerNorm, one wave per row, 16-byte accesses, the row held in registers
// (exact two-pass mean / variance from one read).  C % 8 == 0, C <= 512*CPL.
template <int DT, int CPL>
__global__ __launch_bounds__(256) void layernorm_wave_kernel(const uint16_t* __restrict__ x,
                                                             const uint16_t* __restrict__ gamma,
                                                             const uint16_t* __restrict__ beta,
                                                             long long rows, int C, float eps,
                                                             uint16_t* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = C >> 3;
  const uint16_t* xr = x + row * C;
  float v[CPL][8];
  float s = 0.f;
  // gamma / beta requested with the row: loaded after the two reductions they put a
  // further memory round trip on every row's critical path
  uint4 gq[CPL], bq[CPL];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      gq[i] = *reinterpret_cast<const uint4*>(gamma + c * 8);
      bq[i] = *reinterpret_cast<const uint4*>(beta + c * 8);
    }
  }
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      unpack8<DT>(*reinterpret_cast<const uint4*>(xr + c * 8), v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
    if (lane + 64 * i < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[i][e] - mean;
        q += d * d;
      }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c >= nch) continue;
    float g[8], b[8];
    unpack8<DT>(gq[i], g);
    unpack8<DT>(bq[i], b);
    uint16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f32<DT>((v[i][e] - mean) * rstd * g[e] + b[e]);
    *reinterpret_cast<uint4*>(y + row * C + c * 8) = *reinterpret_cast<uint4*>(o);
  }
}

// GEGLU with 16-byte accesses: F % 8 == 0
template <int DT>
__global__ __launch_bounds__(256) void geglu_vec_kernel(const uint16_t* __restrict__ h,
                                                        long long rows, int F,
                                                        uint16_t* __restrict__ out) {
  const int fv = F >> 3;
  const long long n = rows * fv;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / fv;
    const int c = (int)(i - r * fv) * 8;
    float a[8], g[8];
    unpack8<DT>(*reinterpret_cast<const uint4*>(h + r * 2 * F + c), a);
    unpack8<DT>(*reinterpret_cast<const uint4*>(h + r * 2 * F + F + c), g);
    uint16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f32<DT>(a[e] * gelu_tanh(g[e]));
    *reinterpret_cast<uint4*>(out + r * F + c) = *reinterpret_cast<uint4*>(o);
  }
}

// ---------------------------------------------------------------------------
// GroupNorm on channels-last activations x [N, HW, C] (the layout the MFMA
// convolutions and the transformer blocks share, so no NCHW<->NHWC copies).
// 1. stats: grid (S, N), block (C/8 channel vectors) x (pixel lanes).  Every
//    thread owns 8 fixed channels (<= 2 groups) and accumulates sum / sum^2 in
//    f64 over its pixels; the block folds them per group and writes a f64
//    partial.  The last block of image n (agent-scope ticket, CDNA guide
//    Guideline 16) folds the S partials into (mean, rstd) per group and
//    re-arms the ticket, so the launch replays unchanged in a hipGraph.
// 2. apply: per-channel scale/shift for image n in LDS, then one fma (+SiLU)
//    per element with 16-byte accesses.
// ---------------------------------------------------------------------------
constexpr int kGnMaxC = 4096;

// Two-source input (the UNet up path's skip concatenation, never materialised
// by a separate copy): channels [0, Cx) come from x [N, HW, Cx], channels
// [Cx, C) from x2 [N, HW, C - Cx]; Cx == C is the plain one-source case.
struct GnSrc {
  const uint16_t* x;
  const uint16_t* x2;
  int Cx;
  // 8 channels starting at c (c % 8 == 0, Cx % 8 == 0) of pixel p of image n
  __device__ __forceinline__ const uint16_t* at(int n, int HW, int C, size_t p, int c) const {
    return c < Cx ? x + ((size_t)n * HW + p) * Cx + c
                  : x2 + ((size_t)n * HW + p) * (C - Cx) + (c - Cx);
  }
};

template <int DT>
__global__ __launch_bounds__(512) void gn_nhwc_stats_kernel(GnSrc src, int HW,
                                                            int C, int G, double* __restrict__ part,
                                                            unsigned int* __restrict__ tickets,
                                                            float* __restrict__ stats) {
  const int Tx = C >> 3, Ty = blockDim.x / Tx;
  const int cv = threadIdx.x % Tx, py = threadIdx.x / Tx;
  const int n = blockIdx.y, S = gridDim.x, sp = blockIdx.x;
  const int Cg = C / G;
  const int g0 = (cv * 8) / Cg;
  const int per = (HW + S - 1) / S, p0 = sp * per, p1 = min(HW, p0 + per);
  double s0 = 0.0, q0 = 0.0, s1 = 0.0, q1 = 0.0;
  if (py < Ty) {
    const uint16_t* base = src.at(n, HW, C, 0, cv * 8);
    const int ld = cv * 8 < src.Cx ? src.Cx : C - src.Cx;
    // all (up to 8) of this thread's pixel vectors requested before any is consumed: one
    // memory round trip per 8 pixels instead of per pixel
    constexpr int U = 8;
    for (int p = p0 + py; p < p1; p += U * Ty) {
      uint4 raw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int pp = p + u * Ty;
        raw[u] = pp < p1 ? *reinterpret_cast<const uint4*>(base + (size_t)pp * ld)
                         : make_uint4(0, 0, 0, 0);
      }
      float a0 = 0.f, b0 = 0.f, a1 = 0.f, b1 = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float f[8];
        unpack8<DT>(raw[u], f);  // zero vectors past p1 add nothing
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if ((cv * 8 + e) / Cg == g0) { a0 += f[e]; b0 += f[e] * f[e]; }
          else { a1 += f[e]; b1 += f[e] * f[e]; }
        }
      }
      s0 += a0; q0 += b0; s1 += a1; q1 += b1;
    }
  }
  __shared__ double red[512 * 4];
  __shared__ int last;
  red[threadIdx.x * 4 + 0] = s0; red[threadIdx.x * 4 + 1] = q0;
  red[threadIdx.x * 4 + 2] = s1; red[threadIdx.x * 4 + 3] = q1;
  __syncthreads();
  double* pn = part + ((size_t)n * S + sp) * G * 2;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    double ts = 0.0, tq = 0.0;
    const int vlo = (g * Cg) / 8, vhi = ((g + 1) * Cg - 1) / 8;
    for (int v = vlo; v <= vhi; ++v) {
      const int slot = ((v * 8) / Cg == g) ? 0 : 2;
      for (int y = 0; y < Ty; ++y) {
        ts += red[(y * Tx + v) * 4 + slot];
        tq += red[(y * Tx + v) * 4 + slot + 1];
      }
    }
    pn[2 * g] = ts;
    pn[2 * g + 1] = tq;
  }
  // publish partial; the last block of image n folds all S of them
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&tickets[n], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (unsigned)(S - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tickets[n] = 0u;
    }
  }
  __syncthreads();
  if (!last) return;
  // fold the S partials with every thread: (group, slice) lanes, then LDS
  const int nthr = blockDim.x, lpg = nthr / G;
  {
    const int g = threadIdx.x % G, sl = threadIdx.x / G;
    double ts = 0.0, tq = 0.0;
    if (sl < lpg) {
      // 8 partials requested per round trip (a serial chain of S / lpg loads was the
      // tail of the whole launch)
      constexpr int U = 8;
      for (int k = sl; k < S; k += U * lpg) {
        double ps[U], pq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int kk = k + u * lpg;
          const double* q = part + ((size_t)n * S + (kk < S ? kk : 0)) * G * 2 + 2 * g;
          ps[u] = kk < S ? __builtin_nontemporal_load(q) : 0.0;
          pq[u] = kk < S ? __builtin_nontemporal_load(q + 1) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          ts += ps[u];
          tq += pq[u];
        }
      }
    }
    red[threadIdx.x * 2] = ts;
    red[threadIdx.x * 2 + 1] = tq;
  }
  __syncthreads();
  if (threadIdx.x < G) {
    const int g = threadIdx.x;
    double ts = 0.0, tq = 0.0;
    for (int sl = 0; sl < lpg; ++sl) {
      ts += red[(sl * G + g) * 2];
      tq += red[(sl * G + g) * 2 + 1];
    }
    const double cnt = (double)HW * Cg;
    const double mean = ts / cnt;
    const double var = fmax(tq / cnt - mean * mean, 0.0);
    stats[((size_t)n * G + g) * 2] = (float)mean;
    stats[((size_t)n * G + g) * 2 + 1] = (float)var;
  }
}

// cat (optional): the raw two-source input written out as one [N, HW, C]
// tensor for the consumers that need it unnormalised (the resnet's 1x1 shortcut)
template <int DT, bool SILU>
__global__ __launch_bounds__(256) void gn_nhwc_apply_kernel(GnSrc src,
                                                            const uint16_t* __restrict__ gamma,
                                                            const uint16_t* __restrict__ beta,
                                                            const float* __restrict__ stats,
                                                            int HW, int C, int G, float eps,
                                                            uint16_t* __restrict__ y,
                                                            uint16_t* __restrict__ cat) {
  __shared__ float sc[kGnMaxC], sh[kGnMaxC];
  const int n = blockIdx.y, Cg = C / G;
  const size_t nv = (size_t)HW * (C >> 3);
  const size_t base = (size_t)n * HW * C;
  const size_t vstep = (size_t)gridDim.x * blockDim.x;
  auto load = [&](size_t v) {
    return *reinterpret_cast<const uint4*>(src.at(n, HW, C, v / (C >> 3), (int)(v % (C >> 3)) * 8));
  };
  // the first vector is requested before the scale / shift table is built (its stats /
  // gamma / beta reads and the barrier overlap the load), then one vector ahead
  size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 nxt = make_uint4(0, 0, 0, 0);
  if (v < nv) nxt = load(v);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int g = c / Cg;
    const float mean = stats[((size_t)n * G + g) * 2];
    const float rstd = rsqrtf(stats[((size_t)n * G + g) * 2 + 1] + eps);
    const float a = rstd * to_f32<DT>(gamma[c]);
    sc[c] = a;
    sh[c] = to_f32<DT>(beta[c]) - mean * a;
  }
  __syncthreads();
  for (; v < nv; v += vstep) {
    const int c0 = (int)(v % (C >> 3)) * 8;
    const uint4 raw = nxt;
    if (v + vstep < nv) nxt = load(v + vstep);
    if (cat != nullptr) *reinterpret_cast<uint4*>(cat + base + v * 8) = raw;
    float f[8];
    unpack8<DT>(raw, f);
    uint16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = fmaf(f[e], sc[c0 + e], sh[c0 + e]);
      if (SILU) t = silu(t);
      o[e] = from_f32<DT>(t);
    }
    *reinterpret_cast<uint4*>(y + base + v * 8) = *reinterpret_cast<uint4*>(o);
  }
}

}  // namespace cake

using namespace cake;

#define DISPATCH_DT(dt, ...)                       \
  do {                                             \
    if ((dt) == kBF16) { constexpr int DT = kBF16; __VA_ARGS__; } \
    else if ((dt) == kF16) { constexpr int DT = kF16; __VA_ARGS__; } \
    else return (int)hipErrorInvalidValue;         \
  } while (0)

// part: workspace of B*G*16*3 floats
CAKE_API int cake_groupnorm(int dt, const void* x, const void* gamma, const void* beta, int B,
                            int C, long long HW, int G, float eps, int silu_act, float* part,
                            void* y, hipStream_t st) {
  if (C % G) return (int)hipErrorInvalidValue;
  const long long ge = (long long)(C / G) * HW;
  const long long chunks = (ge + 2047) / 2048;
  const long long nblk = (long long)B * G * chunks;
  if (nblk > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  DISPATCH_DT(dt, {
    hipLaunchKernelGGL((gn_stats_kernel<DT>), dim3(B * G, kGnSplit), dim3(256), 0, st,
                       (const uint16_t*)x, ge, part);
    if (silu_act)
      hipLaunchKernelGGL((gn_apply_kernel<DT, true>), dim3((unsigned)nblk), dim3(256), 0, st,
                         (const uint16_t*)x, (const uint16_t*)gamma, (const uint16_t*)beta, part, C,
                         G, HW, eps, (uint16_t*)y);
    else
      hipLaunchKernelGGL((gn_apply_kernel<DT, false>), dim3((unsigned)nblk), dim3(256), 0, st,
                         (const uint16_t*)x, (const uint16_t*)gamma, (const uint16_t*)beta, part, C,
                         G, HW, eps, (uint16_t*)y);
  });
  return (int)hipGetLastError();
}

CAKE_API int cake_layernorm(int dt, const void* x, const void* gamma, const void* beta,
                            long long rows, int C, float eps, void* y, hipStream_t st) {
  if (rows > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const bool al = ((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) % 16 == 0;
  if (C % 8 == 0 && C <= 2048 && al) {
    const unsigned g = (unsigned)((rows + 3) / 4);
    if (C <= 512)
      DISPATCH_DT(dt, hipLaunchKernelGGL((layernorm_wave_kernel<DT, 1>), dim3(g), dim3(256), 0, st,
                                         (const uint16_t*)x, (const uint16_t*)gamma,
                                         (const uint16_t*)beta, rows, C, eps, (uint16_t*)y));
    else if (C <= 1024)
      DISPATCH_DT(dt, hipLaunchKernelGGL((layernorm_wave_kernel<DT, 2>), dim3(g), dim3(256), 0, st,
                                         (const uint16_t*)x, (const uint16_t*)gamma,
                                         (const uint16_t*)beta, rows, C, eps, (uint16_t*)y));
    else
      DISPATCH_DT(dt, hipLaunchKernelGGL((layernorm_wave_kernel<DT, 4>), dim3(g), dim3(256), 0, st,
                                         (const uint16_t*)x, (const uint16_t*)gamma,
                                         (const uint16_t*)beta, rows, C, eps, (uint16_t*)y));
    return (int)hipGetLastError();
  }
  DISPATCH_DT(dt, hipLaunchKernelGGL((layernorm_kernel<DT>), dim3((unsigned)rows), dim3(256), 0,
                                     st, (const uint16_t*)x, (const uint16_t*)gamma,
                                     (const uint16_t*)beta, C, eps, (uint16_t*)y));
  return (int)hipGetLastError();
}

CAKE_API int cake_geglu(int dt, const void* h, long long rows, int F, void* out, hipStream_t st) {
  const bool al = ((uintptr_t)h | (uintptr_t)out) % 16 == 0;
  if (F % 8 == 0 && al) {
    const long long n = rows * (F / 8);
    const long long g = std::min<long long>((n + 255) / 256, 16384);
    DISPATCH_DT(dt, hipLaunchKernelGGL((geglu_vec_kernel<DT>), dim3((unsigned)g), dim3(256), 0, st,
                                       (const uint16_t*)h, rows, F, (uint16_t*)out));
    return (int)hipGetLastError();
  }
  long long n = rows * F;
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  DISPATCH_DT(dt, hipLaunchKernelGGL((geglu_kernel<DT>), dim3((unsigned)g), dim3(256), 0, st,
                                     (const uint16_t*)h, rows, F, (uint16_t*)out));
  return (int)hipGetLastError();
}

// Channels-last GroupNorm.  part: N*S*G*2 f64 (S = cake_groupnorm_nhwc_splits),
// tickets: N u32 zeroed once (re-armed by the kernel), stats: N*G*2 f32.
CAKE_API int cake_groupnorm_nhwc_splits(int HW) {
  const int s = HW / 16;  // >= 16 pixels per workgroup, <= 256 partials per image
  return s < 1 ? 1 : (s > 256 ? 256 : s);
}

// Two-source form: x [N, HW, Cx] ++ x2 [N, HW, C - Cx] along channels (x2 null
// when Cx == C); cat (optional) receives the concatenated raw input.
CAKE_API int cake_groupnorm_nhwc2(int dt, const void* x, const void* x2, int Cx, void* cat,
                                  const void* gamma, const void* beta, int N, int HW, int C, int G,
                                  float eps, int silu_act, double* part, unsigned int* tickets,
                                  float* stats, void* y, hipStream_t st) {
  if (C % G || C % 8 || C > kGnMaxC || C / 8 > 512 || N <= 0 || HW <= 0 || (C / G) < 1 || G > 256)
    return (int)hipErrorInvalidValue;
  if (Cx <= 0 || Cx > C || Cx % 8 || (Cx < C && x2 == nullptr)) return (int)hipErrorInvalidValue;
  // every 8-channel vector must span at most two groups
  if ((C / G) < 8 && 8 % (C / G)) return (int)hipErrorInvalidValue;
  if ((C / G) < 4) return (int)hipErrorInvalidValue;
  const int Tx = C / 8, Ty = Tx >= 512 ? 1 : 512 / Tx;
  const int S = cake_groupnorm_nhwc_splits(HW);
  const size_t nv = (size_t)HW * (C / 8);
  const unsigned ab = (unsigned)std::min<size_t>((nv + 255) / 256, 1024);
  const GnSrc src{(const uint16_t*)x, (const uint16_t*)x2, Cx};
  DISPATCH_DT(dt, {
    hipLaunchKernelGGL((gn_nhwc_stats_kernel<DT>), dim3(S, N), dim3(Tx * Ty), 0, st, src, HW, C,
                       G, part, tickets, stats);
    if (silu_act)
      hipLaunchKernelGGL((gn_nhwc_apply_kernel<DT, true>), dim3(ab, N), dim3(256), 0, st, src,
                         (const uint16_t*)gamma, (const uint16_t*)beta, stats, HW, C, G, eps,
                         (uint16_t*)y, (uint16_t*)cat);
    else
      hipLaunchKernelGGL((gn_nhwc_apply_kernel<DT, false>), dim3(ab, N), dim3(256), 0, st, src,
                         (const uint16_t*)gamma, (const uint16_t*)beta, stats, HW, C, G, eps,
                         (uint16_t*)y, (uint16_t*)cat);
  });
  return (int)hipGetLastError();
}

CAKE_API int cake_groupnorm_nhwc(int dt, const void* x, const void* gamma, const void* beta, int N,
                                 int HW, int C, int G, float eps, int silu_act, double* part,
                                 unsigned int* tickets, float* stats, void* y, hipStream_t st) {
  return cake_groupnorm_nhwc2(dt, x, nullptr, C, nullptr, gamma, beta, N, HW, C, G, eps, silu_act,
                              part, tickets, stats, y, st);
}
