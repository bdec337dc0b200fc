// Row-wise and elementwise kernels: embedding gather, RMSNorm, RoPE + KV-cache
// write for multi-token (prefill) steps, SwiGLU, residual add.
//
// Reference ops replaced:
//   K01 embedding index_select   cake-core/src/models/llama3/llama.rs:74
//   K02 RmsNorm                  cake-core/src/models/llama3/transformer.rs:60,68
//   K05 rope (non-interleaved)   cake-core/src/models/llama3/attention.rs:25-35
//   K06 kv cat                   cake-core/src/models/llama3/cache.rs:93-122
//   K15 silu * up                cake-core/src/models/llama3/mlp.rs:16
// Decode never uses these (the GEMV prologues/epilogues fuse them); prefill
// runs GEMMs on MFMA and uses these for the glue.
#include "common.h"

namespace cake {

template <int DT>
__global__ void embed_kernel(const uint16_t* __restrict__ table, const int* __restrict__ tok,
                             int H, float* __restrict__ out) {
  const int t = blockIdx.x;
  const uint16_t* row = table + (size_t)tok[t] * H;
  float* o = out + (size_t)t * H;
  for (int i = threadIdx.x * 8; i < H; i += blockDim.x * 8) {
    float f[8];
    unpack8<DT>(*reinterpret_cast<const uint4*>(row + i), f);
    *reinterpret_cast<float4*>(o + i) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(o + i + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
}

// out[t] = x[t] * rsqrt(mean(x[t]^2) + eps) * w  (x f32, out 16-bit)
template <int DT>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const float* __restrict__ x,
                                                      const uint16_t* __restrict__ w,
                                                      float eps, int H,
                                                      uint16_t* __restrict__ out) {
  __shared__ float red[16];
  const float* xr = x + (size_t)blockIdx.x * H;
  float ss = 0.f;
  for (int i = threadIdx.x * 4; i < H; i += blockDim.x * 4) {
    const float4 v = *reinterpret_cast<const float4*>(xr + i);
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = block_sum(ss, red);
  const float r = rsqrtf(ss / (float)H + eps);
  uint16_t* o = out + (size_t)blockIdx.x * H;
  for (int i = threadIdx.x * 4; i < H; i += blockDim.x * 4) {
    const float4 v = *reinterpret_cast<const float4*>(xr + i);
    const uint2 wv = *reinterpret_cast<const uint2*>(w + i);
    uint2 ov;
    ov.x = (uint32_t)from_f32<DT>(v.x * r * to_f32<DT>((uint16_t)(wv.x & 0xffff))) |
           ((uint32_t)from_f32<DT>(v.y * r * to_f32<DT>((uint16_t)(wv.x >> 16))) << 16);
    ov.y = (uint32_t)from_f32<DT>(v.z * r * to_f32<DT>((uint16_t)(wv.y & 0xffff))) |
           ((uint32_t)from_f32<DT>(v.w * r * to_f32<DT>((uint16_t)(wv.y >> 16))) << 16);
    *reinterpret_cast<uint2*>(o + i) = ov;
  }
}

// The same for H <= 1024 * NV: the row's x and w slices are loaded once, all up front,
// into registers (one round of load latency instead of a dependent chain per 1024
// columns and a second pass over x)
template <int DT, int NV>
__global__ __launch_bounds__(256) void rmsnorm_reg_kernel(const float* __restrict__ x,
                                                          const uint16_t* __restrict__ w,
                                                          float eps, int H,
                                                          uint16_t* __restrict__ out) {
  __shared__ float red[16];
  const float* xr = x + (size_t)blockIdx.x * H;
  float4 v[NV];
  uint2 wv[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i = (threadIdx.x + j * 256) * 4;
    if (i < H) {
      v[j] = *reinterpret_cast<const float4*>(xr + i);
      wv[j] = *reinterpret_cast<const uint2*>(w + i);
    } else {
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      wv[j] = make_uint2(0u, 0u);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
    ss += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
  ss = block_sum(ss, red);
  const float r = rsqrtf(ss / (float)H + eps);
  uint16_t* o = out + (size_t)blockIdx.x * H;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i = (threadIdx.x + j * 256) * 4;
    if (i >= H) continue;
    uint2 ov;
    ov.x = (uint32_t)from_f32<DT>(v[j].x * r * to_f32<DT>((uint16_t)(wv[j].x & 0xffff))) |
           ((uint32_t)from_f32<DT>(v[j].y * r * to_f32<DT>((uint16_t)(wv[j].x >> 16))) << 16);
    ov.y = (uint32_t)from_f32<DT>(v[j].z * r * to_f32<DT>((uint16_t)(wv[j].y & 0xffff))) |
           ((uint32_t)from_f32<DT>(v[j].w * r * to_f32<DT>((uint16_t)(wv[j].y >> 16))) << 16);
    *reinterpret_cast<uint2*>(o + i) = ov;
  }
}

// Prefill RoPE: q [T, nh*hd] roped in place; k roped and v copied into the
// cache rows pos0+t of [nkv][S][hd].
template <int DT>
__global__ void rope_kv_kernel(uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                               const uint16_t* __restrict__ v, int ldq, int ld, int nh, int nkv,
                               int hd,
                               const float* __restrict__ inv_freq, int pos0, int S,
                               uint16_t* __restrict__ kc, uint16_t* __restrict__ vc) {
  const int t = blockIdx.x, pos = pos0 + t, half = hd >> 1;
  const int nq = nh * half, nk = nkv * half;
  for (int p = threadIdx.x; p < nq + 2 * nk; p += blockDim.x) {
    if (p < nq + nk) {
      const bool isq = p < nq;
      const int pp = isq ? p : p - nq;
      const int head = pp / half, i = pp - head * half;
      float s, c;
      sincosf((float)pos * inv_freq[i], &s, &c);
      const uint16_t* src = isq ? q + (size_t)t * ldq : k + (size_t)t * ld;
      const float a = to_f32<DT>(src[head * hd + i]);
      const float b = to_f32<DT>(src[head * hd + i + half]);
      const uint16_t oa = from_f32<DT>(a * c - b * s), ob = from_f32<DT>(a * s + b * c);
      if (isq) {
        q[(size_t)t * ldq + head * hd + i] = oa;
        q[(size_t)t * ldq + head * hd + i + half] = ob;
      } else {
        const size_t off = ((size_t)head * S + pos) * hd + i;
        kc[off] = oa;
        kc[off + half] = ob;
      }
    } else {
      const int pp = p - nq - nk;
      const int head = pp / half, i = pp - head * half;
      const size_t off = ((size_t)head * S + pos) * hd + i;
      const uint16_t* src = v + (size_t)t * ld + head * hd;
      vc[off] = src[i];
      vc[off + half] = src[i + half];
    }
  }
}

// Same, 8 elements per item with 16-byte accesses (hd % 16 == 0, 16-byte aligned rows and
// bases): per token, nh + nkv rope items of half/8 vectors each (the a / b halves of a
// head loaded and stored as whole 16-byte rows), then nkv * hd/8 V copies.  The scalar
// form moved 2-byte elements one pair per thread per iteration (18 us per 2048-token
// layer of 8B prefill).
template <int DT>
__global__ __launch_bounds__(256) void rope_kv_vec_kernel(
    uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    int ldq, int ld, int nh, int nkv, int hd, const float* __restrict__ inv_freq, int pos0, int S,
    uint16_t* __restrict__ kc, uint16_t* __restrict__ vc) {
  const int t = blockIdx.x, pos = pos0 + t, half = hd >> 1, hv = half >> 3;
  const int nrope = (nh + nkv) * hv, nv = nkv * (hd >> 3);
  // the token's rotation angles once (shared by its nh + nkv heads), not per head
  __shared__ float s_sn[128], s_cs[128];
  for (int i = threadIdx.x; i < half; i += blockDim.x) sincosf((float)pos * inv_freq[i], &s_sn[i], &s_cs[i]);
  __syncthreads();
  for (int p = threadIdx.x; p < nrope + nv; p += blockDim.x) {
    if (p < nrope) {
      const int head = p / hv, i0 = (p - head * hv) * 8;
      const bool isq = head < nh;
      const int hh = isq ? head : head - nh;
      const uint16_t* src = isq ? q + (size_t)t * ldq + hh * hd : k + (size_t)t * ld + hh * hd;
      float a[8], b[8];
      unpack8<DT>(*reinterpret_cast<const uint4*>(src + i0), a);
      unpack8<DT>(*reinterpret_cast<const uint4*>(src + i0 + half), b);
      uint16_t oa[8], ob[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sn = s_sn[i0 + e], cs = s_cs[i0 + e];
        oa[e] = from_f32<DT>(a[e] * cs - b[e] * sn);
        ob[e] = from_f32<DT>(a[e] * sn + b[e] * cs);
      }
      uint16_t* dst = isq ? q + (size_t)t * ldq + hh * hd : kc + ((size_t)hh * S + pos) * hd;
      *reinterpret_cast<uint4*>(dst + i0) = *reinterpret_cast<const uint4*>(oa);
      *reinterpret_cast<uint4*>(dst + i0 + half) = *reinterpret_cast<const uint4*>(ob);
    } else {
      const int pp = p - nrope, per = hd >> 3;
      const int head = pp / per, c = (pp - head * per) * 8;
      *reinterpret_cast<uint4*>(vc + ((size_t)head * S + pos) * hd + c) =
          *reinterpret_cast<const uint4*>(v + (size_t)t * ld + head * hd + c);
    }
  }
}

// act = silu(g) * u   (16-bit in/out), gu = [T, 2, I] packed or separate.
template <int DT>
__global__ void silu_mul_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u,
                                size_t n, uint16_t* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = from_f32<DT>(silu(to_f32<DT>(g[i])) * to_f32<DT>(u[i]));
}

// out[t][i] = silu(gu[t][i]) * gu[t][I + i]  (fused gate|up GEMM output), 8 per thread
template <int DT>
__global__ void silu_mul_rows_kernel(const uint16_t* __restrict__ gu, size_t T, int I,
                                     uint16_t* __restrict__ out) {
  const int iv = I >> 3;
  const size_t n = T * iv;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t t = i / iv;
    const int c = (int)(i - t * iv) * 8;
    float g[8], u[8];
    unpack8<DT>(*reinterpret_cast<const uint4*>(gu + t * 2 * I + c), g);
    unpack8<DT>(*reinterpret_cast<const uint4*>(gu + t * 2 * I + I + c), u);
    uint16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f32<DT>(silu(g[e]) * u[e]);
    *reinterpret_cast<uint4*>(out + t * I + c) = *reinterpret_cast<uint4*>(o);
  }
}

// resid (f32) += y (16-bit), 8 per thread
template <int DT>
__global__ void add_resid8_kernel(float* __restrict__ resid, const uint16_t* __restrict__ y,
                                  size_t n8) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (size_t)gridDim.x * blockDim.x) {
    float f[8];
    unpack8<DT>(*reinterpret_cast<const uint4*>(y + i * 8), f);
    float4* r = reinterpret_cast<float4*>(resid + i * 8);
    float4 a = r[0], b = r[1];
    a.x += f[0]; a.y += f[1]; a.z += f[2]; a.w += f[3];
    b.x += f[4]; b.y += f[5]; b.z += f[6]; b.w += f[7];
    r[0] = a;
    r[1] = b;
  }
}

// resid (f32) += y (16-bit)
template <int DT>
__global__ void add_resid_kernel(float* __restrict__ resid, const uint16_t* __restrict__ y,
                                 size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    resid[i] += to_f32<DT>(y[i]);
}

// Streaming-read probe (scripts/decode_ceiling.py): reads n16 16-byte words
// with the decode GEMVs' non-temporal loads, 8 per lane in flight, and does no
// other work — the speed-of-light reference for a bandwidth-bound kernel of the
// same byte count (the sink is written only on an impossible value).
__global__ __launch_bounds__(256) void stream_read_kernel(const uint4* __restrict__ p, size_t n16,
                                                          unsigned int* __restrict__ sink) {
  constexpr int U = 8;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  unsigned int acc = 0;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld_nt16(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) {
    const uint4 v = ld_nt16(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// Weight upload conversion (native engine, csrc/engine/llama_engine.cpp): a checkpoint
// tensor in bf16 / f16 / f32 (SK 0 / 1 / 2) -> the model's 16-bit dtype.
template <int SK, int DT>
__global__ __launch_bounds__(256) void cast16_kernel(const void* __restrict__ src,
                                                     uint16_t* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    float v;
    if constexpr (SK == 2) v = reinterpret_cast<const float*>(src)[i];
    else v = to_f32<SK>(reinterpret_cast<const uint16_t*>(src)[i]);
    dst[i] = from_f32<DT>(v);
  }
}

// Tensor-parallel prefill all-reduce (native engine): out (+)= sum of the W slices
// src[w * stride .. + n) that the ranks wrote into this rank's (uncached) slab.
__global__ __launch_bounds__(256) void sum_slices_kernel(float* __restrict__ out,
                                                         const float* __restrict__ src, int W,
                                                         long long stride, long long n,
                                                         int accumulate) {
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * 256 * 4) {
    if (i + 4 <= n) {
      float4 a = accumulate ? *reinterpret_cast<const float4*>(out + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int w = 0; w < W; ++w) {
        const float4 v = *reinterpret_cast<const float4*>(src + w * stride + i);
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
      *reinterpret_cast<float4*>(out + i) = a;
    } else {
      for (long long j = i; j < n; ++j) {
        float a = accumulate ? out[j] : 0.f;
        for (int w = 0; w < W; ++w) a += src[w * stride + j];
        out[j] = a;
      }
    }
  }
}

// Seeded N(mean, std^2) fill of a 16-bit tensor, stateless: element i's value depends
// only on (key, i) — a splitmix64 hash of the element pair index feeds one Box-Muller
// draw per two elements — so any launch geometry (and any rank filling its own slice)
// gives the same bits.  Random-init weights for the native engine's synthetic-checkpoint
// mode (benchmarks: no network, no checkpoint; cake_engine_open with init = 1).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float2 normal_pair(uint64_t key, uint64_t pair) {
  const uint64_t r = mix64(key ^ mix64(pair + 0x9e3779b97f4a7c15ULL));
  const float u1 = (float)((uint32_t)(r >> 40) + 1u) * (1.0f / 16777216.f);  // (0, 1]
  const float u2 = (float)(uint32_t)(r & 0xffffffu) * (1.0f / 16777216.f);  // [0, 1)
  const float rad = sqrtf(-2.f * __logf(u1));
  float s, c;
  __sincosf(6.283185307179586f * u2, &s, &c);
  return make_float2(rad * c, rad * s);
}

template <int DT>
__global__ __launch_bounds__(256) void fill_normal_kernel(uint16_t* __restrict__ out, size_t n,
                                                          float mean, float std, uint64_t key) {
  const size_t n8 = n / 8;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < n8;
       g += (size_t)gridDim.x * blockDim.x) {
    uint32_t w[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float2 z = normal_pair(key, g * 4 + p);
      w[p] = (uint32_t)from_f32<DT>(mean + std * z.x) | ((uint32_t)from_f32<DT>(mean + std * z.y) << 16);
    }
    reinterpret_cast<uint4*>(out)[g] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  // tail (n % 8 elements): the first threads of block 0
  if (blockIdx.x == 0 && threadIdx.x < (n - n8 * 8)) {
    const size_t i = n8 * 8 + threadIdx.x;
    const float2 z = normal_pair(key, i / 2);
    out[i] = from_f32<DT>(mean + std * ((i & 1) ? z.y : z.x));
  }
}

}  // namespace cake

using namespace cake;

CAKE_API int cake_sum_slices(float* out, const float* src, int W, long long stride, long long n,
                             int accumulate, hipStream_t st) {
  if (W < 1 || n < 0 || stride < n || (stride % 4) || ((uintptr_t)out % 16) || ((uintptr_t)src % 16))
    return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  long long g = (n / 4 + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(sum_slices_kernel, dim3((unsigned)g), dim3(256), 0, st, out, src, W, stride, n,
                     accumulate);
  return (int)hipGetLastError();
}

CAKE_API int cake_stream_read(const void* p, size_t bytes, int blocks, unsigned int* sink,
                              hipStream_t st) {
  if (bytes % 16 || blocks < 1 || ((uintptr_t)p % 16)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stream_read_kernel, dim3(blocks), dim3(256), 0, st, (const uint4*)p,
                     bytes / 16, sink);
  return (int)hipGetLastError();
}

#define DISPATCH_DT(dt, ...)                       \
  do {                                             \
    if ((dt) == kBF16) { constexpr int DT = kBF16; __VA_ARGS__; } \
    else if ((dt) == kF16) { constexpr int DT = kF16; __VA_ARGS__; } \
    else return (int)hipErrorInvalidValue;         \
  } while (0)

static inline int ew_grid(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 4096 ? g : 4096);
}

CAKE_API int cake_cast16(int src_kind, int dt, const void* src, void* dst, size_t n,
                         hipStream_t st) {
  if (src_kind < 0 || src_kind > 2) return (int)hipErrorInvalidValue;
  const dim3 g(ew_grid(n)), b(256);
#define CAKE_CAST(SKV)                                                                      \
  DISPATCH_DT(dt, hipLaunchKernelGGL((cast16_kernel<SKV, DT>), g, b, 0, st, src, (uint16_t*)dst, n))
  if (src_kind == 0) CAKE_CAST(0);
  else if (src_kind == 1) CAKE_CAST(1);
  else CAKE_CAST(2);
#undef CAKE_CAST
  return (int)hipGetLastError();
}

CAKE_API int cake_fill_normal(int dt, void* dst, size_t n, float mean, float std,
                              unsigned long long key, hipStream_t st) {
  if ((uintptr_t)dst % 16) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  size_t g = (n / 8 + 255) / 256;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  DISPATCH_DT(dt, hipLaunchKernelGGL((fill_normal_kernel<DT>), dim3((unsigned)g), dim3(256), 0, st,
                                     (uint16_t*)dst, n, mean, std, (uint64_t)key));
  return (int)hipGetLastError();
}

CAKE_API int cake_embed(int dt, const void* table, const int* tok, int T, int H, float* out,
                        hipStream_t st) {
  if (H % 8) return (int)hipErrorInvalidValue;
  DISPATCH_DT(dt, hipLaunchKernelGGL((embed_kernel<DT>), dim3(T), dim3(256), 0, st,
                                     (const uint16_t*)table, tok, H, out));
  return (int)hipGetLastError();
}

static int g_rmsnorm_reg = 1;  // 0: the two-pass loop kernel (A/B, tests)
CAKE_API void cake_rmsnorm_set_reg(int on) { g_rmsnorm_reg = on; }

CAKE_API int cake_rmsnorm(int dt, const float* x, const void* w, float eps, int T, int H,
                          void* out, hipStream_t st) {
  if (H % 4) return (int)hipErrorInvalidValue;
  // register-resident rows up to 8192 columns (every Llama hidden size); wider rows loop
  if (H <= 8192 && g_rmsnorm_reg) {
#define CAKE_RMS(NV) hipLaunchKernelGGL((rmsnorm_reg_kernel<DT, NV>), dim3(T), dim3(256), 0, st, x, \
                                        (const uint16_t*)w, eps, H, (uint16_t*)out)
    DISPATCH_DT(dt, if (H <= 2048) CAKE_RMS(2); else if (H <= 4096) CAKE_RMS(4); else CAKE_RMS(8));
#undef CAKE_RMS
    return (int)hipGetLastError();
  }
  DISPATCH_DT(dt, hipLaunchKernelGGL((rmsnorm_kernel<DT>), dim3(T), dim3(256), 0, st, x,
                                     (const uint16_t*)w, eps, H, (uint16_t*)out));
  return (int)hipGetLastError();
}

// q rows are `ldq` elements apart, k / v rows `ld` apart (separate tensors, or
// column slices of one fused [T, (nh + 2 nkv) hd] projection output)
CAKE_API int cake_rope_kv(int dt, void* q, const void* k, const void* v, int ldq, int ld, int T, int nh,
                          int nkv, int hd, const float* inv_freq, int pos0, int S, void* kc,
                          void* vc, hipStream_t st) {
  const bool vec = hd % 16 == 0 && hd <= 256 && ldq % 8 == 0 && ld % 8 == 0 &&
                   ((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)kc | (uintptr_t)vc) % 16 == 0;
  if (vec) {
    DISPATCH_DT(dt, hipLaunchKernelGGL((rope_kv_vec_kernel<DT>), dim3(T), dim3(256), 0, st,
                                       (uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, ldq,
                                       ld, nh, nkv, hd, inv_freq, pos0, S, (uint16_t*)kc,
                                       (uint16_t*)vc));
    return (int)hipGetLastError();
  }
  DISPATCH_DT(dt, hipLaunchKernelGGL((rope_kv_kernel<DT>), dim3(T), dim3(256), 0, st,
                                     (uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, ldq, ld, nh,
                                     nkv, hd, inv_freq, pos0, S, (uint16_t*)kc,
                                     (uint16_t*)vc));
  return (int)hipGetLastError();
}

CAKE_API int cake_silu_mul(int dt, const void* g, const void* u, size_t n, void* out,
                           hipStream_t st) {
  DISPATCH_DT(dt, hipLaunchKernelGGL((silu_mul_kernel<DT>), dim3(ew_grid(n)), dim3(256), 0, st,
                                     (const uint16_t*)g, (const uint16_t*)u, n,
                                     (uint16_t*)out));
  return (int)hipGetLastError();
}

CAKE_API int cake_silu_mul_rows(int dt, const void* gu, size_t T, int I, void* out,
                                hipStream_t st) {
  if (I % 8 || ((uintptr_t)gu | (uintptr_t)out) % 16) return (int)hipErrorInvalidValue;
  DISPATCH_DT(dt, hipLaunchKernelGGL((silu_mul_rows_kernel<DT>), dim3(ew_grid(T * I / 8)),
                                     dim3(256), 0, st, (const uint16_t*)gu, T, I,
                                     (uint16_t*)out));
  return (int)hipGetLastError();
}

CAKE_API int cake_add_resid(int dt, float* resid, const void* y, size_t n, hipStream_t st) {
  if (n % 8 == 0 && ((uintptr_t)resid % 32 == 0) && ((uintptr_t)y % 16 == 0)) {
    DISPATCH_DT(dt, hipLaunchKernelGGL((add_resid8_kernel<DT>), dim3(ew_grid(n / 8)), dim3(256),
                                       0, st, resid, (const uint16_t*)y, n / 8));
    return (int)hipGetLastError();
  }
  DISPATCH_DT(dt, hipLaunchKernelGGL((add_resid_kernel<DT>), dim3(ew_grid(n)), dim3(256), 0,
                                     st, resid, (const uint16_t*)y, n));
  return (int)hipGetLastError();
}

// Test hook for the wave reductions of common.h (one wave): out[0:64] wave_sum,
// [64:128] wave_max, [128:192] x + x[l^8], [192:256] x + x[l^16], [256:320] x + x[l^32].
__global__ __launch_bounds__(64) void wave_reduce_probe_kernel(const float* x, float* out) {
  const int l = threadIdx.x;
  const float v = x[l];
  out[l] = wave_sum(v);
  out[64 + l] = wave_max(v);
  out[128 + l] = xor_add<8>(v);
  out[192 + l] = xor_add<16>(v);
  out[256 + l] = xor_add<32>(v);
}

CAKE_API int cake_wave_reduce_probe(const float* x, float* out, hipStream_t st) {
  hipLaunchKernelGGL(wave_reduce_probe_kernel, dim3(1), dim3(64), 0, st, x, out);
  return (int)hipGetLastError();
}
