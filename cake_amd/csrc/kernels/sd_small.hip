// Stable Diffusion step glue as device kernels:
//
//   * timestep_embed: sinusoidal embedding of the step's timestep, read from a
//     device table at a device step index (candle stable_diffusion
//     Timesteps: sin/cos of t * exp(-ln(1e4) i / (half - shift)), optional
//     flip), so the UNet step replays unchanged in a hipGraph across steps;
//   * sched_step: classifier-free-guidance combine + scheduler update + the next
//     step's UNet input, in one pass (cake-core/src/models/sd/sd.rs:470-504:
//     cat([x, x]) -> scale_model_input -> unet -> chunk -> u + g (c - u) ->
//     scheduler.step).  Every scheduler the reference uses is
//       prev = A x + B eps + N z        (z ~ N(0, 1), Euler-ancestral only)
//     with per-step scalars (A, B, N) and the next input scale S precomputed on
//     the host into a device table:
//       DDIM eps:  A = sqrt(a_prev / a_t), B = sqrt(1 - a_prev) - sqrt(a_prev (1 - a_t) / a_t)
//       DDIM v:    A = sqrt(a_prev a_t) + sqrt((1 - a_prev)(1 - a_t)),
//                  B = sqrt((1 - a_prev) a_t) - sqrt(a_prev (1 - a_t))
//       Euler-a:   A = 1, B = s_down - s_from, N = s_up
//     z is a counter-based Philox4x32-10 normal (Box-Muller) keyed by the seed
//     with counter (element, step), so the replayed step draws fresh noise;
//   * step_advance: step += 1 (the tables are indexed by it);
//   * to_rgb8: decoded image [B][3][H][W] or [B][H][W][3] (16-bit) ->
//     u8 HWC of clamp(x / 2 + 0.5, 0, 1) * 255 (sd.rs:544-547, truncating cast).
#include "common.h"

namespace cake {

__device__ __forceinline__ uint4 philox4(uint32_t c0, uint32_t c1, uint32_t k0, uint32_t k1) {
  uint32_t c2 = 0u, c3 = 0u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c1 = lo1; c3 = lo0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ float normal_from(uint32_t a, uint32_t b) {
  const float u1 = ((float)(a >> 8) + 0.5f) * 5.9604644775390625e-08f;  // (0, 1)
  const float u2 = (float)(b >> 8) * 5.9604644775390625e-08f;
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

template <int DT, bool OUT16>
__global__ void timestep_embed_kernel(const float* __restrict__ t_table,
                                      const int* __restrict__ step, int B, int dim, int flip,
                                      float shift, void* __restrict__ out) {
  const int half = dim / 2;
  const float t = t_table[step ? *step : 0];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * dim; i += gridDim.x * blockDim.x) {
    const int j = i % dim;
    const int k = j < half ? j : j - half;
    const float e = __expf(-9.210340371976184f * (float)k / ((float)half - shift)) * t;
    const bool first_sin = j < half;
    const float v = (first_sin != (flip != 0)) ? sinf(e) : cosf(e);
    if constexpr (OUT16) reinterpret_cast<uint16_t*>(out)[i] = from_f32<DT>(v);
    else reinterpret_cast<float*>(out)[i] = v;
  }
}

// latents f32 [n] (x), pred 16-bit [(cfg ? 2 : 1) * n] (unet output: [uncond; cond]),
// coef[step] = (A, B, N, S_next); next_in 16-bit [(cfg ? 2 : 1) * n] (optional).
template <int DT>
__global__ void sched_step_kernel(float* __restrict__ x, const uint16_t* __restrict__ pred,
                                  long long n, int cfg, float guidance,
                                  const float4* __restrict__ coef, const int* __restrict__ step,
                                  const uint32_t* __restrict__ key, uint16_t* __restrict__ next_in) {
  const int s = *step;
  const float4 c = coef[s];
  const uint32_t k0 = key[0], k1 = key[1];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float e = to_f32<DT>(pred[i]);
    if (cfg) {
      const float cond = to_f32<DT>(pred[i + n]);
      e = e + guidance * (cond - e);
    }
    float y = c.x * x[i] + c.y * e;
    if (c.z != 0.f) {
      const uint4 r = philox4((uint32_t)i, (uint32_t)s, k0, k1);
      y += c.z * normal_from(r.x, r.y);
    }
    x[i] = y;
    if (next_in != nullptr) {
      const uint16_t v = from_f32<DT>(y * c.w);
      next_in[i] = v;
      if (cfg) next_in[i + n] = v;
    }
  }
}

__global__ void step_advance_kernel(int* __restrict__ step) { *step += 1; }

// x f32 [n]: x = x * scale  +  optional 16-bit copy (UNet input of the first step)
template <int DT>
__global__ void scale_copy_kernel(const float* __restrict__ x, long long n, float scale, int dup,
                                  uint16_t* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const uint16_t v = from_f32<DT>(x[i] * scale);
    out[i] = v;
    if (dup) out[i + n] = v;
  }
}

template <int DT>
__global__ void to_rgb8_kernel(const uint16_t* __restrict__ img, int B, int H, int W, int nhwc,
                               uint8_t* __restrict__ out) {
  const long long total = (long long)B * H * W * 3;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(o % 3);
    const long long p = o / 3;  // (b, y, x)
    const long long b = p / ((long long)H * W), yx = p % ((long long)H * W);
    const long long src = nhwc ? o : (b * 3 + c) * (long long)H * W + yx;
    float v = to_f32<DT>(img[src]) * 0.5f + 0.5f;
    v = fminf(fmaxf(v, 0.f), 1.f) * 255.f;
    out[o] = (uint8_t)v;  // truncation, like the reference's f32 -> u8 cast
  }
}

// CLIP text embedding: out[r, :] = tok[ids[r]] + pos[r % T] (the reference's token +
// position embedding sum, clip.rs; one rounding of the f32 sum, as torch's 16-bit add)
template <int DT>
__global__ __launch_bounds__(256) void clip_embed_kernel(const uint16_t* __restrict__ tok,
                                                         const uint16_t* __restrict__ pos,
                                                         const int* __restrict__ ids, int rows,
                                                         int T, int D, int V,
                                                         uint16_t* __restrict__ out) {
  const long long n = (long long)rows * D;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int r = (int)(i / D), d = (int)(i - (long long)r * D);
    int id = ids[r];
    id = id < 0 ? 0 : (id >= V ? V - 1 : id);
    const float v = to_f32<DT>(tok[(size_t)id * D + d]) + to_f32<DT>(pos[(size_t)(r % T) * D + d]);
    out[i] = from_f32<DT>(v);
  }
}

// 16-bit -> f32 (host read-back of component outputs)
template <int DT>
__global__ __launch_bounds__(256) void widen_kernel(const uint16_t* __restrict__ x, long long n,
                                                    float* __restrict__ y) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    y[i] = to_f32<DT>(x[i]);
}

static inline int grid_for_n(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace cake

using namespace cake;

CAKE_API int cake_timestep_embed(int dt, const float* t_table, const int* step, int B, int dim,
                                 int flip, float shift, int out16, void* out, hipStream_t st) {
  if (B <= 0 || dim <= 0 || dim % 2) return (int)hipErrorInvalidValue;
  const int g = grid_for_n((long long)B * dim);
  if (!out16) hipLaunchKernelGGL((timestep_embed_kernel<kBF16, false>), dim3(g), dim3(256), 0, st,
                                 t_table, step, B, dim, flip, shift, out);
  else if (dt == kBF16) hipLaunchKernelGGL((timestep_embed_kernel<kBF16, true>), dim3(g), dim3(256),
                                           0, st, t_table, step, B, dim, flip, shift, out);
  else if (dt == kF16) hipLaunchKernelGGL((timestep_embed_kernel<kF16, true>), dim3(g), dim3(256), 0,
                                          st, t_table, step, B, dim, flip, shift, out);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// seed: device int64 (read by the kernel, so a captured step serves any seed)
CAKE_API int cake_sched_step(int dt, float* x, const void* pred, long long n, int cfg,
                             float guidance, const void* coef, const int* step,
                             const void* seed, void* next_in, hipStream_t st) {
  if (n <= 0 || seed == nullptr) return (int)hipErrorInvalidValue;
  const int g = grid_for_n(n);
  const uint32_t* key = (const uint32_t*)seed;
  if (dt == kBF16)
    hipLaunchKernelGGL((sched_step_kernel<kBF16>), dim3(g), dim3(256), 0, st, x,
                       (const uint16_t*)pred, n, cfg, guidance, (const float4*)coef, step, key,
                       (uint16_t*)next_in);
  else if (dt == kF16)
    hipLaunchKernelGGL((sched_step_kernel<kF16>), dim3(g), dim3(256), 0, st, x,
                       (const uint16_t*)pred, n, cfg, guidance, (const float4*)coef, step, key,
                       (uint16_t*)next_in);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

CAKE_API int cake_step_advance(int* step, hipStream_t st) {
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, st, step);
  return (int)hipGetLastError();
}

CAKE_API int cake_scale_copy(int dt, const float* x, long long n, float scale, int dup, void* out,
                             hipStream_t st) {
  const int g = grid_for_n(n);
  if (dt == kBF16)
    hipLaunchKernelGGL((scale_copy_kernel<kBF16>), dim3(g), dim3(256), 0, st, x, n, scale, dup,
                       (uint16_t*)out);
  else if (dt == kF16)
    hipLaunchKernelGGL((scale_copy_kernel<kF16>), dim3(g), dim3(256), 0, st, x, n, scale, dup,
                       (uint16_t*)out);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

CAKE_API int cake_to_rgb8(int dt, const void* img, int B, int H, int W, int nhwc, void* out,
                          hipStream_t st) {
  const int g = grid_for_n((long long)B * H * W * 3);
  if (dt == kBF16)
    hipLaunchKernelGGL((to_rgb8_kernel<kBF16>), dim3(g), dim3(256), 0, st, (const uint16_t*)img,
                       B, H, W, nhwc, (uint8_t*)out);
  else if (dt == kF16)
    hipLaunchKernelGGL((to_rgb8_kernel<kF16>), dim3(g), dim3(256), 0, st, (const uint16_t*)img,
                       B, H, W, nhwc, (uint8_t*)out);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

CAKE_API int cake_clip_embed(int dt, const void* tok, const void* pos, const int* ids, int rows,
                             int T, int D, int V, void* out, hipStream_t st) {
  if (rows <= 0 || T <= 0 || D <= 0 || V <= 0) return (int)hipErrorInvalidValue;
  const int g = grid_for_n((long long)rows * D);
  if (dt == kBF16)
    hipLaunchKernelGGL((clip_embed_kernel<kBF16>), dim3(g), dim3(256), 0, st,
                       (const uint16_t*)tok, (const uint16_t*)pos, ids, rows, T, D, V,
                       (uint16_t*)out);
  else if (dt == kF16)
    hipLaunchKernelGGL((clip_embed_kernel<kF16>), dim3(g), dim3(256), 0, st,
                       (const uint16_t*)tok, (const uint16_t*)pos, ids, rows, T, D, V,
                       (uint16_t*)out);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

CAKE_API int cake_widen16(int dt, const void* x, long long n, float* y, hipStream_t st) {
  if (n <= 0) return (int)hipErrorInvalidValue;
  const int g = grid_for_n(n);
  if (dt == kBF16)
    hipLaunchKernelGGL((widen_kernel<kBF16>), dim3(g), dim3(256), 0, st, (const uint16_t*)x, n, y);
  else if (dt == kF16)
    hipLaunchKernelGGL((widen_kernel<kF16>), dim3(g), dim3(256), 0, st, (const uint16_t*)x, n, y);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
