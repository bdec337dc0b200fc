// Shared device helpers for the cake_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64: lane = threadIdx.x & 63, wave = threadIdx.x >> 6.
//   * 16-bit storage types are carried as raw uint16 bit patterns (bf16 or f16,
//     selected by the DT template parameter) and widened to f32 in registers.
//     All accumulation is f32.
//   * Every exported entry point is `extern "C"`, takes raw device pointers and a
//     hipStream_t, and returns a hipError_t as int, so the launches are captured
//     unchanged inside hipGraphs (the Python side passes torch's current stream).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define CAKE_API extern "C" __attribute__((visibility("default")))

namespace cake {

enum DType : int { kBF16 = 0, kF16 = 1, kF32 = 2 };

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// round to nearest even, NaN stays NaN: one v_cvt_pk_bf16_f32 on gfx950
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  _Float16 v;
  __builtin_memcpy(&v, &h, 2);
  return (float)v;
}

__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  _Float16 v = (_Float16)f;
  uint16_t h;
  __builtin_memcpy(&h, &v, 2);
  return h;
}

template <int DT>
__device__ __forceinline__ float to_f32(uint16_t h) {
  if constexpr (DT == kBF16) return bf16_to_f32(h);
  else return f16_to_f32(h);
}

template <int DT>
__device__ __forceinline__ uint16_t from_f32(float f) {
  if constexpr (DT == kBF16) return f32_to_bf16(f);
  else return f32_to_f16(f);
}

// Unpack 8 packed 16-bit values (one 16-byte load) into f32.
template <int DT>
__device__ __forceinline__ void unpack8(const uint4 v, float* o) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = to_f32<DT>((uint16_t)(w[i] & 0xffffu));
    o[2 * i + 1] = to_f32<DT>((uint16_t)(w[i] >> 16));
  }
}

// Wave-wide butterfly reductions without LDS: DPP (quad_perm xor 1 / xor 2,
// row_half_mirror, row_mirror) inside each 16-lane row, then the gfx950 lane-swap
// instructions across rows (v_permlane16_swap: rows 0|1 and 2|3; v_permlane32_swap:
// halves).  Every lane ends with the same bits.  (The __shfl_xor form was six
// dependent ds_bpermute round trips per reduction.)
template <int CTRL> __device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  v += dpp_f<kDppMirror>(v);
  const int b = __builtin_bit_cast(int, v);
  const auto p = __builtin_amdgcn_permlane16_swap(b, b, false, false);
  v = __builtin_bit_cast(float, (int)p[0]) + __builtin_bit_cast(float, (int)p[1]);
  const int c = __builtin_bit_cast(int, v);
  const auto q = __builtin_amdgcn_permlane32_swap(c, c, false, false);
  return __builtin_bit_cast(float, (int)q[0]) + __builtin_bit_cast(float, (int)q[1]);
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<kDppXor1>(v));
  v = fmaxf(v, dpp_f<kDppXor2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_f<kDppMirror>(v));
  const int b = __builtin_bit_cast(int, v);
  const auto p = __builtin_amdgcn_permlane16_swap(b, b, false, false);
  v = fmaxf(__builtin_bit_cast(float, (int)p[0]), __builtin_bit_cast(float, (int)p[1]));
  const int c = __builtin_bit_cast(int, v);
  const auto q = __builtin_amdgcn_permlane32_swap(c, c, false, false);
  return fmaxf(__builtin_bit_cast(float, (int)q[0]), __builtin_bit_cast(float, (int)q[1]));
}

// v + v[lane ^ OFF] (same bits in both lanes of a pair), OFF in {8, 16, 32}.
template <int OFF> __device__ __forceinline__ float xor_add(float v) {
  static_assert(OFF == 8 || OFF == 16 || OFF == 32, "xor_add offset");
  if constexpr (OFF == 8) {
    return v + dpp_f<0x128>(v);  // row_ror:8 == lane ^ 8 inside a 16-lane row
  } else {
    const int b = __builtin_bit_cast(int, v);
    const auto p = OFF == 16 ? __builtin_amdgcn_permlane16_swap(b, b, false, false)
                             : __builtin_amdgcn_permlane32_swap(b, b, false, false);
    return __builtin_bit_cast(float, (int)p[0]) + __builtin_bit_cast(float, (int)p[1]);
  }
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// Streaming (read-once) 16-byte load: weights in batch-1 decode are touched by
// exactly one wave, so keep them from displacing reusable lines.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// x * sigmoid(x) with v_rcp (1 ulp) instead of the IEEE division sequence: the
// SwiGLU / SiLU GEMM epilogues evaluate it once per output element
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-x));
}

// tanh-approximated GELU (candle's gelu / diffusers "gelu-approximate"):
// 0.5 x (1 + tanh(u)) == x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3) — one
// v_exp + one v_rcp instead of libm tanhf (~50 instructions with a branch), which
// made the GEGLU epilogue of SD's FF-in GEMM VALU-bound.
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x * x, x);
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-u2));
}

// MFMA operand / accumulator vectors (16x16x32: 8 x 16-bit per lane, 4 f32 acc)
typedef __bf16 cbf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 cf16x8 __attribute__((ext_vector_type(8)));
typedef float cf32x4 __attribute__((ext_vector_type(4)));

// D = A(16x32) B(32x16) + C; lane l holds A[l&15][8(l>>4)..+8] and B[8(l>>4)..+8][l&15]
// (16-byte k-contiguous fragments), D[4(l>>4)+e][l&15] in element e.
template <int DT>
__device__ __forceinline__ cf32x4 cmfma(const uint4 a, const uint4 b, cf32x4 c) {
  if constexpr (DT == kBF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, a),
                                                   __builtin_bit_cast(cbf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(cf16x8, a),
                                                  __builtin_bit_cast(cf16x8, b), c, 0, 0, 0);
}

// LDS byte offset of a __shared__ pointer (for inline-asm ds_* operands)
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// LDS-DMA (global_load_lds) operand types and an s_waitcnt immediate that
// constrains only the vector-memory counter (gfx9 encoding).
typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
constexpr int vm_wait(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

// 16 bytes global -> LDS; the LDS destination of lane l is lds_wave_base + 16 l.
__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds_wave_base, 16, 0, 0);
}

}  // namespace cake
