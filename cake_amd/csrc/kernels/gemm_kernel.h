// MFMA GEMM kernels, tile configurations and the per-(dtype, epilogue) launcher.
// Shared by gemm.hip (C API, split-K finalize) and the gemm_inst_*.hip translation
// units that instantiate the launchers in parallel (one TU per dtype x epilogue half:
// the fully unrolled interleaved schedules make one TU take minutes).
#pragma once
// (design notes: gemm.hip)
#include "common.h"

#include <type_traits>

namespace cake {

constexpr int kGBK = 64;  // k per step (128-byte rows)

enum GemmEpi : int {
  kEpiStore = 0,   // C16 = acc (+ bias)
  kEpiResid32 = 1, // R32 += acc (+ bias)
  kEpiAdd16 = 2,   // C16 = acc (+ bias) + R16
  kEpiSwiglu = 3,  // C16[:, f] = silu(acc_gate) * acc_up
  kEpiGeglu = 4,   // C16[:, f] = acc_h * gelu_tanh(acc_gate)
  kEpiPartial = 5, // W32[split] = acc (split-K slab, virtual column order)
  kEpiStore32 = 6, // R32 = acc (+ bias)              (f32 output, e.g. conv time biases)
  kEpiSilu = 7,    // C16 = act(acc (+ bias)), act = GemmArgs::act: SiLU (time-embedding
                   // MLP), quick_gelu / erf-GELU (CLIP MLP); host ids 7 / 8 / 9
};

// the activation of kEpiSilu (runtime-uniform: one kernel instance for all three)
__device__ __forceinline__ float gemm_act(int act, float x) {
  if (act == 1) return x * __frcp_rn(1.f + __expf(-1.702f * x));  // quick_gelu
  if (act == 2) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));  // GELU (erf)
  return silu(x);
}

struct GemmArgs {
  const uint16_t* a;     // [M][lda]
  const uint16_t* b;     // [Nw][ldb] weight rows
  uint16_t* c;           // [M][ldc] 16-bit output
  const uint16_t* bias;  // [N] or null
  float* r32;            // [M][ldr] f32 residual (kEpiResid32)
  const uint16_t* r16;   // [M][ldr] 16-bit residual (kEpiAdd16)
  float* ws;             // [splits][M][Nv] f32 slabs (kEpiPartial)
  const uint16_t* zeros; // >= 16 zero bytes (DMA source for out-of-range rows / k)
  long long lda, ldb, ldc, ldr;
  int M, N, K;           // N = output columns (features); Nv = virtual B rows
  int Nv, half;          // gated: Nv = 2 * half, half = N
  int gated;             // B row order interleaves 16-row blocks of two halves
  int tiles_m, tiles_n, kps;  // k elements per split
  int act;               // kEpiSilu activation: 0 SiLU, 1 quick_gelu, 2 GELU (erf)
  // in-kernel split-K pair (gemm_4w.h, splits == 2): the first split of a tile to finish
  // parks its accumulators in ws (one 256x256 f32 slab per tile), the second adds them and
  // runs the epilogue; tick = [kPairTiles arrival counters | kPairTiles ready flags]
  int pair;
  unsigned* tick;
  int dp_tiles;          // pair: tiles [0, dp_tiles) run whole, the rest as k-half pairs
};
constexpr int kPairTiles = 16384;

// virtual B row -> weight row (gated: [16 gate rows | 16 up rows] per 32-row block)
__device__ __forceinline__ int wrow(const GemmArgs& g, int v) {
  if (!g.gated) return v;
  const int blk = v >> 5, w = v & 31;
  return w < 16 ? blk * 16 + w : g.half + blk * 16 + (w - 16);
}


// MFMA with the accumulator pinned to AGPRs (tied "+a" operand): for 128x128 wave
// tiles (256 accumulator registers) hipcc's own allocation rotates the accumulators
// through VGPR copies around every MFMA.  Chained MFMAs on one accumulator need no
// wait states; the A/B fragments come from counted LDS reads.
typedef unsigned cu32x4 __attribute__((ext_vector_type(4)));

template <int DT>
__device__ __forceinline__ void amfma(cf32x4& acc, const uint4& a, const uint4& b) {
  const cu32x4 av = __builtin_bit_cast(cu32x4, a), bv = __builtin_bit_cast(cu32x4, b);
  if constexpr (DT == kBF16)
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(av), "v"(bv));
  else
    asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(av), "v"(bv));
}

// same, volatile: kept in program order among the loads it is interleaved with
template <int DT>
__device__ __forceinline__ void amfma_v(cf32x4& acc, const uint4& a, const uint4& b) {
  const cu32x4 av = __builtin_bit_cast(cu32x4, a), bv = __builtin_bit_cast(cu32x4, b);
  if constexpr (DT == kBF16)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(av), "v"(bv));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(av), "v"(bv));
}

// acc = 0 in the AGPR file (0 x 0 + 0; the fresh zero VGPRs need 2 wait states)
__device__ __forceinline__ void azero(cf32x4& acc) {
  const cu32x4 z = {0u, 0u, 0u, 0u};
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "=a"(acc) : "v"(z));
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E) — the interleaved
// schedule's indices must be constants however long the sweep (a #pragma unroll of a
// 64 x 32 nest can stay rolled, sending the accumulators to scratch).
template <int B, class F, int... Is>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, B + Is>{}), ...);  // flat expansion, no recursion
}
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) static_for_impl<B>(f, std::make_integer_sequence<int, E - B>{});
}

// same with a compile-time byte offset in the instruction (one base VGPR per tile)
template <int OFF>
__device__ __forceinline__ uint4 ds_read16_off(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16-bit");
  uint4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF));
  return v;
}

__device__ __forceinline__ uint4 ds_read16(uint32_t addr) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

// Epilogue operands that come from global memory — the bias columns and the residual
// row segment of each strip — requested AHEAD of use: the bias once per wave, a strip's
// residual before the previous strip is stored.  Loaded inside the strip (as before)
// every strip waited one full memory round trip behind the previous strip's stores
// (the compiler cannot hoist a load over stores that may alias it): +4.5-6.7 us per SD
// add16 projection in isolation.
// Measured per epilogue (profiles/r3_gemm_epilogue_ab.jsonl): the 16-bit residual add
// (SD projections, +6-21 %) and the gated bias (+1-3 %) gain; the f32 residual / plain
// stores did not (the extra live registers cost the 256-wide tiles a spill), so those keep
// their in-strip loads (PRE = false).
template <int DT, int EPI, int NF> struct EpiOps {
  static constexpr int WTN = NF * 16;
  static constexpr bool GATED = (EPI == kEpiSwiglu || EPI == kEpiGeglu);
  static constexpr int OUTC = GATED ? WTN / 2 : WTN;
  static constexpr int CPL = OUTC / 4;
  static constexpr bool PRE = (EPI == kEpiAdd16 || GATED);
  static constexpr bool RES = EPI == kEpiAdd16;
  float bias[PRE ? (GATED ? 2 * CPL : CPL) : 1];
  float res[2][RES ? CPL : 1];

  static constexpr int VW = CPL % 8 == 0 ? 8 : 4;  // vector width (16 / 8-byte accesses)

  // 16-bit values [n0, n0 + CPL) of row p (columns < n valid) as f32
  __device__ __forceinline__ static void load16(const uint16_t* p, int n0, int n, bool vec,
                                                float* o) {
    if (vec) {
      if constexpr (VW == 8) {
#pragma unroll
        for (int c = 0; c < CPL; c += 8) {
          float f[8];
          unpack8<DT>(*reinterpret_cast<const uint4*>(p + n0 + c), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[c + e] = f[e];
        }
      } else {
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
          const uint2 v = *reinterpret_cast<const uint2*>(p + n0 + c);
          o[c] = to_f32<DT>((uint16_t)v.x); o[c + 1] = to_f32<DT>((uint16_t)(v.x >> 16));
          o[c + 2] = to_f32<DT>((uint16_t)v.y); o[c + 3] = to_f32<DT>((uint16_t)(v.y >> 16));
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < CPL; ++c) o[c] = n0 + c < n ? to_f32<DT>(p[n0 + c]) : 0.f;
    }
  }

  __device__ __forceinline__ void load_bias(const GemmArgs& g, int vcol0, int lane) {
    if constexpr (PRE) {
      const int ec = (lane & 3) * CPL;
      if (g.bias == nullptr) {
#pragma unroll
        for (int c = 0; c < (GATED ? 2 * CPL : CPL); ++c) bias[c] = 0.f;
        return;
      }
      const int n0 = GATED ? vcol0 / 2 + ec : vcol0 + ec;
      const bool vec = n0 + CPL <= g.N && (n0 & (VW - 1)) == 0 && (!GATED || (g.half & (VW - 1)) == 0);
      load16(g.bias, n0, g.N, vec, bias);
      if constexpr (GATED) load16(g.bias + g.half, n0, g.N, vec, bias + CPL);
    }
  }

  template <int B>
  __device__ __forceinline__ void load_res(const GemmArgs& g, int m, int vcol0, int lane) {
    if constexpr (RES) {
      const int n0 = vcol0 + (lane & 3) * CPL;
      if (m >= g.M) return;
      const bool vec = n0 + CPL <= g.N && ((g.ldr | n0) & (VW - 1)) == 0;
      load16(g.r16 + (size_t)m * g.ldr, n0, g.N, vec, res[B]);
    }
  }
};

// CPL 16-bit outputs of one lane: 16-byte stores (8-byte when CPL % 8 != 0: the 80-column
// wave tiles), element stores at the right edge (n valid columns) or misaligned rows
// (align = row stride | first column, in elements)
template <int CPL>
__device__ __forceinline__ void store16(uint16_t* dst, const uint16_t* v, bool full,
                                        long long align, int n) {
  constexpr int VW = CPL % 8 == 0 ? 8 : 4;
  if (full && (align & (VW - 1)) == 0) {
    if constexpr (CPL % 8 == 0) {
#pragma unroll
      for (int c = 0; c < CPL; c += 8)
        *reinterpret_cast<uint4*>(dst + c) = *reinterpret_cast<const uint4*>(v + c);
    } else {
#pragma unroll
      for (int c = 0; c < CPL; c += 4)
        *reinterpret_cast<uint2*>(dst + c) = *reinterpret_cast<const uint2*>(v + c);
    }
  } else {
    for (int c = 0; c < CPL; ++c) if (c < n) dst[c] = v[c];
  }
}

// One 16-row strip of a wave's output (NF 16x16 accumulator tiles = NF*16 virtual
// columns starting at vcol0), staged through the wave's LDS slice stg and written
// with the epilogue EPI (bias / residual from ops, buffer B).
// add (split-K pair, gemm_4w.h): this thread's parked partner accumulators of the strip,
// float4 j at add[j * 256], summed in before staging
template <int DT, int EPI, int NF, int B>
__device__ __forceinline__ void epi_strip(const GemmArgs& g, const cf32x4 (&tiles)[NF], float* stg,
                                          int m_strip0, int vcol0, int split, int lane,
                                          const EpiOps<DT, EPI, NF>& ops,
                                          const float4* add = nullptr) {
  constexpr int WTN = NF * 16;
  constexpr int STG_LD = WTN + 4;
  constexpr bool GATED = (EPI == kEpiSwiglu || EPI == kEpiGeglu);
  constexpr int OUTC = GATED ? WTN / 2 : WTN;  // output columns of this strip
  constexpr int CPL = OUTC / 4;                // columns per lane (4 lanes per row)
  const int er = lane >> 2, ec = (lane & 3) * CPL;
  {
    if (add) {
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const float4 o = add[j * 256];
        const float ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          stg[((lane >> 4) * 4 + e) * STG_LD + j * 16 + (lane & 15)] = tiles[j][e] + ov[e];
      }
    } else {
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          stg[((lane >> 4) * 4 + e) * STG_LD + j * 16 + (lane & 15)] = tiles[j][e];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int m = m_strip0 + er;
    if (m < g.M) {
      const float* srow = stg + er * STG_LD;
      if constexpr (EPI == kEpiPartial) {
        float* dst = g.ws + ((size_t)split * g.M + m) * g.Nv;
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
          const int n = vcol0 + ec + c;
          const float4 v = *reinterpret_cast<const float4*>(srow + ec + c);
          if (n + 3 < g.Nv) *reinterpret_cast<float4*>(dst + n) = v;
          else {
            const float vv[4] = {v.x, v.y, v.z, v.w};
            for (int q = 0; q < 4; ++q) if (n + q < g.Nv) dst[n + q] = vv[q];
          }
        }
      } else if constexpr (GATED) {
        // output column f of this lane: virtual cols (32-block b): gate at 32b + c, up at 32b + 16 + c
        const int f0 = vcol0 / 2 + ec;  // vcol0 is a multiple of 32
        uint16_t outv[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int lc = ec + c;                           // output col within the wave
          const int vc = (lc >> 4) * 32 + (lc & 15);       // gate's staged column
          const float a = srow[vc] + ops.bias[c], b = srow[vc + 16] + ops.bias[CPL + c];
          float y;
          if constexpr (EPI == kEpiSwiglu) y = silu(a) * b;
          else y = a * gelu_tanh(b);
          outv[c] = from_f32<DT>(y);
        }
        store16<CPL>(g.c + (size_t)m * g.ldc + f0, outv, f0 + CPL <= g.N, g.ldc | f0, g.N - f0);
      } else {
        const int n0c = vcol0 + ec;
        float v[CPL];
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
          const float4 t4 = *reinterpret_cast<const float4*>(srow + ec + c);
          v[c] = t4.x; v[c + 1] = t4.y; v[c + 2] = t4.z; v[c + 3] = t4.w;
        }
        const bool full = n0c + CPL <= g.N;
        if constexpr (EpiOps<DT, EPI, NF>::PRE) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) v[c] += ops.bias[c];
        } else if (g.bias != nullptr) {
#pragma unroll
          for (int c = 0; c < CPL; ++c)
            if (full || n0c + c < g.N) v[c] += to_f32<DT>(g.bias[n0c + c]);
        }
        if constexpr (EPI == kEpiResid32 || EPI == kEpiStore32) {
          constexpr bool ADD = EPI == kEpiResid32;
          float* r = g.r32 + (size_t)m * g.ldr + n0c;
          if (full && ((g.ldr | n0c) & 3) == 0) {
#pragma unroll
            for (int c = 0; c < CPL; c += 4) {
              float4 o = ADD ? *reinterpret_cast<float4*>(r + c) : make_float4(0.f, 0.f, 0.f, 0.f);
              o.x += v[c]; o.y += v[c + 1]; o.z += v[c + 2]; o.w += v[c + 3];
              *reinterpret_cast<float4*>(r + c) = o;
            }
          } else {
            for (int c = 0; c < CPL; ++c)
              if (n0c + c < g.N) r[c] = ADD ? r[c] + v[c] : v[c];
          }
        } else {
          if constexpr (EPI == kEpiAdd16) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) v[c] += ops.res[B][c];
          }
          if constexpr (EPI == kEpiSilu) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) v[c] = gemm_act(g.act, v[c]);
          }
          uint16_t outv[CPL];
#pragma unroll
          for (int c = 0; c < CPL; ++c) outv[c] = from_f32<DT>(v[c]);
          store16<CPL>(g.c + (size_t)m * g.ldc + n0c, outv, full, g.ldc | n0c, g.N - n0c);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // strip consumed before the next one overwrites it
  }
}

// Wide read-out: a strip (16 rows x the wave's columns) staged through LDS as above, then
// read out LPR lanes per row (8 when an output row is whole 128-byte lines, else 4), a
// lane's 16-byte (80-column tiles: 8-byte) chunks interleaved with its row neighbours'
// (chunk c of lane q at output column (LPR c + q) x the chunk's elements), so a store
// instruction covers each row it touches with one contiguous run (8 rows x 128 B on the
// 64 / 128-column tiles).  epi_strip's read-out (4 lanes per row, CPL contiguous columns
// each) wrote 16-32 bytes into each of up to 32 lines per instruction: the four-wave tile's
// stores took 12-24 % of its time (profiles/r6_gemm_stamps.jsonl).
template <int DT, int EPI, int NF> struct EpiW {
  static constexpr int WTN = NF * 16;
  static constexpr bool GATED = (EPI == kEpiSwiglu || EPI == kEpiGeglu);
  static constexpr bool F32 = (EPI == kEpiResid32 || EPI == kEpiStore32 || EPI == kEpiPartial);
  static constexpr int OUTC = GATED ? WTN / 2 : WTN;  // output columns of a strip
  static constexpr int ESZ = F32 ? 4 : 2;
  static constexpr int ROWB = OUTC * ESZ;             // bytes of one output row of a strip
  // 8 lanes per row when the row is whole 128-byte lines, else 4; 16-byte chunks when a
  // row splits into them evenly over its lanes, else 8-byte (the 80-column tiles)
  static constexpr int LPR = ROWB % 128 == 0 ? 8 : 4;
  static constexpr int CB = ROWB % (LPR * 16) == 0 ? 16 : 8;
  static constexpr int CE = CB / ESZ;                 // output elements per chunk
  static constexpr int NCH = ROWB / (LPR * CB);       // a lane's chunks per row
  static constexpr int CPL = NCH * CE;                // a lane's columns per row
  static constexpr int RPP = 64 / LPR;                // rows per read-out pass
  static constexpr int NP = 16 / RPP;                 // passes per 16-row strip
  static constexpr bool OK = ROWB % (LPR * CB) == 0 && CE >= 4 && (!F32 || CE == 4);
  static constexpr bool RES = EPI == kEpiAdd16;
  static constexpr bool PRE = (EPI == kEpiAdd16 || GATED);
  float bias[PRE ? (GATED ? 2 * CPL : CPL) : 1];
  float res[2][RES ? NP * CPL : 1];  // [buffer][pass x CPL]

  __device__ __forceinline__ static int col(int lane, int c) {
    return (c * LPR + lane % LPR) * CE;
  }
  __device__ __forceinline__ static int row(int lane, int p) { return lane / LPR + RPP * p; }

  // CE (4 / 8) 16-bit values at p + n (columns < lim valid) as f32
  __device__ __forceinline__ static void loadc(const uint16_t* p, int n, int lim, bool vec,
                                               float* o) {
    if (vec && n + CE <= lim) {
      if constexpr (CE == 8) {
        unpack8<DT>(*reinterpret_cast<const uint4*>(p + n), o);
      } else {
        const uint2 v = *reinterpret_cast<const uint2*>(p + n);
        o[0] = to_f32<DT>((uint16_t)v.x); o[1] = to_f32<DT>((uint16_t)(v.x >> 16));
        o[2] = to_f32<DT>((uint16_t)v.y); o[3] = to_f32<DT>((uint16_t)(v.y >> 16));
      }
    } else {
#pragma unroll
      for (int e = 0; e < CE; ++e) o[e] = n + e < lim ? to_f32<DT>(p[n + e]) : 0.f;
    }
  }

  __device__ __forceinline__ void load_bias(const GemmArgs& g, int vcol0, int lane) {
    if constexpr (PRE) {
      if (g.bias == nullptr) {
#pragma unroll
        for (int c = 0; c < (GATED ? 2 * CPL : CPL); ++c) bias[c] = 0.f;
        return;
      }
      const int base = GATED ? vcol0 / 2 : vcol0;
      const bool vec = (base & (CE - 1)) == 0 && (!GATED || (g.half & (CE - 1)) == 0);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        loadc(g.bias, base + col(lane, c), g.N, vec, bias + c * CE);
        if constexpr (GATED)
          loadc(g.bias + g.half, base + col(lane, c), g.N, vec, bias + CPL + c * CE);
      }
    }
  }

  // the add16 residual of this lane's rows of a strip
  template <int B>
  __device__ __forceinline__ void load_res(const GemmArgs& g, int m0, int vcol0, int lane) {
    if constexpr (RES) {
      const bool vec = ((g.ldr | vcol0) & (CE - 1)) == 0;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int m = m0 + row(lane, p);
        if (m >= g.M) continue;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          loadc(g.r16 + (size_t)m * g.ldr, vcol0 + col(lane, c), g.N, vec, res[B] + p * CPL + c * CE);
      }
    }
  }
};

// a strip's accumulators (+ the split-K partner's, add) into the wave's staging slice
template <int NF>
__device__ __forceinline__ void stage_strip_w(const cf32x4 (&tiles)[NF], float* stg, int lane,
                                              const float4* add) {
  constexpr int STG_LD = NF * 16 + 4;
  if (add) {
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const float4 o = add[j * 256];
      const float ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        stg[((lane >> 4) * 4 + e) * STG_LD + j * 16 + (lane & 15)] = tiles[j][e] + ov[e];
    }
  } else {
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        stg[((lane >> 4) * 4 + e) * STG_LD + j * 16 + (lane & 15)] = tiles[j][e];
  }
}

// a staged strip read out 8 lanes per row and written with the epilogue EPI
template <int DT, int EPI, int NF, int B>
__device__ __forceinline__ void readout_strip_w(const GemmArgs& g, const float* stg, int m_strip0,
                                                int vcol0, int split, int lane,
                                                const EpiW<DT, EPI, NF>& ops) {
  using W = EpiW<DT, EPI, NF>;
  constexpr int STG_LD = NF * 16 + 4;
  constexpr int CE = W::CE;
  // resid32: every chunk's residual requested before the first add / store (one memory
  // round trip per strip, not one per chunk: the stores could alias later loads)
  constexpr bool R32 = EPI == kEpiResid32;
  float4 rold[R32 ? W::NP : 1][R32 ? W::NCH : 1];
  if constexpr (R32) {
#pragma unroll
    for (int p = 0; p < W::NP; ++p) {
      const int m = m_strip0 + W::row(lane, p);
#pragma unroll
      for (int c = 0; c < W::NCH; ++c) {
        const int n = vcol0 + W::col(lane, c);
        rold[p][c] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < g.M && n + 4 <= g.N && ((g.ldr | n) & 3) == 0)
          rold[p][c] = *reinterpret_cast<const float4*>(g.r32 + (size_t)m * g.ldr + n);
      }
    }
  }
#pragma unroll
  for (int p = 0; p < W::NP; ++p) {
    const int row = W::row(lane, p);
    const int m = m_strip0 + row;
    if (m >= g.M) continue;
    const float* srow = stg + row * STG_LD;
#pragma unroll
    for (int c = 0; c < W::NCH; ++c) {
      const int lc = W::col(lane, c);  // output column within the wave's strip
      if constexpr (EPI == kEpiPartial) {
        float* dst = g.ws + ((size_t)split * g.M + m) * g.Nv;
        const int n = vcol0 + lc;
        const float4 v = *reinterpret_cast<const float4*>(srow + lc);
        if (n + 3 < g.Nv) *reinterpret_cast<float4*>(dst + n) = v;
        else {
          const float vv[4] = {v.x, v.y, v.z, v.w};
          for (int q = 0; q < 4; ++q) if (n + q < g.Nv) dst[n + q] = vv[q];
        }
      } else if constexpr (W::GATED) {
        const int f0 = vcol0 / 2 + lc;
        const int vc = (lc >> 4) * 32 + (lc & 15);  // the gate's staged column
        uint16_t outv[CE];
#pragma unroll
        for (int e = 0; e < CE; ++e) {
          const float a = srow[vc + e] + ops.bias[c * CE + e];
          const float b = srow[vc + 16 + e] + ops.bias[W::CPL + c * CE + e];
          float y;
          if constexpr (EPI == kEpiSwiglu) y = silu(a) * b;
          else y = a * gelu_tanh(b);
          outv[e] = from_f32<DT>(y);
        }
        store16<CE>(g.c + (size_t)m * g.ldc + f0, outv, f0 + CE <= g.N, g.ldc | f0, g.N - f0);
      } else if constexpr (W::F32) {
        const int n = vcol0 + lc;
        const float4 t = *reinterpret_cast<const float4*>(srow + lc);
        float v[4] = {t.x, t.y, t.z, t.w};
        if (g.bias != nullptr)
#pragma unroll
          for (int e = 0; e < 4; ++e) if (n + e < g.N) v[e] += to_f32<DT>(g.bias[n + e]);
        float* r = g.r32 + (size_t)m * g.ldr + n;
        if (n + 4 <= g.N && ((g.ldr | n) & 3) == 0) {
          float4 o = R32 ? rold[R32 ? p : 0][R32 ? c : 0] : make_float4(0.f, 0.f, 0.f, 0.f);
          o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
          *reinterpret_cast<float4*>(r) = o;
        } else {
          constexpr bool ADD = R32;
          for (int e = 0; e < 4; ++e)
            if (n + e < g.N) r[e] = ADD ? r[e] + v[e] : v[e];
        }
      } else {
        const int n = vcol0 + lc;
        float v[CE];
#pragma unroll
        for (int e = 0; e < CE; e += 4) {
          const float4 t = *reinterpret_cast<const float4*>(srow + lc + e);
          v[e] = t.x; v[e + 1] = t.y; v[e + 2] = t.z; v[e + 3] = t.w;
        }
        if constexpr (W::PRE) {
#pragma unroll
          for (int e = 0; e < CE; ++e) v[e] += ops.bias[c * CE + e];
        } else if (g.bias != nullptr) {
#pragma unroll
          for (int e = 0; e < CE; ++e) if (n + e < g.N) v[e] += to_f32<DT>(g.bias[n + e]);
        }
        if constexpr (EPI == kEpiAdd16) {
#pragma unroll
          for (int e = 0; e < CE; ++e) v[e] += ops.res[B][p * W::CPL + c * CE + e];
        }
        if constexpr (EPI == kEpiSilu) {
#pragma unroll
          for (int e = 0; e < CE; ++e) v[e] = gemm_act(g.act, v[e]);
        }
        uint16_t outv[CE];
#pragma unroll
        for (int e = 0; e < CE; ++e) outv[e] = from_f32<DT>(v[e]);
        store16<CE>(g.c + (size_t)m * g.ldc + n, outv, n + CE <= g.N, g.ldc | n, g.N - n);
      }
    }
  }
}


// PR bit 0: s_setprio(1) around the MFMA clusters; bit 1: AGPR-pinned accumulators;
// bit 2: interleaved schedule (needs bit 1)
template <int DT, int BM, int BN, int WM, int WN, int NS, int EPI, int PR>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(GemmArgs g) {
  constexpr bool AG = (PR & 2) != 0;
  constexpr bool IL = (PR & 4) != 0;
  static_assert(!IL || AG, "the interleaved schedule pins AGPR-accumulator MFMAs");
  constexpr int NT = 64 * WM * WN;
  constexpr int NWAVE = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // per-wave tile
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int ROWS = BM + BN;                // 128-byte rows per k-step
  constexpr int IPW = ROWS / 8 / NWAVE;        // DMA wave-instructions per wave per k-step
  constexpr int BUF = ROWS * 128;              // bytes per LDS buffer
  static_assert(ROWS % (8 * NWAVE) == 0 && BM % 16 == 0 && BN % 32 == 0, "tile geometry");
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile geometry");
  static_assert(WTN % 32 == 0 || !(EPI == kEpiSwiglu || EPI == kEpiGeglu),
                "gated epilogues pair 16-column blocks within a wave");
  constexpr int STG_LD = WTN + 4;              // epilogue staging row stride (floats)
  constexpr int STG = 16 * STG_LD * 4;         // bytes per wave
  constexpr int LDS_BYTES = (NS * BUF > NWAVE * STG) ? NS * BUF : NWAVE * STG;
  static_assert(NS == 2 || NS == 3 || (IL && NS == 4), "LDS stages");
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / WN, wc = wave % WN;

  // ---- XCD-aware grouped tile order --------------------------------------
  const int ntiles = g.tiles_m * g.tiles_n;
  const int bid = blockIdx.x;
  int id;
  {
    const int q = ntiles / 8, r = ntiles % 8, x = bid % 8, i = bid / 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;  // bijective undealing
  }
  constexpr int GROUP = 8;
  const int per_group = GROUP * g.tiles_n;
  const int grp = id / per_group;
  const int first_m = grp * GROUP;
  const int gm = min(GROUP, g.tiles_m - first_m);
  const int tm = first_m + (id % per_group) % gm;
  const int tn = (id % per_group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.y;
  const int kb = split * g.kps, ke = min(g.K, kb + g.kps);
  const int nk = (ke - kb + kGBK - 1) / kGBK;

  // ---- DMA sources of this lane (fixed rows; k advances) -----------------
  // Precomputed per instruction, or (LAZY: many DMA instructions per wave, where the
  // pointer array would crowd out the accumulators) recomputed at each issue.
  constexpr bool LAZY = IL && IPW > 8;
  constexpr int NSRC = LAZY ? 1 : IPW;
  const uint16_t* src[NSRC];
  int chunk[NSRC];
  auto row_src = [&](int i, int& ch) __attribute__((always_inline)) -> const uint16_t* {
    int t = (wave * IPW + i) * 8 + (lane >> 3);  // tile row (A rows, then B rows)
    if constexpr (LAZY) asm volatile("" : "+v"(t));  // recompute per issue: no hoisting
    ch = (lane & 7) ^ ((t >> 1) & 7);
    if (t < BM) {
      const int m = m0 + t;
      return m < g.M ? g.a + (size_t)m * g.lda : nullptr;
    }
    const int v = n0 + (t - BM);
    return v < g.Nv ? g.b + (size_t)wrow(g, v) * g.ldb : nullptr;
  };
  if constexpr (!LAZY) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) src[i] = row_src(i, chunk[i]);
  }
  const uint32_t lds0 = lds_off(smem);
  auto stage_one = [&](int step, int buf, int i) __attribute__((always_inline)) {
    const uint16_t* s0;
    int ch;
    if constexpr (LAZY) {
      s0 = row_src(i, ch);
    } else {
      s0 = src[i];
      ch = chunk[i];
    }
    const int k = kb + step * kGBK + ch * 8;
    const uint16_t* p = (s0 != nullptr && k < ke) ? s0 + k : g.zeros;
    glds16(p, smem + buf * BUF + (wave * IPW + i) * 1024);
  };
  auto stage = [&](int step, int buf) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) stage_one(step, buf, i);
  };

  // ---- fragment addresses: row (lane & 15) of a 16-row group, slot swizzled
  const int swz = (lane & 15) >> 1;
  const uint32_t lrow = (uint32_t)(lane & 15) * 128;
  const uint32_t off0 = (uint32_t)((((lane >> 4)) ^ swz) * 16);      // k 0..31
  const uint32_t off1 = (uint32_t)(((4 + (lane >> 4)) ^ swz) * 16);  // k 32..63
  const uint32_t a_base = lds0 + (uint32_t)(wr * WTM) * 128 + lrow;
  const uint32_t b_base = lds0 + (uint32_t)(BM + wc * WTN) * 128 + lrow;

  cf32x4 acc[FM][FN];
  if constexpr (AG) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) azero(acc[i][j]);
  } else {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto mma = [&](cf32x4& c, const uint4& a, const uint4& b) {
    if constexpr (AG) amfma<DT>(c, a, b);
    else c = cmfma<DT>(a, b, c);
  };

  // One barrier per k-step, placed between the k 0..31 and k 32..63 halves so
  // that LDS latency never sits in front of the MFMAs:
  //   [kk1 reads of t] [kk0 MFMAs of t] wait | vmcnt(DMA t+1) barrier
  //   [DMA t+NS into t's buffer] [kk0 reads of t+1] [kk1 MFMAs of t] wait
  // The barrier publishes every wave's DMA of step t+1 and proves every wave
  // finished reading step t's buffer (its kk1 reads completed before it), so
  // the DMA issued right after it may overwrite that buffer.
  uint4 af0[FM], bf0[FN], af1[FM], bf1[FN];
  if constexpr (IL) {
    // Same pipeline as below, with every LDS read and DMA issued BETWEEN the MFMAs
    // (program order pinned: volatile MFMAs and reads) instead of in bursts in
    // front of them, so the matrix pipe never idles while a wave issues its
    // loads.  Every step issues exactly IPW DMAs (past the end: the zeros page
    // into the consumed buffer) so the counted waits are the same every step.
    constexpr int NM = FM * FN, NR = FM + FN, NL = IPW + NR;
    if (nk > 0) {
#pragma unroll
      for (int p = 0; p + 1 < NS; ++p) stage(p, p);
      __builtin_amdgcn_s_waitcnt(vm_wait((NS - 2) * IPW));
      asm volatile("s_barrier" ::: "memory");
      stage(NS - 1, NS - 1);
#pragma unroll
      for (int i = 0; i < FM; ++i) af0[i] = ds_read16(a_base + i * 16 * 128 + off0);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf0[j] = ds_read16(b_base + j * 16 * 128 + off0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    int buf = 0;
    for (int t = 0; t < nk; ++t) {
      const uint32_t ab = a_base + buf * BUF, bb = b_base + buf * BUF;
      // load r goes after MFMA floor(r * NM / NR)
      static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
        constexpr int m = decltype(mi)::value;
        amfma_v<DT>(acc[m / FN][m % FN], af0[m / FN], bf0[m % FN]);
        static_for<(m * NR + NM - 1) / NM, ((m + 1) * NR + NM - 1) / NM>([&](auto ri)
                                                                      __attribute__((always_inline)) {
          constexpr int r = decltype(ri)::value;
          if constexpr (r < FM) af1[r] = ds_read16_off<r * 16 * 128>(ab + off1);
          else bf1[r - FM] = ds_read16_off<(r - FM) * 16 * 128>(bb + off1);
        });
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int nbuf = buf + 1 == NS ? 0 : buf + 1;
      __builtin_amdgcn_s_waitcnt(vm_wait((NS - 2) * IPW));  // DMA of step t+1 landed
      asm volatile("s_barrier" ::: "memory");
      const uint32_t na = a_base + nbuf * BUF, nb = b_base + nbuf * BUF;
      static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
        constexpr int m = decltype(mi)::value;
        amfma_v<DT>(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN]);
        static_for<(m * NL + NM - 1) / NM, ((m + 1) * NL + NM - 1) / NM>([&](auto li)
                                                                      __attribute__((always_inline)) {
          constexpr int l = decltype(li)::value;
          if constexpr (l < IPW) {
            stage_one(t + NS, buf, l);
          } else {
            constexpr int r = l - IPW;
            if constexpr (r < FM) af0[r] = ds_read16_off<r * 16 * 128>(na + off0);
            else bf0[r - FM] = ds_read16_off<(r - FM) * 16 * 128>(nb + off0);
          }
        });
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      buf = nbuf;
    }
  } else {
  if (nk > 0) stage(0, 0);
  if (NS == 3 && nk > 1) stage(1, 1);
  if (nk > 0) {
    if (NS == 3 && nk > 1) __builtin_amdgcn_s_waitcnt(vm_wait(IPW));
    else __builtin_amdgcn_s_waitcnt(vm_wait(0));
    asm volatile("s_barrier" ::: "memory");
    if (NS - 1 < nk) stage(NS - 1, NS - 1);
#pragma unroll
    for (int i = 0; i < FM; ++i) af0[i] = ds_read16(a_base + i * 16 * 128 + off0);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf0[j] = ds_read16(b_base + j * 16 * 128 + off0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  int buf = 0;
  for (int t = 0; t < nk; ++t) {
    const uint32_t ab = a_base + buf * BUF, bb = b_base + buf * BUF;
#pragma unroll
    for (int i = 0; i < FM; ++i) af1[i] = ds_read16(ab + i * 16 * 128 + off1);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf1[j] = ds_read16(bb + j * 16 * 128 + off1);
    if (PR & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mma(acc[i][j], af0[i], bf0[j]);
    if (PR & 1) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int nbuf = buf + 1 == NS ? 0 : buf + 1;
    if (t + 1 < nk) {
      // DMAs still allowed in flight: step t+2's (3 stages, issued last iteration)
      if (NS == 3 && t + 2 < nk) __builtin_amdgcn_s_waitcnt(vm_wait(IPW));
      else __builtin_amdgcn_s_waitcnt(vm_wait(0));
      asm volatile("s_barrier" ::: "memory");
      if (t + NS < nk) stage(t + NS, buf);
      const uint32_t na = a_base + nbuf * BUF, nb = b_base + nbuf * BUF;
#pragma unroll
      for (int i = 0; i < FM; ++i) af0[i] = ds_read16(na + i * 16 * 128 + off0);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf0[j] = ds_read16(nb + j * 16 * 128 + off0);
    }
    if (PR & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mma(acc[i][j], af1[i], bf1[j]);
    if (PR & 1) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    buf = nbuf;
  }
  }

  // ---- epilogue: 16-row strips staged through this wave's LDS slice --------
  if constexpr (AG) {  // MFMA D -> VALU read: >= 12 wait states after the last MFMA
#pragma unroll
    for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
  }
  __builtin_amdgcn_s_waitcnt(vm_wait(0));
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float* stg = reinterpret_cast<float*>(smem + wave * STG);
  const int row_m0 = m0 + wr * WTM;
  const int vcol0 = n0 + wc * WTN;  // first virtual column of this wave
  if constexpr (EpiW<DT, EPI, FN>::OK) {  // wide read-out (every tile shape in use)
    EpiW<DT, EPI, FN> ops;
    ops.load_bias(g, vcol0, lane);
    ops.template load_res<0>(g, row_m0, vcol0, lane);
    static_for<0, FM>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      if constexpr (i + 1 < FM) ops.template load_res<(i + 1) & 1>(g, row_m0 + (i + 1) * 16, vcol0, lane);
      stage_strip_w<FN>(acc[i], stg, lane, nullptr);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      readout_strip_w<DT, EPI, FN, i & 1>(g, stg, row_m0 + i * 16, vcol0, split, lane, ops);
      __builtin_amdgcn_wave_barrier();  // strip consumed before the next one overwrites it
    });
  } else {
    EpiOps<DT, EPI, FN> ops;
    ops.load_bias(g, vcol0, lane);
    ops.template load_res<0>(g, row_m0 + (lane >> 2), vcol0, lane);
    static_for<0, FM>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      // the next strip's residual goes out before this strip's stores
      if constexpr (i + 1 < FM) ops.template load_res<(i + 1) & 1>(g, row_m0 + (i + 1) * 16 + (lane >> 2), vcol0, lane);
      epi_strip<DT, EPI, FN, i & 1>(g, acc[i], stg, row_m0 + i * 16, vcol0, split, lane, ops);
    });
  }
}

// Split-K finalize: out = epilogue(sum over splits of the slabs).  One thread
// per 4 output columns of one row.
template <int DT, int EPI>
__global__ __launch_bounds__(256) void gemm_splitk_finalize(GemmArgs g, int splits) {
  const int m = blockIdx.y;
  const int f = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (f >= g.N) return;
  const size_t slab = (size_t)g.M * g.Nv;
  float v[4] = {0.f, 0.f, 0.f, 0.f}, u[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr bool GATED = (EPI == kEpiSwiglu || EPI == kEpiGeglu);
  for (int s = 0; s < splits; ++s) {
    const float* row = g.ws + s * slab + (size_t)m * g.Nv;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int fq = f + q;
      if (fq >= g.N) break;
      if constexpr (GATED) {
        const int vc = (fq >> 4) * 32 + (fq & 15);
        v[q] += row[vc];
        u[q] += row[vc + 16];
      } else {
        v[q] += row[fq];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int fq = f + q;
    if (fq >= g.N) break;
    float y;
    if constexpr (GATED) {
      if (g.bias != nullptr) {
        v[q] += to_f32<DT>(g.bias[fq]);
        u[q] += to_f32<DT>(g.bias[g.half + fq]);
      }
    }
    if constexpr (EPI == kEpiSwiglu) y = silu(v[q]) * u[q];
    else if constexpr (EPI == kEpiGeglu) y = v[q] * gelu_tanh(u[q]);
    else {
      y = v[q] + (g.bias != nullptr ? to_f32<DT>(g.bias[fq]) : 0.f);
      if constexpr (EPI == kEpiAdd16) y += to_f32<DT>(g.r16[(size_t)m * g.ldr + fq]);
      if constexpr (EPI == kEpiSilu) y = gemm_act(g.act, y);
    }
    if constexpr (EPI == kEpiResid32) g.r32[(size_t)m * g.ldr + fq] += y;
    else if constexpr (EPI == kEpiStore32) g.r32[(size_t)m * g.ldr + fq] = y;
    else g.c[(size_t)m * g.ldc + fq] = from_f32<DT>(y);
  }
}


// tile configurations (BM, BN, WM, WN, LDS stages, PR flags).  Measured
// (profiles/r2_gemm_sweep_agpr.jsonl, r2_gemm_sweep_il.jsonl): AGPR-pinned
// accumulators +10-20 % on the 4-wave tiles, the interleaved schedule a further
// +5-13 % on every tile (8-wave 256x256: 1144 -> 1286 TFLOP/s at 8192^3); 8 and 11
// are the non-interleaved forms kept for A/B; a 4-wave 256x256 tile (128x128
// per wave; with or without the interleaved schedule: 0.5x of tile 5), an 8-phase
// staggered-wave-group 256x256 tile (0.74x of tile 5, profiles/r2_gemm_8phase_rejected.jsonl)
// and s_setprio measured slower / neutral and were dropped.  14-19: 160-column tiles, whose
// grids fill the 256 CUs exactly on the SD widths (640 / 1280 = 4 / 8 x 160: 2048 x 1280 at
// 64 x 160 and 8192 x 640 at 128 x 160 are 256 tiles) at a higher operand reuse per tile
// than 64 x 64 (45.7 / 71 FLOP per staged byte against 32).
#define CAKE_GEMM_CFGS(X)    \
  X(0, 128, 128, 2, 2, 2, 6) \
  X(1, 64, 128, 1, 4, 2, 6)  \
  X(2, 256, 128, 2, 2, 3, 6) \
  X(3, 128, 256, 2, 2, 3, 6) \
  X(4, 64, 64, 2, 2, 2, 6)   \
  X(5, 256, 256, 2, 4, 2, 6) \
  X(6, 256, 128, 4, 2, 3, 6) \
  X(7, 128, 128, 2, 2, 3, 6) \
  X(8, 128, 128, 2, 2, 2, 2) \
  X(11, 256, 256, 2, 4, 2, 0) \
  X(12, 64, 128, 1, 4, 3, 6) \
  X(13, 64, 64, 2, 2, 4, 6)  \
  X(14, 64, 160, 2, 2, 2, 6) \
  X(15, 64, 160, 4, 1, 2, 6) \
  X(16, 128, 160, 4, 1, 2, 6) \
  X(17, 128, 160, 2, 2, 2, 6) \
  X(18, 64, 160, 2, 2, 3, 6) \
  X(19, 128, 160, 2, 2, 3, 6)

}  // namespace cake

#include "gemm_pp.h"
#include "gemm_rs.h"
#include "gemm_4w.h"

namespace cake {

template <int EPI>
constexpr bool gated_ok(int wave_cols) {
  return wave_cols % 32 == 0 || !(EPI == kEpiSwiglu || EPI == kEpiGeglu);
}

template <int DT, int EPI>
int launch_gemm(int cfg, dim3 grid, hipStream_t st, const GemmArgs& g) {
  if (cfg == kPPCfg) {
    hipLaunchKernelGGL((gemm_pp_kernel<DT, EPI>), grid, dim3(512), 0, st, g);
    return (int)hipGetLastError();
  }
  if (cfg == kRSCfg) {
    hipLaunchKernelGGL((gemm_rs_kernel<DT, EPI>), grid, dim3(256), 0, st, g);
    return (int)hipGetLastError();
  }
  if (cfg == k4WCfg) {
    hipLaunchKernelGGL((gemm_4w_kernel<DT, EPI, 256, 256>), grid, dim3(256), 0, st, g);
    return (int)hipGetLastError();
  }
  if (cfg == k4WCfg192) {
    hipLaunchKernelGGL((gemm_4w_kernel<DT, EPI, 256, 192>), grid, dim3(256), 0, st, g);
    return (int)hipGetLastError();
  }
  if (cfg == k4WCfg128) {
    hipLaunchKernelGGL((gemm_4w_kernel<DT, EPI, 128, 256>), grid, dim3(256), 0, st, g);
    return (int)hipGetLastError();
  }
  if (cfg == k4WCfg + k4WSched) {
    hipLaunchKernelGGL((gemm_4w_kernel<DT, EPI, 256, 256, 1>), grid, dim3(256), 0, st, g);
    return (int)hipGetLastError();
  }
  if (cfg == k4WCfg192 + k4WSched) {
    hipLaunchKernelGGL((gemm_4w_kernel<DT, EPI, 256, 192, 1>), grid, dim3(256), 0, st, g);
    return (int)hipGetLastError();
  }
  if (cfg == k4WCfg128 + k4WSched) {
    hipLaunchKernelGGL((gemm_4w_kernel<DT, EPI, 128, 256, 1>), grid, dim3(256), 0, st, g);
    return (int)hipGetLastError();
  }

#define X(id, BM, BN, WM, WN, NS, PR)                                                        \
  if (cfg == id) {                                                                           \
    if constexpr (gated_ok<EPI>(BN / WN)) {                                                  \
      hipLaunchKernelGGL((gemm_kernel<DT, BM, BN, WM, WN, NS, EPI, PR>), grid,               \
                         dim3(64 * WM * WN), 0, st, g);                                      \
      return (int)hipGetLastError();                                                        \
    } else {                                                                                 \
      return (int)hipErrorInvalidValue;                                                      \
    }                                                                                        \
  }
  CAKE_GEMM_CFGS(X)
#undef X
  return (int)hipErrorInvalidValue;
}

}  // namespace cake
