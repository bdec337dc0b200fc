// KV-cached GQA decode attention (flash-decoding split-K).
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
//   * Decode is flash-decoding with the split count chosen on device from the
//     live length (so one captured launch serves every position): each
//     workgroup streams its key range in 64-key chunks, computes a local
//     softmax and P·V in f32, and the last-arriving split merges the
//     (max, sum, o[hd]) partials (one launch per layer).
//   * Prefill attention is the MFMA flash kernel (flash_attn.hip).
#include "common.h"

namespace cake {

// ---------------------------------------------------------------------------
// decode (flash-decoding, split-K over the live context)
// ---------------------------------------------------------------------------
// Grid (nkv, maxsplit).  One workgroup = (kv head g, split s) and runs all
// NREP query heads of the GQA group (one wave each), so every K/V byte is read
// from HBM once per token.  The number of live splits is derived ON DEVICE from
// the live length Tk = pos + 1 (the launch is graph-replayed at every
// position): ns = min(maxsplit, ceil(Tk / min_keys)); each split owns a
// contiguous range of whole 64-key chunks.  Chunks are streamed
// global -> registers (every load of the next chunk is issued before the
// current chunk is computed) -> LDS (K rows padded 16 B: conflict-free
// row-per-lane ds_read_b128).  Per wave: lane j scores key j, online softmax
// in base 2 (scale * log2 e folded into q), P·V with lanes over head dims.
//
// Combine: splits publish (m, l, o[HD]) with write-through (sc1) stores, drain
// (vmcnt 0), barrier, then one relaxed agent-scope ticket add per workgroup;
// the workgroup whose add returns ns - 1 reads every partial with sc1 loads
// (MI355X_MICROARCH "Valid forms", row 1) and writes the head outputs.  ns == 1
// (short contexts) writes the output directly.
constexpr int kChunk = 64;        // keys per LDS chunk (one per lane)
constexpr int kMaxSplit = 64;     // splits per kv head (partials merged lane-parallel)
static int g_attn_min_keys = 64;  // min keys per split (tunable)

template <int NREP> struct AttnGeom {
  static constexpr int NW = NREP < 4 ? 4 : NREP;  // waves (>= 4 so loads stay wide)
  static constexpr int NT = 64 * NW;
};

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int DT, int HD, int NREP>
__global__ __launch_bounds__(AttnGeom<NREP>::NT) void attn_decode_kernel(
    const float* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int* __restrict__ pos_ptr, int S, float scale_log2,
    float* __restrict__ part, unsigned int* __restrict__ tickets, uint16_t* __restrict__ out,
    int min_keys) {
  constexpr int NT = AttnGeom<NREP>::NT;
  constexpr int NW = AttnGeom<NREP>::NW;
  constexpr int DPL = HD / 64;              // output dims per lane
  constexpr int CPR = HD / 8;               // 16-byte pieces per row
  constexpr int PIECES = kChunk * CPR;      // pieces per chunk (each of K and V)
  constexpr int IPW = PIECES / 64 / NW;     // LDS-DMA wave-instructions per wave (each of K, V)
  static_assert(IPW >= 1 && PIECES % (64 * NW) == 0, "chunk/wave geometry");
  // one LDS array (LDS-DMA pipelines need it: MI355X guide, GEMM item 4a):
  // [2 buffers][K chunk | V chunk] 16-bit, then q (f32, pre-scaled), then p rows
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * PIECES * 8 + NREP * HD * 2 +
                                                        NREP * kChunk * 2 + 2];
  float* qs = reinterpret_cast<float*>(smem + 2 * 2 * PIECES * 8);
  float* ps = qs + NREP * HD;
  unsigned int& last_flag = *reinterpret_cast<unsigned int*>(ps + NREP * kChunk);

  const int g = blockIdx.x, s = blockIdx.y;
  const int Tk = *pos_ptr + 1;
  int ns = (Tk + min_keys - 1) / min_keys;
  if (ns > (int)gridDim.y) ns = gridDim.y;
  int kps = (Tk + ns - 1) / ns;
  kps = (kps + kChunk - 1) / kChunk * kChunk;
  ns = (Tk + kps - 1) / kps;
  if (s >= ns) return;
  const int kb = s * kps, ke = min(Tk, kb + kps);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;


  const uint16_t* kg = kc + (size_t)g * S * HD;
  const uint16_t* vg = vc + (size_t)g * S * HD;
  // Stage chunk [c0, c0 + 64) into buffer b.  LDS piece P (row P / CPR, slot
  // P % CPR) of K holds key piece slot ^ (row % CPR): an XOR swizzle applied on
  // the SOURCE address (the DMA writes lane-linear), so the row-per-lane
  // ds_read_b128 of the scores is conflict-free.  V stays linear.  Rows past
  // the live end re-read the last live row (never outside the cache).
  auto stage = [&](int c0, int b) {
    const int last = ke - 1 - c0;
    uint16_t* kd = smem + b * 2 * PIECES * 8;
    uint16_t* vd = kd + PIECES * 8;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int P = (wave * IPW + i) * 64 + lane;
      const int r = P / CPR, c = P % CPR;
      const int rr = r < last ? r : last;
      glds16(kg + (size_t)(c0 + rr) * HD + (c ^ (r % CPR)) * 8, kd + (wave * IPW + i) * 64 * 8);
      glds16(vg + (size_t)(c0 + rr) * HD + c * 8, vd + (wave * IPW + i) * 64 * 8);
    }
  };

  float m = -INFINITY, l = 0.f, o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  stage(kb, 0);
  // q after the first chunk's DMA: one round trip covers both (hipcc drains the
  // DMA together with the q loads before the LDS stores below)
  for (int i = tid; i < NREP * HD; i += NT) qs[i] = q[(size_t)g * NREP * HD + i] * scale_log2;
  __syncthreads();
  int buf = 0;
  for (int c0 = kb; c0 < ke; c0 += kChunk, buf ^= 1) {
    const int kn = min(kChunk, ke - c0);
    if (c0 + kChunk < ke) {  // next chunk streams while this one computes
      stage(c0 + kChunk, buf ^ 1);
      __builtin_amdgcn_s_waitcnt(vm_wait(2 * IPW));
    } else {
      __builtin_amdgcn_s_waitcnt(vm_wait(0));
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMA for this chunk has landed
    const uint16_t* Ks = smem + buf * 2 * PIECES * 8;
    const uint16_t* Vs = Ks + PIECES * 8;
    if (wave < NREP) {
      float sc = -INFINITY;
      if (lane < kn) {
        const uint16_t* kr = Ks + lane * HD;
        const float* qh = qs + wave * HD;
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < CPR; ++c) {
          float kf[8];
          unpack8<DT>(*reinterpret_cast<const uint4*>(kr + ((c ^ (lane % CPR)) * 8)), kf);
          const float4 qa = *reinterpret_cast<const float4*>(qh + c * 8);
          const float4 qb = *reinterpret_cast<const float4*>(qh + c * 8 + 4);
          acc = fmaf(qa.x, kf[0], acc); acc = fmaf(qa.y, kf[1], acc);
          acc = fmaf(qa.z, kf[2], acc); acc = fmaf(qa.w, kf[3], acc);
          acc = fmaf(qb.x, kf[4], acc); acc = fmaf(qb.y, kf[5], acc);
          acc = fmaf(qb.z, kf[6], acc); acc = fmaf(qb.w, kf[7], acc);
        }
        sc = acc;
      }
      const float mn = fmaxf(m, wave_max(sc));
      const float alpha = exp2f(m - mn);  // 0 on the first chunk (m = -inf)
      const float p = lane < kn ? exp2f(sc - mn) : 0.f;
      l = l * alpha + wave_sum(p);
      m = mn;
      float* pw = ps + wave * kChunk;
      pw[lane] = p;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's p row is in LDS
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[d] *= alpha;
      const int kn4 = kn & ~3;
      for (int j = 0; j < kn4; j += 4) {
        const float4 p4 = *reinterpret_cast<const float4*>(pw + j);
        const float pj[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint16_t* vr = Vs + (j + e) * HD + lane * DPL;
          if constexpr (DPL == 2) {
            const uint32_t w2 = *reinterpret_cast<const uint32_t*>(vr);
            o[0] = fmaf(pj[e], to_f32<DT>((uint16_t)(w2 & 0xffffu)), o[0]);
            o[1] = fmaf(pj[e], to_f32<DT>((uint16_t)(w2 >> 16)), o[1]);
          } else {
#pragma unroll
            for (int d = 0; d < DPL; ++d) o[d] = fmaf(pj[e], to_f32<DT>(vr[d]), o[d]);
          }
        }
      }
      for (int j = kn4; j < kn; ++j) {
        const uint16_t* vr = Vs + j * HD + lane * DPL;
#pragma unroll
        for (int d = 0; d < DPL; ++d) o[d] = fmaf(pw[j], to_f32<DT>(vr[d]), o[d]);
      }
    }
    // every wave is done with this buffer before the next iteration restages it
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  const int h = g * NREP + wave;
  if (ns == 1) {  // the whole context in this split: finish here
    if (wave < NREP) {
      const float inv = 1.f / l;
#pragma unroll
      for (int d = 0; d < DPL; ++d) out[(size_t)h * HD + lane * DPL + d] = from_f32<DT>(o[d] * inv);
    }
    return;
  }

  // publish the partial: write-through stores -> drain -> barrier -> ticket
  if (wave < NREP) {
    float* dst = part + ((size_t)h * kMaxSplit + s) * (HD + 2);
    if (lane == 0) { st_sc1(dst, m); st_sc1(dst + 1, l); }
#pragma unroll
    for (int d = 0; d < DPL; ++d) st_sc1(dst + 2 + lane * DPL + d, o[d]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned int t =
        __hip_atomic_fetch_add(&tickets[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned int last = (t == (unsigned int)(ns - 1)) ? 1u : 0u;
    if (last) tickets[g] = 0u;  // re-arm for the next launch (kernel boundary orders it)
    last_flag = last;
  }
  __syncthreads();
  if (!last_flag || wave >= NREP) return;

  // merge the ns <= 64 partials of this wave's head: lane t owns split t's (m, l)
  const float* src = part + (size_t)h * kMaxSplit * (HD + 2);
  const float mt = lane < ns ? ld_sc1(src + lane * (HD + 2)) : -INFINITY;
  const float lt = lane < ns ? ld_sc1(src + lane * (HD + 2) + 1) : 0.f;
  const float M = wave_max(mt);
  const float wt = lane < ns ? exp2f(mt - M) : 0.f;
  const float L = wave_sum(wt * lt);
  float* pw = ps + wave * kChunk;
  pw[lane] = wt;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  float acc[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) acc[d] = 0.f;
#pragma unroll 8
  for (int t = 0; t < ns; ++t) {
    const float w = pw[t];
    const float* pt = src + t * (HD + 2) + 2 + lane * DPL;
#pragma unroll
    for (int d = 0; d < DPL; ++d) acc[d] = fmaf(w, ld_sc1(pt + d), acc[d]);
  }
  const float inv = 1.f / L;
#pragma unroll
  for (int d = 0; d < DPL; ++d) out[(size_t)h * HD + lane * DPL + d] = from_f32<DT>(acc[d] * inv);
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

// part: workspace [nh][64][hd+2] f32; tickets: [nkv] u32, zero-initialised
// once (the kernel re-arms them).
static inline int attn_max_split(int S) {
  const int n = (S + kChunk - 1) / kChunk;
  return n < kMaxSplit ? n : kMaxSplit;
}

CAKE_API int cake_attn_set_min_keys(int min_keys) {
  if (min_keys < kChunk || min_keys % kChunk) return (int)hipErrorInvalidValue;
  g_attn_min_keys = min_keys;
  return 0;
}

template <int DT, int HD>
static int launch_decode(int n_rep, dim3 grid, hipStream_t st, const float* q, const void* kc,
                         const void* vc, const int* pos, int S, float sl2, float* part,
                         unsigned int* tickets, void* out) {
#define CAKE_DEC(NR)                                                                          \
  hipLaunchKernelGGL((attn_decode_kernel<DT, HD, NR>), grid, dim3(AttnGeom<NR>::NT), 0, st, q, \
                     (const uint16_t*)kc, (const uint16_t*)vc, pos, S, sl2, part, tickets,    \
                     (uint16_t*)out, g_attn_min_keys)
  switch (n_rep) {
    case 1: CAKE_DEC(1); break;
    case 2: CAKE_DEC(2); break;
    case 4: CAKE_DEC(4); break;
    case 8: CAKE_DEC(8); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef CAKE_DEC
  return (int)hipGetLastError();
}

CAKE_API int cake_attn_decode(int dt, const float* q, const void* kc, const void* vc,
                              const int* pos, int S, int nh, int nkv, int hd, float scale,
                              float* part, unsigned int* tickets, void* out, hipStream_t st) {
  if (nkv <= 0 || nh % nkv || S <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid(nkv, attn_max_split(S));
  const float sl2 = scale * 1.4426950408889634f;
  DISPATCH_DT_HD(dt, hd, return (launch_decode<DT, HD>(nh / nkv, grid, st, q, kc, vc, pos, S, sl2,
                                                       part, tickets, out)));
  return (int)hipErrorInvalidValue;
}
