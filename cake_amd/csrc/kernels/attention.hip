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
// Grid (nkv, maxsplit), 4 waves per workgroup.  A workgroup = (kv head g,
// split s) and computes all NREP query heads of the GQA group, so every K/V
// byte is read from HBM once per token.  The live length Tk = pos + 1 is read
// on the device (the launch is graph-replayed at every position) and cut into
// 64-key chunks; a split owns `cps` consecutive chunks (cps = max(min_chunks,
// ceil(chunks / maxsplit))), its 4 waves take one chunk each (looping when
// cps > 4).  A chunk is ONE round trip: every load is issued before the first
// use — K rows by LDS-DMA into this wave's LDS slice (16-byte slots XOR-
// swizzled on the source address so the row-per-lane ds_read_b128 is
// conflict-free), V rows straight to registers (lane = two head dims), q once
// per workgroup.  Per wave: lane j scores key j for each head, online softmax
// in base 2 (scale * log2 e folded into q), P·V with lanes over head dims.
// The waves merge in LDS; with one split (short contexts: Tk <= 64 * min_chunks)
// that is the output, with no further hand-off.
//
// Splits publish (m, l, o[HD]) with write-through (sc1) stores, drain
// (vmcnt 0), barrier, then one relaxed agent-scope ticket add per workgroup;
// the workgroup whose add returns ns - 1 reads every partial with sc1 loads
// (MI355X_MICROARCH "Valid forms", row 1) and writes the head outputs.
constexpr int kChunk = 64;         // keys per wave chunk (one per lane)
constexpr int kMaxSplit = 64;      // splits per kv head (partials merged lane-parallel)
constexpr int kAttnWaves = 4;
static int g_attn_min_chunks = 4;  // min chunks per split (tunable)

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int DT, int HD, int NREP>
__global__ __launch_bounds__(64 * kAttnWaves) void attn_decode_kernel(
    const float* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int* __restrict__ pos_ptr, int S, float scale_log2,
    float* __restrict__ part, unsigned int* __restrict__ tickets, uint16_t* __restrict__ out,
    int min_chunks) {
  constexpr int NW = kAttnWaves, NT = 64 * NW;
  constexpr int DPL = HD / 64;              // head dims per lane (P·V)
  constexpr int CPR = HD / 8;               // 16-byte pieces per K row
  constexpr int KIPW = kChunk * CPR / 64;   // K LDS-DMA wave-instructions per chunk
  constexpr int KBYTES = kChunk * HD * 2;   // one wave's K slice
  constexpr int HPW = (NREP + NW - 1) / NW; // heads merged per wave
  // one LDS array: [NW][K chunk] 16-bit | q [NREP][HD] f32 | p [NW][NREP][64] |
  // merge [NW][NREP][HD + 2] | flag
  constexpr int OFF_Q = NW * KBYTES;
  constexpr int OFF_P = OFF_Q + NREP * HD * 4;
  constexpr int OFF_M = OFF_P + NW * NREP * kChunk * 4;
  constexpr int OFF_F = OFF_M + NW * NREP * (HD + 2) * 4;
  __shared__ __attribute__((aligned(16))) uint8_t smem[OFF_F + 16];
  float* qs = reinterpret_cast<float*>(smem + OFF_Q);
  float* ps = reinterpret_cast<float*>(smem + OFF_P);
  float* ms = reinterpret_cast<float*>(smem + OFF_M);
  unsigned int& last_flag = *reinterpret_cast<unsigned int*>(smem + OFF_F);

  const int g = blockIdx.x, s = blockIdx.y;
  const int Tk = *pos_ptr + 1;
  const int C = (Tk + kChunk - 1) / kChunk;
  int cps = (C + (int)gridDim.y - 1) / (int)gridDim.y;
  cps = cps > min_chunks ? cps : min_chunks;
  const int ns = (C + cps - 1) / cps;
  if (s >= ns) return;
  const int c_end = min(C, (s + 1) * cps);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint16_t* kg = kc + (size_t)g * S * HD;
  const uint16_t* vg = vc + (size_t)g * S * HD;
  uint8_t* kslice = smem + wave * KBYTES;

  float m[NREP], l[NREP], o[NREP][DPL];
#pragma unroll
  for (int h = 0; h < NREP; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[h][d] = 0.f;
  }
  bool first = true;
  for (int c = s * cps + wave; c < c_end || first; c += NW) {
    const bool active = c < c_end;
    const int k0 = c * kChunk;
    const int kn = active ? min(kChunk, Tk - k0) : 0;
    // ---- issue every load of this chunk (one round trip).  V first: with the
    // LDS-DMA issued last hipcc keeps all of them in flight (K DMA first made it
    // drain vmcnt(0) before the 16th DMA) --------------------------------------
    uint32_t vr[kChunk][1];
    if (active) {
#pragma unroll
      for (int r = 0; r < kChunk; ++r) {
        const int rr = r < kn ? r : kn - 1;
        if constexpr (DPL == 2)
          vr[r][0] = *reinterpret_cast<const uint32_t*>(vg + (size_t)(k0 + rr) * HD + lane * 2);
        else
          vr[r][0] = (uint32_t)vg[(size_t)(k0 + rr) * HD + lane];
      }
#pragma unroll
      for (int i = 0; i < KIPW; ++i) {
        const int P = i * 64 + lane;              // LDS slot (row P / CPR, piece P % CPR)
        const int r = P / CPR, pc = P % CPR;
        const int rr = r < kn ? r : kn - 1;       // never past the live rows
        glds16(kg + (size_t)(k0 + rr) * HD + ((pc ^ (r % CPR)) * 8), kslice + i * 1024);
      }
    }
    if (first) {  // q of the whole GQA group, pre-scaled (loads overlap the chunk's)
      for (int i = tid; i < NREP * HD; i += NT) qs[i] = q[(size_t)g * NREP * HD + i] * scale_log2;
      __builtin_amdgcn_s_waitcnt(vm_wait(0));
      __syncthreads();
      first = false;
    } else {
      __builtin_amdgcn_s_waitcnt(vm_wait(0));
      __builtin_amdgcn_wave_barrier();
    }
    if (!active) break;
    // ---- scores: lane j <-> key k0 + j, all heads ------------------------
    float sc[NREP];
#pragma unroll
    for (int h = 0; h < NREP; ++h) sc[h] = 0.f;
    const uint8_t* krow = kslice + lane * HD * 2;
#pragma unroll
    for (int pc = 0; pc < CPR; ++pc) {
      float kf[8];
      unpack8<DT>(*reinterpret_cast<const uint4*>(krow + ((pc ^ (lane % CPR)) * 16)), kf);
#pragma unroll
      for (int h = 0; h < NREP; ++h) {
        const float4 qa = *reinterpret_cast<const float4*>(qs + h * HD + pc * 8);
        const float4 qb = *reinterpret_cast<const float4*>(qs + h * HD + pc * 8 + 4);
        float a = sc[h];
        a = fmaf(qa.x, kf[0], a); a = fmaf(qa.y, kf[1], a);
        a = fmaf(qa.z, kf[2], a); a = fmaf(qa.w, kf[3], a);
        a = fmaf(qb.x, kf[4], a); a = fmaf(qb.y, kf[5], a);
        a = fmaf(qb.z, kf[6], a); a = fmaf(qb.w, kf[7], a);
        sc[h] = a;
      }
    }
    float* pw = ps + wave * NREP * kChunk;
#pragma unroll
    for (int h = 0; h < NREP; ++h) {
      const float sv = lane < kn ? sc[h] : -INFINITY;
      const float mn = fmaxf(m[h], wave_max(sv));
      const float alpha = exp2f(m[h] - mn);  // 0 on the first chunk (m = -inf)
      const float p = lane < kn ? exp2f(sv - mn) : 0.f;
      l[h] = l[h] * alpha + wave_sum(p);
      m[h] = mn;
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[h][d] *= alpha;
      pw[h * kChunk + lane] = p;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's p rows are in LDS
    __builtin_amdgcn_wave_barrier();
    // ---- P·V: lanes over head dims, V rows from registers ----------------
#pragma unroll
    for (int r0 = 0; r0 < kChunk; r0 += 4) {
#pragma unroll
      for (int h = 0; h < NREP; ++h) {
        const float4 p4 = *reinterpret_cast<const float4*>(pw + h * kChunk + r0);
        const float pj[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (DPL == 2) {
            const uint32_t w2 = vr[r0 + e][0];
            o[h][0] = fmaf(pj[e], to_f32<DT>((uint16_t)(w2 & 0xffffu)), o[h][0]);
            o[h][1] = fmaf(pj[e], to_f32<DT>((uint16_t)(w2 >> 16)), o[h][1]);
          } else {
            o[h][0] = fmaf(pj[e], to_f32<DT>((uint16_t)vr[r0 + e][0]), o[h][0]);
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // p rows read before the next chunk rewrites them
  }

  // ---- merge the waves of this split in LDS -------------------------------
#pragma unroll
  for (int h = 0; h < NREP; ++h) {
    float* mw = ms + (wave * NREP + h) * (HD + 2);
    if (lane == 0) { mw[0] = m[h]; mw[1] = l[h]; }
#pragma unroll
    for (int d = 0; d < DPL; ++d) mw[2 + lane * DPL + d] = o[h][d];
  }
  __syncthreads();
  float hm[HPW], hl[HPW], ho[HPW][DPL];
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int h = wave + i * NW;
    hm[i] = -INFINITY; hl[i] = 0.f;
#pragma unroll
    for (int d = 0; d < DPL; ++d) ho[i][d] = 0.f;
    if (h >= NREP) continue;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, ms[(w * NREP + h) * (HD + 2)]);
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float* mw = ms + (w * NREP + h) * (HD + 2);
      const float sc = mw[0] == -INFINITY ? 0.f : exp2f(mw[0] - M);
      L = fmaf(sc, mw[1], L);
#pragma unroll
      for (int d = 0; d < DPL; ++d) ho[i][d] = fmaf(sc, mw[2 + lane * DPL + d], ho[i][d]);
    }
    hm[i] = M; hl[i] = L;
  }
  if (ns == 1) {  // the whole context in this split: finish here
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int h = wave + i * NW;
      if (h >= NREP) continue;
      const float inv = 1.f / hl[i];
#pragma unroll
      for (int d = 0; d < DPL; ++d)
        out[((size_t)g * NREP + h) * HD + lane * DPL + d] = from_f32<DT>(ho[i][d] * inv);
    }
    return;
  }

  // ---- publish the split's partial: write-through stores -> drain -> ticket
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int h = wave + i * NW;
    if (h >= NREP) continue;
    float* dst = part + (((size_t)g * NREP + h) * kMaxSplit + s) * (HD + 2);
    if (lane == 0) { st_sc1(dst, hm[i]); st_sc1(dst + 1, hl[i]); }
#pragma unroll
    for (int d = 0; d < DPL; ++d) st_sc1(dst + 2 + lane * DPL + d, ho[i][d]);
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
  if (!last_flag) return;

  // ---- merge the ns <= 64 split partials: lane t owns split t's (m, l) ----
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int h = wave + i * NW;
    if (h >= NREP) continue;
    const float* src = part + ((size_t)g * NREP + h) * kMaxSplit * (HD + 2);
    const float mt = lane < ns ? ld_sc1(src + lane * (HD + 2)) : -INFINITY;
    const float lt = lane < ns ? ld_sc1(src + lane * (HD + 2) + 1) : 0.f;
    const float M = wave_max(mt);
    const float wt = lane < ns ? exp2f(mt - M) : 0.f;
    const float L = wave_sum(wt * lt);
    float acc[DPL];
#pragma unroll
    for (int d = 0; d < DPL; ++d) acc[d] = 0.f;
    for (int t0 = 0; t0 < ns; t0 += 8) {
      float vals[8][DPL];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int d = 0; d < DPL; ++d)
          vals[u][d] = t0 + u < ns ? ld_sc1(src + (t0 + u) * (HD + 2) + 2 + lane * DPL + d) : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float w = __shfl(wt, (t0 + u) & 63, 64);
#pragma unroll
        for (int d = 0; d < DPL; ++d) acc[d] = fmaf(w, vals[u][d], acc[d]);
      }
    }
    const float inv = 1.f / L;
#pragma unroll
    for (int d = 0; d < DPL; ++d)
      out[((size_t)g * NREP + h) * HD + lane * DPL + d] = from_f32<DT>(acc[d] * inv);
  }
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
  g_attn_min_chunks = min_keys / kChunk;
  return 0;
}

template <int DT, int HD>
static int launch_decode(int n_rep, dim3 grid, hipStream_t st, const float* q, const void* kc,
                         const void* vc, const int* pos, int S, float sl2, float* part,
                         unsigned int* tickets, void* out) {
#define CAKE_DEC(NR)                                                                          \
  hipLaunchKernelGGL((attn_decode_kernel<DT, HD, NR>), grid, dim3(64 * kAttnWaves), 0, st, q,  \
                     (const uint16_t*)kc, (const uint16_t*)vc, pos, S, sl2, part, tickets,    \
                     (uint16_t*)out, g_attn_min_chunks)
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
