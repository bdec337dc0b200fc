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
// current chunk is computed) -> LDS (K rows XOR-swizzled: conflict-free
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

// Chunk [c0, c0 + 64) of one kv head, staged global -> registers -> LDS: piece P
// (row P / CPR, slot P % CPR) of K lands at slot ^ (row % CPR) (the XOR swizzle
// makes the row-per-lane ds_read_b128 of the scores conflict-free), V linear.
// Rows past the live end re-read the last live row (never outside the cache).
template <int HD, int NW, int IPW>
__device__ __forceinline__ void kv_load(u32x4 (&rk)[IPW], u32x4 (&rv)[IPW], const uint16_t* kg,
                                        const uint16_t* vg, int c0, int ke, int wave, int lane) {
  constexpr int CPR = HD / 8;
  const int last = ke - 1 - c0;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int P = (wave * IPW + i) * 64 + lane;
    const int r = P / CPR, c = P % CPR;
    const size_t src = (size_t)(c0 + (r < last ? r : last)) * HD + c * 8;
    rk[i] = *reinterpret_cast<const u32x4*>(kg + src);
    rv[i] = *reinterpret_cast<const u32x4*>(vg + src);
  }
}

template <int HD, int IPW>
__device__ __forceinline__ void kv_store(const u32x4 (&rk)[IPW], const u32x4 (&rv)[IPW],
                                         uint16_t* kd, int wave, int lane) {
  constexpr int CPR = HD / 8;
  uint16_t* vd = kd + kChunk * HD;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int P = (wave * IPW + i) * 64 + lane;
    const int r = P / CPR, c = P % CPR;
    *reinterpret_cast<u32x4*>(kd + (r * CPR + (c ^ (r % CPR))) * 8) = rk[i];
    *reinterpret_cast<u32x4*>(vd + P * 8) = rv[i];
  }
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
  constexpr int IPW = PIECES / 64 / NW;     // 16-byte pieces per thread per chunk (each of K, V)
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
  // past 1024 keys two chunks per split: every extra chunk per split costs about
  // one load round trip (~1.8 us), every extra split ~0.05-0.1 us of merge
  // (profiles/r2_decode_attn_pv*.jsonl: 2048 keys 11.7 us in 17 splits vs 12.4 in 33)
  const int keys = max(max(min_keys, Tk > 1024 ? 2 * kChunk : kChunk), (Tk + kMaxSplit - 1) / kMaxSplit);
  int ns = (Tk + keys - 1) / keys;
  if (ns > (int)gridDim.y) ns = gridDim.y;
  int kps = (Tk + ns - 1) / ns;
  kps = (kps + kChunk - 1) / kChunk * kChunk;
  ns = (Tk + kps - 1) / kps;
  if (s >= ns) return;
  const int kb = s * kps, ke = min(Tk, kb + kps);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;


  const uint16_t* kg = kc + (size_t)g * S * HD;
  const uint16_t* vg = vc + (size_t)g * S * HD;
  // The loads of the next chunk are issued before the current chunk is computed
  // and stored to the other LDS buffer after it (register staging: the compiler's
  // vmcnt covers exactly these loads, where an LDS-DMA stage made every LDS read
  // wait for the in-flight DMA as well).
  u32x4 rk[IPW], rv[IPW];
  // P·V mapping: lane = key group kgi (keys kgi*VT .. +VT of the chunk) x dim
  // group dg (dims dg*8 .. +8): one ds_read_b128 per key per lane, VT of them
  // independent per chunk; the key groups' partial sums are only combined once,
  // after the last chunk (the online-softmax rescale is the same for every lane)
  constexpr int DG = HD / 8, KG = 64 / DG, VT = kChunk / KG;
  const int dg = lane % DG, kgi = lane / DG;
  float m = -INFINITY, l = 0.f, o[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) o[d] = 0.f;
  for (int i = tid; i < NREP * HD; i += NT) qs[i] = q[(size_t)g * NREP * HD + i] * scale_log2;
  kv_load<HD, NW, IPW>(rk, rv, kg, vg, kb, ke, wave, lane);
  kv_store<HD, IPW>(rk, rv, smem, wave, lane);
  __syncthreads();
  int buf = 0;
  for (int c0 = kb; c0 < ke; c0 += kChunk, buf ^= 1) {
    const int kn = min(kChunk, ke - c0);
    const bool more = c0 + kChunk < ke;
    if (more) kv_load<HD, NW, IPW>(rk, rv, kg, vg, c0 + kChunk, ke, wave, lane);  // in flight
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
      for (int d = 0; d < 8; ++d) o[d] *= alpha;
      // keys past kn have p = 0 and V rows re-read from the live range (finite)
      float pv[VT];
#pragma unroll
      for (int t = 0; t < VT; t += 4) {
        const float4 p4 = *reinterpret_cast<const float4*>(pw + kgi * VT + t);
        pv[t] = p4.x; pv[t + 1] = p4.y; pv[t + 2] = p4.z; pv[t + 3] = p4.w;
      }
      const uint16_t* vcol = Vs + (size_t)kgi * VT * HD + dg * 8;
#pragma unroll
      for (int t = 0; t < VT; ++t) {
        float vf[8];
        unpack8<DT>(*reinterpret_cast<const uint4*>(vcol + t * HD), vf);
#pragma unroll
        for (int d = 0; d < 8; ++d) o[d] = fmaf(pv[t], vf[d], o[d]);
      }
    }
    // (that buffer was released by the previous barrier)
    if (more) kv_store<HD, IPW>(rk, rv, smem + (buf ^ 1) * 2 * kChunk * HD, wave, lane);
    __syncthreads();           // next chunk visible; this buffer free for reuse
  }

  // combine the key groups: afterwards every lane of dim group dg holds its 8 sums
#pragma unroll
  for (int off = DG; off < 64; off <<= 1) {
#pragma unroll
    for (int d = 0; d < 8; ++d) o[d] += __shfl_xor(o[d], off, 64);
  }
  const int h = g * NREP + wave;
  if (ns == 1) {  // the whole context in this split: finish here
    if (wave < NREP && kgi == 0) {
      const float inv = 1.f / l;
      uint16_t ob[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) ob[d] = from_f32<DT>(o[d] * inv);
      *reinterpret_cast<uint4*>(out + (size_t)h * HD + dg * 8) = *reinterpret_cast<const uint4*>(ob);
    }
    return;
  }

  // publish the partial: write-through stores -> drain -> barrier -> ticket
  if (wave < NREP) {
    float* dst = part + ((size_t)h * kMaxSplit + s) * (HD + 2);
    if (lane == 0) { st_sc1(dst, m); st_sc1(dst + 1, l); }
    if (kgi == 0) {
#pragma unroll
      for (int d = 0; d < 8; ++d) st_sc1(dst + 2 + dg * 8 + d, o[d]);
    }
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
  // 16 partials' loads in flight per round trip (ns <= 64: at most 4 rounds)
  for (int t0 = 0; t0 < ns; t0 += 16) {
    float v[16][DPL];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int t = t0 + u < ns ? t0 + u : ns - 1;
      const float* pt = src + t * (HD + 2) + 2 + lane * DPL;
#pragma unroll
      for (int d = 0; d < DPL; ++d) v[u][d] = ld_sc1(pt + d);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const float w = t0 + u < ns ? pw[t0 + u] : 0.f;
#pragma unroll
      for (int d = 0; d < DPL; ++d) acc[d] = fmaf(w, v[u][d], acc[d]);
    }
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
