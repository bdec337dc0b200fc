// KV-cached GQA decode attention core (flash-decoding split-K), included by
// attention.hip.
//
// Replaces the reference's attention core:
//   cake-core/src/models/llama3/attention.rs:89-119  (repeat_kv, f32 upcast,
//   q·kᵀ/√d, causal mask, softmax, ·v, transpose back) and the KV growth of
//   cake-core/src/models/llama3/cache.rs:93-122 (Tensor::cat per step).
//
// One workgroup = (kv head g, split s) and runs all NREP query heads of the GQA
// group (one wave each), so every K/V byte is read from HBM once per token.
// The number of live splits is derived ON DEVICE from the live length
// Tk = pos + 1 (the launch is graph-replayed at every position):
// ns = min(maxsplit, ceil(Tk / keys)); each split owns a contiguous range of
// whole 64-key chunks.  Chunks are streamed global -> registers (every load of
// the next chunk is issued before the current chunk is computed) -> LDS (K rows
// XOR-swizzled: conflict-free row-per-lane ds_read_b128).  Per wave: lane j
// scores key j, online softmax in base 2 (scale * log2 e folded into q), P·V
// with lanes over (key group x 8 head dims).
//
// Combine: splits publish (m, l, o[HD]) with write-through (sc1) stores, drain
// (vmcnt 0), barrier, then one relaxed agent-scope ticket add per workgroup;
// the workgroup whose add returns ns - 1 reads every partial with sc1 loads
// (MI355X_MICROARCH "Valid forms", row 1) and writes the head outputs.  ns == 1
// (short contexts) writes the output directly.
//
// (Rejected after measuring: attention and o_proj as one launch whose o_proj
// blocks stream their weights while attention runs and wait on an agent-scope
// counter — 17.3 us vs 5.5 + 7.2 us for the two launches, the attention loads
// queue behind the weight stream; profiles/r2_decode_rejected_experiments.jsonl.)
#pragma once
#include "common.h"

namespace cake {

constexpr int kChunk = 64;        // keys per LDS chunk (one per lane)
constexpr int kMaxSplit = 64;     // splits per kv head (partials merged lane-parallel)

template <int NREP> struct AttnGeom {
  static constexpr int NW = NREP < 4 ? 4 : NREP;  // waves (>= 4 so loads stay wide)
  static constexpr int NT = 64 * NW;
};

// LDS (16-bit elements): 2 x [K chunk | V chunk], q (f32, pre-scaled), p rows, a flag
template <int HD, int NREP>
constexpr int attn_smem_elems() {
  return 2 * 2 * kChunk * HD + NREP * HD * 2 + NREP * kChunk * 2 + 2;
}

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Chunk [c0, c0 + 64) of one kv head, staged global -> registers -> LDS: piece P
// (row P / CPR, slot P % CPR) of K lands at slot ^ (row % CPR) (the XOR swizzle
// makes the row-per-lane ds_read_b128 of the scores conflict-free), V linear.
// Rows past `ke` re-read the last row before it (never outside the cache).
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

// V rows past `last` (the chunk's last live row) are stored as zeros: their
// p is 0, and a row loaded before the live length was known (split 0's
// speculative first chunk) may hold any bits, NaN included.
template <int HD, int IPW>
__device__ __forceinline__ void kv_store(const u32x4 (&rk)[IPW], const u32x4 (&rv)[IPW],
                                         uint16_t* kd, int wave, int lane, int last) {
  constexpr int CPR = HD / 8;
  uint16_t* vd = kd + kChunk * HD;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int P = (wave * IPW + i) * 64 + lane;
    const int r = P / CPR, c = P % CPR;
    *reinterpret_cast<u32x4*>(kd + (r * CPR + (c ^ (r % CPR))) * 8) = rk[i];
    const u32x4 z = {0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4*>(vd + P * 8) = r <= last ? rv[i] : z;
  }
}

struct AttnDecArgs {
  const float* q;          // [nh*hd] f32 (roped)
  const uint16_t* kc;      // [nkv][S][hd]
  const uint16_t* vc;
  const int* pos;          // device scalar
  int S;
  float scale_log2;
  float* part;             // [nh][kMaxSplit][hd+2] f32
  unsigned int* tickets;   // [2 nkv + 2]: arrival tickets / epochs, then the error word
  uint16_t* out;           // [nh*hd]
  int min_keys, maxsplit;
  unsigned long long* stamps;  // diagnostics (nullptr in production): per-WG phase clocks
  int target;                  // core 2: splits aimed at (keys per split = Tk / target)
  int single;                  // core 2: live lengths up to this run as one split
  int drop_partials;           // test hook: splits >= 1 never publish (forces a timeout)
};

// Phase clock of workgroup (g, s) for the latency breakdown (scripts/attn_stamps.py):
// slot k of 8, shader-clock ticks (s_memtime) from thread 0.
#define ATTN_STAMP(k)                                                              \
  do {                                                                             \
    if (a.stamps != nullptr && threadIdx.x == 0)                                   \
      stamp[k] = __builtin_amdgcn_s_memtime();                                     \
  } while (0)

// Merge the ns <= 64 split partials of head h (one wave; lane t owns split t's m, l)
// into the head's output row.  The first round's loads — every split's (m, l) and the
// o rows of the first kMergeRound splits — are all issued before any is used, so up
// to kMergeRound splits cost one memory round trip (agent-scope loads go past the
// XCD's L2: each round trip is a long one).  pw: 64 floats of scratch LDS.
constexpr int kMergeRound = 16;

template <int DT, int HD>
__device__ __forceinline__ void attn_merge_head(const AttnDecArgs& a, int h, int ns, int lane,
                                                float* pw) {
  constexpr int DPL = HD / 64;  // output dims per lane
  constexpr int MR = kMergeRound;
  const float* src = a.part + (size_t)h * kMaxSplit * (HD + 2);
  const float mt = lane < ns ? ld_sc1(src + lane * (HD + 2)) : -INFINITY;
  const float lt = lane < ns ? ld_sc1(src + lane * (HD + 2) + 1) : 0.f;
  float v[MR][DPL];
#pragma unroll
  for (int u = 0; u < MR; ++u) {
    const int t = u < ns ? u : ns - 1;
    const float* pt = src + t * (HD + 2) + 2 + lane * DPL;
#pragma unroll
    for (int d = 0; d < DPL; ++d) v[u][d] = ld_sc1(pt + d);
  }
  const float M = wave_max(mt);
  const float wt = lane < ns ? exp2f(mt - M) : 0.f;
  const float L = wave_sum(wt * lt);
  pw[lane] = wt;
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the weights are in LDS
  __builtin_amdgcn_wave_barrier();
  float acc[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) acc[d] = 0.f;
#pragma unroll
  for (int u = 0; u < MR; ++u) {
    const float w = u < ns ? pw[u] : 0.f;
#pragma unroll
    for (int d = 0; d < DPL; ++d) acc[d] = fmaf(w, v[u][d], acc[d]);
  }
  for (int t0 = MR; t0 < ns; t0 += MR) {  // ns > 16: further rounds
#pragma unroll
    for (int u = 0; u < MR; ++u) {
      const int t = t0 + u < ns ? t0 + u : ns - 1;
      const float* pt = src + t * (HD + 2) + 2 + lane * DPL;
#pragma unroll
      for (int d = 0; d < DPL; ++d) v[u][d] = ld_sc1(pt + d);
    }
#pragma unroll
    for (int u = 0; u < MR; ++u) {
      const float w = t0 + u < ns ? pw[t0 + u] : 0.f;
#pragma unroll
      for (int d = 0; d < DPL; ++d) acc[d] = fmaf(w, v[u][d], acc[d]);
    }
  }
  const float inv = 1.f / L;
  uint16_t* dst = a.out + (size_t)h * HD + lane * DPL;
#pragma unroll
  for (int d = 0; d < DPL; ++d) dst[d] = from_f32<DT>(acc[d] * inv);
}

template <int DT, int HD, int NREP>
__device__ __forceinline__ void attn_decode_block(const AttnDecArgs& a, int g, int s,
                                                  uint16_t* smem) {
  constexpr int NT = AttnGeom<NREP>::NT;
  constexpr int NW = AttnGeom<NREP>::NW;
  constexpr int DPL = HD / 64;              // output dims per lane (merge)
  constexpr int CPR = HD / 8;               // 16-byte pieces per row
  constexpr int PIECES = kChunk * CPR;      // pieces per chunk (each of K and V)
  constexpr int IPW = PIECES / 64 / NW;     // 16-byte pieces per thread per chunk (each of K, V)
  static_assert(IPW >= 1 && PIECES % (64 * NW) == 0, "chunk/wave geometry");
  float* qs = reinterpret_cast<float*>(smem + 2 * 2 * PIECES * 8);
  float* ps = qs + NREP * HD;
  unsigned int& last_flag = *reinterpret_cast<unsigned int*>(ps + NREP * kChunk);

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  unsigned long long stamp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ATTN_STAMP(0);
  const uint16_t* kg = a.kc + (size_t)g * a.S * HD;
  const uint16_t* vg = a.vc + (size_t)g * a.S * HD;
  // The loads of the next chunk are issued before the current chunk is computed
  // and stored to the other LDS buffer after it (register staging: the compiler's vmcnt covers
  // exactly these loads, where an LDS-DMA stage made every LDS read wait for the
  // in-flight DMA as well).
  u32x4 rk[IPW], rv[IPW];
  // Split 0 always starts at key 0: its q rows and first chunk are requested
  // together with the position, so a short context costs one memory round trip
  // instead of three (rows are clamped to the cache; kv_store zeroes dead V rows).
  constexpr int QPT = (NREP * HD + NT - 1) / NT;
  float qr[QPT];
  if (s == 0) {
    kv_load<HD, NW, IPW>(rk, rv, kg, vg, 0, a.S, wave, lane);
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
      const int i = tid + j * NT;
      qr[j] = i < NREP * HD ? a.q[(size_t)g * NREP * HD + i] : 0.f;
    }
  }
  const int Tk = *a.pos + 1;
  ATTN_STAMP(1);
  // past 1024 keys two chunks per split: every extra chunk per split costs about
  // one load round trip (~1.8 us), every extra split ~0.05-0.1 us of merge
  // (profiles/r2_decode_attn_pv*.jsonl: 2048 keys 11.7 us in 17 splits vs 12.4 in 33)
  const int keys = max(max(a.min_keys, Tk > 1024 ? 2 * kChunk : kChunk),
                       (Tk + kMaxSplit - 1) / kMaxSplit);
  int ns = (Tk + keys - 1) / keys;
  if (ns > a.maxsplit) ns = a.maxsplit;
  int kps = (Tk + ns - 1) / ns;
  kps = (kps + kChunk - 1) / kChunk * kChunk;
  ns = (Tk + kps - 1) / kps;
  if (s >= ns) return;
  const int kb = s * kps, ke = min(Tk, kb + kps);
  // P·V mapping: lane = key group kgi (keys kgi*VT .. +VT of the chunk) x dim
  // group dg (dims dg*8 .. +8): one ds_read_b128 per key per lane, VT of them
  // independent per chunk; the key groups' partial sums are only combined once,
  // after the last chunk (the online-softmax rescale is the same for every lane)
  constexpr int DG = HD / 8, KG = 64 / DG, VT = kChunk / KG;
  static_assert(DG == 8 || DG == 16, "key-group combine covers hd 64 and 128");
  const int dg = lane % DG, kgi = lane / DG;
  float m = -INFINITY, l = 0.f, o[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) o[d] = 0.f;
  if (s != 0) {
    kv_load<HD, NW, IPW>(rk, rv, kg, vg, kb, ke, wave, lane);
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
      const int i = tid + j * NT;
      qr[j] = i < NREP * HD ? a.q[(size_t)g * NREP * HD + i] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int i = tid + j * NT;
    if (i < NREP * HD) qs[i] = qr[j] * a.scale_log2;
  }
  kv_store<HD, IPW>(rk, rv, smem, wave, lane, ke - 1 - kb);
  __syncthreads();
  ATTN_STAMP(2);
  int buf = 0;
  for (int c0 = kb; c0 < ke; c0 += kChunk, buf ^= 1) {
    const int kn = min(kChunk, ke - c0);
    const bool more = c0 + kChunk < ke;
    if (more) kv_load<HD, NW, IPW>(rk, rv, kg, vg, c0 + kChunk, ke, wave, lane);  // in flight
    const uint16_t* Ks = smem + buf * 2 * PIECES * 8;
    const uint16_t* Vs = Ks + PIECES * 8;
    // q stays in LDS: hoisted out of the chunk loop it pinned 128 VGPRs per lane;
    // its reads are broadcasts
    asm volatile("" ::: "memory");
    if (wave < NREP) {
      float sc = -INFINITY;
      if (lane < kn) {
        // K piece c of this lane's row sits at byte (lane*HD*2 + 16*(c ^ lane%CPR)) =
        // kx ^ 16c; kx is made opaque here so the 16 piece addresses are formed in
        // the loop (hoisted, they pinned 16 VGPRs across it)
        unsigned int kx = (unsigned int)(lane * HD * 2 + 16 * (lane % CPR));
        asm volatile("" : "+v"(kx));
        const char* kb8 = reinterpret_cast<const char*>(Ks);
        const float* qh = qs + wave * HD;
        float acc0 = 0.f, acc1 = 0.f;  // two chains: half the dependent-FMA latency
        // CQ row pieces (K + q LDS reads) in flight at a time: unbounded, the
        // scheduler hoisted all of them next to the in-flight chunk registers
        constexpr int CQ = CPR < 4 ? CPR : 4;
#pragma unroll
        for (int c0 = 0; c0 < CPR; c0 += CQ) {
#pragma unroll
          for (int c = c0; c < c0 + CQ; ++c) {
            float kf[8];
            unpack8<DT>(*reinterpret_cast<const uint4*>(kb8 + (kx ^ (16u * c))), kf);
            const float4 qa = *reinterpret_cast<const float4*>(qh + c * 8);
            const float4 qb = *reinterpret_cast<const float4*>(qh + c * 8 + 4);
            acc0 = fmaf(qa.x, kf[0], acc0); acc1 = fmaf(qa.y, kf[1], acc1);
            acc0 = fmaf(qa.z, kf[2], acc0); acc1 = fmaf(qa.w, kf[3], acc1);
            acc0 = fmaf(qb.x, kf[4], acc0); acc1 = fmaf(qb.y, kf[5], acc1);
            acc0 = fmaf(qb.z, kf[6], acc0); acc1 = fmaf(qb.w, kf[7], acc1);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        sc = acc0 + acc1;
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
      // keys past kn have p = 0 and zeroed V rows
      float pv[VT];
#pragma unroll
      for (int t = 0; t < VT; t += 4) {
        const float4 p4 = *reinterpret_cast<const float4*>(pw + kgi * VT + t);
        pv[t] = p4.x; pv[t + 1] = p4.y; pv[t + 2] = p4.z; pv[t + 3] = p4.w;
      }
      const uint16_t* vcol = Vs + (size_t)kgi * VT * HD + dg * 8;
      // VH keys' V reads in flight at a time (bounds the registers the scheduler
      // may give to LDS reads)
      constexpr int VH = VT < 4 ? VT : 4;
#pragma unroll
      for (int t0 = 0; t0 < VT; t0 += VH) {
        uint4 vr[VH];
#pragma unroll
        for (int t = 0; t < VH; ++t) vr[t] = *reinterpret_cast<const uint4*>(vcol + (t0 + t) * HD);
#pragma unroll
        for (int t = 0; t < VH; ++t) {
          float vf[8];
          unpack8<DT>(vr[t], vf);
#pragma unroll
          for (int d = 0; d < 8; ++d) o[d] = fmaf(pv[t0 + t], vf[d], o[d]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // (that buffer was released by the previous barrier)
    if (more) kv_store<HD, IPW>(rk, rv, smem + (buf ^ 1) * 2 * kChunk * HD, wave, lane,
                                ke - 1 - (c0 + kChunk));
    __syncthreads();           // next chunk visible; this buffer free for reuse
  }

  ATTN_STAMP(3);
  // combine the key groups: afterwards every lane of dim group dg holds its 8 sums
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    if constexpr (DG <= 8) o[d] = xor_add<8>(o[d]);
    o[d] = xor_add<32>(xor_add<16>(o[d]));
  }
  ATTN_STAMP(4);
  auto flush_stamps = [&](int n) {
    if (a.stamps != nullptr && tid == 0) {
      unsigned long long* d = a.stamps + ((size_t)s * gridDim.x + g) * 8;
      for (int k = 0; k < 8; ++k) d[k] = k < n ? stamp[k] : 0ull;
    }
  };
  const int h = g * NREP + wave;
  if (ns == 1) {  // the whole context in this split: finish here
    ATTN_STAMP(5);
    flush_stamps(6);
    if (wave < NREP && kgi == 0) {
      const float inv = 1.f / l;
      uint16_t ob[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) ob[d] = from_f32<DT>(o[d] * inv);
      *reinterpret_cast<uint4*>(a.out + (size_t)h * HD + dg * 8) =
          *reinterpret_cast<const uint4*>(ob);
    }
    return;
  }

  // publish the partial: write-through stores -> drain -> barrier -> ticket
  if (wave < NREP) {
    float* dst = a.part + ((size_t)h * kMaxSplit + s) * (HD + 2);
    if (lane == 0) { st_sc1(dst, m); st_sc1(dst + 1, l); }
    if (kgi == 0) {
#pragma unroll
      for (int d = 0; d < 8; ++d) st_sc1(dst + 2 + dg * 8 + d, o[d]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ATTN_STAMP(5);
  if (tid == 0) {
    const unsigned int t =
        __hip_atomic_fetch_add(&a.tickets[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned int last = (t == (unsigned int)(ns - 1)) ? 1u : 0u;
    if (last) a.tickets[g] = 0u;  // re-arm for the next launch (kernel boundary orders it)
    last_flag = last;
  }
  __syncthreads();
  ATTN_STAMP(6);
  if (!last_flag) flush_stamps(7);
  if (!last_flag || wave >= NREP) return;

  attn_merge_head<DT, HD>(a, h, ns, lane, ps + wave * kChunk);
  ATTN_STAMP(7);
  flush_stamps(8);
}

}  // namespace cake
