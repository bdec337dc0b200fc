// KV-cached GQA decode attention, v2: wave-independent key streams with MFMA scores.
// Included by attention.hip (same arguments / partial layout / ticket combine as
// attn_core.h, selected with cake_attn_set_impl(2)).
//
// Replaces the reference's attention core:
//   cake-core/src/models/llama3/attention.rs:89-119 and cache.rs:93-122.
//
// Why a second core: v1 stages 64-key chunks global -> registers -> LDS and every
// wave then re-reads q (f32, broadcast) and its K row / V columns from LDS, with a
// workgroup barrier per chunk — about 2.2 µs per extra chunk of a split
// (profiles/r2_decode_attn_pv*.jsonl: 1 split of 512 keys 20 µs vs 8 splits 8.7).
// Here nothing of K/V goes through LDS and the waves never wait for each other
// before the end of the split:
//   * a wave owns 16-key blocks (w, w + NW, ...) of its split and keeps its own
//     online-softmax state (m, l, o) for the NREP query heads of the group;
//   * scores S^T[16 keys x 16 cols] = K_blk[16 x HD] . Q^T on v_mfma_f32_16x16x32
//     (A = K rows straight from global memory: lane l holds row l&15, dims
//     32 d + 8 (l>>4); B = q as bf16 / f16 in registers, columns >= NREP zero) —
//     HD/32 MFMAs per block;
//   * the block's p (and the per-head rescale) go to a 1 KB wave-private LDS tile,
//     and P.V runs on the VALU from V rows also loaded straight from global
//     (lane -> 8 dims x HD/32 keys): NREP x 8 f32 accumulators per lane;
//   * the next block's K/V loads are issued before the current block is computed;
//   * at the end: key-group sums across lanes (permlane swaps), the NW waves'
//     states merged once through LDS, and the split's partial published to the
//     ticket combine of attn_core.h (or written out directly when ns == 1).
// Dead keys (past the live length, or speculative rows of split 0 loaded before
// the position arrived) are masked in the scores and zeroed in V.
#pragma once
#include <type_traits>

#include "attn_core.h"

namespace cake {

constexpr int kBlk = 16;  // keys per wave block (MFMA M dimension)
// bound on the merge's granule polls (s_sleep 1 apart): a producer that never publishes
// ends the poll instead of hanging the GPU, and sets the error word tickets[2 nkv]
// (the output of that launch is invalid; the host raises on it: ops.hip.attn_error)
constexpr int kAttnMaxPolls = 1 << 20;

__device__ __noinline__ void attn_poll_timeout(unsigned int* err) {
  __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int OFF> __device__ __forceinline__ float xor_max(float v) {
  static_assert(OFF == 16 || OFF == 32, "xor_max offset");
  const int b = __builtin_bit_cast(int, v);
  const auto p = OFF == 16 ? __builtin_amdgcn_permlane16_swap(b, b, false, false)
                           : __builtin_amdgcn_permlane32_swap(b, b, false, false);
  return fmaxf(__builtin_bit_cast(float, (int)p[0]), __builtin_bit_cast(float, (int)p[1]));
}

// LDS floats of the v2 core: per wave a p tile [16 keys][16 cols] + alpha[16], then
// the end-of-split wave states (m[16], l[16], o[NREP][HD]) of all NW waves.
template <int HD, int NREP, int NW>
constexpr int attn2_smem_floats() {
  return NW * (kBlk * 16 + 16) + NW * (32 + NREP * HD) + 1;
}

// Core 2's workgroup: 4 waves (8 for 8-head groups).  Rejected after measuring: 12
// waves for <= 4-head groups (every wave one 16-key block up to 192 keys, so the key loop
// is no longer a chain of load round trips) ran the 8B decode attention at 7.48 us vs
// 5.48 (bench context, Tk <= 72): the wave-state merge and barrier scale with the wave
// count while most waves hold no keys (profiles/r4_decode_attn_waves.md).
template <int NREP> struct AttnGeom2 {
  static constexpr int NW = AttnGeom<NREP>::NW;
  static constexpr int NT = 64 * NW;
};

// host/device split policy of the v2 core (mirrored by ops.hip.attn_splits)
__device__ __forceinline__ void attn2_splits(int Tk, int min_keys, int maxsplit, int target,
                                             int single, int& ns, int& kps) {
  if (Tk <= single) {  // one split: no partials, no merge (cheaper up to ~320 keys)
    ns = 1;
    kps = (Tk + kBlk - 1) / kBlk * kBlk;
    return;
  }
  int keys = (Tk + target - 1) / target;
  keys = (keys + kBlk - 1) / kBlk * kBlk;
  if (keys < min_keys) keys = min_keys;
  ns = (Tk + keys - 1) / keys;
  if (ns > maxsplit) ns = maxsplit;
  kps = (Tk + ns - 1) / ns;
  kps = (kps + kBlk - 1) / kBlk * kBlk;
  ns = (Tk + kps - 1) / kps;
}

// Agent-coherent (sc1, L2-served, L1 bypassed) 16-byte buffer loads: the fused QKV ->
// attention tail (gemv.hip qkv_attn_kernel) reads q and the new K/V row that other
// workgroups of the same launch stored write-through (MI355X_MICROARCH "Valid forms").
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sc1_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ uint4 ld16_sc1(__amdgpu_buffer_rsrc_t r, size_t byte_off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 16);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// FUSED: called by the last-arriving workgroup of kv group g inside the QKV launch —
// q / K / V loads are sc1 and the whole context runs as one split (the host picks the
// fused launch where attn2_splits gives one split; longer contexts stay correct, one
// workgroup walking every key).  ng = number of kv heads (the standalone grid's x).
// PFD: key blocks per wave in flight (1: the next block's loads issued with the current
// block's compute; 2: two ahead, and split 0 requests its first TWO blocks per wave at
// launch — up to 2 NW x 16 keys need no load round trip inside the loop).
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// hook: called once per wave right after the block's first loads (K/V of the first one
// or two key blocks, q) are issued and before anything waits on them — a caller's own
// loads issued there queue BEHIND the attention's (vmcnt retires in order) instead of in
// front of them (attn_oproj.hip: the o_proj weight tile)
// ONE: the head-parallel short-context launch (attn_head_kernel): one split, plain loads,
// no epoch word (tickets untouched); g is then a QUERY head (NREP 1) and kvh its kv head.
template <int DT, int HD, int NREP, bool FUSED = false, int NW = AttnGeom2<NREP>::NW,
          int PFD = 2, class Hook = NoHook, bool ONE = false>
__device__ __forceinline__ void attn2_decode_block(const AttnDecArgs& a, int g, int s,
                                                   float* lds, int ng, const Hook& hook = Hook(),
                                                   int kvh = -1) {
  static_assert(PFD == 1 || PFD == 2 || PFD == 4, "prefetch depth 1, 2 or 4");
  constexpr int DS = HD / 32;    // MFMA k-steps (A fragments) per key block
  constexpr int NCH = HD / 8;    // 8-dim chunks per row
  constexpr int KPL = NCH / 4;   // keys per lane in P.V (16 keys over 64 / NCH key groups)
  static_assert(NCH == 8 || NCH == 16, "hd 64 or 128");
  static_assert(NREP <= 16, "GQA group <= 16 heads");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, rg = lane >> 4;       // MFMA column (head) / row group
  const int ch = lane % NCH, kg = lane / NCH;      // P.V: dim chunk / key group
  float* pt = lds + wave * (kBlk * 16 + 16);       // this wave's p tile + alpha row
  float* alph = pt + kBlk * 16;
  float* st = lds + NW * (kBlk * 16 + 16);         // end-of-split wave states
  unsigned long long stamp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ATTN_STAMP(0);
  const int kv = kvh < 0 ? g : kvh;
  const uint16_t* kgp = a.kc + (size_t)kv * a.S * HD;
  const uint16_t* vgp = a.vc + (size_t)kv * a.S * HD;

  // one block's operands: K A-fragments and V rows of this lane
  // PFD slots of one block's operands (slot index a compile-time constant everywhere)
  uint4 kf[PFD][DS], vf[PFD][KPL];
  __amdgpu_buffer_rsrc_t krs, vrs;
  if constexpr (FUSED) { krs = sc1_rsrc(kgp); vrs = sc1_rsrc(vgp); }
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, PFD - 1>;
  auto load_blk = [&](auto slot, int key0, int last) {
    constexpr int SL = decltype(slot)::value;
#pragma unroll
    for (int d = 0; d < DS; ++d) {
      const int r = min(key0 + col, last);
      const size_t o = (size_t)r * HD + d * 32 + rg * 8;
      if constexpr (FUSED) kf[SL][d] = ld16_sc1(krs, o * 2);
      else kf[SL][d] = *reinterpret_cast<const uint4*>(kgp + o);
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const int r = min(key0 + kg * KPL + j, last);
      const size_t o = (size_t)r * HD + ch * 8;
      if constexpr (FUSED) vf[SL][j] = ld16_sc1(vrs, o * 2);
      else vf[SL][j] = *reinterpret_cast<const uint4*>(vgp + o);
    }
  };

  // split 0 starts at key 0: its first blocks are requested with the position
  // (rows clamped to the cache; dead rows are masked / zeroed below)
  if (s == 0) load_blk(I0{}, wave * kBlk, a.S - 1);
  // q (f32, roped) -> pre-scaled 16-bit B fragments: column col = head g*NREP + col.
  // The q loads go out right after the first block's, and split 0's second speculative
  // block after q: loads retire in order, so q (needed by the first MFMA) never waits
  // behind the second block.
  uint4 qf[DS];
  {
    float qv[DS][8];
    float4 qx[DS][2];
#pragma unroll
    for (int d = 0; d < DS; ++d) {
      if (col < NREP) {
        const size_t qo = (size_t)(g * NREP + col) * HD + d * 32 + rg * 8;
        if constexpr (FUSED) {
          const __amdgpu_buffer_rsrc_t qr = sc1_rsrc(a.q);
          qx[d][0] = __builtin_bit_cast(float4, ld16_sc1(qr, qo * 4));
          qx[d][1] = __builtin_bit_cast(float4, ld16_sc1(qr, qo * 4 + 16));
        } else {
          qx[d][0] = *reinterpret_cast<const float4*>(a.q + qo);
          qx[d][1] = *reinterpret_cast<const float4*>(a.q + qo + 4);
        }
      } else {
        qx[d][0] = qx[d][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PFD == 2) {
      if (s == 0) load_blk(I1{}, (wave + NW) * kBlk, a.S - 1);
    } else if constexpr (PFD == 4) {
      if (s == 0) {
        load_blk(std::integral_constant<int, 1>{}, (wave + NW) * kBlk, a.S - 1);
        load_blk(std::integral_constant<int, 2>{}, (wave + 2 * NW) * kBlk, a.S - 1);
        load_blk(std::integral_constant<int, 3>{}, (wave + 3 * NW) * kBlk, a.S - 1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    hook();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int d = 0; d < DS; ++d) {
      const float4 x0 = qx[d][0], x1 = qx[d][1];
      qv[d][0] = x0.x; qv[d][1] = x0.y; qv[d][2] = x0.z; qv[d][3] = x0.w;
      qv[d][4] = x1.x; qv[d][5] = x1.y; qv[d][6] = x1.z; qv[d][7] = x1.w;
    }
#pragma unroll
    for (int d = 0; d < DS; ++d) {
      uint16_t h[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = from_f32<DT>(qv[d][e] * a.scale_log2);
      qf[d] = *reinterpret_cast<const uint4*>(h);
    }
  }
  const int Tk = *a.pos + 1;
  unsigned int epoch = 0;
  if constexpr (!ONE) epoch = a.tickets[ng + g];  // this launch's granule tag - 1
  ATTN_STAMP(1);
  int ns, kps;
  if constexpr (FUSED || ONE) {
    ns = 1;
    kps = (Tk + kBlk - 1) / kBlk * kBlk;
  } else {
    attn2_splits(Tk, a.min_keys, a.maxsplit, a.target, a.single, ns, kps);
  }
  if (s >= ns) return;
  const int kb = s * kps, ke = min(Tk, kb + kps);
  const int nblk = (ke - kb + kBlk - 1) / kBlk;

  float m = -INFINITY, l = 0.f;   // of head `col` (identical across row groups)
  float o[NREP][8];
#pragma unroll
  for (int h = 0; h < NREP; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[h][e] = 0.f;

  int b = wave;
  if (s != 0) {
    if (b < nblk) load_blk(I0{}, kb + b * kBlk, ke - 1);
    if constexpr (PFD == 2)
      if (b + NW < nblk) load_blk(I1{}, kb + (b + NW) * kBlk, ke - 1);
    if constexpr (PFD == 4) {
      if (b + NW < nblk) load_blk(std::integral_constant<int, 1>{}, kb + (b + NW) * kBlk, ke - 1);
      if (b + 2 * NW < nblk)
        load_blk(std::integral_constant<int, 2>{}, kb + (b + 2 * NW) * kBlk, ke - 1);
      if (b + 3 * NW < nblk)
        load_blk(std::integral_constant<int, 3>{}, kb + (b + 3 * NW) * kBlk, ke - 1);
    }
  }
  ATTN_STAMP(2);
  // one key block from slot `slot`; the block PFD x NW further on is requested into the
  // freed slot before this one is computed
  auto block = [&](auto slot, int b) {
    constexpr int SL = decltype(slot)::value;
    const int key0 = kb + b * kBlk;
    uint4 kc[DS], vc[KPL];
#pragma unroll
    for (int d = 0; d < DS; ++d) kc[d] = kf[SL][d];
#pragma unroll
    for (int j = 0; j < KPL; ++j) vc[j] = vf[SL][j];
    if (b + PFD * NW < nblk) load_blk(slot, key0 + PFD * NW * kBlk, ke - 1);
    // scores: S[key 4 rg + e][col]
    cf32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < DS; ++d) acc = cmfma<DT>(kc[d], qf[d], acc);
    float sc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) sc[e] = key0 + 4 * rg + e < ke ? acc[e] : -INFINITY;
    float bm = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
    bm = xor_max<32>(xor_max<16>(bm));
    const float mn = fmaxf(m, bm);
    const float alpha = exp2f(m - mn);  // 0 on the first block (m = -inf)
    float p[4], ps = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) { p[e] = exp2f(sc[e] - mn); ps += p[e]; }
    ps = xor_add<32>(xor_add<16>(ps));
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int e = 0; e < 4; ++e) pt[(4 * rg + e) * 16 + col] = p[e];
    if (rg == 0) alph[col] = alpha;
    if (b == wave) ATTN_STAMP(6);  // diagnostics: first block's scores done (one split only)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the tile is in LDS
    __builtin_amdgcn_wave_barrier();
    // P.V on this lane's KPL keys x 8 dims; dead keys' V rows are zero
    float al[NREP];
#pragma unroll
    for (int h = 0; h < NREP; ++h) al[h] = alph[h];
#pragma unroll
    for (int h = 0; h < NREP; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) o[h][e] *= al[h];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const int key = key0 + kg * KPL + j;
      float vv[8];
      unpack8<DT>(vc[j], vv);
      if (key >= ke) {
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[e] = 0.f;
      }
      const float* prow = pt + (kg * KPL + j) * 16;
#pragma unroll
      for (int h = 0; h < NREP; ++h) {
        const float ph = prow[h];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[h][e] = fmaf(ph, vv[e], o[h][e]);
      }
    }
    __builtin_amdgcn_wave_barrier();  // tile reads done before the next block's writes
  };
  if constexpr (PFD == 1) {
    for (; b < nblk; b += NW) block(I0{}, b);
  } else if constexpr (PFD == 2) {
    for (; b < nblk; b += 2 * NW) {
      block(I0{}, b);
      if (b + NW < nblk) block(I1{}, b + NW);
    }
  } else {
    for (; b < nblk; b += 4 * NW) {
      block(I0{}, b);
      if (b + NW < nblk) block(std::integral_constant<int, 1>{}, b + NW);
      if (b + 2 * NW < nblk) block(std::integral_constant<int, 2>{}, b + 2 * NW);
      if (b + 3 * NW < nblk) block(std::integral_constant<int, 3>{}, b + 3 * NW);
    }
  }
  ATTN_STAMP(3);
  // sum the key groups: lanes of one dim chunk (lane % NCH) end with the wave's o
#pragma unroll
  for (int h = 0; h < NREP; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = o[h][e];
      if constexpr (NCH == 8) v = xor_add<8>(v);
      o[h][e] = xor_add<32>(xor_add<16>(v));
    }
  // wave states -> LDS: m/l of head col (lanes 0..15), o[h][ch*8..] (lanes 0..NCH-1)
  float* ws = st + wave * (32 + NREP * HD);
  if (lane < 16) { ws[lane] = m; ws[16 + lane] = l; }
  if (kg == 0) {
#pragma unroll
    for (int h = 0; h < NREP; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) ws[32 + h * HD + ch * 8 + e] = o[h][e];
  }
  __syncthreads();
  ATTN_STAMP(4);
  // merge the NW waves: thread -> outputs (h, d) = tid, tid + NT, ...
  constexpr int NT = NW * 64;
  constexpr int NOUT = NREP * HD;
  constexpr int OPT = (NOUT + NT - 1) / NT;
  float mo[OPT], lo[OPT], ao[OPT];
#pragma unroll
  for (int i = 0; i < OPT; ++i) {
    const int idx = tid + i * NT;
    const int h = idx / HD, d = idx - h * HD;
    float M = -INFINITY;
    if (idx < NOUT) {
#pragma unroll
      for (int w = 0; w < NW; ++w) M = fmaxf(M, st[w * (32 + NREP * HD) + h]);
    }
    float L = 0.f, A = 0.f;
    if (idx < NOUT) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float* wsw = st + w * (32 + NREP * HD);
        const float wt = exp2f(wsw[h] - M);  // waves without keys: m = -inf -> 0
        L = fmaf(wt, wsw[16 + h], L);
        A = fmaf(wt, wsw[32 + h * HD + d], A);
      }
    }
    mo[i] = M; lo[i] = L; ao[i] = A;
  }
  if (ns == 1) {  // the whole context in this split: finish here
    ATTN_STAMP(5);
#pragma unroll
    for (int i = 0; i < OPT; ++i) {
      const int idx = tid + i * NT;
      if (idx < NOUT) a.out[(size_t)g * NOUT + idx] = from_f32<DT>(ao[i] / lo[i]);
    }
    if constexpr (!ONE) {
      if (a.stamps != nullptr && tid == 0) {
        unsigned long long* dd = a.stamps + ((size_t)s * ng + g) * 8;
        for (int k = 0; k < 8; ++k) dd[k] = (k < 6 || k == 6) ? stamp[k] : 0ull;
      }
      if (tid == 0) a.tickets[ng + g] = epoch + 1u;
    }
    return;
  }
  // Splits >= 1 publish their partial as 8-byte {value, tag} granules (one sc1 store
  // each; a reader that sees the tag sees the value: no fence, no drain, no ticket) and
  // exit.  Split 0 keeps its own partial in LDS and merges: one wave per head polls
  // the other splits' granules until every tag is this launch's (tag = epoch + 1; the
  // per-kv-head epoch lives in tickets[nkv + g] and is advanced by split 0 at the end,
  // so stale granules of earlier launches never match).
  const unsigned long long tagw = (unsigned long long)(epoch + 1u) << 32;
  unsigned long long* gpart = reinterpret_cast<unsigned long long*>(a.part);
  if (s != 0) {
#pragma unroll
    for (int i = 0; i < OPT; ++i) {
      const int idx = tid + i * NT;
      if (idx < NOUT && !a.drop_partials) {
        const int h = idx / HD, d = idx - h * HD;
        unsigned long long* dst = gpart + ((size_t)(g * NREP + h) * kMaxSplit + s) * (HD + 2);
        if (d == 0) {
          __hip_atomic_store(dst, tagw | __float_as_uint(mo[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(dst + 1, tagw | __float_as_uint(lo[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __hip_atomic_store(dst + 2 + d, tagw | __float_as_uint(ao[i]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    ATTN_STAMP(5);
    if (a.stamps != nullptr && tid == 0) {
      unsigned long long* dd = a.stamps + ((size_t)s * ng + g) * 8;
      for (int k = 0; k < 8; ++k) dd[k] = k < 6 ? stamp[k] : 0ull;
    }
    return;
  }
  // split 0: own partial -> LDS (the p tiles are free now), then the per-head merge
  float* own = lds;  // [NREP][HD + 2]: m, l, o[HD]
  static_assert(NREP * (HD + 2) <= NW * (kBlk * 16 + 16), "own partial fits the p tiles");
  __syncthreads();  // every wave is done with its p tile
#pragma unroll
  for (int i = 0; i < OPT; ++i) {
    const int idx = tid + i * NT;
    if (idx < NOUT) {
      const int h = idx / HD, d = idx - h * HD;
      if (d == 0) { own[h * (HD + 2)] = mo[i]; own[h * (HD + 2) + 1] = lo[i]; }
      own[h * (HD + 2) + 2 + d] = ao[i];
    }
  }
  __syncthreads();
  ATTN_STAMP(5);
  if (wave < NREP) {
    constexpr int DPL = HD / 64;  // output dims per lane
    const int h = wave;
    const unsigned long long* src = gpart + (size_t)(g * NREP + h) * kMaxSplit * (HD + 2);
    const float* ow = own + h * (HD + 2);
    // One poll round covers (m, l) of split `lane` and the o rows of splits 1..16 (all
    // of them at the default 16-split target): every granule requested at once, the
    // round repeated until every tag is this launch's.
    constexpr int RU = 16;  // o rows (splits) per round
    float mt = lane == 0 ? ow[0] : -INFINITY, lt = lane == 0 ? ow[1] : 0.f;
    unsigned long long v[RU][DPL];
    for (int tries = 0;; ++tries) {
      bool ok = true;
      if (lane >= 1 && lane < ns) {
        const unsigned long long gm = __hip_atomic_load(src + lane * (HD + 2), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long gl = __hip_atomic_load(src + lane * (HD + 2) + 1, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        ok = (gm >> 32) == (tagw >> 32) && (gl >> 32) == (tagw >> 32);
        mt = __uint_as_float((unsigned int)gm);
        lt = __uint_as_float((unsigned int)gl);
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int t = 1 + u < ns ? 1 + u : ns - 1;
#pragma unroll
        for (int d = 0; d < DPL; ++d) {
          v[u][d] = __hip_atomic_load(src + t * (HD + 2) + 2 + lane * DPL + d, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
          ok = ok && (v[u][d] >> 32) == (tagw >> 32);
        }
      }
      if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;
      if (tries > kAttnMaxPolls) {
        if (lane == 0) attn_poll_timeout(a.tickets + 2 * ng);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const float M = wave_max(mt);
    const float wt = lane < ns ? exp2f(mt - M) : 0.f;
    const float L = wave_sum(wt * lt);
    float acc[DPL];
#pragma unroll
    for (int d = 0; d < DPL; ++d) acc[d] = __shfl(wt, 0, 64) * ow[2 + lane * DPL + d];
    for (int t0 = 1;; t0 += RU) {
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const float w = __shfl(wt, t0 + u < ns ? t0 + u : 63, 64);
        const float wu = t0 + u < ns ? w : 0.f;
#pragma unroll
        for (int d = 0; d < DPL; ++d) acc[d] = fmaf(wu, __uint_as_float((unsigned int)v[u][d]), acc[d]);
      }
      if (t0 + RU >= ns) break;
      // further rounds (more than 17 splits: a split target above 16)
      for (int tries = 0;; ++tries) {
        bool ok = true;
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int t = t0 + RU + u < ns ? t0 + RU + u : ns - 1;
#pragma unroll
          for (int d = 0; d < DPL; ++d) {
            v[u][d] = __hip_atomic_load(src + t * (HD + 2) + 2 + lane * DPL + d, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
            ok = ok && (v[u][d] >> 32) == (tagw >> 32);
          }
        }
        if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;
        if (tries > kAttnMaxPolls) {
          if (lane == 0) attn_poll_timeout(a.tickets + 2 * ng);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    const float inv = 1.f / L;
    uint16_t* dst = a.out + (size_t)(g * NREP + h) * HD + lane * DPL;
#pragma unroll
    for (int d = 0; d < DPL; ++d) dst[d] = from_f32<DT>(acc[d] * inv);
  }
  ATTN_STAMP(7);
  if (tid == 0) a.tickets[ng + g] = epoch + 1u;  // the next launch's tag
  if (a.stamps != nullptr && tid == 0) {
    unsigned long long* dd = a.stamps + ((size_t)s * ng + g) * 8;
    for (int k = 0; k < 8; ++k) dd[k] = (k == 6) ? stamp[5] : stamp[k];
  }
}

}  // namespace cake
