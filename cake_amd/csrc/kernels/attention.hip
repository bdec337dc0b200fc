// KV-cached GQA attention (decode split-K + causal prefill).
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
//   * Decode is flash-decoding: grid (nkv, S/64) — each workgroup owns 64 keys
//     (one per lane), computes a local softmax and P·V in f32, and writes
//     (max, sum, o[hd]) partials; the last-arriving split merges them (one
//     launch per layer).  The grid is sized for max_seq so the launch is
//     hipGraph-replayable; blocks past the live length exit immediately.
//   * Prefill: one wave per (query row, head) with an online softmax over
//     64-key tiles; the causal limit is offset-aware (pos0 + t), which fixes the
//     reference's index_pos==0-only mask and enables
//     chunked prefill.
#include "common.h"

namespace cake {

constexpr int kKeysPerSplit = 64;

// Decode attention moves a few hundred KB while HBM sits idle for ~5 us; extra
// workgroups appended to its grid (blockIdx.y >= nsplit) read the o_proj
// weights that the next launch needs, with ordinary (allocating) loads, so they
// land in the memory-side Infinity Cache (MALL, 256 MB) and the GEMV reads them
// from there.  Read-only: the loaded words are folded into a register that an
// empty volatile asm consumes, which keeps the loads alive without any store.
template <int NT>
__device__ __forceinline__ void prefetch_blocks(const uint4* __restrict__ p, size_t nchunks,
                                                int b, int nb) {
  const size_t per = (nchunks + nb - 1) / nb;
  const size_t lo = (size_t)b * per;
  const size_t hi = lo + per < nchunks ? lo + per : nchunks;
  unsigned int acc = 0u;
  constexpr int UN = 8;
  size_t i = lo + threadIdx.x;
  for (; i + (UN - 1) * NT < hi; i += UN * NT) {
    uint4 v[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) v[u] = p[i + u * NT];
#pragma unroll
    for (int u = 0; u < UN; ++u) acc ^= v[u].x ^ v[u].w;
  }
  for (; i < hi; i += NT) { const uint4 v = p[i]; acc ^= v.x ^ v.w; }
  asm volatile("" ::"v"(acc));
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
// One workgroup = (kv head g, 64-key split s), NREP waves (one per query head
// of the GQA group).  K/V rows of the split are staged into LDS with coalesced
// 16-byte loads (K rows padded by 16 B so the per-lane row reads are
// conflict-free), scores/softmax/P·V run from LDS, and the split's
// (max, sum, o[HD]) partial goes to a workspace.  The LAST split to finish
// (agent-scope release/acquire ticket per kv head) merges all partials and
// writes the head outputs, so no separate combine launch exists; a
// single-split context (Tk <= 64) writes its output directly.
template <int DT, int HD, int NREP>
__global__ __launch_bounds__(64 * NREP) void attn_decode_kernel(
    const float* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int* __restrict__ pos_ptr, int S, float scale,
    float* __restrict__ part, int nsplit, unsigned int* __restrict__ tickets,
    uint16_t* __restrict__ out, const uint4* __restrict__ pf, size_t pf_chunks) {
  constexpr int DPL = HD / 64;         // output dims per lane
  constexpr int KROW = HD + 8;         // padded K row (elements)
  constexpr int CPR = HD / 8;          // 16-byte chunks per row
  constexpr int NT = 64 * NREP;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[kKeysPerSplit * KROW];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[kKeysPerSplit * HD];
  __shared__ __attribute__((aligned(16))) float qs[NREP * HD];
  __shared__ float ps[NREP * kKeysPerSplit];
  __shared__ unsigned int last_flag;

  const int g = blockIdx.x, s = blockIdx.y;
  if (s >= nsplit) {  // Infinity-Cache warm-up of the next GEMV's weights (see header)
    prefetch_blocks<64 * NREP>(pf, pf_chunks, (s - nsplit) * gridDim.x + g,
                               (gridDim.y - nsplit) * gridDim.x);
    return;
  }
  const int Tk = *pos_ptr + 1;
  const int k0 = s * kKeysPerSplit;
  if (k0 >= Tk) return;
  const int kn = min(kKeysPerSplit, Tk - k0);
  const int ns = (Tk + kKeysPerSplit - 1) / kKeysPerSplit;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int h = g * NREP + wave;

  const uint4* kg = reinterpret_cast<const uint4*>(kc + ((size_t)g * S + k0) * HD);
  const uint4* vg = reinterpret_cast<const uint4*>(vc + ((size_t)g * S + k0) * HD);
  for (int i = tid; i < kn * CPR; i += NT) {
    const int r = i / CPR, c = i - r * CPR;
    *reinterpret_cast<uint4*>(Ks + r * KROW + c * 8) = kg[i];
    reinterpret_cast<uint4*>(Vs)[i] = vg[i];
  }
  for (int i = tid; i < NREP * HD; i += NT) qs[i] = q[(size_t)g * NREP * HD + i];
  __syncthreads();

  // scores: lane j <-> key k0 + j
  float sc = -INFINITY;
  if (lane < kn) {
    const uint16_t* kr = Ks + lane * KROW;
    const float* qh = qs + wave * HD;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < CPR; ++c) {
      float kf[8];
      unpack8<DT>(*reinterpret_cast<const uint4*>(kr + c * 8), kf);
      const float4 qa = *reinterpret_cast<const float4*>(qh + c * 8);
      const float4 qb = *reinterpret_cast<const float4*>(qh + c * 8 + 4);
      acc = fmaf(qa.x, kf[0], acc); acc = fmaf(qa.y, kf[1], acc);
      acc = fmaf(qa.z, kf[2], acc); acc = fmaf(qa.w, kf[3], acc);
      acc = fmaf(qb.x, kf[4], acc); acc = fmaf(qb.y, kf[5], acc);
      acc = fmaf(qb.z, kf[6], acc); acc = fmaf(qb.w, kf[7], acc);
    }
    sc = acc * scale;
  }
  const float m = wave_max(sc);
  const float p = lane < kn ? __expf(sc - m) : 0.f;
  const float l = wave_sum(p);
  ps[wave * kKeysPerSplit + lane] = p;
  __syncthreads();

  float o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  const float* pw = ps + wave * kKeysPerSplit;
#pragma unroll 8
  for (int j = 0; j < kn; ++j) {
    const float pj = pw[j];
    const uint16_t* vr = Vs + j * HD + lane * DPL;
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[d] = fmaf(pj, to_f32<DT>(vr[d]), o[d]);
  }

  if (ns == 1) {  // whole context in this split: finish here
    const float inv = 1.f / l;
#pragma unroll
    for (int d = 0; d < DPL; ++d) out[(size_t)h * HD + lane * DPL + d] = from_f32<DT>(o[d] * inv);
    return;
  }

  float* dst = part + ((size_t)h * nsplit + s) * (HD + 2);
  if (lane == 0) { dst[0] = m; dst[1] = l; }
#pragma unroll
  for (int d = 0; d < DPL; ++d) dst[2 + lane * DPL + d] = o[d];

  // publish: stores -> vmcnt(0) -> barrier -> release(agent) -> ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned int t =
        __hip_atomic_fetch_add(&tickets[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned int last = (t == (unsigned int)(ns - 1)) ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tickets[g] = 0u;  // re-arm for the next launch
    }
    last_flag = last;
  }
  __syncthreads();
  if (!last_flag) return;

  // combine all ns partials of this wave's head
  const float* src = part + (size_t)h * nsplit * (HD + 2);
  float M = -INFINITY;
  for (int t = 0; t < ns; ++t) M = fmaxf(M, src[t * (HD + 2)]);
  float L = 0.f, acc[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) acc[d] = 0.f;
#pragma unroll 4
  for (int t = 0; t < ns; ++t) {
    const float* pt = src + t * (HD + 2);
    const float w = __expf(pt[0] - M);
    L = fmaf(w, pt[1], L);
#pragma unroll
    for (int d = 0; d < DPL; ++d) acc[d] = fmaf(w, pt[2 + lane * DPL + d], acc[d]);
  }
  const float inv = 1.f / L;
#pragma unroll
  for (int d = 0; d < DPL; ++d) out[(size_t)h * HD + lane * DPL + d] = from_f32<DT>(acc[d] * inv);
}

// ---------------------------------------------------------------------------
// prefill (T query rows at positions pos0 .. pos0+T-1, causal)
// q: [T, nh, HD] (16-bit, roped); out: [T, nh, HD] (16-bit)
// ---------------------------------------------------------------------------
template <int DT, int HD>
__global__ __launch_bounds__(256) void attn_prefill_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, int pos0, int T, int S, int nh, int nkv,
    float scale, uint16_t* __restrict__ out) {
  constexpr int DPL = HD / 64;
  __shared__ float qs[4 * HD];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.x;
  const int t = blockIdx.y * 4 + wave;
  const int g = h / (nh / nkv);
  const bool active = t < T;
  if (active)
    for (int i = lane; i < HD; i += 64)
      qs[wave * HD + i] = to_f32<DT>(q[((size_t)t * nh + h) * HD + i]);
  __syncthreads();
  if (!active) return;
  const float* qh = qs + wave * HD;
  const int Tk = pos0 + t + 1;
  const uint16_t* kbase = kc + (size_t)g * S * HD;
  const uint16_t* vbase = vc + (size_t)g * S * HD;
  float m = -INFINITY, l = 0.f, o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  for (int k0 = 0; k0 < Tk; k0 += 64) {
    const int kn = min(64, Tk - k0);
    float sc = -INFINITY;
    if (lane < kn) {
      const uint4* kr = reinterpret_cast<const uint4*>(kbase + (size_t)(k0 + lane) * HD);
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < HD / 8; ++c) {
        float kf[8];
        unpack8<DT>(kr[c], kf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(qh[c * 8 + e], kf[e], acc);
      }
      sc = acc * scale;
    }
    const float mt = wave_max(sc);
    const float mn = fmaxf(m, mt);
    const float alpha = __expf(m - mn);  // m=-inf on the first tile -> 0
    const float p = lane < kn ? __expf(sc - mn) : 0.f;
    l = l * alpha + wave_sum(p);
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[d] *= alpha;
    for (int j = 0; j < kn; ++j) {
      const float pj = __shfl(p, j, 64);
      const uint16_t* vr = vbase + (size_t)(k0 + j) * HD + lane * DPL;
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[d] = fmaf(pj, to_f32<DT>(vr[d]), o[d]);
    }
    m = mn;
  }
  const float inv = 1.f / l;
#pragma unroll
  for (int d = 0; d < DPL; ++d)
    out[((size_t)t * nh + h) * HD + lane * DPL + d] = from_f32<DT>(o[d] * inv);
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

// part: workspace [nh][nsplit][hd+2] f32, nsplit = ceil(S / 64);
// tickets: [nkv] u32, zero-initialised once (the kernel re-arms them).
template <int DT, int HD>
static int launch_decode(int n_rep, dim3 grid, hipStream_t st, const float* q, const void* kc,
                         const void* vc, const int* pos, int S, float scale, float* part,
                         int nsplit, unsigned int* tickets, void* out, const void* pf,
                         size_t pf_chunks) {
#define CAKE_DEC(NR)                                                                         \
  hipLaunchKernelGGL((attn_decode_kernel<DT, HD, NR>), grid, dim3(64 * NR), 0, st, q,        \
                     (const uint16_t*)kc, (const uint16_t*)vc, pos, S, scale, part, nsplit,  \
                     tickets, (uint16_t*)out, (const uint4*)pf, pf_chunks)
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

// pf/pf_bytes/pf_rows: optional read-only weight range to warm into the
// Infinity Cache with pf_rows extra grid rows (nkv workgroups each).
CAKE_API int cake_attn_decode_pf(int dt, const float* q, const void* kc, const void* vc,
                                 const int* pos, int S, int nh, int nkv, int hd, float scale,
                                 float* part, unsigned int* tickets, void* out, const void* pf,
                                 size_t pf_bytes, int pf_rows, hipStream_t st) {
  const int n_rep = nh / nkv;
  if (nh % nkv || n_rep > 8 || pf_bytes % 16 || pf_rows < 0) return (int)hipErrorInvalidValue;
  if (pf == nullptr || pf_bytes == 0) pf_rows = 0;
  const int nsplit = (S + kKeysPerSplit - 1) / kKeysPerSplit;
  const dim3 grid(nkv, nsplit + pf_rows);
  DISPATCH_DT_HD(dt, hd, return (launch_decode<DT, HD>(n_rep, grid, st, q, kc, vc, pos, S, scale,
                                                       part, nsplit, tickets, out, pf,
                                                       pf_bytes / 16)));
  return (int)hipErrorInvalidValue;
}

CAKE_API int cake_attn_decode(int dt, const float* q, const void* kc, const void* vc,
                              const int* pos, int S, int nh, int nkv, int hd, float scale,
                              float* part, unsigned int* tickets, void* out, hipStream_t st) {
  return cake_attn_decode_pf(dt, q, kc, vc, pos, S, nh, nkv, hd, scale, part, tickets, out,
                             nullptr, 0, 0, st);
}

CAKE_API int cake_attn_prefill(int dt, const void* q, const void* kc, const void* vc,
                               int pos0, int T, int S, int nh, int nkv, int hd, float scale,
                               void* out, hipStream_t st) {
  if (nh % nkv) return (int)hipErrorInvalidValue;
  DISPATCH_DT_HD(dt, hd,
                 hipLaunchKernelGGL((attn_prefill_kernel<DT, HD>), dim3(nh, (T + 3) / 4),
                                    dim3(256), 0, st, (const uint16_t*)q,
                                    (const uint16_t*)kc, (const uint16_t*)vc, pos0, T, S, nh,
                                    nkv, scale, (uint16_t*)out));
  return (int)hipGetLastError();
}
