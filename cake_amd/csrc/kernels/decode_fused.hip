// Fused decode step: GQA attention (split-K) + o_proj GEMV + residual, ONE launch.
//
// Why: at batch 1 the attention of a decode step reads almost nothing (the
// KV rows of one token history, ~100 KB) and is latency-bound for ~5 us, during
// which HBM sits idle; o_proj then streams 32 MB (8B) as a separate launch with
// its own ramp/drain.  Here every workgroup first issues the loads of its o_proj
// weight rows into registers, then helps with attention, then waits for the
// attention output and finishes o_proj from registers — the weight stream runs
// underneath the attention.  Replaces attention.rs:96-120 + o_proj (K09-K14).
//
// Attention units (kv head, 64-key split) run on the lowest workgroup ids
// before those workgroups wait on anything; every workgroup then spins
// (bounded, one lane, s_sleep) on a done-counter.  Inter-workgroup hand-offs
// use the agent-scope release/acquire recipe of the CDNA guide (§6 Guideline
// 16): stores -> vmcnt(0) -> barrier -> release fence -> relaxed atomic;
// consumer: relaxed poll -> acquire fence.  The done-counter is re-armed by
// the QKV kernel that precedes each launch (stream order), so no exit ticket
// is needed and the launch replays unchanged inside a hipGraph.
#include "common.h"

namespace cake {

constexpr int kAoThreads = 256;
constexpr int kKeys = 64;

struct AOArgs {
  const float* q;           // [nh*HD] f32 roped
  const uint16_t* kc;       // [nkv][S][HD] (this layer)
  const uint16_t* vc;
  const int* pos;           // device scalar
  int S, nkv;
  float scale;
  float* part;              // [nh][nsplit][HD+2]
  int nsplit;
  unsigned int* tickets;    // [nkv] split-combine tickets
  unsigned int* ctl;        // [1] kv-head groups done (re-armed by the QKV kernel)
  uint16_t* attn_out;       // [nh*HD]
  const uint16_t* wo;       // [N, K]
  int K, N;
  float* resid;             // [N] f32, += wo @ attn_out
  int* err;                 // set to 1 on a spin timeout
  int sleep;                // poll back-off, in units of s_sleep 8 (~512 clk)
};

__device__ __forceinline__ void publish_release() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// One attention unit: kv head g, keys [64s, 64s+64).  4 waves; wave w handles
// query heads w, w+4 (NREP = 8) of the group.  Returns via LDS-free globals.
template <int DT, int HD, int NREP>
__device__ void attn_unit(const AOArgs& a, int g, int s, int Tk, uint16_t* Ks, uint16_t* Vs,
                          float* qs, float* ps, unsigned int* flag) {
  constexpr int DPL = HD / 64, KROW = HD + 8, CPR = HD / 8;
  constexpr int HPW = NREP > 4 ? NREP / 4 : 1;  // heads per wave
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int k0 = s * kKeys;
  const int kn = min(kKeys, Tk - k0);
  const int ns = (Tk + kKeys - 1) / kKeys;
  const uint4* kg = reinterpret_cast<const uint4*>(a.kc + ((size_t)g * a.S + k0) * HD);
  const uint4* vg = reinterpret_cast<const uint4*>(a.vc + ((size_t)g * a.S + k0) * HD);
  for (int i = tid; i < kn * CPR; i += kAoThreads) {
    const int r = i / CPR, c = i - r * CPR;
    *reinterpret_cast<uint4*>(Ks + r * KROW + c * 8) = kg[i];
    reinterpret_cast<uint4*>(Vs)[i] = vg[i];
  }
  for (int i = tid; i < NREP * HD; i += kAoThreads) qs[i] = a.q[(size_t)g * NREP * HD + i];
  __syncthreads();
  float m[HPW], l[HPW], o[HPW][DPL];
#pragma unroll
  for (int hh = 0; hh < HPW; ++hh) {
    const int hl = wave + 4 * hh;  // local head index in the group
    if (hl >= NREP) { m[hh] = 0.f; l[hh] = 0.f; continue; }
    float sc = -INFINITY;
    if (lane < kn) {
      const uint16_t* kr = Ks + lane * KROW;
      const float* qh = qs + hl * HD;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < CPR; ++c) {
        float kf[8];
        unpack8<DT>(*reinterpret_cast<const uint4*>(kr + c * 8), kf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(qh[c * 8 + e], kf[e], acc);
      }
      sc = acc * a.scale;
    }
    m[hh] = wave_max(sc);
    const float p = lane < kn ? __expf(sc - m[hh]) : 0.f;
    l[hh] = wave_sum(p);
    ps[hl * kKeys + lane] = p;
  }
  __syncthreads();
#pragma unroll
  for (int hh = 0; hh < HPW; ++hh) {
    const int hl = wave + 4 * hh;
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[hh][d] = 0.f;
    if (hl >= NREP) continue;
    const float* pw = ps + hl * kKeys;
#pragma unroll 8
    for (int j = 0; j < kn; ++j) {
      const float pj = pw[j];
      const uint16_t* vr = Vs + j * HD + lane * DPL;
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[hh][d] = fmaf(pj, to_f32<DT>(vr[d]), o[hh][d]);
    }
  }
  bool finished = false;  // this workgroup wrote the group's final outputs
  if (ns == 1) {
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) {
      const int hl = wave + 4 * hh;
      if (hl >= NREP) continue;
      const int h = g * NREP + hl;
      const float inv = 1.f / l[hh];
#pragma unroll
      for (int d = 0; d < DPL; ++d)
        a.attn_out[(size_t)h * HD + lane * DPL + d] = from_f32<DT>(o[hh][d] * inv);
    }
    finished = true;
  } else {
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) {
      const int hl = wave + 4 * hh;
      if (hl >= NREP) continue;
      const int h = g * NREP + hl;
      float* dst = a.part + ((size_t)h * a.nsplit + s) * (HD + 2);
      if (lane == 0) { dst[0] = m[hh]; dst[1] = l[hh]; }
#pragma unroll
      for (int d = 0; d < DPL; ++d) dst[2 + lane * DPL + d] = o[hh][d];
    }
    publish_release();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t =
          __hip_atomic_fetch_add(&a.tickets[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned last = t == (unsigned)(ns - 1) ? 1u : 0u;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        a.tickets[g] = 0u;
      }
      *flag = last;
    }
    __syncthreads();
    if (*flag) {
#pragma unroll
      for (int hh = 0; hh < HPW; ++hh) {
        const int hl = wave + 4 * hh;
        if (hl >= NREP) continue;
        const int h = g * NREP + hl;
        const float* src = a.part + (size_t)h * a.nsplit * (HD + 2);
        float M = -INFINITY;
        for (int t = 0; t < ns; ++t) M = fmaxf(M, src[t * (HD + 2)]);
        float L = 0.f, acc[DPL];
#pragma unroll
        for (int d = 0; d < DPL; ++d) acc[d] = 0.f;
        for (int t = 0; t < ns; ++t) {
          const float* pt = src + t * (HD + 2);
          const float w = __expf(pt[0] - M);
          L = fmaf(w, pt[1], L);
#pragma unroll
          for (int d = 0; d < DPL; ++d) acc[d] = fmaf(w, pt[2 + lane * DPL + d], acc[d]);
        }
        const float inv = 1.f / L;
#pragma unroll
        for (int d = 0; d < DPL; ++d)
          a.attn_out[(size_t)h * HD + lane * DPL + d] = from_f32<DT>(acc[d] * inv);
      }
      finished = true;
    }
  }
  // a completed kv-head group: publish its outputs (release) and count it
  if (finished) {
    publish_release();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&a.ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();  // LDS reuse by the next unit
}

template <int DT, int HD, int NREP, int PFC>
__global__ __launch_bounds__(kAoThreads, 2) void attn_oproj_kernel(AOArgs a) {
  constexpr int KROW = HD + 8;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[kKeys * KROW];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[kKeys * HD];
  __shared__ __attribute__((aligned(16))) float qs[NREP * HD];
  __shared__ float ps[NREP * kKeys];
  __shared__ unsigned int sh[2];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int npairs = (a.N + 1) >> 1;
  const int stride = gridDim.x * (kAoThreads / 64);
  const int p0 = blockIdx.x * (kAoThreads / 64) + wave;

  // 1. attention: workgroup u < units executes unit u (kv head u % nkv, split
  //    u / nkv) before it waits on anything.  Units sit on the lowest
  //    workgroup ids (dispatched first); the wait below is bounded, so even an
  //    out-of-order dispatch degrades to an error flag, never a hang.
  const int Tk = *a.pos + 1;
  const int ns = (Tk + kKeys - 1) / kKeys;
  const int units = a.nkv * ns;
  for (int u = blockIdx.x; u < units; u += gridDim.x)
    attn_unit<DT, HD, NREP>(a, u % a.nkv, u / a.nkv, Tk, Ks, Vs, qs, ps, &sh[1]);

  // 2. stream this wave's first o_proj pair into registers while the
  //    remaining attention units finish elsewhere
  uint4 ra[PFC > 0 ? PFC : 1], rb[PFC > 0 ? PFC : 1];
  if (PFC > 0 && p0 < npairs) {
    const uint4* a4 = reinterpret_cast<const uint4*>(a.wo + (size_t)(2 * p0) * a.K);
    const uint4* b4 = reinterpret_cast<const uint4*>(a.wo + (size_t)min(2 * p0 + 1, a.N - 1) * a.K);
#pragma unroll
    for (int c = 0; c < PFC; ++c) {
      ra[c] = ld_nt16(a4 + c * 64 + lane);
      rb[c] = ld_nt16(b4 + c * 64 + lane);
    }
  }

  // 3. wait until every kv-head group is complete (bounded spin, one lane).
  //    ctl[1] is re-armed to 0 by the QKV kernel that precedes this launch.
  if (tid == 0) {
    unsigned int spins = 0;
    while (__hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           (unsigned)a.nkv) {
      for (int z = 0; z < a.sleep; ++z) __builtin_amdgcn_s_sleep(8);
      if (++spins > (1u << 22)) { atomicExch(a.err, 1); break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // 4. stage attention output (bf16/f16 [K]) into LDS (reuses the K tile)
  uint16_t* xs = Ks;  // K*2 bytes <= 16 KB  (checked on the host)
  for (int i = tid * 8; i < a.K; i += kAoThreads * 8)
    *reinterpret_cast<uint4*>(xs + i) = *reinterpret_cast<const uint4*>(a.attn_out + i);
  __syncthreads();

  // 5. o_proj + residual
  const int nch = a.K >> 3;
  for (int p = p0; p < npairs; p += stride) {
    const uint16_t* wa = a.wo + (size_t)(2 * p) * a.K;
    const uint16_t* wb = a.wo + (size_t)min(2 * p + 1, a.N - 1) * a.K;
    float aa = 0.f, ab = 0.f;
    int c_start = 0;
    if (PFC > 0 && p == p0) {
#pragma unroll
      for (int c = 0; c < PFC; ++c) {
        float xv[8], fa[8], fb[8];
        unpack8<DT>(reinterpret_cast<const uint4*>(xs)[c * 64 + lane], xv);
        unpack8<DT>(ra[c], fa);
        unpack8<DT>(rb[c], fb);
#pragma unroll
        for (int e = 0; e < 8; ++e) { aa = fmaf(fa[e], xv[e], aa); ab = fmaf(fb[e], xv[e], ab); }
      }
      c_start = PFC * 64;
    }
    const uint4* a4 = reinterpret_cast<const uint4*>(wa);
    const uint4* b4 = reinterpret_cast<const uint4*>(wb);
    for (int c0 = c_start; c0 < nch; c0 += 64 * 4) {
      uint4 va[4], vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + u * 64 + lane;
        va[u] = c < nch ? ld_nt16(a4 + c) : make_uint4(0, 0, 0, 0);
        vb[u] = c < nch ? ld_nt16(b4 + c) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + u * 64 + lane;
        if (c >= nch) continue;
        float xv[8], fa[8], fb[8];
        unpack8<DT>(reinterpret_cast<const uint4*>(xs)[c], xv);
        unpack8<DT>(va[u], fa);
        unpack8<DT>(vb[u], fb);
#pragma unroll
        for (int e = 0; e < 8; ++e) { aa = fmaf(fa[e], xv[e], aa); ab = fmaf(fb[e], xv[e], ab); }
      }
    }
    aa = wave_sum(aa);
    ab = wave_sum(ab);
    if (lane == 0) {
      a.resid[2 * p] += aa;
      if (2 * p + 1 < a.N) a.resid[2 * p + 1] += ab;
    }
  }
}

}  // namespace cake

using namespace cake;

// ctl: 3 u32 zero-initialised once; err: 1 int; tickets: nkv u32 zeroed once.
CAKE_API int cake_attn_oproj(int dt, const float* q, const void* kc, const void* vc,
                             const int* pos, int S, int nh, int nkv, int hd, float scale,
                             float* part, unsigned int* tickets, unsigned int* ctl, void* attn_out,
                             const void* wo, int N, float* resid, int* err, int grid,
                             int prefetch, int sleep_units, hipStream_t st) {
  const int n_rep = nh / nkv;
  const int K = nh * hd;
  if (nh % nkv || hd != 128 || (n_rep != 4 && n_rep != 8) || K % 8 || K * 2 > 64 * (hd + 8) * 2 ||
      K / 8 < 64 * 8 || grid <= 0)
    return (int)hipErrorInvalidValue;
  AOArgs a{q, (const uint16_t*)kc, (const uint16_t*)vc, pos, S, nkv, scale, part,
           (S + kKeys - 1) / kKeys, tickets, ctl, (uint16_t*)attn_out, (const uint16_t*)wo, K, N,
           resid, err, sleep_units};
#define CAKE_AO(DTV, NR)                                                                       \
  do {                                                                                         \
    if (prefetch)                                                                              \
      hipLaunchKernelGGL((attn_oproj_kernel<DTV, 128, NR, 8>), dim3(grid), dim3(kAoThreads), 0, \
                         st, a);                                                               \
    else                                                                                       \
      hipLaunchKernelGGL((attn_oproj_kernel<DTV, 128, NR, 0>), dim3(grid), dim3(kAoThreads), 0, \
                         st, a);                                                               \
  } while (0)
  if (dt == kBF16) { if (n_rep == 4) CAKE_AO(kBF16, 4); else CAKE_AO(kBF16, 8); }
  else if (dt == kF16) { if (n_rep == 4) CAKE_AO(kF16, 4); else CAKE_AO(kF16, 8); }
  else return (int)hipErrorInvalidValue;
#undef CAKE_AO
  return (int)hipGetLastError();
}
