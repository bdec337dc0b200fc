// Decode GEMV kernels (shared by gemv.hip, gemv_mlp.hip, gemv_head.hip: the launchers
// are split across translation units so their many (dtype, U, prefetch, NX)
// instantiations compile in parallel).  Design notes: gemv.hip.
#pragma once
#include "common.h"

namespace cake {

constexpr int kGemvThreads = 256;  // 4 waves
constexpr int kGemvWaves = kGemvThreads / 64;
constexpr int kGemvMaxBlocks = 1024;

// ---------------------------------------------------------------------------
// x staging (prologues)
// ---------------------------------------------------------------------------

// Normalise a f32 row into LDS:  xs[i] = x[i] * rsqrt(mean(x^2) + eps) * w[i].
template <int DT>
__device__ __forceinline__ void stage_rmsnorm(const float* __restrict__ x,
                                              const uint16_t* __restrict__ w,
                                              float eps, int K, float* xs) {
  __shared__ float red[16];
  float ss = 0.f;
  for (int i = threadIdx.x * 4; i < K; i += kGemvThreads * 4) {
    const float4 v = *reinterpret_cast<const float4*>(x + i);
    *reinterpret_cast<float4*>(xs + i) = v;
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = block_sum(ss, red);
  const float r = rsqrtf(ss / (float)K + eps);
  for (int i = threadIdx.x * 4; i < K; i += kGemvThreads * 4) {
    float4 v = *reinterpret_cast<float4*>(xs + i);
    const uint2 wv = *reinterpret_cast<const uint2*>(w + i);
    v.x *= r * to_f32<DT>((uint16_t)(wv.x & 0xffff));
    v.y *= r * to_f32<DT>((uint16_t)(wv.x >> 16));
    v.z *= r * to_f32<DT>((uint16_t)(wv.y & 0xffff));
    v.w *= r * to_f32<DT>((uint16_t)(wv.y >> 16));
    *reinterpret_cast<float4*>(xs + i) = v;
  }
  __syncthreads();
}

// Copy a 16-bit activation row into LDS (kept 16-bit: 70B down_proj has K=28672).
__device__ __forceinline__ void stage_plain16(const uint16_t* __restrict__ x, int K,
                                              uint16_t* xs) {
  for (int i = threadIdx.x * 8; i < K; i += kGemvThreads * 8)
    *reinterpret_cast<uint4*>(xs + i) = *reinterpret_cast<const uint4*>(x + i);
  __syncthreads();
}

// Split x prologues (NX > 0, used with a weight prefetch PFC > 0): the x loads
// are issued FIRST, then the wave's first weight rows, then the x half is
// finished.  Loads retire in order (vmcnt), so issuing the weights first — the
// plain prologue order — made the norm wait for the whole weight batch; in this
// order the norm waits only for x, and its reduction / LDS round trips overlap
// the weight stream.  K = 1024 NX (RMSNorm, f32 row) or 2048 NX (16-bit row).
template <int DT, int NX> struct NormPre {  // K <= 1024 NX, K % 4 == 0
  float4 x[NX];
  uint2 w[NX];
  __device__ __forceinline__ void load(const float* __restrict__ xg, const uint16_t* __restrict__ wg,
                                       int K) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = (j * kGemvThreads + threadIdx.x) * 4;
      x[j] = i < K ? *reinterpret_cast<const float4*>(xg + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      w[j] = i < K ? *reinterpret_cast<const uint2*>(wg + i) : make_uint2(0u, 0u);
    }
  }
  __device__ __forceinline__ void finish(float eps, int K, float* xs) {
    __shared__ float red[16];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < NX; ++j) ss += x[j].x * x[j].x + x[j].y * x[j].y + x[j].z * x[j].z + x[j].w * x[j].w;
    ss = block_sum(ss, red);
    const float r = rsqrtf(ss / (float)K + eps);
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = (j * kGemvThreads + threadIdx.x) * 4;
      float4 v = x[j];
      v.x *= r * to_f32<DT>((uint16_t)(w[j].x & 0xffff));
      v.y *= r * to_f32<DT>((uint16_t)(w[j].x >> 16));
      v.z *= r * to_f32<DT>((uint16_t)(w[j].y & 0xffff));
      v.w *= r * to_f32<DT>((uint16_t)(w[j].y >> 16));
      if (i < K) *reinterpret_cast<float4*>(xs + i) = v;
    }
    __syncthreads();
  }
};

template <int NX> struct Plain16Pre {  // K <= 2048 NX, K % 8 == 0
  uint4 v[NX];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ xg, int K) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = (j * kGemvThreads + threadIdx.x) * 8;
      v[j] = i < K ? *reinterpret_cast<const uint4*>(xg + i) : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __device__ __forceinline__ void finish(int K, uint16_t* xs) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = (j * kGemvThreads + threadIdx.x) * 8;
      if (i < K) *reinterpret_cast<uint4*>(xs + i) = v[j];
    }
    __syncthreads();
  }
};

template <int DT, bool XF32>
__device__ __forceinline__ void load_x8(const void* xs, int chunk, float* o) {
  if constexpr (XF32) {
    const float4* p = reinterpret_cast<const float4*>(xs) + chunk * 2;
    const float4 a = p[0], b = p[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  } else {
    unpack8<DT>(reinterpret_cast<const uint4*>(xs)[chunk], o);
  }
}

// ---------------------------------------------------------------------------
// core: one wave computes dot products of a PAIR of weight rows with the x row
// staged in LDS.  U = 16-byte chunks per row in flight per lane per iteration
// (2*U loads outstanding).  PFC = chunks per row per lane of the wave's FIRST
// pair issued before the x prologue (RMSNorm / staging) so the HBM stream
// overlaps it; for K = 4096 PFC = 8 is the whole pair (64 VGPRs).  All
// register arrays are indexed by compile-time constants (no scratch).
// ---------------------------------------------------------------------------
template <int DT, bool XF32>
__device__ __forceinline__ void fma_chunk(const void* xs, int chunk, const uint4 va,
                                          const uint4 vb, float& acc_a, float& acc_b) {
  float xv[8], fa[8], fb[8];
  load_x8<DT, XF32>(xs, chunk, xv);
  unpack8<DT>(va, fa);
  unpack8<DT>(vb, fb);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    acc_a = fmaf(fa[e], xv[e], acc_a);
    acc_b = fmaf(fb[e], xv[e], acc_b);
  }
}

// accumulate chunks [c_start, nch) of rows wa, wb
template <int DT, bool XF32, int U>
__device__ __forceinline__ void dot_range(const uint16_t* __restrict__ wa,
                                          const uint16_t* __restrict__ wb, const void* xs,
                                          int nch, int c_start, float& acc_a, float& acc_b) {
  const int lane = threadIdx.x & 63;
  const uint4* a4 = reinterpret_cast<const uint4*>(wa);
  const uint4* b4 = reinterpret_cast<const uint4*>(wb);
  const int full = c_start + ((nch - c_start) / (64 * U)) * (64 * U);
  for (int c0 = c_start; c0 < full; c0 += 64 * U) {
    uint4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = ld_nt16(a4 + c0 + u * 64 + lane);
      vb[u] = ld_nt16(b4 + c0 + u * 64 + lane);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) fma_chunk<DT, XF32>(xs, c0 + u * 64 + lane, va[u], vb[u], acc_a, acc_b);
  }
  for (int c = full + lane; c < nch; c += 64) fma_chunk<DT, XF32>(xs, c, a4[c], b4[c], acc_a, acc_b);
}

template <int N> struct Regs { uint4 a[N], b[N]; };
template <> struct Regs<0> { uint4 a[1], b[1]; };

// issue the first PFC chunks of (wa, wb)
template <int PFC>
__device__ __forceinline__ void prefetch_rows(const uint16_t* wa, const uint16_t* wb, Regs<PFC>& r) {
  if constexpr (PFC > 0) {
    const int lane = threadIdx.x & 63;
    const uint4* a4 = reinterpret_cast<const uint4*>(wa);
    const uint4* b4 = reinterpret_cast<const uint4*>(wb);
#pragma unroll
    for (int c = 0; c < PFC; ++c) {
      r.a[c] = ld_nt16(a4 + c * 64 + lane);
      r.b[c] = ld_nt16(b4 + c * 64 + lane);
    }
  }
}

// Walk the wave's pairs p0, p0+stride, ...: map(p, wa, wb) gives the rows,
// epi(p, da, db) consumes the two dot products (full wave sums).
template <int DT, bool XF32, int U, int PFC, class Map, class Epi>
__device__ __forceinline__ void run_pairs(const Map& map, const Epi& epi, const void* xs, int K,
                                          int npairs, int p0, int stride, const Regs<PFC>& pre) {
  const int nch = K >> 3;
  int p = p0;
  if constexpr (PFC > 0) {
    // Unconditional (an idle wave works on a clamped pair and drops it): a use of
    // the prefetched registers inside a branch lets the compiler sink the
    // prefetch loads past the x prologue's barrier, serialising them again.
    const uint16_t *wa, *wb;
    map(p < npairs ? p : npairs - 1, wa, wb);
    const int lane = threadIdx.x & 63;
    float aa = 0.f, ab = 0.f;
#pragma unroll
    for (int c = 0; c < PFC; ++c) fma_chunk<DT, XF32>(xs, c * 64 + lane, pre.a[c], pre.b[c], aa, ab);
    dot_range<DT, XF32, U>(wa, wb, xs, nch, PFC * 64, aa, ab);
    aa = wave_sum(aa);
    ab = wave_sum(ab);
    if (p < npairs) epi(p, aa, ab);
    p += stride;
  }
  for (; p < npairs; p += stride) {
    const uint16_t *wa, *wb;
    map(p, wa, wb);
    float aa = 0.f, ab = 0.f;
    dot_range<DT, XF32, U>(wa, wb, xs, nch, 0, aa, ab);
    epi(p, wave_sum(aa), wave_sum(ab));
  }
}

// ---------------------------------------------------------------------------
// QKV + RoPE + KV-cache write
// ---------------------------------------------------------------------------
struct QkvArgs {
  const float* resid;      // [K] f32
  const uint16_t* norm_w;  // [K]
  float eps;
  const uint16_t* wq;  // [nh*hd, K]
  const uint16_t* wk;  // [nkv*hd, K]
  const uint16_t* wv;  // [nkv*hd, K]
  int K, nh, nkv, hd;
  const float* inv_freq;  // [hd/2]
  const int* pos;         // device scalar: position of this token
  float* q_out;           // [nh*hd] f32 (roped)
  uint16_t* kcache;       // [nkv][S][hd] (this layer)
  uint16_t* vcache;
  int S;
};

struct QkvRow {
  const uint16_t* base;
  int kind, head, i;  // kind 0=q 1=k 2=v
  size_t ra;
};

__device__ __forceinline__ QkvRow qkv_row(const QkvArgs& a, int p) {
  const int half = a.hd >> 1;
  const int slot = p / half;
  QkvRow r;
  r.i = p - slot * half;
  if (slot < a.nh) { r.kind = 0; r.head = slot; r.base = a.wq; }
  else if (slot < a.nh + a.nkv) { r.kind = 1; r.head = slot - a.nh; r.base = a.wk; }
  else { r.kind = 2; r.head = slot - a.nh - a.nkv; r.base = a.wv; }
  r.ra = (size_t)r.head * a.hd + r.i;
  return r;
}

template <int DT, int U, int PFC, int NX>
__global__ __launch_bounds__(kGemvThreads) void qkv_rope_kernel(QkvArgs a) {
  extern __shared__ float xs[];
  const int half = a.hd >> 1;
  const int npairs = (a.nh + 2 * a.nkv) * half;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int p0 = blockIdx.x * kGemvWaves + wave;
  // base selected by address arithmetic, not a pointer select: a select between
  // kernel-argument fields becomes a memory load of the argument block, which
  // would stand (in vmcnt order) in front of the split prologue's x loads
  // (offsets from wq keep the global address space visible: no flat loads)
  const uint16_t* wq = a.wq;
  const ptrdiff_t dk = a.wk - a.wq, dv = a.wv - a.wq;
  const int nh = a.nh, nqk = a.nh + a.nkv, hd = a.hd, K = a.K;
  auto map = [=](int p, const uint16_t*& wa, const uint16_t*& wb) {
    const int slot = p / half;
    const bool isq = slot < nh, isk = !isq && slot < nqk;
    const uint16_t* base = wq + (isq ? 0 : (isk ? dk : dv));
    const int head = slot - (isq ? 0 : (isk ? nh : nqk));
    const size_t ra = (size_t)head * hd + (p - slot * half);
    wa = base + ra * K;
    wb = base + (ra + half) * K;
  };
  Regs<PFC> pre;
  NormPre<DT, NX> xp;
  const uint16_t *wa0, *wb0;  // rows first: their address math may load (kernarg select)
  map(p0 < npairs ? p0 : npairs - 1, wa0, wb0);
  if constexpr (NX > 0) xp.load(a.resid, a.norm_w, a.K);
  __builtin_amdgcn_sched_barrier(0);  // x loads strictly before the weights (in-order vmcnt)
  if (NX > 0 || (PFC > 0 && p0 < npairs)) prefetch_rows<PFC>(wa0, wb0, pre);  // NX: exact vmcnt
  // the RoPE frequency of the wave's first pair, requested now: loaded in the
  // epilogue it was one more memory round trip at the end of every wave
  const int pc = p0 < npairs ? p0 : npairs - 1;
  const float f0 = a.inv_freq[pc - (pc / half) * half];
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (NX > 0) xp.finish(a.eps, a.K, xs);
  else stage_rmsnorm<DT>(a.resid, a.norm_w, a.eps, a.K, xs);
  const int pos = *a.pos;
  auto epi = [&](int p, float da, float db) {
    if (lane != 0) return;
    const QkvRow r = qkv_row(a, p);
    float oa = da, ob = db;
    if (r.kind < 2) {
      float s, c;
      sincosf((float)pos * (p == p0 ? f0 : a.inv_freq[r.i]), &s, &c);
      oa = da * c - db * s;
      ob = da * s + db * c;
    }
    if (r.kind == 0) {
      a.q_out[r.ra] = oa;
      a.q_out[r.ra + half] = ob;
    } else {
      uint16_t* cache = r.kind == 1 ? a.kcache : a.vcache;
      const size_t off = ((size_t)r.head * a.S + pos) * a.hd + r.i;
      cache[off] = from_f32<DT>(oa);
      cache[off + half] = from_f32<DT>(ob);
    }
  };
  run_pairs<DT, true, U, PFC>(map, epi, xs, a.K, npairs, p0, gridDim.x * kGemvWaves, pre);
}

// ---------------------------------------------------------------------------
// RMSNorm + gate/up + SiLU*mul
// ---------------------------------------------------------------------------
template <int DT, int U, int PFC, int NX>
__global__ __launch_bounds__(kGemvThreads) void swiglu_kernel(
    const float* __restrict__ resid, const uint16_t* __restrict__ norm_w, float eps,
    const uint16_t* __restrict__ wg, const uint16_t* __restrict__ wu, int K, int I,
    uint16_t* __restrict__ act) {
  extern __shared__ float xs[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j0 = blockIdx.x * kGemvWaves + wave;
  auto map = [&](int j, const uint16_t*& wa, const uint16_t*& wb) {
    wa = wg + (size_t)j * K;
    wb = wu + (size_t)j * K;
  };
  Regs<PFC> pre;
  NormPre<DT, NX> xp;
  const int jp = j0 < I ? j0 : I - 1;
  const uint16_t *wa0 = wg + (size_t)jp * K, *wb0 = wu + (size_t)jp * K;
  if constexpr (NX > 0) xp.load(resid, norm_w, K);
  __builtin_amdgcn_sched_barrier(0);  // x loads strictly before the weights (in-order vmcnt)
  // NX: unconditional (an idle wave re-reads the last row), so the vmcnt is exact
  if (NX > 0 || (PFC > 0 && j0 < I)) prefetch_rows<PFC>(wa0, wb0, pre);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (NX > 0) xp.finish(eps, K, xs);
  else stage_rmsnorm<DT>(resid, norm_w, eps, K, xs);
  auto epi = [&](int j, float g, float u) {
    if (lane == 0) act[j] = from_f32<DT>(silu(g) * u);
  };
  run_pairs<DT, true, U, PFC>(map, epi, xs, K, I, j0, gridDim.x * kGemvWaves, pre);
}

// ---------------------------------------------------------------------------
// out (+)= W x   with 16-bit x: o_proj / down_proj (accumulate into the f32
// residual stream) — or plain f32 output.
// ---------------------------------------------------------------------------
template <int DT, int U, int PFC, int NX, bool ACCUM>
__global__ __launch_bounds__(kGemvThreads) void gemv_x16_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, int K, int N,
    float* __restrict__ out) {
  extern __shared__ float smem[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int npairs = (N + 1) >> 1;
  const int p0 = blockIdx.x * kGemvWaves + wave;
  auto map = [&](int p, const uint16_t*& wa, const uint16_t*& wb) {
    wa = w + (size_t)(2 * p) * K;
    wb = w + (size_t)min(2 * p + 1, N - 1) * K;
  };
  Regs<PFC> pre;
  Plain16Pre<NX> xp;
  const uint16_t *wa0, *wb0;
  map(p0 < npairs ? p0 : npairs - 1, wa0, wb0);
  if constexpr (NX > 0) xp.load(x, K);
  __builtin_amdgcn_sched_barrier(0);  // x loads strictly before the weights (in-order vmcnt)
  if (NX > 0 || (PFC > 0 && p0 < npairs)) prefetch_rows<PFC>(wa0, wb0, pre);  // NX: exact vmcnt
  // ACCUM: the residual words of the wave's first pair, requested now (read in
  // the epilogue they were one more memory round trip at the end of every wave;
  // no other wave of this launch writes them)
  float r0a = 0.f, r0b = 0.f;
  if constexpr (ACCUM) {
    const int pc = p0 < npairs ? p0 : npairs - 1;
    r0a = out[2 * pc];
    r0b = out[min(2 * pc + 1, N - 1)];
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (NX > 0) xp.finish(K, xs);
  else stage_plain16(x, K, xs);
  auto epi = [&](int p, float da, float db) {
    if (lane != 0) return;
    const int ra = 2 * p, rb = 2 * p + 1;
    if (ACCUM) out[ra] = da + (p == p0 ? r0a : out[ra]); else out[ra] = da;
    if (rb < N) { if (ACCUM) out[rb] = db + (p == p0 ? r0b : out[rb]); else out[rb] = db; }
  };
  run_pairs<DT, false, U, PFC>(map, epi, xs, K, npairs, p0, gridDim.x * kGemvWaves, pre);
}

// Greedy token selection fused into the lm_head (SEL): repeat penalty on the logits of
// the last `last_n` history tokens, argmax (ties -> smallest index), and the step
// finalizer (tok, history, pos) — what repeat_penalty_kernel + argmax_kernel +
// finalize_kernel (sampling.hip) do in three more launches after the lm_head.
struct HeadSel {
  const int* hist;         // token history [max_hist]
  const int* hist_len;     // device scalar
  int last_n;              // <= 256 (4 window tokens per lane)
  float penalty;           // 1 = none
  unsigned long long* slot;  // best key (ordered(logit) << 32 | ~index), 0 between launches
  unsigned int* ticket;      // finished workgroups, 0 between launches
  int* tok;                // next input token
  int* hist_w;             // history (written by the last workgroup)
  int* hist_len_w;
  int* pos;
  int max_hist;
  const uint16_t* embed;   // optional: the next step's input, resid = embed[tok] (f32)
  float* emb_out;
  int H;
};

__device__ __forceinline__ unsigned int ordered_key(float f) {
  const unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// RMSNorm(f32 row) then f32 output: the lm_head (SEL: + greedy selection, see HeadSel).
template <int DT, int U, int PFC, int NX, bool SEL>
__global__ __launch_bounds__(kGemvThreads) void gemv_norm_f32_kernel(
    const float* __restrict__ resid, const uint16_t* __restrict__ norm_w, float eps,
    const uint16_t* __restrict__ w, int K, int N, float* __restrict__ out, HeadSel hs) {
  extern __shared__ float xs[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int npairs = (N + 1) >> 1;
  const int p0 = blockIdx.x * kGemvWaves + wave;
  auto map = [&](int p, const uint16_t*& wa, const uint16_t*& wb) {
    wa = w + (size_t)(2 * p) * K;
    wb = w + (size_t)min(2 * p + 1, N - 1) * K;
  };
  // SEL: the history length is requested ahead of the x prologue (one load in front of
  // it), the window itself after it (queued behind the first weight rows; first needed
  // by the first pair's epilogue)
  int hlen = 0;
  if constexpr (SEL) hlen = hs.penalty != 1.f ? *hs.hist_len : 0;
  Regs<PFC> pre;
  NormPre<DT, NX> xp;
  const uint16_t *wa0, *wb0;
  map(p0 < npairs ? p0 : npairs - 1, wa0, wb0);
  if constexpr (NX > 0) xp.load(resid, norm_w, K);
  __builtin_amdgcn_sched_barrier(0);  // x loads strictly before the weights (in-order vmcnt)
  if (NX > 0 || (PFC > 0 && p0 < npairs)) prefetch_rows<PFC>(wa0, wb0, pre);  // NX: exact vmcnt
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (NX > 0) xp.finish(eps, K, xs);
  else stage_rmsnorm<DT>(resid, norm_w, eps, K, xs);
  int win[4] = {-1, -1, -1, -1};
  if constexpr (SEL) {
    const int n = min(hs.last_n, hlen), start = hlen - n;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j * 64 + lane < n) win[j] = hs.hist[start + j * 64 + lane];
  }
  unsigned long long best = 0ull;
  auto epi = [&](int p, float da, float db) {
    const int ra = 2 * p, rb = 2 * p + 1;
    if constexpr (SEL) {
      // penalty: the row is one of the window's tokens (each token once, like the
      // unique-token loop of repeat_penalty_kernel)
      if (hs.penalty != 1.f) {
        const bool ia = win[0] == ra || win[1] == ra || win[2] == ra || win[3] == ra;
        const bool ib = win[0] == rb || win[1] == rb || win[2] == rb || win[3] == rb;
        if (__builtin_amdgcn_ballot_w64(ia) != 0ull) da = da >= 0.f ? da / hs.penalty : da * hs.penalty;
        if (__builtin_amdgcn_ballot_w64(ib) != 0ull) db = db >= 0.f ? db / hs.penalty : db * hs.penalty;
      }
      const unsigned long long ka =
          ((unsigned long long)ordered_key(da) << 32) | (0xffffffffu - (unsigned int)ra);
      best = ka > best ? ka : best;
      if (rb < N) {
        const unsigned long long kb =
            ((unsigned long long)ordered_key(db) << 32) | (0xffffffffu - (unsigned int)rb);
        best = kb > best ? kb : best;
      }
    }
    if (lane != 0) return;
    out[ra] = da;
    if (rb < N) out[rb] = db;
  };
  run_pairs<DT, true, U, PFC>(map, epi, xs, K, npairs, p0, gridDim.x * kGemvWaves, pre);
  if constexpr (SEL) {
    // block max -> one returning 8-byte device atomic on the slot, drained before the
    // ticket (atomics on both sides: the last workgroup reads the slot atomically)
    __shared__ unsigned long long red[kGemvWaves];
    __shared__ int is_last;
    if (lane == 0) red[wave] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long b = red[0];
#pragma unroll
      for (int i = 1; i < kGemvWaves; ++i) b = red[i] > b ? red[i] : b;
      const unsigned long long old =
          __hip_atomic_fetch_max(hs.slot, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::"v"((unsigned int)old) : "memory");
      const unsigned int t =
          __hip_atomic_fetch_add(hs.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      is_last = t == gridDim.x - 1;
    }
    __syncthreads();
    if (is_last) {  // block-uniform
      __shared__ int sel_tok;
      if (threadIdx.x == 0) {
        const unsigned long long key =
            __hip_atomic_fetch_max(hs.slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int t = (int)(0xffffffffu - (unsigned int)(key & 0xffffffffull));
        *hs.tok = t;
        const int len = *hs.hist_len_w;
        if (len < hs.max_hist) { hs.hist_w[len] = t; *hs.hist_len_w = len + 1; }
        *hs.pos += 1;
        // re-arm for the next launch (the kernel boundary orders these for it)
        __hip_atomic_store(hs.slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hs.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sel_tok = t;
      }
      if (hs.embed != nullptr) {
        // the next step's input row (what embed_kernel would launch for): every other
        // workgroup has finished reading resid (their tickets preceded this one)
        __syncthreads();
        const uint16_t* row = hs.embed + (size_t)sel_tok * hs.H;
        for (int i = threadIdx.x * 8; i < hs.H; i += kGemvThreads * 8) {
          float f[8];
          unpack8<DT>(*reinterpret_cast<const uint4*>(row + i), f);
          *reinterpret_cast<float4*>(hs.emb_out + i) = make_float4(f[0], f[1], f[2], f[3]);
          *reinterpret_cast<float4*>(hs.emb_out + i + 4) = make_float4(f[4], f[5], f[6], f[7]);
        }
      }
    }
  }
}

// Launch geometry per kernel kind (tunable at run time; defaults from the
// rocprofv3-measured sweep in profiles/): U = chunks in flight per row,
// PF = prefetch the first weight batch before the x prologue, MB = grid cap.
struct GemvTune { int U, PF, MB; };
// kX16 = 16-bit-input GEMVs with K > 8192 (down_proj), kX16S = K <= 8192 (o_proj)
enum GemvKind { kQkv = 0, kSwiglu = 1, kX16 = 2, kNormF32 = 3, kX16S = 4, kNumKinds = 5 };
// measured in the decode graph (8B, tok/s): profiles/r2_gemv_split_prologue_sweep*.jsonl —
// prefetching the first weight rows behind the split x prologue is +10% (323 -> 357); the
// round-3 re-sweep (profiles/r3_decode_gemv_tuning_ingraph.jsonl) moved QKV to U 2 / PF 4
// (+0.3 %, every round) and left the rest
// the run-time tuning table (defined in gemv.hip, set by cake_gemv_set_tuning)
extern GemvTune g_tune[kNumKinds];

static inline int grid_for(int npairs, int max_blocks) {
  int g = (npairs + kGemvWaves - 1) / kGemvWaves;
  return g < max_blocks ? g : max_blocks;
}

}  // namespace cake

using namespace cake;

#define DISPATCH_DT(dt, ...)                       \
  do {                                             \
    if ((dt) == kBF16) { constexpr int DT = kBF16; __VA_ARGS__; } \
    else if ((dt) == kF16) { constexpr int DT = kF16; __VA_ARGS__; } \
    else return (int)hipErrorInvalidValue;         \
  } while (0)

// Expand BODY for the run-time (U, PFC) choice; PFC falls back to 0 when a
// row is shorter than PFC*64 chunks (small test shapes).
#define CAKE_TUNE_U(PFCV, ...)                                                       \
  if (t.U == 2) { constexpr int U = 2; constexpr int PF = PFCV; __VA_ARGS__; }       \
  else if (t.U == 8) { constexpr int U = 8; constexpr int PF = PFCV; __VA_ARGS__; }  \
  else { constexpr int U = 4; constexpr int PF = PFCV; __VA_ARGS__; }
// NX: split x prologue (only with a weight prefetch): RMSNorm rows K <= 1024 NX,
// 16-bit rows K <= 2048 NX (guarded tails: the TP shards' K); larger K use the
// plain prologue (NX = 0).
#define CAKE_NX_NORM(K, ...)                                                         \
  if constexpr (PF > 0) {                                                            \
    if ((K) <= 4096) { constexpr int NX = 4; __VA_ARGS__; }                          \
    else if ((K) <= 8192) { constexpr int NX = 8; __VA_ARGS__; }                     \
    else { constexpr int NX = 0; __VA_ARGS__; }                                      \
  } else { constexpr int NX = 0; __VA_ARGS__; }
#define CAKE_NX_X16(K, ...)                                                          \
  if constexpr (PF > 0) {                                                            \
    if ((K) <= 2048) { constexpr int NX = 1; __VA_ARGS__; }                          \
    else if ((K) <= 4096) { constexpr int NX = 2; __VA_ARGS__; }                     \
    else if ((K) <= 8192) { constexpr int NX = 4; __VA_ARGS__; }                     \
    else if ((K) <= 14336) { constexpr int NX = 7; __VA_ARGS__; }                    \
    else if ((K) <= 28672) { constexpr int NX = 14; __VA_ARGS__; }                   \
    else { constexpr int NX = 0; __VA_ARGS__; }                                      \
  } else { constexpr int NX = 0; __VA_ARGS__; }
#define DISPATCH_TUNE(t, K, ...)                                                     \
  do {                                                                               \
    const int pfc_ = ((K) / 8 >= 64 * (t).PF) ? (t).PF : 0;                          \
    if (pfc_ == 8) { CAKE_TUNE_U(8, __VA_ARGS__) }                                   \
    else if (pfc_ == 4) { CAKE_TUNE_U(4, __VA_ARGS__) }                              \
    else { CAKE_TUNE_U(0, __VA_ARGS__) }                                             \
  } while (0)

