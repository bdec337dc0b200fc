// Persistent batch-1 decode megakernel: every transformer block of a decode
// step (and optionally ln_f + lm_head) in ONE launch.
//
// Replaces, for T = 1, the per-layer chain of the reference
//   cake-core/src/models/llama3/transformer.rs:51-73   (block forward)
//   cake-core/src/models/llama3/attention.rs:49-120    (qkv, rope, kv, attention, o_proj)
//   cake-core/src/models/llama3/mlp.rs:15-18           (SwiGLU)
//   cake-core/src/models/llama3/llama.rs:119-137       (ln_f + lm_head -> f32)
// that the multi-kernel path (gemv.hip + attention.hip) runs as 5 launches per
// layer.
//
// Why: batch-1 decode is a pure HBM weight stream (8B: 15 GB per token).  With
// one launch per projection every kernel boundary drains the chip (tail
// waves, end-of-kernel cache write-back, launch ramp, the RMSNorm prologue
// before the first weight byte is requested): ~27 us per layer measured on
// MI355X on top of ~62 us of streaming (profiles/r1_v2_decode8b_kernels.txt).
//
// Design (MI355X-first):
//   * Grid = one workgroup per CU, all co-resident (the dynamic LDS request is
//     > 80 KB so two never share a CU).  A workgroup is 8 COMPUTE waves + 1
//     CONTROL wave.
//   * Compute waves only ever issue weight loads.  Each owns a fixed stream of
//     "batches" (2 weight rows x 4 16-byte chunks per lane = 8 KB) across all
//     phases and layers, triple-buffered in registers with a uniform load count
//     per batch, so the compiler's in-order vmcnt bookkeeping keeps two batches
//     in flight while one is consumed — including across phase boundaries:
//     weights never depend on activations, so the first batches of the next
//     projection are already in flight while the workgroup waits at a barrier.
//     Dot products go to LDS, never to global memory.
//   * gfx9 has ONE in-order vmcnt for loads and stores, so any store or
//     activation load issued by a streaming wave would queue behind its 16 KB
//     of in-flight weights.  The control wave therefore does everything else:
//     epilogue stores, the grid barrier (one agent-scope counter, bounded by a
//     wall-clock deadline), staging of the next x into LDS (RMSNorm included),
//     and the GQA attention of (kv head, 64-key split) units with an
//     agent-scope ticket combine — all while the compute waves' prefetches
//     keep HBM busy.
//   * Cross-workgroup data is written with agent-scope (sc1) stores and read
//     with sc1 loads, stores drained (vmcnt(0)) before the barrier arrival;
//     nothing needs an L2 write-back or invalidate inside the launch.
//   * No read-modify-write of the residual: o_proj / down write their outputs
//     (YO / YD) and the next staging computes resid + y in f32 (exactly the
//     multi-kernel path's `resid += y`), each workgroup writing its slice of the
//     updated residual into a ping-pong buffer.
//   * Compile-time wave roles, register-resident buffers, no scratch.
#include "common.h"

namespace cake {
namespace mega {

constexpr int NW = 8;             // compute waves per workgroup
constexpr int NT = (NW + 1) * 64; // + control wave
constexpr int KB = 4;             // 16-byte chunks per lane per row per batch
constexpr int BATCH_ELEMS = KB * 64 * 8;  // elements of one row per batch (2048)
constexpr int KEYS = 64;          // keys per attention unit (one per lane)
constexpr int kMaxLayers = 128;   // layer-table capacity (LDS)

enum Phase : int { kQKV = 0, kATT = 1, kO = 2, kSWI = 3, kDOWN = 4, kHEAD = 5, kFIN = 6 };

struct Layer {
  const uint16_t *ln1, *wqkv, *wo, *ln2, *wg, *wu, *wd;
  uint16_t *kc, *vc;  // this layer's cache [nkv][S][hd]
};

struct Args {
  const Layer* layers;
  int L;
  int H, I, nh, nkv, hd, S, KS;
  float eps, scale;
  const float* inv_freq;
  const int* pos;
  float* resid;         // [H] f32: input (embedding row); output (no head: after the last layer)
  uint64_t* yo_t;       // [H] tagged f32: o_proj output
  uint64_t* yd_t;       // [H] tagged f32: down_proj output
  uint64_t* qkv_t;      // [KS][nq + 2*nk] tagged f32: q/k/v (K-split) partial dot products
  uint32_t* attn_t;     // [nh*hd] tagged 16-bit: attention output
  uint32_t* act_t;      // [I] tagged 16-bit: SwiGLU activation
  float* attn_part;     // [nh][ceil(S/64)][hd + 2] f32 split partials
  unsigned* tickets;    // [nkv], zero at rest (the last split re-arms)
  unsigned* launch_ctr; // launch id: tags of this launch; workgroup 0 increments it at the end
  int* err;             // 1 = a dependency wait timed out
  const uint16_t* norm_f;  // optional head (nullptr: final residual written instead)
  const uint16_t* lm_head;
  int V;
  float* logits;
  long long* trace;     // optional [NP][grid][8] timestamps (debug)
  int xcap;             // floats of the x / attention LDS region
  int kmax;             // max units of one compute wave in one phase (LDS result slots)
  long long timeout;    // dependency-wait deadline, s_memrealtime ticks (100 MHz)
};

// ----------------------------------------------------------------------------
// coherent (agent-scope, sc1) accesses for data exchanged inside the launch
// ----------------------------------------------------------------------------
// Buffer resources bound the access: a load past num_records returns 0
// instead of faulting, so the control wave's staging loads can be issued
// unconditionally (no per-load branches -> the compiler keeps them all in flight).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes = 0x7fffffff) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
// 16 bytes at byte offset `off`, sc1 (cache-policy aux bit 4)
__device__ __forceinline__ uint4 ld_sc1_16(__amdgpu_buffer_rsrc_t r, int off) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld_8(__amdgpu_buffer_rsrc_t r, int off) {
  typedef unsigned int v2u __attribute__((ext_vector_type(2)));
  const v2u v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ float ld_sc1_f32b(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}
__device__ __forceinline__ float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, int off) {
  const uint4 u = ld_sc1_16(r, off);
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                     __uint_as_float(u.w));
}
__device__ __forceinline__ float ld_sc1_f32(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f32(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u16(uint16_t* p, uint16_t v) {
  __hip_atomic_store(reinterpret_cast<unsigned short*>(p), (unsigned short)v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void cfence() { asm volatile("" ::: "memory"); }
// Workgroup rendezvous WITHOUT a memory fence: a compute wave's in-flight
// weight loads must not be drained here.  LDS traffic is ordered explicitly.
__device__ __forceinline__ void wg_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  cfence();
}

// ----------------------------------------------------------------------------
// phases
// ----------------------------------------------------------------------------
struct Geo {
  int nq, nk, R, NP;  // NP = 5*L + 1 phases (the last is HEAD or FIN)
  int gw, nwv;        // global compute-wave index / count
  bool head;
  const Layer* lt;    // the layer table, copied into LDS (a VMEM read of it
                      // would have to wait behind the in-flight weights)
};

__device__ __forceinline__ int ph_kind(const Args& a, const Geo& g, int p) {
  if (p < 5 * a.L) return p % 5;
  return g.head ? kHEAD : kFIN;
}

__device__ __forceinline__ int ph_units(const Args& a, const Geo& g, int kind) {
  switch (kind) {
    case kQKV: return (g.R >> 1) * a.KS;
    case kO: return a.H >> 1;
    case kSWI: return a.I;
    case kDOWN: return a.H >> 1;
    case kHEAD: return a.V >> 1;
  }
  return 0;
}

// batches per unit
__device__ __forceinline__ int ph_nb(const Args& a, const Geo& g, int kind) {
  switch (kind) {
    case kQKV: return a.H / a.KS / BATCH_ELEMS;
    case kO: return g.nq / BATCH_ELEMS;
    case kSWI: return a.H / BATCH_ELEMS;
    case kDOWN: return a.I / BATCH_ELEMS;
    case kHEAD: return a.H / BATCH_ELEMS;
  }
  return 0;
}

// ----------------------------------------------------------------------------
// compute-wave batch stream
// ----------------------------------------------------------------------------
// Weight batches are loaded with inline-asm global loads that the compiler
// does not track: the compute wave's vmcnt queue then holds ONLY these loads,
// in issue order, and `wait_buf` waits for exactly one buffer while the other
// two stay in flight (the compiler's own waitcnt insertion is conservative
// across this loop's phase-transition control flow and would drain all three).
struct Buf {
  u32x4 a[KB], b[KB];
};

__device__ __forceinline__ u32x4 asm_ld_nt(const void* p) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
  return r;
}

// all loads issued after B's: the other two buffers
constexpr int kVmInFlight = 2 * 2 * KB;
__device__ __forceinline__ void wait_buf(Buf& B) {
  static_assert(KB == 4, "wait_buf lists the buffer registers explicitly");
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(B.a[0]), "+v"(B.a[1]), "+v"(B.a[2]), "+v"(B.a[3]), "+v"(B.b[0]),
                 "+v"(B.b[1]), "+v"(B.b[2]), "+v"(B.b[3])
               : "n"(kVmInFlight));
}

__device__ __forceinline__ void unpack8v(const u32x4 v, float* o, bool bf16) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (bf16) {
      o[2 * i] = __uint_as_float(w[i] << 16);
      o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    } else {
      o[2 * i] = f16_to_f32((uint16_t)(w[i] & 0xffffu));
      o[2 * i + 1] = f16_to_f32((uint16_t)(w[i] >> 16));
    }
  }
}

struct Cur {
  int p, u, bi, k;  // phase, unit, batch within unit, unit ordinal within the phase
};

// move to the first valid batch at or after (p, u) — skipping phases where
// this wave has no unit; p == NP is the end of the stream
__device__ __forceinline__ void seek(const Args& a, const Geo& g, Cur& c) {
  while (c.p < g.NP) {
    const int kind = ph_kind(a, g, c.p);
    if (kind != kATT && kind != kFIN && c.u < ph_units(a, g, kind)) return;
    ++c.p;
    c.u = g.gw;
    c.bi = 0;
    c.k = 0;
  }
}

__device__ __forceinline__ void advance(const Args& a, const Geo& g, Cur& c) {
  if (c.p >= g.NP) return;
  if (++c.bi < ph_nb(a, g, ph_kind(a, g, c.p))) return;
  c.bi = 0;
  c.u += g.nwv;
  ++c.k;
  seek(a, g, c);
}

// chunk pointers of this lane for the batch at c (a dummy, valid batch at the
// end of the stream keeps the per-batch load count uniform)
__device__ __forceinline__ void rows_of(const Args& a, const Geo& g, const Cur& c, int lane,
                                        const uint4*& ra, const uint4*& rb) {
  const uint16_t *pa, *pb;
  const int H = a.H;
  const int kind = c.p < g.NP ? ph_kind(a, g, c.p) : -1;
  const int off = c.bi * (KB * 64) + lane;
  if (kind == kHEAD) {
    pa = a.lm_head + (size_t)(2 * c.u) * H;
    pb = pa + H;
  } else if (kind < 0) {
    pa = g.lt[0].wqkv;
    pb = pa;
    ra = reinterpret_cast<const uint4*>(pa) + lane;
    rb = ra;
    return;
  } else {
    const Layer& Ly = g.lt[c.p / 5];
    switch (kind) {
      case kQKV: {
        const int pr = a.KS == 2 ? (c.u >> 1) : c.u;
        const int kh = a.KS == 2 ? (c.u & 1) : 0;
        pa = Ly.wqkv + (size_t)(2 * pr) * H + kh * (H / 2);
        pb = pa + H;
        break;
      }
      case kO:
        pa = Ly.wo + (size_t)(2 * c.u) * g.nq;
        pb = pa + g.nq;
        break;
      case kSWI:
        pa = Ly.wg + (size_t)c.u * H;
        pb = Ly.wu + (size_t)c.u * H;
        break;
      default:  // kDOWN
        pa = Ly.wd + (size_t)(2 * c.u) * a.I;
        pb = pa + a.I;
        break;
    }
  }
  ra = reinterpret_cast<const uint4*>(pa) + off;
  rb = reinterpret_cast<const uint4*>(pb) + off;
}

__device__ __forceinline__ void issue(const Args& a, const Geo& g, const Cur& c, int lane,
                                      Buf& B) {
  const uint4 *ra, *rb;
  rows_of(a, g, c, lane, ra, rb);
#pragma unroll
  for (int i = 0; i < KB; ++i) B.a[i] = asm_ld_nt(ra + i * 64);
#pragma unroll
  for (int i = 0; i < KB; ++i) B.b[i] = asm_ld_nt(rb + i * 64);
}

template <int DT, bool XF32>
__device__ __forceinline__ void consume(Buf& B, const void* xs, int ci0, float& sa, float& sb) {
  wait_buf(B);
#pragma unroll
  for (int i = 0; i < KB; ++i) {
    float xv[8], fa[8], fb[8];
    const int ci = ci0 + i * 64;
    if constexpr (XF32) {
      const float4* p = reinterpret_cast<const float4*>(xs) + ci * 2;
      const float4 u = p[0], v = p[1];
      xv[0] = u.x; xv[1] = u.y; xv[2] = u.z; xv[3] = u.w;
      xv[4] = v.x; xv[5] = v.y; xv[6] = v.z; xv[7] = v.w;
    } else {
      unpack8<DT>(reinterpret_cast<const uint4*>(xs)[ci], xv);
    }
    unpack8v(B.a[i], fa, DT == kBF16);
    unpack8v(B.b[i], fb, DT == kBF16);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sa = fmaf(fa[e], xv[e], sa);
      sb = fmaf(fb[e], xv[e], sb);
    }
  }
}

// ----------------------------------------------------------------------------
// control wave: tagged data (no grid barrier)
// ----------------------------------------------------------------------------
// Every value exchanged between workgroups is stored together with a tag of
// (launch, phase) in ONE atomic 64-bit (f32) or 32-bit (16-bit value) sc1
// store; a consumer polls exactly the data it needs until every tag matches.
// One memory round trip per phase boundary instead of store-drain + atomic
// arrive + poll + reload.  Each phase consumes ALL outputs of the previous
// one, so a buffer is never rewritten before every consumer has read it.
__device__ __forceinline__ uint32_t tag32(unsigned launch, int p) {
  return (launch * 512u + (unsigned)p) | 0x80000000u;
}
__device__ __forceinline__ uint32_t tag16(unsigned launch, int p) {
  return ((launch * 512u + (unsigned)p) & 0x7fffu) | 0x8000u;
}
__device__ __forceinline__ void st_tag64(uint64_t* p, float v, uint32_t tag) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_tag32(uint32_t* p, uint16_t v, uint32_t t16) {
  __hip_atomic_store(p, (t16 << 16) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// deadline bookkeeping of one wait; returns false once it has expired (err set)
__device__ __forceinline__ bool still_waiting(const Args& a, long long t0) {
  __builtin_amdgcn_s_sleep(1);
  if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout ||
      __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
    if ((threadIdx.x & 63) == 0)
      __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return true;
}

constexpr int SU = 8;  // float4 groups per lane per staging batch (2 tagged-f32 16-byte loads each)

// x = r (+ y), r <- x (the workgroup's LDS copy of the residual stream),
// xs = RMSNorm(x) * w.  y: tagged f32 [H] of phase tag `t` (nullptr: none).
template <int DT>
__device__ __forceinline__ bool stage_norm(const Args& a, float* r, const uint64_t* y, uint32_t t,
                                           const uint16_t* w, float* xs, float* ws) {
  const int lane = threadIdx.x & 63;
  const int K = a.H;  // multiple of 64 * 4 * 8; batches past K read 0 (bounded resources)
  const auto ry = rsrc(y ? (const void*)y : (const void*)a.resid, y ? K * 8 : 0);
  const auto rw = rsrc(w, K * 2);
  float ss = 0.f;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int base = 0; base < K; base += 64 * 4 * SU) {
    uint2 wv[SU];
#pragma unroll
    for (int j = 0; j < SU; ++j) wv[j] = ld_8(rw, (base + (j * 64 + lane) * 4) * 2);
    uint4 yv[2 * SU];
    for (;;) {
#pragma unroll
      for (int j = 0; j < SU; ++j) {
        const int i = base + (j * 64 + lane) * 4;
        yv[2 * j] = ld_sc1_16(ry, i * 8);
        yv[2 * j + 1] = ld_sc1_16(ry, i * 8 + 16);
      }
      bool ok = true;
      if (y) {
#pragma unroll
        for (int j = 0; j < SU; ++j) {
          const bool in = base + (j * 64 + lane) * 4 < K;
          ok = ok && (!in || (yv[2 * j].y == t && yv[2 * j].w == t && yv[2 * j + 1].y == t &&
                              yv[2 * j + 1].w == t));
        }
      }
      if (__all(ok)) break;
      if (!still_waiting(a, t0)) return false;
    }
#pragma unroll
    for (int j = 0; j < SU; ++j) {
      const int i = base + (j * 64 + lane) * 4;
      if (i >= K) continue;
      float4 x = *reinterpret_cast<float4*>(r + i);
      if (y) {
        x.x += __uint_as_float(yv[2 * j].x);
        x.y += __uint_as_float(yv[2 * j].z);
        x.z += __uint_as_float(yv[2 * j + 1].x);
        x.w += __uint_as_float(yv[2 * j + 1].z);
        *reinterpret_cast<float4*>(r + i) = x;
      }
      *reinterpret_cast<float4*>(xs + i) = x;
      *reinterpret_cast<float4*>(ws + i) =
          make_float4(to_f32<DT>((uint16_t)(wv[j].x & 0xffff)), to_f32<DT>((uint16_t)(wv[j].x >> 16)),
                      to_f32<DT>((uint16_t)(wv[j].y & 0xffff)), to_f32<DT>((uint16_t)(wv[j].y >> 16)));
      ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    }
  }
  ss = wave_sum(ss);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const float rn = rsqrtf(ss / (float)K + a.eps);
  // xs = x * (rn * w): the multi-kernel path's rounding
#pragma unroll 4
  for (int i = lane * 4; i < K; i += 64 * 4) {
    float4 v = *reinterpret_cast<float4*>(xs + i);
    const float4 wf = *reinterpret_cast<const float4*>(ws + i);
    v.x *= rn * wf.x;
    v.y *= rn * wf.y;
    v.z *= rn * wf.z;
    v.w *= rn * wf.w;
    *reinterpret_cast<float4*>(xs + i) = v;
  }
  return true;
}

// xs[0..K) = tagged 16-bit src of tag t (K multiple of 4)
__device__ __forceinline__ bool stage16(const Args& a, const uint32_t* src, int K, uint32_t t,
                                        uint16_t* xs) {
  const int lane = threadIdx.x & 63;
  const auto r = rsrc(src, K * 4);
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int base = 0; base < K; base += 64 * 4 * 2 * SU) {
    uint4 v[2 * SU];
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < 2 * SU; ++j) v[j] = ld_sc1_16(r, (base + (j * 64 + lane) * 4) * 4);
#pragma unroll
      for (int j = 0; j < 2 * SU; ++j) {
        const bool in = base + (j * 64 + lane) * 4 < K;
        ok = ok && (!in || ((v[j].x >> 16) == t && (v[j].y >> 16) == t &&
                            (v[j].z >> 16) == t && (v[j].w >> 16) == t));
      }
      if (__all(ok)) break;
      if (!still_waiting(a, t0)) return false;
    }
#pragma unroll
    for (int j = 0; j < 2 * SU; ++j) {
      const int i = base + (j * 64 + lane) * 4;
      if (i < K)
        *reinterpret_cast<uint2*>(xs + i) =
            make_uint2((v[j].x & 0xffffu) | (v[j].y << 16), (v[j].z & 0xffffu) | (v[j].w << 16));
    }
  }
  return true;
}

// ----------------------------------------------------------------------------
// control wave: attention unit (kv head g, keys [64 s, 64 s + 64) of pos+1)
// ----------------------------------------------------------------------------
// K and V tiles of keys [64 s, 64 s + 64) of kv head g into LDS with
// global_load_lds_dwordx4 (1 KiB per instruction, lane-linear).  Issued during
// the QKV phase for the workgroup's first attention unit of the layer (the
// cache rows < pos do not depend on this token), so the tile has landed when
// the attention phase starts.  K: instruction c, lane L fetches (row (L - c)
// & 63, chunk c) so that lane r later reads its chunk c from slot
// c*64 + ((r + c) & 63) without bank conflicts.  Rows past the context re-read
// row 0 of the tile (finite values, weighted by p = 0).
template <int HD>
__device__ __forceinline__ void attn_tiles(const Args& a, const Layer& Ly, int g, int s, int Tk,
                                           uint4* kt, uint16_t* vt) {
  constexpr int CPR = HD / 8;
  typedef const __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  const int lane = threadIdx.x & 63;
  const int k0 = s * KEYS;
  const int kn_cnt = min(KEYS, Tk - k0);
  const uint4* kg = reinterpret_cast<const uint4*>(Ly.kc + ((size_t)g * a.S + k0) * HD);
  const uint4* vg = reinterpret_cast<const uint4*>(Ly.vc + ((size_t)g * a.S + k0) * HD);
#pragma unroll
  for (int c = 0; c < CPR; ++c) {
    const int r = (lane - c) & 63;
    const uint4* src = kg + (r < kn_cnt ? r : 0) * CPR + c;
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(kt + c * 64), 16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < CPR; ++j) {
    const int i = j * 64 + lane;  // chunk index within the tile
    const uint4* src = (i / CPR < kn_cnt) ? vg + i : vg + (i % CPR);
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(vt + j * 512), 16, 0, 0);
  }
}

// One attention unit = query head hq (of kv group g = hq / NREP), keys
// [64 s, 64 s + 64) of Tk = pos + 1, on the control wave.  have_tiles: the
// K/V tiles were prefetched into kt / vt during the QKV phase.
template <int DT, int HD, int NREP>
__device__ __forceinline__ bool attn_unit(const Args& a, const Geo& geo, const Layer& Ly, int hq,
                                          int s, int ns, int pos, float* lds, uint4* kt,
                                          uint16_t* vt, bool have_tiles, const float* rope_cs,
                                          const float* rope_sn, uint32_t tq, uint32_t to16,
                                          long long* trp) {
#define CAKE_TR(i) if (trp != nullptr && lane == 0) trp[i] = (long long)__builtin_amdgcn_s_memrealtime()
  constexpr int DPL = HD / 64;
  constexpr int HALF = HD / 2;
  constexpr int CPR = HD / 8;
  const int lane = threadIdx.x & 63;
  const int g = hq / NREP;
  const int Tk = pos + 1;
  float* qs = lds;         // [HD] roped q (f32)
  float* kn = qs + HD;     // [HD] new key (16-bit rounded)
  float* vn = kn + HD;     // [HD] new value
  float* ps = vn + HD;     // [64] probabilities / merge weights
  const int k0 = s * KEYS;
  const int kn_cnt = min(KEYS, Tk - k0);
  const int kk = k0 + lane;
  if (!have_tiles) attn_tiles<HD>(a, Ly, g, s, Tk, kt, vt);

  // 1. sum the K-split partials of q (head hq), k, v (group g), polled until
  //    every tag is this launch's QKV phase (the second half's resource is
  //    empty when KS == 1); RoPE from the launch's cos/sin table
  {
    constexpr int N2 = 3 * HD / 2;  // 16-byte loads = 2 tagged values
    constexpr int NJ = (N2 + 63) / 64;
    const auto r0 = rsrc(a.qkv_t, geo.R * 8);
    const auto r1 = rsrc(a.qkv_t + geo.R, a.KS == 2 ? geo.R * 8 : 0);
    uint4 v0[NJ], v1[NJ];
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int i = (j * 64 + lane) * 2, slot = i / HD, d = i - slot * HD;
        int row;
        if (slot == 0) row = hq * HD + d;
        else if (slot == 1) row = geo.nq + g * HD + d;
        else row = geo.nq + geo.nk + g * HD + d;
        const bool in = i < 3 * HD;
        if (!in) row = geo.R;  // past the end: reads 0
        v0[j] = ld_sc1_16(r0, row * 8);
        v1[j] = ld_sc1_16(r1, row * 8);
        ok = ok && (!in || (v0[j].y == tq && v0[j].w == tq &&
                            (a.KS == 1 || (v1[j].y == tq && v1[j].w == tq))));
      }
      if (__all(ok)) break;
      if (!still_waiting(a, t0)) return false;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = (j * 64 + lane) * 2;
      if (i < 3 * HD)  // qs, kn, vn are contiguous
        *reinterpret_cast<float2*>(qs + i) =
            make_float2(__uint_as_float(v0[j].x) + __uint_as_float(v1[j].x),
                        __uint_as_float(v0[j].z) + __uint_as_float(v1[j].z));
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  for (int i = lane; i < 3 * HALF; i += 64) {
    const int slot = i / HALF, d = i - slot * HALF;
    float* base = qs + slot * HD;
    const float da = base[d], db = base[d + HALF];
    float oa = da, ob = db;
    if (slot <= 1) {  // q and k are rotated, v is not
      const float sn = rope_sn[d], cs = rope_cs[d];
      oa = da * cs - db * sn;
      ob = da * sn + db * cs;
    }
    if (slot >= 1) {  // k, v are stored 16-bit: attend to the rounded value
      const uint16_t ha = from_f32<DT>(oa), hb = from_f32<DT>(ob);
      oa = to_f32<DT>(ha);
      ob = to_f32<DT>(hb);
      if (s == ns - 1 && hq % NREP == 0) {  // one unit per group appends the row
        uint16_t* cache = (slot == 1 ? Ly.kc : Ly.vc) + ((size_t)g * a.S + pos) * HD;
        cache[d] = ha;
        cache[d + HALF] = hb;
      }
    }
    base[d] = oa;
    base[d + HALF] = ob;
  }
  CAKE_TR(4);
  // K / V tiles landed (row pos, if in this split, comes from kn / vn)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (pos >= k0 && pos < k0 + kn_cnt) {
    for (int d = lane; d < HD; d += 64) vt[(pos - k0) * HD + d] = from_f32<DT>(vn[d]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // 2. scores: lane <-> key kk
  float sc = -INFINITY;
  if (lane < kn_cnt) {
    float acc = 0.f;
    const bool fresh = (kk == pos);
#pragma unroll 4
    for (int c = 0; c < CPR; ++c) {
      float kf[8];
      if (!fresh) {
        unpack8<DT>(kt[c * 64 + ((lane + c) & 63)], kf);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) kf[e] = kn[c * 8 + e];
      }
      const float4 q0 = *reinterpret_cast<const float4*>(qs + c * 8);
      const float4 q1 = *reinterpret_cast<const float4*>(qs + c * 8 + 4);
      acc = fmaf(q0.x, kf[0], acc); acc = fmaf(q0.y, kf[1], acc);
      acc = fmaf(q0.z, kf[2], acc); acc = fmaf(q0.w, kf[3], acc);
      acc = fmaf(q1.x, kf[4], acc); acc = fmaf(q1.y, kf[5], acc);
      acc = fmaf(q1.z, kf[6], acc); acc = fmaf(q1.w, kf[7], acc);
    }
    sc = acc * a.scale;
  }
  const float m = wave_max(sc);
  const float pl = lane < kn_cnt ? __expf(sc - m) : 0.f;
  const float l = wave_sum(pl);
  ps[lane] = pl;  // zero past the context
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  CAKE_TR(5);

  // 3. P.V from the LDS tile, 8 keys per step; lane owns dims lane*DPL ..
  float o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  const int kn8 = (kn_cnt + 7) & ~7;
  for (int j = 0; j < kn8; j += 8) {
    const float4 pa = *reinterpret_cast<const float4*>(ps + j);
    const float4 pb = *reinterpret_cast<const float4*>(ps + j + 4);
    const float pj[8] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (DPL == 2) {
        const uint32_t w2 = *reinterpret_cast<const uint32_t*>(vt + (j + u) * HD + lane * 2);
        o[0] = fmaf(pj[u], to_f32<DT>((uint16_t)(w2 & 0xffff)), o[0]);
        o[1] = fmaf(pj[u], to_f32<DT>((uint16_t)(w2 >> 16)), o[1]);
      } else {
#pragma unroll
        for (int d = 0; d < DPL; ++d)
          o[d] = fmaf(pj[u], to_f32<DT>(vt[(j + u) * HD + lane * DPL + d]), o[d]);
      }
    }
  }
  CAKE_TR(6);

  uint32_t* outp = a.attn_t + (size_t)hq * HD + lane * DPL;
  if (ns == 1) {  // whole context in this unit
    const float inv = 1.f / l;
#pragma unroll
    for (int d = 0; d < DPL; ++d) st_tag32(outp + d, from_f32<DT>(o[d] * inv), to16);
    return true;
  }
  const int nsplit = (a.S + KEYS - 1) / KEYS;
  {
    float* dst = a.attn_part + ((size_t)hq * nsplit + s) * (HD + 2);
    if (lane == 0) { st_sc1_f32(dst, m); st_sc1_f32(dst + 1, l); }
#pragma unroll
    for (int d = 0; d < DPL; ++d) st_sc1_f32(dst + 2 + lane * DPL + d, o[d]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned last = 0;
  if (lane == 0) {
    const unsigned t =
        __hip_atomic_fetch_add(a.tickets + hq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == (unsigned)(ns - 1)) ? 1u : 0u;
    if (last) __hip_atomic_store(a.tickets + hq, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  last = __shfl(last, 0, 64);
  CAKE_TR(7);
  if (!last) return true;
  // the last split merges all ns (<= 64: one per lane) partials of head hq;
  // every load is unconditional (rows past ns read 0 from the bounded resource)
  constexpr int MU = 8;
  const int hstride = nsplit * (HD + 2);
  const auto rp = rsrc(a.attn_part + (size_t)hq * hstride, hstride * 4);
  const int rowl = lane < ns ? lane : nsplit;  // nsplit: past this head's rows
  const float mt0 = ld_sc1_f32b(rp, (rowl * (HD + 2)) * 4);
  const float lt = ld_sc1_f32b(rp, (rowl * (HD + 2) + 1) * 4);
  const float mt = lane < ns ? mt0 : -INFINITY;
  const float M = wave_max(mt);
  const float wt = lane < ns ? __expf(mt - M) : 0.f;
  const float Ls = wave_sum(wt * lt);
  ps[lane] = wt;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float acc[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) acc[d] = 0.f;
  for (int t0 = 0; t0 < ns; t0 += MU) {
    float ov[MU][DPL];
#pragma unroll
    for (int u = 0; u < MU; ++u)
#pragma unroll
      for (int d = 0; d < DPL; ++d)
        ov[u][d] = ld_sc1_f32b(rp, ((t0 + u) * (HD + 2) + 2 + lane * DPL + d) * 4);
#pragma unroll
    for (int u = 0; u < MU; ++u) {
      const float w = ps[(t0 + u) & 63];
      const float wv = (t0 + u < ns) ? w : 0.f;
#pragma unroll
      for (int d = 0; d < DPL; ++d) acc[d] = fmaf(wv, ov[u][d], acc[d]);
    }
  }
  const float inv = 1.f / Ls;
#pragma unroll
  for (int d = 0; d < DPL; ++d) st_tag32(outp + d, from_f32<DT>(acc[d] * inv), to16);
  return true;
#undef CAKE_TR
}

// ----------------------------------------------------------------------------
// control wave: store this workgroup's results of GEMV phase p
// ----------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ void store_results(const Args& a, const Geo& g, int kind,
                                              const float* res, uint32_t t, uint32_t t16) {
  const int lane = threadIdx.x & 63;
  const int nunits = ph_units(a, g, kind);
  // res[w][k][2]: unit u = (blockIdx*NW + w) + k*nwv
  for (int i = lane; i < NW * a.kmax; i += 64) {
    const int w = i / a.kmax, k = i - w * a.kmax;
    const int u = blockIdx.x * NW + w + k * g.nwv;
    if (u >= nunits) continue;
    const float da = res[2 * i], db = res[2 * i + 1];
    switch (kind) {
      case kQKV: {
        const int pr = a.KS == 2 ? (u >> 1) : u;
        const int kh = a.KS == 2 ? (u & 1) : 0;
        st_tag64(a.qkv_t + (size_t)kh * g.R + 2 * pr, da, t);
        st_tag64(a.qkv_t + (size_t)kh * g.R + 2 * pr + 1, db, t);
        break;
      }
      case kO:
        st_tag64(a.yo_t + 2 * u, da, t);
        st_tag64(a.yo_t + 2 * u + 1, db, t);
        break;
      case kDOWN:
        st_tag64(a.yd_t + 2 * u, da, t);
        st_tag64(a.yd_t + 2 * u + 1, db, t);
        break;
      case kSWI:
        st_tag32(a.act_t + u, from_f32<DT>(silu(da) * db), t16);
        break;
      default:  // kHEAD (consumed by the next kernel)
        a.logits[2 * u] = da;
        a.logits[2 * u + 1] = db;
        break;
    }
  }
}

// ----------------------------------------------------------------------------
// the kernel
// ----------------------------------------------------------------------------
template <int DT, int HD, int NREP>
__global__ __launch_bounds__(NT) void decode_mega_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ int abort_flag;
  __shared__ Layer ltab[kMaxLayers];
  __shared__ float rope_cs[64], rope_sn[64];  // cos / sin(pos * inv_freq) of this launch
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  Geo g;
  g.nq = a.nh * HD;
  g.nk = a.nkv * HD;
  g.R = g.nq + 2 * g.nk;
  g.NP = 5 * a.L + 1;
  g.nwv = gridDim.x * NW;
  g.head = a.lm_head != nullptr;
  for (int i = threadIdx.x; i < a.L * (int)(sizeof(Layer) / 8); i += NT)
    reinterpret_cast<uint64_t*>(ltab)[i] = reinterpret_cast<const uint64_t*>(a.layers)[i];
  __syncthreads();
  g.lt = ltab;
  float* res = lds;                                // [NW][kmax][2] dot products
  float* xs = lds + ((NW * a.kmax * 2 + 3) & ~3);  // x staging / attention scratch (16 B aligned)
  float* ws = xs + a.xcap;                         // norm weights (f32) while staging
  float* rl = ws + a.H;                            // the workgroup's residual stream (f32)
  uint4* kt = reinterpret_cast<uint4*>(rl + a.H);  // attention K tile (swizzled) [64 * HD * 2 B]
  uint16_t* vt = reinterpret_cast<uint16_t*>(kt) + 64 * HD;  // attention V tile [64][HD]

  if (wave == NW) {
    // ============================ control wave ============================
    const int pos = *a.pos;
    const unsigned launch = *a.launch_ctr;
    if (lane == 0) abort_flag = 0;
    if (lane < HD / 2) {  // same expression as the multi-kernel path's qkv epilogue
      float sn, cs;
      sincosf((float)pos * a.inv_freq[lane], &sn, &cs);
      rope_cs[lane] = cs;
      rope_sn[lane] = sn;
    }
    // the workgroup's copy of the residual stream: embedding row in
    for (int i = lane * 4; i < a.H; i += 256)
      *reinterpret_cast<float4*>(rl + i) = *reinterpret_cast<const float4*>(a.resid + i);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    for (int p = 0; p < g.NP; ++p) {
      const int kind = ph_kind(a, g, p);
      const int l = p / 5;
      const bool tr = a.trace != nullptr && lane == 0;
      long long* trp = tr ? a.trace + ((size_t)p * gridDim.x + blockIdx.x) * 8 : nullptr;
      if (tr) trp[0] = trp[1] = (long long)__builtin_amdgcn_s_memrealtime();
      const uint32_t tprev = tag32(launch, p - 1), tprev16 = tag16(launch, p - 1);
      bool ok = true;
      switch (kind) {  // stage phase p's input (waits for the previous phase's tags)
        case kQKV: {
          ok = stage_norm<DT>(a, rl, p > 0 ? a.yd_t : nullptr, tprev, g.lt[l].ln1, xs, ws);
          // K/V tiles of this workgroup's first attention unit of the layer
          const int ns = (pos + KEYS) / KEYS;
          if ((int)blockIdx.x < a.nh * ns) {
            const int hq = blockIdx.x / ns, s = blockIdx.x % ns;
            attn_tiles<HD>(a, g.lt[l], hq / NREP, s, pos + 1, kt, vt);
          }
          break;
        }
        case kO:
          ok = stage16(a, a.attn_t, g.nq, tprev16, reinterpret_cast<uint16_t*>(xs));
          break;
        case kSWI:
          ok = stage_norm<DT>(a, rl, a.yo_t, tprev, g.lt[l].ln2, xs, ws);
          break;
        case kDOWN:
          ok = stage16(a, a.act_t, a.I, tprev16, reinterpret_cast<uint16_t*>(xs));
          break;
        case kHEAD:
          ok = stage_norm<DT>(a, rl, a.yd_t, tprev, a.norm_f, xs, ws);
          break;
        case kFIN: {  // final residual: this workgroup's slice of rl + yd
          const int slice = (a.H + gridDim.x - 1) / gridDim.x;
          const int s0 = blockIdx.x * slice, s1 = min(a.H, s0 + slice);
          const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
          for (int i = s0 + lane; i < s1; i += 64) {
            unsigned long long e;
            for (;;) {
              e = __hip_atomic_load(reinterpret_cast<unsigned long long*>(a.yd_t + i),
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if ((uint32_t)(e >> 32) == tprev) break;
              if (!still_waiting(a, t0)) { ok = false; break; }
            }
            if (!ok) break;
            a.resid[i] = rl[i] + __uint_as_float((uint32_t)e);
          }
          ok = __all(ok);
          break;
        }
        default:
          break;
      }
      if (!ok) {
        if (lane == 0) abort_flag = 1;
        wg_barrier();  // B_p: release the compute waves, which exit
        return;
      }
      if (tr) trp[2] = (long long)__builtin_amdgcn_s_memrealtime();
      wg_barrier();  // B_p
      if (kind == kATT) {
        const int Tk = pos + 1;
        const int ns = (Tk + KEYS - 1) / KEYS;
        for (int u = blockIdx.x; u < a.nh * ns && ok; u += gridDim.x)
          ok = attn_unit<DT, HD, NREP>(a, g, g.lt[l], u / ns, u % ns, ns, pos, xs, kt, vt,
                                       u == (int)blockIdx.x, rope_cs, rope_sn, tprev,
                                       tag16(launch, p), trp);
        if (!ok) {  // the compute waves wait at A_p, then at B_{p+1}
          if (lane == 0) abort_flag = 1;
          wg_barrier();
          wg_barrier();
          return;
        }
      }
      wg_barrier();  // A_p: the compute waves' dot products of phase p are in LDS
      if (tr) trp[3] = (long long)__builtin_amdgcn_s_memrealtime();
      if (kind != kATT && kind != kFIN)
        store_results<DT>(a, g, kind, res, tag32(launch, p), tag16(launch, p));
    }
    // every workgroup has read this launch's id (all of them produced the
    // last phase's inputs): the next launch uses fresh tags
    if (blockIdx.x == 0 && lane == 0)
      __hip_atomic_fetch_add(a.launch_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ============================ compute waves ============================
  g.gw = blockIdx.x * NW + wave;
  Cur ic{0, g.gw, 0, 0};
  seek(a, g, ic);
  Cur cc = ic;
  Buf B0, B1, B2;
  issue(a, g, ic, lane, B0);
  advance(a, g, ic);
  issue(a, g, ic, lane, B1);
  advance(a, g, ic);
  issue(a, g, ic, lane, B2);
  advance(a, g, ic);
  float sa = 0.f, sb = 0.f;
  int cur = 0;  // the phase whose x is staged
  wg_barrier();  // B_0
  if (abort_flag) return;

  // one batch: bring the workgroup to cc's phase, consume B, refill B
#define CAKE_MEGA_STEP(B)                                                                  \
  {                                                                                        \
    while (cur < cc.p) {                                                                   \
      wg_barrier(); /* A_cur */                                                            \
      if (++cur < g.NP) {                                                                  \
        wg_barrier(); /* B_cur */                                                          \
        if (abort_flag) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); return; }       \
      }                                                                                    \
    }                                                                                      \
    if (cc.p >= g.NP) break;                                                               \
    {                                                                                      \
      const int kind = ph_kind(a, g, cc.p);                                                \
      int ci0 = cc.bi * (KB * 64) + lane;                                                  \
      if (kind == kQKV && a.KS == 2) ci0 += (cc.u & 1) * (a.H / 16);                       \
      if (kind == kO || kind == kDOWN) consume<DT, false>(B, xs, ci0, sa, sb);             \
      else consume<DT, true>(B, xs, ci0, sa, sb);                                          \
      if (cc.bi == ph_nb(a, g, kind) - 1) {                                                \
        const float da = wave_sum(sa), db = wave_sum(sb);                                  \
        sa = sb = 0.f;                                                                     \
        if (lane == 0) {                                                                   \
          float* r = res + 2 * (wave * a.kmax + cc.k);                                     \
          r[0] = da;                                                                       \
          r[1] = db;                                                                       \
        }                                                                                  \
      }                                                                                    \
    }                                                                                      \
    issue(a, g, ic, lane, B);                                                              \
    advance(a, g, ic);                                                                     \
    advance(a, g, cc);                                                                     \
  }

  for (;;) {
    CAKE_MEGA_STEP(B0)
    CAKE_MEGA_STEP(B1)
    CAKE_MEGA_STEP(B2)
  }
#undef CAKE_MEGA_STEP
  // the stream ended inside phase cur: finish the remaining rendezvous
  while (cur < g.NP) {
    wg_barrier();  // A_cur
    if (++cur < g.NP) {
      wg_barrier();  // B_cur
      if (abort_flag) break;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace mega
}  // namespace cake

using namespace cake;
using namespace cake::mega;

static int g_mega_cus = 0;

// result slots per compute wave per phase for a grid of `grid` workgroups
static int mega_kmax(int H, int I, int nh, int nkv, int hd, int V, int KS, int grid) {
  const long nwv = (long)grid * NW;
  const long R = (long)(nh + 2 * nkv) * hd;
  long m = 0;
  const long units[5] = {(R / 2) * KS, H / 2, I, H / 2, V / 2};
  for (long u : units) m = u > m ? u : m;
  return (int)((m + nwv - 1) / nwv);
}

static size_t mega_xcap(int H, int I, int nh, int nkv, int hd) {
  const int nrep = nh / nkv;
  size_t x = (size_t)H * 4;
  if ((size_t)I * 2 > x) x = (size_t)I * 2;
  if ((size_t)nh * hd * 2 > x) x = (size_t)nh * hd * 2;
  (void)nrep;
  const size_t att = sizeof(float) * (3 * (size_t)hd + 64);
  if (att > x) x = att;
  return ((x + 15) & ~size_t(15)) / 4;
}

static size_t mega_lds(int H, int I, int nh, int nkv, int hd, int kmax) {
  // [results NW*kmax*2 f32 | pad to 16 B] [x / attention: xcap f32] [norm weights: H f32]
  // [residual stream: H f32] [attention K and V tiles: 2 * 64 * hd * 2 B]
  size_t need = (((size_t)NW * kmax * 2 + 3) & ~size_t(3)) * 4 +
                mega_xcap(H, I, nh, nkv, hd) * 4 + (size_t)H * 8 + (size_t)4 * 64 * hd;
  // > 80 KB: at most one workgroup per CU (the grid is one workgroup per CU)
  if (need < 96 * 1024) need = 96 * 1024;
  return need;
}

CAKE_API int cake_mega_grid() {
  if (g_mega_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&g_mega_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess)
      return 0;
  }
  return g_mega_cus;
}

CAKE_API int cake_mega_supported(int H, int I, int nh, int nkv, int hd, int V) {
  if (nkv <= 0 || nh % nkv) return 0;
  const int nrep = nh / nkv;
  if (!(nrep == 1 || nrep == 2 || nrep == 4 || nrep == 8)) return 0;
  if (!(hd == 64 || hd == 128)) return 0;
  if (H % BATCH_ELEMS || I % BATCH_ELEMS || (nh * hd) % BATCH_ELEMS) return 0;
  if (V % 2) return 0;
  return 1;
}

// KS = 2 (split the QKV projection's K in halves) when it balances the waves better
CAKE_API int cake_mega_ks(int H, int nh, int nkv, int hd, int grid) {
  if (grid <= 0) grid = cake_mega_grid();
  if (H % (2 * BATCH_ELEMS)) return 1;
  const long nwv = (long)grid * NW;
  const long pairs = (long)(nh + 2 * nkv) * hd / 2;
  const double e1 = (double)pairs / (((pairs + nwv - 1) / nwv) * nwv);
  const double e2 = (double)(2 * pairs) / (((2 * pairs + nwv - 1) / nwv) * nwv);
  return e2 > e1 + 1e-9 ? 2 : 1;
}

CAKE_API int cake_decode_mega(int dt, const void* layers, int L, int H, int I, int nh, int nkv,
                              int hd, int S, int KS, float eps, float scale,
                              const float* inv_freq, const int* pos, float* resid, void* yo_t,
                              void* yd_t, void* qkv_t, void* attn_t, void* act_t,
                              float* attn_part, unsigned* tickets, unsigned* launch_ctr, int* err,
                              const void* norm_f, const void* lm_head, int V, float* logits,
                              int grid, double timeout_s, long long* trace, hipStream_t st) {
  if (!cake_mega_supported(H, I, nh, nkv, hd, V) || L < 1 || L > kMaxLayers)
    return (int)hipErrorInvalidValue;
  if (!(KS == 1 || (KS == 2 && H % (2 * BATCH_ELEMS) == 0))) return (int)hipErrorInvalidValue;
  if (grid <= 0) grid = cake_mega_grid();
  if (grid <= 0) return (int)hipErrorInvalidValue;
  const int kmax = mega_kmax(H, I, nh, nkv, hd, lm_head ? V : 2, KS, grid);
  const size_t lds = mega_lds(H, I, nh, nkv, hd, kmax);
  if (lds > 150 * 1024) return (int)hipErrorInvalidValue;
  Args a;
  a.layers = (const Layer*)layers;
  a.L = L;
  a.H = H; a.I = I; a.nh = nh; a.nkv = nkv; a.hd = hd; a.S = S; a.KS = KS;
  a.eps = eps; a.scale = scale;
  a.inv_freq = inv_freq; a.pos = pos;
  a.resid = resid;
  a.yo_t = (uint64_t*)yo_t; a.yd_t = (uint64_t*)yd_t; a.qkv_t = (uint64_t*)qkv_t;
  a.attn_t = (uint32_t*)attn_t; a.act_t = (uint32_t*)act_t;
  a.attn_part = attn_part; a.tickets = tickets;
  a.launch_ctr = launch_ctr; a.err = err;
  a.norm_f = (const uint16_t*)norm_f; a.lm_head = (const uint16_t*)lm_head;
  a.V = lm_head ? V : 0;
  a.logits = logits;
  a.kmax = kmax;
  a.trace = trace;
  a.xcap = (int)mega_xcap(H, I, nh, nkv, hd);
  a.timeout = (long long)((timeout_s > 0 ? timeout_s : 0.25) * 1e8);
  const int nrep = nh / nkv;
#define CAKE_MEGA(DTV, HDV, NR)                                                            \
  do {                                                                                     \
    auto kern = decode_mega_kernel<DTV, HDV, NR>;                                          \
    static size_t lds_set = 0;                                                             \
    if (lds > lds_set) {                                                                   \
      const hipError_t e = hipFuncSetAttribute(                                            \
          (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);        \
      if (e != hipSuccess) return (int)e;                                                  \
      lds_set = lds;                                                                       \
    }                                                                                      \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, st, a);                            \
  } while (0)
#define CAKE_MEGA_NR(DTV, HDV)                  \
  switch (nrep) {                               \
    case 1: CAKE_MEGA(DTV, HDV, 1); break;      \
    case 2: CAKE_MEGA(DTV, HDV, 2); break;      \
    case 4: CAKE_MEGA(DTV, HDV, 4); break;      \
    default: CAKE_MEGA(DTV, HDV, 8); break;     \
  }
  if (dt == kBF16) {
    if (hd == 128) { CAKE_MEGA_NR(kBF16, 128) } else { CAKE_MEGA_NR(kBF16, 64) }
  } else if (dt == kF16) {
    if (hd == 128) { CAKE_MEGA_NR(kF16, 128) } else { CAKE_MEGA_NR(kF16, 64) }
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef CAKE_MEGA_NR
#undef CAKE_MEGA
  return (int)hipGetLastError();
}
