// Persistent batch-1 decode: every transformer layer of one token in ONE launch.
//
// Replaces the reference's per-token layer loop:
//   cake-core/src/models/llama3/llama.rs:72-138 (block loop of one token),
//   transformer.rs:51-73 (pre-norm block), attention.rs:38-123 (q/k/v, rope, KV
//   append, GQA softmax(QK^T)V, o_proj), mlp.rs:13-33 (SwiGLU), cache.rs:93-122.
//
// Why one launch: the five-launch layer (gemv.hip + attention.hip) streams each
// weight matrix near the HBM rate, but every kernel boundary drains the chip: the
// next launch's first weight bytes are requested only after the previous launch's
// last wave has retired (MI355X_MICROARCH "boundary", ~1.2-1.9 us, 160 per 8B token).
//
// Engine (one workgroup of 8 waves per CU, all resident):
//   * wave 7 is the LOADER: it streams this CU's weight rows of every op of every
//     layer, in order, into an LDS ring of 16 KB slots with LDS-DMA
//     (global_load_lds, nt), keeping up to 4 slots in flight and publishing each
//     landed slot with an LDS word.  It never waits for activations, so the HBM
//     stream runs on through every dependency edge until the ring is full
//     (MI355X_MICROARCH "prefetch-credit", "ldsdma-fill").
//   * waves 0-6 are CONSUMERS: slot i goes to consumer i % 7; a consumer copies its
//     slot to registers, frees it, and takes dot products (v_dot2 f32 <- 2 x 16-bit)
//     with the op's input row, which is staged in LDS as 16-bit (the model dtype,
//     as the reference's Linear sees it).  Partial sums go to LDS per (row pair,
//     consumer) and are added in a fixed order (deterministic).
//   * edges (all-to-all dependencies between ops): every output word is published as
//     an 8-byte {tag, value} granule by one agent-scope (sc1, write-through) store;
//     consumers load the granules of the next op's input and re-poll only the ones
//     whose tag is not yet this launch's (MI355X_MICROARCH "Valid forms" R2: the data
//     is its own flag, no fences).  While they gather, the loader keeps one slot in
//     flight ("thinned"), so the gather's loads do not queue behind the ring fill.
//     Each (layer, edge) has its own granule array; the tag is a launch epoch in
//     device memory, advanced by the last workgroup to exit.
//   * attention: nkv x ns units (ns splits of the live keys, chosen on device from
//     the position) on workgroups spread over the XCDs; split 0 of each group merges
//     and skips o_proj.  Old keys come from the cache, the current position's key /
//     value from the QKV granules.
//   * consumers synchronise among themselves with an LDS counter (the loader never
//     joins a barrier); every global spin is bounded (s_memrealtime): a timeout sets
//     an error word the host checks, and stops every later spin of the launch.
#include "../kernels/common.h"

namespace cake {
namespace mk {

typedef unsigned long long u64;
constexpr int kBlk = 512;       // K elements per row block (1 KB of 16-bit weights)
constexpr int kKeys = 16;       // keys per attention wave block (MFMA M)
constexpr int kMaxSplitMk = 16;
constexpr int kMaxG = 512;
constexpr int kNW = 8;          // waves per workgroup
constexpr int kNL = 2;          // loader waves (the last kNL)
constexpr int kNC = kNW - kNL;  // consumer waves 0 .. kNC-1
constexpr int kNCT = kNC * 64;  // consumer threads
constexpr int kSlot = 16384;    // ring slot bytes: 8 pair-blocks (row a + row b, 1 KB each)
constexpr int kPB = 8;          // pair-blocks per slot
constexpr int kMaxFly = 3;      // slots a loader may keep in flight beyond the one it waits for
constexpr int kMaxRing = 8;

struct Layer {  // device-side pointer table, one entry per layer
  const uint16_t* ln1;
  const uint16_t* wqkv;  // [(nh + 2 nkv) hd, H]: q rows, then k, then v
  const uint16_t* wo;    // [H, nh hd]
  const uint16_t* ln2;
  const uint16_t* wgu;   // [2 I, H]: gate rows, then up
  const uint16_t* wd;    // [H, I]
  uint16_t* kc;          // [nkv][S][hd]
  uint16_t* vc;
};

struct Args {
  const Layer* layers;
  int L, H, I, nh, nkv, hd, S;
  float eps, scale_log2;
  const float* inv_freq;  // [hd/2]
  const int* pos;         // device scalar
  float* resid;           // layer-0 input, final output (f32 [H])
  u64* gran;              // granule workspace, gstride words per layer
  long long gstride;
  unsigned* ctl;          // [0] epoch [1] exit ticket [2] error flag [3] error site
  int maxsplit, single, target, min_keys;
  int ring;               // ring slots
  int thin;               // loader keeps one slot in flight while consumers gather
  int fly;                // slots each loader keeps in flight beyond the one it waits for
  int o_all;              // o_proj rows on every workgroup (1) or not on the mergers (0)
  unsigned long long timeout;  // s_memrealtime ticks (100 MHz)
  unsigned long long* stamps;  // diagnostics (nullptr in production): per-WG phase clocks
};
constexpr int kStampsPerLayer = 14;  // 10 consumer + 4 loader phase clocks

// granule offsets inside one layer's block (words)
struct GOff { long long res, q, kv, att, mid, act, part; };
__host__ __device__ inline GOff goff(int H, int I, int nh, int nkv, int hd, int maxsplit) {
  GOff o;
  o.res = 0;
  o.q = o.res + H;
  o.kv = o.q + (long long)nh * hd;
  o.att = o.kv + (long long)nkv * hd;
  o.mid = o.att + (long long)nh * hd / 2;
  o.act = o.mid + H;
  o.part = o.act + I / 2;
  return o;
}
__host__ __device__ inline long long gstride_words(int H, int I, int nh, int nkv, int hd,
                                                   int maxsplit) {
  const GOff o = goff(H, I, nh, nkv, hd, maxsplit);
  const long long n = o.part + (long long)nh * maxsplit * (hd + 2);
  return (n + 15) / 16 * 16;
}

// ---------------------------------------------------------------------------
// global-address-space access: pointers read from the layer table are generic, and
// generic (flat) loads count against lgkmcnt too.  Every device-memory access goes
// through an address_space(1) pointer (global_load / global_store).
// ---------------------------------------------------------------------------
#define CAKE_G __attribute__((address_space(1)))
#define CAKE_C __attribute__((address_space(4)))
template <class T> __device__ __forceinline__ const CAKE_G T* gp(const T* p) {
  return (const CAKE_G T*)p;
}
template <class T> __device__ __forceinline__ CAKE_G T* gpw(T* p) { return (CAKE_G T*)p; }
__device__ __forceinline__ uint4 ldg16(const void* p) {
  const u32x4 v = *(const CAKE_G u32x4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ u64 gld(const u64* p) {
  return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gst(u64* p, unsigned tag, unsigned v) {
  __hip_atomic_store(gpw(p), ((u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ctl_ld(unsigned* p) {
  return __hip_atomic_load(gpw(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ctl_st(unsigned* p, unsigned v) {
  __hip_atomic_store(gpw(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned pack2(float a, float b, int dt) {
  const uint16_t x = dt == kBF16 ? f32_to_bf16(a) : f32_to_f16(a);
  const uint16_t y = dt == kBF16 ? f32_to_bf16(b) : f32_to_f16(b);
  return (unsigned)x | ((unsigned)y << 16);
}
// LDS words (ring control, consumer barrier): workgroup-scope atomics + LDS-only fences
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// threadIdx.x behind a volatile asm: lane-derived values are recomputed where used
// instead of being hoisted out of the layer loop (each hoisted value held a VGPR for
// the whole kernel and pushed the register allocator into scratch spills)
__device__ __forceinline__ int otid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

// Poll state of one thread: `dead` once any spin of this launch gave up.
struct Spin {
  unsigned long long t0;
  bool dead;
};

__device__ __noinline__ void spin_fail(unsigned* ctl, int site) {
  ctl_st(ctl + 3, (unsigned)site);
  ctl_st(ctl + 2, 1u);
}

// Load granules idx[j] (j < J, idx < n) until every tag == tag; values out.
template <int J>
__device__ __forceinline__ void poll(const u64* g, const int (&idx)[J], int n, unsigned tag,
                                     unsigned (&val)[J], const Args& a, Spin& sp, int site) {
  u64 v[J];
#pragma unroll
  for (int j = 0; j < J; ++j) v[j] = gld(g + (idx[j] < n ? idx[j] : 0));
#pragma unroll
  for (int j = 0; j < J; ++j)
    if (idx[j] >= n) v[j] = (u64)tag << 32;
  if (!sp.dead) {
    for (unsigned it = 0;; ++it) {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < J; ++j) ok = ok && (unsigned)(v[j] >> 32) == tag;
      if (ok) break;
      if ((it & 255u) == 255u) {
        if (__builtin_amdgcn_s_memrealtime() - sp.t0 > a.timeout) {
          spin_fail(a.ctl, site);
          sp.dead = true;
          break;
        }
        if (ctl_ld(a.ctl + 2) != 0u) {
          sp.dead = true;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < J; ++j)
        if (idx[j] < n && (unsigned)(v[j] >> 32) != tag) v[j] = gld(g + idx[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < J; ++j) val[j] = (unsigned)v[j];
}

// Consumer-only barrier: an LDS arrival counter (the loader wave never joins).
struct CBar {
  unsigned* cnt;
  unsigned gen;
};
__device__ __forceinline__ void cbar(CBar& b) {
  b.gen += kNC;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(b.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (lds_ld(b.cnt) < b.gen) __builtin_amdgcn_s_sleep(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// n granules of packed 16-bit pairs -> dst32[0..n) (LDS), consumer threads.
__device__ __forceinline__ void gather_u32(const u64* g, int n, unsigned tag, unsigned* dst,
                                           const Args& a, Spin& sp, int site) {
  const int ct = otid();
  for (int base = 0; base < n; base += 8 * kNCT) {
    int idx[8];
    unsigned v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) idx[j] = base + j * kNCT + ct;
    poll<8>(g, idx, n, tag, v, a, sp, site);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (idx[j] < n) dst[idx[j]] = v[j];
  }
}

// Residual row (H f32: granules, or plain memory written by an earlier launch) ->
// xs[H] = model-dtype(raw * w * rsqrt(mean(raw^2) + eps)), and the f32 rows
// [row_lo, row_lo + nrow) (the residual rows this workgroup's next epilogue adds to)
// into rows[]; consumer threads, 8 words per thread in flight per pass (raw * w staged
// in LDS at stage[H], so no per-thread arrays of H / threads entries are live); ends
// with a consumer barrier.
template <int DT>
__device__ __forceinline__ void gather_norm(const u64* g, const float* plain, int H, unsigned tag,
                                            const uint16_t* w, float eps, float* rows,
                                            int row_lo, int nrow, uint16_t* xs, float* stage,
                                            float* red, CBar& cb, const Args& a, Spin& sp,
                                            int site) {
  const int ct = otid();
  float ss = 0.f;
  for (int base = 0; base < H; base += 8 * kNCT) {
    int idx[8];
    unsigned v[8];
    float wv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      idx[j] = base + j * kNCT + ct;
      wv[j] = to_f32<DT>(gp(w)[idx[j] < H ? idx[j] : 0]);
    }
    if (plain != nullptr) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __float_as_uint(gp(plain)[idx[j] < H ? idx[j] : 0]);
    } else {
      poll<8>(g, idx, H, tag, v, a, sp, site);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = __uint_as_float(v[j]);
      if (idx[j] < H) {
        ss = fmaf(f, f, ss);
        stage[idx[j]] = f * wv[j];
        if ((unsigned)(idx[j] - row_lo) < (unsigned)nrow) rows[idx[j] - row_lo] = f;
      }
    }
  }
  ss = wave_sum(ss);
  if ((ct & 63) == 0) red[ct >> 6] = ss;
  cbar(cb);
  float tot = 0.f;
#pragma unroll
  for (int w2 = 0; w2 < kNC; ++w2) tot += red[w2];
  const float r = rsqrtf(tot / (float)H + eps);
  for (int i = ct; i < H; i += kNCT) xs[i] = from_f32<DT>(stage[i] * r);
  cbar(cb);
}

// ---------------------------------------------------------------------------
// ops: this CU's contiguous range of row pairs of one matrix
// ---------------------------------------------------------------------------
enum OpKind { kQKV = 0, kRows2 = 1, kGU = 2 };
struct Op {
  const uint16_t* base;
  int kind, K, pbeg, npl, bpp;
  unsigned up;  // kGU: byte distance gate row -> up row
};
__device__ __forceinline__ Op make_op(const uint16_t* base, int kind, int K, int P, int nparts,
                                      int ip, int align, unsigned up) {
  Op o;
  o.base = base;
  o.kind = kind;
  o.K = K;
  o.up = up;
  const int Pa = P / align;
  const int s = (int)((long long)ip * Pa / nparts) * align;
  const int e = (int)((long long)(ip + 1) * Pa / nparts) * align;
  o.pbeg = s;
  o.npl = ip < 0 ? 0 : e - s;
  o.bpp = K / kBlk;
  return o;
}
// byte offsets of local pair pl's two rows
template <int HD>
__device__ __forceinline__ void op_rows(const Op& o, int pl, unsigned long long& oa,
                                        unsigned long long& ob) {
  const int p = o.pbeg + pl;
  const unsigned long long rb = (unsigned long long)o.K * 2u;
  if (o.kind == kQKV) {
    constexpr int half = HD / 2;
    const int slot = p / half;
    oa = (unsigned long long)(slot * HD + (p - slot * half)) * rb;
    ob = oa + (unsigned long long)half * rb;
  } else if (o.kind == kRows2) {
    oa = (unsigned long long)(2 * p) * rb;
    ob = oa + rb;
  } else {
    oa = (unsigned long long)p * rb;
    ob = oa + o.up;
  }
}

// The ops of layer l for this workgroup, in stream order: QKV, o_proj (npl 0 on a
// merger), gate/up, down.
template <int HD>
__device__ __forceinline__ Op layer_op(const Args& a, const CAKE_C Layer* ly, int k, int G,
                                       int wg, int o_ip) {
  const int H = a.H, I = a.I, nh = a.nh, nkv = a.nkv;
  if (k == 0) return make_op(ly->wqkv, kQKV, H, (nh + 2 * nkv) * (HD / 2), G, wg, 1, 0u);
  if (k == 1)
    return a.o_all ? make_op(ly->wo, kRows2, nh * HD, H / 2, G, wg, 1, 0u)
                   : make_op(ly->wo, kRows2, nh * HD, H / 2, G - nkv, o_ip, 1, 0u);
  if (k == 2) return make_op(ly->wgu, kGU, H, I, G, wg, 2, (unsigned)I * (unsigned)H * 2u);
  return make_op(ly->wd, kRows2, I, H / 2, G, wg, 1, 0u);
}

// ---------------------------------------------------------------------------
// the loader wave
// ---------------------------------------------------------------------------
// One ring slot: 16 x 1 KB global -> LDS, lane l of load k landing at dst + 1024 k + 16 l,
// non-temporal.  In ONE asm statement (M0 stepped between the loads) so hipcc neither
// counts the loads nor inserts its conservative vmcnt(0) in front of the loader's own
// LDS control accesses; completion is counted by hand (vmcnt below).
__device__ __forceinline__ void glds_slot(const char* const (&p)[16], unsigned dst) {
  unsigned keep;
#define CAKE_GL(k) "global_load_lds_dwordx4 %[p" #k "], off nt\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
  asm volatile("s_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[dst]\n\ts_nop 0\n\t"
               CAKE_GL(0) CAKE_GL(1) CAKE_GL(2) CAKE_GL(3) CAKE_GL(4) CAKE_GL(5) CAKE_GL(6)
               CAKE_GL(7) CAKE_GL(8) CAKE_GL(9) CAKE_GL(10) CAKE_GL(11) CAKE_GL(12) CAKE_GL(13)
               CAKE_GL(14) CAKE_GL(15) "s_mov_b32 m0, %[keep]"
               : [keep] "=&s"(keep)
               : [dst] "s"(dst), [p0] "v"(p[0]), [p1] "v"(p[1]), [p2] "v"(p[2]), [p3] "v"(p[3]),
                 [p4] "v"(p[4]), [p5] "v"(p[5]), [p6] "v"(p[6]), [p7] "v"(p[7]), [p8] "v"(p[8]),
                 [p9] "v"(p[9]), [p10] "v"(p[10]), [p11] "v"(p[11]), [p12] "v"(p[12]),
                 [p13] "v"(p[13]), [p14] "v"(p[14]), [p15] "v"(p[15])
               : "memory", "scc");
#undef CAKE_GL
}

struct RingCtl {
  unsigned full[kMaxRing];  // slot sequence + 1 of the landed fill
  unsigned free_[kMaxRing]; // slot sequence + 1 of the fill consumed
  unsigned cb;              // consumer barrier counter
  unsigned gath;            // consumers are gathering (loader thins)
  unsigned pad[2];
  float red[16];
};

// phase clock of this workgroup (s_memrealtime, 100 MHz, comparable across CUs):
// [wg][layer * kStampsPerLayer + k], then kernel start / end
#define MK_STAMP(idx)                                                                     \
  do {                                                                                    \
    if (a.stamps != nullptr && threadIdx.x == 0)                                          \
      a.stamps[(size_t)blockIdx.x * (a.L * kStampsPerLayer + 2) + (idx)] =                \
          __builtin_amdgcn_s_memrealtime();                                               \
  } while (0)

// Loader wave li (of kNL) fills the ring slots whose sequence number is li mod kNL.
template <int HD>
__device__ void loader_run(const Args& a, int G, int wg, int o_ip, unsigned ring_lds,
                           RingCtl* rc, Spin& sp, int li) {
  const int lane = otid() & 63;
  const unsigned NS = (unsigned)a.ring;
  const char* dummy = reinterpret_cast<const char*>(a.gran) + lane * 16;  // never-written words
  unsigned seq = 0;   // slot sequence of the op being walked (all loaders count all slots)
  unsigned fly = 0;   // this loader's slots in flight
  unsigned last = 0;  // this loader's most recent slot
  auto mark_all = [&]() {
    for (unsigned k = 0; k < fly; ++k) {
      const unsigned q = last - k * kNL;
      lds_st(&rc->full[q % NS], q + 1u);
    }
    fly = 0;
  };
  for (int l = 0; l < a.L; ++l) {
    const CAKE_C Layer* ly = (const CAKE_C Layer*)a.layers + l;
    for (int k = 0; k < 4; ++k) {
      const Op o = layer_op<HD>(a, ly, k, G, wg, o_ip);
      const int tot = o.npl * o.bpp;
      const int nsl = (tot + kPB - 1) / kPB;
      const char* base = reinterpret_cast<const char*>(o.base);
      for (int s = (int)(((unsigned)li + kNL - seq % kNL) % kNL); s < nsl; s += kNL) {
        const unsigned i = seq + (unsigned)s;
        const unsigned r = i % NS;
        if (i >= NS && lds_ld(&rc->free_[r]) < i - NS + 1u) {
          // ring full: publish everything in flight (consumers free a slot only after
          // they have seen it land), then wait for the slot
          __builtin_amdgcn_s_waitcnt(vm_wait(0));
          mark_all();
          for (unsigned it = 0; lds_ld(&rc->free_[r]) < i - NS + 1u; ++it) {
            __builtin_amdgcn_s_sleep(1);
            if ((it & 1023u) == 1023u && (sp.dead || ctl_ld(a.ctl + 2) != 0u ||
                                          __builtin_amdgcn_s_memrealtime() - sp.t0 > a.timeout)) {
              sp.dead = true;
              break;
            }
          }
        }
        const char* pv[16];
        const int q0 = s * kPB;
        int pl = q0 / o.bpp, kb = q0 - pl * o.bpp;
        unsigned long long oa, ob;
        op_rows<HD>(o, pl, oa, ob);
#pragma unroll
        for (int j = 0; j < kPB; ++j) {
          const bool ok = q0 + j < tot;
          const unsigned long long kbo = (unsigned long long)kb * (kBlk * 2) + lane * 16;
          pv[2 * j] = ok ? base + oa + kbo : dummy;
          pv[2 * j + 1] = ok ? base + ob + kbo : dummy;
          if (++kb == o.bpp) {
            kb = 0;
            ++pl;
            op_rows<HD>(o, pl, oa, ob);
          }
        }
        glds_slot(pv, __builtin_amdgcn_readfirstlane(ring_lds + r * kSlot));
        if (li == 0) {  // diagnostics: loader 0's first issue of o_proj / its last, gate/up, down
          const int si = k == 1 && s == 0 ? 10 : k == 1 && s + kNL >= nsl ? 11
                       : k == 2 && s == 0 ? 12 : k == 3 && s == 0 ? 13 : -1;
          if (a.stamps != nullptr && si >= 0 && lane == 0)
            a.stamps[(size_t)blockIdx.x * (a.L * kStampsPerLayer + 2) + l * kStampsPerLayer + si] =
                __builtin_amdgcn_s_memrealtime();
        }
        ++fly;
        last = i;
        if (a.thin && lds_ld(&rc->gath) != 0u) {
          __builtin_amdgcn_s_waitcnt(vm_wait(0));
          mark_all();
        } else if (fly > (unsigned)a.fly) {
          // the oldest of this loader's slots has landed once at most a.fly newer ones
          // (2 kPB loads each) are outstanding
          switch (a.fly) {
            case 0: __builtin_amdgcn_s_waitcnt(vm_wait(0)); break;
            case 1: __builtin_amdgcn_s_waitcnt(vm_wait(2 * kPB)); break;
            case 2: __builtin_amdgcn_s_waitcnt(vm_wait(4 * kPB)); break;
            default: __builtin_amdgcn_s_waitcnt(vm_wait(6 * kPB)); break;
          }
          const unsigned q = last - (unsigned)a.fly * kNL;
          lds_st(&rc->full[q % NS], q + 1u);
          --fly;
        }
      }
      seq += (unsigned)nsl;
    }
  }
  __builtin_amdgcn_s_waitcnt(vm_wait(0));
  mark_all();
}

// ---------------------------------------------------------------------------
// consumers: the slots of one op
// ---------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ float dot8(const uint4 w, const uint4 x, float acc) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  typedef _Float16 hf2 __attribute__((ext_vector_type(2)));
  const unsigned wv[4] = {w.x, w.y, w.z, w.w}, xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if constexpr (DT == kBF16)
      acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, wv[e]),
                                            __builtin_bit_cast(bf2, xv[e]), acc, false);
    else
      acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(hf2, wv[e]), __builtin_bit_cast(hf2, xv[e]),
                                   acc, false);
  }
  return acc;
}

// Consumer wave c: the op's slots seq0 + s (s % kNC == (c - seq0) mod kNC); partial dot
// products accumulated into part[(pl * kNC + c) * 2 + {0, 1}] (column c: this wave only).
template <int DT>
__device__ __forceinline__ void consume_op(const Op& o, unsigned seq0, const uint8_t* ring,
                                           RingCtl* rc, const uint16_t* xs, float* part, int NS,
                                           const Args& a, Spin& sp) {
  const int ct = otid();
  const int c = __builtin_amdgcn_readfirstlane(ct >> 6), lane = ct & 63;
  const int tot = o.npl * o.bpp;
  const int nsl = (tot + kPB - 1) / kPB;
  for (int t = lane; t < o.npl; t += 64) {
    part[(t * kNC + c) * 2] = 0.f;
    part[(t * kNC + c) * 2 + 1] = 0.f;
  }
  const int first = (int)(((unsigned)c + kNC - seq0 % kNC) % kNC);
  for (int s = first; s < nsl; s += kNC) {
    const unsigned i = seq0 + s;
    const int r = (int)(i % (unsigned)NS);
    for (unsigned it = 0; lds_ld(&rc->full[r]) < i + 1u; ++it) {
      __builtin_amdgcn_s_sleep(0);
      if ((it & 4095u) == 4095u && (sp.dead || ctl_ld(a.ctl + 2) != 0u ||
                                    __builtin_amdgcn_s_memrealtime() - sp.t0 > a.timeout)) {
        sp.dead = true;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    const uint8_t* sl = ring + (size_t)r * kSlot + lane * 16;
    uint4 wa[kPB], wb[kPB];
#pragma unroll
    for (int j = 0; j < kPB; ++j) {
      wa[j] = *reinterpret_cast<const uint4*>(sl + (2 * j) * 1024);
      wb[j] = *reinterpret_cast<const uint4*>(sl + (2 * j + 1) * 1024);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the slot is in registers
    lds_st(&rc->free_[r], i + 1u);
    const int q0 = s * kPB;
    int pl = q0 / o.bpp, kb = q0 - pl * o.bpp;
    float aa = 0.f, ab = 0.f;
    int pc = pl;
#pragma unroll
    for (int j = 0; j < kPB; ++j) {
      if (q0 + j < tot) {
        if (pl != pc) {
          const float sa = wave_sum(aa), sb = wave_sum(ab);
          if (lane == 0) {
            part[(pc * kNC + c) * 2] += sa;
            part[(pc * kNC + c) * 2 + 1] += sb;
          }
          aa = ab = 0.f;
          pc = pl;
        }
        const uint4 xv = *reinterpret_cast<const uint4*>(xs + kb * kBlk + lane * 8);
        aa = dot8<DT>(wa[j], xv, aa);
        ab = dot8<DT>(wb[j], xv, ab);
      }
      if (++kb == o.bpp) { kb = 0; ++pl; }
    }
    const float sa = wave_sum(aa), sb = wave_sum(ab);
    if (lane == 0) {
      part[(pc * kNC + c) * 2] += sa;
      part[(pc * kNC + c) * 2 + 1] += sb;
    }
  }
}

__device__ __forceinline__ void pair_sum(const float* part, int t, float& da, float& db) {
  da = 0.f;
  db = 0.f;
#pragma unroll
  for (int c = 0; c < kNC; ++c) {
    da += part[(t * kNC + c) * 2];
    db += part[(t * kNC + c) * 2 + 1];
  }
}

// ---------------------------------------------------------------------------
// attention unit (kv head g, split s): core2-style wave-independent key blocks on the
// consumer waves
// ---------------------------------------------------------------------------
__device__ __forceinline__ void splits_for(int Tk, int min_keys, int maxsplit, int target,
                                           int single, int& ns, int& kps) {
  if (Tk <= single) {
    ns = 1;
    kps = (Tk + kKeys - 1) / kKeys * kKeys;
    return;
  }
  int keys = (Tk + target - 1) / target;
  keys = (keys + kKeys - 1) / kKeys * kKeys;
  if (keys < min_keys) keys = min_keys;
  ns = (Tk + keys - 1) / keys;
  if (ns > maxsplit) ns = maxsplit;
  kps = (Tk + ns - 1) / ns;
  kps = (kps + kKeys - 1) / kKeys * kKeys;
  ns = (Tk + kps - 1) / kps;
}

template <int OFF> __device__ __forceinline__ float xmax(float v) {
  const int b = __builtin_bit_cast(int, v);
  const auto p = OFF == 16 ? __builtin_amdgcn_permlane16_swap(b, b, false, false)
                           : __builtin_amdgcn_permlane32_swap(b, b, false, false);
  return fmaxf(__builtin_bit_cast(float, (int)p[0]), __builtin_bit_cast(float, (int)p[1]));
}

template <int HD, int NREP, int NW>
constexpr int attn_lds_floats() {
  // p tiles + alpha, wave states, q (f32), new k/v rows (16-bit), output row (16-bit)
  return NW * (kKeys * 16 + 16) + NW * (32 + NREP * HD) + NREP * HD + HD + NREP * HD / 2 + 16;
}

template <int DT, int HD, int NREP, int NW>
__device__ __forceinline__ void attn_unit(const Args& a, const uint16_t* kcache,
                                          const uint16_t* vcache, const GOff& go, u64* gl,
                                          unsigned tag,
                          int g, int s, int ns, int kps, int pos, float* lds, Spin& sp, CBar& cb) {
  constexpr int NT = NW * 64;
  constexpr int DS = HD / 32, NCH = HD / 8, KPL = NCH / 4;
  static_assert(NCH == 8 || NCH == 16, "hd 64 or 128");
  static_assert(NREP <= 16, "GQA group");
  const int tid = otid(), wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, rg = lane >> 4;
  const int ch = lane % NCH, kg = lane / NCH;
  float* pt = lds + wave * (kKeys * 16 + 16);
  float* alph = pt + kKeys * 16;
  float* st = lds + NW * (kKeys * 16 + 16);
  float* qs = st + NW * (32 + NREP * HD);
  uint16_t* kn = reinterpret_cast<uint16_t*>(qs + NREP * HD);  // [HD] new key row
  uint16_t* vn = kn + HD;                                       // [HD] new value row
  uint16_t* ob = vn + HD;                                       // [NREP * HD] output
  const int Tk = pos + 1;
  const int kb = s * kps, ke = min(Tk, kb + kps);
  const int nblk = (ke - kb + kKeys - 1) / kKeys;
  const uint16_t* kgp = kcache + (size_t)g * a.S * HD;
  const uint16_t* vgp = vcache + (size_t)g * a.S * HD;
  const int half = HD / 2;

  uint4 kf[DS], vf[KPL];
  auto load_blk = [&](int key0) {
    const int last = ke - 1;
#pragma unroll
    for (int d = 0; d < DS; ++d) {
      const int r = min(key0 + col, last);
      kf[d] = ldg16(kgp + (size_t)r * HD + d * 32 + rg * 8);
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const int r = min(key0 + kg * KPL + j, last);
      vf[j] = ldg16(vgp + (size_t)r * HD + ch * 8);
    }
  };
  // old keys were written by earlier launches: their loads go out before the q edge
  int b = wave;
  if (b < nblk) load_blk(kb + b * kKeys);

  // q of the group (f32 granules) and, for the split holding the current key, the
  // new k/v rows (pair granules (i, i + hd/2))
  const bool has_new = ke == Tk;
  {
    const int nq = NREP * HD;
    const int nn = has_new ? HD : 0;  // HD/2 k pairs + HD/2 v pairs
    constexpr int J = (NREP * HD + HD + NT - 1) / NT;
    int idx[J];
    unsigned v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) idx[j] = j * NT + tid;
    // two arrays behind one index space: [0, nq) q, [nq, nq + nn) k then v pairs
    u64 w[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int i = idx[j];
      const u64* src = i < nq ? gl + go.q + (size_t)g * nq + i
                              : gl + go.kv + (i - nq < half ? (size_t)g * half + (i - nq)
                                                            : (size_t)a.nkv * half + (size_t)g * half + (i - nq - half));
      w[j] = i < nq + nn ? gld(src) : ((u64)tag << 32);
      if (!sp.dead) {
        for (unsigned it = 0; (unsigned)(w[j] >> 32) != tag; ++it) {
          if ((it & 255u) == 255u &&
              (__builtin_amdgcn_s_memrealtime() - sp.t0 > a.timeout ||
               ctl_ld(a.ctl + 2) != 0u)) {
            if (__builtin_amdgcn_s_memrealtime() - sp.t0 > a.timeout) spin_fail(a.ctl, 10);
            sp.dead = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          w[j] = gld(src);
        }
      }
      v[j] = (unsigned)w[j];
      if (i < nq) {
        qs[i] = __uint_as_float(v[j]);
      } else if (i < nq + nn) {
        const int p = i - nq;
        uint16_t* row = p < half ? kn : vn;
        const int ii = p < half ? p : p - half;
        row[ii] = (uint16_t)(v[j] & 0xffffu);
        row[ii + half] = (uint16_t)(v[j] >> 16);
      }
    }
  }
  cbar(cb);
  uint4 qf[DS];
#pragma unroll
  for (int d = 0; d < DS; ++d) {
    uint16_t h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = col < NREP ? qs[col * HD + d * 32 + rg * 8 + e] : 0.f;
      h[e] = from_f32<DT>(x * a.scale_log2);
    }
    qf[d] = *reinterpret_cast<const uint4*>(h);
  }

  float m = -INFINITY, l = 0.f;
  float o[NREP][8];
#pragma unroll
  for (int h = 0; h < NREP; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[h][e] = 0.f;

  for (; b < nblk; b += NW) {
    const int key0 = kb + b * kKeys;
    uint4 kc[DS], vc[KPL];
#pragma unroll
    for (int d = 0; d < DS; ++d) kc[d] = kf[d];
#pragma unroll
    for (int j = 0; j < KPL; ++j) vc[j] = vf[j];
    if (b + NW < nblk) load_blk(key0 + NW * kKeys);
    // the current position's row comes from the granules (the cache row is being
    // written by another workgroup in this launch)
    if (key0 + col == pos) {
#pragma unroll
      for (int d = 0; d < DS; ++d) kc[d] = *reinterpret_cast<const uint4*>(kn + d * 32 + rg * 8);
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j)
      if (key0 + kg * KPL + j == pos) vc[j] = *reinterpret_cast<const uint4*>(vn + ch * 8);
    cf32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < DS; ++d) acc = cmfma<DT>(kc[d], qf[d], acc);
    float sc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) sc[e] = key0 + 4 * rg + e < ke ? acc[e] : -INFINITY;
    float bm = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
    bm = xmax<32>(xmax<16>(bm));
    const float mn = fmaxf(m, bm);
    const float alpha = exp2f(m - mn);
    float p[4], ps = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) { p[e] = exp2f(sc[e] - mn); ps += p[e]; }
    ps = xor_add<32>(xor_add<16>(ps));
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int e = 0; e < 4; ++e) pt[(4 * rg + e) * 16 + col] = p[e];
    if (rg == 0) alph[col] = alpha;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
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
    __builtin_amdgcn_wave_barrier();
  }
  // key-group sums, wave states -> LDS, merge the NW waves
#pragma unroll
  for (int h = 0; h < NREP; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = o[h][e];
      if constexpr (NCH == 8) v = xor_add<8>(v);
      o[h][e] = xor_add<32>(xor_add<16>(v));
    }
  float* ws = st + wave * (32 + NREP * HD);
  if (lane < 16) { ws[lane] = m; ws[16 + lane] = l; }
  if (kg == 0) {
#pragma unroll
    for (int h = 0; h < NREP; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) ws[32 + h * HD + ch * 8 + e] = o[h][e];
  }
  cbar(cb);
  constexpr int NOUT = NREP * HD;
  constexpr int OPT = (NOUT + NT - 1) / NT;
  float mo[OPT], lo[OPT], ao[OPT];
#pragma unroll
  for (int i = 0; i < OPT; ++i) {
    const int idx = tid + i * NT;
    const int h = idx / HD, d = idx - h * HD;
    float M = -INFINITY, L = 0.f, A = 0.f;
    if (idx < NOUT) {
#pragma unroll
      for (int w = 0; w < NW; ++w) M = fmaxf(M, st[w * (32 + NREP * HD) + h]);
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
  u64* att = gl + go.att + (size_t)g * NOUT / 2;
  if (ns == 1) {
#pragma unroll
    for (int i = 0; i < OPT; ++i) {
      const int idx = tid + i * NT;
      if (idx < NOUT) ob[idx] = from_f32<DT>(ao[i] / lo[i]);
    }
  } else if (s != 0) {
    // partial {m, l, o[HD]} of each head as f32 granules
    u64* gp = gl + go.part;
#pragma unroll
    for (int i = 0; i < OPT; ++i) {
      const int idx = tid + i * NT;
      if (idx < NOUT) {
        const int h = idx / HD, d = idx - h * HD;
        u64* dst = gp + ((size_t)(g * NREP + h) * a.maxsplit + s) * (HD + 2);
        if (d == 0) {
          gst(dst, tag, __float_as_uint(mo[i]));
          gst(dst + 1, tag, __float_as_uint(lo[i]));
        }
        gst(dst + 2 + d, tag, __float_as_uint(ao[i]));
      }
    }
    cbar(cb);  // LDS (st) reuse by the caller
    return;
  } else {
    // split 0: own partial -> LDS (p tiles are free), one wave per head merges
    float* own = lds;
    static_assert(NREP * (HD + 2) <= NW * (kKeys * 16 + 16), "own partial fits the p tiles");
    cbar(cb);
#pragma unroll
    for (int i = 0; i < OPT; ++i) {
      const int idx = tid + i * NT;
      if (idx < NOUT) {
        const int h = idx / HD, d = idx - h * HD;
        if (d == 0) { own[h * (HD + 2)] = mo[i]; own[h * (HD + 2) + 1] = lo[i]; }
        own[h * (HD + 2) + 2 + d] = ao[i];
      }
    }
    cbar(cb);
    for (int h = wave; h < NREP; h += NW) {
      constexpr int DPL = HD / 64;
      const u64* src = gl + go.part + (size_t)(g * NREP + h) * a.maxsplit * (HD + 2);
      const float* ow = own + h * (HD + 2);
      // lane t < ns holds split t's (m, l); o rows of splits 1..ns-1, DPL dims per lane
      float mt = lane == 0 ? ow[0] : -INFINITY, lt = lane == 0 ? ow[1] : 0.f;
      float acc[DPL];
      {
        int id2[2];
        unsigned v2[2];
        id2[0] = (lane >= 1 && lane < ns) ? lane * (HD + 2) : 1 << 30;
        id2[1] = (lane >= 1 && lane < ns) ? lane * (HD + 2) + 1 : 1 << 30;
        poll<2>(src, id2, 1 << 29, tag, v2, a, sp, 11);
        if (lane >= 1 && lane < ns) { mt = __uint_as_float(v2[0]); lt = __uint_as_float(v2[1]); }
      }
      const float M = wave_max(mt);
      const float wt = lane < ns ? exp2f(mt - M) : 0.f;
      const float L = wave_sum(wt * lt);
      const float w0 = __shfl(wt, 0, 64);
#pragma unroll
      for (int d = 0; d < DPL; ++d) acc[d] = w0 * ow[2 + lane * DPL + d];
      // o rows of 8 splits per poll round (all requested before any is used)
      constexpr int RU = 8;
      for (int t0 = 1; t0 < ns; t0 += RU) {
        int id[RU * DPL];
        unsigned vv[RU * DPL];
#pragma unroll
        for (int u = 0; u < RU; ++u)
#pragma unroll
          for (int d = 0; d < DPL; ++d)
            id[u * DPL + d] = t0 + u < ns ? (t0 + u) * (HD + 2) + 2 + lane * DPL + d : 1 << 30;
        poll<RU * DPL>(src, id, 1 << 29, tag, vv, a, sp, 12);
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const float wtt = __shfl(wt, t0 + u < 64 ? t0 + u : 63, 64);
          if (t0 + u < ns) {
#pragma unroll
            for (int d = 0; d < DPL; ++d) acc[d] = fmaf(wtt, __uint_as_float(vv[u * DPL + d]), acc[d]);
          }
        }
      }
      const float inv = 1.f / L;
#pragma unroll
      for (int d = 0; d < DPL; ++d) ob[h * HD + lane * DPL + d] = from_f32<DT>(acc[d] * inv);
    }
  }
  cbar(cb);
  // publish the group's output: 2 x 16-bit per granule
  for (int i = tid; i < NOUT / 2; i += NT) {
    const unsigned w = (unsigned)ob[2 * i] | ((unsigned)ob[2 * i + 1] << 16);
    gst(att + i, tag, w);
  }
  cbar(cb);
}


// ---------------------------------------------------------------------------
// the persistent kernel
// ---------------------------------------------------------------------------
__device__ __forceinline__ int merger_wg(int g, int G, int nkv) {
  return g * (G / nkv) + (g & 7);
}

// LDS layout (bytes): ring | RingCtl | rows f32[kMaxRows] | part f32[maxpl][kNC][2] | xs
constexpr int kMaxRows = 64;  // residual rows of one workgroup's o_proj / down share
struct Lds {
  unsigned ring, ctl, raw, part, xs, total;
};
__host__ __device__ inline Lds lds_layout(int H, int I, int nh, int hd, int nrep, int G, int ring) {
  Lds o;
  const int maxpl = (I + G - 1) / G + 2;
  o.ring = 0;
  o.ctl = o.ring + (unsigned)ring * kSlot;
  o.raw = o.ctl + (unsigned)((sizeof(RingCtl) + 15) / 16 * 16);
  o.part = o.raw + (unsigned)kMaxRows * 4u;
  o.xs = o.part + (unsigned)(maxpl * kNC * 2 * 4 + 15) / 16 * 16;
  unsigned xs = (unsigned)H * 6u;  // 16-bit normalised row + its f32 staging
  const unsigned x16 = (unsigned)(nh * hd > I ? nh * hd : I) * 2u;
  if (x16 > xs) xs = x16;
  const unsigned at = 4u * (unsigned)(kNC * (kKeys * 16 + 16) + kNC * (32 + nrep * hd) + nrep * hd +
                                      hd + nrep * hd / 2 + 16);
  if (at > xs) xs = at;
  o.total = o.xs + xs;
  return o;
}

template <int DT, int HD, int NREP>
__global__ __launch_bounds__(kNW * 64) void mk_decode_kernel(Args a) {
  constexpr int half = HD / 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int G = gridDim.x, wg = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int H = a.H, I = a.I, nh = a.nh, nkv = a.nkv, S = a.S;
  const int KO = nh * HD;
  const Lds lay = lds_layout(H, I, nh, HD, NREP, G, a.ring);
  uint8_t* ring = smem + lay.ring;
  RingCtl* rc = reinterpret_cast<RingCtl*>(smem + lay.ctl);
  float* rows = reinterpret_cast<float*>(smem + lay.raw);
  float* part = reinterpret_cast<float*>(smem + lay.part);
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem + lay.xs);

  if (threadIdx.x < sizeof(RingCtl) / 4) reinterpret_cast<unsigned*>(rc)[threadIdx.x] = 0u;
  __syncthreads();

  Spin sp;
  sp.t0 = __builtin_amdgcn_s_memrealtime();
  sp.dead = ctl_ld(a.ctl + 2) != 0u;
  const unsigned tag = ctl_ld(a.ctl) + 1u;
  const int pos = *gp(a.pos);
  int ns, kps;
  splits_for(pos + 1, a.min_keys, a.maxsplit, a.target, a.single, ns, kps);
  // attention role
  int my_g = -1, my_s = -1, n_merg_below = 0;
  for (int g = 0; g < nkv; ++g) {
    const int base = merger_wg(g, G, nkv);
    if (wg >= base && wg < base + ns) { my_g = g; my_s = wg - base; }
    if (base < wg) ++n_merg_below;
  }
  const bool is_attn = my_g >= 0;
  const bool is_merger = is_attn && my_s == 0;
  const int o_ip = is_merger ? -1 : wg - n_merg_below;  // index among o_proj workgroups
  const GOff go = goff(H, I, nh, nkv, HD, a.maxsplit);
  MK_STAMP(a.L * kStampsPerLayer);

  if (wave >= kNC) {
    loader_run<HD>(a, G, wg, o_ip,
                   (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)ring, rc,
                   sp, wave - kNC);
  } else {
    CBar cb{&rc->cb, 0u};
    unsigned seq = 0;
    auto set_gath = [&](unsigned v) {
      if (otid() == 0) lds_st(&rc->gath, v);
    };
    for (int l = 0; l < a.L; ++l) {
      const int tid = otid();
      const CAKE_C Layer* ly = (const CAKE_C Layer*)a.layers + l;
      u64* gl = a.gran + (size_t)l * a.gstride;
      const int sb = l * kStampsPerLayer;
      // ---------------- QKV + RoPE + KV write ----------------
      set_gath(1u);
      const Op oo = layer_op<HD>(a, ly, 1, G, wg, o_ip);
      gather_norm<DT>(gl + go.res, l == 0 ? a.resid : nullptr, H, tag, ly->ln1, a.eps, rows,
                      2 * oo.pbeg, 2 * oo.npl, xs, reinterpret_cast<float*>(xs + H),
                          rc->red, cb, a, sp, 1);
      set_gath(0u);
      MK_STAMP(sb + 0);
      {
        const Op o = layer_op<HD>(a, ly, 0, G, wg, o_ip);
        consume_op<DT>(o, seq, ring, rc, xs, part, a.ring, a, sp);
        seq += (o.npl * o.bpp + kPB - 1) / kPB;
        cbar(cb);
        MK_STAMP(sb + 1);
        uint16_t* kc = ly->kc;
        uint16_t* vc = ly->vc;
        for (int t = tid; t < o.npl; t += kNCT) {
          float da, db;
          pair_sum(part, t, da, db);
          const int p = o.pbeg + t;
          const int slot = p / half, i = p - slot * half;
          const int kind = slot < nh ? 0 : (slot < nh + nkv ? 1 : 2);
          const int head = slot - (kind == 0 ? 0 : (kind == 1 ? nh : nh + nkv));
          float oa = da, ob = db;
          if (kind < 2) {
            float sn, cs;
            sincosf((float)pos * gp(a.inv_freq)[i], &sn, &cs);
            oa = da * cs - db * sn;
            ob = da * sn + db * cs;
          }
          if (kind == 0) {
            gst(gl + go.q + (size_t)head * HD + i, tag, __float_as_uint(oa));
            gst(gl + go.q + (size_t)head * HD + i + half, tag, __float_as_uint(ob));
          } else {
            uint16_t* cache = kind == 1 ? kc : vc;
            const size_t off = ((size_t)head * S + pos) * HD + i;
            const uint16_t ha = from_f32<DT>(oa), hb = from_f32<DT>(ob);
            gpw(cache)[off] = ha;
            gpw(cache)[off + half] = hb;
            gst(gl + go.kv + (size_t)(kind - 1) * nkv * half + (size_t)head * half + i, tag,
                (unsigned)ha | ((unsigned)hb << 16));
          }
        }
        cbar(cb);
        MK_STAMP(sb + 2);
      }
      // ---------------- attention ----------------
      if (is_attn)
        attn_unit<DT, HD, NREP, kNC>(a, ly->kc, ly->vc, go, gl, tag, my_g, my_s, ns, kps, pos,
                                     reinterpret_cast<float*>(xs), sp, cb);
      // ---------------- o_proj + residual ----------------
      {
        const Op o = layer_op<HD>(a, ly, 1, G, wg, o_ip);
        if (o.npl > 0) {
          set_gath(1u);
          gather_u32(gl + go.att, KO / 2, tag, reinterpret_cast<unsigned*>(xs), a, sp, 2);
          set_gath(0u);
          cbar(cb);
          MK_STAMP(sb + 3);
          consume_op<DT>(o, seq, ring, rc, xs, part, a.ring, a, sp);
          seq += (o.npl * o.bpp + kPB - 1) / kPB;
          cbar(cb);
          MK_STAMP(sb + 4);
          for (int t = tid; t < o.npl; t += kNCT) {
            float da, db;
            pair_sum(part, t, da, db);
            const int row = 2 * (o.pbeg + t);
            gst(gl + go.mid + row, tag, __float_as_uint(rows[2 * t] + da));
            gst(gl + go.mid + row + 1, tag, __float_as_uint(rows[2 * t + 1] + db));
          }
          cbar(cb);
        }
      }
      // ---------------- RMSNorm + gate/up + SwiGLU ----------------
      set_gath(1u);
      const Op od = layer_op<HD>(a, ly, 3, G, wg, o_ip);
      gather_norm<DT>(gl + go.mid, nullptr, H, tag, ly->ln2, a.eps, rows, 2 * od.pbeg,
                      2 * od.npl, xs, reinterpret_cast<float*>(xs + H), rc->red, cb, a,
                          sp, 3);
      set_gath(0u);
      MK_STAMP(sb + 5);
      {
        const Op o = layer_op<HD>(a, ly, 2, G, wg, o_ip);
        consume_op<DT>(o, seq, ring, rc, xs, part, a.ring, a, sp);
        seq += (o.npl * o.bpp + kPB - 1) / kPB;
        cbar(cb);
        MK_STAMP(sb + 6);
        for (int t = tid; 2 * t < o.npl; t += kNCT) {
          float g0, u0, g1, u1;
          pair_sum(part, 2 * t, g0, u0);
          pair_sum(part, 2 * t + 1, g1, u1);
          const int j = o.pbeg + 2 * t;
          gst(gl + go.act + j / 2, tag, pack2(silu(g0) * u0, silu(g1) * u1, DT));
        }
        cbar(cb);
      }
      // ---------------- down_proj + residual ----------------
      set_gath(1u);
      gather_u32(gl + go.act, I / 2, tag, reinterpret_cast<unsigned*>(xs), a, sp, 4);
      set_gath(0u);
      cbar(cb);
      MK_STAMP(sb + 7);
      {
        const Op o = layer_op<HD>(a, ly, 3, G, wg, o_ip);
        consume_op<DT>(o, seq, ring, rc, xs, part, a.ring, a, sp);
        seq += (o.npl * o.bpp + kPB - 1) / kPB;
        cbar(cb);
        MK_STAMP(sb + 8);
        u64* gn = gl + a.gstride;
        const bool last = l + 1 == a.L;
        for (int t = tid; t < o.npl; t += kNCT) {
          float da, db;
          pair_sum(part, t, da, db);
          const int row = 2 * (o.pbeg + t);
          const float va = rows[2 * t] + da, vb = rows[2 * t + 1] + db;
          if (!last) {
            gst(gn + go.res + row, tag, __float_as_uint(va));
            gst(gn + go.res + row + 1, tag, __float_as_uint(vb));
          } else {
            gpw(a.resid)[row] = va;
            gpw(a.resid)[row + 1] = vb;
          }
        }
        cbar(cb);
        MK_STAMP(sb + 9);
      }
    }
  }
  MK_STAMP(a.L * kStampsPerLayer + 1);
  // exit: the last workgroup advances the epoch (the next launch's tag)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(gpw(a.ctl + 1), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)G - 1u) {
      ctl_st(a.ctl + 1, 0u);
      ctl_st(a.ctl, tag);
    }
  }
}

}  // namespace mk
}  // namespace cake

using namespace cake;

namespace {
int g_mk_grid = 0;
unsigned long long* g_mk_stamps = nullptr;  // diagnostics only
int g_mk_thin = 1;
int g_mk_ring = 0;  // 0 = as many slots as fit
int g_mk_fly = 1;
int g_mk_o_all = 1;

int mk_grid() {
  if (g_mk_grid > 0) return g_mk_grid;
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  g_mk_grid = n;
  return n;
}

constexpr unsigned kLdsMax = 160 * 1024;

int ring_slots(int H, int I, int nh, int hd, int nrep, int G) {
  const mk::Lds z = mk::lds_layout(H, I, nh, hd, nrep, G, 0);
  if (z.total >= kLdsMax) return 0;
  int n = (int)((kLdsMax - z.total) / mk::kSlot);
  if (n > mk::kMaxRing) n = mk::kMaxRing;
  if (g_mk_ring > 0 && g_mk_ring < n) n = g_mk_ring;
  return n;
}

template <int DT, int HD, int NREP>
int mk_launch(const mk::Args& a, int G, size_t lds, hipStream_t st) {
  auto kern = mk::mk_decode_kernel<DT, HD, NREP>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kLdsMax) != hipSuccess)
      return (int)hipErrorInvalidValue;
    attr_set = true;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, mk::kNW * 64, lds) !=
          hipSuccess ||
      per_cu < 1)
    return (int)hipErrorLaunchOutOfResources;
  hipLaunchKernelGGL(kern, dim3(G), dim3(mk::kNW * 64), lds, st, a);
  return (int)hipGetLastError();
}
}  // namespace

// Granule words per layer of the workspace (one block per layer, zero-initialised
// once together with ctl; the kernel never needs them re-zeroed).
CAKE_API long long cake_mk_gstride(int H, int I, int nh, int nkv, int hd) {
  return mk::gstride_words(H, I, nh, nkv, hd, mk::kMaxSplitMk);
}

CAKE_API int cake_mk_grid() { return mk_grid(); }

// Diagnostics: per-workgroup phase clocks, [grid][L * 10 + 2] u64 (nullptr = off).
CAKE_API int cake_mk_set_stamps(void* p) {
  g_mk_stamps = (unsigned long long*)p;
  return 0;
}

// Tuning / A-B: loader thinning during gathers (0/1), a cap on the ring slots (0 = as
// many as fit in LDS) and the slots each loader keeps in flight beyond the one it waits
// for (0..3): HBM saturates at a small in-flight depth per CU, and every slot in flight
// is one not yet landed — ring space that banks no credit across an edge.
CAKE_API int cake_mk_set_tuning(int thin, int ring, int fly, int o_all) {
  if (ring < 0 || ring > mk::kMaxRing || fly < 0 || fly > mk::kMaxFly)
    return (int)hipErrorInvalidValue;
  g_mk_thin = thin != 0;
  g_mk_ring = ring;
  g_mk_fly = fly;
  g_mk_o_all = o_all != 0;
  return 0;
}

// Shapes the persistent decode supports (0 = supported).
CAKE_API int cake_mk_supported(int H, int I, int nh, int nkv, int hd) {
  const int G = mk_grid();
  if (G <= 0) return 1;
  if (H % mk::kBlk || I % mk::kBlk || (nh * hd) % mk::kBlk) return 2;
  if (hd != 128 || nkv <= 0 || nh % nkv) return 3;
  const int nrep = nh / nkv;
  if (nrep != 4 && nrep != 8) return 4;
  if (H % 8) return 5;
  if (G < nkv * (mk::kMaxSplitMk + 8) || G - nkv < 1 || G > mk::kMaxG) return 6;
  if (ring_slots(H, I, nh, hd, nrep, G) < 2) return 7;
  if ((H / 2) < G || (nh + 2 * nkv) * hd / 2 < G) return 8;
  if (2 * ((H / 2 + G - nkv - 1) / (G - nkv)) > mk::kMaxRows) return 9;
  return 0;
}

// layers: device array of L mk::Layer (8 pointers each); gran: L * gstride words;
// ctl: 4 words; all zero-initialised before the first launch.
CAKE_API int cake_mk_decode(int dt, const void* layers, int L, int H, int I, int nh, int nkv,
                            int hd, int S, float eps, float scale, const float* inv_freq,
                            const int* pos, float* resid, void* gran, unsigned* ctl,
                            double timeout_s, hipStream_t st) {
  if (cake_mk_supported(H, I, nh, nkv, hd) != 0 || L <= 0 || S <= 0 || !layers || !gran || !ctl)
    return (int)hipErrorInvalidValue;
  const int G = mk_grid();
  const int nrep = nh / nkv;
  mk::Args a;
  a.layers = (const mk::Layer*)layers;
  a.L = L; a.H = H; a.I = I; a.nh = nh; a.nkv = nkv; a.hd = hd; a.S = S;
  a.eps = eps;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.inv_freq = inv_freq;
  a.pos = pos;
  a.resid = resid;
  a.gran = (mk::u64*)gran;
  a.gstride = mk::gstride_words(H, I, nh, nkv, hd, mk::kMaxSplitMk);
  a.ctl = ctl;
  a.maxsplit = mk::kMaxSplitMk;
  a.single = 320;
  a.target = 16;
  a.min_keys = 64;
  a.ring = ring_slots(H, I, nh, hd, nrep, G);
  a.thin = g_mk_thin;
  a.fly = g_mk_fly;
  a.o_all = g_mk_o_all;
  a.timeout = (unsigned long long)(timeout_s * 1e8);
  a.stamps = g_mk_stamps;
  const size_t lds = mk::lds_layout(H, I, nh, hd, nrep, G, a.ring).total;
  if (dt == kBF16) {
    return nrep == 4 ? mk_launch<kBF16, 128, 4>(a, G, lds, st) : mk_launch<kBF16, 128, 8>(a, G, lds, st);
  } else if (dt == kF16) {
    return nrep == 4 ? mk_launch<kF16, 128, 4>(a, G, lds, st) : mk_launch<kF16, 128, 8>(a, G, lds, st);
  }
  return (int)hipErrorInvalidValue;
}
