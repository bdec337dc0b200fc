// Persistent batch-1 decode: every transformer layer of one token in ONE launch.
//
// Replaces the reference's per-token layer loop:
//   cake-core/src/models/llama3/llama.rs:72-138 (block loop of one token),
//   transformer.rs:51-73 (pre-norm block), attention.rs:38-123 (q/k/v, rope, KV
//   append, GQA softmax(QK^T)V, o_proj), mlp.rs:13-33 (SwiGLU), cache.rs:93-122.
//
// Why one launch: the five-launch layer (gemv.hip + attention.hip) streams each
// weight matrix near the HBM rate, but every kernel boundary drains the chip:
// the next launch's first weight bytes are requested only after the previous
// launch's last wave has retired (~1.2-1.9 us per boundary, 160 per 8B token;
// MI355X_MICROARCH "boundary").  Here each workgroup (one per CU, all resident)
// requests its FIRST weight block of the next op before it waits for that op's
// input vector, so the HBM stream runs through every dependency edge.
//
// Structure (G = #CUs workgroups of NW waves, one per CU):
//   * op = QKV+RoPE | attention | o_proj+residual | RMSNorm+gate/up+SwiGLU |
//     down_proj+residual.  A GEMV op's row pairs are split into contiguous
//     per-workgroup ranges; inside a workgroup the (pair x 512-element K block)
//     space is split evenly over the waves, each wave keeps U blocks of both rows
//     in flight (double-buffered registers), partial dot products go to LDS per
//     (pair, wave) and are summed in a fixed order (deterministic).
//   * edges (the all-to-all dependencies): every output word is published as an
//     8-byte {tag, value} granule with one agent-scope (sc1, write-through) store;
//     consumers sweep the granules with agent-scope loads until every tag is this
//     launch's (MI355X_MICROARCH "Valid forms" R2: the data is its own flag, no
//     fences).  Each (layer, edge) has its own granule array; the tag is a launch
//     epoch kept in device memory and advanced by the last workgroup to exit, so
//     graph replays never see a previous launch's words.
//   * attention: nkv x ns units (ns splits of the live keys, chosen on device
//     from the position) run on workgroups spread over the XCDs; the
//     workgroups holding split 0 (the mergers) skip o_proj, so the attention
//     chain overlaps everyone else's o_proj weight prefetch.  Old keys come from
//     the cache (written by earlier launches), the current position's key/value
//     from the QKV granules.
//   * every spin is bounded (s_memrealtime); a timeout sets an error word the
//     host checks, and stops every later spin of the launch instead of hanging.
#include "common.h"

namespace cake {
namespace mk {

typedef unsigned long long u64;
constexpr int kBlk = 512;    // K elements per weight block: 64 lanes x 8
constexpr int kKeys = 16;    // keys per attention wave block (MFMA M)
constexpr int kMaxSplitMk = 16;

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
  unsigned long long timeout;  // s_memrealtime ticks (100 MHz)
  unsigned long long* stamps;  // diagnostics (nullptr in production): per-WG phase clocks
};
constexpr int kStampsPerLayer = 10;

// granule offsets inside one layer's block (words)
// sentinels: per edge one granule per producing workgroup (kMaxG slots)
constexpr int kMaxG = 512;
enum Edge { kERes = 0, kEQkv = 1, kEAtt = 2, kEMid = 3, kEAct = 4, kNumEdges = 5 };
struct GOff { long long res, q, kv, att, mid, act, part, sent; };
__host__ __device__ inline GOff goff(int H, int I, int nh, int nkv, int hd, int maxsplit) {
  GOff o;
  o.res = 0;
  o.q = o.res + H;
  o.kv = o.q + (long long)nh * hd;
  o.att = o.kv + (long long)nkv * hd;
  o.mid = o.att + (long long)nh * hd / 2;
  o.act = o.mid + H;
  o.part = o.act + I / 2;
  o.sent = o.part + (long long)nh * maxsplit * (hd + 2);
  return o;
}
__host__ __device__ inline long long gstride_words(int H, int I, int nh, int nkv, int hd,
                                                   int maxsplit) {
  const GOff o = goff(H, I, nh, nkv, hd, maxsplit);
  const long long n = o.sent + (long long)kNumEdges * kMaxG;
  return (n + 15) / 16 * 16;
}

// ---------------------------------------------------------------------------
// global-address-space access: pointers read from the layer table are generic, and
// generic (flat) loads count against lgkmcnt too, so every LDS wait would also wait
// for the whole in-flight weight stream.  Every device-memory access below goes
// through an address_space(1) pointer (global_load / global_store).
// ---------------------------------------------------------------------------
#define CAKE_G __attribute__((address_space(1)))
template <class T> __device__ __forceinline__ const CAKE_G T* gp(const T* p) {
  return (const CAKE_G T*)p;
}
template <class T> __device__ __forceinline__ CAKE_G T* gpw(T* p) { return (CAKE_G T*)p; }
__device__ __forceinline__ uint4 ldg_nt16(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load((const CAKE_G u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ldg16(const void* p) {
  const u32x4 v = *(const CAKE_G u32x4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}

// granules
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
  for (int j = 0; j < J; ++j) v[j] = idx[j] < n ? gld(g + idx[j]) : ((u64)tag << 32);
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

// n granules of packed 16-bit pairs -> dst32[0..n) (LDS), all threads.
template <int NT>
__device__ __forceinline__ void gather_u32(const u64* g, int n, unsigned tag, unsigned* dst,
                                           const Args& a, Spin& sp, int site) {
  for (int base = 0; base < n; base += 8 * NT) {
    int idx[8];
    unsigned v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) idx[j] = base + j * NT + otid();
    poll<8>(g, idx, n, tag, v, a, sp, site);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (idx[j] < n) dst[idx[j]] = v[j];
  }
}

// The poller wave: wait until the sentinels [0, n) of one edge carry `tag` (each
// producing workgroup stores its sentinel after its data granules).  One wave polls
// n words per pass instead of every thread polling every data granule — that storm of
// agent-scope loads competed with the weight stream.  The data granules keep their
// own tags, so a sentinel seen before some data (no store ordering is assumed) only
// costs that thread a short re-poll in the sweep.
__device__ __forceinline__ void wait_sent(const u64* sent, int n, unsigned tag, const Args& a,
                                          Spin& sp, int site) {
  const int lane = otid() & 63;
  for (int base = 0; base < n; base += 4 * 64) {
    int idx[4];
    unsigned v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) idx[j] = base + j * 64 + lane;
    poll<4>(sent, idx, n, tag, v, a, sp, site);
  }
}

// Residual row (H f32: granules, or plain memory written by an earlier launch)
// -> raw[H] (LDS) and xs[H] = raw * rsqrt(mean(raw^2) + eps) * w (LDS).
template <int DT, int NT, int J>
__device__ __forceinline__ void gather_norm(const u64* g, const float* plain, int H, unsigned tag,
                                            const uint16_t* w, float eps, float* raw, float* xs,
                                            float* red, const Args& a, Spin& sp, int site) {
  int idx[J];
  unsigned v[J];
  float wv[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    idx[j] = j * NT + otid();
    wv[j] = idx[j] < H ? to_f32<DT>(gp(w)[idx[j]]) : 0.f;
  }
  if (plain != nullptr) {
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = idx[j] < H ? __float_as_uint(gp(plain)[idx[j]]) : 0u;
  } else {
    poll<J>(g, idx, H, tag, v, a, sp, site);
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const float f = __uint_as_float(v[j]);
    if (idx[j] < H) { raw[idx[j]] = f; ss = fmaf(f, f, ss); }
  }
  ss = block_sum(ss, red);
  const float r = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int j = 0; j < J; ++j)
    if (idx[j] < H) xs[idx[j]] = __uint_as_float(v[j]) * r * wv[j];
}

// ---------------------------------------------------------------------------
// weight-streaming GEMV core
// ---------------------------------------------------------------------------
template <int U> struct Batch { uint4 a[U], b[U]; };

// One op's share of a workgroup: pairs [pbeg, pbeg + npl); this wave's blocks [b0, b1)
// of the flattened (pair, 512-element K block) space, bpp blocks per pair.
struct Rng { int pbeg, npl, bpp, b0, b1; };

__device__ __forceinline__ Rng make_rng(int P, int nparts, int ip, int K, int wave, int NW,
                                        int align) {
  Rng r;
  const int Pa = P / align;
  const int s = (int)((long long)ip * Pa / nparts) * align;
  const int e = (int)((long long)(ip + 1) * Pa / nparts) * align;
  r.pbeg = s;
  r.npl = ip < 0 ? 0 : e - s;
  r.bpp = K / kBlk;
  const int tot = r.npl * r.bpp;
  r.b0 = wave * tot / NW;
  r.b1 = (wave + 1) * tot / NW;
  return r;
}

// Weight rows are read through a buffer resource over the whole matrix: a block past
// the wave's range gets an out-of-range offset, which the hardware answers with zeros
// and no memory traffic — so every load is unconditional (a load under a branch left
// its result in a phi, and the compiler waited for it right there).
// (the base pointer comes from the layer table through a vector load: readfirstlane
// makes it provably uniform, else every buffer load became a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  const unsigned long long v = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  void* b = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, (int)bytes, 0x00020000);
}
constexpr unsigned kOob = 0xFFFFFFF0u;
__device__ __forceinline__ uint4 bload_nt(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2);  // aux 2 = nt
  return make_uint4(v.x, v.y, v.z, v.w);
}

// map.offs(pair_local, oa, ob): byte offsets of the pair's two rows in map.rs
template <int U, class Map>
__device__ __forceinline__ void issue(const Map& map, int bpp, int b, int b1, Batch<U>& B) {
  const unsigned lo = (unsigned)(otid() & 63) * 16u;
  int pl = b / bpp, kb = b - pl * bpp;
  unsigned oa, ob;
  map.offs(pl, oa, ob);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool ok = b + u < b1;
    const unsigned kbo = (unsigned)kb * (kBlk * 2) + lo;
    B.a[u] = bload_nt(map.rs, ok ? oa + kbo : kOob);
    B.b[u] = bload_nt(map.rs, ok ? ob + kbo : kOob);
    if (++kb == bpp) {
      kb = 0;
      ++pl;
      map.offs(pl, oa, ob);
    }
  }
}

template <int DT, bool XF32>
__device__ __forceinline__ void fma8(const void* xs, int chunk, const uint4 va, const uint4 vb,
                                     float& aa, float& ab) {
  float xv[8], fa[8], fb[8];
  if constexpr (XF32) {
    const float4* p = reinterpret_cast<const float4*>(xs) + chunk * 2;
    const float4 x0 = p[0], x1 = p[1];
    xv[0] = x0.x; xv[1] = x0.y; xv[2] = x0.z; xv[3] = x0.w;
    xv[4] = x1.x; xv[5] = x1.y; xv[6] = x1.z; xv[7] = x1.w;
  } else {
    unpack8<DT>(reinterpret_cast<const uint4*>(xs)[chunk], xv);
  }
  unpack8<DT>(va, fa);
  unpack8<DT>(vb, fb);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    aa = fmaf(fa[e], xv[e], aa);
    ab = fmaf(fb[e], xv[e], ab);
  }
}

// Walk this wave's blocks [b0, b1) with `cur` = the already-issued first batch;
// part[(pl * NW + wave) * 2 + {0,1}] = this wave's partial dot products of pair pl.
template <int DT, bool XF32, int U, int NW, class Map>
__device__ __forceinline__ void walk(const Map& map, const void* xs, const Rng& r, Batch<U>& cur,
                                     float* part) {
  const int lane = otid() & 63, wave = __builtin_amdgcn_readfirstlane(otid() >> 6);
  if (r.b1 <= r.b0) return;
  float aa = 0.f, ab = 0.f;
  int pl_cur = r.b0 / r.bpp;
  for (int b = r.b0; b < r.b1; b += U) {
    Batch<U> nxt;
    if (b + U < r.b1) issue<U>(map, r.bpp, b + U, r.b1, nxt);
    int pl = b / r.bpp, kb = b - pl * r.bpp;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b + u < r.b1) {
        if (pl != pl_cur) {
          const float sa = wave_sum(aa), sb = wave_sum(ab);
          if (lane == 0) {
            part[(pl_cur * NW + wave) * 2] = sa;
            part[(pl_cur * NW + wave) * 2 + 1] = sb;
          }
          aa = ab = 0.f;
          pl_cur = pl;
        }
        fma8<DT, XF32>(xs, kb * 64 + lane, cur.a[u], cur.b[u], aa, ab);
      }
      if (++kb == r.bpp) { kb = 0; ++pl; }
    }
    cur = nxt;
  }
  const float sa = wave_sum(aa), sb = wave_sum(ab);
  if (lane == 0) {
    part[(pl_cur * NW + wave) * 2] = sa;
    part[(pl_cur * NW + wave) * 2 + 1] = sb;
  }
}

// Sum of the partials of local pair t over the waves whose block range touches it.
template <int NW>
__device__ __forceinline__ void pair_sum(const float* part, const Rng& r, int t, float& da,
                                         float& db) {
  const int tot = r.npl * r.bpp, lo = t * r.bpp, hi = lo + r.bpp;
  da = 0.f;
  db = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int b0 = w * tot / NW, b1 = (w + 1) * tot / NW;
    if (b0 < hi && b1 > lo && b1 > b0) {
      da += part[(t * NW + w) * 2];
      db += part[(t * NW + w) * 2 + 1];
    }
  }
}

// ---------------------------------------------------------------------------
// attention unit (kv head g, split s): core2-style wave-independent key blocks
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
__device__ __forceinline__ void attn_unit(const Args& a, const uint16_t* kcache, const uint16_t* vcache, const GOff& go, u64* gl, unsigned tag,
                          int g, int s, int ns, int kps, int pos, float* lds, Spin& sp) {
  constexpr int NT = NW * 64;
  constexpr int DS = HD / 32, NCH = HD / 8, KPL = NCH / 4;
  static_assert(NCH == 8 || NCH == 16, "hd 64 or 128");
  static_assert(NREP <= 16 && NREP <= NW, "GQA group");
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
  __syncthreads();
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
  __syncthreads();
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
    __syncthreads();  // LDS (st) reuse by the caller
    return;
  } else {
    // split 0: own partial -> LDS (p tiles are free), one wave per head merges
    float* own = lds;
    static_assert(NREP * (HD + 2) <= NW * (kKeys * 16 + 16), "own partial fits the p tiles");
    __syncthreads();
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
    if (wave < NREP) {
      constexpr int DPL = HD / 64;
      const int h = wave;
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
  __syncthreads();
  // publish the group's output: 2 x 16-bit per granule
  for (int i = tid; i < NOUT / 2; i += NT) {
    const unsigned w = (unsigned)ob[2 * i] | ((unsigned)ob[2 * i + 1] << 16);
    gst(att + i, tag, w);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// the persistent kernel
// ---------------------------------------------------------------------------
__device__ __forceinline__ int merger_wg(int g, int G, int nkv) {
  return g * (G / nkv) + (g & 7);
}

// Row maps: pair (local index pl) -> byte offsets of its two weight rows.
template <int HD> struct MapQKV {  // rows (slot hd + i, slot hd + i + hd/2) of wqkv
  __amdgpu_buffer_rsrc_t rs;
  int pbeg, K;
  __device__ __forceinline__ void offs(int pl, unsigned& oa, unsigned& ob) const {
    constexpr int half = HD / 2;
    const int p = pbeg + pl;
    const int slot = p / half;
    const unsigned ra = (unsigned)(slot * HD + (p - slot * half));
    oa = ra * (unsigned)K * 2u;
    ob = oa + (unsigned)(half * K * 2);
  }
};
struct MapRows2 {  // rows 2p, 2p + 1
  __amdgpu_buffer_rsrc_t rs;
  int pbeg, K;
  __device__ __forceinline__ void offs(int pl, unsigned& oa, unsigned& ob) const {
    oa = (unsigned)(2 * (pbeg + pl)) * (unsigned)K * 2u;
    ob = oa + (unsigned)K * 2u;
  }
};
struct MapGU {  // gate row j and up row j (I rows further)
  __amdgpu_buffer_rsrc_t rs;
  int pbeg, K;
  unsigned up;  // byte distance gate -> up
  __device__ __forceinline__ void offs(int pl, unsigned& oa, unsigned& ob) const {
    oa = (unsigned)(pbeg + pl) * (unsigned)K * 2u;
    ob = oa + up;
  }
};

// phase clock of this workgroup (s_memrealtime, 100 MHz, comparable across CUs):
// [wg][layer * kStampsPerLayer + k], then kernel start / end
#define MK_STAMP(idx)                                                                     \
  do {                                                                                    \
    if (a.stamps != nullptr && threadIdx.x == 0)                                          \
      a.stamps[(size_t)blockIdx.x * (a.L * kStampsPerLayer + 2) + (idx)] =                \
          __builtin_amdgcn_s_memrealtime();                                               \
  } while (0)

template <int DT, int NW, int U, int HD, int NREP>
__global__ __launch_bounds__(NW * 64) void mk_decode_kernel(Args a) {
  constexpr int NT = NW * 64;
  constexpr int half = HD / 2;
  constexpr int POLL = NW - 1;  // the poller wave (issues its own prefetch after polling)
  extern __shared__ float smem[];
  const int G = gridDim.x, wg = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const bool poller = wave == POLL;
  const int H = a.H, I = a.I, nh = a.nh, nkv = a.nkv, S = a.S;
  const int KO = nh * HD;
  // LDS: rawA[H] rawB[H] part[maxpl][NW][2] red[32] xs[...]
  const int maxpl = (I + G - 1) / G + 2;
  float* rawA = smem;
  float* rawB = rawA + H;
  float* part = rawB + H;
  float* red = part + maxpl * NW * 2;
  float* xs = red + 32;

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
  const int Pq = (nh + 2 * nkv) * half;
  const long long bq = (long long)Pq * 2 * H * 2, bo = (long long)H * KO * 2;
  const long long bgu = 2LL * I * H * 2, bd = (long long)H * I * 2;
  const unsigned gu_off = (unsigned)I * (unsigned)H * 2u;

  MK_STAMP(a.L * kStampsPerLayer);
  Batch<U> pre;
  {
    const CAKE_G Layer* ly = gp(a.layers);
    const Rng r = make_rng(Pq, G, wg, H, wave, NW, 1);
    issue<U>(MapQKV<HD>{rsrc(ly->wqkv, bq), r.pbeg, H}, r.bpp, r.b0, r.b1, pre);
  }

  for (int l = 0; l < a.L; ++l) {
    const int tid = otid();
    const CAKE_G Layer* ly = gp(a.layers + l);
    u64* gl = a.gran + (size_t)l * a.gstride;
    u64* sent = gl + go.sent;
    // ---------------- QKV + RoPE + KV write ----------------
    if (l > 0 && poller) {
      wait_sent(sent + kERes * kMaxG, G, tag, a, sp, 21);
      const Rng r = make_rng(Pq, G, wg, H, wave, NW, 1);
      issue<U>(MapQKV<HD>{rsrc(ly->wqkv, bq), r.pbeg, H}, r.bpp, r.b0, r.b1, pre);
    }
    __syncthreads();
    gather_norm<DT, NT, 16>(gl + go.res, l == 0 ? a.resid : nullptr, H, tag, ly->ln1, a.eps,
                            rawA, xs, red, a, sp, 1);
    __syncthreads();
    const int sb = l * kStampsPerLayer;
    MK_STAMP(sb + 0);
    {
      const Rng r = make_rng(Pq, G, wg, H, wave, NW, 1);
      walk<DT, true, U, NW>(MapQKV<HD>{rsrc(ly->wqkv, bq), r.pbeg, H}, xs, r, pre, part);
    }
    if (!is_attn && o_ip >= 0 && !poller) {
      const Rng r = make_rng(H / 2, G - nkv, o_ip, KO, wave, NW, 1);
      issue<U>(MapRows2{rsrc(ly->wo, bo), r.pbeg, KO}, r.bpp, r.b0, r.b1, pre);
    }
    __syncthreads();
    MK_STAMP(sb + 1);
    {
      const Rng r = make_rng(Pq, G, wg, H, wave, NW, 1);
      uint16_t* kc = ly->kc;
      uint16_t* vc = ly->vc;
      for (int t = tid; t < r.npl; t += NT) {
        float da, db;
        pair_sum<NW>(part, r, t, da, db);
        const int p = r.pbeg + t;
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
    }
    __syncthreads();
    if (tid == 0) gst(sent + kEQkv * kMaxG + wg, tag, 1u);
    MK_STAMP(sb + 2);
    // ---------------- attention ----------------
    if (is_attn) {
      if (poller) wait_sent(sent + kEQkv * kMaxG, G, tag, a, sp, 22);
      __syncthreads();
      attn_unit<DT, HD, NREP, NW>(a, ly->kc, ly->vc, go, gl, tag, my_g, my_s, ns, kps, pos, xs, sp);
      if (my_s == 0 && tid == 0) gst(sent + kEAtt * kMaxG + my_g, tag, 1u);
      // o_proj prefetch, unconditional in this block so the batch is not live across the
      // attention code (a merger's range is empty: every load is out of range, no traffic)
      const Rng r = make_rng(H / 2, G - nkv, o_ip, KO, wave, NW, 1);
      issue<U>(MapRows2{rsrc(ly->wo, bo), r.pbeg, KO}, r.bpp, r.b0, r.b1, pre);
    }
    if (is_merger && tid == 0) gst(sent + kEMid * kMaxG + wg, tag, 1u);  // no o_proj rows
    // ---------------- o_proj + residual ----------------
    if (o_ip >= 0) {
      if (poller) wait_sent(sent + kEAtt * kMaxG, nkv, tag, a, sp, 23);
      if (!is_attn && poller) {
        const Rng r = make_rng(H / 2, G - nkv, o_ip, KO, wave, NW, 1);
        issue<U>(MapRows2{rsrc(ly->wo, bo), r.pbeg, KO}, r.bpp, r.b0, r.b1, pre);
      }
      __syncthreads();
      gather_u32<NT>(gl + go.att, KO / 2, tag, reinterpret_cast<unsigned*>(xs), a, sp, 2);
      __syncthreads();
      MK_STAMP(sb + 3);
      const Rng r = make_rng(H / 2, G - nkv, o_ip, KO, wave, NW, 1);
      walk<DT, false, U, NW>(MapRows2{rsrc(ly->wo, bo), r.pbeg, KO}, xs, r, pre, part);
    }
    if (!poller) {
      const Rng r = make_rng(I, G, wg, H, wave, NW, 2);
      issue<U>(MapGU{rsrc(ly->wgu, bgu), r.pbeg, H, gu_off}, r.bpp, r.b0, r.b1, pre);
    }
    __syncthreads();
    MK_STAMP(sb + 4);
    if (o_ip >= 0) {
      const Rng r = make_rng(H / 2, G - nkv, o_ip, KO, wave, NW, 1);
      for (int t = tid; t < r.npl; t += NT) {
        float da, db;
        pair_sum<NW>(part, r, t, da, db);
        const int row = 2 * (r.pbeg + t);
        gst(gl + go.mid + row, tag, __float_as_uint(rawA[row] + da));
        gst(gl + go.mid + row + 1, tag, __float_as_uint(rawA[row + 1] + db));
      }
      __syncthreads();
      if (tid == 0) gst(sent + kEMid * kMaxG + wg, tag, 1u);
    }
    // ---------------- RMSNorm + gate/up + SwiGLU ----------------
    if (poller) {
      wait_sent(sent + kEMid * kMaxG, G, tag, a, sp, 24);
      const Rng r = make_rng(I, G, wg, H, wave, NW, 2);
      issue<U>(MapGU{rsrc(ly->wgu, bgu), r.pbeg, H, gu_off}, r.bpp, r.b0, r.b1, pre);
    }
    __syncthreads();
    gather_norm<DT, NT, 16>(gl + go.mid, nullptr, H, tag, ly->ln2, a.eps, rawB, xs, red, a, sp, 3);
    __syncthreads();
    MK_STAMP(sb + 5);
    {
      const Rng r = make_rng(I, G, wg, H, wave, NW, 2);
      walk<DT, true, U, NW>(MapGU{rsrc(ly->wgu, bgu), r.pbeg, H, gu_off}, xs, r, pre, part);
    }
    if (!poller) {
      const Rng r = make_rng(H / 2, G, wg, I, wave, NW, 1);
      issue<U>(MapRows2{rsrc(ly->wd, bd), r.pbeg, I}, r.bpp, r.b0, r.b1, pre);
    }
    __syncthreads();
    MK_STAMP(sb + 6);
    {
      const Rng r = make_rng(I, G, wg, H, wave, NW, 2);
      for (int t = tid; 2 * t < r.npl; t += NT) {
        float g0, u0, g1, u1;
        pair_sum<NW>(part, r, 2 * t, g0, u0);
        pair_sum<NW>(part, r, 2 * t + 1, g1, u1);
        const int j = r.pbeg + 2 * t;
        gst(gl + go.act + j / 2, tag, pack2(silu(g0) * u0, silu(g1) * u1, DT));
      }
    }
    __syncthreads();
    if (tid == 0) gst(sent + kEAct * kMaxG + wg, tag, 1u);
    // ---------------- down_proj + residual ----------------
    if (poller) {
      wait_sent(sent + kEAct * kMaxG, G, tag, a, sp, 25);
      const Rng r = make_rng(H / 2, G, wg, I, wave, NW, 1);
      issue<U>(MapRows2{rsrc(ly->wd, bd), r.pbeg, I}, r.bpp, r.b0, r.b1, pre);
    }
    __syncthreads();
    gather_u32<NT>(gl + go.act, I / 2, tag, reinterpret_cast<unsigned*>(xs), a, sp, 4);
    __syncthreads();
    MK_STAMP(sb + 7);
    {
      const Rng r = make_rng(H / 2, G, wg, I, wave, NW, 1);
      walk<DT, false, U, NW>(MapRows2{rsrc(ly->wd, bd), r.pbeg, I}, xs, r, pre, part);
    }
    if (l + 1 < a.L && !poller) {
      const CAKE_G Layer* ln = ly + 1;
      const Rng r = make_rng(Pq, G, wg, H, wave, NW, 1);
      issue<U>(MapQKV<HD>{rsrc(ln->wqkv, bq), r.pbeg, H}, r.bpp, r.b0, r.b1, pre);
    }
    __syncthreads();
    MK_STAMP(sb + 8);
    {
      const Rng r = make_rng(H / 2, G, wg, I, wave, NW, 1);
      u64* gn = gl + a.gstride;
      const bool last = l + 1 == a.L;
      for (int t = tid; t < r.npl; t += NT) {
        float da, db;
        pair_sum<NW>(part, r, t, da, db);
        const int row = 2 * (r.pbeg + t);
        const float va = rawB[row] + da, vb = rawB[row + 1] + db;
        if (!last) {
          gst(gn + go.res + row, tag, __float_as_uint(va));
          gst(gn + go.res + row + 1, tag, __float_as_uint(vb));
        } else {
          gpw(a.resid)[row] = va;
          gpw(a.resid)[row + 1] = vb;
        }
      }
      if (!last) {
        __syncthreads();
        if (tid == 0) gst(gn + go.sent + kERes * kMaxG + wg, tag, 1u);
      }
    }
    MK_STAMP(sb + 9);
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

// LDS bytes of one workgroup
inline size_t lds_bytes(int H, int I, int nh, int hd, int nrep, int G, int NW) {
  const int maxpl = (I + G - 1) / G + 2;
  size_t xs = (size_t)H;                       // f32 normalized row
  const size_t x16 = (size_t)((nh * hd > I ? nh * hd : I) + 1) / 2;  // 16-bit rows as floats
  if (x16 > xs) xs = x16;
  const size_t at = (size_t)NW * (kKeys * 16 + 16) + (size_t)NW * (32 + nrep * hd) +
                    (size_t)nrep * hd + hd + (size_t)nrep * hd / 2 + 16;
  if (at > xs) xs = at;
  return sizeof(float) * (2 * (size_t)H + (size_t)maxpl * NW * 2 + 32 + xs);
}

}  // namespace mk
}  // namespace cake

using namespace cake;

namespace {
constexpr int kMkNW = 8;
constexpr int kMkU = 8;
int g_mk_grid = 0;
unsigned long long* g_mk_stamps = nullptr;  // diagnostics only

int mk_grid() {
  if (g_mk_grid > 0) return g_mk_grid;
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  g_mk_grid = n;
  return n;
}

template <int DT, int HD, int NREP>
int mk_launch(const mk::Args& a, int G, size_t lds, hipStream_t st) {
  auto kern = mk::mk_decode_kernel<DT, kMkNW, kMkU, HD, NREP>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return (int)hipErrorInvalidValue;
    attr_set = true;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, kMkNW * 64, lds) !=
          hipSuccess ||
      per_cu < 1)
    return (int)hipErrorLaunchOutOfResources;
  hipLaunchKernelGGL(kern, dim3(G), dim3(kMkNW * 64), lds, st, a);
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

// Shapes the persistent decode supports (0 = supported).
CAKE_API int cake_mk_supported(int H, int I, int nh, int nkv, int hd) {
  const int G = mk_grid();
  if (G <= 0) return 1;
  if (H % mk::kBlk || I % mk::kBlk || (nh * hd) % mk::kBlk) return 2;
  if (hd != 128 || nkv <= 0 || nh % nkv) return 3;
  const int nrep = nh / nkv;
  if (nrep != 4 && nrep != 8) return 4;
  if (H > 16 * kMkNW * 64) return 5;
  if (G < nkv * (mk::kMaxSplitMk + 8) || G - nkv < 1 || G > mk::kMaxG) return 6;
  if (mk::lds_bytes(H, I, nh, hd, nrep, G, kMkNW) > 160 * 1024) return 7;
  if ((H / 2) < G || (nh + 2 * nkv) * hd / 2 < G) return 8;
  return 0;
}

// layers: device array of L mk::Layer (11 pointers each); gran: L * gstride words;
// ctl: 4 words; all zero-initialised before the first launch.
CAKE_API int cake_mk_decode(int dt, const void* layers, int L, int H, int I, int nh, int nkv,
                            int hd, int S, float eps, float scale, const float* inv_freq,
                            const int* pos, float* resid, void* gran, unsigned* ctl,
                            double timeout_s, hipStream_t st) {
  if (cake_mk_supported(H, I, nh, nkv, hd) != 0 || L <= 0 || S <= 0 || !layers || !gran || !ctl)
    return (int)hipErrorInvalidValue;
  const int G = mk_grid();
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
  a.timeout = (unsigned long long)(timeout_s * 1e8);
  a.stamps = g_mk_stamps;
  const int nrep = nh / nkv;
  const size_t lds = mk::lds_bytes(H, I, nh, hd, nrep, G, kMkNW);
  if (dt == kBF16) {
    return nrep == 4 ? mk_launch<kBF16, 128, 4>(a, G, lds, st) : mk_launch<kBF16, 128, 8>(a, G, lds, st);
  } else if (dt == kF16) {
    return nrep == 4 ? mk_launch<kF16, 128, 4>(a, G, lds, st) : mk_launch<kF16, 128, 8>(a, G, lds, st);
  }
  return (int)hipErrorInvalidValue;
}
