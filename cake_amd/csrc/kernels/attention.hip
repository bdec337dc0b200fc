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
//     workgroup streams its key range, computes a local softmax and P·V in f32,
//     and the (max, sum, o[hd]) partials are merged inside the same launch —
//     core 2 (default, attn_core2.h): 16-key blocks per wave, one split up to 320
//     keys, else ~16 splits whose partials go out as epoch-tagged granules that
//     split 0 polls and merges; core 1 (attn_core.h): 64-key LDS chunks, the
//     last-arriving split merges behind a ticket.
//   * Prefill attention is the MFMA flash kernel (flash_attn.hip).
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "attn_core.h"
#include "attn_core2.h"

namespace cake {

// Grid (nkv, maxsplit): see attn_core.h for the split / chunk / combine scheme.
static int g_attn_min_keys = 64;  // min keys per split (tunable)
// core 2: number of splits aimed at past target * min_keys keys: fewer, longer splits
// trade loop time for a cheaper ticket + merge tail (16 splits: 8B decode +3.4 % tok/s at
// 2048 keys, +5.7 % at 4000 vs 64; profiles/r3_decode_ab.jsonl); tunable
static int g_attn_target = 16;
// core 2: live lengths up to this many keys run as ONE split per kv head — its merge
// tail (partials out, polled back in: ~6.5k cycles, profiles/r3_attn_stamps_granule_v2.jsonl)
// costs what ~240 more keys of one split's loop cost (~27 cycles per key)
static int g_attn_single = 320;
static int g_attn_drop_partials = 0;  // test hook (cake_attn_debug_drop_partials)
// core 2: key blocks per wave in flight (attn2_decode_block PFD); 0 = by the launch's
// split cap: 1 for grids of <= 8 splits per kv head (the graph bucket of short contexts:
// 5.47 vs 5.96 us per 8B layer at 33-177 keys, the deeper prefetch's larger code costs
// more than it saves), 2 above (8B decode at 2048 keys +0.7 % tok/s;
// profiles/r4_decode_attn_prefetch.md); tunable
static int g_attn_prefetch = 0;

template <int DT, int HD, int NREP>
__global__ __launch_bounds__(AttnGeom<NREP>::NT) void attn_decode_kernel(AttnDecArgs a) {
  // one LDS array (LDS-DMA pipelines need it: MI355X guide, GEMM item 4a)
  __shared__ __attribute__((aligned(16))) uint16_t smem[attn_smem_elems<HD, NREP>()];
  attn_decode_block<DT, HD, NREP>(a, blockIdx.x, blockIdx.y, smem);
}

template <int DT, int HD, int NREP, int PFD>
__global__ __launch_bounds__(AttnGeom2<NREP>::NT) void attn2_decode_kernel(AttnDecArgs a) {
  __shared__ __attribute__((aligned(16)))
      float lds[attn2_smem_floats<HD, NREP, AttnGeom2<NREP>::NW>()];
  attn2_decode_block<DT, HD, NREP, false, AttnGeom2<NREP>::NW, PFD>(a, blockIdx.x, blockIdx.y,
                                                                    lds, gridDim.x);
}

// Head-parallel short-context decode: one workgroup per QUERY head (grid nh), NW waves
// over the key blocks, the whole context as one split.  Against the per-kv-head launch
// (nkv workgroups, each carrying its group's nrep heads) the same keys are read nrep
// times (from L2), but P.V and the end merge carry one head instead of nrep and 4x more
// workgroups issue the loads.  Engines launch it for live lengths up to g_attn_heads_max.
template <int DT, int HD, int NW, int PFD>
__global__ __launch_bounds__(64 * NW) void attn_head_kernel(AttnDecArgs a, int nrep) {
  __shared__ __attribute__((aligned(16))) float lds[attn2_smem_floats<HD, 1, NW>()];
  const int h = blockIdx.x;
  attn2_decode_block<DT, HD, 1, false, NW, PFD, NoHook, true>(a, h, 0, lds, gridDim.x, NoHook(),
                                                             h / nrep);
}

}  // namespace cake

using namespace cake;

// 1 = LDS-staged chunk core (attn_core.h), 2 = wave-stream MFMA core (attn_core2.h).
// Core 2 is the default: equal at short context, 2 % more tok/s at a 2048-token one
// (profiles/r3_decode_ab.jsonl).
static int g_attn_impl = 2;
CAKE_API int cake_attn_set_impl(int impl) {
  if (impl != 1 && impl != 2) return (int)hipErrorInvalidValue;
  g_attn_impl = impl;
  return 0;
}

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

// Launch-time cap on the splits per kv head (0 = none): a graph captured for short
// live lengths launches only the workgroups those lengths can use (the idle ones of
// a max_seq-sized grid cost ~3.7 us per layer at 4096; the kernel stays correct
// for any cap — fewer, longer splits).
static int g_attn_split_cap = 0;
static unsigned long long* g_attn_stamps = nullptr;  // diagnostics only
CAKE_API int cake_attn_set_stamps(void* p) {
  g_attn_stamps = (unsigned long long*)p;
  return 0;
}
CAKE_API int cake_attn_set_split_cap(int cap) {
  if (cap < 0 || cap > kMaxSplit) return (int)hipErrorInvalidValue;
  g_attn_split_cap = cap;
  return 0;
}

CAKE_API int cake_attn_set_target_splits(int target) {
  if (target < 1 || target > kMaxSplit) return (int)hipErrorInvalidValue;
  g_attn_target = target;
  return 0;
}

CAKE_API int cake_attn_set_prefetch(int depth) {
  if (depth < 0 || depth > 2) return (int)hipErrorInvalidValue;
  g_attn_prefetch = depth;
  return 0;
}

CAKE_API int cake_attn_set_single_max(int keys) {
  if (keys < 0) return (int)hipErrorInvalidValue;
  g_attn_single = keys;
  return 0;
}

// Test hook: core 2's splits >= 1 skip publishing their partials, so split 0's merge
// runs into its poll bound and must raise the error word (tests/test_kernels_gpu.py).
CAKE_API int cake_attn_debug_drop_partials(int on) {
  g_attn_drop_partials = on != 0;
  return 0;
}

// Host mirror of the device split policy (attn2_splits / core 1's chunk rule) for a live
// length Tk under the current settings: the native engine picks position-bucket graphs
// with it (as ops.hip.attn_splits does for Python).
CAKE_API int cake_attn_splits(int Tk) {
  if (Tk < 1) Tk = 1;
  if (g_attn_impl == 2) {
    int ns, kps;
    if (Tk <= g_attn_single) return 1;
    int keys = (Tk + g_attn_target - 1) / g_attn_target;
    keys = (keys + 15) / 16 * 16;
    if (keys < g_attn_min_keys) keys = g_attn_min_keys;
    ns = (Tk + keys - 1) / keys;
    if (ns > kMaxSplit) ns = kMaxSplit;
    kps = (Tk + ns - 1) / ns;
    kps = (kps + 15) / 16 * 16;
    return (Tk + kps - 1) / kps;
  }
  int keys = g_attn_min_keys;
  if (Tk > 1024 && keys < 128) keys = 128;
  if (keys < (Tk + 63) / 64) keys = (Tk + 63) / 64;
  return (Tk + keys - 1) / keys;
}

CAKE_API int cake_attn_max_split(int S) { return S > 0 ? attn_max_split(S) : 0; }

CAKE_API int cake_attn_set_min_keys(int min_keys) {
  if (min_keys < kChunk || min_keys % kChunk) return (int)hipErrorInvalidValue;
  g_attn_min_keys = min_keys;
  return 0;
}

// Core 2's split 0 spins on the partials of the other splits of its head, so every
// workgroup of the grid must be resident at once.  A grid larger than the empty device can
// hold (70B: 8 KV heads x 64 splits = 512 workgroups at one per CU) is launched with fewer
// splits — the device-side split policy reads its cap from the launch (maxsplit), so each
// split covers more keys and the merge stays exact — and only a device that cannot hold
// even one split per KV head runs core 1's last-arriver merge.  The occupancy query is
// made once per kernel (a small table keyed by the kernel's address) and a trimmed grid is
// reported once.
template <class K>
static long long resident_blocks(K kern, int threads) {
  static std::mutex mu;
  static int cus = 0;
  static std::vector<std::pair<const void*, int>> per_cu_of;
  std::lock_guard<std::mutex> g(mu);
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
  }
  int per_cu = -1;
  for (const auto& e : per_cu_of)
    if (e.first == (const void*)kern) per_cu = e.second;
  if (per_cu < 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, threads, 0) !=
        hipSuccess)
      return 0;
    per_cu_of.push_back({(const void*)kern, per_cu});
  }
  return (long long)per_cu * cus;
}

// the splits of a core-2 grid of `heads` x `splits` workgroups that fit the device at once
// (0: not even one per head)
template <class K>
static int resident_splits(K kern, int threads, int heads, int splits) {
  static bool warned = false;
  const long long cap = resident_blocks(kern, threads);
  if (cap < heads) return 0;
  if ((long long)heads * splits <= cap) return splits;
  const int fit = (int)(cap / heads);
  // the grid is trimmed to what fits (core 2's splits walk more keys each); logged on request
  if (!warned && std::getenv("CAKE_ATTN_LOG") != nullptr) {
    warned = true;
    std::fprintf(stderr, "[cake] decode attention: %d x %d workgroups trimmed to residency "
                 "(%lld): core 2 with %d splits per KV head\n", heads, splits, cap, fit);
  }
  return fit;
}

template <int DT, int HD>
static int launch_decode(int n_rep, dim3 grid, hipStream_t st, const AttnDecArgs& a) {
#define CAKE_DEC2(NR, PF)                                                                     \
  if (const int fit = resident_splits(attn2_decode_kernel<DT, HD, NR, PF>, AttnGeom2<NR>::NT,  \
                                      (int)grid.x, (int)grid.y)) {                            \
    AttnDecArgs a2 = a;                                                                       \
    a2.maxsplit = fit;                                                                        \
    hipLaunchKernelGGL((attn2_decode_kernel<DT, HD, NR, PF>), dim3(grid.x, fit),              \
                       dim3(AttnGeom2<NR>::NT), 0, st, a2);                                   \
  } else                                                                                      \
    hipLaunchKernelGGL((attn_decode_kernel<DT, HD, NR>), grid, dim3(AttnGeom<NR>::NT), 0, st, a)
#define CAKE_DEC(NR)                                                                          \
  if (g_attn_impl == 2 && (g_attn_prefetch == 2 || (g_attn_prefetch == 0 && grid.y > 8)))    \
    { CAKE_DEC2(NR, 2); }                                                                     \
  else if (g_attn_impl == 2) { CAKE_DEC2(NR, 1); }                                            \
  else                                                                                        \
    hipLaunchKernelGGL((attn_decode_kernel<DT, HD, NR>), grid, dim3(AttnGeom<NR>::NT), 0, st, a)
  switch (n_rep) {
    case 1: CAKE_DEC(1); break;
    case 2: CAKE_DEC(2); break;
    case 4: CAKE_DEC(4); break;
    case 8: CAKE_DEC(8); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef CAKE_DEC
#undef CAKE_DEC2
  return (int)hipGetLastError();
}

CAKE_API int cake_attn_decode(int dt, const float* q, const void* kc, const void* vc,
                              const int* pos, int S, int nh, int nkv, int hd, float scale,
                              float* part, unsigned int* tickets, void* out, hipStream_t st) {
  if (nkv <= 0 || nh % nkv || S <= 0) return (int)hipErrorInvalidValue;
  const int ms = attn_max_split(S);
  const int splits = g_attn_split_cap > 0 && g_attn_split_cap < ms ? g_attn_split_cap : ms;
  const dim3 grid(nkv, splits);
  const AttnDecArgs a{q, (const uint16_t*)kc, (const uint16_t*)vc, pos, S,
                      scale * 1.4426950408889634f, part, tickets, (uint16_t*)out,
                      g_attn_min_keys, splits, g_attn_stamps, g_attn_target,
                      g_attn_single, g_attn_drop_partials};
  DISPATCH_DT_HD(dt, hd, return (launch_decode<DT, HD>(nh / nkv, grid, st, a)));
  return (int)hipErrorInvalidValue;
}

// ---- head-parallel short-context launch (attn_head_kernel)
static int g_attn_heads_max = 0;  // live lengths <= this take it (0: off)
static int g_attn_head_waves = 2;
static int g_attn_head_pfd = 2;  // key blocks per wave in flight (2 or 4)

CAKE_API int cake_attn_set_head_prefetch(int pfd) {
  if (pfd != 2 && pfd != 4) return (int)hipErrorInvalidValue;
  g_attn_head_pfd = pfd;
  return 0;
}

CAKE_API int cake_attn_set_heads(int max_keys, int waves) {
  if (max_keys < 0 || (waves != 1 && waves != 2 && waves != 4 && waves != 8 && waves != 16))
    return (int)hipErrorInvalidValue;
  g_attn_heads_max = max_keys;
  g_attn_head_waves = waves;
  return 0;
}

CAKE_API int cake_attn_heads_max() { return g_attn_heads_max; }

// out [nh][hd] (16-bit) for the position *pos (live length *pos + 1); any length is
// correct (one workgroup walks every key), short ones are what it is fast for.
CAKE_API int cake_attn_decode_heads(int dt, const float* q, const void* kc, const void* vc,
                                    const int* pos, int S, int nh, int nkv, int hd, float scale,
                                    void* out, hipStream_t st) {
  if (nkv <= 0 || nh % nkv || S <= 0) return (int)hipErrorInvalidValue;
  const AttnDecArgs a{q, (const uint16_t*)kc, (const uint16_t*)vc, pos, S,
                      scale * 1.4426950408889634f, nullptr, nullptr, (uint16_t*)out,
                      g_attn_min_keys, 1, nullptr, g_attn_target, S, 0};
  const int nrep = nh / nkv;
#define CAKE_HEADS(NW)                                                                         \
  do {                                                                                         \
    if (g_attn_head_pfd == 4)                                                                  \
      hipLaunchKernelGGL((attn_head_kernel<DT, HD, NW, 4>), dim3(nh), dim3(64 * NW), 0, st, a, \
                         nrep);                                                                \
    else                                                                                       \
      hipLaunchKernelGGL((attn_head_kernel<DT, HD, NW, 2>), dim3(nh), dim3(64 * NW), 0, st, a, \
                         nrep);                                                                \
  } while (0)
  DISPATCH_DT_HD(dt, hd, {
    if (g_attn_head_waves == 1) CAKE_HEADS(1);
    else if (g_attn_head_waves == 2) CAKE_HEADS(2);
    else if (g_attn_head_waves == 4) CAKE_HEADS(4);
    else if (g_attn_head_waves == 8) CAKE_HEADS(8);
    else CAKE_HEADS(16);
    return (int)hipGetLastError();
  });
#undef CAKE_HEADS
  return (int)hipErrorInvalidValue;
}
