// MFMA GEMM for every T > 1 linear layer: y = x W^T (+ fused epilogue).
//
// Replaces the reference's candle Linear -> cuBLAS gemm for the Llama prefill
// projections (cake-core/src/models/llama3/attention.rs:49-60 q/k/v, :120 o;
// mlp.rs:14-18 gate/up/down) and every Stable Diffusion / CLIP linear
// (candle-transformers stable_diffusion attention/FF/proj layers reached from
// cake-core/src/models/sd/{unet,vae,clip}.rs), SURVEY K03 / K34-K36 / K40.
//
//   A = x [M][K] (activations, row stride lda), B = W [N][K] (HF weight layout,
//   row stride ldb): both operands are k-contiguous, so every MFMA fragment is
//   one 16-byte LDS read.  f32 accumulation on v_mfma_f32_16x16x32_{bf16,f16}.
//
// Structure (gfx950):
//   * Workgroup tile BM x BN x 64, 256 threads = WM x WN waves, per-wave tile
//     (BM/WM) x (BN/WN) as FM x FN 16x16 MFMA tiles.
//   * Operands staged global -> LDS by LDS-DMA (global_load_lds_dwordx4, no
//     VGPR round trip) into two buffers; the DMA of k-step t+2 is in flight
//     while step t computes.  The 128-byte rows are XOR-swizzled in 16-byte
//     slots (slot ^= (row >> 1) & 7) on the SOURCE address (the DMA writes
//     lane-linear), which makes the fragment ds_read_b128 conflict-free.
//   * Fragment reads are inline-asm ds_read_b128 with an explicit lgkmcnt wait:
//     hipcc cannot see them, so it does not drain the in-flight DMA (vmcnt(0))
//     in front of them, which it does for compiler-visible LDS reads of a
//     buffer a DMA may write.  Waits on the DMA are counted (vmcnt(N)) and the
//     barriers are raw s_barrier (MI355X guide: "Pipelining across barriers").
//   * XCD-aware grouped tile order: round-robin block -> XCD dealing is undone
//     so each XCD's blocks cover a compact group of tiles (shared A rows / W
//     rows hit that XCD's L2).
//   * Split-K (grid.y) for grids smaller than the chip: f32 partial slabs and
//     a second kernel that reduces them and applies the epilogue.
//   * Epilogues (C staged through LDS per 16-row strip, 16-32 byte vector
//     stores): plain store (+bias), f32 residual accumulate (Llama o/down
//     proj: resid += y), 16-bit add (+bias, +residual: SD proj_out), SwiGLU
//     (silu(gate) * up from the fused gate|up weight) and GEGLU
//     (h * gelu_tanh(gate), SD FeedForward).  For the gated forms the B rows
//     are read in a virtual order that interleaves 16-row blocks of the two
//     halves, so gate and up of one feature land in the same lane.
#include "gemm_kernel.h"

namespace cake {
// the launchers are instantiated in gemm_inst_{bf16,f16}_{a,b}.hip
#define CAKE_GEMM_EXTERN(DT, E) extern template int launch_gemm<DT, E>(int, dim3, hipStream_t, const GemmArgs&);
#define CAKE_GEMM_EXTERN_ALL(DT) CAKE_GEMM_EXTERN(DT, kEpiStore) CAKE_GEMM_EXTERN(DT, kEpiResid32) \
  CAKE_GEMM_EXTERN(DT, kEpiAdd16) CAKE_GEMM_EXTERN(DT, kEpiSwiglu) CAKE_GEMM_EXTERN(DT, kEpiGeglu) \
  CAKE_GEMM_EXTERN(DT, kEpiPartial) CAKE_GEMM_EXTERN(DT, kEpiStore32) CAKE_GEMM_EXTERN(DT, kEpiSilu)
CAKE_GEMM_EXTERN_ALL(kBF16)
CAKE_GEMM_EXTERN_ALL(kF16)
#undef CAKE_GEMM_EXTERN_ALL
#undef CAKE_GEMM_EXTERN
}  // namespace cake

using namespace cake;

// split-K pair tickets of gemm_4w (zero at load; every pair leaves its tile's zero)
__device__ unsigned g_pair_tick[2 * kPairTiles];

static unsigned* pair_ticks() {
  static unsigned* p = nullptr;
  if (!p) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_pair_tick)) == hipSuccess) p = static_cast<unsigned*>(a);
  }
  return p;
}

static inline void cfg_dims(int cfg, int& bm, int& bn) {
  if (cfg >= k4WCfg + k4WSched && cfg <= k4WCfg128 + k4WSched) cfg -= k4WSched;  // three-barrier twins
  if (cfg == kPPCfg || cfg == kRSCfg || cfg == k4WCfg) { bm = bn = 256; return; }
  if (cfg == k4WCfg192) { bm = 256; bn = 192; return; }
  if (cfg == k4WCfg128) { bm = 128; bn = 256; return; }
#define X(id, BM, BN, WM, WN, NS, PR) if (cfg == id) { bm = BM; bn = BN; return; }
  CAKE_GEMM_CFGS(X)
#undef X
  bm = bn = 0;
}

CAKE_API int cake_gemm_tile(int cfg, int* bm, int* bn) {
  cfg_dims(cfg, *bm, *bn);
  return *bm > 0 ? 0 : (int)hipErrorInvalidValue;
}

// the gated epilogues pair 16-column gate / up blocks inside one wave: 32-column multiples
template <int DT>
static int dispatch_epi(int epi, int cfg, dim3 grid, hipStream_t st, const GemmArgs& g) {
  switch (epi) {
    case kEpiStore: return launch_gemm<DT, kEpiStore>(cfg, grid, st, g);
    case kEpiResid32: return launch_gemm<DT, kEpiResid32>(cfg, grid, st, g);
    case kEpiAdd16: return launch_gemm<DT, kEpiAdd16>(cfg, grid, st, g);
    case kEpiSwiglu: return launch_gemm<DT, kEpiSwiglu>(cfg, grid, st, g);
    case kEpiGeglu: return launch_gemm<DT, kEpiGeglu>(cfg, grid, st, g);
    case kEpiPartial: return launch_gemm<DT, kEpiPartial>(cfg, grid, st, g);
    case kEpiStore32: return launch_gemm<DT, kEpiStore32>(cfg, grid, st, g);
    case kEpiSilu: return launch_gemm<DT, kEpiSilu>(cfg, grid, st, g);
  }
  return (int)hipErrorInvalidValue;
}

template <int DT>
static int dispatch_finalize(int epi, dim3 grid, hipStream_t st, const GemmArgs& g, int splits) {
  switch (epi) {
#define F(E) case E: hipLaunchKernelGGL((gemm_splitk_finalize<DT, E>), grid, dim3(256), 0, st, g, splits); break;
    F(kEpiStore) F(kEpiResid32) F(kEpiAdd16) F(kEpiSwiglu) F(kEpiGeglu) F(kEpiStore32)
    F(kEpiSilu)
#undef F
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// Split plan of one call: the k split actually run (whole 64-element steps per split) and,
// for a four-wave tile at splits 2, the in-kernel pair's tiles (0: the slab + finalize
// form).  cake_gemm and cake_gemm_ws_floats both decide through this one function, so a
// workspace sized by the query always covers the launch.
struct SplitPlan {
  int splits, kps, bm, bn, ntiles, npair;
};
static SplitPlan split_plan(int cfg, int splits, int M, long long Nv, int K) {
  SplitPlan p{};
  cfg_dims(cfg, p.bm, p.bn);
  int kps = (K + splits - 1) / splits;
  kps = (kps + kGBK - 1) / kGBK * kGBK;
  p.kps = kps;
  p.splits = (K + kps - 1) / kps;
  if (p.bm == 0) return p;
  p.ntiles = (int)(((M + p.bm - 1) / p.bm) * ((Nv + p.bn - 1) / p.bn));
  const int npair = p.ntiles <= 256 ? p.ntiles : p.ntiles % 256;
  if (four_wave_cfg(cfg) && p.splits == 2 && npair > 0 &&
      npair <= 128 + (p.ntiles <= 256 ? 128 : 0) && p.ntiles <= kPairTiles &&
      (long long)npair * p.bm * p.bn <= 2LL * M * Nv && pair_ticks())
    p.npair = npair;
  return p;
}

// f32 workspace (elements) a cake_gemm call with these arguments needs: the pair's slabs
// (npair x BM x BN) or splits x M x Nv partial rows, 0 when it runs unsplit
CAKE_API long long cake_gemm_ws_floats(int cfg, int splits, int M, int N, int K, int gated) {
  if (splits < 1 || M <= 0 || N <= 0 || K <= 0) return 0;
  const long long Nv = gated ? 2LL * N : N;
  const SplitPlan p = split_plan(cfg, splits, M, Nv, K);
  if (p.npair > 0) return (long long)p.npair * p.bm * p.bn;
  return p.splits > 1 ? (long long)p.splits * M * Nv : 0;
}

// y = epilogue(x W^T).  N = output features (gated: W has 2N rows, gate rows
// [0, N), up/gate-2 rows [N, 2N)).  splits > 1 needs ws = splits * M * Nv f32.
// Requirements (host-checked in ops/gemm.py): K % 8 == 0, lda/ldb % 8 == 0,
// 16-byte aligned operand bases, gated => N % 16 == 0.
CAKE_API int cake_gemm(int dt, int epi, int cfg, int splits, const void* a, long long lda,
                       const void* b, long long ldb, void* c, long long ldc, const void* bias,
                       void* resid, long long ldr, float* ws, const void* zeros, int M, int N,
                       int K, hipStream_t st) {
  int act = 0;
  if (epi == 8 || epi == 9) {  // quick_gelu / GELU: the activation epilogue, other act
    act = epi - 7;
    epi = kEpiSilu;
  }
  int bm, bn;
  cfg_dims(cfg, bm, bn);
  if (bm == 0 || M <= 0 || N <= 0 || K <= 0 || K % 8 || lda % 8 || ldb % 8 || splits < 1)
    return (int)hipErrorInvalidValue;
  const bool gated = (epi == kEpiSwiglu || epi == kEpiGeglu);
  if (gated && N % 16) return (int)hipErrorInvalidValue;
  const bool four = four_wave_cfg(cfg);
  if (cfg == kRSCfg || four) {  // whole 64-element k steps; 31-bit offsets
    const long long wrows = gated ? 2LL * N : N;
    if (K % kGBK || ((long long)(M - 1) * lda + K) * 2 >= 0x7fffffffLL ||
        ((wrows - 1) * ldb + K) * 2 >= 0x7fffffffLL)
      return (int)hipErrorInvalidValue;
  }
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = (uint16_t*)c;
  g.bias = (const uint16_t*)bias;
  g.r32 = (epi == kEpiResid32 || epi == kEpiStore32) ? (float*)resid : nullptr;
  g.r16 = (epi == kEpiAdd16) ? (const uint16_t*)resid : nullptr;
  g.ws = ws; g.zeros = (const uint16_t*)zeros;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldr = ldr;
  g.M = M; g.N = N; g.K = K;
  g.gated = gated ? 1 : 0;
  g.act = act;
  g.half = N;
  g.Nv = gated ? 2 * N : N;
  g.tiles_m = (M + bm - 1) / bm;
  g.tiles_n = (g.Nv + bn - 1) / bn;
  const SplitPlan sp = split_plan(cfg, splits, M, g.Nv, K);
  splits = sp.splits;
  g.kps = sp.kps;
  const dim3 grid(g.tiles_m * g.tiles_n, splits);
  // splits == 2 on a four-wave tile: the tiles past the last whole wave (all of them when
  // there are at most 256) run as in-kernel k-half pairs, the rest whole; one slab per
  // paired tile in ws (cake_gemm_ws_floats), no finalize launch
  const int ntiles = g.tiles_m * g.tiles_n;
  const int npair = sp.npair;
  if (npair > 0 && ws != nullptr) {
    g.pair = 1;
    g.tick = pair_ticks();
    g.dp_tiles = ntiles - npair;
    const dim3 pgrid(g.dp_tiles + 2 * npair, 1);
    return (dt == kBF16) ? dispatch_epi<kBF16>(epi, cfg, pgrid, st, g)
           : (dt == kF16) ? dispatch_epi<kF16>(epi, cfg, pgrid, st, g)
                          : (int)hipErrorInvalidValue;
  }
  const int kernel_epi = splits > 1 ? (int)kEpiPartial : epi;
  if (splits > 1 && ws == nullptr) return (int)hipErrorInvalidValue;
  int rc = (dt == kBF16) ? dispatch_epi<kBF16>(kernel_epi, cfg, grid, st, g)
         : (dt == kF16) ? dispatch_epi<kF16>(kernel_epi, cfg, grid, st, g)
                        : (int)hipErrorInvalidValue;
  if (rc != 0 || splits == 1) return rc;
  const dim3 fgrid((N + 1023) / 1024, M);
  return (dt == kBF16) ? dispatch_finalize<kBF16>(epi, fgrid, st, g, splits)
                       : dispatch_finalize<kF16>(epi, fgrid, st, g, splits);
}
