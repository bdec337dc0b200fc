// Ping-pong 256x256 MFMA GEMM (plan cfg 20): the large Llama prefill projections.
//
// Included by gemm_kernel.h (launch_gemm dispatches cfg 20 here); same GemmArgs, tile
// order, LDS image and epilogues as gemm_kernel.
//
// Why a second kernel: gemm_kernel's 8-wave 256x256 tile (cfg 5) interleaves every LDS
// read and LDS-DMA issue of a wave between that same wave's MFMAs; with two waves per
// SIMD both waves then compete for issue in every gap and the matrix pipe idles while
// one of them sits in a DMA issue (60-185 cycles each, MI355X_MICROARCH.md 'LDS-DMA
// piece').  Here the two waves of a SIMD take turns instead:
//
//   * 8 waves = 2 (M) x 4 (N), 128 x 64 outputs per wave (FM 8 x FN 4 16x16 tiles,
//     AGPR accumulators), 512 threads, 128 KB LDS (two 64 KB k-tile buffers), BK 64.
//   * A k-tile is 4 phases, one output quadrant (64 x 32) x K 64 = 16 MFMAs each, in
//     snake order Q(0,0) Q(0,1) Q(1,1) Q(1,0) so each phase re-uses one operand from
//     registers: the phases read A-lo + B-lo (12 ds_read_b128), B-hi (4), A-hi (8), -.
//   * Every phase: [LDS reads; 2 LDS-DMA issues; lgkmcnt(0)] barrier [16 MFMAs]
//     barrier.  Waves 4-7 run one barrier behind waves 0-3 (one extra s_barrier up
//     front), so between any two barriers one wave of each SIMD is in its MFMA cluster
//     while the other issues its loads: the matrix pipe has a wave to run at all times.
//   * Staging by read time, two k-tiles ahead where the buffer allows it: the four
//     128-row units of a k-tile (A-lo rows, B-lo rows, B-hi rows, A-hi rows) are each
//     re-staged right after the phase that last reads them (B-lo of tile t+1 in phase 1
//     of tile t; A-lo / B-hi / A-hi of tile t+2 in phases 2 / 3 / 4 of tile t), so a
//     DMA has 4-7 phases to land.  One counted wait per k-tile (vmcnt(6) in phase 4,
//     before its barrier) retires everything tile t+1 reads; the lgkmcnt(0) before each
//     phase's first barrier retires the reads a later phase's DMA overwrites.
//   * The k-loop always issues the same DMAs (past the end of K: the zeros page into a
//     consumed region), so the counted waits hold on every tile.
#pragma once

namespace cake {

constexpr int kPPCfg = 20;  // plan cfg id of this kernel (BM = BN = 256)

template <int DT, int EPI>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmArgs g) {
  constexpr int BM = 256, BN = 256, WTM = 128, WTN = 64, FM = 8, FN = 4;
  constexpr int BUF = (BM + BN) * 128;          // bytes per k-tile buffer (64 KB)
  constexpr int STG_LD = WTN + 4, STG = 16 * STG_LD * 4;
  static_assert(8 * STG <= 2 * BUF, "epilogue staging fits the operand buffers");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3;

  // ---- XCD-aware grouped tile order (as gemm_kernel) ---------------------
  const int ntiles = g.tiles_m * g.tiles_n;
  int id;
  {
    const int bid = blockIdx.x;
    const int q = ntiles / 8, r = ntiles % 8, x = bid % 8, i = bid / 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
  }
  constexpr int GROUP = 8;
  const int per_group = GROUP * g.tiles_n;
  const int first_m = (id / per_group) * GROUP;
  const int gm = min(GROUP, g.tiles_m - first_m);
  const int m0 = (first_m + (id % per_group) % gm) * BM;
  const int n0 = ((id % per_group) / gm) * BN;
  const int split = blockIdx.y;
  const int kb = split * g.kps, ke = min(g.K, kb + g.kps);
  const int nk = (ke - kb + kGBK - 1) / kGBK;

  // ---- staging units: 16 blocks of 8 LDS rows each; this wave issues blocks 2w, 2w+1
  // unit 0: A rows wr*128 + [0, 64)   unit 3: A rows wr*128 + [64, 128)
  // unit 1: B rows wc*64 + [0, 32)    unit 2: B rows wc*64 + [32, 64)   (B at row 256)
  auto unit_row = [](int u, int b) -> int {
    if (u == 0) return (b >> 3) * 128 + (b & 7) * 8;
    if (u == 3) return (b >> 3) * 128 + 64 + (b & 7) * 8;
    return 256 + (b >> 2) * 64 + (u == 2 ? 32 : 0) + (b & 3) * 8;
  };
  const uint16_t* src[4][2];
  int chunk[4][2];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = unit_row(u, wave * 2 + i) + (lane >> 3);  // this lane's LDS row
      chunk[u][i] = (lane & 7) ^ ((t >> 1) & 7);               // swizzled source chunk
      if (t < BM) {
        const int m = m0 + t;
        src[u][i] = m < g.M ? g.a + (size_t)m * g.lda : nullptr;
      } else {
        const int v = n0 + (t - BM);
        src[u][i] = v < g.Nv ? g.b + (size_t)wrow(g, v) * g.ldb : nullptr;
      }
    }
  auto stage = [&](auto UI, int tile, auto BI) __attribute__((always_inline)) {
    constexpr int u = decltype(UI)::value, bsel = decltype(BI)::value;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = kb + tile * kGBK + chunk[u][i] * 8;
      const uint16_t* p = (src[u][i] != nullptr && k < ke) ? src[u][i] + k : g.zeros;
      glds16(p, smem + bsel * BUF + unit_row(u, wave * 2 + i) * 128);
    }
  };
  using U0 = std::integral_constant<int, 0>;
  using U1 = std::integral_constant<int, 1>;
  using U2 = std::integral_constant<int, 2>;
  using U3 = std::integral_constant<int, 3>;

  // ---- fragment addresses (swizzled 16-byte slots, as gemm_kernel) -----------
  const int swz = (lane & 15) >> 1;
  const uint32_t lrow = (uint32_t)(lane & 15) * 128;
  const uint32_t off0 = (uint32_t)(((lane >> 4) ^ swz) * 16);       // k 0..31
  const uint32_t off1 = (uint32_t)(((4 + (lane >> 4)) ^ swz) * 16); // k 32..63
  const uint32_t lds0 = lds_off(smem);
  const uint32_t a_base = lds0 + (uint32_t)(wr * WTM) * 128 + lrow;
  const uint32_t b_base = lds0 + (uint32_t)(BM + wc * WTN) * 128 + lrow;

  cf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) azero(acc[i][j]);

  uint4 af[4][2], b0f[2][2], b1f[2][2];  // A quadrant rows, B columns lo / hi; [tile][k half]
  // A rows mh*64 + [0, 64) of buffer BSEL
  auto read_a = [&](auto BI, auto MH) __attribute__((always_inline)) {
    constexpr int o = decltype(MH)::value * 64 * 128;
    const uint32_t base = a_base + (decltype(BI)::value ? BUF : 0);
    static_for<0, 4>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      af[i][0] = ds_read16_off<o + i * 16 * 128>(base + off0);
      af[i][1] = ds_read16_off<o + i * 16 * 128>(base + off1);
    });
  };
  auto read_b = [&](auto BI, auto NH, uint4 (&bf)[2][2]) __attribute__((always_inline)) {
    constexpr int o = decltype(NH)::value * 32 * 128;
    const uint32_t base = b_base + (decltype(BI)::value ? BUF : 0);
    static_for<0, 2>([&](auto jj) __attribute__((always_inline)) {
      constexpr int j = decltype(jj)::value;
      bf[j][0] = ds_read16_off<o + j * 16 * 128>(base + off0);
      bf[j][1] = ds_read16_off<o + j * 16 * 128>(base + off1);
    });
  };
  // quadrant (mh, nh) x K 64: 16 MFMAs
  auto mma = [&](auto MH, auto NH, const uint4 (&bf)[2][2]) __attribute__((always_inline)) {
    constexpr int mh = decltype(MH)::value, nh = decltype(NH)::value;
    static_for<0, 8>([&](auto xi) __attribute__((always_inline)) {
      constexpr int x = decltype(xi)::value, i = x >> 1, j = x & 1;
      amfma_v<DT>(acc[mh * 4 + i][nh * 2 + j], af[i][0], bf[j][0]);
      amfma_v<DT>(acc[mh * 4 + i][nh * 2 + j], af[i][1], bf[j][1]);
    });
  };
  // the end of a phase's load section and its MFMA cluster between the two barriers
  auto sync_loads = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto end_mfma = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;

  // one k-tile from buffer B (0 / 1)
  auto ktile = [&](auto BI, int t) __attribute__((always_inline)) {
    using NB = std::integral_constant<int, 1 - decltype(BI)::value>;
    // phase 1: Q(0,0) -- A-lo, B-lo; stage B-lo of tile t+1 (other buffer)
    read_a(BI, Z{});
    read_b(BI, Z{}, b0f);
    stage(U1{}, t + 1, NB{});
    sync_loads();
    __builtin_amdgcn_s_setprio(1);
    mma(Z{}, Z{}, b0f);
    __builtin_amdgcn_s_setprio(0);
    end_mfma();
    // phase 2: Q(0,1) -- B-hi; stage A-lo of tile t+2 (this buffer: read in phase 1)
    read_b(BI, O{}, b1f);
    stage(U0{}, t + 2, BI);
    sync_loads();
    __builtin_amdgcn_s_setprio(1);
    mma(Z{}, O{}, b1f);
    __builtin_amdgcn_s_setprio(0);
    end_mfma();
    // phase 3: Q(1,1) -- A-hi; stage B-hi of tile t+2
    read_a(BI, O{});
    stage(U2{}, t + 2, BI);
    sync_loads();
    __builtin_amdgcn_s_setprio(1);
    mma(O{}, O{}, b1f);
    __builtin_amdgcn_s_setprio(0);
    end_mfma();
    // phase 4: Q(1,0) -- no reads; stage A-hi of tile t+2; retire tile t+1's DMAs
    stage(U3{}, t + 2, BI);
    __builtin_amdgcn_s_waitcnt(vm_wait(6));
    sync_loads();
    __builtin_amdgcn_s_setprio(1);
    mma(O{}, Z{}, b0f);
    __builtin_amdgcn_s_setprio(0);
    end_mfma();
  };

  // prologue: all of tile 0, tile 1 but its B-lo (phase 1 of tile 0 stages that)
  stage(U0{}, 0, Z{});
  stage(U1{}, 0, Z{});
  stage(U2{}, 0, Z{});
  stage(U3{}, 0, Z{});
  stage(U0{}, 1, O{});
  stage(U2{}, 1, O{});
  stage(U3{}, 1, O{});
  __builtin_amdgcn_s_waitcnt(vm_wait(6));
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  if (wr == 1) asm volatile("s_barrier" ::: "memory");  // waves 4-7: one barrier behind
  __builtin_amdgcn_sched_barrier(0);
  for (int t = 0; t < nk; t += 2) {
    ktile(Z{}, t);
    if (t + 1 < nk) ktile(O{}, t + 1);
  }
  if (wr == 0) asm volatile("s_barrier" ::: "memory");  // the matching barrier

  // ---- epilogue (as gemm_kernel) -----------------------------------------
#pragma unroll
  for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
  __builtin_amdgcn_s_waitcnt(vm_wait(0));
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float* stg = reinterpret_cast<float*>(smem + wave * STG);
  const int row_m0 = m0 + wr * WTM;
  const int vcol0 = n0 + wc * WTN;
  EpiOps<DT, EPI, FN> ops;
  ops.load_bias(g, vcol0, lane);
  ops.template load_res<0>(g, row_m0 + (lane >> 2), vcol0, lane);
  static_for<0, FM>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    if constexpr (i + 1 < FM)
      ops.template load_res<(i + 1) & 1>(g, row_m0 + (i + 1) * 16 + (lane >> 2), vcol0, lane);
    epi_strip<DT, EPI, FN, i & 1>(g, acc[i], stg, row_m0 + i * 16, vcol0, split, lane, ops);
  });
}

}  // namespace cake
