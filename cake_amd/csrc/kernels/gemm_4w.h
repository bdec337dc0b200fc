// Four-wave 256x256 MFMA GEMM (plan cfg 22): the large Llama prefill projections.
//
// Included by gemm_kernel.h (launch_gemm dispatches cfg 22 here); same GemmArgs, tile
// order, swizzled LDS image, fragment reads, interleaved schedule and epilogues as
// gemm_kernel's IL path.
//
// The shape of the winning library kernel on this chip (hipBLASLt's 256x256x64 tile,
// profiles/r6_gemm_pmc_8192.txt): one wave per SIMD, 128 x 128 outputs per wave, LDS-DMA
// staging, 32 fragment reads per k-step.  gemm_kernel's 4-wave form of the same tile
// measured 0.5x (round 2) because each of its 16 DMA issues per wave and k-step
// recomputed a 64-bit source pointer and a zeros-page select in VALU; here a DMA is one
// buffer_load_dwordx4 ... lds:
//   * one per-lane byte offset VGPR per operand (the lane's row in its 32-row group and
//     its swizzled 16-byte chunk), the group's row offset and the k step in the scalar
//     soffset, the LDS destination in M0;
//   * rows past the matrix read through the descriptor's range check (zeros, no fault),
//     so no per-issue select and no zeros page; gated (SwiGLU / GEGLU) weights keep a
//     constant row stride per group (16 gate + 16 up rows), so the same form covers them.
//   Needs K and the split's k range in whole 64-element steps and operands under 2 GB
//   (host-checked).
#pragma once

namespace cake {

constexpr int k4WCfg = 22;     // plan cfg id of the 256 x 256 tile
constexpr int k4WCfg192 = 23;  // 256 x 192 (8B q|k|v: 6144 = 32 x 192 columns, 256 tiles at
                               // 2048 tokens instead of 192)
constexpr int k4WCfg128 = 24;  // 128 x 256 (8B o / down at 2048 tokens: 256 tiles, not 128)
constexpr int k4WDeep = 3;     // cfg + 3: the same tiles with DEEP staging (25, 26, 27)
inline bool four_wave_cfg(int cfg) { return cfg >= k4WCfg && cfg <= k4WCfg128 + k4WDeep; }

// DEEP (cfg 25-27): the LDS image split by k half, so each half of step t+2 is staged as
// soon as the half of step t it replaces has been read (kk0 half during the first MFMA
// half of step t, kk1 half during the second), two barriers per step with vmcnt(2 x the
// half's DMAs): a DMA has ~1.5 steps to land instead of ~0.5-1.  Half-rows are 64 bytes
// (four 16-byte slots); slot s of row r holds chunk s ^ F[(r >> 2) & 3], F = {0, 2, 3, 1},
// which spreads every ds_read_b128 lane group over 16 distinct bank quads.
template <int DT, int EPI, int BM, int BN, bool DEEP = false>
__global__ __launch_bounds__(256) void gemm_4w_kernel(GemmArgs g) {
  static_assert((BM == 256 && (BN == 256 || BN == 192)) || (BM == 128 && BN == 256),
                "four-wave tile shapes");
  constexpr int WTM = BM / 2, WTN = BN / 2, FM = WTM / 16, FN = WTN / 16;
  constexpr int BUF = (BM + BN) * 128;  // 64 / 56 / 48 KB per k-step buffer
  constexpr int IPW = (BM + BN) / 32;   // DMA wave-instructions per wave per k-step
  constexpr int NA = BM / 32;           // of which A
  static_assert(IPW == FM + FN, "the second half alternates one DMA with one fragment read");
  constexpr int STG_LD = WTN + 4, STG = 16 * STG_LD * 4;
  static_assert(4 * STG <= 2 * BUF - 16, "epilogue staging fits the operand buffers");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  // ---- XCD-aware grouped tile order (as gemm_kernel) ---------------------
  // Paired split-K (g.pair): workgroups [0, dp_tiles) run whole tiles, the rest run the
  // remaining tiles as pairs of k halves (2 workgroups per tile) — the last partial wave
  // of a grid at half length instead of full (8B gate|up at 2048 tokens: 896 tiles =
  // 3 full waves + 128 paired tiles), or every tile paired when there are too few.
  const int ntiles = g.tiles_m * g.tiles_n;
  int id, split = blockIdx.y;
  {
    const int bid = blockIdx.x;
    const int dp = g.pair ? g.dp_tiles : ntiles;
    if (bid < dp) {
      const int q = dp / 8, r = dp % 8, x = bid % 8, i = bid / 8;
      id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
      if (g.pair) split = -1;  // a whole tile
    } else {
      id = dp + (bid - dp) / 2;
      split = (bid - dp) & 1;
    }
  }
  constexpr int GROUP = 8;
  const int per_group = GROUP * g.tiles_n;
  const int first_m = (id / per_group) * GROUP;
  const int gm = min(GROUP, g.tiles_m - first_m);
  const int m0 = (first_m + (id % per_group) % gm) * BM;
  const int n0 = ((id % per_group) / gm) * BN;
  const int kb = split < 0 ? 0 : split * g.kps;
  const int ke = split < 0 ? g.K : min(g.K, kb + g.kps);
  const int nk = (ke - kb) / kGBK;

  // ---- DMA: instruction i of this wave fills LDS rows i*32 + wave*8 + [0, 8) (A rows
  // for i < NA, B rows after); lane l -> row + l/8, slot l%8 holding source chunk
  // (l%8) ^ ((row >> 1) & 7), the same for every i
  const int rA = wave * 8 + (lane >> 3);
  const int chunk = (lane & 7) ^ ((rA >> 1) & 7);
  const long long brows = g.gated ? 2LL * g.half : (long long)g.Nv;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(g.a), (short)0, (int)(((long long)(g.M - 1) * g.lda + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(g.b), (short)0, (int)(((brows - 1) * g.ldb + g.K) * 2), 0x00020000);
  const uint32_t voff_a = (uint32_t)(((long long)(m0 + rA) * g.lda + chunk * 8) * 2);
  long long brow0;  // weight row of this lane in B group 0
  if (!g.gated) brow0 = n0 + rA;
  else brow0 = (rA < 16 ? 0LL : (long long)g.half - 16) + n0 / 2 + rA;
  const uint32_t voff_b = (uint32_t)((brow0 * g.ldb + chunk * 8) * 2);
  // scalar byte offsets of each 32-row group (A: 32 rows; B: 32 virtual rows = 16
  // weight rows of each half when gated)
  const uint32_t gstride_a = (uint32_t)(32LL * g.lda * 2);
  const uint32_t gstride_b = (uint32_t)((g.gated ? 16LL : 32LL) * g.ldb * 2);
  const uint32_t kbase = (uint32_t)kb * 2;
  // a step past the split's end: soffset 2^31 - 1 puts every lane out of range (zeros,
  // no memory traffic; voffsets stay below 2^31, so the sum cannot wrap)
  auto stage_one = [&](int step, int buf, int i) __attribute__((always_inline)) {
    const uint32_t ks = kbase + (uint32_t)step * (kGBK * 2);
    auto* dst = (__attribute__((address_space(3))) void*)(smem + buf * BUF + (i * 4 + wave) * 1024);
    const bool live = step < nk;
    if (i < NA)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, dst, 16, voff_a, live ? (int)(ks + i * gstride_a) : 0x7fffffff, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, dst, 16, voff_b, live ? (int)(ks + (i - NA) * gstride_b) : 0x7fffffff, 0, 0);
  };
  auto stage = [&](int step, int buf) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) stage_one(step, buf, i);
  };

  cf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) azero(acc[i][j]);
  if constexpr (DEEP) {
    constexpr int HB = (BM + BN) * 64;  // bytes per half-k region
    constexpr int IPH = (BM + BN) / 64; // DMAs per wave per half (16 rows of 64 B each)
    constexpr int NAH = BM / 64;        // of which A
    static_assert(IPH * 2 == FM + FN, "a half's DMAs alternate with its fragment reads");
    // DMA j of this wave fills half-rows (j * 4 + wave) * 16 + [0, 16); lane l -> row
    // + l / 4, slot l % 4, holding chunk (l % 4) ^ F[(l >> 4) & 3] of the half
    const int hrow = wave * 16 + (lane >> 2);
    const int fsw = (0x78 >> (2 * ((lane >> 4) & 3))) & 3;
    const int hch = (lane & 3) ^ fsw;
    const uint32_t hvoff_a = (uint32_t)(((long long)(m0 + hrow) * g.lda + hch * 8) * 2);
    long long hbrow;
    if (!g.gated) hbrow = n0 + hrow;
    else hbrow = ((wave & 1) ? (long long)g.half : 0LL) + (n0 / 32 + (wave >> 1)) * 16 + (lane >> 2);
    const uint32_t hvoff_b = (uint32_t)((hbrow * g.ldb + hch * 8) * 2);
    const uint32_t hstride_a = (uint32_t)(64LL * g.lda * 2);
    const uint32_t hstride_b = (uint32_t)((g.gated ? 32LL : 64LL) * g.ldb * 2);
    auto stage_half = [&](int step, int buf, int h, int j) __attribute__((always_inline)) {
      const uint32_t ks = kbase + (uint32_t)step * (kGBK * 2) + (uint32_t)h * 64;
      auto* dst = (__attribute__((address_space(3))) void*)(smem + (buf * 2 + h) * HB +
                                                            (j * 4 + wave) * 1024);
      const bool live = step < nk;
      if (j < NAH)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            ra, dst, 16, hvoff_a, live ? (int)(ks + j * hstride_a) : 0x7fffffff, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rb, dst, 16, hvoff_b, live ? (int)(ks + (j - NAH) * hstride_b) : 0x7fffffff, 0, 0);
    };
    // fragment (16 rows x 8 k) of tile row r0: row r0 + (l & 15), slot (l >> 4) ^ F[...]
    const uint32_t lds0 = lds_off(smem);
    const uint32_t foff = (uint32_t)(lane & 15) * 64 +
                          (uint32_t)((((lane >> 4) & 3) ^ ((0x78 >> (2 * ((lane >> 2) & 3))) & 3)) * 16);
    const uint32_t fa = lds0 + (uint32_t)(wr * WTM) * 64 + foff;
    const uint32_t fb = lds0 + (uint32_t)(BM + wc * WTN) * 64 + foff;
    constexpr int NM = FM * FN, NR = FM + FN;
    uint4 af0[FM], bf0[FN], af1[FM], bf1[FN];
    // prologue: both halves of steps 0 and 1, then step 0's k 0..31 fragments
    for (int st = 0; st < 2; ++st)
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < IPH; ++j) stage_half(st, st, h, j);
    __builtin_amdgcn_s_waitcnt(vm_wait(2 * IPH));
    asm volatile("s_barrier" ::: "memory");
#pragma unroll
    for (int i = 0; i < FM; ++i) af0[i] = ds_read16(fa + i * 16 * 64);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf0[j] = ds_read16(fb + j * 16 * 64);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    auto half_step = [&](auto BI, int t) __attribute__((always_inline)) {
      constexpr int b = decltype(BI)::value;
      const uint32_t a1 = fa + (b * 2 + 1) * HB, b1 = fb + (b * 2 + 1) * HB;
      const uint32_t a0n = fa + ((1 - b) * 2) * HB, b0n = fb + ((1 - b) * 2) * HB;
      // MFMAs on k 0..31 of t | reads of t's k 32..63, the k 0..31 DMAs of t + 2
      static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
        constexpr int m = decltype(mi)::value;
        amfma_v<DT>(acc[m / FN][m % FN], af0[m / FN], bf0[m % FN]);
        static_for<(m * 2 * NR + NM - 1) / NM, ((m + 1) * 2 * NR + NM - 1) / NM>([&](auto li)
                                                                        __attribute__((always_inline)) {
          constexpr int l = decltype(li)::value;
          if constexpr (l % 2 == 1) {
            constexpr int r = l / 2;
            if constexpr (r < FM) af1[r] = ds_read16_off<r * 16 * 64>(a1);
            else bf1[r - FM] = ds_read16_off<(r - FM) * 16 * 64>(b1);
          } else if constexpr ((l / 2) % 2 == 0) {  // DMAs spread over the phase
            stage_half(t + 2, b, 0, l / 4);
          }
        });
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(vm_wait(2 * IPH));  // t + 1's k 0..31 landed
      asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // MFMAs on k 32..63 of t | reads of t + 1's k 0..31, the k 32..63 DMAs of t + 2
      static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
        constexpr int m = decltype(mi)::value;
        amfma_v<DT>(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN]);
        static_for<(m * 2 * NR + NM - 1) / NM, ((m + 1) * 2 * NR + NM - 1) / NM>([&](auto li)
                                                                        __attribute__((always_inline)) {
          constexpr int l = decltype(li)::value;
          if constexpr (l % 2 == 1) {
            constexpr int r = l / 2;
            if constexpr (r < FM) af0[r] = ds_read16_off<r * 16 * 64>(a0n);
            else bf0[r - FM] = ds_read16_off<(r - FM) * 16 * 64>(b0n);
          } else if constexpr ((l / 2) % 2 == 0) {  // DMAs spread over the phase
            stage_half(t + 2, b, 1, l / 4);
          }
        });
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(vm_wait(2 * IPH));  // t + 1's k 32..63 landed
      asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    using Z = std::integral_constant<int, 0>;
    using O = std::integral_constant<int, 1>;
    for (int t = 0; t < nk; t += 2) {
      half_step(Z{}, t);
      if (t + 1 < nk) half_step(O{}, t + 1);
    }
  } else {
  // ---- fragment addresses (as gemm_kernel) ----------------------------------
  const int swz = (lane & 15) >> 1;
  const uint32_t lrow = (uint32_t)(lane & 15) * 128;
  const uint32_t off0 = (uint32_t)(((lane >> 4) ^ swz) * 16);
  const uint32_t off1 = (uint32_t)(((4 + (lane >> 4)) ^ swz) * 16);
  const uint32_t lds0 = lds_off(smem);
  const uint32_t a_base = lds0 + (uint32_t)(wr * WTM) * 128 + lrow;
  const uint32_t b_base = lds0 + (uint32_t)(BM + wc * WTN) * 128 + lrow;


  // The interleaved two-stage schedule of gemm_kernel (IL, NS = 2):
  //   [kk1 reads of t | kk0 MFMAs of t] wait | vmcnt(DMA t+1) barrier
  //   [DMA t+2 into t's buffer + kk0 reads of t+1 | kk1 MFMAs of t] wait
  // Every step issues all 16 DMAs (past the split's end: out of the descriptors' range,
  // zeros) so the counted waits hold.
  constexpr int NM = FM * FN, NR = FM + FN, NL = IPW + NR;
  uint4 af0[FM], bf0[FN], af1[FM], bf1[FN];
  stage(0, 0);
  __builtin_amdgcn_s_waitcnt(vm_wait(0));
  asm volatile("s_barrier" ::: "memory");
  stage(1, 1);
#pragma unroll
  for (int i = 0; i < FM; ++i) af0[i] = ds_read16(a_base + i * 16 * 128 + off0);
#pragma unroll
  for (int j = 0; j < FN; ++j) bf0[j] = ds_read16(b_base + j * 16 * 128 + off0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int buf = 0;
  for (int t = 0; t < nk; ++t) {
    const uint32_t ab = a_base + buf * BUF, bb = b_base + buf * BUF;
    static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
      constexpr int m = decltype(mi)::value;
      amfma_v<DT>(acc[m / FN][m % FN], af0[m / FN], bf0[m % FN]);
      static_for<(m * NR + NM - 1) / NM, ((m + 1) * NR + NM - 1) / NM>([&](auto ri)
                                                                    __attribute__((always_inline)) {
        constexpr int r = decltype(ri)::value;
        if constexpr (r < FM) af1[r] = ds_read16_off<r * 16 * 128>(ab + off1);
        else bf1[r - FM] = ds_read16_off<(r - FM) * 16 * 128>(bb + off1);
      });
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int nbuf = buf ^ 1;
    __builtin_amdgcn_s_waitcnt(vm_wait(0));  // DMA of step t+1 landed
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t na = a_base + nbuf * BUF, nb = b_base + nbuf * BUF;
    const int s2 = t + 2;
    static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
      constexpr int m = decltype(mi)::value;
      amfma_v<DT>(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN]);
      static_for<(m * NL + NM - 1) / NM, ((m + 1) * NL + NM - 1) / NM>([&](auto li)
                                                                    __attribute__((always_inline)) {
        constexpr int l = decltype(li)::value;
        if constexpr (l % 2 == 0 && l / 2 < IPW) {  // DMAs and reads alternate
          stage_one(s2, buf, l / 2);
        } else {
          constexpr int r = (l - 1) / 2;
          if constexpr (r < FM) af0[r] = ds_read16_off<r * 16 * 128>(na + off0);
          else bf0[r - FM] = ds_read16_off<(r - FM) * 16 * 128>(nb + off0);
        }
      });
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    buf = nbuf;
  }

  }

  // ---- epilogue (as gemm_kernel) -----------------------------------------
#pragma unroll
  for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
  __builtin_amdgcn_s_waitcnt(vm_wait(0));
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const float4* padd = nullptr;
  if (g.pair && split >= 0) {
    // split-K pair: ticket per tile (agent scope).  The first arrival stores its
    // accumulators to the tile's slab ([i][j][thread] float4, coalesced), releases and
    // raises the ready flag, and is done; the second waits for the flag (the first is
    // already past its ticket, so it is running: no residency assumption), acquires,
    // adds the slab and runs the epilogue, then clears the tile's counters for the next
    // launch.  a + b in either order: the same bits whichever split arrives first.
    const int pid = id - g.dp_tiles;  // this pair's slot
    unsigned* tk = g.tick + pid;
    unsigned* fl = g.tick + kPairTiles + pid;
    volatile uint32_t* bc = reinterpret_cast<volatile uint32_t*>(smem + 2 * BUF - 16);
    if (tid == 0) bc[0] = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const bool first = bc[0] == 0;
    float4* slab = reinterpret_cast<float4*>(g.ws + (size_t)pid * (BM * BN)) + tid;
    if (first) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const cf32x4 v = acc[i][j];
          slab[(i * FN + j) * 256] = make_float4(v[0], v[1], v[2], v[3]);
        }
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(fl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
        __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(fl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    padd = slab;  // the epilogue strips add the first split's accumulators
  }
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
    epi_strip<DT, EPI, FN, i & 1>(g, acc[i], stg, row_m0 + i * 16, vcol0, split, lane, ops,
                                  padd ? padd + i * FN * 256 : nullptr);
  });
}

}  // namespace cake
