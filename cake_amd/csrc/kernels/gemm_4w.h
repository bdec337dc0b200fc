// Four-wave MFMA GEMM tiles 256x256 / 256x192 / 128x256 (plan cfg 22-24, and 25-27 on the
// three-barrier schedule): the large Llama prefill projections.
//
// Included by gemm_kernel.h (launch_gemm dispatches cfg 22-27 here); same GemmArgs, tile
// order, swizzled LDS image, fragment reads and epilogues as gemm_kernel's IL path.
//
// The shape of the winning library kernel on this chip (hipBLASLt's 256x256x64 tile,
// profiles/r6_gemm_pmc_8192.txt): one wave per SIMD, 128 x 128 outputs per wave, LDS-DMA
// staging, 32 fragment reads per k-step.  At one wave per SIMD every instruction beside
// the MFMAs is paid in MFMA gaps (16 cycles, 8 of them free), so a DMA piece is three
// instructions and nothing else (k-loop stamps: profiles/r6_gemm_stamps.jsonl):
//   * buffer_load_dwordx4 ... offen lds with one per-lane byte offset VGPR per operand (the
//     lane's row in its 32-row group and its swizzled 16-byte chunk) and the group's row
//     offset as a loop-invariant scalar soffset;
//   * the k step in the descriptor: its base advanced and num_records shrunk per step (a
//     handful of scalar ops per step, not per piece); rows past the matrix and steps past
//     the split read through the range check as zeros (no per-issue select, no zeros
//     page); gated (SwiGLU / GEGLU) weights keep a constant row stride per group (16 gate
//     + 16 up rows), so the same form covers them;
//   * the M0 write (buffer base + the piece's offset as an immediate) and the DMA in one
//     asm statement with the MFMA it is scheduled behind, which also covers M0's wait state.
//   Needs K and the split's k range in whole 64-element steps and operands under 2 GB
//   (host-checked).
#pragma once

// Diagnostic build only (scripts/gemm_stamp.hip defines CAKE_GEMM_STAMPS and the
// g_gemm_stamps buffer): s_memtime at the k-loop's segment boundaries, summed per wave.
#ifdef CAKE_GEMM_STAMPS
#define CAKE_STAMP(v)                                                                   \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
#else
#define CAKE_STAMP(v) \
  do {                \
  } while (0)
#endif

namespace cake {

constexpr int k4WCfg = 22;     // plan cfg id of the 256 x 256 tile
constexpr int k4WCfg192 = 23;  // 256 x 192 (8B q|k|v: 6144 = 32 x 192 columns, 256 tiles at
                               // 2048 tokens instead of 192)
constexpr int k4WCfg128 = 24;  // 128 x 256 (8B o / down at 2048 tokens: 256 tiles, not 128)
constexpr int k4WSched = 3;    // cfg + 3: the same tiles on the three-barrier schedule (25-27)
inline bool four_wave_cfg(int cfg) { return cfg >= k4WCfg && cfg <= k4WCfg128 + k4WSched; }
// op k of an alternating sequence of nr reads and nd DMAs (the longer list's tail last):
// kind 0 = read, 1 = DMA, and its index within its list
constexpr int alt_kind(int nr, int nd, int k) {
  return k < 2 * (nr < nd ? nr : nd) ? k % 2 : (nr > nd ? 0 : 1);
}
constexpr int alt_idx(int nr, int nd, int k) {
  const int mn = nr < nd ? nr : nd;
  return k < 2 * mn ? k / 2 : mn + (k - 2 * mn);
}

// LDS-DMA of one 1 KiB piece (buffer_load_dwordx4 ... offen lds) with the M0 write in the
// same statement (M0 is not preserved around inline asm); d = the buffer descriptor as an
// SGPR quad.  amfma_dma issues an MFMA between the M0 write and the DMA, which covers the
// write's wait state (no s_nop) and keeps the DMA beside the MFMA it was scheduled with.
template <int OFF>
__device__ __forceinline__ void dma16(uint32_t mb, uint32_t voff, cu32x4 d, uint32_t soff) {
  asm volatile("s_add_u32 m0, %0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(mb), "v"(voff), "s"(d), "s"(soff), "i"(OFF) : "memory");
}
template <int DT, int OFF>
__device__ __forceinline__ void amfma_dma(cf32x4& acc, const uint4& a, const uint4& b, uint32_t mb,
                                          uint32_t voff, cu32x4 d, uint32_t soff) {
  const cu32x4 av = __builtin_bit_cast(cu32x4, a), bv = __builtin_bit_cast(cu32x4, b);
  if constexpr (DT == kBF16)
    asm volatile("s_add_u32 m0, %3, %7\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
                 "buffer_load_dwordx4 %4, %5, %6 offen lds"
                 : "+a"(acc)
                 : "v"(av), "v"(bv), "s"(mb), "v"(voff), "s"(d), "s"(soff), "i"(OFF)
                 : "memory");
  else
    asm volatile("s_add_u32 m0, %3, %7\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
                 "buffer_load_dwordx4 %4, %5, %6 offen lds"
                 : "+a"(acc)
                 : "v"(av), "v"(bv), "s"(mb), "v"(voff), "s"(d), "s"(soff), "i"(OFF)
                 : "memory");
}

// SCHED 1 (cfg 25-27): the same tiles on a three-barrier schedule (the DMAs of step t+2
// issued as soon as every wave has read the operand region they overwrite).
template <int DT, int EPI, int BM, int BN, int SCHED = 0>
__global__ __launch_bounds__(256) void gemm_4w_kernel(GemmArgs g) {
  static_assert((BM == 256 && (BN == 256 || BN == 192)) || (BM == 128 && BN == 256),
                "four-wave tile shapes");
  constexpr int WTM = BM / 2, WTN = BN / 2, FM = WTM / 16, FN = WTN / 16;
  constexpr int BUF = (BM + BN) * 128;  // 64 / 56 / 48 KB per k-step buffer
  constexpr int IPW = (BM + BN) / 32;   // DMA wave-instructions per wave per k-step
  constexpr int NA = BM / 32;           // of which A
  static_assert(IPW == FM + FN, "the second half alternates one DMA with one fragment read");
  constexpr int STG_LD = WTN + 4, STG = 16 * STG_LD * 4;
  static_assert(8 * STG <= 2 * BUF - 16, "epilogue staging (2 slices per wave) fits the operand buffers");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
#ifdef CAKE_GEMM_STAMPS
  unsigned long long st_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_entry;
  CAKE_STAMP(t_entry);
#endif
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
  const int nrec_a = (int)(((long long)(g.M - 1) * g.lda + g.K) * 2);
  const int nrec_b = (int)(((brows - 1) * g.ldb + g.K) * 2);
  const uint32_t voff_a = (uint32_t)(((long long)(m0 + rA) * g.lda + chunk * 8) * 2);
  long long brow0;  // weight row of this lane in B group 0
  if (!g.gated) brow0 = n0 + rA;
  else brow0 = (rA < 16 ? 0LL : (long long)g.half - 16) + n0 / 2 + rA;
  const uint32_t voff_b = (uint32_t)((brow0 * g.ldb + chunk * 8) * 2);
  // scalar byte offsets of each 32-row group (A: 32 rows; B: 32 virtual rows = 16
  // weight rows of each half when gated): loop-invariant SGPRs
  const uint32_t gstride_a = (uint32_t)(32LL * g.lda * 2);
  const uint32_t gstride_b = (uint32_t)((g.gated ? 16LL : 32LL) * g.ldb * 2);
  // The k step lives in the descriptors: base advanced to the step's first column and
  // num_records shrunk by as much (a step past the split's end: 0 records, every lane out
  // of range -> zeros, no memory traffic).  Per DMA that leaves the M0 write and the DMA
  // itself in the MFMA stream, the rest is a handful of scalar ops per k-step.
  // descriptor words: base (48 bits, stride 0), num_records, flags (raw, offen)
  auto desc_at = [&](const uint16_t* base, int nrec, int step) __attribute__((always_inline)) {
    const int k0 = kb + step * kGBK;
    const unsigned long long p = (unsigned long long)(base + k0);
    cu32x4 d;
    d[0] = __builtin_amdgcn_readfirstlane((unsigned)p);
    d[1] = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32) & 0xFFFFu);
    d[2] = __builtin_amdgcn_readfirstlane(step < nk ? (unsigned)(nrec - 2 * k0) : 0u);
    d[3] = 0x00020000u;
    return d;
  };
  auto src_a = [&](int step) __attribute__((always_inline)) { return desc_at(g.a, nrec_a, step); };
  auto src_b = [&](int step) __attribute__((always_inline)) { return desc_at(g.b, nrec_b, step); };
  const uint32_t m0_base = __builtin_amdgcn_readfirstlane(lds_off(smem) + (uint32_t)wave * 1024);
  // M0 (= buffer base + 4 KiB per piece, the piece offset an immediate) / voffset / soffset
  // of DMA I (A pieces for I < NA) into buffer buf
  auto dma_mb = [&](int buf) __attribute__((always_inline)) {
    return m0_base + (uint32_t)(buf * BUF);
  };
  auto dma_voff = [&](int i) __attribute__((always_inline)) { return i < NA ? voff_a : voff_b; };
  auto dma_soff = [&](int i) __attribute__((always_inline)) {
    return i < NA ? (uint32_t)i * gstride_a : (uint32_t)(i - NA) * gstride_b;
  };
  auto stage_one = [&](const cu32x4& sa, const cu32x4& sb, int buf, auto I)
                       __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    dma16<i * 4096>(dma_mb(buf), dma_voff(i), i < NA ? sa : sb, dma_soff(i));
  };
  // MFMA with DMA I fused behind it
  auto mfma_dma = [&](cf32x4& c, const uint4& a, const uint4& b, const cu32x4& sa,
                      const cu32x4& sb, int buf, auto I) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    amfma_dma<DT, i * 4096>(c, a, b, dma_mb(buf), dma_voff(i), i < NA ? sa : sb, dma_soff(i));
  };
  auto stage = [&](int step, int buf) {
    const cu32x4 sa = src_a(step), sb = src_b(step);
    static_for<0, IPW>([&](auto I) __attribute__((always_inline)) { stage_one(sa, sb, buf, I); });
  };

  cf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) azero(acc[i][j]);
  // ---- fragment addresses (as gemm_kernel) ----------------------------------
  const int swz = (lane & 15) >> 1;
  const uint32_t lrow = (uint32_t)(lane & 15) * 128;
  const uint32_t off0 = (uint32_t)(((lane >> 4) ^ swz) * 16);
  const uint32_t off1 = (uint32_t)(((4 + (lane >> 4)) ^ swz) * 16);
  const uint32_t lds0 = lds_off(smem);
  const uint32_t a_base = lds0 + (uint32_t)(wr * WTM) * 128 + lrow;
  const uint32_t b_base = lds0 + (uint32_t)(BM + wc * WTN) * 128 + lrow;
  constexpr int NM = FM * FN, NR = FM + FN, NB = IPW - NA;
  uint4 af0[FM], bf0[FN], af1[FM], bf1[FN];

  if constexpr (SCHED == 1) {
    // Three barriers per k-step; a step's operand regions are restaged as soon as every
    // wave has read them, so the DMAs spread over two thirds of the step:
    //   phase 1 (k 0..31 MFMAs of t): [B k 32..63 reads] lgkm+barrier (B of t free)
    //     [A k 32..63 reads + B DMAs of t+2] lgkm+barrier (A of t free) [A DMAs]
    //   phase 2 (k 32..63 MFMAs of t): [A DMAs] vmcnt(this step's) + barrier
    //     (t+1 landed) [k 0..31 reads of t+1] lgkm
    // Each wait + barrier follows an MFMA issue, so the pipe runs while the waves align.
    // (placements measured: barriers at NM/8 and NM/2, or all A DMAs before phase 2 with its
    // barrier at MFMA 1, ran within 3 % / 3-6 % slower, profiles/r6_gemm_three_barrier_ab.txt)
    constexpr int Q1 = NM / 4, Q2 = (NM * 5) / 8, P1 = NM / 4;
    constexpr int NA1 = NA / 2;  // A DMAs in phase 1's tail, the rest in phase 2's head
    static_assert(Q1 >= FN / 2 && Q2 - Q1 - 1 >= (FM + NB) / 2, "op density");
    stage(0, 0);
    stage(1, 1);
    __builtin_amdgcn_s_waitcnt(vm_wait(IPW));
    asm volatile("s_barrier" ::: "memory");
#pragma unroll
    for (int i = 0; i < FM; ++i) af0[i] = ds_read16(a_base + i * 16 * 128 + off0);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf0[j] = ds_read16(b_base + j * 16 * 128 + off0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    int buf = 0;
    for (int t = 0; t < nk; ++t) {
      const uint32_t ab = a_base + buf * BUF, bb = b_base + buf * BUF;
      const int nbuf = buf ^ 1;
      const uint32_t na = a_base + nbuf * BUF, nb = b_base + nbuf * BUF;
      const cu32x4 sa = src_a(t + 2), sb = src_b(t + 2);
      // ops k of n spread over MFMAs [lo, hi): op k after MFMA lo + floor(k (hi-lo) / n)
      static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
        constexpr int m = decltype(mi)::value;
        // the first op placed after this MFMA, when it is a DMA, goes in the MFMA's statement
        constexpr int L2 = Q2 - Q1 - 1, n2 = FM + NB, m2 = m - Q1 - 1;
        constexpr int L3 = NM - Q2 - 1, m3 = m - Q2 - 1;
        constexpr int k2 = (m2 * n2 + L2 - 1) / L2, k2e = ((m2 + 1) * n2 + L2 - 1) / L2;
        constexpr int k3 = (m3 * NA1 + L3 - 1) / L3, k3e = ((m3 + 1) * NA1 + L3 - 1) / L3;
        constexpr int fd = (m > Q1 && m < Q2 && k2 < k2e && alt_kind(FM, NB, k2) == 1)
                               ? NA + alt_idx(FM, NB, k2)
                               : (m > Q2 && k3 < k3e) ? k3 : -1;
        if constexpr (fd >= 0) mfma_dma(acc[m / FN][m % FN], af0[m / FN], bf0[m % FN], sa, sb, buf, std::integral_constant<int, fd>{});
        else amfma_v<DT>(acc[m / FN][m % FN], af0[m / FN], bf0[m % FN]);
        if constexpr (m < Q1) {
          static_for<(m * FN + Q1 - 1) / Q1, ((m + 1) * FN + Q1 - 1) / Q1>([&](auto ji)
                                                                    __attribute__((always_inline)) {
            constexpr int j = decltype(ji)::value;
            bf1[j] = ds_read16_off<j * 16 * 128>(bb + off1);
          });
        } else if constexpr (m == Q1 || m == Q2) {
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (m < Q2) {
          static_for<k2 + (fd >= 0 ? 1 : 0), k2e>([&](auto ki) __attribute__((always_inline)) {
            constexpr int k = decltype(ki)::value;  // reads and DMAs alternate
            if constexpr (alt_kind(FM, NB, k) == 0)
              af1[alt_idx(FM, NB, k)] = ds_read16_off<alt_idx(FM, NB, k) * 16 * 128>(ab + off1);
            else
              stage_one(sa, sb, buf, std::integral_constant<int, NA + alt_idx(FM, NB, k)>{});
          });
        } else {
          static_for<k3 + (fd >= 0 ? 1 : 0), k3e>([&](auto ki) __attribute__((always_inline)) {
            stage_one(sa, sb, buf, ki);
          });
        }
      });
      static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
        constexpr int m = decltype(mi)::value;
        constexpr int n1 = NA - NA1;
        constexpr int k1 = (m * n1 + P1 - 1) / P1, k1e = ((m + 1) * n1 + P1 - 1) / P1;
        constexpr int fd = (m < P1 && k1 < k1e) ? NA1 + k1 : -1;
        if constexpr (fd >= 0) mfma_dma(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN], sa, sb, buf, std::integral_constant<int, fd>{});
        else amfma_v<DT>(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN]);
        if constexpr (m < P1) {
          static_for<k1 + (fd >= 0 ? 1 : 0), k1e>([&](auto ki) __attribute__((always_inline)) {
            stage_one(sa, sb, buf, std::integral_constant<int, NA1 + decltype(ki)::value>{});
          });
        } else if constexpr (m == P1) {
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_waitcnt(vm_wait(IPW));  // step t+1's DMAs landed
          asm volatile("s_barrier" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        } else {
          constexpr int L = NM - P1 - 1, mm = m - P1 - 1;
          static_for<(mm * NR + L - 1) / L, ((mm + 1) * NR + L - 1) / L>([&](auto ri)
                                                                   __attribute__((always_inline)) {
            constexpr int r = decltype(ri)::value;
            if constexpr (r < FM) af0[r] = ds_read16_off<r * 16 * 128>(na + off0);
            else bf0[r - FM] = ds_read16_off<(r - FM) * 16 * 128>(nb + off0);
          });
        }
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      buf = nbuf;
    }
  } else {

  // The interleaved two-stage schedule of gemm_kernel (IL, NS = 2):
  //   [kk1 reads of t | kk0 MFMAs of t] wait | vmcnt(DMA t+1) barrier
  //   [DMA t+2 into t's buffer + kk0 reads of t+1 | kk1 MFMAs of t] wait
  // Every step issues all 16 DMAs (past the split's end: out of the descriptors' range,
  // zeros) so the counted waits hold.
  constexpr int NL = IPW + NR;
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
  unsigned long long tp = 0, t1 = 0, t2 = 0, t3 = 0;
  CAKE_STAMP(tp);
#ifdef CAKE_GEMM_STAMPS
  st_[4] = tp - t_entry;  // prologue: tile decode, descriptors, first two steps' DMAs
#endif
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
    CAKE_STAMP(t1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int nbuf = buf ^ 1;
    __builtin_amdgcn_s_waitcnt(vm_wait(0));  // DMA of step t+1 landed
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    CAKE_STAMP(t2);
    const uint32_t na = a_base + nbuf * BUF, nb = b_base + nbuf * BUF;
    const cu32x4 sa = src_a(t + 2), sb = src_b(t + 2);
    static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
      constexpr int m = decltype(mi)::value;
      constexpr int l0 = (m * NL + NM - 1) / NM, l1 = ((m + 1) * NL + NM - 1) / NM;
      constexpr bool fuse = l0 < l1 && l0 % 2 == 0 && l0 / 2 < IPW;
      if constexpr (fuse) mfma_dma(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN], sa, sb, buf, std::integral_constant<int, l0 / 2>{});
      else amfma_v<DT>(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN]);
      static_for<l0 + (fuse ? 1 : 0), l1>([&](auto li) __attribute__((always_inline)) {
        constexpr int l = decltype(li)::value;
        if constexpr (l % 2 == 0 && l / 2 < IPW) {  // DMAs and reads alternate
          stage_one(sa, sb, buf, std::integral_constant<int, l / 2>{});
        } else {
          constexpr int r = (l - 1) / 2;
          if constexpr (r < FM) af0[r] = ds_read16_off<r * 16 * 128>(na + off0);
          else bf0[r - FM] = ds_read16_off<(r - FM) * 16 * 128>(nb + off0);
        }
      });
    });
    CAKE_STAMP(t3);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    buf = nbuf;
#ifdef CAKE_GEMM_STAMPS
    unsigned long long t4;
    CAKE_STAMP(t4);
    st_[0] += t1 - tp; st_[1] += t2 - t1; st_[2] += t3 - t2; st_[3] += t4 - t3;
    tp = t4;
#endif
  }
#ifdef CAKE_GEMM_STAMPS
  st_[5] = tp;  // loop end; the epilogue's length is taken at the kernel's end
#endif
  (void)tp; (void)t1; (void)t2; (void)t3;

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
  if constexpr (EpiW<DT, EPI, FN>::OK) {
    EpiW<DT, EPI, FN> ops;
    ops.load_bias(g, vcol0, lane);
    ops.template load_res<0>(g, row_m0, vcol0, lane);
#ifdef CAKE_GEMM_STAMPS
    unsigned long long ts0, ts1;
    CAKE_STAMP(ts0);
    st_[7] = ts0 - st_[5];  // loop end -> first strip
#endif
    // two staging slices per wave: strip i+1 is staged while strip i is read out (one
    // LDS wait per strip; a wave's LDS accesses complete in order, so restaging a slice
    // after the reads of the strip before it needs no wait)
    float* sg0 = reinterpret_cast<float*>(smem + (wave * 2) * STG);
    float* sg1 = reinterpret_cast<float*>(smem + (wave * 2 + 1) * STG);
    stage_strip_w<FN>(acc[0], sg0, lane, padd);
    static_for<0, FM>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      if constexpr (i + 1 < FM) {
        stage_strip_w<FN>(acc[i + 1], (i & 1) ? sg0 : sg1, lane,
                          padd ? padd + (i + 1) * FN * 256 : nullptr);
        ops.template load_res<(i + 1) & 1>(g, row_m0 + (i + 1) * 16, vcol0, lane);
      }
      readout_strip_w<DT, EPI, FN, i & 1>(g, (i & 1) ? sg1 : sg0, row_m0 + i * 16, vcol0, split,
                                          lane, ops);
    });
#ifdef CAKE_GEMM_STAMPS
    CAKE_STAMP(ts1);
    st_[6] = ts1 - ts0;  // the strips (staging + read-out + store issue)
#endif
  } else {  // 96-column wave tiles (256 x 192): 4 lanes per row
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
#ifdef CAKE_GEMM_STAMPS
  {
    unsigned long long t_end;
#ifndef CAKE_STAMP_NODRAIN
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's stores issued and done
#endif
    CAKE_STAMP(t_end);
    st_[5] = t_end - st_[5];
    if (lane == 0)
      for (int i = 0; i < 8; ++i) g_gemm_stamps[((size_t)blockIdx.x * 4 + wave) * 8 + i] = st_[i];
  }
#endif
}

}  // namespace cake
