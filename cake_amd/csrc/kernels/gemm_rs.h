// Register-staged 256x256 MFMA GEMM (plan cfg 21): the large Llama prefill projections.
//
// Included by gemm_kernel.h (launch_gemm dispatches cfg 21 here); same GemmArgs, tile
// order, swizzled LDS image, fragment reads and epilogues as gemm_kernel.
//
// Why: the 8-wave 256x256 tile (cfg 5) and its ping-pong form (cfg 20, gemm_pp.h) stage
// operands by LDS-DMA, 64 KB per k-tile = 16 DMA issues per SIMD, each holding its wave's
// issue for 60-185 cycles (MI355X_MICROARCH.md 'LDS-DMA piece') against the 2048 cycles
// of MFMA work per k-tile: both measured the same 1.32-1.33 PF/s at 8192^3, where the
// matrix pipe sat idle a third of the time (profiles/r3_gemm_large_pmc.txt: hipBLASLt's
// register-staged 4-wave kernel keeps it 1.34x busier per clock).  Here:
//
//   * 4 waves (one per SIMD, 512 registers each), 2 x 2, 128 x 128 outputs per wave:
//     FM = FN = 8 16x16 tiles, 256 AGPR accumulators; per k-tile a wave reads 32
//     fragments (128 KB of LDS per CU, 2/3 of cfg 5's 192 KB).
//   * Operands by buffer_load_dwordx4 into 16 staging registers x 4 per lane (64 KB per
//     k-tile over 256 lanes), ds_write_b128 into the other of two 64 KB LDS buffers:
//     one load costs its wave a few issue cycles, one 16-byte LDS store 13.
//   * Per k-tile t (buffer b):  [64 MFMAs on k 0..31 | in their gaps: 16 fragment reads of
//     k 32..63, 16 stores of the staged tile t+1 into buffer b^1, then 16 loads of tile
//     t+2 into the same registers]  lgkmcnt(0) barrier  [64 MFMAs on k 32..63 | 16
//     fragment reads of k 0..31 of tile t+1 from b^1].  One barrier per k-tile; a load
//     has a whole k-tile (~2k cycles) to land before its store.
//   * Out-of-range rows and the loads past the last k-tile read through the buffer
//     descriptor's range check (zeros, no memory traffic): no zeros page, no per-load
//     select.  Needs K and the split's k range in whole 64-element steps (host-checked)
//     and operands under 2 GB.
#pragma once

namespace cake {

constexpr int kRSCfg = 21;  // plan cfg id of this kernel (BM = BN = 256)

__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  cu32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(r), "s"(soff));
  return __builtin_bit_cast(uint4, v);
}

template <int OFF>
__device__ __forceinline__ void ds_write16_off(uint32_t addr, const uint4& v) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16-bit");
  const cu32x4 d = __builtin_bit_cast(cu32x4, v);
  asm volatile("ds_write_b128 %0, %1 offset:%2" : : "v"(addr), "v"(d), "i"(OFF));
}

template <int DT, int EPI>
__global__ __launch_bounds__(256) void gemm_rs_kernel(GemmArgs g) {
  constexpr int BM = 256, BN = 256, WTM = 128, WTN = 128, FM = 8, FN = 8;
  constexpr int BUF = (BM + BN) * 128;  // 64 KB per k-tile buffer
  constexpr int NLD = 16;               // staging loads per lane per k-tile
  constexpr int STG_LD = WTN + 4, STG = 16 * STG_LD * 4;
  static_assert(4 * STG <= 2 * BUF, "epilogue staging fits the operand buffers");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 1, wc = wave & 1;

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
  const int nk = (ke - kb) / kGBK;

  // ---- staging: load i of this lane = 16-byte chunk (tid & 7) of LDS row i*32 + tid/8
  // (rows 0-255 A, 256-511 B); offsets in bytes from the operand base at k = kb
  const long long brows = g.gated ? 2LL * g.half : (long long)g.Nv;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(g.a), (short)0, (int)(((long long)(g.M - 1) * g.lda + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(g.b), (short)0, (int)(((brows - 1) * g.ldb + g.K) * 2), 0x00020000);
  uint32_t voff[NLD];
  const int ch = tid & 7;
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const int r = i * 32 + (tid >> 3);
    if (i < 8) {
      const int m = m0 + r;
      voff[i] = m < g.M ? (uint32_t)(((long long)m * g.lda + kb + ch * 8) * 2) : 0x80000000u;
    } else {
      const int v = n0 + (r - BM);
      voff[i] = v < g.Nv ? (uint32_t)(((long long)wrow(g, v) * g.ldb + kb + ch * 8) * 2)
                         : 0x80000000u;
    }
  }
  // LDS destination of load i: row i*32 + tid/8, slot ch ^ ((row >> 1) & 7); the slot
  // swizzle depends on tid only (i*32 rows shift row >> 1 by multiples of 16)
  const uint32_t lds0 = lds_off(smem);
  const uint32_t wbase = lds0 + (uint32_t)(tid >> 3) * 128 + (uint32_t)((ch ^ ((tid >> 4) & 7)) * 16);
  uint4 stg_r[NLD];
  // k-tile `t` (relative to kb) -> soffset; past the split: out of every descriptor's range
  auto soff_of = [&](int t) -> uint32_t { return t < nk ? (uint32_t)t * 128u : 0x80000000u; };

  // ---- fragment addresses (as gemm_kernel) ----------------------------------
  const int swz = (lane & 15) >> 1;
  const uint32_t lrow = (uint32_t)(lane & 15) * 128;
  const uint32_t off0 = (uint32_t)(((lane >> 4) ^ swz) * 16);
  const uint32_t off1 = (uint32_t)(((4 + (lane >> 4)) ^ swz) * 16);
  const uint32_t a_base = lds0 + (uint32_t)(wr * WTM) * 128 + lrow;
  const uint32_t b_base = lds0 + (uint32_t)(BM + wc * WTN) * 128 + lrow;

  cf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) azero(acc[i][j]);
  uint4 af0[FM], bf0[FN], af1[FM], bf1[FN];

  // ---- prologue: tile 0 -> LDS buffer 0, tile 1 -> registers, k 0..31 fragments of tile 0
  {
    const uint32_t s0 = soff_of(0);
    static_for<0, NLD>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      stg_r[i] = buf_ld16(i < 8 ? ra : rb, voff[i], s0);
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    static_for<0, NLD>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      ds_write16_off<i * 32 * 128>(wbase, stg_r[i]);
    });
    const uint32_t s1 = soff_of(1);
    static_for<0, NLD>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      stg_r[i] = buf_ld16(i < 8 ? ra : rb, voff[i], s1);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
#pragma unroll
    for (int i = 0; i < FM; ++i) af0[i] = ds_read16(a_base + i * 16 * 128 + off0);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf0[j] = ds_read16(b_base + j * 16 * 128 + off0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }

  constexpr int NM = FM * FN;  // 64 MFMAs per k half
  // k-tile t from buffer BI: the schedule of the header comment
  auto ktile = [&](auto BI, int t) __attribute__((always_inline)) {
    constexpr int b = decltype(BI)::value;
    const uint32_t ab = a_base + b * BUF, bb = b_base + b * BUF;
    const uint32_t na = a_base + (1 - b) * BUF, nb = b_base + (1 - b) * BUF;
    const uint32_t wb = wbase + (1 - b) * BUF;
    const uint32_t s2 = soff_of(t + 2);
    // half 1: MFMAs on k 0..31; reads of k 32..63 after MFMAs 0-15, tile t+1's stores
    // after 16-31 (its loads were issued one k-tile ago), tile t+2's loads after 32-47
    static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
      constexpr int m = decltype(mi)::value;
      amfma_v<DT>(acc[m / FN][m % FN], af0[m / FN], bf0[m % FN]);
      if constexpr (m < 16) {
        if constexpr (m < FM) af1[m] = ds_read16_off<m * 16 * 128>(ab + off1);
        else bf1[m - FM] = ds_read16_off<(m - FM) * 16 * 128>(bb + off1);
      } else if constexpr (m < 32) {
        if constexpr (m == 16) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ds_write16_off<(m - 16) * 32 * 128>(wb, stg_r[m - 16]);
      } else if constexpr (m < 48) {
        stg_r[m - 32] = buf_ld16(m - 32 < 8 ? ra : rb, voff[m - 32], s2);
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");  // tile t+1 in buffer b^1, buffer b's reads done
    __builtin_amdgcn_sched_barrier(0);
    // half 2: MFMAs on k 32..63; reads of tile t+1's k 0..31 from buffer b^1
    static_for<0, NM>([&](auto mi) __attribute__((always_inline)) {
      constexpr int m = decltype(mi)::value;
      amfma_v<DT>(acc[m / FN][m % FN], af1[m / FN], bf1[m % FN]);
      if constexpr (m % 4 == 0) {
        constexpr int r = m / 4;
        if constexpr (r < FM) af0[r] = ds_read16_off<r * 16 * 128>(na + off0);
        else bf0[r - FM] = ds_read16_off<(r - FM) * 16 * 128>(nb + off0);
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  for (int t = 0; t < nk; t += 2) {
    ktile(Z{}, t);
    if (t + 1 < nk) ktile(O{}, t + 1);
  }

  // ---- epilogue (as gemm_kernel) -----------------------------------------
#pragma unroll
  for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[FM - 1][j]));
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
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
