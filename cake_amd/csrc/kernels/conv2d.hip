// Implicit-GEMM 2-D convolution on MFMA (gfx950 v_mfma_f32_16x16x32_{bf16,f16}),
// channels-last (NHWC) activations.
//
// Replaces the reference's candle conv2d (cuDNN/im2col) in every UNet / VAE
// ResnetBlock2D, down/up sampler and 1x1 shortcut (reference
// forwarders cake-core/src/models/sd/unet.rs, vae.rs).
//
//   out[p][oc] = sum_{ky,kx,ic} W[oc][ky][kx][ic] * X[n][iy][ix][ic]
//                + bias[oc] (+ bias2[n][oc]) (+ resid[p][oc])
//   p = (n, oy, ox), iy = oy*stride - pad + ky (nearest-2x upsampled input when
//   `up`: the virtual input is 2H x 2W and reads X[iy>>1][ix>>1]).
//
// GEMM view: rows = output channels (A = packed weights, k-contiguous),
// columns = output pixels (B = implicit im2col; with NHWC and the (ky,kx,ic)
// k order a 64-deep k-step is one tap x 64 contiguous channels, i.e. one
// 128-byte line per pixel).  Both operands are therefore 16-byte
// k-contiguous MFMA fragments; the accumulator layout (row = 4*(lane>>4)+r)
// gives each lane 4 consecutive channels of one pixel -> 8-byte stores.
// The time-embedding add of ResnetBlock2D (bias2) and the block's residual
// (resid) are fused in the epilogue; the 2x nearest upsample is fused into the
// B-operand addressing.
//
// Tiling: 256 threads = 2x2 waves, tile BM(oc) x BN(pix) x 64(k), register
// staged double-buffered LDS (global loads of step s+1 in flight during the
// MFMAs of step s), 16-byte chunks XOR-swizzled per row (conflict-free
// ds_read_b128 fragment reads), XCD-aware block->tile remap so neighbouring
// tiles (sharing the input tile through L2) land on one XCD.  Small grids use
// split-K with f32 slabs + a finalize launch carrying the epilogue.
#include "common.h"

namespace cake {

constexpr int kCBK = 64;  // k per step (one tap x 64 input channels)

struct ConvArgs {
  const uint16_t* x;      // [N][H][W][IC]
  const uint16_t* w;      // [OC][KH][KW][IC]
  const uint16_t* bias;   // [OC] or null
  const float* bias2;     // [N][OC] f32 or null
  const uint16_t* resid;  // [N][OH][OW][OC] or null
  uint16_t* out;          // [N][OH][OW][OC]
  float* ws;              // split-K slabs [splits][P][OC]
  const uint16_t* zeros;  // >= 16 zero bytes (LDS-DMA source for padding)
  int N, H, W, IC, OC, OH, OW, KH, KW, stride, pad, up;
  int P, ksteps, ks_per_split, tiles_m, tiles_n;
  int bias2_ld;           // row stride of bias2 (elements; OC when packed)
  int in_nchw;            // x is [N][IC][H][W] (direct small-IC kernel only: UNet conv_in)
  int out_nchw;           // out is [N][OC][OH][OW] (no resid: UNet conv_out)
};


// element offset of (row, 16-byte chunk) in a [rows][64] swizzled tile
__device__ __forceinline__ int swz(int row, int chunk) { return (row * 8 + (chunk ^ (row & 7))) * 8; }

template <int DT>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, int oc, int p, const float* v) {
  float r[4] = {v[0], v[1], v[2], v[3]};
  if (a.bias) {
    const uint2 b = *reinterpret_cast<const uint2*>(a.bias + oc);
    r[0] += to_f32<DT>(b.x & 0xffff); r[1] += to_f32<DT>(b.x >> 16);
    r[2] += to_f32<DT>(b.y & 0xffff); r[3] += to_f32<DT>(b.y >> 16);
  }
  if (a.bias2) {
    const int n = p / (a.OH * a.OW);
    const float4 b = *reinterpret_cast<const float4*>(a.bias2 + (size_t)n * a.bias2_ld + oc);
    r[0] += b.x; r[1] += b.y; r[2] += b.z; r[3] += b.w;
  }
  if (a.out_nchw) {  // planar output: the UNet's last conv writes the external layout
    const int ohw = a.OH * a.OW, n = p / ohw, px = p - n * ohw;
#pragma unroll
    for (int i = 0; i < 4; ++i) a.out[((size_t)n * a.OC + oc + i) * ohw + px] = from_f32<DT>(r[i]);
    return;
  }
  const size_t o = (size_t)p * a.OC + oc;
  if (a.resid) {
    const uint2 q = *reinterpret_cast<const uint2*>(a.resid + o);
    r[0] += to_f32<DT>(q.x & 0xffff); r[1] += to_f32<DT>(q.x >> 16);
    r[2] += to_f32<DT>(q.y & 0xffff); r[3] += to_f32<DT>(q.y >> 16);
  }
  uint2 st;
  st.x = (uint32_t)from_f32<DT>(r[0]) | ((uint32_t)from_f32<DT>(r[1]) << 16);
  st.y = (uint32_t)from_f32<DT>(r[2]) | ((uint32_t)from_f32<DT>(r[3]) << 16);
  *reinterpret_cast<uint2*>(a.out + o) = st;
}

template <int DT, int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(ConvArgs a) {
  constexpr int FM = BM / 32, FN = BN / 32;  // 16x16 fragments per wave (2x2 waves)
  constexpr int LA = BM / 32, LB = BN / 32;  // 16-byte chunks staged per thread per operand
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (BM + BN) * kCBK];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware remap (bijective for any tile count): logical tiles that share
  // an XCD are contiguous, and consecutive logical tiles share the pixel tile.
  int bid = blockIdx.x;
  {
    const int nwg = a.tiles_m * a.tiles_n, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int m0 = (bid % a.tiles_m) * BM, n0 = (bid / a.tiles_m) * BN;
  const int s_beg = blockIdx.y * a.ks_per_split;
  const int s_end = min(a.ksteps, s_beg + a.ks_per_split);

  // per-thread staging rows: chunk c of rows rb + 32*i
  const int c = tid & 7, rb = tid >> 3;
  const int cpt = a.IC >> 6;  // k-steps per tap
  const int VH = a.H << a.up, VW = a.W << a.up;
  const uint16_t* wrow[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int oc = m0 + rb + 32 * i;
    wrow[i] = oc < a.OC ? a.w + (size_t)oc * a.KH * a.KW * a.IC + c * 8 : nullptr;
  }
  int piy[LB], pix[LB];
  const uint16_t* pbase[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int p = n0 + rb + 32 * i;
    if (p < a.P) {
      const int hw = a.OH * a.OW, n = p / hw, rem = p - n * hw, oy = rem / a.OW, ox = rem - oy * a.OW;
      piy[i] = oy * a.stride - a.pad;
      pix[i] = ox * a.stride - a.pad;
      pbase[i] = a.x + (size_t)n * a.H * a.W * a.IC + c * 8;
    } else {
      piy[i] = -(1 << 28);  // never in bounds
      pix[i] = 0;
      pbase[i] = a.x;
    }
  }

  uint4 ra[LA], rbv[LB];
  auto gload = [&](int s) {
    const int tap = s / cpt, icb = (s - tap * cpt) << 6;
    const int ky = tap / a.KW, kx = tap - ky * a.KW;
#pragma unroll
    for (int i = 0; i < LA; ++i)
      ra[i] = wrow[i] ? *reinterpret_cast<const uint4*>(wrow[i] + (size_t)s * kCBK) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int iy = piy[i] + ky, ix = pix[i] + kx;
      if (iy >= 0 && iy < VH && ix >= 0 && ix < VW)
        rbv[i] = *reinterpret_cast<const uint4*>(
            pbase[i] + ((size_t)(iy >> a.up) * a.W + (ix >> a.up)) * a.IC + icb);
      else
        rbv[i] = make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
    uint16_t* As = smem + buf * (BM + BN) * kCBK;
    uint16_t* Bs = As + BM * kCBK;
#pragma unroll
    for (int i = 0; i < LA; ++i) *reinterpret_cast<uint4*>(As + swz(rb + 32 * i, c)) = ra[i];
#pragma unroll
    for (int i = 0; i < LB; ++i) *reinterpret_cast<uint4*>(Bs + swz(rb + 32 * i, c)) = rbv[i];
  };

  cf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};

  if (s_beg < s_end) {
    gload(s_beg);
    sstore(0);
    __syncthreads();
  }
  for (int s = s_beg; s < s_end; ++s) {
    const int buf = (s - s_beg) & 1;
    const bool more = s + 1 < s_end;
    if (more) gload(s + 1);
    const uint16_t* As = smem + buf * (BM + BN) * kCBK;
    const uint16_t* Bs = As + BM * kCBK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + swz(wm * (BM / 2) + i * 16 + l16, ks * 4 + g4));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bf[j] = *reinterpret_cast<const uint4*>(Bs + swz(wn * (BN / 2) + j * 16 + l16, ks * 4 + g4));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = cmfma<DT>(af[i], bf[j], acc[i][j]);
    }
    if (more) sstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds oc = base + 4*g4 + r (r = 0..3) of pixel base + l16
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int oc = m0 + wm * (BM / 2) + i * 16 + 4 * g4;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = n0 + wn * (BN / 2) + j * 16 + l16;
      if (oc >= a.OC || p >= a.P) continue;
      const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (gridDim.y > 1) {
        *reinterpret_cast<float4*>(a.ws + ((size_t)blockIdx.y * a.P + p) * a.OC + oc) =
            make_float4(v[0], v[1], v[2], v[3]);
      } else {
        conv_epilogue<DT>(a, oc, p, v);
      }
    }
  }
}


// Same GEMM with LDS-DMA staging (global_load_lds_dwordx4): no VGPR round trip
// and no ds_write pass.  The LDS image stays lane-linear per wave instruction
// (8 rows x 128 B = 1 KiB); the XOR swizzle is applied on the SOURCE address
// (lane L of a piece fetches logical chunk (L&7)^(L>>3) of row L>>3), and
// out-of-range rows / padding taps read a zero line.  Two buffers, two raw
// barriers per k-step: [issue s+1] -> vmcnt(pieces of s+1) -> barrier ->
// MFMAs on s -> lgkmcnt(0) -> barrier (WAR before s+2 overwrites).
template <int DT, int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv_glds_kernel(ConvArgs a) {
  constexpr int FM = BM / 32, FN = BN / 32;
  constexpr int IA = BM / 32, IB = BN / 32;  // 1-KiB pieces per wave per operand
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (BM + BN) * kCBK];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  int bid = blockIdx.x;
  {
    const int nwg = a.tiles_m * a.tiles_n, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int m0 = (bid % a.tiles_m) * BM, n0 = (bid / a.tiles_m) * BN;
  const int s_beg = blockIdx.y * a.ks_per_split;
  const int s_end = min(a.ksteps, s_beg + a.ks_per_split);

  const int lrow = lane >> 3, lch = (lane & 7) ^ lrow;
  const int cpt = a.IC >> 6;
  const int VH = a.H << a.up, VW = a.W << a.up;
  const uint16_t* zero = a.zeros;
  const uint16_t* wsrc[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int oc = m0 + (wave * IA + i) * 8 + lrow;
    wsrc[i] = oc < a.OC ? a.w + (size_t)oc * a.KH * a.KW * a.IC + lch * 8 : nullptr;
  }
  int piy[IB], pix[IB];
  const uint16_t* pbase[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int p = n0 + (wave * IB + i) * 8 + lrow;
    if (p < a.P) {
      const int hw = a.OH * a.OW, n = p / hw, rem = p - n * hw, oy = rem / a.OW, ox = rem - oy * a.OW;
      piy[i] = oy * a.stride - a.pad;
      pix[i] = ox * a.stride - a.pad;
      pbase[i] = a.x + (size_t)n * a.H * a.W * a.IC + lch * 8;
    } else {
      piy[i] = -(1 << 28);
      pix[i] = 0;
      pbase[i] = a.x;
    }
  }
  auto issue = [&](int s, int buf) {
    const int tap = s / cpt, icb = (s - tap * cpt) << 6;
    const int ky = tap / a.KW, kx = tap - ky * a.KW;
    uint16_t* As = smem + buf * (BM + BN) * kCBK;
    uint16_t* Bs = As + BM * kCBK;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const uint16_t* g = wsrc[i] ? wsrc[i] + (size_t)s * kCBK : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)(As + (wave * IA + i) * 8 * kCBK), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int iy = piy[i] + ky, ix = pix[i] + kx;
      const uint16_t* g = (iy >= 0 && iy < VH && ix >= 0 && ix < VW)
                              ? pbase[i] + ((size_t)(iy >> a.up) * a.W + (ix >> a.up)) * a.IC + icb
                              : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)(Bs + (wave * IB + i) * 8 * kCBK), 16, 0, 0);
    }
  };

  cf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};

  if (s_beg < s_end) issue(s_beg, 0);
  for (int s = s_beg; s < s_end; ++s) {
    const int buf = (s - s_beg) & 1;
    if (s + 1 < s_end) {
      issue(s + 1, buf ^ 1);
      __builtin_amdgcn_s_waitcnt(vm_wait(IA + IB));
    } else {
      __builtin_amdgcn_s_waitcnt(vm_wait(0));
    }
    asm volatile("s_barrier" ::: "memory");
    const uint16_t* As = smem + buf * (BM + BN) * kCBK;
    const uint16_t* Bs = As + BM * kCBK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + swz(wm * (BM / 2) + i * 16 + l16, ks * 4 + g4));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bf[j] = *reinterpret_cast<const uint4*>(Bs + swz(wn * (BN / 2) + j * 16 + l16, ks * 4 + g4));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = cmfma<DT>(af[i], bf[j], acc[i][j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int oc = m0 + wm * (BM / 2) + i * 16 + 4 * g4;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = n0 + wn * (BN / 2) + j * 16 + l16;
      if (oc >= a.OC || p >= a.P) continue;
      const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (gridDim.y > 1) {
        *reinterpret_cast<float4*>(a.ws + ((size_t)blockIdx.y * a.P + p) * a.OC + oc) =
            make_float4(v[0], v[1], v[2], v[3]);
      } else {
        conv_epilogue<DT>(a, oc, p, v);
      }
    }
  }
}

// Halo-tiled variant for stride-1 KxK convolutions (3x3 in every ResnetBlock2D
// and the fused-upsample conv).  A block owns BM output channels x a TH x TW
// spatial output tile of one image (TH*TW <= BN).  For each 64-channel input
// chunk the (TH+KH-1) x (TW+KW-1) input halo is staged ONCE by LDS-DMA and
// serves all KH*KW taps from LDS: the implicit-GEMM B operand is re-read
// through L2 once per chunk instead of once per tap (the im2col kernels above
// are L2-bandwidth bound at ~16 TB/s; this cuts their L2 bytes ~2.5x).
// Step order: s = chunk * taps + tap.  The halo of chunk c+1 is issued at tap 0
// of chunk c into the other halo buffer (a whole chunk of lookahead); the
// weight tile of step s+1 is issued during step s.
template <int DT, int BM, int BN, int WM, int WN, int HPW>
__global__ __launch_bounds__(64 * WM * WN, 8 / (WM * WN)) void conv_halo_kernel(
    ConvArgs a, int TH, int TW, int tiles_y, int tiles_x) {
  constexpr int NW = WM * WN;                       // waves
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;  // fragments per wave
  constexpr int IA = BM / 8 / NW;                   // weight pieces per wave per step
  constexpr int HROWS = HPW * NW * 8;               // halo rows per buffer
  static_assert(IA * 8 * NW == BM, "weight tile must split into whole pieces");
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (BM + HROWS) * kCBK];
  uint16_t* const Abuf = smem;                    // [2][BM][64]
  uint16_t* const Hbuf = smem + 2 * BM * kCBK;    // [2][HROWS][64]

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int wm = wave / WN, wn = wave % WN;
  int bid = blockIdx.x;
  {
    const int nwg = a.tiles_m * a.tiles_n, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int m0 = (bid % a.tiles_m) * BM;
  int t = bid / a.tiles_m;
  const int txi = t % tiles_x; t /= tiles_x;
  const int tyi = t % tiles_y;
  const int n = t / tiles_y;
  const int oy0 = tyi * TH, ox0 = txi * TW;
  const int HW_ = TW + a.KW - 1;          // halo width
  const int HR = (TH + a.KH - 1) * HW_;   // halo rows in use
  const int VH = a.H << a.up, VW = a.W << a.up;
  const int taps = a.KH * a.KW, nchunk = a.IC >> 6;
  const int nsteps = taps * nchunk;

  const int lrow = lane >> 3, lch = (lane & 7) ^ lrow;
  const uint16_t* zero = a.zeros;
  // weight rows of this lane's pieces
  const uint16_t* wsrc[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int oc = m0 + (wave * IA + i) * 8 + lrow;
    wsrc[i] = oc < a.OC ? a.w + (size_t)oc * taps * a.IC + lch * 8 : nullptr;
  }
  // halo rows of this lane's pieces: element offset of the input pixel, or -1
  long long hoff[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int r = (wave * HPW + i) * 8 + lrow;
    hoff[i] = -1;
    if (r < HR) {
      const int hy = r / HW_, hx = r - hy * HW_;
      const int vy = oy0 - a.pad + hy, vx = ox0 - a.pad + hx;
      if (vy >= 0 && vy < VH && vx >= 0 && vx < VW)
        hoff[i] = (((long long)n * a.H + (vy >> a.up)) * a.W + (vx >> a.up)) * a.IC + lch * 8;
    }
  }
  auto issue_w = [&](int s, int buf) {
    const int chunk = s / taps, tap = s - chunk * taps;
    const size_t koff = (size_t)tap * a.IC + chunk * kCBK;
    uint16_t* As = Abuf + buf * BM * kCBK;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const uint16_t* g = wsrc[i] ? wsrc[i] + koff : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)(As + (wave * IA + i) * 8 * kCBK), 16, 0, 0);
    }
  };
  auto issue_h = [&](int chunk, int buf) {
    uint16_t* Hs = Hbuf + buf * HROWS * kCBK;
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const uint16_t* g = hoff[i] >= 0 ? a.x + hoff[i] + chunk * kCBK : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)(Hs + (wave * HPW + i) * 8 * kCBK), 16, 0, 0);
    }
  };

  // this lane's B-fragment halo rows at tap (0,0)
  int hb[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int pi = wn * (BN / WN) + j * 16 + l16;
    const int ty = pi / TW, tx = pi - ty * TW;
    hb[j] = pi < TH * TW ? ty * HW_ + tx : 0;
  }

  cf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = cf32x4{0.f, 0.f, 0.f, 0.f};

  issue_h(0, 0);
  issue_w(0, 0);
  for (int s = 0; s < nsteps; ++s) {
    const int chunk = s / taps, tap = s - chunk * taps;
    const bool more = s + 1 < nsteps;
    const bool next_halo = tap == 0 && chunk + 1 < nchunk;
    if (next_halo) issue_h(chunk + 1, (chunk + 1) & 1);
    if (more) issue_w(s + 1, (s + 1) & 1);
    if (more && next_halo) __builtin_amdgcn_s_waitcnt(vm_wait(IA + HPW));
    else if (more) __builtin_amdgcn_s_waitcnt(vm_wait(IA));
    else __builtin_amdgcn_s_waitcnt(vm_wait(0));
    asm volatile("s_barrier" ::: "memory");
    const uint16_t* As = Abuf + (s & 1) * BM * kCBK;
    const uint16_t* Hs = Hbuf + (chunk & 1) * HROWS * kCBK;
    const int ky = tap / a.KW, kx = tap - ky * a.KW;
    const int toff = ky * HW_ + kx;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + swz(wm * (BM / WM) + i * 16 + l16, ks * 4 + g4));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bf[j] = *reinterpret_cast<const uint4*>(Hs + swz(hb[j] + toff, ks * 4 + g4));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = cmfma<DT>(af[i], bf[j], acc[i][j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int pi = wn * (BN / WN) + j * 16 + l16;
    const int ty = pi / TW, tx = pi - ty * TW;
    const int oy = oy0 + ty, ox = ox0 + tx;
    if (pi >= TH * TW || oy >= a.OH || ox >= a.OW) continue;
    const int p = (n * a.OH + oy) * a.OW + ox;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int oc = m0 + wm * (BM / WM) + i * 16 + 4 * g4;
      if (oc >= a.OC) continue;
      const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      conv_epilogue<DT>(a, oc, p, v);
    }
  }
}

// split-K combine: one thread per 4 output channels of one pixel
template <int DT>
__global__ __launch_bounds__(256) void conv_splitk_finalize(ConvArgs a, int splits) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)a.P * (a.OC >> 2);
  if (q >= total) return;
  const int p = (int)(q / (a.OC >> 2)), oc = (int)(q % (a.OC >> 2)) * 4;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < splits; ++s) {
    const float4 t = *reinterpret_cast<const float4*>(a.ws + ((size_t)s * a.P + p) * a.OC + oc);
    v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
  }
  conv_epilogue<DT>(a, oc, p, v);
}

// Direct 3x3 convolution for the few-input-channel layers (UNet / VAE conv_in on
// the 4 latent channels, the VAE encoder's RGB input): K = 9 * IC is too short
// for the implicit GEMM's 64-wide K steps, and the work is small (P x OC x 36
// FMAs), so it runs on the VALU.  The whole filter sits in LDS as f32
// [9*IC][OC]; a thread owns 8 output channels of one pixel (channel group
// fastest, so a wave's stores are contiguous), keeps its 9*IC input taps in
// registers and reads the filter rows as LDS broadcasts / 32-byte vectors.
// Bias, per-sample bias2 and the residual are fused as in conv_epilogue.
constexpr int kSmallCMaxW = 18432;  // f32 filter elements in LDS (72 KB: OC <= 512 at IC = 4)

template <int DT, int IC>
__global__ __launch_bounds__(256) void conv_smallc_kernel(ConvArgs a) {
  constexpr int KK = 9 * IC;
  __shared__ __attribute__((aligned(16))) float wsm[kSmallCMaxW];
  const int OC = a.OC;
  for (int i = threadIdx.x; i < KK * OC; i += 256) {
    const int k = i / OC, oc = i - k * OC;  // packed w [OC][3][3][IC]: k = (kh*3+kw)*IC + ic
    wsm[i] = to_f32<DT>(a.w[(size_t)oc * KK + k]);
  }
  __syncthreads();
  const int G = OC >> 3, ohw = a.OH * a.OW;
  const long long total = (long long)a.P * G;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (long long)gridDim.x * 256) {
    const int p = (int)(t / G), og = (int)(t - (long long)p * G);
    const int n = p / ohw, r = p - n * ohw, oh = r / a.OW, ow = r - oh * a.OW;
    float xin[KK];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ih = oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
        const bool ok = ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
        const int ihc = ok ? ih : 0, iwc = ok ? iw : 0;
        if (a.in_nchw) {  // planar input (the UNet's external layout)
          const size_t plane = (size_t)a.H * a.W;
          const uint16_t* src = a.x + (size_t)n * IC * plane + (size_t)ihc * a.W + iwc;
#pragma unroll
          for (int c = 0; c < IC; ++c)
            xin[(kh * 3 + kw) * IC + c] = ok ? to_f32<DT>(src[c * plane]) : 0.f;
        } else {
          const uint16_t* src = a.x + (((size_t)n * a.H + ihc) * a.W + iwc) * IC;
#pragma unroll
          for (int c = 0; c < IC; ++c) xin[(kh * 3 + kw) * IC + c] = ok ? to_f32<DT>(src[c]) : 0.f;
        }
      }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float* wr = wsm + og * 8;
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      const float4 w0 = *reinterpret_cast<const float4*>(wr + k * OC);
      const float4 w1 = *reinterpret_cast<const float4*>(wr + k * OC + 4);
      acc[0] = fmaf(xin[k], w0.x, acc[0]); acc[1] = fmaf(xin[k], w0.y, acc[1]);
      acc[2] = fmaf(xin[k], w0.z, acc[2]); acc[3] = fmaf(xin[k], w0.w, acc[3]);
      acc[4] = fmaf(xin[k], w1.x, acc[4]); acc[5] = fmaf(xin[k], w1.y, acc[5]);
      acc[6] = fmaf(xin[k], w1.z, acc[6]); acc[7] = fmaf(xin[k], w1.w, acc[7]);
    }
    conv_epilogue<DT>(a, og * 8, p, acc);
    conv_epilogue<DT>(a, og * 8 + 4, p, acc + 4);
  }
}

// ---------------------------------------------------------------------------
// 1x1 convolution with few channels (IC, OC <= 16): the VAE's quant_conv (8 -> 8) and
// post_quant_conv (4 -> 4) on the latent — a per-pixel 16x16 matrix-vector product,
// bandwidth-bound, so one thread per pixel on the VALU with the filter in LDS (f32).
// Either side may be planar (NCHW: the module's external layout, read / written here
// instead of a layout-copy kernel) or channels-last.
// ---------------------------------------------------------------------------
constexpr int kPwMaxC = 16;

template <int DT>
__global__ __launch_bounds__(256) void conv1x1_small_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ w,
                                                            const uint16_t* __restrict__ bias,
                                                            uint16_t* __restrict__ out, int N,
                                                            int HW, int IC, int OC, int in_nchw,
                                                            int out_nchw) {
  __shared__ float wsm[kPwMaxC * kPwMaxC + kPwMaxC];
  for (int i = threadIdx.x; i < IC * OC; i += 256) wsm[i] = to_f32<DT>(w[i]);
  if (threadIdx.x < OC) wsm[kPwMaxC * kPwMaxC + threadIdx.x] = bias ? to_f32<DT>(bias[threadIdx.x]) : 0.f;
  __syncthreads();
  const long long P = (long long)N * HW;
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < P; p += (long long)gridDim.x * 256) {
    const int n = (int)(p / HW), r = (int)(p - (long long)n * HW);
    float xin[kPwMaxC];
#pragma unroll
    for (int c = 0; c < kPwMaxC; ++c)
      xin[c] = c < IC ? to_f32<DT>(in_nchw ? x[((size_t)n * IC + c) * HW + r] : x[(size_t)p * IC + c])
                      : 0.f;
#pragma unroll
    for (int o = 0; o < kPwMaxC; ++o) {
      if (o >= OC) break;
      float acc = wsm[kPwMaxC * kPwMaxC + o];
#pragma unroll
      for (int c = 0; c < kPwMaxC; ++c)
        if (c < IC) acc = fmaf(wsm[o * IC + c], xin[c], acc);
      const uint16_t v = from_f32<DT>(acc);
      if (out_nchw) out[((size_t)n * OC + o) * HW + r] = v;
      else out[(size_t)p * OC + o] = v;
    }
  }
}

}  // namespace cake

using namespace cake;

// x [N, IC, HW] (layout bit 0) or [N, HW, IC]; w [OC, IC]; out [N, OC, HW] (bit 1) or
// [N, HW, OC]; IC, OC in 1..16.
CAKE_API int cake_conv1x1_small(int dt, const void* x, const void* w, const void* bias, void* out,
                                int N, int HW, int IC, int OC, int layout, hipStream_t st) {
  if (IC < 1 || IC > kPwMaxC || OC < 1 || OC > kPwMaxC || N <= 0 || HW <= 0 || layout < 0 ||
      layout > 3)
    return (int)hipErrorInvalidValue;
  const long long P = (long long)N * HW;
  const unsigned grid = (unsigned)std::min<long long>((P + 255) / 256, 4096);
#define CAKE_PW(DTV)                                                                          \
  hipLaunchKernelGGL((conv1x1_small_kernel<DTV>), dim3(grid), dim3(256), 0, st,              \
                     (const uint16_t*)x, (const uint16_t*)w, (const uint16_t*)bias,          \
                     (uint16_t*)out, N, HW, IC, OC, layout & 1, (layout >> 1) & 1)
  if (dt == kBF16) CAKE_PW(kBF16);
  else if (dt == kF16) CAKE_PW(kF16);
  else return (int)hipErrorInvalidValue;
#undef CAKE_PW
  return (int)hipGetLastError();
}

// Workspace (f32 elements) the launcher needs for split-K with `splits` > 1.
CAKE_API long long cake_conv2d_workspace(int P, int OC, int splits) {
  return splits > 1 ? (long long)splits * P * OC : 0;
}

// cfg: 0 = 128x128, 1 = 64x128, 2 = 128x64, 3 = 64x64 (oc x pixel tile);
//      +4 = the same tiles with LDS-DMA staging (needs `zeros`);
//      8/9 = halo kernel, 128/64 oc x (th x tw <= 128 pixels), 10/11 = 128/64 oc x
//      (th x tw <= 64 pixels), 12/13 = 128/64 oc x (th x tw <= 256 pixels, 8 waves);
//      stride 1 only, no split-K; 14 = direct 3x3 kernel for IC 3 / 4 (conv_in).
// layout: bit 0 = x NCHW (cfg 14 only), bit 1 = out NCHW (no resid)
CAKE_API int cake_conv2d_nhwc2(int dt, const void* x, const void* w, const void* bias,
                               const float* bias2, const void* resid, void* out, float* ws,
                               const void* zeros,
                               int N, int H, int W, int IC, int OC, int KH, int KW, int stride,
                               int pad, int up, int cfg, int splits, int th, int tw,
                               int bias2_ld, int layout, hipStream_t st) {
  const int in_nchw = layout & 1, out_nchw = (layout >> 1) & 1;
  if ((in_nchw && cfg != 14) || (out_nchw && resid) || layout < 0 || layout > 3)
    return (int)hipErrorInvalidValue;
  if (cfg == 14) {  // direct small-IC 3x3 kernel
    if ((IC != 3 && IC != 4) || KH != 3 || KW != 3 || OC % 8 || 9 * IC * OC > kSmallCMaxW ||
        N <= 0 || stride <= 0 || up || (bias2 && bias2_ld > 0 && (bias2_ld % 4 || bias2_ld < OC)))
      return (int)hipErrorInvalidValue;
    const int OH = (H + 2 * pad - 3) / stride + 1, OW = (W + 2 * pad - 3) / stride + 1;
    if (OH <= 0 || OW <= 0) return (int)hipErrorInvalidValue;
    ConvArgs a{(const uint16_t*)x, (const uint16_t*)w, (const uint16_t*)bias, bias2,
               (const uint16_t*)resid, (uint16_t*)out, nullptr, nullptr, N, H, W, IC, OC, OH, OW,
               3, 3, stride, pad, 0, N * OH * OW, 0, 0, 0, 0};
    a.bias2_ld = bias2_ld > 0 ? bias2_ld : OC;
    a.in_nchw = in_nchw;
    a.out_nchw = out_nchw;
    const long long work = (long long)a.P * (OC / 8);
    const unsigned grid = (unsigned)std::min<long long>((work + 255) / 256, 2048);
#define CAKE_SMALLC(DTV)                                                                         \
    if (IC == 3) hipLaunchKernelGGL((conv_smallc_kernel<DTV, 3>), dim3(grid), dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((conv_smallc_kernel<DTV, 4>), dim3(grid), dim3(256), 0, st, a);
    if (dt == kBF16) { CAKE_SMALLC(kBF16); }
    else if (dt == kF16) { CAKE_SMALLC(kF16); }
    else return (int)hipErrorInvalidValue;
#undef CAKE_SMALLC
    return (int)hipGetLastError();
  }
  if (IC % 64 || OC % 4 || N <= 0 || stride <= 0 || KH <= 0 || KW <= 0 || splits <= 0 ||
      (bias2 && bias2_ld > 0 && (bias2_ld % 4 || bias2_ld < OC)) ||
      (up && stride != 1) || cfg < 0 || cfg > 13 || (splits > 1 && !ws) || (cfg > 3 && !zeros))
    return (int)hipErrorInvalidValue;
  const int VH = H << up, VW = W << up;
  const int OH = (VH + 2 * pad - KH) / stride + 1, OW = (VW + 2 * pad - KW) / stride + 1;
  if (OH <= 0 || OW <= 0) return (int)hipErrorInvalidValue;
  if (cfg >= 8) {
    const int bn = cfg >= 12 ? 256 : cfg < 10 ? 128 : 64, bm = (cfg & 1) ? 64 : 128;
    const int hrows = cfg >= 12 ? 384 : (cfg < 10 ? 6 : 4) * 32;
    const int nthr = cfg >= 12 ? 512 : 256;
    if (stride != 1 || th <= 0 || tw <= 0 || th * tw > bn || (th + KH - 1) * (tw + KW - 1) > hrows)
      return (int)hipErrorInvalidValue;
    const int ty = (OH + th - 1) / th, tx = (OW + tw - 1) / tw;
    ConvArgs a{(const uint16_t*)x, (const uint16_t*)w, (const uint16_t*)bias, bias2,
               (const uint16_t*)resid, (uint16_t*)out, nullptr, (const uint16_t*)zeros, N, H, W,
               IC, OC, OH, OW, KH, KW, 1, pad, up, N * OH * OW, KH * KW * (IC / 64), 0,
               (OC + bm - 1) / bm, N * ty * tx};
    a.bias2_ld = bias2_ld > 0 ? bias2_ld : OC;
    a.in_nchw = in_nchw;
    a.out_nchw = out_nchw;
    const dim3 grid(a.tiles_m * a.tiles_n);
#define CAKE_HALO(DTV)                                                                                     \
    switch (cfg) {                                                                                         \
      case 8: hipLaunchKernelGGL((conv_halo_kernel<DTV, 128, 128, 2, 2, 6>), grid, dim3(nthr), 0, st, a, th, tw, ty, tx); break; \
      case 9: hipLaunchKernelGGL((conv_halo_kernel<DTV, 64, 128, 2, 2, 6>), grid, dim3(nthr), 0, st, a, th, tw, ty, tx); break;  \
      case 10: hipLaunchKernelGGL((conv_halo_kernel<DTV, 128, 64, 2, 2, 4>), grid, dim3(nthr), 0, st, a, th, tw, ty, tx); break; \
      case 11: hipLaunchKernelGGL((conv_halo_kernel<DTV, 64, 64, 2, 2, 4>), grid, dim3(nthr), 0, st, a, th, tw, ty, tx); break;  \
      case 12: hipLaunchKernelGGL((conv_halo_kernel<DTV, 128, 256, 2, 4, 6>), grid, dim3(nthr), 0, st, a, th, tw, ty, tx); break; \
      default: hipLaunchKernelGGL((conv_halo_kernel<DTV, 64, 256, 2, 4, 6>), grid, dim3(nthr), 0, st, a, th, tw, ty, tx); break;  \
    }
    if (dt == kBF16) { CAKE_HALO(kBF16); }
    else if (dt == kF16) { CAKE_HALO(kF16); }
    else return (int)hipErrorInvalidValue;
#undef CAKE_HALO
    return (int)hipGetLastError();
  }
  static const int BMs[8] = {128, 64, 128, 64, 128, 64, 128, 64};
  static const int BNs[8] = {128, 128, 64, 64, 128, 128, 64, 64};
  ConvArgs a{(const uint16_t*)x, (const uint16_t*)w, (const uint16_t*)bias, bias2,
             (const uint16_t*)resid, (uint16_t*)out, ws, (const uint16_t*)zeros, N, H, W, IC, OC, OH, OW, KH, KW,
             stride, pad, up, N * OH * OW, KH * KW * (IC / 64), 0, 0, 0};
  a.bias2_ld = bias2_ld > 0 ? bias2_ld : OC;
    a.in_nchw = in_nchw;
    a.out_nchw = out_nchw;
  a.tiles_m = (OC + BMs[cfg] - 1) / BMs[cfg];
  a.tiles_n = (a.P + BNs[cfg] - 1) / BNs[cfg];
  splits = splits > a.ksteps ? a.ksteps : splits;
  a.ks_per_split = (a.ksteps + splits - 1) / splits;
  splits = (a.ksteps + a.ks_per_split - 1) / a.ks_per_split;
  const dim3 grid(a.tiles_m * a.tiles_n, splits);
#define CAKE_CONV(DTV)                                                                        \
  do {                                                                                        \
    switch (cfg) {                                                                            \
      case 0: hipLaunchKernelGGL((conv_igemm_kernel<DTV, 128, 128>), grid, dim3(256), 0, st, a); break; \
      case 1: hipLaunchKernelGGL((conv_igemm_kernel<DTV, 64, 128>), grid, dim3(256), 0, st, a); break;  \
      case 2: hipLaunchKernelGGL((conv_igemm_kernel<DTV, 128, 64>), grid, dim3(256), 0, st, a); break;  \
      case 3: hipLaunchKernelGGL((conv_igemm_kernel<DTV, 64, 64>), grid, dim3(256), 0, st, a); break;  \
      case 4: hipLaunchKernelGGL((conv_glds_kernel<DTV, 128, 128>), grid, dim3(256), 0, st, a); break; \
      case 5: hipLaunchKernelGGL((conv_glds_kernel<DTV, 64, 128>), grid, dim3(256), 0, st, a); break;  \
      case 6: hipLaunchKernelGGL((conv_glds_kernel<DTV, 128, 64>), grid, dim3(256), 0, st, a); break;  \
      default: hipLaunchKernelGGL((conv_glds_kernel<DTV, 64, 64>), grid, dim3(256), 0, st, a); break;  \
    }                                                                                         \
    if (splits > 1) {                                                                         \
      const size_t total = (size_t)a.P * (OC / 4);                                            \
      hipLaunchKernelGGL((conv_splitk_finalize<DTV>), dim3((unsigned)((total + 255) / 256)),   \
                         dim3(256), 0, st, a, splits);                                        \
    }                                                                                         \
  } while (0)
  if (dt == kBF16) CAKE_CONV(kBF16);
  else if (dt == kF16) CAKE_CONV(kF16);
  else return (int)hipErrorInvalidValue;
#undef CAKE_CONV
  return (int)hipGetLastError();
}

CAKE_API int cake_conv2d_nhwc(int dt, const void* x, const void* w, const void* bias,
                              const float* bias2, const void* resid, void* out, float* ws,
                              const void* zeros,
                              int N, int H, int W, int IC, int OC, int KH, int KW, int stride,
                              int pad, int up, int cfg, int splits, int th, int tw,
                              int bias2_ld, hipStream_t st) {
  return cake_conv2d_nhwc2(dt, x, w, bias, bias2, resid, out, ws, zeros, N, H, W, IC, OC, KH, KW,
                           stride, pad, up, cfg, splits, th, tw, bias2_ld, 0, st);
}
