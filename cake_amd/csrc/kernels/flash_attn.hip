// Flash-attention forward on MFMA (gfx950 v_mfma_f32_16x16x32_{bf16,f16}).
//
// One kernel serves every multi-query attention in the framework:
//   * Llama prefill (causal, offset-aware positions, GQA via kv-head index,
//     reading K/V straight from the [nkv][S][hd] KV cache) — replaces the
//     reference's materialised [nh,T,Tk] f32 scores + 5-launch softmax
//     (cake-core/src/models/llama3/attention.rs:96-118);
//   * Stable Diffusion self/cross attention (SpatialTransformer, head dims
//     40/64/80/160) and the CLIP causal attention.
// Tensors are addressed through (batch, head, row) element strides, so the
// projection outputs are consumed in place ([B, N, H*D] layouts) with no
// permute/contiguous copies.
//
// Tiling: workgroup = 4 waves = 64 query rows (16 per wave), key tiles of 64.
// Q lives in registers as MFMA A-fragments; each K tile is staged in LDS
// (row-padded: conflict-free 16-byte reads), V is staged TRANSPOSED so both
// PV operands are contiguous 16-byte LDS reads.  S = Q·Kᵀ runs as 4 16x16
// MFMA tiles per wave; the online softmax (exp2 domain) works directly on the
// accumulator layout (row = 4*(lane>>4)+r, col = lane&15) — the O accumulator
// shares that row layout, so the rescale is a per-register multiply.  P goes
// through a small per-wave LDS tile to become the A operand of P·V.
// DP = head dim padded to a multiple of 32 (zero-filled, never stored).
#include "common.h"

namespace cake {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct FlashArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  int B, H, Hkv, N, M, D;
  long long q_sb, q_sh, q_sn;
  long long k_sb, k_sh, k_sn;
  long long v_sb, v_sh, v_sn;
  long long o_sb, o_sh, o_sn;
  float scale_log2;  // softmax scale * log2(e)
  int causal;
  int pos0;          // absolute position of query row 0 (keys start at 0)
};

constexpr int kBM = 64, kBN = 64, kKP = 8;  // rows, keys, LDS row pad (elements)

template <int DT>
__device__ __forceinline__ f32x4 mfma16(const uint4 a, const uint4 b, f32x4 c) {
  if constexpr (DT == kBF16) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
}

template <int DT, int DP>
__global__ __launch_bounds__(256) void flash_fwd_kernel(FlashArgs a) {
  constexpr int KS = DP / 32;   // k-steps of Q·Kᵀ
  constexpr int DT16 = DP / 16; // output column tiles
  __shared__ __attribute__((aligned(16))) uint16_t Ks[kBN * (DP + kKP)];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[DP * (kBN + kKP)];
  __shared__ __attribute__((aligned(16))) uint16_t Ps[4 * 16 * (kBN + kKP)];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.x * kBM;
  const int h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (a.H / a.Hkv);
  const uint16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const uint16_t* kb = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vb = a.v + b * a.v_sb + hk * a.v_sh;
  const bool d_vec = (a.D % 8) == 0;

  // Q fragments (A operand): row = l16, k = ks*32 + 8*g4 + j
  uint4 qf[KS];
  {
    const int row = m0 + wave * 16 + l16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = ks * 32 + 8 * g4;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < a.N && d0 < a.D) {
        const uint16_t* p = qb + (long long)row * a.q_sn + d0;
        if (d_vec) v = *reinterpret_cast<const uint4*>(p);
        else {
          uint16_t t[8];
          for (int j = 0; j < 8; ++j) t[j] = d0 + j < a.D ? p[j] : 0;
          v = *reinterpret_cast<uint4*>(t);
        }
      }
      qf[ks] = v;
    }
  }

  f32x4 acc[DT16];
#pragma unroll
  for (int t = 0; t < DT16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mrow[r] = -INFINITY; lrow[r] = 0.f; }

  int kend = a.M;
  if (a.causal) kend = min(kend, a.pos0 + m0 + kBM);
  uint16_t* pw = Ps + wave * 16 * (kBN + kKP);

  for (int kt = 0; kt < kend; kt += kBN) {
    // ---- stage K (row-major, padded) and V (transposed) into LDS
    constexpr int CH = DP / 8;  // 16-byte chunks per row
    for (int i = tid; i < kBN * CH; i += 256) {
      const int r = i / CH, c = i - r * CH;
      const int key = kt + r, d0 = c * 8;
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (key < a.M && d0 < a.D) {
        const uint16_t* kp = kb + (long long)key * a.k_sn + d0;
        const uint16_t* vp = vb + (long long)key * a.v_sn + d0;
        if (d_vec) {
          kv = *reinterpret_cast<const uint4*>(kp);
          vv = *reinterpret_cast<const uint4*>(vp);
        } else {
          uint16_t tk[8], tv[8];
          for (int j = 0; j < 8; ++j) {
            tk[j] = d0 + j < a.D ? kp[j] : 0;
            tv[j] = d0 + j < a.D ? vp[j] : 0;
          }
          kv = *reinterpret_cast<uint4*>(tk);
          vv = *reinterpret_cast<uint4*>(tv);
        }
      }
      *reinterpret_cast<uint4*>(Ks + r * (DP + kKP) + d0) = kv;
      const uint16_t* ve = reinterpret_cast<const uint16_t*>(&vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) Vt[(d0 + j) * (kBN + kKP) + r] = ve[j];
    }
    __syncthreads();

    // ---- S = Q Kᵀ  (4 tiles of 16 keys)
    f32x4 s[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const uint16_t* krow = Ks + (nt * 16 + l16) * (DP + kKP) + 8 * g4;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        s[nt] = mfma16<DT>(qf[ks], *reinterpret_cast<const uint4*>(krow + ks * 32), s[nt]);
    }

    // ---- mask + online softmax (rows 4*g4 + r, columns l16 of each tile)
    float tmax[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qi = a.pos0 + m0 + wave * 16 + 4 * g4 + r;
      float mx = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int kj = kt + nt * 16 + l16;
        float x = s[nt][r] * a.scale_log2;
        if (kj >= a.M || (a.causal && kj > qi)) x = -INFINITY;
        s[nt][r] = x;
        mx = fmaxf(mx, x);
      }
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      tmax[r] = mx;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(mrow[r], tmax[r]);
      const float alpha = mn == -INFINITY ? 1.f : exp2f(mrow[r] - mn);
      float rs = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float p = mn == -INFINITY ? 0.f : exp2f(s[nt][r] - mn);
        s[nt][r] = p;
        rs += p;
      }
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) rs += __shfl_xor(rs, off, 64);
      lrow[r] = lrow[r] * alpha + rs;
      mrow[r] = mn;
#pragma unroll
      for (int t = 0; t < DT16; ++t) acc[t][r] *= alpha;
    }

    // ---- P -> LDS (per wave), then O += P V
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pw[(4 * g4 + r) * (kBN + kKP) + nt * 16 + l16] = from_f32<DT>(s[nt][r]);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes done
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < kBN / 32; ++ks) {
      const uint4 pa = *reinterpret_cast<const uint4*>(pw + l16 * (kBN + kKP) + ks * 32 + 8 * g4);
#pragma unroll
      for (int t = 0; t < DT16; ++t) {
        const uint4 vbf =
            *reinterpret_cast<const uint4*>(Vt + (t * 16 + l16) * (kBN + kKP) + ks * 32 + 8 * g4);
        acc[t] = mfma16<DT>(pa, vbf, acc[t]);
      }
    }
    __syncthreads();  // Ks/Vt/Ps reused by the next tile
  }

  // ---- epilogue: O / l
  uint16_t* ob = a.o + b * a.o_sb + h * a.o_sh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + wave * 16 + 4 * g4 + r;
    if (row >= a.N) continue;
    const float inv = lrow[r] > 0.f ? 1.f / lrow[r] : 0.f;
#pragma unroll
    for (int t = 0; t < DT16; ++t) {
      const int d = t * 16 + l16;
      if (d < a.D) ob[(long long)row * a.o_sn + d] = from_f32<DT>(acc[t][r] * inv);
    }
  }
}

}  // namespace cake

using namespace cake;

template <int DT>
static int launch_flash(const FlashArgs& a, hipStream_t st) {
  const dim3 grid((a.N + kBM - 1) / kBM, a.H, a.B);
  const int dp = ((a.D + 31) / 32) * 32;
#define CAKE_FL(P) \
  hipLaunchKernelGGL((flash_fwd_kernel<DT, P>), grid, dim3(256), 0, st, a); break;
  switch (dp) {
    case 32: CAKE_FL(32)
    case 64: CAKE_FL(64)
    case 96: CAKE_FL(96)
    case 128: CAKE_FL(128)
    case 160: CAKE_FL(160)
    case 192: CAKE_FL(192)
    case 256: CAKE_FL(256)
    default: return (int)hipErrorInvalidValue;
  }
#undef CAKE_FL
  return (int)hipGetLastError();
}

// strides in ELEMENTS: s[0]=batch, s[1]=head, s[2]=row for q, k, v, o (12 values)
CAKE_API int cake_flash_attn(int dt, const void* q, const void* k, const void* v, void* o, int B,
                             int H, int Hkv, int N, int M, int D, const long long* strides,
                             float scale, int causal, int pos0, hipStream_t st) {
  if (H <= 0 || Hkv <= 0 || H % Hkv || D <= 0 || D > 256 || N <= 0 || M <= 0)
    return (int)hipErrorInvalidValue;
  FlashArgs a{(const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o,
              B, H, Hkv, N, M, D,
              strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
              strides[6], strides[7], strides[8], strides[9], strides[10], strides[11],
              scale * 1.4426950408889634f, causal, pos0};
  if (dt == kBF16) return launch_flash<kBF16>(a, st);
  if (dt == kF16) return launch_flash<kF16>(a, st);
  return (int)hipErrorInvalidValue;
}
