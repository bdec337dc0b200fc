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

#include <cstdlib>

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
  int pair;          // v2 causal: workgroup x runs q tiles x and n-1-x (equal work)
  // v2 non-causal key split (grid.z = B * ksplit): split s walks keys [s*kchunk, (s+1)*kchunk)
  // and writes its normalised f32 O rows to po and their log2-sum-exp to plse
  // ([B * ksplit][H][N](D)); flash_merge_kernel combines the splits.
  int ksplit = 1, kchunk = 0;
  float* po = nullptr;
  float* plse = nullptr;
  long long ws_bytes = 0;  // host: bytes at po (ksplit * B * H * N * (D + 1) f32)
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

// ---------------------------------------------------------------------------
// v2: 32x32x16 MFMA, swapped QKᵀ, P straight from the accumulators.
//
// Workgroup = 4 waves x 32 query rows; key tiles of 64 (two 32-key subtiles).
// Per wave and tile:
//   Sᵀ[key][q] = K·Qᵀ            (A = K rows from LDS, B = Q rows in registers)
//     -> lane (q = lane&31, half h) holds the scores of its query row for
//        keys (r&3) + 8(r>>2) + 4h: the row max is 31 in-lane fmax + ONE
//        cross-half shuffle, the row sum stays lane-partial until the end.
//   Oᵀ[d][q] += Vᵀ·Pᵀ            (B = the Sᵀ accumulator registers packed to
//        16-bit: an accumulator tile is the next MFMA's B operand when the
//        product sums over its rows; CDNA guide §3.  A = Vᵀ rows from LDS,
//        in the matching permuted key order: two 8-byte reads per fragment)
// K is staged row-major with a 16-byte XOR swizzle (conflict-free
// ds_read_b128), V transposed (row stride 68 elements: conflict-free
// ds_read_b64), both double-buffered; the next tile's global loads are issued
// before the MFMAs and written to LDS after them (issue-early / write-late).
// DP = head dim padded to 64 or 128.
// ---------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int DT>
__device__ __forceinline__ f32x16 mfma32(const uint4 a, const uint4 b, f32x16 c) {
  if constexpr (DT == kBF16) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
}

template <int DP>
__device__ __forceinline__ int k_swz(int row, int chunk) {
  // 16-byte chunk position inside a K row (conflict-free ds_read_b128 for the
  // 16-lane groups {0-3,12-15,20-27}, ...; MI355X_MICROARCH §LDS)
  if constexpr (DP == 64) return chunk ^ ((row >> 1) & 7);
  else return chunk ^ (row & 15);
}

__device__ __forceinline__ uint32_t pack2(uint16_t lo, uint16_t hi) {
  return (uint32_t)lo | ((uint32_t)hi << 16);
}

// two f32 -> packed 16-bit pair (RNE; hipcc emits v_cvt_pk_bf16_f32 on gfx950)
template <int DT>
__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  if constexpr (DT == kBF16) {
    const __bf16 a = (__bf16)lo, b = (__bf16)hi;
    return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
  } else {
    // the two-element vector form lowers to one v_cvt_pk_f16_f32 (RNE); two scalar
    // casts + shift/or took three instructions per pair
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 v = {(_Float16)lo, (_Float16)hi};
    return __builtin_bit_cast(uint32_t, v);
  }
}

constexpr int kVTS = 68;

// deferred-max threshold of flash2 (log2 units): p <= 2^8 between rescales
constexpr float kDefer = 8.f;

template <int DT, int DP, int NW>
__global__ __launch_bounds__(64 * NW, 2) void flash2_fwd_kernel(FlashArgs a) {
  constexpr int KS = DP / 16;   // QKᵀ k-steps
  constexpr int NCH = DP / 8;   // 16-byte chunks per K/V row
  constexpr int DTL = DP / 32;  // Oᵀ tiles
  constexpr int NT = 64 * NW;   // threads
  constexpr int NPR = 32 * NCH / NT;  // (key pair, chunk) items per thread per tile
  static_assert(NPR * NT == 32 * NCH, "staging must divide evenly");
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 64 * DP + 2 * DP * kVTS];
  uint16_t* const Kb = smem;
  uint16_t* const Vb = smem + 2 * 64 * DP;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l32 = lane & 31, h = lane >> 5;
  const int hq = blockIdx.y, b = blockIdx.z / a.ksplit, sk = blockIdx.z - b * a.ksplit;
  // Causal load balance: q tile x costs ~x key tiles, so with a grid that fills the
  // chip once, the last tiles' workgroups set the kernel time at ~2x the mean.
  // Paired, workgroup x runs tiles x and n-1-x back to back (n+1 tiles' work each).
  const int nqt = (a.N + 32 * NW - 1) / (32 * NW);
  const int bx = blockIdx.x;
  const int npass = (a.pair && nqt - 1 - bx != bx) ? 2 : 1;
  for (int pass = 0; pass < npass; ++pass) {
  if (pass) __syncthreads();  // every wave is past its LDS reads of the first tile
  const int mblk = (pass ? nqt - 1 - bx : bx) * (32 * NW);
  const int qrow = mblk + wave * 32 + l32;
  const int hk = hq / (a.H / a.Hkv);
  const uint16_t* qb = a.q + b * a.q_sb + hq * a.q_sh;
  const uint16_t* kb = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vb = a.v + b * a.v_sb + hk * a.v_sh;

  // Q as the B operand: lane holds Q[qrow][16ks + 8h .. +8]
  uint4 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int d0 = 16 * ks + 8 * h;
    qf[ks] = (qrow < a.N && d0 < a.D)
                 ? *reinterpret_cast<const uint4*>(qb + (long long)qrow * a.q_sn + d0)
                 : make_uint4(0, 0, 0, 0);
  }

  f32x16 o[DTL];
#pragma unroll
  for (int t = 0; t < DTL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int qpos = qrow + a.pos0;
  const int qmin = mblk + wave * 32 + a.pos0;  // smallest query position of this wave

  int kend = a.M;
  if (a.causal) kend = min(kend, a.pos0 + mblk + 32 * NW);
  int j0 = 0;
  if (a.ksplit > 1) {  // this split's key tiles (causal rows past the split: empty partials)
    j0 = sk * a.kchunk / 64;
    kend = min(kend, (sk + 1) * a.kchunk);
  }
  const int ntiles = (kend + 63) / 64;

  // staging: pair pi -> keys 2*(pi / NCH) + {0,1}, chunk pi % NCH.  Per-thread element
  // offsets of tile 0 are computed once; a tile adds the wave-uniform j * 64 rows.
  uint4 kr[NPR][2], vr[NPR][2];
  long long koff[NPR], voff[NPR];
  int krow[NPR];
  bool cok[NPR];
#pragma unroll
  for (int i = 0; i < NPR; ++i) {
    const int pi = tid + NT * i, kp = pi / NCH, c = pi - kp * NCH;
    krow[i] = 2 * kp;
    cok[i] = c * 8 < a.D;
    koff[i] = (long long)(2 * kp) * a.k_sn + c * 8;
    voff[i] = (long long)(2 * kp) * a.v_sn + c * 8;
  }
  auto gload = [&](int j) {
    const uint16_t* kj = kb + (long long)j * 64 * a.k_sn;
    const uint16_t* vj = vb + (long long)j * 64 * a.v_sn;
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool ok = j * 64 + krow[i] + e < a.M && cok[i];
        kr[i][e] = ok ? *reinterpret_cast<const uint4*>(kj + koff[i] + e * a.k_sn)
                      : make_uint4(0, 0, 0, 0);
        vr[i][e] = ok ? *reinterpret_cast<const uint4*>(vj + voff[i] + e * a.v_sn)
                      : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto sstore = [&](int buf) {
    uint16_t* Ks = Kb + buf * 64 * DP;
    uint16_t* Vt = Vb + buf * DP * kVTS;
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
      const int pi = tid + NT * i, kp = pi / NCH, c = pi - kp * NCH;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int row = 2 * kp + e;
        *reinterpret_cast<uint4*>(Ks + row * DP + k_swz<DP>(row, c) * 8) = kr[i][e];
      }
      const uint16_t* v0 = reinterpret_cast<const uint16_t*>(&vr[i][0]);
      const uint16_t* v1 = reinterpret_cast<const uint16_t*>(&vr[i][1]);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *reinterpret_cast<uint32_t*>(Vt + (c * 8 + e) * kVTS + 2 * kp) = pack2(v0[e], v1[e]);
    }
  };

  if (ntiles > j0) {
    gload(j0);
    sstore(0);
  }
  __syncthreads();
  for (int j = j0; j < ntiles; ++j) {
    const int buf = (j - j0) & 1;
    const bool more = j + 1 < ntiles;
    const uint16_t* Ks = Kb + buf * 64 * DP;
    const uint16_t* Vt = Vb + buf * DP * kVTS;

    // ---- Sᵀ = K Qᵀ over two 32-key subtiles.  A subtile's K fragments are all read
    // before its MFMAs (DP 64: both subtiles' up front): read -> wait -> MFMA per fragment
    // exposed the LDS latency KS times per subtile.
    f32x16 s[2];
    constexpr int KT = DP == 64 ? 2 : 1;  // subtiles whose fragments are read together
#pragma unroll
    for (int t0 = 0; t0 < 2; t0 += KT) {
      uint4 kf[KT][KS];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const int row = 32 * (t0 + u) + l32;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          kf[u][ks] =
              *reinterpret_cast<const uint4*>(Ks + row * DP + k_swz<DP>(row, 2 * ks + h) * 8);
      }
      if constexpr (DP == 64) __builtin_amdgcn_sched_barrier(0);  // reads before the MFMAs
#pragma unroll
      for (int u = 0; u < KT; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[t0 + u][r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[t0 + u] = mfma32<DT>(kf[u][ks], qf[ks], s[t0 + u]);
      }
    }

    // the next tile's global loads go out AFTER the QKᵀ MFMAs: issued at the top of the
    // iteration, the first MFMA's wait (vmcnt(0), emitted by the compiler for the q
    // registers) drained them at once and the prefetch hid nothing
    if (more) gload(j + 1);
    // ---- online softmax; the row spans lanes l, l^32.  Scores stay raw (the
    // scale is folded into one fma per exp2); masking only on boundary tiles.
    const bool edge = j * 64 + 64 > a.M || (a.causal && j * 64 + 63 > qmin);
    if (edge) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = j * 64 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (key >= a.M || (a.causal && key > qpos)) s[t][r] = -INFINITY;
        }
    }
    // row max: four independent max chains, then the lane l / l^32 exchange on
    // permlane32_swap (no LDS round trip as with ds_bpermute)
    float mq[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mq[r & 3] = fmaxf(mq[r & 3], s[t][r]);
    float mt = fmaxf(fmaxf(mq[0], mq[1]), fmaxf(mq[2], mq[3]));
    {
      const int bi = __builtin_bit_cast(int, mt);
      const auto sw = __builtin_amdgcn_permlane32_swap(bi, bi, false, false);
      mt = fmaxf(__builtin_bit_cast(float, (int)sw[0]), __builtin_bit_cast(float, (int)sw[1]));
    }
    // Deferred max (FA-style threshold): the running max moves only when a tile's max
    // exceeds it by more than 2^kDefer in probability units, so p stays <= 2^kDefer and
    // most tiles skip the O rescale (skipped when no lane of the wave moved its max).
    const bool grow = m == -INFINITY || (mt - m) * a.scale_log2 > kDefer;
    const float mn = grow ? fmaxf(m, mt) : m;  // raw-score units
    const float mc = mn == -INFINITY ? 0.f : mn * a.scale_log2;
    float rq[4] = {0.f, 0.f, 0.f, 0.f};  // four independent row-sum chains
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[t][r], a.scale_log2, -mc));
        s[t][r] = p;
        rq[r & 3] += p;
      }
    const float rs = (rq[0] + rq[1]) + (rq[2] + rq[3]);
    if (__builtin_amdgcn_ballot_w64(grow) != 0ull) {
      const float alpha = __builtin_amdgcn_exp2f(m * a.scale_log2 - mc);  // m = -inf -> 0
      l *= alpha;
#pragma unroll
      for (int t = 0; t < DTL; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
    }
    l += rs;
    m = mn;

    // ---- Oᵀ += Vᵀ Pᵀ: k-step (t, s2) covers keys 32t + 16s2 + {8(j>>2) + 4h + (j&3)}
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        uint4 pf;
        pf.x = cvt_pk<DT>(s[t][8 * s2 + 0], s[t][8 * s2 + 1]);
        pf.y = cvt_pk<DT>(s[t][8 * s2 + 2], s[t][8 * s2 + 3]);
        pf.z = cvt_pk<DT>(s[t][8 * s2 + 4], s[t][8 * s2 + 5]);
        pf.w = cvt_pk<DT>(s[t][8 * s2 + 6], s[t][8 * s2 + 7]);
        const int k0 = 32 * t + 16 * s2 + 4 * h;
#pragma unroll
        for (int dt = 0; dt < DTL; ++dt) {
          const uint16_t* vrow = Vt + (32 * dt + l32) * kVTS + k0;
          const uint2 lo = *reinterpret_cast<const uint2*>(vrow);
          const uint2 hi = *reinterpret_cast<const uint2*>(vrow + 8);
          o[dt] = mfma32<DT>(make_uint4(lo.x, lo.y, hi.x, hi.y), pf, o[dt]);
        }
      }
    if (more) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: O[q][d] = Oᵀ[d][q] / l  (d = 32dt + 8g + 4h + i)
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (a.ksplit > 1) {  // key split: f32 partial rows + log2-sum-exp for the merge
    if (qrow < a.N) {
      const size_t row = ((size_t)blockIdx.z * a.H + hq) * a.N + qrow;
      float* prow = a.po + row * a.D;
#pragma unroll
      for (int dt = 0; dt < DTL; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = 32 * dt + 8 * g + 4 * h;
          if (d < a.D)
            *reinterpret_cast<float4*>(prow + d) =
                make_float4(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv,
                            o[dt][4 * g + 3] * inv);
        }
      if (h == 0) a.plse[row] = lt > 0.f ? m * a.scale_log2 + __log2f(lt) : -INFINITY;
    }
    continue;
  }
  if (qrow < a.N) {
    uint16_t* orow = a.o + b * a.o_sb + hq * a.o_sh + (long long)qrow * a.o_sn;
#pragma unroll
    for (int dt = 0; dt < DTL; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        if (d < a.D) {
          uint2 st;
          st.x = pack2(from_f32<DT>(o[dt][4 * g + 0] * inv), from_f32<DT>(o[dt][4 * g + 1] * inv));
          st.y = pack2(from_f32<DT>(o[dt][4 * g + 2] * inv), from_f32<DT>(o[dt][4 * g + 3] * inv));
          *reinterpret_cast<uint2*>(orow + d) = st;
        }
      }
  }
  }  // pass
}

// Merge of the key splits: O = sum_s 2^(lse_s - max) O_s / sum_s 2^(lse_s - max); one thread
// per 4 head dims of one (b, h, q) row.
template <int DT>
__global__ __launch_bounds__(256) void flash_merge_kernel(FlashArgs a) {
  const int dq = a.D / 4;
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t rows = (size_t)a.B * a.H * a.N;
  if (t >= rows * dq) return;
  const size_t r = t / dq;
  const int d = (int)(t - r * dq) * 4;
  const int q = (int)(r % a.N), hq = (int)((r / a.N) % a.H), b = (int)(r / ((size_t)a.N * a.H));
  const size_t hn = (size_t)a.H * a.N;
  float lse[4], mx = -INFINITY;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    lse[s] = s < a.ksplit ? a.plse[(size_t)(b * a.ksplit + s) * hn + (size_t)hq * a.N + q]
                          : -INFINITY;
    mx = fmaxf(mx, lse[s]);
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float wsum = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s >= a.ksplit || lse[s] == -INFINITY) continue;
    const float w = __builtin_amdgcn_exp2f(lse[s] - mx);
    const float4 v = *reinterpret_cast<const float4*>(
        a.po + ((size_t)(b * a.ksplit + s) * hn + (size_t)hq * a.N + q) * a.D + d);
    acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
    wsum += w;
  }
  const float inv = wsum > 0.f ? 1.f / wsum : 0.f;
  uint2 st;
  st.x = pack2(from_f32<DT>(acc.x * inv), from_f32<DT>(acc.y * inv));
  st.y = pack2(from_f32<DT>(acc.z * inv), from_f32<DT>(acc.w * inv));
  *reinterpret_cast<uint2*>(a.o + b * a.o_sb + hq * a.o_sh + (long long)q * a.o_sn + d) = st;
}

}  // namespace cake

using namespace cake;

static int g_flash_ksplit = -1;  // v2 key splits: 0 = auto, 1 = off, 2 / 4 forced;
                                 // -1: from CAKE_FLASH_KSPLIT (default auto)

static int flash_ksplit() {
  if (g_flash_ksplit < 0) {
    const char* e = getenv("CAKE_FLASH_KSPLIT");
    const int k = e ? atoi(e) : 0;
    g_flash_ksplit = (k == 1 || k == 2 || k == 4) ? k : 0;
  }
  return g_flash_ksplit;
}
static int g_flash_impl = -1;  // -1: from CAKE_FLASH_IMPL (default 2)
static long long g_flash_pair_min = 512;  // unpaired workgroups needed before pairing
static int g_flash_nw = 0;                 // v2 waves per workgroup override (0 = auto)

static int flash_impl() {
  if (g_flash_impl < 0) {
    const char* e = getenv("CAKE_FLASH_IMPL");
    g_flash_impl = e ? atoi(e) : 2;
  }
  return g_flash_impl;
}

template <int DT>
static int launch_flash(const FlashArgs& a, hipStream_t st) {
  // v2 needs 16-byte rows (D % 8 == 0, 8-byte aligned strides) and D <= 128
  auto al = [](const void* p, int n) { return ((uintptr_t)p % n) == 0; };
  const bool v2 = flash_impl() >= 2 && a.D % 8 == 0 && a.D <= 128 && a.q_sn % 8 == 0 &&
                  a.k_sn % 8 == 0 && a.v_sn % 8 == 0 && a.o_sn % 4 == 0 && a.q_sb % 8 == 0 &&
                  a.q_sh % 8 == 0 && a.k_sb % 8 == 0 && a.k_sh % 8 == 0 && a.v_sb % 8 == 0 &&
                  a.v_sh % 8 == 0 && a.o_sb % 4 == 0 && a.o_sh % 4 == 0 && al(a.q, 16) &&
                  al(a.k, 16) && al(a.v, 16) && al(a.o, 8);
  if (v2) {
    // rows per workgroup: 128 (4 waves); smaller only for tiny grids (measured:
    // 4-wave workgroups win even at 128 workgroups on 256 CUs)
    int nw = 4;
    const int nw_min = a.D <= 64 ? 1 : 2;  // DP=128 staging registers need >= 2 waves
    while (nw > nw_min && (long long)((a.N + 32 * nw - 1) / (32 * nw)) * a.H * a.B < 32) nw >>= 1;
    if (g_flash_nw >= nw_min && g_flash_nw <= 4) nw = g_flash_nw;
    const int nqt = (a.N + 32 * nw - 1) / (32 * nw);
    FlashArgs p = a;
    // pair causal q tiles once the unpaired grid fills every CU twice (below that,
    // halving the workgroups costs more parallelism than the balance gains)
    p.pair = a.causal && nqt >= 2 && (long long)nqt * a.H * a.B >= g_flash_pair_min;
    // Non-causal grids with fewer workgroups than CUs (SD 1.5's 1024-token self-attention:
    // 128) leave most of the chip idle: split the keys (>= 256 per split, up to two
    // workgroups per CU) and merge the f32 partial rows in a second launch (44.8 -> 28.1 us
    // there).  At >= 256 workgroups the split measured neutral (SDXL's 320: 35.4 us either
    // way; profiles/r4_flash_key_split.jsonl), so it stays off.
    p.ksplit = 1;
    // causal: only a forced split (cake_flash_set_ksplit 2 / 4; measured A/B)
    if ((!a.causal || flash_ksplit() > 1) && a.D % 4 == 0 && a.po != nullptr) {
      const long long wgs = (long long)nqt * a.H * a.B;
      int ks = 1;
      if (flash_ksplit() == 0) {
        if (wgs < 256)
          while (ks < 4 && wgs * ks < 512 && a.M / (2 * ks) >= 256) ks *= 2;
      } else {
        ks = flash_ksplit();
      }
      const long long need = (long long)ks * a.B * a.H * a.N * (a.D + 1) * 4;
      if (ks > 1 && need <= a.ws_bytes) {
        p.ksplit = ks;
        p.kchunk = ((a.M + ks - 1) / ks + 63) / 64 * 64;
        p.plse = a.po + (size_t)ks * a.B * a.H * a.N * a.D;
      }
    }
    const dim3 g2(p.pair ? (nqt + 1) / 2 : nqt, a.H, a.B * p.ksplit);
#define CAKE_FL2(P, W) hipLaunchKernelGGL((flash2_fwd_kernel<DT, P, W>), g2, dim3(64 * W), 0, st, p)
    if (a.D <= 64) {
      if (nw == 4) CAKE_FL2(64, 4); else if (nw == 2) CAKE_FL2(64, 2); else CAKE_FL2(64, 1);
    } else {
      if (nw == 4) CAKE_FL2(128, 4); else CAKE_FL2(128, 2);
    }
#undef CAKE_FL2
    if (p.ksplit > 1) {
      const size_t n = (size_t)a.B * a.H * a.N * (a.D / 4);
      hipLaunchKernelGGL((flash_merge_kernel<DT>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                         st, p);
    }
    return (int)hipGetLastError();
  }
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

// 1 = the 16-row 16x16x32 kernel, 2 = the 32x32x16 swapped-QKᵀ kernel (when shapes allow)
CAKE_API void cake_flash_set_impl(int v) { g_flash_impl = v; }
CAKE_API void cake_flash_set_nw(int nw) { g_flash_nw = nw; }
// causal q-tile pairing threshold (unpaired workgroups); <= 0 never pairs
CAKE_API void cake_flash_set_pair_min(long long n) { g_flash_pair_min = n > 0 ? n : (1ll << 62); }

// key splits of the non-causal v2 path: 0 = auto, 1 = never, 2 / 4 = forced (tests)
CAKE_API void cake_flash_set_ksplit(int k) { g_flash_ksplit = (k == 1 || k == 2 || k == 4) ? k : 0; }

// strides in ELEMENTS: s[0]=batch, s[1]=head, s[2]=row for q, k, v, o (12 values).
// ws (optional, f32, ws_bytes): partial rows for the non-causal key split.
CAKE_API int cake_flash_attn_ws(int dt, const void* q, const void* k, const void* v, void* o, int B,
                                int H, int Hkv, int N, int M, int D, const long long* strides,
                                float scale, int causal, int pos0, void* ws, long long ws_bytes,
                                hipStream_t st) {
  if (H <= 0 || Hkv <= 0 || H % Hkv || D <= 0 || D > 256 || N <= 0 || M <= 0)
    return (int)hipErrorInvalidValue;
  FlashArgs a{(const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o,
              B, H, Hkv, N, M, D,
              strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
              strides[6], strides[7], strides[8], strides[9], strides[10], strides[11],
              scale * 1.4426950408889634f, causal, pos0, 0};
  a.po = (float*)ws;
  a.ws_bytes = ws ? ws_bytes : 0;
  if (dt == kBF16) return launch_flash<kBF16>(a, st);
  if (dt == kF16) return launch_flash<kF16>(a, st);
  return (int)hipErrorInvalidValue;
}

CAKE_API int cake_flash_attn(int dt, const void* q, const void* k, const void* v, void* o, int B,
                             int H, int Hkv, int N, int M, int D, const long long* strides,
                             float scale, int causal, int pos0, hipStream_t st) {
  return cake_flash_attn_ws(dt, q, k, v, o, B, H, Hkv, N, M, D, strides, scale, causal, pos0,
                            nullptr, 0, st);
}
