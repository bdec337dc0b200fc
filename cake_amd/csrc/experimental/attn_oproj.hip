// Decode attention + o_proj as ONE launch, for the live lengths the attention runs as a
// single split (short contexts: the bench's and most chat turns').
//
// The two launches it replaces (attention.hip, then the o_proj GEMV of gemv.hip) cost a
// kernel boundary plus the attention's whole dependent chain — q load, K/V blocks,
// online softmax, wave merge — with the chip idle: ~5.6 us against ~1.9 us of its own
// bytes (profiles/r4_decode8b_p32_kernel_table.txt), then o_proj streams its 33.6 MB.
// Here the o_proj weights stream WHILE the attention runs:
//
//   * the o_proj input columns of kv group g (its NREP query heads x hd) multiply
//     W_o[:, g NREP hd .. ] only, so o_proj splits over the kv groups exactly
//     (out = sum_g W_o[:, cols(g)] . attn[cols(g)]);
//   * workgroup (j, g) — row block j of RB output rows, kv group g — first issues its
//     W_o[rows(j), cols(g)] loads into registers (nt: read once), then runs the group's
//     attention (attn_core2.h, one split, output into LDS), then the dot products
//     against the registers: no weight byte waits for the attention, no attention step
//     waits for a weight byte;
//   * every group's attention is recomputed by the H / RB workgroups of that group
//     (blockIdx % nkv = g: with 8 kv heads one XCD per group, so the group's K/V rows
//     are read from HBM once and from that XCD's L2 after): a few KB per workgroup at
//     the short lengths this kernel serves;
//   * the nkv per-group partial rows of a row block are summed in a fixed order by the
//     last-arriving workgroup (relaxed agent-scope ticket), so results are deterministic.
//     Partials travel as 8-byte {f32, tag} granules (one store each; the tag is the row
//     block's launch epoch + 1): the last arriver polls for the tags instead of either
//     side fencing — a release fence per workgroup writes back the L2 and cost ~50 us per
//     launch here (MI355X_MICROARCH 'barrier-counter' / 'publish-large').
//
// Reference: cake-core/src/models/llama3/attention.rs:96-120 (scores, softmax, P.V,
// o_proj); SURVEY K09-K13 + K03 (o_proj) + K14 (residual).
#include <cstdio>

#include "../kernels/attn_core2.h"

namespace cake {

// output rows per workgroup: 64, or 32 for 8-head groups (whose 8-wave workgroup holds
// 2 chunks per lane per row: 64 rows would spill the weight registers)
constexpr int kAoRows = 64;
__host__ __device__ constexpr int ao_rows(int nrep) { return nrep == 8 ? 32 : kAoRows; }

struct AttnOprojArgs {
  const float* q;          // [nh*hd] f32 (roped)
  const uint16_t* kc;      // [nkv][S][hd] this layer's cache
  const uint16_t* vc;
  const int* pos;          // device scalar: this token's position
  int S;
  float scale_log2;
  const uint16_t* wo;      // [H][ldw] o_proj weight (16-bit)
  int ldw;                 // row length of wo (= nh * hd of this rank)
  int H;                   // output rows
  float* out;              // [H] f32: out (+)= W_o . attn
  int accumulate;
  unsigned long long* ws;  // [nkv][H] {f32 partial, tag} granules
  unsigned int* tickets;   // [NRB] arrival counters (zero between launches), [NRB] epochs,
                           // then [2 nkv + 2] scratch for the attention core's epoch words
  unsigned int* err;       // error word (a poll that gave up), or null
  int nkv;
};

// sum over aligned groups of N lanes (N = 16, 32, 64): every lane of a group ends with it
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(N == 16 || N == 32 || N == 64, "lane group");
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  v += dpp_f<kDppMirror>(v);
  if constexpr (N >= 32) v = xor_add<16>(v);
  if constexpr (N == 64) v = xor_add<32>(v);
  return v;
}

template <int DT, int HD, int NREP>
__global__ __launch_bounds__(AttnGeom2<NREP>::NT) void attn_oproj_kernel(AttnOprojArgs p) {
  constexpr int NW = AttnGeom2<NREP>::NW;
  constexpr int NT = 64 * NW;
  constexpr int RB = ao_rows(NREP);
  constexpr int NCOL = NREP * HD;         // o_proj input columns of one kv group
  constexpr int CH = NCOL / 8;            // 16-byte chunks of one row segment
  constexpr int LPR = CH < 64 ? CH : 64;  // lanes per row
  constexpr int RPW = 64 / LPR;           // rows per wave instruction
  constexpr int CPL = CH / LPR;           // chunks per lane per row
  constexpr int RPWV = RB / NW;           // rows per wave
  constexpr int IT = RPWV / RPW;
  static_assert(CH % LPR == 0 && RPWV % RPW == 0 && IT >= 1, "o_proj tiling");
  __shared__ __attribute__((aligned(16))) float lds[attn2_smem_floats<HD, NREP, NW>()];
  __shared__ __attribute__((aligned(16))) uint16_t xs[NCOL];
  __shared__ int is_last;
  const int nkv = p.nkv;
  const int g = blockIdx.x % nkv, j = blockIdx.x / nkv;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sub = lane / LPR, cl = lane - sub * LPR;
  const int row0 = j * RB + wave * RPWV;
  const int nrb = p.H / 32;  // ticket / epoch slots (the smallest row block)
  const unsigned int epoch =
      __hip_atomic_load(p.tickets + nrb + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  // (1) this workgroup's weight tile, in flight during the attention: issued by the
  // attention core's hook, right BEHIND its first K/V blocks and q (loads retire in
  // order: issued in front, the weights would delay every attention step)
  uint4 w[IT][CPL];
  const uint16_t* wg = p.wo + (size_t)g * NCOL;
  auto issue_weights = [&]() {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const uint4* wr =
          reinterpret_cast<const uint4*>(wg + (size_t)(row0 + it * RPW + sub) * p.ldw);
#pragma unroll
      for (int c = 0; c < CPL; ++c) w[it][c] = ld_nt16(wr + cl + c * LPR);
    }
  };

  // (2) the group's attention, one split, output (16-bit, as the standalone kernel
  // writes it) into LDS: the core stores at out[g * NCOL + idx]
  AttnDecArgs at{};
  at.q = p.q;
  at.kc = p.kc;
  at.vc = p.vc;
  at.pos = p.pos;
  at.S = p.S;
  at.scale_log2 = p.scale_log2;
  at.part = nullptr;
  at.tickets = p.tickets + 2 * nrb;  // scratch epoch words (never a tag in one split)
  at.out = xs - (size_t)g * NCOL;
  at.min_keys = 64;
  at.maxsplit = 1;
  at.stamps = nullptr;
  at.target = 16;
  at.single = p.S;  // every live length is one split here
  at.drop_partials = 0;
  // two key blocks per wave requested up front (PFD 2): up to 2 NW x 16 keys of the
  // attention need no load issued behind the weights
  attn2_decode_block<DT, HD, NREP, false, NW, 2>(at, g, 0, lds, nkv, issue_weights);
  __syncthreads();

  // (3) partial o_proj rows of this group: lanes of a row group sum their chunks
  float acc[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      float wv[8], xv[8];
      unpack8<DT>(w[it][c], wv);
      unpack8<DT>(*reinterpret_cast<const uint4*>(xs + (cl + c * LPR) * 8), xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) a = fmaf(wv[e], xv[e], a);
    }
    acc[it] = group_sum<LPR>(a);
  }
  const unsigned long long tag = (unsigned long long)(epoch + 1u) << 32;
  if (cl == 0) {
#pragma unroll
    for (int it = 0; it < IT; ++it)
      __hip_atomic_store(p.ws + (size_t)g * p.H + row0 + it * RPW + sub,
                         tag | __float_as_uint(acc[it]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // (4) the last of the nkv groups of row block j sums the partials (g order: fixed)
  if (threadIdx.x == 0) {
    const unsigned int t =
        __hip_atomic_fetch_add(p.tickets + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = t == (unsigned int)(nkv - 1);
  }
  __syncthreads();
  if (!is_last) return;  // workgroup-uniform
  bool timed_out = false;
  for (int i = threadIdx.x; i < RB; i += NT) {
    const int r = j * RB + i;
    float s = 0.f;
    for (int gg = 0; gg < nkv; ++gg) {
      unsigned long long v;
      for (int tries = 0;; ++tries) {  // the granule of this launch (its tag) — bounded
        v = __hip_atomic_load(p.ws + (size_t)gg * p.H + r, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
        if ((v >> 32) == (tag >> 32)) break;
        if (tries > kAttnMaxPolls) { timed_out = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      s += __uint_as_float((unsigned int)v);
    }
    p.out[r] = p.accumulate ? p.out[r] + s : s;
  }
  if (timed_out && p.err) attn_poll_timeout(p.err);
  __syncthreads();
  if (threadIdx.x == 0) {  // re-arm for the next launch (the kernel boundary orders these)
    __hip_atomic_store(p.tickets + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p.tickets + nrb + j, epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace cake

using namespace cake;

// Shapes the fused launch covers: GQA group 1/2/4/8, head_dim 64/128, H a multiple of
// the row block, and the o_proj row length nh * hd (this rank's heads).
CAKE_API int cake_attn_oproj_supported(int nh, int nkv, int hd, int H) {
  if (nkv <= 0 || nh % nkv || (hd != 64 && hd != 128) || H <= 0 || H % kAoRows) return 0;
  const int nrep = nh / nkv;  // (H % 64 == 0 covers the 32-row blocks too)
  if (nrep != 1 && nrep != 2 && nrep != 4 && nrep != 8) return 0;
  const int ncol = nrep * hd;
  return ncol >= 128 && ncol <= 1024;
}

// workspace: {f32, tag} granules of the partial rows (as f32 words: 2 per granule), then
// the ticket / epoch words (u32, zeroed once)
CAKE_API long long cake_attn_oproj_ws_floats(int nkv, int H) { return 2ll * nkv * H; }
CAKE_API long long cake_attn_oproj_ticket_words(int nkv, int H) {
  return 2ll * (H / 32) + 2 * nkv + 2;  // slots for the smallest row block
}

CAKE_API int cake_attn_oproj(int dt, const float* q, const void* kc, const void* vc,
                             const int* pos, int S, int nh, int nkv, int hd, float scale,
                             const void* wo, int ldw, int H, float* out, int accumulate,
                             float* ws, unsigned int* tickets, unsigned int* err,
                             hipStream_t st) {
  if (!cake_attn_oproj_supported(nh, nkv, hd, H) || S <= 0 || ldw < nh * hd || !ws || !tickets ||
      ((uintptr_t)ws % 8))
    return (int)hipErrorInvalidValue;
  AttnOprojArgs p{q, (const uint16_t*)kc, (const uint16_t*)vc, pos, S,
                  scale * 1.4426950408889634f, (const uint16_t*)wo, ldw, H, out, accumulate,
                  reinterpret_cast<unsigned long long*>(ws), tickets, err, nkv};
  const int nrep = nh / nkv;
  const dim3 grid(nkv * (H / ao_rows(nrep)));
#define CAKE_AO(DTV, HDV, NR)                                                                  \
  hipLaunchKernelGGL((attn_oproj_kernel<DTV, HDV, NR>), grid, dim3(AttnGeom2<NR>::NT), 0, st, p)
#define CAKE_AO_128(DTV)                         \
  switch (nrep) {                                \
    case 1: CAKE_AO(DTV, 128, 1); break;         \
    case 2: CAKE_AO(DTV, 128, 2); break;         \
    case 4: CAKE_AO(DTV, 128, 4); break;         \
    default: CAKE_AO(DTV, 128, 8); break;        \
  }
#define CAKE_AO_64(DTV)  /* nrep 1 x hd 64 = 64 columns: not covered */ \
  switch (nrep) {                                \
    case 2: CAKE_AO(DTV, 64, 2); break;          \
    case 4: CAKE_AO(DTV, 64, 4); break;          \
    default: CAKE_AO(DTV, 64, 8); break;         \
  }
  if (dt == kBF16 && hd == 128) { CAKE_AO_128(kBF16); }
  else if (dt == kBF16) { CAKE_AO_64(kBF16); }
  else if (dt == kF16 && hd == 128) { CAKE_AO_128(kF16); }
  else if (dt == kF16) { CAKE_AO_64(kF16); }
  else return (int)hipErrorInvalidValue;
#undef CAKE_AO_128
#undef CAKE_AO_64
#undef CAKE_AO
  return (int)hipGetLastError();
}
