// One-shot all-reduce for tensor-parallel decode on one node (xGMI mesh).
//
// Tensor parallelism is the MI355X-first answer to batch-1 decode on N GPUs:
// where the reference shards LAYERS over workers (cake-core/src/models/llama3/
// llama.rs:95-114 — every token visits every worker in turn, so N GPUs decode
// no faster than one), each rank here holds 1/N of every layer's heads and MLP
// rows and streams 1/N of the weights per token.  The price is two all-reduces
// of the hidden state per layer (after o_proj and after down_proj), i.e. 64
// small (16 KiB f32) collectives per 8B token — latency-bound, so they are done
// as ONE kernel each, without the host and inside the decode graph:
//
//   every rank stores its partial vector into EVERY peer's inbox (one system-
//   scope 8-byte store per word: {f32 word, tag}, the hop.hip granule), then
//   polls its own inbox until all N-1 peers' words carry the expected tag and
//   sums them with its own partial.  On an 8-GPU MI355X node every pair of GPUs
//   has its own xGMI link, so the N-1 pushes go out in parallel.
//
// The tag is a per-rank device counter advanced by the last workgroup to finish
// (agent-scope ticket), so graph replays stay in lock step; the inbox has two
// parity banks, so a fast rank's next all-reduce cannot overwrite words a slow
// peer has not read yet (it cannot get two ahead: finishing all-reduce k needs
// every peer's contribution to k).  Polls are bounded by a wall-clock timeout
// (s_memrealtime) that sets an error word instead of hanging the GPU.
//
// Ops: SUM of f32 vectors (out = sum, or out += sum into the f32 residual
// stream), MAX of one 64-bit argmax key (vocab-sharded lm_head: the key is
// (ordered logit << 32 | ~global index), so the max is the global argmax with
// the smallest index on ties, exactly as the single-GPU argmax_kernel), and
// GATHER of the vocab-sharded logits into a full vector on every rank (sampled
// decoding: top-k / top-p need the global distribution; every rank then draws
// the same token from the same full vector).
#include "common.h"

namespace cake {

constexpr int kArThreads = 256;
constexpr int kArMaxRanks = 8;

struct ArArgs {
  unsigned long long* peer[kArMaxRanks];  // peers' inboxes (own slot unused)
  const unsigned long long* inbox;        // this rank's inbox [2][N][n]
  unsigned int* seq;                      // [0] = tag counter, [1] = done ticket
  int* err;
  int rank, world, n;
  unsigned long long timeout_ticks;
};

__device__ __forceinline__ unsigned long long ar_poll(const unsigned long long* p,
                                                      unsigned int tag, unsigned long long t0,
                                                      unsigned long long limit, bool& late) {
  unsigned long long g;
  for (;;) {
    g = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((unsigned int)(g >> 32) == tag || late) return g;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit) late = true;
  }
}

// The last workgroup advances the tag (every workgroup has read it by then).
__device__ __forceinline__ void ar_finish(const ArArgs& a, unsigned int tag) {
  __shared__ unsigned int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int t = __hip_atomic_fetch_add(a.seq + 1, 1u, __ATOMIC_ACQ_REL,
                                                  __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __hip_atomic_store(a.seq + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.seq, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// out[i] (+)= sum over ranks of partial[i], i < n
template <bool ACC>
__global__ __launch_bounds__(kArThreads) void ar_sum_kernel(ArArgs a, const float* __restrict__ partial,
                                                            float* __restrict__ out) {
  const unsigned int tag = __hip_atomic_load(a.seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const size_t bank = (size_t)(tag & 1u) * a.world * a.n;
  const int i0 = blockIdx.x * kArThreads + threadIdx.x, stride = gridDim.x * kArThreads;
  for (int i = i0; i < a.n; i += stride) {
    const unsigned long long g =
        (unsigned long long)__float_as_uint(partial[i]) | ((unsigned long long)tag << 32);
    for (int r = 0; r < a.world; ++r)
      if (r != a.rank)
        __hip_atomic_store(a.peer[r] + bank + (size_t)a.rank * a.n + i, g, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool late = false;
  for (int i = i0; i < a.n; i += stride) {
    float s = partial[i];
    for (int r = 0; r < a.world; ++r) {
      if (r == a.rank) continue;
      const unsigned long long g = ar_poll(a.inbox + bank + (size_t)r * a.n + i, tag, t0,
                                           a.timeout_ticks, late);
      s += __uint_as_float((uint32_t)g);
    }
    if constexpr (ACC) out[i] += s;
    else out[i] = s;
  }
  if (late) atomicOr(a.err, 1);
  ar_finish(a, tag);
}

// slot (u64 argmax key): max over ranks, in place (n = 2 words: lo, hi)
__global__ __launch_bounds__(64) void ar_max_key_kernel(ArArgs a, unsigned long long* slot) {
  const unsigned int tag = __hip_atomic_load(a.seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const size_t bank = (size_t)(tag & 1u) * a.world * 2;
  const unsigned long long key = *slot;
  const int lane = threadIdx.x;
  if (lane < 2) {
    const uint32_t w = lane == 0 ? (uint32_t)key : (uint32_t)(key >> 32);
    const unsigned long long g = (unsigned long long)w | ((unsigned long long)tag << 32);
    for (int r = 0; r < a.world; ++r)
      if (r != a.rank)
        __hip_atomic_store(a.peer[r] + bank + (size_t)a.rank * 2 + lane, g, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool late = false;
  unsigned long long best = key;
  // lane r < world polls rank r's two words
  if (lane < a.world && lane != a.rank) {
    const unsigned long long lo = ar_poll(a.inbox + bank + (size_t)lane * 2, tag, t0,
                                          a.timeout_ticks, late);
    const unsigned long long hi = ar_poll(a.inbox + bank + (size_t)lane * 2 + 1, tag, t0,
                                          a.timeout_ticks, late);
    const unsigned long long k = (lo & 0xffffffffull) | ((hi & 0xffffffffull) << 32);
    best = k > best ? k : best;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(best, off, 64);
    best = o > best ? o : best;
  }
  if (late) atomicOr(a.err, 1);
  __syncthreads();
  if (lane == 0) *slot = best;
  ar_finish(a, tag);
}

// full[0, n) on every rank <- the ranks' contiguous shards: this rank owns
// [off, off + n_local) = shard[0, n_local).  The inbox holds 2 banks x n granules;
// every rank writes its shard at its global offset in every peer's bank.
__global__ __launch_bounds__(kArThreads) void ar_gather_kernel(ArArgs a, const float* __restrict__ shard,
                                                               int off, int n_local,
                                                               float* __restrict__ full) {
  const unsigned int tag = __hip_atomic_load(a.seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const size_t bank = (size_t)(tag & 1u) * a.n;
  const int i0 = blockIdx.x * kArThreads + threadIdx.x, stride = gridDim.x * kArThreads;
  for (int i = i0; i < n_local; i += stride) {
    const float v = shard[i];
    const unsigned long long g = (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
    for (int r = 0; r < a.world; ++r)
      if (r != a.rank)
        __hip_atomic_store(a.peer[r] + bank + off + i, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    full[off + i] = v;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool late = false;
  for (int i = i0; i < a.n; i += stride) {
    if (i >= off && i < off + n_local) continue;
    const unsigned long long g = ar_poll(a.inbox + bank + i, tag, t0, a.timeout_ticks, late);
    full[i] = __uint_as_float((uint32_t)g);
  }
  if (late) atomicOr(a.err, 1);
  ar_finish(a, tag);
}

}  // namespace cake

using namespace cake;

static int ar_args(ArArgs& a, void* const* peers, const void* inbox, unsigned int* seq, int* err,
                   int rank, int world, int n, double timeout_s) {
  if (world < 1 || world > kArMaxRanks || rank < 0 || rank >= world || n <= 0 || !inbox ||
      !seq || !err || timeout_s <= 0)
    return (int)hipErrorInvalidValue;
  for (int r = 0; r < kArMaxRanks; ++r) {
    a.peer[r] = (r < world && r != rank) ? (unsigned long long*)peers[r] : nullptr;
    if (r < world && r != rank && a.peer[r] == nullptr) return (int)hipErrorInvalidValue;
  }
  a.inbox = (const unsigned long long*)inbox;
  a.seq = seq;
  a.err = err;
  a.rank = rank;
  a.world = world;
  a.n = n;
  a.timeout_ticks = (unsigned long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  return 0;
}

// Inbox granules needed for vectors of n words: 2 parity banks x world x n.
CAKE_API long long cake_ar_inbox_words(int world, int n) { return 2ll * world * n; }

// out (+)= sum over ranks of partial (f32[n]); partial and out may alias when !accumulate.
CAKE_API int cake_ar_sum(const float* partial, float* out, int n, int accumulate, void* const* peers,
                         const void* inbox, unsigned int* seq, int* err, int rank, int world,
                         double timeout_s, hipStream_t st) {
  ArArgs a;
  const int rc = ar_args(a, peers, inbox, seq, err, rank, world, n, timeout_s);
  if (rc) return rc;
  int g = (n + kArThreads - 1) / kArThreads;
  if (g > 64) g = 64;
  if (accumulate)
    hipLaunchKernelGGL((ar_sum_kernel<true>), dim3(g), dim3(kArThreads), 0, st, a, partial, out);
  else
    hipLaunchKernelGGL((ar_sum_kernel<false>), dim3(g), dim3(kArThreads), 0, st, a, partial, out);
  return (int)hipGetLastError();
}

// *slot = max over ranks of *slot (u64 argmax key); the inbox must hold n = 2 words.
CAKE_API int cake_ar_max_key(unsigned long long* slot, void* const* peers, const void* inbox,
                             unsigned int* seq, int* err, int rank, int world, double timeout_s,
                             hipStream_t st) {
  ArArgs a;
  const int rc = ar_args(a, peers, inbox, seq, err, rank, world, 2, timeout_s);
  if (rc) return rc;
  hipLaunchKernelGGL(ar_max_key_kernel, dim3(1), dim3(64), 0, st, a, slot);
  return (int)hipGetLastError();
}

// full (f32[n]) on every rank <- concatenation of the ranks' shards (shard = this
// rank's [off, off + n_local)); the inbox must hold 2 x n granules.
CAKE_API int cake_ar_gather(const float* shard, int off, int n_local, float* full, int n,
                            void* const* peers, const void* inbox, unsigned int* seq, int* err,
                            int rank, int world, double timeout_s, hipStream_t st) {
  ArArgs a;
  const int rc = ar_args(a, peers, inbox, seq, err, rank, world, n, timeout_s);
  if (rc) return rc;
  if (off < 0 || n_local < 0 || off + n_local > n) return (int)hipErrorInvalidValue;
  int g = (n + kArThreads * 8 - 1) / (kArThreads * 8);
  if (g > 64) g = 64;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(ar_gather_kernel, dim3(g), dim3(kArThreads), 0, st, a, shard, off, n_local, full);
  return (int)hipGetLastError();
}
