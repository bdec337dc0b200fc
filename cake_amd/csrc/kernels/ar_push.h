// Tensor-parallel all-reduce granule push, shared by allreduce.hip and the GEMV
// epilogue that produces the partial sums (gemv.hip): each f32 word travels to
// every peer as ONE system-scope 8-byte store {word, tag} into the peer's inbox
// bank for this all-reduce (see allreduce.hip for the protocol).
#pragma once
#include "common.h"

namespace cake {

constexpr int kArMaxRanks = 8;

struct ArPush {
  unsigned long long* peer[kArMaxRanks];  // peers' inboxes [2][world][n] (own: unused)
  const unsigned int* seq;                // this channel's tag counter (read-only here)
  int rank, world, n;
};

// Tag of the all-reduce about to run on this channel (the pull kernel advances it).
__device__ __forceinline__ unsigned int ar_next_tag(const unsigned int* seq) {
  return __hip_atomic_load(seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

__device__ __forceinline__ void ar_push_word(const ArPush& p, unsigned int tag, int i, float v) {
  const size_t bank = (size_t)(tag & 1u) * p.world * p.n;
  const unsigned long long g =
      (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
  for (int r = 0; r < p.world; ++r)
    if (r != p.rank)
      __hip_atomic_store(p.peer[r] + bank + (size_t)p.rank * p.n + i, g, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace cake
