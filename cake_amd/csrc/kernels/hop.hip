// Device-side pipeline hop: the hidden state of one token moves rank -> rank
// as a peer-to-peer store stream over xGMI, with no host involvement, so each
// rank's whole decode step (receive, its layers, send) is ONE hipGraph replay.
//
// Replaces the reference's per-token TCP round trip of the hidden state
// (cake-core/src/cake/client.rs:50-59, 116-124 -> worker.rs:236-252), which
// copies the tensor device -> host -> socket -> host -> device on both ends
// (proto/message.rs:22-38).
//
// Protocol (the "low-latency" flag-in-data form): every 32-bit payload word
// travels in one naturally aligned 8-byte granule {word, tag} written by ONE
// system-scope store, so a reader that sees the expected tag also sees the word
// (no fences, no separate flag).  The tag is a per-(sender, inbox) sequence
// number kept in device memory on both sides and advanced by the kernels
// themselves, so graph replays stay in lock step.  The receiver's inbox lives
// in uncached device memory on the receiving GPU (hipDeviceMallocUncached),
// exported to the sender through a HIP IPC handle; the receiver polls with
// system-scope loads and a bounded wall-clock timeout (s_memrealtime, 100 MHz)
// that raises an error word instead of hanging the GPU when a peer dies.
//
// Payload encodings: f32 words (exact), or bf16 pairs (half the bytes; the
// reference ships activations in the 16-bit model dtype anyway) followed by
// `nhdr` raw 32-bit header words (position, stream id, flags).
#include "common.h"

namespace cake {

constexpr int kHopThreads = 512;

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}

// src: H f32 hidden values followed by nhdr 32-bit header words (one buffer).
template <bool BF16>
__global__ __launch_bounds__(kHopThreads) void hop_send_kernel(
    const float* __restrict__ src, int H, int nhdr, unsigned long long* __restrict__ dst,
    unsigned int* __restrict__ seq) {
  const unsigned int tag = *seq + 1u;
  const int nw = (BF16 ? H / 2 : H) + nhdr;
  const uint32_t* hw = reinterpret_cast<const uint32_t*>(src + H);
  for (int i = threadIdx.x; i < nw; i += kHopThreads) {
    uint32_t w;
    const int nh = BF16 ? H / 2 : H;
    if (i < nh) {
      if constexpr (BF16) {
        const float2 v = reinterpret_cast<const float2*>(src)[i];
        w = pack_bf16x2(v.x, v.y);
      } else {
        w = __float_as_uint(src[i]);
      }
    } else {
      w = hw[i - nh];
    }
    const unsigned long long g = (unsigned long long)w | ((unsigned long long)tag << 32);
    __hip_atomic_store(dst + i, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();  // every thread has read *seq
  if (threadIdx.x == 0) *seq = tag;
}

template <bool BF16>
__global__ __launch_bounds__(kHopThreads) void hop_recv_kernel(
    const unsigned long long* __restrict__ inbox, int H, int nhdr, float* __restrict__ dst,
    unsigned int* __restrict__ seq, int* __restrict__ err, unsigned long long timeout_ticks) {
  const unsigned int tag = *seq + 1u;
  const int nh = BF16 ? H / 2 : H;
  const int nw = nh + nhdr;
  uint32_t* hw = reinterpret_cast<uint32_t*>(dst + H);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  // fail fast: once a receive of this rank timed out (the error word is set until the
  // host reads and clears it), later receives of the same run do not wait again — a
  // dead peer costs one timeout, not one per queued replay
  bool timed_out = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  for (int i = threadIdx.x; i < nw; i += kHopThreads) {
    unsigned long long g;
    for (;;) {
      g = __hip_atomic_load(inbox + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((unsigned int)(g >> 32) == tag || timed_out) break;
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) timed_out = true;
    }
    const uint32_t w = (uint32_t)g;
    if (i < nh) {
      if constexpr (BF16) {
        reinterpret_cast<float2*>(dst)[i] =
            make_float2(bf16_to_f32((uint16_t)(w & 0xffffu)), bf16_to_f32((uint16_t)(w >> 16)));
      } else {
        dst[i] = __uint_as_float(w);
      }
    } else {
      hw[i - nh] = w;
    }
  }
  if (timed_out) atomicOr(err, 1);
  __syncthreads();
  if (threadIdx.x == 0) *seq = tag;
}

// ---------------------------------------------------------------------------
// Bulk hop: a multi-megabyte message (the split UNet's feature map and skip tensors)
// rank -> rank inside the step graphs.  Granules double the bytes and one workgroup
// cannot fill an xGMI link, so the bulk form moves 16-byte chunks with a grid:
//   send: every workgroup copies its share of the source segments straight into the
//     receiver's inbox (uncached device memory on the receiving GPU, IPC-mapped here)
//     with system-scope (sc0 sc1) buffer stores, waits for its stores to be
//     acknowledged (s_waitcnt 0), then counts itself in; the last workgroup to arrive
//     stores the message tag into the inbox's flag word (one system-scope 8-byte
//     store) and advances the channel's send sequence.  No release fence: every data
//     store is complete before the counter that enables the flag moves.
//   recv: one workgroup polls the flag (system scope, bounded by the wall-clock
//     timeout; fail fast on an already-raised error word) and advances the receive
//     sequence, then a copy grid moves the inbox into the local state buffer with
//     system-scope loads (the inbox is uncached: no stale line can be read).
// A channel carries one message per step; the sender cannot overwrite an inbox before
// the receiver copied it out, because the split-UNet step is a ring (the next message
// on a channel depends on the receiver's output of this step).
constexpr int kBulkThreads = 256;
constexpr int kBulkSegs = 32;
constexpr int kBulkSys = 17;  // cache policy sc0 | sc1: system scope

struct BulkSegs {
  const uint4* src[kBulkSegs];
  unsigned long long n16[kBulkSegs];   // 16-byte chunks of segment k
  unsigned long long off16[kBulkSegs]; // its offset in the message, in chunks
  int n;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t bulk_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff,
                                           0x00020000);
}

__global__ __launch_bounds__(kBulkThreads) void bulk_send_kernel(
    BulkSegs s, uint4* __restrict__ dst, unsigned long long* __restrict__ flag,
    unsigned int* __restrict__ seq, unsigned int* __restrict__ count) {
  const size_t nt = (size_t)gridDim.x * kBulkThreads;
  const size_t t = (size_t)blockIdx.x * kBulkThreads + threadIdx.x;
  for (int k = 0; k < s.n; ++k) {
    const uint4* src = s.src[k];
    const __amdgpu_buffer_rsrc_t r = bulk_rsrc(dst + s.off16[k]);
    const size_t n = s.n16[k];
    size_t i = t;
    for (; i + 3 * nt < n; i += 4 * nt) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src[i + u * nt];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const u32x4 w = {v[u].x, v[u].y, v[u].z, v[u].w};
        __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)((i + u * nt) * 16), 0, kBulkSys);
      }
    }
    for (; i < n; i += nt) {
      const uint4 v = src[i];
      const u32x4 w = {v.x, v.y, v.z, v.w};
      __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)(i * 16), 0, kBulkSys);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // this thread's stores are acknowledged
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {  // last workgroup: every chunk has landed
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned int tag = *seq + 1u;
      __hip_atomic_store(flag, ((unsigned long long)tag << 32) | tag, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      *seq = tag;
    }
  }
}

// one workgroup waits for the flag (a waiting grid would hold every CU while the ranks
// that share a GPU in the rehearsal need them to produce the message), then the copy
// grid runs behind it on the same stream
__global__ __launch_bounds__(64) void bulk_wait_kernel(const unsigned long long* __restrict__ flag,
                                                       unsigned int* __restrict__ seq,
                                                       int* __restrict__ err,
                                                       unsigned long long timeout_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned int tag = *seq + 1u;
  bool timed_out = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (!timed_out) {
    const unsigned long long g = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((unsigned int)g == tag && (unsigned int)(g >> 32) == tag) break;
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) timed_out = true;
  }
  if (timed_out) atomicOr(err, 1);
  *seq = tag;
}

__global__ __launch_bounds__(kBulkThreads) void bulk_copy_kernel(const uint4* __restrict__ rx,
                                                                 unsigned long long n16,
                                                                 uint4* __restrict__ dst) {
  const __amdgpu_buffer_rsrc_t r = bulk_rsrc(rx);
  const size_t nt = (size_t)gridDim.x * kBulkThreads;
  size_t i = (size_t)blockIdx.x * kBulkThreads + threadIdx.x;
  for (; i + 3 * nt < n16; i += 4 * nt) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)((i + u * nt) * 16), 0, kBulkSys);
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[i + u * nt] = make_uint4(v[u].x, v[u].y, v[u].z, v[u].w);
  }
  for (; i < n16; i += nt) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, kBulkSys);
    dst[i] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

}  // namespace cake

using namespace cake;

// Inbox memory: uncached device memory (coherent with peer writes), zeroed.
CAKE_API int cake_hop_alloc(size_t bytes, void** ptr) {
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, bytes);
}

CAKE_API int cake_hop_free(void* ptr) { return (int)hipFree(ptr); }

CAKE_API int cake_ipc_handle(void* ptr, void* out64) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) <= 64, "IPC handle size");
  __builtin_memcpy(out64, &h, sizeof(h));
  return 0;
}

CAKE_API int cake_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

CAKE_API int cake_ipc_open(const void* in64, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, in64, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

CAKE_API int cake_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// Words (= 8-byte granules) of one hop message.
CAKE_API int cake_hop_words(int H, int nhdr, int bf16) { return (bf16 ? H / 2 : H) + nhdr; }

CAKE_API int cake_hop_send(const float* src, int H, int nhdr, int bf16, void* dst_inbox,
                           unsigned int* seq, hipStream_t st) {
  if (H <= 0 || nhdr < 0 || (bf16 && H % 2)) return (int)hipErrorInvalidValue;
  if (bf16)
    hipLaunchKernelGGL((hop_send_kernel<true>), dim3(1), dim3(kHopThreads), 0, st, src, H, nhdr,
                       (unsigned long long*)dst_inbox, seq);
  else
    hipLaunchKernelGGL((hop_send_kernel<false>), dim3(1), dim3(kHopThreads), 0, st, src, H, nhdr,
                       (unsigned long long*)dst_inbox, seq);
  return (int)hipGetLastError();
}

CAKE_API int cake_hop_recv(const void* inbox, int H, int nhdr, int bf16, float* dst,
                           unsigned int* seq, int* err, double timeout_s, hipStream_t st) {
  if (H <= 0 || nhdr < 0 || (bf16 && H % 2) || timeout_s <= 0) return (int)hipErrorInvalidValue;
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);  // 100 MHz
  if (bf16)
    hipLaunchKernelGGL((hop_recv_kernel<true>), dim3(1), dim3(kHopThreads), 0, st,
                       (const unsigned long long*)inbox, H, nhdr, dst, seq, err, ticks);
  else
    hipLaunchKernelGGL((hop_recv_kernel<false>), dim3(1), dim3(kHopThreads), 0, st,
                       (const unsigned long long*)inbox, H, nhdr, dst, seq, err, ticks);
  return (int)hipGetLastError();
}

// Bulk hop (see bulk_send_kernel).  The inbox is `rx_bytes` of message plus one 64-byte
// flag line (cake_hop_alloc(rx_bytes + 64)); offsets and sizes are multiples of 16 and a
// message stays below 2 GB (32-bit buffer offsets).  seq / count / err: device words of
// this end of the channel (zeroed once; the receiver has no counter).
static int bulk_grid(unsigned long long n16) {
  const unsigned long long per = (unsigned long long)kBulkThreads * 4;
  unsigned long long g = (n16 + per - 1) / per;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return (int)g;
}

CAKE_API int cake_bulk_send(const void* const* srcs, const unsigned long long* bytes,
                            const unsigned long long* offs, int nseg, void* dst_rx,
                            unsigned long long rx_bytes, unsigned int* seq, unsigned int* count,
                            hipStream_t st) {
  if (nseg < 1 || nseg > kBulkSegs || rx_bytes % 16 || rx_bytes >= (1ull << 31))
    return (int)hipErrorInvalidValue;
  BulkSegs s{};
  s.n = nseg;
  unsigned long long most = 0;
  for (int k = 0; k < nseg; ++k) {
    if (bytes[k] % 16 || offs[k] % 16 || (reinterpret_cast<uintptr_t>(srcs[k]) & 15) ||
        offs[k] + bytes[k] > rx_bytes)
      return (int)hipErrorInvalidValue;
    s.src[k] = reinterpret_cast<const uint4*>(srcs[k]);
    s.n16[k] = bytes[k] / 16;
    s.off16[k] = offs[k] / 16;
    if (s.n16[k] > most) most = s.n16[k];
  }
  uint4* dst = reinterpret_cast<uint4*>(dst_rx);
  auto* flag = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(dst_rx) + rx_bytes);
  hipLaunchKernelGGL(bulk_send_kernel, dim3(bulk_grid(most)), dim3(kBulkThreads), 0, st, s, dst,
                     flag, seq, count);
  return (int)hipGetLastError();
}

CAKE_API int cake_bulk_recv(const void* rx, unsigned long long bytes, void* dst,
                            unsigned int* seq, int* err, double timeout_s, hipStream_t st) {
  if (bytes % 16 || bytes >= (1ull << 31) || (reinterpret_cast<uintptr_t>(dst) & 15) ||
      timeout_s <= 0)
    return (int)hipErrorInvalidValue;
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);  // 100 MHz
  const auto* flag = reinterpret_cast<const unsigned long long*>(
      reinterpret_cast<const char*>(rx) + bytes);
  hipLaunchKernelGGL(bulk_wait_kernel, dim3(1), dim3(64), 0, st, flag, seq, err, ticks);
  hipLaunchKernelGGL(bulk_copy_kernel, dim3(bulk_grid(bytes / 16)), dim3(kBulkThreads), 0, st,
                     reinterpret_cast<const uint4*>(rx), bytes / 16,
                     reinterpret_cast<uint4*>(dst));
  return (int)hipGetLastError();
}
