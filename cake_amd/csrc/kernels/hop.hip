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
