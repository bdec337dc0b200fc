// Diagnostic build: where the four-wave 256x256 GEMM's k-loop (gemm_4w.h, cfg 22) spends
// its cycles.  Compiles the kernel with CAKE_GEMM_STAMPS (s_memtime at the segment
// boundaries of every k-step, summed per wave); never linked into the library.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -inline-threshold=100000 \
//         scripts/gemm_stamp.hip -o scripts/gemm_stamp
//   ./scripts/gemm_stamp [M N K]
//
// Segments per k-step (shares are meaningful, absolute lengths include the stamps' own
// cost of ~40 cycles each):
//   A  first half's 64 MFMAs + the next half's 16 fragment reads (issue stream)
//   B  LDS-read drain + vmcnt(0) (the next step's DMA) + barrier
//   C  second half's 64 MFMAs + 16 DMAs + 16 fragment reads (issue stream)
//   D  LDS-read drain at the step's end
// and per tile: prologue (entry -> loop) and epilogue (loop end -> the tile's stores done).
#define CAKE_GEMM_STAMPS 1
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <hip/hip_runtime.h>

__device__ unsigned long long g_gemm_stamps[4096 * 4 * 8];

#include "../cake_amd/csrc/kernels/gemm_kernel.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// uniform [-1, 1) bf16 from a hash (random operands: zero-filled data clocks higher)
__global__ void fill_kernel(uint16_t* p, size_t n, unsigned seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned h = (unsigned)i * 2654435761u ^ seed;
  h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
  const float f = (float)(h & 0xFFFFFF) / 8388608.0f - 1.0f;
  p[i] = (uint16_t)(__float_as_uint(f) >> 16);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 8192;
  const int N = argc > 2 ? std::atoi(argv[2]) : 8192;
  const int K = argc > 3 ? std::atoi(argv[3]) : 8192;
  if (M % 256 || N % 256 || K % 64 || (size_t)(M / 256) * (N / 256) > 4096) {
    std::fprintf(stderr, "M, N multiples of 256, K of 64, at most 4096 tiles\n");
    return 2;
  }
  uint16_t *a, *b, *c;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&b, (size_t)N * K * 2));
  CK(hipMalloc(&c, (size_t)M * N * 2));
  fill_kernel<<<(unsigned)(((size_t)M * K + 255) / 256), 256>>>(a, (size_t)M * K, 1u);
  fill_kernel<<<(unsigned)(((size_t)N * K + 255) / 256), 256>>>(b, (size_t)N * K, 2u);
  cake::GemmArgs g{};
  g.a = a; g.b = b; g.c = c;
  g.lda = K; g.ldb = K; g.ldc = N;
  g.M = M; g.N = N; g.K = K; g.Nv = N; g.half = N;
  g.tiles_m = M / 256; g.tiles_n = N / 256; g.kps = K;
  const dim3 grid(g.tiles_m * g.tiles_n, 1);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 8; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((cake::gemm_4w_kernel<0, cake::kEpiStore, 256, 256, 0>), grid, dim3(256),
                       0, 0, g);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const size_t nw = (size_t)grid.x * 4;
  std::vector<unsigned long long> st(nw * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_gemm_stamps), st.size() * 8));
  const double steps = (double)K / 64;
  double seg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (size_t w = 0; w < nw; ++w)
    for (int i = 0; i < 8; ++i) seg[i] += (double)st[w * 8 + i];
  double tot = 0;
  for (int i = 0; i < 8; ++i) seg[i] /= nw;
  for (int i = 0; i < 4; ++i) tot += seg[i] / steps;
  const double tile = seg[0] + seg[1] + seg[2] + seg[3] + seg[4] + seg[5];
  const char* names[4] = {"A mfma64+reads16", "B drain+vmcnt0+barrier", "C mfma64+dma16+reads16",
                          "D drain"};
  std::printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"best_ms\": %.4f, \"tflops\": %.1f, "
              "\"cycles_per_kstep\": %.1f",
              M, N, K, best, 2.0 * M * N * K / best / 1e9, tot);
  for (int i = 0; i < 4; ++i)
    std::printf(", \"%s\": [%.1f, %.3f]", names[i], seg[i] / steps, seg[i] / steps / tot);
  std::printf(", \"tile_cycles\": %.0f, \"prologue\": [%.0f, %.3f], \"epilogue\": [%.0f, %.3f], "
              "\"epi_lead\": %.0f, \"epi_strips\": %.0f}\n",
              tile, seg[4], seg[4] / tile, seg[5], seg[5] / tile, seg[7], seg[6]);
  return 0;
}
