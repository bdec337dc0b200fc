// Instantiates the GEMM launchers (gemm_kernel.h) for bf16, epilogues Geglu, Partial, Store32, Silu;
// split from gemm.hip so the heavy instantiations compile in parallel.
#include "gemm_kernel.h"

namespace cake {
template int launch_gemm<kBF16, kEpiGeglu>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kBF16, kEpiPartial>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kBF16, kEpiStore32>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kBF16, kEpiSilu>(int, dim3, hipStream_t, const GemmArgs&);
}  // namespace cake
