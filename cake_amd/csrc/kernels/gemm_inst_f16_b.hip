// Instantiates the GEMM launchers (gemm_kernel.h) for f16, epilogues Geglu, Partial, Store32, Silu;
// split from gemm.hip so the heavy instantiations compile in parallel.
#include "gemm_kernel.h"

namespace cake {
template int launch_gemm<kF16, kEpiGeglu>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kF16, kEpiPartial>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kF16, kEpiStore32>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kF16, kEpiSilu>(int, dim3, hipStream_t, const GemmArgs&);
}  // namespace cake
