// Instantiates the GEMM launchers (gemm_kernel.h) for f16, epilogues Store, Resid32, Add16, Swiglu;
// split from gemm.hip so the heavy instantiations compile in parallel.
#include "gemm_kernel.h"

namespace cake {
template int launch_gemm<kF16, kEpiStore>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kF16, kEpiResid32>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kF16, kEpiAdd16>(int, dim3, hipStream_t, const GemmArgs&);
template int launch_gemm<kF16, kEpiSwiglu>(int, dim3, hipStream_t, const GemmArgs&);
}  // namespace cake
