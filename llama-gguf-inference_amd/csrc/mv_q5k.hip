// mv_q5k.hip — the single-token matvec instantiations for T_Q5_K weights (mv_kernels.h).
#include "mv_kernels.h"

// mv_q5k_x86.hip includes this file with LLMI_MV_X86 = 1 (the x86-numerics instantiations)
#ifndef LLMI_MV_X86
#define LLMI_MV_X86 0
#endif

namespace llmi {
template hipError_t mv_dispatch_epi<0, true, T_Q5_K, LLMI_MV_X86>(const MVArgs&, int, dim3, size_t, hipStream_t);
template hipError_t mv_dispatch_epi<0, false, T_Q5_K, LLMI_MV_X86>(const MVArgs&, int, dim3, size_t, hipStream_t);
template hipError_t mv_qkv2_launch<true, T_Q5_K, T_Q6_K, LLMI_MV_X86>(const MVArgs&, int, dim3, size_t, hipStream_t);
template hipError_t mv_qkv2_launch<false, T_Q5_K, T_Q6_K, LLMI_MV_X86>(const MVArgs&, int, dim3, size_t, hipStream_t);
}  // namespace llmi
