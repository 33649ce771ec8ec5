// mv_q80.hip — the single-token matvec instantiations for T_Q8_0 weights (mv_kernels.h).
#include "mv_kernels.h"

// mv_q80_x86.hip includes this file with LLMI_MV_X86 = 1 (the x86-numerics instantiations)
#ifndef LLMI_MV_X86
#define LLMI_MV_X86 0
#endif

namespace llmi {
template hipError_t mv_dispatch_epi<1, true, T_Q8_0, LLMI_MV_X86>(const MVArgs&, int, dim3, size_t, hipStream_t);
template hipError_t mv_dispatch_epi<1, false, T_Q8_0, LLMI_MV_X86>(const MVArgs&, int, dim3, size_t, hipStream_t);
}  // namespace llmi
