// mv_q6k.hip — the single-token matvec instantiations for T_Q6_K weights (mv_kernels.h).
#include "mv_kernels.h"

namespace llmi {
template hipError_t mv_dispatch_epi<0, true, T_Q6_K>(const MVArgs&, int, dim3, size_t, hipStream_t);
template hipError_t mv_dispatch_epi<0, false, T_Q6_K>(const MVArgs&, int, dim3, size_t, hipStream_t);
}  // namespace llmi
