// mv_q80.hip — the single-token matvec instantiations for T_Q8_0 weights (mv_kernels.h).
#include "mv_kernels.h"

namespace llmi {
template hipError_t mv_dispatch_epi<1, true, T_Q8_0>(const MVArgs&, int, dim3, size_t, hipStream_t);
template hipError_t mv_dispatch_epi<1, false, T_Q8_0>(const MVArgs&, int, dim3, size_t, hipStream_t);
}  // namespace llmi
