// mv_q5k_x86.hip — the x86-numerics (X86 = 1) instantiations of mv_q5k.hip, a separate
// translation unit so the two builds compile in parallel.
#define LLMI_MV_X86 1
#include "mv_q5k.hip"
