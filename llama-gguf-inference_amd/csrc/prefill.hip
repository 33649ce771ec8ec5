// prefill.hip — the batched-prefill translation unit (prefill.hip.inc: MFMA prompt prefill).
#include "kernels.h"
#include "launch_util.h"
#include "mv_device.h"
#include "pf_device.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

namespace llmi {
#include "prefill.hip.inc"
}  // namespace llmi
