// launch_util.h — host-side launch helper shared by the kernel translation units
// (kernels.hip, the per-type matvec units mv_*.hip, prefill.hip).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

namespace llmi {

// Launch-event hook (llmi_profile_kernels, kernels.hip): while armed, the timed launches
// record `start` when the first kernel of the op begins and `stop` when the last one ends
// (hipExtLaunchKernelGGL), i.e. kernel execution time without dependent-launch gaps.
hipEvent_t launch_event(bool stop);

// CUs of the current device, cached per device (in-process replicas run one scheduler
// thread per GPU; a benign race writes the same value twice)
static inline int cu_count() {
    static int cache[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    int n = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
    if (n == 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 0) n = 0;
        __atomic_store_n(&cache[dev], n, __ATOMIC_RELAXED);
    }
    return n;
}

template <typename K, typename... Args>
static void launch_k(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, bool first, bool last, Args... args) {
    hipEvent_t e0 = first ? launch_event(false) : nullptr, e1 = last ? launch_event(true) : nullptr;
    if (e0 || e1) hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, s, e0, e1, 0, args...);
    else hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}

}  // namespace llmi
