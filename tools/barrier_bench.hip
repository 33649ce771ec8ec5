// barrier_bench.hip — microbenchmark of in-launch grid barriers on MI355X (one workgroup
// per CU), to price the phase seams of a persistent decode step against the ~1.2-1.5 us
// dependent-kernel boundary.  Each variant runs N barriers in one launch; between
// barriers every workgroup optionally publishes `pub` floats with write-through (sc1)
// stores and then reads a 4096-float vector written by other workgroups with sc1 loads
// (the residual hand-off of a decode layer).  Every spin is bounded: a timed-out wait
// sets a fault word and the kernel finishes.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/barrier_bench tools/barrier_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef unsigned __attribute__((address_space(1))) gu32;
constexpr unsigned kSpin = 1u << 22;

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
    return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// variant 0: one counter; 1: 8 shards (blockIdx % 8), lanes 0-7 of wave 0 poll one
// shard each; 2: 8 shards, last arriver of a shard bumps a top counter, one lane polls it
template <int V>
__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned phase, unsigned nwg, unsigned* fault) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int tid = threadIdx.x;
    bool ok = true;
    if (V == 0) {
        if (tid == 0) {
            __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (phase + 1) * nwg;
            unsigned s = 0;
            while (ld_sc1(bar) < target) {
                if (++s > kSpin) { ok = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    } else if (V == 1) {
        if (tid == 0) __hip_atomic_fetch_add(bar + 16 * (blockIdx.x & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tid < 8) {
            const unsigned cnt = (nwg - tid + 7) / 8;  // workgroups b with b % 8 == tid
            const unsigned target = (phase + 1) * cnt;
            unsigned s = 0;
            while (ld_sc1(bar + 16 * tid) < target) {
                if (++s > kSpin) { ok = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    } else {
        if (tid == 0) {
            const unsigned sh = blockIdx.x & 7, cnt = (nwg - sh + 7) / 8;
            const unsigned old = __hip_atomic_fetch_add(bar + 16 * sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == (phase + 1) * cnt) __hip_atomic_fetch_add(bar + 16 * 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (phase + 1) * 8;
            unsigned s = 0;
            while (ld_sc1(bar + 16 * 8) < target) {
                if (++s > kSpin) { ok = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    if (!ok) atomicOr(fault, 1u);
    __syncthreads();
    return ok;
}

template <int V>
__global__ __launch_bounds__(1024) void k_bar(unsigned* bar, int n, float* vec, int pub, float* sink, unsigned* fault) {
    float acc = 0.f;
    for (int p = 0; p < n; ++p) {
        if (pub) {  // publish this WG's slice of the vector (write-through), then read all of it
            const int per = (4096 + gridDim.x - 1) / gridDim.x;
            for (int i = threadIdx.x; i < per; i += blockDim.x) {
                const int e = blockIdx.x * per + i;
                if (e < 4096) __hip_atomic_store((gu32*)(vec + (p & 1) * 4096 + e), __float_as_uint((float)(p + e)), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (!grid_barrier<V>(bar, (unsigned)p, gridDim.x, fault)) return;
        if (pub) {
            for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
                const float v = __uint_as_float(ld_sc1((const unsigned*)(vec + (p & 1) * 4096 + i)));
                if (v != (float)(p + i)) atomicOr(fault, 2u);  // stale read
                acc += v;
            }
        }
    }
    if (acc == 1234.5f) sink[0] = acc;
}

int main(int argc, char** argv) {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned *bar, *fault;
    float *vec, *sink;
    CK(hipMalloc(&bar, 4096));
    CK(hipMalloc(&fault, 16));
    CK(hipMalloc(&vec, 2 * 4096 * 4));
    CK(hipMalloc(&sink, 16));
    CK(hipMemset(fault, 0, 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nwg = argc > 1 ? atoi(argv[1]) : cus;
    printf("CUs %d, grid %d x 1024 threads\n", cus, nwg);
    for (int pub = 0; pub < 2; ++pub)
        for (int v = 0; v < 3; ++v) {
            double t[2] = {0, 0};
            const int ns[2] = {1, 201};
            for (int k = 0; k < 2; ++k) {
                float best = 1e30f;
                for (int rep = 0; rep < 5; ++rep) {
                    CK(hipMemset(bar, 0, 4096));
                    CK(hipEventRecord(e0, 0));
                    if (v == 0) hipLaunchKernelGGL(k_bar<0>, dim3(nwg), dim3(1024), 0, 0, bar, ns[k], vec, pub, sink, fault);
                    if (v == 1) hipLaunchKernelGGL(k_bar<1>, dim3(nwg), dim3(1024), 0, 0, bar, ns[k], vec, pub, sink, fault);
                    if (v == 2) hipLaunchKernelGGL(k_bar<2>, dim3(nwg), dim3(1024), 0, 0, bar, ns[k], vec, pub, sink, fault);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (ms < best) best = ms;
                }
                t[k] = best * 1e3;
            }
            unsigned f = 0;
            CK(hipMemcpy(&f, fault, 4, hipMemcpyDeviceToHost));
            printf("variant %d pub %d: launch(1 barrier) %.2f us, per barrier %.3f us, fault %u\n", v, pub, t[0],
                   (t[1] - t[0]) / 200.0, f);
        }
    return 0;
}
