// mfma64_probe.hip — what v_mfma_f64_16x16x4_f64 does on gfx950 (k_pf_fa's instruction):
//  1. summation semantics: a k-ordered chain of fma roundings (the oracle's sequential
//     double sum), a pairwise tree, or one rounding of a wider sum, told apart by
//     products [2^53, 1, 1, -2^53] (sequential 0, pairwise 1, exact 2) and a C of 2^53
//     with products [1, 1, 0, 0] (sequential 2^53, exact 2^53 + 2);
//  2. issue rate and dependent latency per SIMD (s_memtime around back-to-back MFMAs
//     on 1 / 4 / 8 independent accumulators, one wave);
//  3. whole-chip FP64 MFMA TFLOP/s (every CU, 4 or 8 waves each).
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma64_probe.hip -o tools/mfma64_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_sem(const double* a, const double* b, const double* c, double* d) {
    const int l = threadIdx.x;
    d4 acc = {c[0], c[0], c[0], c[0]};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) d[l * 4 + i] = acc[i];
}

template <int NACC>
__global__ void k_rate(double x, int iters, double* out, long long* cyc) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
    const double a = x + threadIdx.x, b = x - threadIdx.x;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    const long long t1 = clock64();
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

// B operand rebuilt before every MFMA: MODE 1 f16 -> f32 -> f64 (two VALU cvts, one on
// the f64 path), MODE 2 f32 -> f64 only, MODE 3 f16 -> f32 only (b fed as (double) of a
// loop-invariant f32 plus an f32 add), MODE 4 eight extra f32 VALU ops per MFMA
template <int NACC, int MODE>
__global__ void k_rate_b(double x, int iters, double* out, long long* cyc) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
    const double a = x + threadIdx.x;
    float f = (float)threadIdx.x;
    unsigned h = 0x3c00u + threadIdx.x;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) {
            double b;
            if constexpr (MODE == 1) b = (double)(float)__builtin_bit_cast(_Float16, (unsigned short)(h + it + i));
            else if constexpr (MODE == 2) b = (double)(f + (float)(it + i));
            else if constexpr (MODE == 3) b = x + (double)(int)(h + it + i);
            else {
                float g = f + (float)it;
#pragma unroll
                for (int k = 0; k < 8; ++k) g = g * 1.0001f + 0.5f;
                f = g;
                b = x;
            }
            acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
        }
    }
    const long long t1 = clock64();
    double s = f;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

// 8 waves = 2 per SIMD: waves 0-3 run MFMAs only, waves 4-7 VALU f32 FMAs only (8
// independent chains) -- do the two kinds share a SIMD's time or overlap?
__global__ void k_mix(int iters, int valu_iters, double* out, long long* cyc) {
    const int w = threadIdx.x >> 6;
    const long long t0 = clock64();
    double s = 0;
    if (w < 4) {
        d4 acc[4];
        for (int i = 0; i < 4; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
        const double a = 1.0 + threadIdx.x, b = 2.0;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
        for (int i = 0; i < 4; ++i) s += acc[i][0];
    } else if (valu_iters > 0) {
        float g[8];
        for (int k = 0; k < 8; ++k) g[k] = threadIdx.x + k;
        for (int it = 0; it < valu_iters; ++it)
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = g[k] * 1.0001f + 0.5f;
        for (int k = 0; k < 8; ++k) s += g[k];
    }
    const long long t1 = clock64();
    out[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
}

// the same mix for the f16 MFMA k_pf_gemm runs on (v_mfma_f32_16x16x32_f16)
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k_mix16(int iters, int valu_iters, double* out, long long* cyc) {
    const int w = threadIdx.x >> 6;
    const long long t0 = clock64();
    double s = 0;
    if (w < 4) {
        f4 acc[4];
        for (int i = 0; i < 4; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
        h8 a, b;
        for (int k = 0; k < 8; ++k) { a[k] = (_Float16)(threadIdx.x + k); b[k] = (_Float16)1.f; }
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
        for (int i = 0; i < 4; ++i) s += acc[i][0];
    } else if (valu_iters > 0) {
        float g[8];
        for (int k = 0; k < 8; ++k) g[k] = threadIdx.x + k;
        for (int it = 0; it < valu_iters; ++it)
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = g[k] * 1.0001f + 0.5f;
        for (int k = 0; k < 8; ++k) s += g[k];
    }
    const long long t1 = clock64();
    out[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
}

int main() {
    // ---- 1. semantics: row 0 / column 0 of the 16x16 result = sum_k A[0][k] B[k][0]
    double ha[64], hb[64], hc = 0.0, hd[256];
    for (int l = 0; l < 64; ++l) { ha[l] = 0.0; hb[l] = 0.0; }
    // lane l holds A[l & 15][l >> 4] and B[l >> 4][l & 15]: k = l >> 4 for row / col 0
    const double p[4] = {ldexp(1.0, 53), 1.0, 1.0, -ldexp(1.0, 53)};
    for (int k = 0; k < 4; ++k) { ha[16 * k] = p[k]; hb[16 * k] = 1.0; }
    double *da, *db, *dc, *dd, *dout;
    long long* dcyc;
    hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dc, 8); hipMalloc(&dd, sizeof hd);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipMemcpy(dc, &hc, 8, hipMemcpyHostToDevice);
    k_sem<<<1, 64>>>(da, db, dc, dd);
    hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
    // C/D row (lane >> 4) + 4 i, col lane & 15: row 0 col 0 = lane 0, reg 0
    printf("{\"products_2p53_1_1_m2p53\": %.17g, ", hd[0]);
    const double p2[4] = {1.0, 1.0, 0.0, 0.0};
    for (int k = 0; k < 4; ++k) ha[16 * k] = p2[k];
    hc = ldexp(1.0, 53);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(dc, &hc, 8, hipMemcpyHostToDevice);
    k_sem<<<1, 64>>>(da, db, dc, dd);
    hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
    printf("\"c2p53_plus_1_1_minus_2p53\": %.17g, ", hd[0] - ldexp(1.0, 53));
    // ---- 2. one wave: cycles per MFMA
    hipMalloc(&dout, sizeof(double) * 256 * 8 * 64);
    hipMalloc(&dcyc, 8);
    long long cyc = 0;
    const int iters = 4096;
    k_rate<1><<<1, 64>>>(1.0, iters, dout, dcyc);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("\"cycles_dependent\": %.2f, ", (double)cyc / iters);
    k_rate<4><<<1, 64>>>(1.0, iters, dout, dcyc);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("\"cycles_per_mfma_4acc\": %.2f, ", (double)cyc / iters / 4);
    k_rate<8><<<1, 64>>>(1.0, iters, dout, dcyc);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("\"cycles_per_mfma_8acc\": %.2f, ", (double)cyc / iters / 8);
    // ---- 3. whole chip
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int wpc = 4; wpc <= 8; wpc += 4) {
        const int big = 20000;
        k_rate<4><<<cus, 64 * wpc>>>(1.0, 100, dout, dcyc);
        hipEventRecord(e0);
        k_rate<4><<<cus, 64 * wpc>>>(1.0, big, dout, dcyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = (double)cus * wpc * big * 4 * 2048.0;
        printf("\"tflops_%dwaves_per_cu\": %.1f%s", wpc, flops / (ms * 1e-3) / 1e12, wpc == 8 ? "" : ", ");
    }
    printf(", \"cus\": %d, ", cus);
    // ---- 4. one wave, VALU work beside each MFMA
    k_rate_b<4, 1><<<1, 64>>>(1.0, iters, dout, dcyc);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("\"cycles_per_mfma_b_f16_f32_f64\": %.2f, ", (double)cyc / iters / 4);
    k_rate_b<4, 2><<<1, 64>>>(1.0, iters, dout, dcyc);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("\"cycles_per_mfma_b_f32_f64\": %.2f, ", (double)cyc / iters / 4);
    k_rate_b<4, 3><<<1, 64>>>(1.0, iters, dout, dcyc);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("\"cycles_per_mfma_b_i32_f64_add\": %.2f, ", (double)cyc / iters / 4);
    k_rate_b<4, 4><<<1, 64>>>(1.0, iters, dout, dcyc);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("\"cycles_per_mfma_8_f32_fma\": %.2f, ", (double)cyc / iters / 4);
    // ---- 5. MFMA waves beside VALU waves on the same SIMDs
    long long* dc8;
    hipMalloc(&dc8, 8 * 8);
    long long c8[8];
    for (int vi : {0, 4 * iters}) {
        k_mix<<<1, 512>>>(iters, vi, dout, dc8);
        hipMemcpy(c8, dc8, 64, hipMemcpyDeviceToHost);
        printf("\"mix_valu%d_mfma_wave_cycles_per_mfma\": %.2f, \"mix_valu%d_valu_wave_cycles\": %lld, ", vi ? 1 : 0,
               (double)c8[0] / iters / 4, vi ? 1 : 0, c8[4]);
    }
    k_mix<<<1, 512>>>(0, 4 * iters, dout, dc8);
    hipMemcpy(c8, dc8, 64, hipMemcpyDeviceToHost);
    printf("\"valu_alone_cycles\": %lld, ", c8[4]);
    for (int vi : {0, 4 * iters}) {
        k_mix16<<<1, 512>>>(4 * iters, vi, dout, dc8);
        hipMemcpy(c8, dc8, 64, hipMemcpyDeviceToHost);
        printf("\"f16_mix_valu%d_mfma_cycles_per_mfma\": %.2f, \"f16_mix_valu%d_valu_wave_cycles\": %lld, ", vi ? 1 : 0,
               (double)c8[0] / iters / 16, vi ? 1 : 0, c8[4]);
    }
    printf("\"end\": 0}\n");
    return 0;
}
