/*
 * ggml_oracle.c — TEST INFRASTRUCTURE ONLY (see ggml_oracle.h): CPU restatement of the
 * reference's NGL=0 llama.cpp decode numerics.  PARITY UNPINNED by the reference
 * (SURVEY.md §8c): llama.cpp is an un-vendored, unpinned dependency
 * (Dockerfile.cpu:11 `FROM ghcr.io/ggml-org/llama.cpp:server`), invoked by
 * scripts/start.sh:235 (`LLAMA_BIN=/app/llama-server`) with `-ngl $NGL` at
 * scripts/start.sh:473-494; NGL=0 is the CPU path (Dockerfile.cpu:84-89).
 *
 * Every routine cites the upstream function it restates [upstream, recalled] and the
 * SURVEY.md row it covers.  Deviations from upstream, all documented in DESIGN.md:
 *   - exp() is llmi_expf (include/llmi_math.h) instead of libm/ggml SIMD exp;
 *   - compiled with -ffp-contract=off (upstream's FMA contraction depends on -march);
 *   - the Q4_K/Q5_K scale unpack uses get_scale_min_k4 (upstream's vec_dot uses the
 *     equivalent utmp/kmask bit trick; both yield the same 8 scales and 8 mins).
 */
#include "ggml_oracle.h"

#include <fcntl.h>
#include <math.h>
#if defined(__AVX2__)
#include <immintrin.h>
#endif
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/llmi_math.h"

#define QK_K 256
#define QK8_0 32

typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; } block_q4_K;
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; } block_q5_K;
typedef struct { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; } __attribute__((packed)) block_q6_K;
typedef struct { uint16_t d; int8_t qs[32]; } __attribute__((packed)) block_q8_0;
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; } block_q8_K;

_Static_assert(sizeof(block_q4_K) == 144, "q4_K");
_Static_assert(sizeof(block_q5_K) == 176, "q5_K");
_Static_assert(sizeof(block_q6_K) == 210, "q6_K");
_Static_assert(sizeof(block_q8_0) == 34, "q8_0");
_Static_assert(sizeof(block_q8_K) == 292, "q8_K");

static __thread char g_err[512];
const char* or_last_error(void) { return g_err; }
#define OR_FAIL(...) do { snprintf(g_err, sizeof g_err, __VA_ARGS__); goto fail; } while (0)

float or_fp16_to_fp32(uint16_t h) { return llmi_h2f(h); }
uint16_t or_fp32_to_fp16(float f) { return llmi_f2h(f); }
static inline float mode_expf(float x);
/* exp as the softmax / SiLU use it: llmi_expf (generic), ggml_v_expf or libm expf (x86 mode) */
float or_expf(float x) { return mode_expf(x); }

/* llmi_expf_glibc (llmi_math.h) against THIS host's libm expf for every float in
 * [lo, hi] (both finite, lo <= hi): the number of inputs whose bits differ, and the
 * first such input in *first.  Test infrastructure: pins the restatement the
 * flash-attention numerics use to a real glibc. */
int64_t or_expf_glibc_check(float lo, float hi, int fma, int stride, float* first) {
    int64_t bad = 0;
    /* walk the float line from lo to hi in order (every stride-th float) */
    float x = lo;
    for (;;) {
        const float a = llmi_expf_glibc(x, fma), b = expf(x);
        if (llmi_f2u(a) != llmi_f2u(b)) {
            if (!bad && first) *first = x;
            ++bad;
        }
        if (x >= hi) break;
        for (int i = 0; i < stride && x < hi; ++i) x = nextafterf(x, hi);
    }
    return bad;
}

size_t or_type_size(int t) {
    switch (t) {
        case OR_F32: return 4; case OR_F16: return 2; case OR_Q8_0: return 34;
        case OR_Q4_K: return 144; case OR_Q5_K: return 176; case OR_Q6_K: return 210;
        case OR_Q8_K: return 292; default: return 0;
    }
}
int or_block_size(int t) {
    switch (t) {
        case OR_F32: case OR_F16: return 1; case OR_Q8_0: return 32;
        case OR_Q4_K: case OR_Q5_K: case OR_Q6_K: case OR_Q8_K: return 256; default: return 0;
    }
}
/* upstream type_traits_cpu[...].vec_dot_type: K-quants -> Q8_K, Q8_0 -> Q8_0, F16 -> F16 */
int or_vec_dot_type(int t) {
    switch (t) {
        case OR_Q4_K: case OR_Q5_K: case OR_Q6_K: return OR_Q8_K;
        case OR_Q8_0: return OR_Q8_0; case OR_F16: return OR_F16; case OR_F32: return OR_F32;
        default: return -1;
    }
}

/* upstream get_scale_min_k4 (ggml-quants.c) — SURVEY.md Appendix A */
static inline void get_scale_min_k4(int j, const uint8_t* q, uint8_t* d, uint8_t* m) {
    if (j < 4) {
        *d = q[j] & 63; *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

/* ---------------- dequantize_row_*  ---------------- */
/* upstream dequantize_row_q4_K */
static void deq_q4_K(const block_q4_K* x, float* y, int64_t k) {
    for (int64_t i = 0; i < k / QK_K; i++) {
        const uint8_t* q = x[i].qs;
        const float d = llmi_h2f(x[i].d), min = llmi_h2f(x[i].dmin);
        int is = 0; uint8_t sc, m;
        for (int j = 0; j < QK_K; j += 64) {
            get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
            const float d1 = d * sc, m1 = min * m;
            get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
            const float d2 = d * sc, m2 = min * m;
            for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
            for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
            q += 32; is += 2;
        }
    }
}
/* upstream dequantize_row_q5_K */
static void deq_q5_K(const block_q5_K* x, float* y, int64_t k) {
    for (int64_t i = 0; i < k / QK_K; i++) {
        const uint8_t* ql = x[i].qs; const uint8_t* qh = x[i].qh;
        const float d = llmi_h2f(x[i].d), min = llmi_h2f(x[i].dmin);
        int is = 0; uint8_t sc, m; uint8_t u1 = 1, u2 = 2;
        for (int j = 0; j < QK_K; j += 64) {
            get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
            const float d1 = d * sc, m1 = min * m;
            get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
            const float d2 = d * sc, m2 = min * m;
            for (int l = 0; l < 32; ++l) *y++ = d1 * ((ql[l] & 0xF) + (qh[l] & u1 ? 16 : 0)) - m1;
            for (int l = 0; l < 32; ++l) *y++ = d2 * ((ql[l] >> 4) + (qh[l] & u2 ? 16 : 0)) - m2;
            ql += 32; is += 2; u1 <<= 2; u2 <<= 2;
        }
    }
}
/* upstream dequantize_row_q6_K */
static void deq_q6_K(const block_q6_K* x, float* y, int64_t k) {
    for (int64_t i = 0; i < k / QK_K; i++) {
        const float d = llmi_h2f(x[i].d);
        const uint8_t* ql = x[i].ql; const uint8_t* qh = x[i].qh; const int8_t* sc = x[i].scales;
        for (int n = 0; n < QK_K; n += 128) {
            for (int l = 0; l < 32; ++l) {
                int is = l / 16;
                const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                y[l + 0] = d * sc[is + 0] * q1;
                y[l + 32] = d * sc[is + 2] * q2;
                y[l + 64] = d * sc[is + 4] * q3;
                y[l + 96] = d * sc[is + 6] * q4;
            }
            y += 128; ql += 64; qh += 32; sc += 8;
        }
    }
}
/* upstream dequantize_row_q8_0 */
static void deq_q8_0(const block_q8_0* x, float* y, int64_t k) {
    for (int64_t i = 0; i < k / QK8_0; i++) {
        const float d = llmi_h2f(x[i].d);
        for (int j = 0; j < QK8_0; ++j) y[i * QK8_0 + j] = x[i].qs[j] * d;
    }
}

int or_dequantize_row(int type, const void* src, float* dst, int64_t n) {
    switch (type) {
        case OR_F32: memcpy(dst, src, (size_t)n * 4); return 0;
        case OR_F16: for (int64_t i = 0; i < n; ++i) dst[i] = llmi_h2f(((const uint16_t*)src)[i]); return 0;
        case OR_Q4_K: deq_q4_K(src, dst, n); return 0;
        case OR_Q5_K: deq_q5_K(src, dst, n); return 0;
        case OR_Q6_K: deq_q6_K(src, dst, n); return 0;
        case OR_Q8_0: deq_q8_0(src, dst, n); return 0;
        default: return -1;
    }
}

/* ---------------- activation quantization ---------------- */
/* upstream quantize_row_q8_K_ref: signed max-abs per 256, iscale=-127/max, bsums per 16 */
void or_quantize_row_q8_K(const float* x, void* vy, int64_t k) {
    block_q8_K* y = vy;
    for (int64_t i = 0; i < k / QK_K; i++) {
        float max = 0, amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            float ax = fabsf(x[j]);
            if (ax > amax) { amax = ax; max = x[j]; }
        }
        if (!amax) {
            y[i].d = 0;
            memset(y[i].qs, 0, QK_K);
            memset(y[i].bsums, 0, sizeof y[i].bsums);  /* upstream leaves bsums stale; zero is what they sum to */
            x += QK_K;
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < QK_K; ++j) {
            int v = llmi_nearest_int(iscale * x[j]);
            y[i].qs[j] = (int8_t)(v < 127 ? v : 127);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t)sum;
        }
        y[i].d = 1 / iscale;
        x += QK_K;
    }
}
/* upstream quantize_row_q8_0_ref: d = amax/127 (stored f16), q = roundf(x/d) */
void or_quantize_row_q8_0(const float* x, void* vy, int64_t k) {
    block_q8_0* y = vy;
    for (int64_t i = 0; i < k / QK8_0; i++) {
        float amax = 0.0f;
        for (int j = 0; j < QK8_0; j++) {
            const float v = x[i * QK8_0 + j];
            amax = fmaxf(amax, fabsf(v));
        }
        const float d = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        y[i].d = llmi_f2h(d);
        for (int j = 0; j < QK8_0; ++j) y[i].qs[j] = (int8_t)roundf(x[i * QK8_0 + j] * id);
    }
}

/* ---------------- vec_dot ---------------- */
/* upstream ggml_vec_dot_q4_K_q8_K_generic */
static float vd_q4_K(int n, const block_q4_K* x, const block_q8_K* y) {
    int8_t aux8[QK_K]; int16_t aux16[8]; float sums[8]; int32_t aux32[8];
    memset(sums, 0, sizeof sums);
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        const uint8_t* q4 = x[i].qs; const int8_t* q8 = y[i].qs;
        memset(aux32, 0, sizeof aux32);
        int8_t* a = aux8;
        for (int j = 0; j < QK_K / 64; ++j) {
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] & 0xF);
            a += 32;
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] >> 4);
            a += 32; q4 += 32;
        }
        uint8_t scales[8], mins[8];
        for (int j = 0; j < 8; ++j) get_scale_min_k4(j, x[i].scales, &scales[j], &mins[j]);
        int sumi = 0;
        for (int j = 0; j < QK_K / 16; ++j) sumi += y[i].bsums[j] * mins[j / 2];
        a = aux8;
        int is = 0;
        for (int j = 0; j < QK_K / 32; ++j) {
            int32_t scale = scales[is++];
            for (int r = 0; r < 4; ++r) {
                for (int l = 0; l < 8; ++l) aux16[l] = (int16_t)(q8[l] * a[l]);
                for (int l = 0; l < 8; ++l) aux32[l] += scale * aux16[l];
                q8 += 8; a += 8;
            }
        }
        const float d = llmi_h2f(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
        const float dmin = llmi_h2f(x[i].dmin) * y[i].d;
        sumf -= dmin * sumi;
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    return sumf;
}
/* upstream ggml_vec_dot_q5_K_q8_K_generic */
static float vd_q5_K(int n, const block_q5_K* x, const block_q8_K* y) {
    int8_t aux8[QK_K]; int16_t aux16[8]; float sums[8]; int32_t aux32[8];
    memset(sums, 0, sizeof sums);
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        const uint8_t* q4 = x[i].qs; const uint8_t* hm = x[i].qh; const int8_t* q8 = y[i].qs;
        memset(aux32, 0, sizeof aux32);
        int8_t* a = aux8;
        uint8_t m = 1;
        for (int j = 0; j < QK_K / 64; ++j) {
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] & 0xF);
            for (int l = 0; l < 32; ++l) a[l] += (hm[l] & m ? 16 : 0);
            a += 32; m <<= 1;
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] >> 4);
            for (int l = 0; l < 32; ++l) a[l] += (hm[l] & m ? 16 : 0);
            a += 32; m <<= 1;
            q4 += 32;
        }
        uint8_t scales[8], mins[8];
        for (int j = 0; j < 8; ++j) get_scale_min_k4(j, x[i].scales, &scales[j], &mins[j]);
        int sumi = 0;
        for (int j = 0; j < QK_K / 16; ++j) sumi += y[i].bsums[j] * mins[j / 2];
        a = aux8;
        int is = 0;
        for (int j = 0; j < QK_K / 32; ++j) {
            int32_t scale = scales[is++];
            for (int r = 0; r < 4; ++r) {
                for (int l = 0; l < 8; ++l) aux16[l] = (int16_t)(q8[l] * a[l]);
                for (int l = 0; l < 8; ++l) aux32[l] += scale * aux16[l];
                q8 += 8; a += 8;
            }
        }
        const float d = llmi_h2f(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
        const float dmin = llmi_h2f(x[i].dmin) * y[i].d;
        sumf -= dmin * sumi;
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    return sumf;
}
/* upstream ggml_vec_dot_q6_K_q8_K_generic */
static float vd_q6_K(int n, const block_q6_K* x, const block_q8_K* y) {
    int8_t aux8[QK_K]; int16_t aux16[8]; float sums[8]; int32_t aux32[8];
    memset(sums, 0, sizeof sums);
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        const uint8_t* q4 = x[i].ql; const uint8_t* qh = x[i].qh; const int8_t* q8 = y[i].qs;
        memset(aux32, 0, sizeof aux32);
        int8_t* a = aux8;
        for (int j = 0; j < QK_K; j += 128) {
            for (int l = 0; l < 32; ++l) {
                a[l + 0] = (int8_t)((q4[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                a[l + 32] = (int8_t)((q4[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                a[l + 64] = (int8_t)((q4[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                a[l + 96] = (int8_t)((q4[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
            }
            a += 128; q4 += 64; qh += 32;
        }
        a = aux8;
        int is = 0;
        for (int j = 0; j < QK_K / 16; ++j) {
            int scale = x[i].scales[is++];
            for (int r = 0; r < 2; ++r) {
                for (int l = 0; l < 8; ++l) aux16[l] = (int16_t)(q8[l] * a[l]);
                for (int l = 0; l < 8; ++l) aux32[l] += scale * aux16[l];
                q8 += 8; a += 8;
            }
        }
        const float d = llmi_h2f(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    return sumf;
}
/* upstream ggml_vec_dot_q8_0_q8_0 (generic tail loop) */
static float vd_q8_0(int n, const block_q8_0* x, const block_q8_0* y) {
    float sumf = 0;
    for (int ib = 0; ib < n / QK8_0; ++ib) {
        int sumi = 0;
        for (int j = 0; j < QK8_0; j++) sumi += x[ib].qs[j] * y[ib].qs[j];
        sumf += sumi * (llmi_h2f(x[ib].d) * llmi_h2f(y[ib].d));
    }
    return sumf;
}
/* upstream ggml_vec_dot_f16 (generic: double accumulation) */
static float vd_f16(int n, const uint16_t* x, const uint16_t* y) {
    double sumf = 0.0;
    for (int i = 0; i < n; ++i) sumf += (double)(llmi_h2f(x[i]) * llmi_h2f(y[i]));
    return (float)sumf;
}
/* upstream ggml_vec_dot_f32 (generic: double accumulation) */
static float vd_f32(int n, const float* x, const float* y) {
    double sumf = 0.0;
    for (int i = 0; i < n; ++i) sumf += (double)(x[i] * y[i]);
    return (float)sumf;
}

/* Unpack one K-quant block into its 256 unsigned quant values in natural element order
 * (Q4_K 0..15, Q5_K 0..31, Q6_K 0..63; the generic functions' unpack loops, without
 * Q6_K's -32), then the 16-element integer dots against the q8_K block: every chunk's
 * integer sums are made of these exactly (sums of products, any grouping). */
static void block_unpack_kq(int wtype, const uint8_t* blk, uint8_t* u) {
    if (wtype == OR_Q6_K) {
        const block_q6_K* x = (const block_q6_K*)blk;
        const uint8_t* ql = x->ql; const uint8_t* qh = x->qh;
        uint8_t* a = u;
        for (int j = 0; j < QK_K; j += 128) {
            for (int l = 0; l < 32; ++l) {
                a[l + 0] = (uint8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4));
                a[l + 32] = (uint8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4));
                a[l + 64] = (uint8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4));
                a[l + 96] = (uint8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4));
            }
            a += 128; ql += 64; qh += 32;
        }
    } else {
        const uint8_t* qs; const uint8_t* hm = NULL;
        if (wtype == OR_Q4_K) qs = ((const block_q4_K*)blk)->qs;
        else { qs = ((const block_q5_K*)blk)->qs; hm = ((const block_q5_K*)blk)->qh; }
        for (int j = 0; j < QK_K / 64; ++j) {
            for (int l = 0; l < 32; ++l) u[64 * j + l] = (uint8_t)(qs[32 * j + l] & 0xF);
            for (int l = 0; l < 32; ++l) u[64 * j + 32 + l] = (uint8_t)(qs[32 * j + l] >> 4);
            if (hm) {
                for (int l = 0; l < 32; ++l) u[64 * j + l] += (hm[l] >> (2 * j)) & 1 ? 16 : 0;
                for (int l = 0; l < 32; ++l) u[64 * j + 32 + l] += (hm[l] >> (2 * j + 1)) & 1 ? 16 : 0;
            }
        }
    }
}
/* The generic functions above for a K-quant row whose quant values are already
 * unpacked (u: the row's block_unpack_kq output) and whose per-block constants are
 * decoded once (RowConst: h2f(d), h2f(dmin), the 6-bit scales/mins or Q6_K's int8
 * scales): the same integer sums (exact in any grouping) and the same fp32 operations
 * in the same order, hoisted out of the token loop of or_prefill. */
typedef struct { float d, dmin; int sc[16], mn[8]; } RowConst;

static void row_consts(int wtype, const uint8_t* blk, RowConst* rc) {
    if (wtype == OR_Q6_K) {
        const block_q6_K* x = (const block_q6_K*)blk;
        rc->d = llmi_h2f(x->d); rc->dmin = 0.f;
        for (int j = 0; j < 16; ++j) rc->sc[j] = x->scales[j];
        return;
    }
    const uint8_t* scales; uint16_t d16, m16;
    if (wtype == OR_Q4_K) { const block_q4_K* x = (const block_q4_K*)blk; scales = x->scales; d16 = x->d; m16 = x->dmin; }
    else { const block_q5_K* x = (const block_q5_K*)blk; scales = x->scales; d16 = x->d; m16 = x->dmin; }
    rc->d = llmi_h2f(d16); rc->dmin = llmi_h2f(m16);
    for (int j = 0; j < 8; ++j) { uint8_t a, b; get_scale_min_k4(j, scales, &a, &b); rc->sc[j] = a; rc->mn[j] = b; }
}

static float vd_generic_unpacked(int wtype, int n, const RowConst* rcs, const uint8_t* u, const void* act) {
    float sums[8]; float sumf = 0;
    for (int l = 0; l < 8; ++l) sums[l] = 0;
    for (int ib = 0; ib < n / QK_K; ++ib) {
        const block_q8_K* y = (const block_q8_K*)act + ib;
        const RowConst* rc = rcs + ib;
        const uint8_t* ub = u + (size_t)ib * QK_K;
        int32_t aux32[8];
        for (int l = 0; l < 8; ++l) aux32[l] = 0;
        if (wtype == OR_Q6_K) {
            for (int j = 0; j < 16; ++j)
                for (int e = 0; e < 16; ++e) aux32[e & 7] += rc->sc[j] * (((int)ub[16 * j + e] - 32) * y->qs[16 * j + e]);
        } else {
            for (int j = 0; j < 8; ++j)
                for (int e = 0; e < 32; ++e) aux32[e & 7] += rc->sc[j] * ((int)ub[32 * j + e] * y->qs[32 * j + e]);
        }
        const float d = rc->d * y->d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
        if (wtype != OR_Q6_K) {
            int sumi = 0;
            for (int j = 0; j < QK_K / 16; ++j) sumi += y->bsums[j] * rc->mn[j / 2];
            const float dmin = rc->dmin * y->d;
            sumf -= dmin * sumi;
        }
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    return sumf;
}

/* ---------------- CPU baseline only: AVX2 dot products ----------------
 * TIMING PATH, NOT THE CHECKER.  The reference's CPU image builds llama.cpp for the host
 * (Dockerfile.cpu:84-89), whose x86 kernels (ggml-cpu arch/x86 quants.c, upstream, not
 * vendored) vectorise these dots with AVX2 maddubs/madd and accumulate the per-block
 * integer sums in 8 fp32 lanes — a different fp32 association from the generic order the
 * parity checks use.  These are written here in that style (unsigned-weights x signed-q8
 * maddubs, 16-bit scale madd, one fp32 FMA per block, Q4_K's 4-lane min accumulator) so
 * bench.py's cpu_baseline times a vectorised CPU path instead of the scalar restatement;
 * they compute exactly the x86 association mode's dots below (bit-identical,
 * tests/test_parity_x86.py).  Results agree with the generic order to float rounding
 * (tests/test_oracle_fast.py), never bit for bit; or_set_fast_dots is off by default and
 * no parity test turns it on. */
static int g_fast = 0;
#if defined(__AVX2__) && defined(__FMA__)
#include <immintrin.h>
static inline float fh2f(uint16_t h) { return _cvtsh_ss(h); }  /* exact, = llmi_h2f */
static inline float hsum8(__m256 v) {
    __m128 a = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
    a = _mm_add_ps(a, _mm_movehl_ps(a, a));
    a = _mm_add_ss(a, _mm_movehdup_ps(a));
    return _mm_cvtss_f32(a);
}
/* the 8 scales and 8 mins of a Q4_K/Q5_K block at once: upstream's utmp/kmask unpack
 * (the same values as get_scale_min_k4 j = 0..7, without its per-j branches) */
static inline void scales_mins_k4(const uint8_t* q, uint8_t* sc, uint8_t* mn) {
    uint32_t u[4];
    memcpy(u, q, 12);
    const uint32_t k1 = 0x3f3f3f3fu, k2 = 0x0f0f0f0fu, k3 = 0x03030303u;
    u[3] = ((u[2] >> 4) & k2) | (((u[1] >> 6) & k3) << 4);
    const uint32_t m01 = u[1] & k1;
    u[1] = (u[2] & k2) | (((u[0] >> 6) & k3) << 4);
    u[2] = m01;
    u[0] &= k1;
    memcpy(sc, u, 8);
    memcpy(mn, u + 2, 8);
}
static inline int kq_mins_dot(const int16_t* bsums, const uint8_t* mn) {
    int s = 0;
    for (int j = 0; j < 16; ++j) s += bsums[j] * mn[j / 2];
    return s;
}
static float fd_q4_K(int n, const block_q4_K* x, const block_q8_K* y) {
    const __m256i m4 = _mm256_set1_epi8(0x0F);
    __m256 acc = _mm256_setzero_ps();
    __m128 accm4 = _mm_setzero_ps();
    for (int i = 0; i < n / QK_K; ++i) {
        uint8_t sc[8], mn[8];
        scales_mins_k4(x[i].scales, sc, mn);
        __m256i sumi = _mm256_setzero_si256();
        for (int j = 0; j < 4; ++j) {
            const __m256i qb = _mm256_loadu_si256((const __m256i*)(x[i].qs + 32 * j));
            const __m256i lo = _mm256_and_si256(qb, m4), hi = _mm256_and_si256(_mm256_srli_epi16(qb, 4), m4);
            const __m256i yl = _mm256_loadu_si256((const __m256i*)(y[i].qs + 64 * j));
            const __m256i yh = _mm256_loadu_si256((const __m256i*)(y[i].qs + 64 * j + 32));
            const __m256i pl = _mm256_madd_epi16(_mm256_maddubs_epi16(lo, yl), _mm256_set1_epi16(sc[2 * j]));
            const __m256i ph = _mm256_madd_epi16(_mm256_maddubs_epi16(hi, yh), _mm256_set1_epi16(sc[2 * j + 1]));
            sumi = _mm256_add_epi32(sumi, _mm256_add_epi32(pl, ph));
        }
        acc = _mm256_fmadd_ps(_mm256_set1_ps(y[i].d * fh2f(x[i].d)), _mm256_cvtepi32_ps(sumi), acc);
        /* upstream's min terms: 4 lanes prod[k] = madd(mins, hadd(bsums)), FMA-accumulated */
        const __m256i q8sums = _mm256_loadu_si256((const __m256i*)y[i].bsums);
        const __m128i q8s = _mm_hadd_epi16(_mm256_castsi256_si128(q8sums), _mm256_extracti128_si256(q8sums, 1));
        const __m128i mins = _mm_cvtepu8_epi16(_mm_loadl_epi64((const __m128i*)mn));
        const __m128i prod = _mm_madd_epi16(mins, q8s);
        accm4 = _mm_fmadd_ps(_mm_set1_ps(-y[i].d * fh2f(x[i].dmin)), _mm_cvtepi32_ps(prod), accm4);
    }
    accm4 = _mm_add_ps(accm4, _mm_movehl_ps(accm4, accm4));
    accm4 = _mm_add_ss(accm4, _mm_movehdup_ps(accm4));
    return hsum8(acc) + _mm_cvtss_f32(accm4);
}
static float fd_q5_K(int n, const block_q5_K* x, const block_q8_K* y) {
    const __m256i m4 = _mm256_set1_epi8(0x0F), b16 = _mm256_set1_epi8(0x10);
    __m256 acc = _mm256_setzero_ps();
    float summs = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        uint8_t sc[8], mn[8];
        scales_mins_k4(x[i].scales, sc, mn);
        const __m256i hb = _mm256_loadu_si256((const __m256i*)x[i].qh);
        __m256i sumi = _mm256_setzero_si256();
        for (int j = 0; j < 4; ++j) {
            const __m256i qb = _mm256_loadu_si256((const __m256i*)(x[i].qs + 32 * j));
            const __m256i ml = _mm256_set1_epi8((char)(1 << (2 * j))), mh = _mm256_set1_epi8((char)(1 << (2 * j + 1)));
            const __m256i lo = _mm256_or_si256(_mm256_and_si256(qb, m4),
                                               _mm256_and_si256(_mm256_cmpeq_epi8(_mm256_and_si256(hb, ml), ml), b16));
            const __m256i hi = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(qb, 4), m4),
                                               _mm256_and_si256(_mm256_cmpeq_epi8(_mm256_and_si256(hb, mh), mh), b16));
            const __m256i yl = _mm256_loadu_si256((const __m256i*)(y[i].qs + 64 * j));
            const __m256i yh = _mm256_loadu_si256((const __m256i*)(y[i].qs + 64 * j + 32));
            const __m256i pl = _mm256_madd_epi16(_mm256_maddubs_epi16(lo, yl), _mm256_set1_epi16(sc[2 * j]));
            const __m256i ph = _mm256_madd_epi16(_mm256_maddubs_epi16(hi, yh), _mm256_set1_epi16(sc[2 * j + 1]));
            sumi = _mm256_add_epi32(sumi, _mm256_add_epi32(pl, ph));
        }
        acc = _mm256_fmadd_ps(_mm256_set1_ps(y[i].d * fh2f(x[i].d)), _mm256_cvtepi32_ps(sumi), acc);
        /* upstream: one scalar summs += dmin * sum(prod), FMA-contracted (gnu11 build) */
        summs = fmaf(-y[i].d * fh2f(x[i].dmin), (float)kq_mins_dot(y[i].bsums, mn), summs);
    }
    return hsum8(acc) + summs;
}
static float fd_q6_K(int n, const block_q6_K* x, const block_q8_K* y) {
    const __m256i m4 = _mm256_set1_epi8(0x0F), m2 = _mm256_set1_epi8(0x30), k32 = _mm256_set1_epi8(32);
    __m256 acc = _mm256_setzero_ps();
    for (int i = 0; i < n / QK_K; ++i) {
        __m256i sumi = _mm256_setzero_si256();
        for (int h = 0; h < 2; ++h) {
            const __m256i l0 = _mm256_loadu_si256((const __m256i*)(x[i].ql + 64 * h));
            const __m256i l1 = _mm256_loadu_si256((const __m256i*)(x[i].ql + 64 * h + 32));
            const __m256i qh = _mm256_loadu_si256((const __m256i*)(x[i].qh + 32 * h));
            __m256i q[4];  /* elements 128h + 32k + l, unsigned 6-bit */
            q[0] = _mm256_or_si256(_mm256_and_si256(l0, m4), _mm256_and_si256(_mm256_slli_epi16(qh, 4), m2));
            q[1] = _mm256_or_si256(_mm256_and_si256(l1, m4), _mm256_and_si256(_mm256_slli_epi16(qh, 2), m2));
            q[2] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l0, 4), m4), _mm256_and_si256(qh, m2));
            q[3] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l1, 4), m4), _mm256_and_si256(_mm256_srli_epi16(qh, 2), m2));
            for (int k = 0; k < 4; ++k) {
                const int e0 = 128 * h + 32 * k;
                const __m256i yv = _mm256_loadu_si256((const __m256i*)(y[i].qs + e0));
                /* (q - 32) * y = q * y - 32 * y: both maddubs in range */
                const __m256i p = _mm256_sub_epi16(_mm256_maddubs_epi16(q[k], yv), _mm256_maddubs_epi16(k32, yv));
                const __m256i s = _mm256_set_m128i(_mm_set1_epi16(x[i].scales[e0 / 16 + 1]), _mm_set1_epi16(x[i].scales[e0 / 16]));
                sumi = _mm256_add_epi32(sumi, _mm256_madd_epi16(p, s));
            }
        }
        acc = _mm256_fmadd_ps(_mm256_set1_ps(y[i].d * fh2f(x[i].d)), _mm256_cvtepi32_ps(sumi), acc);
    }
    return hsum8(acc);
}
static float fd_q8_0(int n, const block_q8_0* x, const block_q8_0* y) {
    __m256 acc = _mm256_setzero_ps();
    const __m256i ones = _mm256_set1_epi16(1);
    for (int ib = 0; ib < n / QK8_0; ++ib) {
        const __m256i a = _mm256_loadu_si256((const __m256i*)x[ib].qs), b = _mm256_loadu_si256((const __m256i*)y[ib].qs);
        const __m256i p = _mm256_madd_epi16(_mm256_maddubs_epi16(_mm256_sign_epi8(a, a), _mm256_sign_epi8(b, a)), ones);
        acc = _mm256_fmadd_ps(_mm256_set1_ps(fh2f(x[ib].d) * fh2f(y[ib].d)), _mm256_cvtepi32_ps(p), acc);
    }
    return hsum8(acc);
}
/* AVX-512BW forms (g_fast == 2; Zen 4/5 and recent Xeon hosts, where a GGML_CPU_ALL_VARIANTS
 * image also loads its AVX-512 variant): the AVX2 kernels above at twice the width, two
 * 32-byte groups per instruction, 16 fp32 lanes per block accumulator -- the same integer
 * sums, a 16-lane fp32 association (timing only, like every fast dot; test_oracle_fast.py).
 * Compiled by target attribute in the x86-64-v3 build and chosen at run time. */
#define OR_AVX512 __attribute__((target("avx512f,avx512bw,avx512vl,avx512dq")))
OR_AVX512 static inline __m512i ld2x256(const void* a, const void* b) {
    return _mm512_inserti64x4(_mm512_castsi256_si512(_mm256_loadu_si256((const __m256i*)a)),
                              _mm256_loadu_si256((const __m256i*)b), 1);
}
OR_AVX512 static inline __m512i set2x16(int a, int b) {  /* int16 a in the low 256 bits, b in the high */
    return _mm512_inserti64x4(_mm512_castsi256_si512(_mm256_set1_epi16((short)a)), _mm256_set1_epi16((short)b), 1);
}
OR_AVX512 static float fd512_q4_K(int n, const block_q4_K* x, const block_q8_K* y) {
    const __m512i m4 = _mm512_set1_epi8(0x0F);
    __m512 acc = _mm512_setzero_ps();
    __m128 accm4 = _mm_setzero_ps();
    for (int i = 0; i < n / QK_K; ++i) {
        uint8_t sc[8], mn[8];
        scales_mins_k4(x[i].scales, sc, mn);
        __m512i sumi = _mm512_setzero_si512();
        for (int jj = 0; jj < 2; ++jj) {  /* 32-byte groups j = 2 jj, 2 jj + 1 */
            const __m512i qb = _mm512_loadu_si512((const void*)(x[i].qs + 64 * jj));
            const __m512i lo = _mm512_and_si512(qb, m4), hi = _mm512_and_si512(_mm512_srli_epi16(qb, 4), m4);
            const int8_t* q8 = y[i].qs + 128 * jj;
            const __m512i yl = ld2x256(q8, q8 + 64), yh = ld2x256(q8 + 32, q8 + 96);
            const __m512i pl = _mm512_madd_epi16(_mm512_maddubs_epi16(lo, yl), set2x16(sc[4 * jj], sc[4 * jj + 2]));
            const __m512i ph = _mm512_madd_epi16(_mm512_maddubs_epi16(hi, yh), set2x16(sc[4 * jj + 1], sc[4 * jj + 3]));
            sumi = _mm512_add_epi32(sumi, _mm512_add_epi32(pl, ph));
        }
        acc = _mm512_fmadd_ps(_mm512_set1_ps(y[i].d * fh2f(x[i].d)), _mm512_cvtepi32_ps(sumi), acc);
        const __m256i q8sums = _mm256_loadu_si256((const __m256i*)y[i].bsums);
        const __m128i q8s = _mm_hadd_epi16(_mm256_castsi256_si128(q8sums), _mm256_extracti128_si256(q8sums, 1));
        const __m128i mins = _mm_cvtepu8_epi16(_mm_loadl_epi64((const __m128i*)mn));
        accm4 = _mm_fmadd_ps(_mm_set1_ps(-y[i].d * fh2f(x[i].dmin)), _mm_cvtepi32_ps(_mm_madd_epi16(mins, q8s)), accm4);
    }
    accm4 = _mm_add_ps(accm4, _mm_movehl_ps(accm4, accm4));
    accm4 = _mm_add_ss(accm4, _mm_movehdup_ps(accm4));
    return _mm512_reduce_add_ps(acc) + _mm_cvtss_f32(accm4);
}
OR_AVX512 static float fd512_q5_K(int n, const block_q5_K* x, const block_q8_K* y) {
    const __m512i m4 = _mm512_set1_epi8(0x0F), b16 = _mm512_set1_epi8(0x10);
    __m512 acc = _mm512_setzero_ps();
    float summs = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        uint8_t sc[8], mn[8];
        scales_mins_k4(x[i].scales, sc, mn);
        const __m512i hb = _mm512_broadcast_i64x4(_mm256_loadu_si256((const __m256i*)x[i].qh));
        __m512i sumi = _mm512_setzero_si512();
        for (int jj = 0; jj < 2; ++jj) {
            const __m512i qb = _mm512_loadu_si512((const void*)(x[i].qs + 64 * jj));
            const __m512i ml = _mm512_inserti64x4(_mm512_set1_epi8((char)(1 << (4 * jj))), _mm256_set1_epi8((char)(1 << (4 * jj + 2))), 1);
            const __m512i mh = _mm512_inserti64x4(_mm512_set1_epi8((char)(1 << (4 * jj + 1))), _mm256_set1_epi8((char)(1 << (4 * jj + 3))), 1);
            const __m512i lo = _mm512_or_si512(_mm512_and_si512(qb, m4),
                                               _mm512_maskz_mov_epi8(_mm512_test_epi8_mask(hb, ml), b16));
            const __m512i hi = _mm512_or_si512(_mm512_and_si512(_mm512_srli_epi16(qb, 4), m4),
                                               _mm512_maskz_mov_epi8(_mm512_test_epi8_mask(hb, mh), b16));
            const int8_t* q8 = y[i].qs + 128 * jj;
            const __m512i yl = ld2x256(q8, q8 + 64), yh = ld2x256(q8 + 32, q8 + 96);
            const __m512i pl = _mm512_madd_epi16(_mm512_maddubs_epi16(lo, yl), set2x16(sc[4 * jj], sc[4 * jj + 2]));
            const __m512i ph = _mm512_madd_epi16(_mm512_maddubs_epi16(hi, yh), set2x16(sc[4 * jj + 1], sc[4 * jj + 3]));
            sumi = _mm512_add_epi32(sumi, _mm512_add_epi32(pl, ph));
        }
        acc = _mm512_fmadd_ps(_mm512_set1_ps(y[i].d * fh2f(x[i].d)), _mm512_cvtepi32_ps(sumi), acc);
        summs = fmaf(-y[i].d * fh2f(x[i].dmin), (float)kq_mins_dot(y[i].bsums, mn), summs);
    }
    return _mm512_reduce_add_ps(acc) + summs;
}
OR_AVX512 static float fd512_q6_K(int n, const block_q6_K* x, const block_q8_K* y) {
    const __m512i m4 = _mm512_set1_epi8(0x0F), m2 = _mm512_set1_epi8(0x30), k32 = _mm512_set1_epi8(32);
    /* int16 index vectors: scale s of 16 elements -> 8 int16 lanes each */
    const __m512i i01 = _mm512_set_epi16(3, 3, 3, 3, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0);
    const __m512i i23 = _mm512_add_epi16(i01, _mm512_set1_epi16(4));
    __m512 acc = _mm512_setzero_ps();
    for (int i = 0; i < n / QK_K; ++i) {
        __m512i sumi = _mm512_setzero_si512();
        for (int h = 0; h < 2; ++h) {
            const __m256i l0 = _mm256_loadu_si256((const __m256i*)(x[i].ql + 64 * h));
            const __m256i l1 = _mm256_loadu_si256((const __m256i*)(x[i].ql + 64 * h + 32));
            const __m256i qh = _mm256_loadu_si256((const __m256i*)(x[i].qh + 32 * h));
            /* (q0 | q1), (q2 | q3): elements 128h + 0..63 and 64..127 */
            const __m512i L01 = _mm512_inserti64x4(_mm512_castsi256_si512(l0), l1, 1);
            const __m512i H = _mm512_broadcast_i64x4(qh);
            const __m512i Hlo = _mm512_inserti64x4(_mm512_castsi256_si512(_mm256_slli_epi16(qh, 4)), _mm256_slli_epi16(qh, 2), 1);
            const __m512i Hhi = _mm512_inserti64x4(_mm512_castsi256_si512(qh), _mm256_srli_epi16(qh, 2), 1);
            (void)H;
            const __m512i q01 = _mm512_or_si512(_mm512_and_si512(L01, m4), _mm512_and_si512(Hlo, m2));
            const __m512i q23 = _mm512_or_si512(_mm512_and_si512(_mm512_srli_epi16(L01, 4), m4), _mm512_and_si512(Hhi, m2));
            const __m512i y01 = _mm512_loadu_si512((const void*)(y[i].qs + 128 * h));
            const __m512i y23 = _mm512_loadu_si512((const void*)(y[i].qs + 128 * h + 64));
            const __m512i p01 = _mm512_sub_epi16(_mm512_maddubs_epi16(q01, y01), _mm512_maddubs_epi16(k32, y01));
            const __m512i p23 = _mm512_sub_epi16(_mm512_maddubs_epi16(q23, y23), _mm512_maddubs_epi16(k32, y23));
            const __m512i s8 = _mm512_broadcast_i32x4(_mm_cvtepi8_epi16(_mm_loadl_epi64((const __m128i*)(x[i].scales + 8 * h))));
            sumi = _mm512_add_epi32(sumi, _mm512_madd_epi16(p01, _mm512_permutexvar_epi16(i01, s8)));
            sumi = _mm512_add_epi32(sumi, _mm512_madd_epi16(p23, _mm512_permutexvar_epi16(i23, s8)));
        }
        acc = _mm512_fmadd_ps(_mm512_set1_ps(y[i].d * fh2f(x[i].d)), _mm512_cvtepi32_ps(sumi), acc);
    }
    return _mm512_reduce_add_ps(acc);
}
OR_AVX512 static float fd512_q8_0(int n, const block_q8_0* x, const block_q8_0* y) {
    __m512 acc = _mm512_setzero_ps();
    const __m512i ones = _mm512_set1_epi16(1);
    int ib = 0;
    for (; ib + 1 < n / QK8_0; ib += 2) {
        const __m512i a = ld2x256(x[ib].qs, x[ib + 1].qs), b = ld2x256(y[ib].qs, y[ib + 1].qs);
        const __m512i ua = _mm512_abs_epi8(a);
        const __m512i sb = _mm512_mask_sub_epi8(b, _mm512_movepi8_mask(a), _mm512_setzero_si512(), b);  /* sign(b, a) */
        const __m512i p = _mm512_madd_epi16(_mm512_maddubs_epi16(ua, sb), ones);
        const __m512 d = _mm512_insertf32x8(_mm512_set1_ps(fh2f(x[ib].d) * fh2f(y[ib].d)),
                                            _mm256_set1_ps(fh2f(x[ib + 1].d) * fh2f(y[ib + 1].d)), 1);
        acc = _mm512_fmadd_ps(d, _mm512_cvtepi32_ps(p), acc);
    }
    float r = _mm512_reduce_add_ps(acc);
    if (ib < n / QK8_0) r += fd_q8_0(QK8_0, x + ib, y + ib);
    return r;
}
/* 1 = AVX2 dots, 2 = AVX-512BW dots (falls back to 1 on hosts without it) */
int or_set_fast_dots(int on) {
    if (on >= 2 && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512f") &&
        __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq")) {
        g_fast = 2;
        return 2;
    }
    g_fast = on ? 1 : 0;
    return on ? 1 : 0;
}
#else
int or_set_fast_dots(int on) { g_fast = 0; (void)on; return 0; }  /* no AVX2 in this build */
#endif

/* ---------------- x86 association mode (parity measurement) ----------------
 * MEASUREMENT PATH, NOT THE CHECKER.  The GPU is bit-identical to the generic order above.
 * The reference's CPU path (Dockerfile.cpu:11 `llama.cpp:server`, NGL=0 at :84-89) runs
 * llama.cpp's x86 build instead, whose kernels associate the same operations differently
 * [upstream ggml-cpu arch/x86/quants.c, vec.h/vec.cpp, simd-mappings.h, ops.cpp; recalled,
 * not vendored; modelled on the AVX2+FMA ("haswell") variant].  or_set_x86_mode() switches
 * the oracle onto that association, so that generic-vs-x86 over a trajectory measures the
 * GPU's distance from the NGL=0 numerics (tools/parity_x86.py, profiles/r04/parity_x86.jsonl).
 * Lanes are emulated in scalar C with fmaf() where upstream uses _mm256_fmadd_ps:
 *   OR_X86_DOTS   ggml_vec_dot_q{4,5,6}_K_q8_K / q8_0_q8_0 AVX2: per 256-block the integer
 *                 sums in 8 int32 lanes (lane k = bytes 4k..4k+3 of every 32-byte vector,
 *                 maddubs + madd), acc[k] = fma(d, (float)sumi[k], acc[k]) with
 *                 d = y.d * fp16(x.d); Q4_K's min terms in 4 lanes acc_m[k] = fma(dmin,
 *                 (float)prod[k], acc_m[k]) with dmin = -y.d * fp16(x.dmin), prod[k] =
 *                 m[2k](bs[4k]+bs[4k+1]) + m[2k+1](bs[4k+2]+bs[4k+3]) (hadd + madd),
 *                 reduced (a0+a2)+(a1+a3); Q5_K's one scalar summs += dmin*(float)sum(prod)
 *                 (FMA-contracted, gnu11 default); result hsum_float_8(acc) [+ mins]
 *   OR_X86_Q80    quantize_row_q8_0 AVX2: id = 127/amax, q = round-half-even(x*id)
 *   OR_X86_F16DOT ggml_vec_dot_f16 AVX2+F16C (KQ over head dims, PV over positions):
 *                 4 x 8 fp32 FMA accumulators (element i -> acc[(i%32)/8][i%8]), reduced
 *                 acc0+acc2, acc1+acc3, then those two, then lo4+hi4 and two hadds
 *   OR_X86_VEXP   ggml_v_expf / ggml_v_silu (AVX2 polynomial exp) in soft_max and SwiGLU,
 *                 and ggml_vec_soft_max_f32's sum: per 8 positions an fp32 hsum, added in double
 *   OR_X86_LIBM   libm expf in soft_max and SiLU (scalar sums) instead of llmi_expf
 *   OR_X86_NOFMA  Q5_K's scalar min term without FMA contraction (-ffp-contract=off build)
 *   OR_X86_FA     flash attention instead of the non-flash path (attn_head_fa below) */
enum { OR_X86_DOTS = 1, OR_X86_Q80 = 2, OR_X86_F16DOT = 4, OR_X86_VEXP = 8, OR_X86_LIBM = 16, OR_X86_NOFMA = 32,
       OR_X86_FA = 64 };
static int g_x86 = 0;
int or_set_x86_mode(int flags) { g_x86 = flags; return g_x86; }
int or_get_x86_mode(void) { return g_x86; }

/* hsum_float_8: (lo4 + hi4), then movehl + add, then movehdup + add_ss */
static inline float x86_hsum8(const float* a) {
    const float t0 = a[4] + a[0], t1 = a[5] + a[1], t2 = a[6] + a[2], t3 = a[7] + a[3];
    return (t0 + t2) + (t1 + t3);
}
static float x86_q4_K(int n, const block_q4_K* x, const block_q8_K* y) {
    float acc[8] = {0}, accm[4] = {0};
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = y[i].d * llmi_h2f(x[i].d);
        const float dmin = -y[i].d * llmi_h2f(x[i].dmin);
        uint8_t sc[8], mn[8];
        for (int j = 0; j < 8; ++j) get_scale_min_k4(j, x[i].scales, &sc[j], &mn[j]);
        int32_t sumi[8] = {0};
        for (int j = 0; j < 4; ++j)
            for (int b = 0; b < 32; ++b) {
                const int q = x[i].qs[32 * j + b];
                sumi[b >> 2] += sc[2 * j] * ((q & 0xF) * y[i].qs[64 * j + b]) + sc[2 * j + 1] * ((q >> 4) * y[i].qs[64 * j + 32 + b]);
            }
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(d, (float)sumi[k], acc[k]);
        const int16_t* bs = y[i].bsums;
        for (int k = 0; k < 4; ++k) {
            const int prod = mn[2 * k] * (bs[4 * k] + bs[4 * k + 1]) + mn[2 * k + 1] * (bs[4 * k + 2] + bs[4 * k + 3]);
            accm[k] = fmaf(dmin, (float)prod, accm[k]);
        }
    }
    const float m = (accm[0] + accm[2]) + (accm[1] + accm[3]);
    return x86_hsum8(acc) + m;
}
static float x86_q5_K(int n, const block_q5_K* x, const block_q8_K* y) {
    float acc[8] = {0}, summs = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = y[i].d * llmi_h2f(x[i].d);
        const float dmin = -y[i].d * llmi_h2f(x[i].dmin);
        uint8_t sc[8], mn[8];
        for (int j = 0; j < 8; ++j) get_scale_min_k4(j, x[i].scales, &sc[j], &mn[j]);
        int32_t sumi[8] = {0};
        for (int j = 0; j < 4; ++j)
            for (int b = 0; b < 32; ++b) {
                const int q = x[i].qs[32 * j + b], h = x[i].qh[b];
                const int lo = (q & 0xF) + (((h >> (2 * j)) & 1) << 4), hi = (q >> 4) + (((h >> (2 * j + 1)) & 1) << 4);
                sumi[b >> 2] += sc[2 * j] * (lo * y[i].qs[64 * j + b]) + sc[2 * j + 1] * (hi * y[i].qs[64 * j + 32 + b]);
            }
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(d, (float)sumi[k], acc[k]);
        int sm = 0;
        for (int j = 0; j < 16; ++j) sm += mn[j / 2] * y[i].bsums[j];
        summs = (g_x86 & OR_X86_NOFMA) ? summs + dmin * (float)sm : fmaf(dmin, (float)sm, summs);
    }
    return x86_hsum8(acc) + summs;
}
static float x86_q6_K(int n, const block_q6_K* x, const block_q8_K* y) {
    float acc[8] = {0};
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = y[i].d * llmi_h2f(x[i].d);
        int32_t sumi[8] = {0};
        for (int h = 0; h < 2; ++h)
            for (int v = 0; v < 4; ++v)
                for (int b = 0; b < 32; ++b) {
                    const int e = 128 * h + 32 * v + b;
                    const uint8_t lq = x[i].ql[64 * h + 32 * (v & 1) + b], hq = x[i].qh[32 * h + b];
                    const int q = ((v < 2 ? lq & 0xF : lq >> 4) | (((hq >> (2 * v)) & 3) << 4)) - 32;
                    sumi[b >> 2] += x[i].scales[e / 16] * (q * y[i].qs[e]);
                }
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(d, (float)sumi[k], acc[k]);
    }
    return x86_hsum8(acc);
}
static float x86_q8_0(int n, const block_q8_0* x, const block_q8_0* y) {
    float acc[8] = {0};
    for (int ib = 0; ib < n / QK8_0; ++ib) {
        const float d = llmi_h2f(x[ib].d) * llmi_h2f(y[ib].d);
        int32_t sumi[8] = {0};
        for (int b = 0; b < 32; ++b) sumi[b >> 2] += x[ib].qs[b] * y[ib].qs[b];
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(d, (float)sumi[k], acc[k]);
    }
    return x86_hsum8(acc);
}
/* quantize_row_q8_0 (x86 AVX2 path) */
static void x86_quantize_row_q8_0(const float* x, void* vy, int64_t k) {
    block_q8_0* y = vy;
    for (int64_t i = 0; i < k / QK8_0; i++) {
        float amax = 0.0f;
        for (int j = 0; j < QK8_0; j++) amax = fmaxf(amax, fabsf(x[i * QK8_0 + j]));
        const float d = amax / 127.f;
        y[i].d = llmi_f2h(d);
        const float id = amax != 0.0f ? 127.f / amax : 0.0f;
        for (int j = 0; j < QK8_0; ++j) y[i].qs[j] = (int8_t)(int)rintf(x[i * QK8_0 + j] * id);
    }
}
/* ggml_vec_dot_f16 (AVX2 + F16C): n a multiple of 32 (head dims; padded KV rows) */
static float x86_dot_f16f(int n, const float* a, const float* b) {
    float acc[4][8];
    memset(acc, 0, sizeof acc);
    const int np = n & ~31;
    for (int i = 0; i < np; ++i) acc[(i & 31) >> 3][i & 7] = fmaf(a[i], b[i], acc[(i & 31) >> 3][i & 7]);
    for (int l = 0; l < 8; ++l) { acc[0][l] = acc[0][l] + acc[2][l]; acc[1][l] = acc[1][l] + acc[3][l]; }
    for (int l = 0; l < 8; ++l) acc[0][l] = acc[0][l] + acc[1][l];
    const float t0 = acc[0][0] + acc[0][4], t1 = acc[0][1] + acc[0][5], t2 = acc[0][2] + acc[0][6], t3 = acc[0][3] + acc[0][7];
    double sumf = (double)((t0 + t1) + (t2 + t3));  /* _mm_hadd_ps twice: lane 0 */
    for (int i = np; i < n; ++i) sumf += (double)(a[i] * b[i]);
    return (float)sumf;
}
/* ggml_v_expf (AVX2 form; the ARM optimized-routines expf polynomial) */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static float x86_v_expf(float x) {
    const float r = 0x1.8p23f;
    const float z = fmaf(x, 0x1.715476p+0f, r);
    const float n = z - r;
    const float b = fmaf(-n, 0x1.7f7d1cp-20f, fmaf(-n, 0x1.62e4p-1f, x));
    const uint32_t e = f2u(z) << 23;
    const float k = u2f(e + f2u(1.0f));
    const float u = b * b;
    const float j = fmaf(fmaf(fmaf(0x1.0e4020p-7f, b, 0x1.573e2ep-5f), u, fmaf(0x1.555e66p-3f, b, 0x1.fffdb6p-2f)), u,
                         0x1.ffffecp-1f * b);
    if (!(fabsf(n) > 126.f)) return fmaf(j, k, k);
    const uint32_t g = n <= 0.f ? 0x82000000u : 0u;
    const float s1 = u2f(g + 0x7f000000u), s2 = u2f(e - g);
    if (fabsf(n) > 192.f) return s1 * s1;
    return fmaf(s2, j, s2) * s1;
}
/* SiLU and exp under the mode's exp (ggml_v_silu: x / (1 + v_expf(-x))) */
static inline float mode_expf(float x) {
    if (g_x86 & OR_X86_VEXP) return x86_v_expf(x);
    if (g_x86 & OR_X86_LIBM) return expf(x);
    return llmi_expf(x);
}
static inline float mode_silu(float x) { return x / (1.0f + mode_expf(-x)); }

float or_vec_dot(int wtype, int n, const void* w, const void* a) {
    if (g_x86 & OR_X86_DOTS) {
        switch (wtype) {
            case OR_Q4_K: return x86_q4_K(n, w, a);
            case OR_Q5_K: return x86_q5_K(n, w, a);
            case OR_Q6_K: return x86_q6_K(n, w, a);
            case OR_Q8_0: return x86_q8_0(n, w, a);
            default: break;
        }
    }
#if defined(__AVX2__) && defined(__FMA__)
    if (g_fast == 2) {
        switch (wtype) {
            case OR_Q4_K: return fd512_q4_K(n, w, a);
            case OR_Q5_K: return fd512_q5_K(n, w, a);
            case OR_Q6_K: return fd512_q6_K(n, w, a);
            case OR_Q8_0: return fd512_q8_0(n, w, a);
            default: break;
        }
    }
    if (g_fast) {
        switch (wtype) {
            case OR_Q4_K: return fd_q4_K(n, w, a);
            case OR_Q5_K: return fd_q5_K(n, w, a);
            case OR_Q6_K: return fd_q6_K(n, w, a);
            case OR_Q8_0: return fd_q8_0(n, w, a);
            default: break;
        }
    }
#endif
    switch (wtype) {
        case OR_Q4_K: return vd_q4_K(n, w, a);
        case OR_Q5_K: return vd_q5_K(n, w, a);
        case OR_Q6_K: return vd_q6_K(n, w, a);
        case OR_Q8_0: return vd_q8_0(n, w, a);
        case OR_F16: return vd_f16(n, w, a);
        case OR_F32: return vd_f32(n, w, a);
        default: return NAN;
    }
}

static size_t act_bytes(int wtype, int64_t cols) {
    int vt = or_vec_dot_type(wtype);
    return (size_t)(cols / or_block_size(vt)) * or_type_size(vt);
}
static void quantize_act(int wtype, const float* x, void* act, int64_t cols) {
    int vt = or_vec_dot_type(wtype);
    if (vt == OR_Q8_K) or_quantize_row_q8_K(x, act, cols);
    else if (vt == OR_Q8_0) { if (g_x86 & OR_X86_Q80) x86_quantize_row_q8_0(x, act, cols); else or_quantize_row_q8_0(x, act, cols); }
    else if (vt == OR_F16) for (int64_t i = 0; i < cols; ++i) ((uint16_t*)act)[i] = llmi_f2h(x[i]);
    else memcpy(act, x, (size_t)cols * 4);
}

/* the activation conversion or_matvec applies for weight type wtype (vec_dot_type of
 * wtype, under the current mode: x86 q8_0 rounding with OR_X86_Q80) */
int or_quantize_act(int wtype, const float* x, void* out, int64_t cols) {
    if (or_vec_dot_type(wtype) < 0 || cols % or_block_size(or_vec_dot_type(wtype))) return -1;
    quantize_act(wtype, x, out, cols);
    return 0;
}

/* upstream ggml_compute_forward_mul_mat for one src1 column: src1 is converted to
 * vec_dot_type once, then vec_dot per src0 row. */
int or_matvec(int wtype, const void* W, int64_t rows, int64_t cols, const float* x, float* y, int nthreads) {
    if (or_vec_dot_type(wtype) < 0 || cols % or_block_size(wtype)) return -1;
    void* act = malloc(act_bytes(wtype, cols));
    if (!act) return -1;
    quantize_act(wtype, x, act, cols);
    const size_t row_bytes = (size_t)(cols / or_block_size(wtype)) * or_type_size(wtype);
    (void)nthreads;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t r = 0; r < rows; ++r)
        y[r] = or_vec_dot(wtype, (int)cols, (const uint8_t*)W + (size_t)r * row_bytes, act);
    free(act);
    return 0;
}

/* upstream ggml_compute_forward_rms_norm_f32 (sum of x*x in ggml_float=double,
 * scale = 1/sqrtf(mean+eps)) followed by ggml_compute_forward_mul (y*w) */
void or_rms_norm_mul(const float* x, const float* w, float* y, int n, float eps) {
    double sum = 0.0;
    for (int i = 0; i < n; ++i) sum += (double)(x[i] * x[i]);
    const float mean = (float)(sum / n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int i = 0; i < n; ++i) y[i] = x[i] * scale;
    for (int i = 0; i < n; ++i) y[i] = y[i] * w[i];
}

/* =======================================================================
 * GGUF v3 reader (independent of the product's loader) — SURVEY.md §8a row a4,
 * format per SURVEY.md Appendix A.
 * ======================================================================= */
enum { G_U8, G_I8, G_U16, G_I16, G_U32, G_I32, G_F32, G_BOOL, G_STR, G_ARR, G_U64, G_I64, G_F64 };

typedef struct { char name[96]; int type; int n_dims; int64_t ne[4]; uint64_t offset; const uint8_t* data; } or_tensor;

typedef struct {
    const uint8_t* p; const uint8_t* end; int ok;
} rd_t;
static uint64_t rd_u(rd_t* r, int n) {
    if (r->p + n > r->end) { r->ok = 0; return 0; }
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v |= (uint64_t)r->p[i] << (8 * i);
    r->p += n; return v;
}
static size_t g_scalar_size(int t) {
    switch (t) {
        case G_U8: case G_I8: case G_BOOL: return 1; case G_U16: case G_I16: return 2;
        case G_U32: case G_I32: case G_F32: return 4; case G_U64: case G_I64: case G_F64: return 8;
        default: return 0;
    }
}
static void rd_skip_value(rd_t* r, int t) {
    if (t == G_STR) { uint64_t n = rd_u(r, 8); if (r->p + n > r->end) r->ok = 0; else r->p += n; return; }
    if (t == G_ARR) {
        int et = (int)rd_u(r, 4); uint64_t n = rd_u(r, 8);
        for (uint64_t i = 0; i < n && r->ok; ++i) rd_skip_value(r, et);
        return;
    }
    size_t s = g_scalar_size(t);
    if (!s || r->p + s > r->end) { r->ok = 0; return; }
    r->p += s;
}
static double rd_num(rd_t* r, int t) {
    uint64_t v = rd_u(r, (int)g_scalar_size(t));
    switch (t) {
        case G_I8: return (int8_t)v; case G_I16: return (int16_t)v; case G_I32: return (int32_t)v;
        case G_I64: return (double)(int64_t)v;
        case G_F32: { uint32_t u = (uint32_t)v; return llmi_u2f(u); }
        case G_F64: { double d; memcpy(&d, &v, 8); return d; }
        default: return (double)v;
    }
}

struct or_model {
    /* file */
    int fd; uint8_t* map; size_t map_len;
    int n_tensors; or_tensor* tensors;
    /* hparams */
    int n_embd, n_layer, n_head, n_head_kv, n_ff, n_vocab, n_rot, head_dim, n_ctx, file_type;
    float eps, rope_base;
    /* weights */
    const or_tensor *tok_embd, *out_norm, *output, *rope_freqs;
    struct { const or_tensor *an, *wq, *wk, *wv, *wo, *fn, *wg, *wu, *wd; } *L;
    /* state */
    uint16_t *kc, *vc;       /* [layer][pos][n_head_kv*head_dim] f16 */
    float *x, *xb, *q, *k, *v, *att, *hb, *hb2, *tmp, *sc;
    float *tap_embd, *tap_final;
    /* or_model_localize: the decode matrices' anonymous copies */
    uint8_t** local; int n_local;
};

static const or_tensor* find_t(const or_model* m, const char* name) {
    for (int i = 0; i < m->n_tensors; ++i) if (!strcmp(m->tensors[i].name, name)) return &m->tensors[i];
    return NULL;
}

static int key_eq(const uint8_t* s, uint64_t n, const char* k) { return strlen(k) == n && !memcmp(s, k, n); }

or_model* or_model_load(const char* path, int n_ctx) {
    or_model* m = calloc(1, sizeof *m);
    if (!m) return NULL;
    m->fd = -1;
    m->rope_base = 10000.0f; m->eps = 1e-5f;
    struct stat st;
    m->fd = open(path, O_RDONLY);
    if (m->fd < 0) OR_FAIL("open %s failed", path);
    if (fstat(m->fd, &st)) OR_FAIL("stat failed");
    m->map_len = (size_t)st.st_size;
    m->map = mmap(NULL, m->map_len, PROT_READ, MAP_PRIVATE, m->fd, 0);
    if (m->map == MAP_FAILED) { m->map = NULL; OR_FAIL("mmap failed"); }
    rd_t r = {m->map, m->map + m->map_len, 1};
    if (rd_u(&r, 4) != 0x46554747u) OR_FAIL("bad magic");
    uint32_t version = (uint32_t)rd_u(&r, 4);
    if (version != 3) OR_FAIL("unsupported GGUF version %u", version);
    uint64_t n_tensors = rd_u(&r, 8), n_kv = rd_u(&r, 8);
    uint64_t alignment = 32;
    int64_t arch_vocab = -1, toks_n = -1;
    for (uint64_t i = 0; i < n_kv && r.ok; ++i) {
        uint64_t kl = rd_u(&r, 8);
        const uint8_t* key = r.p;
        if (r.p + kl > r.end) { r.ok = 0; break; }
        r.p += kl;
        int t = (int)rd_u(&r, 4);
        if (t == G_STR || t == G_ARR) {
            if (t == G_ARR && key_eq(key, kl, "tokenizer.ggml.tokens")) {
                const uint8_t* save = r.p; rd_u(&r, 4); toks_n = (int64_t)rd_u(&r, 8); r.p = save;
            }
            rd_skip_value(&r, t);
            continue;
        }
        double v = rd_num(&r, t);
#define KV(name, field) else if (key_eq(key, kl, name)) m->field = (typeof(m->field))v
        if (key_eq(key, kl, "general.alignment")) alignment = (uint64_t)v;
        KV("llama.embedding_length", n_embd); KV("llama.block_count", n_layer);
        KV("llama.feed_forward_length", n_ff); KV("llama.attention.head_count", n_head);
        KV("llama.attention.head_count_kv", n_head_kv); KV("llama.rope.dimension_count", n_rot);
        KV("llama.attention.layer_norm_rms_epsilon", eps); KV("llama.rope.freq_base", rope_base);
        KV("general.file_type", file_type);
        else if (key_eq(key, kl, "llama.vocab_size")) arch_vocab = (int64_t)v;
#undef KV
    }
    if (!r.ok) OR_FAIL("truncated metadata");
    if (!m->n_embd || !m->n_layer || !m->n_head) OR_FAIL("missing llama.* hyperparameters");
    if (!m->n_head_kv) m->n_head_kv = m->n_head;
    m->head_dim = m->n_embd / m->n_head;
    if (!m->n_rot) m->n_rot = m->head_dim;
    m->n_tensors = (int)n_tensors;
    m->tensors = calloc(n_tensors ? n_tensors : 1, sizeof(or_tensor));
    for (uint64_t i = 0; i < n_tensors && r.ok; ++i) {
        or_tensor* T = &m->tensors[i];
        uint64_t nl = rd_u(&r, 8);
        if (nl >= sizeof T->name || r.p + nl > r.end) OR_FAIL("bad tensor name");
        memcpy(T->name, r.p, nl); r.p += nl;
        T->n_dims = (int)rd_u(&r, 4);
        if (T->n_dims < 1 || T->n_dims > 4) OR_FAIL("bad n_dims");
        for (int d = 0; d < 4; ++d) T->ne[d] = 1;
        for (int d = 0; d < T->n_dims; ++d) T->ne[d] = (int64_t)rd_u(&r, 8);
        T->type = (int)rd_u(&r, 4);
        T->offset = rd_u(&r, 8);
    }
    if (!r.ok) OR_FAIL("truncated tensor infos");
    size_t data_start = (size_t)(r.p - m->map);
    data_start = (data_start + alignment - 1) / alignment * alignment;
    for (int i = 0; i < m->n_tensors; ++i) {
        or_tensor* T = &m->tensors[i];
        int64_t n = T->ne[0] * T->ne[1] * T->ne[2] * T->ne[3];
        size_t bytes = (size_t)(n / or_block_size(T->type)) * or_type_size(T->type);
        if (!or_type_size(T->type)) OR_FAIL("tensor %s: unsupported type %d", T->name, T->type);
        if (data_start + T->offset + bytes > m->map_len) OR_FAIL("tensor %s out of file", T->name);
        T->data = m->map + data_start + T->offset;
    }
    m->tok_embd = find_t(m, "token_embd.weight");
    m->out_norm = find_t(m, "output_norm.weight");
    m->output = find_t(m, "output.weight");
    m->rope_freqs = find_t(m, "rope_freqs.weight");
    if (!m->tok_embd || !m->out_norm) OR_FAIL("missing token_embd/output_norm");
    if (!m->output) m->output = m->tok_embd;  /* tied embeddings */
    m->n_vocab = (int)m->tok_embd->ne[1];
    (void)arch_vocab; (void)toks_n;
    m->L = calloc((size_t)m->n_layer, sizeof *m->L);
    for (int l = 0; l < m->n_layer; ++l) {
        char nm[96];
#define LT(f, s) do { snprintf(nm, sizeof nm, "blk.%d.%s.weight", l, s); m->L[l].f = find_t(m, nm); \
                      if (!m->L[l].f) OR_FAIL("missing %s", nm); } while (0)
        LT(an, "attn_norm"); LT(wq, "attn_q"); LT(wk, "attn_k"); LT(wv, "attn_v"); LT(wo, "attn_output");
        LT(fn, "ffn_norm"); LT(wg, "ffn_gate"); LT(wu, "ffn_up"); LT(wd, "ffn_down");
#undef LT
    }
    if (!m->n_ff) m->n_ff = (int)m->L[0].wg->ne[1];
    m->n_ctx = n_ctx > 0 ? n_ctx : 512;
    const size_t kvd = (size_t)m->n_head_kv * m->head_dim;
    m->kc = calloc((size_t)m->n_layer * m->n_ctx * kvd, 2);
    m->vc = calloc((size_t)m->n_layer * m->n_ctx * kvd, 2);
    const int E = m->n_embd, F = m->n_ff;
    m->x = calloc(E, 4); m->xb = calloc(E, 4); m->q = calloc(E, 4);
    m->k = calloc(kvd, 4); m->v = calloc(kvd, 4); m->att = calloc(E, 4);
    m->hb = calloc(F, 4); m->hb2 = calloc(F, 4); m->tmp = calloc(E > F ? E : F, 4);
    m->sc = calloc((size_t)m->n_head * m->n_ctx, 4);
    m->tap_embd = calloc(E, 4); m->tap_final = calloc(E, 4);
    if (!m->kc || !m->vc || !m->sc) OR_FAIL("out of memory");
    return m;
fail:
    or_model_free(m);
    return NULL;
}

static size_t tensor_bytes(const or_tensor* T) {
    int64_t n = T->ne[0] * T->ne[1] * T->ne[2] * T->ne[3];
    return (size_t)(n / or_block_size(T->type)) * or_type_size(T->type);
}

/* CPU-baseline placement (bench.py cpu_baseline leg; numerics untouched): copy every
 * matrix the decode step streams out of the file mapping into anonymous memory, each row
 * written by the OpenMP thread of nth that or_decode's static row loops will give it
 * (q/k/v and gate/up as the concatenations matvec_multi splits), so under Linux's
 * first-touch policy a row's pages sit on the NUMA node of the thread that reads them.
 * The mapping's page cache sits on the node that wrote the file.  Returns bytes copied. */
static uint8_t* loc_rows(const or_tensor* const* T, int n, int nth, uint8_t** out) {
    int64_t rows0[4] = {0, 0, 0, 0};
    size_t rb[3];
    for (int i = 0; i < n; ++i) {
        rows0[i + 1] = rows0[i] + T[i]->ne[1];
        rb[i] = (size_t)(T[i]->ne[0] / or_block_size(T[i]->type)) * or_type_size(T[i]->type);
        out[i] = aligned_alloc(4096, ((size_t)T[i]->ne[1] * rb[i] + 4095) / 4096 * 4096);
        if (!out[i]) return NULL;
    }
#pragma omp parallel for schedule(static) num_threads(nth > 0 ? nth : 1)
    for (int64_t g = 0; g < rows0[n]; ++g) {
        int i = 0;
        while (g >= rows0[i + 1]) ++i;
        const int64_t r = g - rows0[i];
        memcpy(out[i] + (size_t)r * rb[i], (const uint8_t*)T[i]->data + (size_t)r * rb[i], rb[i]);
    }
    return out[0];
}
int64_t or_model_localize(or_model* m, int nth) {
    if (m->local) return 0;
    const int nm = m->n_layer * 7 + 1;
    m->local = calloc((size_t)nm, sizeof(uint8_t*));
    if (!m->local) return -1;
    int k = 0;
    int64_t bytes = 0;
    for (int l = 0; l < m->n_layer; ++l) {
        const or_tensor* const qkv[3] = {m->L[l].wq, m->L[l].wk, m->L[l].wv};
        const or_tensor* const gu[2] = {m->L[l].wg, m->L[l].wu};
        const or_tensor* const wo[1] = {m->L[l].wo};
        const or_tensor* const wd[1] = {m->L[l].wd};
        const or_tensor* const* sets[4] = {qkv, wo, gu, wd};
        const int ns[4] = {3, 1, 2, 1};
        for (int j = 0; j < 4; ++j) {
            uint8_t* out[3] = {NULL, NULL, NULL};
            if (!loc_rows(sets[j], ns[j], nth, out)) return -1;
            for (int i = 0; i < ns[j]; ++i) {
                m->local[k++] = out[i];
                ((or_tensor*)sets[j][i])->data = out[i];
                bytes += (int64_t)tensor_bytes(sets[j][i]);
            }
        }
    }
    {
        const or_tensor* const o[1] = {m->output};
        uint8_t* out[3] = {NULL, NULL, NULL};
        if (!loc_rows(o, 1, nth, out)) return -1;
        m->local[k++] = out[0];
        ((or_tensor*)m->output)->data = out[0];
        bytes += (int64_t)tensor_bytes(m->output);
    }
    m->n_local = k;
    return bytes;
}

void or_model_free(or_model* m) {
    if (!m) return;
    if (m->local) {
        for (int i = 0; i < m->n_local; ++i) free(m->local[i]);
        free(m->local);
    }
    if (m->map) munmap(m->map, m->map_len);
    if (m->fd >= 0) close(m->fd);
    free(m->tensors); free(m->L); free(m->kc); free(m->vc);
    free(m->x); free(m->xb); free(m->q); free(m->k); free(m->v); free(m->att);
    free(m->hb); free(m->hb2); free(m->tmp); free(m->sc); free(m->tap_embd); free(m->tap_final);
    free(m);
}

void or_model_info(const or_model* m, int64_t* o) {
    o[0] = m->n_embd; o[1] = m->n_layer; o[2] = m->n_head; o[3] = m->n_head_kv; o[4] = m->n_ff;
    o[5] = m->n_vocab; o[6] = m->n_rot; o[7] = m->n_ctx; o[8] = m->head_dim; o[9] = m->file_type;
}

void or_kv_clear(or_model* m) {
    const size_t kvd = (size_t)m->n_head_kv * m->head_dim;
    memset(m->kc, 0, (size_t)m->n_layer * m->n_ctx * kvd * 2);
    memset(m->vc, 0, (size_t)m->n_layer * m->n_ctx * kvd * 2);
}


double or_bytes_per_token(const or_model* m, int ctx) {
    double b = 0;
    for (int l = 0; l < m->n_layer; ++l) {
        b += tensor_bytes(m->L[l].wq) + tensor_bytes(m->L[l].wk) + tensor_bytes(m->L[l].wv) + tensor_bytes(m->L[l].wo);
        b += tensor_bytes(m->L[l].wg) + tensor_bytes(m->L[l].wu) + tensor_bytes(m->L[l].wd);
        b += tensor_bytes(m->L[l].an) + tensor_bytes(m->L[l].fn);
    }
    b += tensor_bytes(m->output) + tensor_bytes(m->out_norm);
    b += (double)tensor_bytes(m->tok_embd) / m->n_vocab;
    b += (double)m->n_layer * 2.0 * m->n_head_kv * m->head_dim * 2.0 * (ctx + 1);
    return b;
}

/* upstream ggml_rope_cache_init + rope_yarn (ext_factor 0, freq_scale 1, attn_factor 1)
 * and the NORM-mode rotation of adjacent pairs in ggml_compute_forward_rope_f32.
 * theta is built by iterative multiplication by theta_scale = powf(base, -2/n_dims). */
static void rope_norm(float* v, int n_heads, int head_dim, int n_rot, int pos, float base, const float* ff) {
    const float theta_scale = powf(base, -2.0f / n_rot);
    float cache[1024];
    float theta = (float)pos;
    for (int i0 = 0; i0 < n_rot; i0 += 2) {
        const float f = ff ? ff[i0 / 2] : 1.0f;
        const float th = 1.0f * (theta / f);
        cache[i0 + 0] = cosf(th) * 1.0f;
        cache[i0 + 1] = sinf(th) * 1.0f;
        theta *= theta_scale;
    }
    for (int h = 0; h < n_heads; ++h) {
        float* s = v + (size_t)h * head_dim;
        for (int i0 = 0; i0 < n_rot; i0 += 2) {
            const float c = cache[i0], sn = cache[i0 + 1];
            const float x0 = s[i0], x1 = s[i0 + 1];
            s[i0] = x0 * c - x1 * sn;
            s[i0 + 1] = x0 * sn + x1 * c;
        }
    }
}

static void matvec_t(const or_tensor* T, const float* x, float* y, int nth) {
    or_matvec(T->type, T->data, T->ne[1], T->ne[0], x, y, nth);
}

/* or_matvec of n tensors with the same input in ONE parallel loop over all their rows
 * (q/k/v, gate/up): the activation conversion once per distinct vec_dot type, one
 * fork/join instead of n.  Each row's dot is or_matvec's. */
static void matvec_multi(const or_tensor* const* T, int n, const float* x, float* const* y, int nth) {
    void* act[3] = {NULL, NULL, NULL};
    int64_t rows0[4] = {0, 0, 0, 0};
    size_t rb[3];
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < i && !act[i]; ++j)
            if (or_vec_dot_type(T[j]->type) == or_vec_dot_type(T[i]->type)) act[i] = act[j];
        if (!act[i]) {
            act[i] = malloc(act_bytes(T[i]->type, T[i]->ne[0]));
            quantize_act(T[i]->type, x, act[i], T[i]->ne[0]);
        }
        rows0[i + 1] = rows0[i] + T[i]->ne[1];
        rb[i] = (size_t)(T[i]->ne[0] / or_block_size(T[i]->type)) * or_type_size(T[i]->type);
    }
#pragma omp parallel for schedule(static) num_threads(nth > 0 ? nth : 1)
    for (int64_t g = 0; g < rows0[n]; ++g) {
        int i = 0;
        while (g >= rows0[i + 1]) ++i;
        const int64_t r = g - rows0[i];
        y[i][r] = or_vec_dot(T[i]->type, (int)T[i]->ne[0], (const uint8_t*)T[i]->data + (size_t)r * rb[i], act[i]);
    }
    for (int i = 0; i < n; ++i) {
        int shared = 0;
        for (int j = 0; j < i; ++j) shared |= act[j] == act[i];
        if (!shared) free(act[i]);
    }
}

/* Flash attention of query head h (OR_X86_FA): upstream's CPU
 * ggml_compute_forward_flash_attn_ext_f16 for one query row with f16 K and V [ggml-cpu
 * ops.cpp, "one_chunk"; upstream, recalled, not vendored] -- what a llama-server started
 * without --flash-attn runs on the CPU when `-fa auto` resolves to on:
 *   q16 = f16(q); S = 0, M = -inf, VKQ16[D] = 0 (f16)
 *   per position t: s = ggml_vec_dot_f16(K[t], q16) * scale (+ 0, the unmasked mask)
 *     s > M: M = s, ms = expf(Mold - M), VKQ16 = f16(f32(VKQ16) * ms)   (vec_scale_f16)
 *     else:  vs = expf(s - M)
 *     VKQ16 = f16(f32(VKQ16) + f32(V[t]) * vs)                           (vec_mad_f16)
 *     S = S * ms + vs
 *   out = f32(VKQ16) * (S == 0 ? 0 : 1 / S)                               (vec_scale_f32)
 * expf is libm's (llmi_expf_glibc with FMA: what glibc's ifunc picks on an FMA host,
 * whichever ggml-cpu variant calls it; pinned to this host's libm, test_oracle_math.py).
 * With OR_X86_F16DOT (the AVX2+F16C build) the dot is the 4 x 8-lane form and vec_mad /
 * the S update are FMA-contracted; without it (the generic scalar build, no FMA) they are
 * a multiply and an add.  Single-query rows only: prompts run through it token by token. */
static void attn_head_fa(const or_model* m, int l, const float* q, int h, int n_kv, float* out) {
    const int HK = m->n_head_kv, D = m->head_dim, kvd = HK * D, g = h / (m->n_head / HK);
    const uint16_t* kl = m->kc + ((size_t)l * m->n_ctx) * kvd;
    const uint16_t* vl = m->vc + ((size_t)l * m->n_ctx) * kvd;
    const float scale = 1.0f / sqrtf((float)D);
    const int x86 = (g_x86 & OR_X86_F16DOT) != 0;
    float qf[512], kf[512], vkq[512];
    uint16_t vkq16[512];
    for (int d = 0; d < D; ++d) { qf[d] = llmi_h2f(llmi_f2h(q[d])); vkq16[d] = 0; }
    float S = 0.0f, M = -INFINITY;
    for (int t = 0; t < n_kv; ++t) {
        const uint16_t* kr = kl + (size_t)t * kvd + (size_t)g * D;
        const uint16_t* vr = vl + (size_t)t * kvd + (size_t)g * D;
        float sc;
        if (x86) {
            for (int d = 0; d < D; ++d) kf[d] = llmi_h2f(kr[d]);
            sc = x86_dot_f16f(D, kf, qf);
        } else {
            double sumf = 0.0;
            for (int d = 0; d < D; ++d) sumf += (double)(llmi_h2f(kr[d]) * qf[d]);
            sc = (float)sumf;
        }
        sc = sc * scale;
        sc = sc + 0.0f;  /* s += slope * mask (0 for every position the query sees) */
        const float Mold = M;
        float ms = 1.0f, vs = 1.0f;
        if (sc > M) {
            M = sc;
            ms = llmi_expf_glibc(Mold - M, 1);
            for (int d = 0; d < D; ++d) vkq16[d] = llmi_f2h(llmi_h2f(vkq16[d]) * ms);
        } else {
            vs = llmi_expf_glibc(sc - M, 1);
        }
        for (int d = 0; d < D; ++d)
            vkq16[d] = llmi_f2h(x86 ? fmaf(llmi_h2f(vr[d]), vs, llmi_h2f(vkq16[d]))
                                    : llmi_h2f(vkq16[d]) + llmi_h2f(vr[d]) * vs);
        S = x86 ? fmaf(S, ms, vs) : S * ms + vs;
    }
    const float S_inv = S == 0.0f ? 0.0f : 1.0f / S;
    for (int d = 0; d < D; ++d) vkq[d] = llmi_h2f(vkq16[d]);
    for (int d = 0; d < D; ++d) out[d] = vkq[d] * S_inv;
}

/* Non-flash attention of query head h (roped q, f32[D]) over the layer's first n_kv
 * cached positions: kq = mul_mat(K_f16, q) with q rounded to f16 (ggml_vec_dot_f16,
 * double sum), soft_max_ext(kq, scale 1/sqrt(D)) with a double sum, kqv =
 * mul_mat(V_f16, kq) with the probabilities rounded to f16.  w: f32[n_kv] scratch. */
static void attn_head(const or_model* m, int l, const float* q, int h, int n_kv, float* w, float* out) {
    if (g_x86 & OR_X86_FA) { attn_head_fa(m, l, q, h, n_kv, out); return; }
    const int HK = m->n_head_kv, D = m->head_dim, kvd = HK * D, g = h / (m->n_head / HK);
    const uint16_t* kl = m->kc + ((size_t)l * m->n_ctx) * kvd;
    const uint16_t* vl = m->vc + ((size_t)l * m->n_ctx) * kvd;
    const float kq_scale = 1.0f / sqrtf((float)D);
    /* f16-rounded q and K/V values as floats (the same values vd_f16 and the PV loop
     * form per element; converted once instead of once per use) */
    float qf[512];
    for (int d = 0; d < D; ++d) qf[d] = llmi_h2f(llmi_f2h(q[d]));
    float mx = -INFINITY;
    const int f16x = (g_x86 & OR_X86_F16DOT) != 0;
    for (int t = 0; t < n_kv; ++t) {
        const uint16_t* kr = kl + (size_t)t * kvd + (size_t)g * D;
        if (f16x) {
            float kf[512];
            for (int d = 0; d < D; ++d) kf[d] = llmi_h2f(kr[d]);
            w[t] = x86_dot_f16f(D, kf, qf) * kq_scale;
        } else {
            double sumf = 0.0;  /* ggml_vec_dot_f16 (generic): double accumulation */
            for (int d = 0; d < D; ++d) sumf += (double)(llmi_h2f(kr[d]) * qf[d]);
            w[t] = (float)sumf * kq_scale;
        }
        mx = fmaxf(mx, w[t]);
    }
    double sum = 0.0;
    if (g_x86 & OR_X86_VEXP) {  /* ggml_vec_soft_max_f32, AVX2: per 8 positions an fp32 hsum */
        int t = 0;
        for (; t + 7 < n_kv; t += 8) {
            float e8[8];
            for (int l = 0; l < 8; ++l) { e8[l] = x86_v_expf(w[t + l] - mx); w[t + l] = e8[l]; }
            sum += (double)x86_hsum8(e8);
        }
        if (t < n_kv) {  /* the row is padded to 32 with masked (-inf -> 0) positions */
            float e8[8] = {0};
            for (int l = 0; t + l < n_kv; ++l) { e8[l] = x86_v_expf(w[t + l] - mx); w[t + l] = e8[l]; }
            sum += (double)x86_hsum8(e8);
        }
    } else {
        for (int t = 0; t < n_kv; ++t) { float e = mode_expf(w[t] - mx); sum += (double)e; w[t] = e; }
    }
    const float inv = (float)(1.0 / sum);
    for (int t = 0; t < n_kv; ++t) w[t] = llmi_h2f(llmi_f2h(w[t] * inv));  /* p rounded to f16 */
    if (f16x) {  /* mul_mat(V^T, p): one f16 dot over the positions (padded to 32 with p = 0) per dim */
        const int np = (n_kv + 31) & ~31;
        float vf[8192], pf[8192];
        if (np > 8192) return;
        for (int t = n_kv; t < np; ++t) pf[t] = 0.f;
        for (int t = 0; t < n_kv; ++t) pf[t] = w[t];
        for (int d = 0; d < D; ++d) {
            for (int t = 0; t < n_kv; ++t) vf[t] = llmi_h2f(vl[(size_t)t * kvd + (size_t)g * D + d]);
            for (int t = n_kv; t < np; ++t) vf[t] = 0.f;
            out[d] = x86_dot_f16f(np, vf, pf);
        }
        return;
    }
    double acc[512];
    for (int d = 0; d < D; ++d) acc[d] = 0.0;
    for (int t = 0; t < n_kv; ++t) {  /* per d the same sequential double sum over t */
        const uint16_t* vr = vl + (size_t)t * kvd + (size_t)g * D;
        for (int d = 0; d < D; ++d) acc[d] += (double)(llmi_h2f(vr[d]) * w[t]);
    }
    for (int d = 0; d < D; ++d) out[d] = (float)acc[d];
}

/* One decode step of llm_build_llama [upstream llama-model.cpp] with the non-flash
 * attention path: kq = mul_mat(K_f16, q) (q rounded to f16, ggml_vec_dot_f16),
 * soft_max_ext(kq, scale = 1/sqrt(head_dim)) with double sum, kqv = mul_mat(V_f16,
 * kq) (probabilities rounded to f16).  SURVEY.md §8a rows a10-a16. */
int or_decode(or_model* m, int32_t token, int32_t pos, float* logits, int nth) {
    if (token < 0 || token >= m->n_vocab) { snprintf(g_err, sizeof g_err, "token %d out of range", token); return -1; }
    if (pos < 0 || pos >= m->n_ctx) { snprintf(g_err, sizeof g_err, "pos %d out of ctx", pos); return 1; }
    const int E = m->n_embd, H = m->n_head, HK = m->n_head_kv, D = m->head_dim, F = m->n_ff;
    const int kvd = HK * D, n_kv = pos + 1;
    const float* ff = m->rope_freqs ? (const float*)m->rope_freqs->data : NULL;
    /* get_rows(token_embd, token) -> dequantize one row */
    {
        const size_t rb = tensor_bytes(m->tok_embd) / m->n_vocab;
        or_dequantize_row(m->tok_embd->type, m->tok_embd->data + (size_t)token * rb, m->x, E);
        memcpy(m->tap_embd, m->x, (size_t)E * 4);
    }
    for (int l = 0; l < m->n_layer; ++l) {
        or_rms_norm_mul(m->x, (const float*)m->L[l].an->data, m->xb, E, m->eps);
        {
            const or_tensor* const T[3] = {m->L[l].wq, m->L[l].wk, m->L[l].wv};
            float* const Y[3] = {m->q, m->k, m->v};
            matvec_multi(T, 3, m->xb, Y, nth);
        }
        rope_norm(m->q, H, D, m->n_rot, pos, m->rope_base, ff);
        rope_norm(m->k, HK, D, m->n_rot, pos, m->rope_base, ff);
        uint16_t* kl = m->kc + ((size_t)l * m->n_ctx) * kvd;
        uint16_t* vl = m->vc + ((size_t)l * m->n_ctx) * kvd;
        for (int i = 0; i < kvd; ++i) { kl[(size_t)pos * kvd + i] = llmi_f2h(m->k[i]); vl[(size_t)pos * kvd + i] = llmi_f2h(m->v[i]); }
#pragma omp parallel for schedule(static) num_threads(nth > 0 ? nth : 1)
        for (int h = 0; h < H; ++h) attn_head(m, l, m->q + (size_t)h * D, h, n_kv, m->sc + (size_t)h * m->n_ctx, m->att + (size_t)h * D);
        matvec_t(m->L[l].wo, m->att, m->tmp, nth);
        for (int i = 0; i < E; ++i) m->x[i] = m->tmp[i] + m->x[i];
        or_rms_norm_mul(m->x, (const float*)m->L[l].fn->data, m->xb, E, m->eps);
        {
            const or_tensor* const T[2] = {m->L[l].wg, m->L[l].wu};
            float* const Y[2] = {m->hb, m->hb2};
            matvec_multi(T, 2, m->xb, Y, nth);
        }
        for (int i = 0; i < F; ++i) m->hb[i] = mode_silu(m->hb[i]) * m->hb2[i];
        matvec_t(m->L[l].wd, m->hb, m->tmp, nth);
        for (int i = 0; i < E; ++i) m->x[i] = m->tmp[i] + m->x[i];
    }
    memcpy(m->tap_final, m->x, (size_t)E * 4);
    if (!logits) return 0;  /* prompt token whose logits nobody reads: KV cache only */
    or_rms_norm_mul(m->x, (const float*)m->out_norm->data, m->xb, E, m->eps);
    or_matvec(m->output->type, m->output->data, m->n_vocab, E, m->xb, logits, nth);
    return 0;
}

/* T consecutive or_decode steps at positions pos0.. with no logits (a prompt), the
 * loops reordered for speed: per layer each weight row is unpacked once and dotted with
 * the T activations (vd_generic_unpacked: or_vec_dot's operations with the row's
 * unpacking and constants hoisted), then attention per (token, head).  Every token's operations are exactly
 * or_decode's (the KV rows a token attends to are written by the same layer before).
 * Leaves the last token's state (x, taps) as or_decode would.  Test infrastructure for
 * the long parity tests (2048-token prompts at 7B widths). */
static void matmul_t(const or_tensor* W, const float* X, int T, float* Y, int nth) {
    const int wtype = W->type;
    const int64_t rows = W->ne[1], cols = W->ne[0];
    const size_t ab = act_bytes(wtype, cols);
    uint8_t* acts = malloc(ab * (size_t)T);
    for (int t = 0; t < T; ++t) quantize_act(wtype, X + (size_t)t * cols, acts + ab * t, cols);
    const size_t row_bytes = (size_t)(cols / or_block_size(wtype)) * or_type_size(wtype);
    const int kq = (wtype == OR_Q4_K || wtype == OR_Q5_K || wtype == OR_Q6_K) && !(g_x86 & OR_X86_DOTS);
#pragma omp parallel num_threads(nth > 0 ? nth : 1)
    {
        uint8_t* u = malloc((size_t)cols);
        RowConst* rcs = malloc(sizeof(RowConst) * (size_t)(cols / QK_K + 1));
        const size_t bb = or_type_size(wtype);
#pragma omp for schedule(dynamic, 8)
        for (int64_t r = 0; r < rows; ++r) {
            const uint8_t* w = (const uint8_t*)W->data + (size_t)r * row_bytes;
            if (kq) {
                for (int64_t ib = 0; ib < cols / QK_K; ++ib) {
                    block_unpack_kq(wtype, w + (size_t)ib * bb, u + ib * QK_K);
                    row_consts(wtype, w + (size_t)ib * bb, rcs + ib);
                }
                for (int t = 0; t < T; ++t) Y[(size_t)t * rows + r] = vd_generic_unpacked(wtype, (int)cols, rcs, u, acts + ab * t);
            } else {
                for (int t = 0; t < T; ++t) Y[(size_t)t * rows + r] = or_vec_dot(wtype, (int)cols, w, acts + ab * t);
            }
        }
        free(u);
        free(rcs);
    }
    free(acts);
}

int or_prefill(or_model* m, const int32_t* tokens, int T, int pos0, int nth) {
    if (T <= 0 || pos0 < 0 || pos0 + T > m->n_ctx) { snprintf(g_err, sizeof g_err, "prefill range out of ctx"); return 1; }
    for (int t = 0; t < T; ++t)
        if (tokens[t] < 0 || tokens[t] >= m->n_vocab) { snprintf(g_err, sizeof g_err, "token %d out of range", tokens[t]); return -1; }
    const int E = m->n_embd, H = m->n_head, HK = m->n_head_kv, D = m->head_dim, F = m->n_ff, kvd = HK * D, QD = H * D;
    const float* ff = m->rope_freqs ? (const float*)m->rope_freqs->data : NULL;
    float* X = malloc((size_t)T * E * 4); float* XB = malloc((size_t)T * E * 4); float* TMP = malloc((size_t)T * E * 4);
    float* Q = malloc((size_t)T * QD * 4); float* K = malloc((size_t)T * kvd * 4); float* V = malloc((size_t)T * kvd * 4);
    float* ATT = malloc((size_t)T * QD * 4); float* HB = malloc((size_t)T * F * 4); float* HB2 = malloc((size_t)T * F * 4);
    const size_t rb = tensor_bytes(m->tok_embd) / m->n_vocab;
    for (int t = 0; t < T; ++t) or_dequantize_row(m->tok_embd->type, m->tok_embd->data + (size_t)tokens[t] * rb, X + (size_t)t * E, E);
    for (int l = 0; l < m->n_layer; ++l) {
        for (int t = 0; t < T; ++t) or_rms_norm_mul(X + (size_t)t * E, (const float*)m->L[l].an->data, XB + (size_t)t * E, E, m->eps);
        matmul_t(m->L[l].wq, XB, T, Q, nth);
        matmul_t(m->L[l].wk, XB, T, K, nth);
        matmul_t(m->L[l].wv, XB, T, V, nth);
        uint16_t* kl = m->kc + ((size_t)l * m->n_ctx) * kvd;
        uint16_t* vl = m->vc + ((size_t)l * m->n_ctx) * kvd;
        for (int t = 0; t < T; ++t) {
            rope_norm(Q + (size_t)t * QD, H, D, m->n_rot, pos0 + t, m->rope_base, ff);
            rope_norm(K + (size_t)t * kvd, HK, D, m->n_rot, pos0 + t, m->rope_base, ff);
            for (int i = 0; i < kvd; ++i) {
                kl[(size_t)(pos0 + t) * kvd + i] = llmi_f2h(K[(size_t)t * kvd + i]);
                vl[(size_t)(pos0 + t) * kvd + i] = llmi_f2h(V[(size_t)t * kvd + i]);
            }
        }
#pragma omp parallel num_threads(nth > 0 ? nth : 1)
        {
            float* w = malloc((size_t)m->n_ctx * 4);
#pragma omp for schedule(dynamic, 1)
            for (int th = 0; th < T * H; ++th) {
                const int t = th / H, h = th % H;
                attn_head(m, l, Q + (size_t)t * QD + (size_t)h * D, h, pos0 + t + 1, w, ATT + (size_t)t * QD + (size_t)h * D);
            }
            free(w);
        }
        matmul_t(m->L[l].wo, ATT, T, TMP, nth);
        for (size_t i = 0; i < (size_t)T * E; ++i) X[i] = TMP[i] + X[i];
        for (int t = 0; t < T; ++t) or_rms_norm_mul(X + (size_t)t * E, (const float*)m->L[l].fn->data, XB + (size_t)t * E, E, m->eps);
        matmul_t(m->L[l].wg, XB, T, HB, nth);
        matmul_t(m->L[l].wu, XB, T, HB2, nth);
        for (size_t i = 0; i < (size_t)T * F; ++i) HB[i] = mode_silu(HB[i]) * HB2[i];
        matmul_t(m->L[l].wd, HB, T, TMP, nth);
        for (size_t i = 0; i < (size_t)T * E; ++i) X[i] = TMP[i] + X[i];
        if (l == m->n_layer - 1) {  /* the last token's taps, as or_decode leaves them */
            memcpy(m->q, Q + (size_t)(T - 1) * QD, (size_t)QD * 4);
            memcpy(m->k, K + (size_t)(T - 1) * kvd, (size_t)kvd * 4);
            memcpy(m->v, V + (size_t)(T - 1) * kvd, (size_t)kvd * 4);
            memcpy(m->att, ATT + (size_t)(T - 1) * QD, (size_t)QD * 4);
            memcpy(m->hb, HB + (size_t)(T - 1) * F, (size_t)F * 4);
        }
    }
    memcpy(m->x, X + (size_t)(T - 1) * E, (size_t)E * 4);
    memcpy(m->tap_final, m->x, (size_t)E * 4);
    free(X); free(XB); free(TMP); free(Q); free(K); free(V); free(ATT); free(HB); free(HB2);
    return 0;
}

int or_tap(const or_model* m, int which, float* out) {
    if (which == 0) memcpy(out, m->tap_embd, (size_t)m->n_embd * 4);
    else if (which == 1) memcpy(out, m->tap_final, (size_t)m->n_embd * 4);
    /* last layer's intermediates of the last step: 2 q (roped), 3 attention output,
     * 4 SwiGLU output, 5 k (roped), 6 v */
    else if (which == 2) memcpy(out, m->q, (size_t)m->n_head * m->head_dim * 4);
    else if (which == 3) memcpy(out, m->att, (size_t)m->n_head * m->head_dim * 4);
    else if (which == 4) memcpy(out, m->hb, (size_t)m->n_ff * 4);
    else if (which == 5) memcpy(out, m->k, (size_t)m->n_head_kv * m->head_dim * 4);
    else if (which == 6) memcpy(out, m->v, (size_t)m->n_head_kv * m->head_dim * 4);
    /* 7 / 8: the last layer's K / V cache, raw f16 [pos][n_head_kv*head_dim] for all n_ctx */
    else if (which == 7 || which == 8) {
        const size_t kvl = (size_t)m->n_ctx * m->n_head_kv * m->head_dim;
        memcpy(out, (which == 7 ? m->kc : m->vc) + (size_t)(m->n_layer - 1) * kvl, kvl * 2);
    }
    else return -1;
    return 0;
}

/* Host DRAM streaming-read rate (bench.py's CPU roofline beside the CPU baseline): every
 * thread sums its share of a `bytes` buffer (touched first), best of `reps` passes.
 * Returns GB/s. */
double or_host_stream_gbps(size_t bytes, int reps, int nth) {
    const size_t n = bytes / 8;
    uint64_t* buf = (uint64_t*)malloc(n * 8);
    if (!buf) return -1.0;
#pragma omp parallel for schedule(static) num_threads(nth > 0 ? nth : 1)
    for (size_t i = 0; i < n; ++i) buf[i] = i;
    double best = 0.0;
    volatile uint64_t sink = 0;
    for (int r = 0; r < reps; ++r) {
        const double t0 = omp_get_wtime();
        uint64_t s = 0;
#pragma omp parallel for schedule(static) reduction(+ : s) num_threads(nth > 0 ? nth : 1)
        for (size_t i = 0; i < n; ++i) s += buf[i];
        const double dt = omp_get_wtime() - t0;
        sink += s;
        if (dt > 0 && (double)bytes / dt / 1e9 > best) best = (double)bytes / dt / 1e9;
    }
    (void)sink;
    free(buf);
    return best;
}
