/*
 * llmi_math.h — scalar numerics shared by the HIP decode path and its CPU oracle.
 *
 * Everything here is plain IEEE-754 single precision with round-to-nearest-even and
 * NO fused multiply-add: both the HIP library and oracle/ are compiled with
 * -ffp-contract=off, so a function below returns the same bits on gfx950 and on x86.
 *
 * Why a private expf: ggml's CPU path (the reference's NGL=0 llama-server, an
 * un-vendored, unpinned dependency — SURVEY.md §8c) evaluates exp() through libm or
 * its own SIMD polynomial depending on the ISA it was built for.  Neither exists on
 * the GPU, and libm/ocml differ in the last ulp.  llmi fixes ONE definition (range
 * reduction + degree-7 Taylor, < 2 ulp vs correctly rounded, checked in
 * tests/test_oracle_math.py) and uses it on both sides, so softmax and SiLU are
 * bit-identical between the oracle and the GPU.  This is a documented deviation
 * from "whatever libm the reference image shipped" (DESIGN.md §Numerics).
 *
 * nearest_int() restates ggml's magic-number rounding used by quantize_row_q8_K_ref
 * (upstream ggml-quants.c).
 */
#ifndef LLMI_MATH_H
#define LLMI_MATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define LLMI_HD static inline __attribute__((always_inline)) __host__ __device__
#else
#define LLMI_HD static inline
#endif

LLMI_HD uint32_t llmi_f2u(float f) {
    union { float f; uint32_t u; } v; v.f = f; return v.u;
}
LLMI_HD float llmi_u2f(uint32_t u) {
    union { float f; uint32_t u; } v; v.u = u; return v.f;
}

/* IEEE half -> float (exact). */
LLMI_HD float llmi_h2f(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    if (exp == 0x1fu) return llmi_u2f(sign | 0x7f800000u | (man << 13));
    if (exp == 0) {
        if (man == 0) return llmi_u2f(sign);
        /* subnormal: man * 2^-24, exact in float */
        float v = (float)man * 5.9604644775390625e-08f;
        return llmi_u2f(sign | llmi_f2u(v));
    }
    return llmi_u2f(sign | ((exp + 112u) << 23) | (man << 13));
}

/* float -> IEEE half, round to nearest even (same result as F16C / v_cvt_f16_f32). */
LLMI_HD uint16_t llmi_f2h(float f) {
    uint32_t x = llmi_f2u(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to +-inf */
    if (ax < 0x38800000u) {                                   /* half subnormal or zero */
        if (ax < 0x33000000u) return (uint16_t)sign;          /* < 2^-25 (ties -> 0) */
        uint32_t e = ax >> 23;
        uint32_t m = (ax & 0x7fffffu) | 0x800000u;
        uint32_t shift = 126u - e;                            /* 14..24 */
        uint32_t q = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1u);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t r = ax - 0x38000000u;                            /* rebias 127 -> 15 */
    r = (r + 0xfffu + ((r >> 13) & 1u)) >> 13;
    return (uint16_t)(sign | r);
}

/* ggml nearest_int(): round-half-even via the 1.5*2^23 magic constant. |fval| <= 4194303. */
LLMI_HD int llmi_nearest_int(float fval) {
    float val = fval + 12582912.f;
    int32_t i = (int32_t)llmi_f2u(val);
    return (i & 0x007fffff) - 0x00400000;
}

/* exp(x) for float, < 2 ulp; identical bits on host and device (no FMA, RNE). */
LLMI_HD float llmi_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return llmi_u2f(0x7f800000u);
    if (x < -103.97208404541015625f) return 0.0f;
    /* n = round(x / ln2) */
    float t = x * 1.44269502162933349609375f;
    float nf = t + 12582912.f;          /* round-half-even to integer */
    nf = nf - 12582912.f;
    int32_t n = (int32_t)nf;
    /* Cody-Waite: ln2 = C1 + C2, C1 has 9 significant bits so n*C1 is exact */
    float r = x - nf * 0.693359375f;
    r = r - nf * -2.12194440e-4f;
    /* e^r, |r| <= 0.347: Taylor to degree 7 (truncation < 5e-9 relative) */
    float p = 1.98412698e-4f;           /* 1/5040 */
    p = p * r + 1.38888889e-3f;         /* 1/720  */
    p = p * r + 8.33333333e-3f;         /* 1/120  */
    p = p * r + 4.16666667e-2f;         /* 1/24   */
    p = p * r + 1.66666667e-1f;         /* 1/6    */
    p = p * r + 0.5f;
    p = p * r + 1.0f;
    p = p * r + 1.0f;
    /* scale by 2^n, in two exact steps when 2^n alone is not a normal float */
    if (n > 127) { p = p * 2.0f; n -= 1; }
    if (n < -126) { p = p * llmi_u2f((uint32_t)(n + 126 + 127) << 23); return p * 1.17549435e-38f; }
    return p * llmi_u2f((uint32_t)(n + 127) << 23);
}

/* ggml SiLU: x / (1 + exp(-x)) with the shared exp. */
LLMI_HD float llmi_silu(float x) { return x / (1.0f + llmi_expf(-x)); }

/* ---------------------------------------------------------------------------------
 * Deterministic counter-based generator for synthetic GGUF weights:
 * byte k of tensor t under seed s is a pure function of (s, t, k), so the HIP
 * generator, the C file writer and any test can reproduce any tensor independently.
 * --------------------------------------------------------------------------------- */
LLMI_HD uint64_t llmi_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
/* 64 random bits for (seed, tensor, counter). */
LLMI_HD uint64_t llmi_rand64(uint64_t seed, uint64_t tensor, uint64_t ctr) {
    return llmi_mix64(llmi_mix64(seed * 0x9e3779b97f4a7c15ull + tensor) + ctr * 0xd1b54a32d192ed03ull);
}
/* uniform float in [0,1) from the top 24 bits */
LLMI_HD float llmi_u01(uint64_t r) { return (float)(uint32_t)(r >> 40) * 5.9604644775390625e-08f; }

#endif /* LLMI_MATH_H */
