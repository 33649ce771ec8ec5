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

/* glibc's expf (sysdeps/ieee754/flt-32/e_expf.c, the ARM optimized-routines algorithm,
 * glibc >= 2.27; upstream, not vendored), restated for the flash-attention numerics
 * (ggml's CPU flash_attn_ext calls libm expf for its online-softmax factors):
 * x*32/ln2 = k + r in double, 2^(k/32) from a 32-entry table of correctly rounded
 * doubles, a degree-3 polynomial in r, one final double -> float rounding.  FMA: the
 * glibc build an x86-64 FMA host dispatches to (__expf_fma) contracts the polynomial's
 * a*b+c; fma != 0 selects that form.  Which form equals THIS host's libm is checked
 * exhaustively over the softmax range by tests/test_oracle_math.py. */
LLMI_HD uint64_t llmi_d2u(double d) {
    union { double d; uint64_t u; } v; v.d = d; return v.u;
}
LLMI_HD double llmi_u2d(uint64_t u) {
    union { double d; uint64_t u; } v; v.u = u; return v.d;
}
LLMI_HD uint64_t llmi_exp2f_tab(uint32_t i) {  /* asuint64(2^(i/32)) - (i << 47) */
    switch (i & 31u) {
        case 0: return 0x3ff0000000000000ull; case 1: return 0x3fefd9b0d3158574ull;
        case 2: return 0x3fefb5586cf9890full; case 3: return 0x3fef9301d0125b51ull;
        case 4: return 0x3fef72b83c7d517bull; case 5: return 0x3fef54873168b9aaull;
        case 6: return 0x3fef387a6e756238ull; case 7: return 0x3fef1e9df51fdee1ull;
        case 8: return 0x3fef06fe0a31b715ull; case 9: return 0x3feef1a7373aa9cbull;
        case 10: return 0x3feedea64c123422ull; case 11: return 0x3feece086061892dull;
        case 12: return 0x3feebfdad5362a27ull; case 13: return 0x3feeb42b569d4f82ull;
        case 14: return 0x3feeab07dd485429ull; case 15: return 0x3feea47eb03a5585ull;
        case 16: return 0x3feea09e667f3bcdull; case 17: return 0x3fee9f75e8ec5f74ull;
        case 18: return 0x3feea11473eb0187ull; case 19: return 0x3feea589994cce13ull;
        case 20: return 0x3feeace5422aa0dbull; case 21: return 0x3feeb737b0cdc5e5ull;
        case 22: return 0x3feec49182a3f090ull; case 23: return 0x3feed503b23e255dull;
        case 24: return 0x3feee89f995ad3adull; case 25: return 0x3feeff76f2fb5e47ull;
        case 26: return 0x3fef199bdd85529cull; case 27: return 0x3fef3720dcef9069ull;
        case 28: return 0x3fef5818dcfba487ull; case 29: return 0x3fef7c97337b9b5full;
        case 30: return 0x3fefa4afa2a490daull; default: return 0x3fefd0765b6e4540ull;
    }
}
LLMI_HD double llmi_fma_d(double a, double b, double c, int fma) { return fma ? __builtin_fma(a, b, c) : a * b + c; }
LLMI_HD float llmi_expf_glibc(float x, int fma) {
    const uint32_t abstop = (llmi_f2u(x) >> 20) & 0x7ffu;
    if (abstop >= 0x42bu) {                 /* |x| >= 88 or nan (top12(88.0f) = 0x42b) */
        if (llmi_f2u(x) == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8u) return x + x;
        if (x > 88.72283172607421875f) return llmi_u2f(0x7f800000u);   /* 0x1.62e42ep6 */
        if (x < -103.97207641601562f) return 0.0f;                     /* -0x1.9fe368p6 */
    }
    const double InvLn2N = 0x1.71547652b82fep+0 * 32, SHIFT = 0x1.8p+52;
    const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                 C2 = 0x1.62e42ff0c52d6p-1 / 32;
    const double xd = (double)x;
    /* the FMA build contracts every add/sub use of InvLn2N * xd, i.e. both: the
     * rounding to k and r are then taken from the exact product */
    double kd = fma ? __builtin_fma(InvLn2N, xd, SHIFT) : InvLn2N * xd + SHIFT;
    const uint64_t ki = llmi_d2u(kd);
    kd -= SHIFT;
    const double r = fma ? __builtin_fma(InvLn2N, xd, -kd) : InvLn2N * xd - kd;
    double z;
    const uint64_t t = llmi_exp2f_tab((uint32_t)ki) + (ki << 47);
    const double s = llmi_u2d(t);
    z = llmi_fma_d(C0, r, C1, fma);
    const double r2 = r * r;
    double y = llmi_fma_d(C2, r, 1.0, fma);
    y = llmi_fma_d(z, r2, y, fma);
    y = y * s;
    return (float)y;
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
