/*
 * llmi_synth.h — synthetic GGUF tensor contents (SURVEY.md §8d "Synthetic inputs").
 *
 * No real model files exist offline, so every benchmark and parity model is built
 * from this generator: blocks are drawn directly in their quantized form (not via a
 * quantizer), with fp16 block scales chosen so dequantized weights have std ~0.02 and
 * mean ~0, which keeps logits O(1..10) and makes a 1e-3 absolute logit tolerance
 * meaningful.  Byte k of block b of tensor t is a pure function of (seed, t, b, k):
 * the C GGUF writer (host) and any checker reproduce a tensor without the others.
 *
 * Block layouts are the upstream ggml ones:
 *   Q4_K 144 B {f16 d, f16 dmin, u8 scales[12], u8 qs[128]}
 *   Q5_K 176 B {f16 d, f16 dmin, u8 scales[12], u8 qh[32], u8 qs[128]}
 *   Q6_K 210 B {u8 ql[128], u8 qh[64], i8 scales[16], f16 d}
 *   Q8_0  34 B {f16 d, i8 qs[32]}
 */
#ifndef LLMI_SYNTH_H
#define LLMI_SYNTH_H

#include "llmi_math.h"

enum {
    LLMI_T_F32 = 0, LLMI_T_F16 = 1, LLMI_T_Q8_0 = 8, LLMI_T_Q4_K = 12,
    LLMI_T_Q5_K = 13, LLMI_T_Q6_K = 14, LLMI_T_Q8_K = 15
};

/* std-0.02 calibration of the fp16 block scale d (see DESIGN.md §Synthetic models) */
#define LLMI_SYN_D_Q4K 7.74e-5f  /* std(d*sc*q - 7.5*d*m) = 258.3*d */
#define LLMI_SYN_D_Q5K 3.79e-5f  /* std(d*sc*q - 15.5*d*m) = 527.2*d */
#define LLMI_SYN_D_Q6K 2.93e-5f  /* std(d*sc*(q-32)) = 682.9*d */
#define LLMI_SYN_D_Q80 2.73e-4f  /* std(d*q), q uniform in [-127,127] = 73.3*d */

/* Writes one quantized block of `type` (block index `bi` inside tensor `tensor`). */
LLMI_HD void llmi_synth_block(int type, uint64_t seed, uint64_t tensor, uint64_t bi, uint8_t* out) {
    uint64_t base = bi * 64u;  /* <= 33 draws per block */
    /* byte generator: 8 bytes per 64-bit draw */
#define LLMI_SB(k) ((uint8_t)(llmi_rand64(seed, tensor, base + 1u + (uint64_t)(k) / 8u) >> (8u * ((uint64_t)(k) % 8u))))
    float jit = 0.75f + 0.5f * llmi_u01(llmi_rand64(seed, tensor, base));
    if (type == LLMI_T_Q4_K || type == LLMI_T_Q5_K) {
        float d = (type == LLMI_T_Q4_K ? LLMI_SYN_D_Q4K : LLMI_SYN_D_Q5K) * jit;
        float dmin = d * (type == LLMI_T_Q4_K ? 7.5f : 15.5f);
        uint16_t hd = llmi_f2h(d), hm = llmi_f2h(dmin);
        out[0] = (uint8_t)hd; out[1] = (uint8_t)(hd >> 8);
        out[2] = (uint8_t)hm; out[3] = (uint8_t)(hm >> 8);
        int rest = (type == LLMI_T_Q4_K) ? 140 : 172;  /* scales + (qh) + qs: uniform bytes */
        for (int k = 0; k < rest; ++k) out[4 + k] = LLMI_SB(k);
    } else if (type == LLMI_T_Q6_K) {
        for (int k = 0; k < 192; ++k) out[k] = LLMI_SB(k);              /* ql, qh */
        for (int k = 0; k < 16; ++k) out[192 + k] = (uint8_t)(int8_t)((int)(LLMI_SB(192 + k) & 127u) - 64);
        uint16_t hd = llmi_f2h(LLMI_SYN_D_Q6K * jit);
        out[208] = (uint8_t)hd; out[209] = (uint8_t)(hd >> 8);
    } else if (type == LLMI_T_Q8_0) {
        uint16_t hd = llmi_f2h(LLMI_SYN_D_Q80 * jit);
        out[0] = (uint8_t)hd; out[1] = (uint8_t)(hd >> 8);
        for (int k = 0; k < 32; ++k) {
            uint32_t r = (uint32_t)(llmi_rand64(seed, tensor, base + 1u + (uint64_t)k) >> 32);
            out[2 + k] = (uint8_t)(int8_t)((int)(r % 255u) - 127);
        }
    }
#undef LLMI_SB
}

/* Element i of a float tensor: norm weights in [0.9, 1.1) (not exactly 1 so a dropped
 * multiply is visible), other f32/f16 tensors ~U(-0.035, 0.035) (std 0.02). */
LLMI_HD float llmi_synth_f32(uint64_t seed, uint64_t tensor, uint64_t i, int is_norm) {
    float u = llmi_u01(llmi_rand64(seed, tensor, i));
    return is_norm ? 0.9f + 0.2f * u : (u - 0.5f) * 0.0693f;
}

#endif /* LLMI_SYNTH_H */
