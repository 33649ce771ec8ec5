// pf_device.h — the f16-MFMA building blocks of the K-quant GEMMs (prefill.hip.inc
// k_pf_gemm, batch.hip k_bmm): the activation fragment layout, one lane's weights of a
// 256-element stage, and the exact B fragments q * scale (prefill.hip.inc header: why
// every integer sum is exact on the f16 MFMA).
#pragma once
#include "mv_device.h"

namespace llmi {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// f16 MFMA fragments of q8 activations: [T/32][stage][32 entries][32 tokens][8 f16], a
// stage = 256 elements (K-quants: one block, entry = 4 l + g; Q8_0: eight 32-blocks)
__host__ __device__ inline size_t pf_aq_off(int t, int stage, int entry, int nstage) {
    return ((((size_t)(t >> 5) * nstage + stage) * 32 + entry) * 32 + (t & 31)) * 16;
}

// bsum pairs as the A fragments of the sumi MFMA (k_pf_quant's abf): [T/32][stage][4 g]
// [32 tokens][8 f16] = (lo, hi) of pairs 2g, 2g + 1 and four zeros, pair = 64 hi + lo
__host__ __device__ inline size_t pf_abf_off(int t, int stage, int g, int nstage) {
    return ((((size_t)(t >> 5) * nstage + stage) * 4 + g) * 32 + (t & 31)) * 16;
}

// one lane's weights of a stage: row lane & 15, chunk(s) of lane group lane >> 4
template <int T>
struct PfW {
    u32x4 q0, q1;      // K-quants: parts 0, 1 of chunk 4 stage + g
    u32x4 hdr;         // Q4_K/Q5_K block header; Q6_K high bits of the chunk
    u32x2 qh;          // Q5_K fifth bits
    uint32_t sc;       // Q6_K chunk scales
    uint32_t d;        // Q6_K fp16 d
    u32x2 q8[8];       // Q8_0: bytes 8g .. 8g+7 of the stage's eight 32-blocks
    u32x4 dd;          // Q8_0: fp16 d of the stage's eight 32-blocks
};
// Row view for the prefill's per-lane rows: plane bases of one row (common.h unit-major
// planes; part p of unit u at qa + (p U + u) 16)
struct RowPtr {
    const uint8_t* qa;
    const uint8_t* hb;
    uint32_t ps;       // bytes from one part of a row's unit to the next (U * 16 * row group)
    const uint8_t* sb;
    const uint8_t* db;
};
template <int T>
__device__ __forceinline__ RowPtr row_ptr(const Seg& s, int row, int cols) {
    RowPtr r;
    const size_t ru = (size_t)row * (size_t)(cols >> 8);
    const uint32_t U = (uint32_t)(cols >> 8);
    r.ps = (U * 16u) << s.rgs;
    r.qa = s.a + piece_off((uint32_t)row, 0, 0, U, unit_parts<T>(), s.rgs);
    r.hb = s.h + piece_off((uint32_t)row, 0, 0, U, unit_hparts<T>(), s.rgs);
    r.sb = s.s + ru * 16;
    r.db = s.d + ru * (T == T_Q8_0 ? 16 : 2);
    return r;
}
// plain (temporal) loads: a lane reads 16 B of a 128-B line whose other 112 B the next 7
// stages read, so the line should stay in L2 (the decode matvec's nontemporal weights are
// read once)
#ifndef LLMI_PF_NT
#define LLMI_PF_NT 0
#endif
__device__ __forceinline__ u32x4 pf_ld16(const uint8_t* p) {
    if constexpr (LLMI_PF_NT) return ldw(p);
    else return *(const u32x4*)p;
}
__device__ __forceinline__ u32x2 pf_ld8(const uint8_t* p) {
    if constexpr (LLMI_PF_NT) return ldw8(p);
    else return *(const u32x2*)p;
}
__device__ __forceinline__ uint32_t pf_ld4(const uint8_t* p) {
    if constexpr (LLMI_PF_NT) return ldw4(p);
    else return *(const uint32_t*)p;
}
template <int T>
__device__ __forceinline__ PfW<T> pf_w_load(const RowPtr& rp, int stage, int) {
    PfW<T> w;
    const uint32_t g = (threadIdx.x & 63) >> 4, st = (uint32_t)stage;
    if constexpr (T == T_Q8_0) {
        // 32-block l of the stage's unit: parts 2l, 2l + 1; bytes 8g .. 8g+7 are in part
        // 2l + g / 2 at 8 (g % 2)
#pragma unroll
        for (int l = 0; l < 8; ++l)
            w.q8[l] = *(const u32x2*)(rp.qa + (2 * l + (g >> 1)) * rp.ps + st * 16 + 8 * (g & 1));
        w.dd = *(const u32x4*)(rp.db + st * 16);
    } else {
        w.q0 = pf_ld16(rp.qa + (2 * g) * rp.ps + st * 16);
        w.q1 = pf_ld16(rp.qa + (2 * g + 1) * rp.ps + st * 16);
        if constexpr (T == T_Q4_K || T == T_Q5_K) {
            w.hdr = *(const u32x4*)(rp.sb + st * 16);
            if constexpr (T == T_Q5_K) w.qh = pf_ld8(rp.hb + (g >> 1) * rp.ps + st * 16 + 8 * (g & 1));
        } else {
            w.hdr = pf_ld16(rp.hb + g * rp.ps + st * 16);
            w.sc = pf_ld4(rp.sb + st * 16 + 4 * g);
            w.d = *(const uint16_t*)(rp.db + st * 2);
        }
    }
    return w;
}

// f16 pair (1024 + x0, 1024 + x1) of two values 0..255 held in the low bytes of the
// two 16-bit halves of `v` (magic-number conversion, exact)
__device__ __forceinline__ uint32_t pf_magic(uint32_t v) { return v | 0x64006400u; }
__device__ __forceinline__ h2 as_h2(uint32_t v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ s2 as_h2s(uint32_t v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ uint32_t as_u(h2 v) { return __builtin_bit_cast(uint32_t, v); }
// (1024 + x) * s - (1024 + off) * s = (x - off) * s, one rounding of an exact integer
__device__ __forceinline__ uint32_t pf_scale(uint32_t magic_pair, h2 s, h2 off_s) {
    return as_u(__builtin_elementwise_fma(as_h2(magic_pair), s, -off_s));
}

template <int T, int NP>
struct PfB {
    h8 b[NP];  // Q6_K: b[0] = (q-32)*sl, b[1] = (q-32)*sh
};
// B fragments of residue l (K-quants) or 32-block l (Q8_0) for this lane (X86: of x86
// lane l, the weights' x86 byte order: a Q6_K dword = 4 elements of ONE sub-block)
template <int T, int X86 = 0>
__device__ __forceinline__ void pf_build_b(const PfW<T>& w, int l, h2 slo, h2 shi, h2 slo_o, h2 shi_o, const h2* s6,
                                           const h2* s6o, h8* out) {
    if constexpr (T == T_Q8_0) {
        const uint32_t lo = w.q8[l].x, hi = w.q8[l].y;
        uint32_t v[4];
        // signed byte b -> b ^ 0x80 = b + 128 (0..255) -> f16 1024 + b + 128; minus 1152
        const uint32_t xl = lo ^ 0x80808080u, xh = hi ^ 0x80808080u;
        v[0] = __builtin_amdgcn_perm(0u, xl, 0x0c010c00u);
        v[1] = __builtin_amdgcn_perm(0u, xl, 0x0c030c02u);
        v[2] = __builtin_amdgcn_perm(0u, xh, 0x0c010c00u);
        v[3] = __builtin_amdgcn_perm(0u, xh, 0x0c030c02u);
        h8 r;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const h2 x = as_h2(pf_magic(v[k])) - h2{(_Float16)1152.f, (_Float16)1152.f};
            r[2 * k] = x[0];
            r[2 * k + 1] = x[1];
        }
        out[0] = r;
    } else {
        const u32x4 q = (l >> 2) ? w.q1 : w.q0;
        const uint32_t d = q[l & 3];
        // bytes 0..3 -> 16-bit halves: (b0, b1), (b2, b3)
        const uint32_t x01 = __builtin_amdgcn_perm(0u, d, 0x0c010c00u), x23 = __builtin_amdgcn_perm(0u, d, 0x0c030c02u);
        uint32_t lo01 = x01 & 0x000F000Fu, lo23 = x23 & 0x000F000Fu;
        uint32_t hi01 = (x01 >> 4) & 0x000F000Fu, hi23 = (x23 >> 4) & 0x000F000Fu;
        if constexpr (T == T_Q5_K) {  // fifth bits: byte i, bit l of the lo / hi word -> bit 4 of half i % 2
            const uint32_t bl = (w.qh.x >> l) & M1, bh = (w.qh.y >> l) & M1;
            lo01 |= __builtin_amdgcn_perm(0u, bl, 0x0c010c00u) << 4;
            lo23 |= __builtin_amdgcn_perm(0u, bl, 0x0c030c02u) << 4;
            hi01 |= __builtin_amdgcn_perm(0u, bh, 0x0c010c00u) << 4;
            hi23 |= __builtin_amdgcn_perm(0u, bh, 0x0c030c02u) << 4;
        }
        if constexpr (T == T_Q6_K) {  // high 2 bits (stored XOR 2): (h ^ 2) << 4 per byte
            const uint32_t hl = (w.hdr[l >> 2] >> (2 * (l & 3))) & M2, hh = (w.hdr[2 + (l >> 2)] >> (2 * (l & 3))) & M2;
            const uint32_t l01 = __builtin_amdgcn_perm(0u, hl, 0x0c010c00u), l23 = __builtin_amdgcn_perm(0u, hl, 0x0c030c02u);
            const uint32_t h01 = __builtin_amdgcn_perm(0u, hh, 0x0c010c00u), h23 = __builtin_amdgcn_perm(0u, hh, 0x0c030c02u);
            lo01 |= (l01 ^ 0x00020002u) << 4;
            lo23 |= (l23 ^ 0x00020002u) << 4;
            hi01 |= (h01 ^ 0x00020002u) << 4;
            hi23 |= (h23 ^ 0x00020002u) << 4;
            // pairs: (lo01) sub-block 4g, (lo23) 4g+1, (hi01) 4g+2, (hi23) 4g+3
            // (X86: lo01 and lo23 sub-block 4g + l/4, hi01 and hi23 4g + 2 + l/4)
            const uint32_t m[4] = {pf_magic(lo01), pf_magic(lo23), pf_magic(hi01), pf_magic(hi23)};
#pragma unroll
            for (int part = 0; part < 2; ++part) {
                h8 r;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int sbk = X86 ? (k >> 1) * 2 + (l >> 2) : k;
                    const h2 x = as_h2(pf_scale(m[k], s6[2 * sbk + part], s6o[2 * sbk + part]));
                    r[2 * k] = x[0];  // fragment order: j = 4h + i
                    r[2 * k + 1] = x[1];
                }
                out[part] = r;
            }
            return;
        }
        // j = 0..3: low nibbles i = 0..3 (x01: i = 0, 1 in its halves; x23: i = 2, 3)
        const h2 a = as_h2(pf_scale(pf_magic(lo01), slo, slo_o)), b = as_h2(pf_scale(pf_magic(lo23), slo, slo_o));
        const h2 c = as_h2(pf_scale(pf_magic(hi01), shi, shi_o)), e = as_h2(pf_scale(pf_magic(hi23), shi, shi_o));
        out[0] = h8{a[0], a[1], b[0], b[1], c[0], c[1], e[0], e[1]};
    }
}

}  // namespace llmi
