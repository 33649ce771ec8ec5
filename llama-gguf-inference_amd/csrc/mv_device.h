// mv_device.h — device helpers of the quantized matvec shared by the single-token
// (kernels.hip), batched (batch.hip) and prefill kernels: cross-lane exchange, the
// activation prologue (RMSNorm + q8_K / q8_0 quantization, bit-exact with ggml), the
// chunk-planar weight loads, the per-chunk integer sums and ggml's generic fp32 order
// (the fold), row-pair bookkeeping, the epilogues and the attention bodies.  Everything
// here is __device__ inline.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"
#include "../../include/llmi_math.h"

namespace llmi {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef short short2_t __attribute__((ext_vector_type(2)));

// Weight loads are nontemporal (nt): every weight byte is read once per token by one
// CU, so keeping it in L2/MALL only evicts the activations and KV.  Measured with the
// statically counted prologue (tools/mvbench.py, graph-replayed): 2-10 % faster on
// every shape (output 128256x4096 Q6_K: 78.8 -> 70.8 us); end to end 555 -> 581 tok/s.
// (Before the prologue stopped waiting on vmcnt(0), nt measured slower.)
#ifndef LLMI_NT
#define LLMI_NT 1
#endif
constexpr bool kNontemporalWeights = LLMI_NT != 0;

__device__ __forceinline__ float h2f(uint32_t h) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(h & 0xffffu));
}
// f32 -> f16 with its own rounding.  The empty asm makes the f32 value opaque: without
// it the compiler folds f2h(a * b) into v_fma_mixlo_f16, ONE rounding of the exact
// product straight to f16, where ggml rounds to f32 first and then to f16 (a tie in
// the f32 product then rounds differently: softmax probabilities left the oracle by one
// f16 ulp, experiments/pf_diag9.py).
__device__ __forceinline__ uint16_t f2h(float f) {
    __asm__("" : "+v"(f));
    return __builtin_bit_cast(uint16_t, (_Float16)f);
}

__device__ __forceinline__ u32x4 ldw(const uint8_t* p) {
    if constexpr (kNontemporalWeights) return __builtin_nontemporal_load((const u32x4*)p);
    else return *(const u32x4*)p;
}
__device__ __forceinline__ u32x2 ldw8(const uint8_t* p) {
    if constexpr (kNontemporalWeights) return __builtin_nontemporal_load((const u32x2*)p);
    else return *(const u32x2*)p;
}
__device__ __forceinline__ uint32_t ldw4(const uint8_t* p) {
    if constexpr (kNontemporalWeights) return __builtin_nontemporal_load((const uint32_t*)p);
    else return *(const uint32_t*)p;
}
__device__ __forceinline__ int dot4(uint32_t a, int b, int c) {
    return __builtin_amdgcn_sdot4((int)a, b, c, false);
}
// ---- cross-lane exchange without LDS round trips (VALU latency): DPP within 16-lane
// rows, v_permlane16/32_swap across rows / halves (gfx950).  xor_partner<o>(v) returns
// v of lane L^o for o in {1,2,4,8,16,32}; for o = 4 / 8 the DPP row_half_mirror /
// row_mirror partner (lane 7-i / 15-i) is used, which equals lane L^4 / L^8 whenever
// the value is already uniform over aligned 4- / 8-lane groups, i.e. inside a
// butterfly after the xor-1/xor-2 (and xor-4) steps.  Every butterfly below runs the
// steps in the order 1, 2, 4, 8, 16, 32 (used only where the result is exact in any order:
// integer sums, max / min keys, double sums that absorb the reordering -- DESIGN.md §5).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int O>
__device__ __forceinline__ uint32_t xor_partner_u32(uint32_t v) {
    if constexpr (O == 1) return dpp_u32<0xB1>(v);        // quad_perm [1,0,3,2]
    else if constexpr (O == 2) return dpp_u32<0x4E>(v);   // quad_perm [2,3,0,1]
    else if constexpr (O == 4) return dpp_u32<0x141>(v);  // row_half_mirror
    else if constexpr (O == 8) return dpp_u32<0x140>(v);  // row_mirror
    else if constexpr (O == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return ((threadIdx.x >> 4) & 1) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return ((threadIdx.x >> 5) & 1) ? r[0] : r[1];
    }
}
template <int O>
__device__ __forceinline__ float xor_partner(float v) { return __uint_as_float(xor_partner_u32<O>(__float_as_uint(v))); }
template <int O>
__device__ __forceinline__ int xor_partner_i(int v) { return (int)xor_partner_u32<O>((uint32_t)v); }
template <int O>
__device__ __forceinline__ double xor_partner_d(double v) {
    const unsigned long long u = __double_as_longlong(v);
    const uint32_t lo = xor_partner_u32<O>((uint32_t)u), hi = xor_partner_u32<O>((uint32_t)(u >> 32));
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
// 64-lane sum, all lanes receive the result (butterfly 1,2,4,8,16,32)
__device__ __forceinline__ float wave_sum(float v) {
    v += xor_partner<1>(v);
    v += xor_partner<2>(v);
    v += xor_partner<4>(v);
    v += xor_partner<8>(v);
    v += xor_partner<16>(v);
    v += xor_partner<32>(v);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
    v += xor_partner_d<1>(v);
    v += xor_partner_d<2>(v);
    v += xor_partner_d<4>(v);
    v += xor_partner_d<8>(v);
    v += xor_partner_d<16>(v);
    v += xor_partner_d<32>(v);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, xor_partner<1>(v));
    v = fmaxf(v, xor_partner<2>(v));
    v = fmaxf(v, xor_partner<4>(v));
    v = fmaxf(v, xor_partner<8>(v));
    v = fmaxf(v, xor_partner<16>(v));
    v = fmaxf(v, xor_partner<32>(v));
    return v;
}
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ----------------------------------------------------------------------------------
// LDS image of the quantized activation: one kRec-byte RECORD per 256-element unit
// (the weights' unit, common.h), in the weights' part order:
//   K-quants (block_q8_K):  [32 p, 32 p + 16)       LO: activation of the low nibbles
//                           [32 p + 16, 32 p + 32)  HI: ... of the high nibbles of part p
//                           (residue order: byte 4m + i of LO = chunk element l + 8i,
//                           of HI = 32 + l + 8i, chunk c = p / 2, l = 4 (p % 2) + m)
//                           [256, 288) bsums int16[16], [288, 292) d
//   Q8_0 (block_q8_0):      [16 p, 16 p + 16) elements 16 p .. +15 (natural order),
//                           [256, 288) d of the eight 32-blocks (f32 of the f16 value)
// A lane reads the record of its own unit: the stride of 19 x 16 B (odd) puts the 16
// lanes of a ds_read_b128 bank group on 16 distinct 16-B bank quads (conflict-free).
// ----------------------------------------------------------------------------------
constexpr int kRec = 304, kRecBs = 256, kRecD = 288;
struct Lds {
    uint8_t* act;
    double* red;
};
__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline size_t lds_red_off(int act, int cols) { return (size_t)(cols >> 8) * kRec; }
// offset of the per-wave fold buffers in a matvec workgroup's LDS (after the activation
// image and the prologue's reduction slots); mv_lds_bytes: kernels.hip
__host__ __device__ inline size_t fold_off(int act, int cols, int waves) {
    return a16(lds_red_off(act, cols) + (size_t)waves * sizeof(double));
}

__device__ __forceinline__ Lds carve(uint8_t* smem, int act, int cols) {
    Lds l;
    l.act = smem;
    l.red = (double*)(smem + lds_red_off(act, cols));
    return l;
}

// workgroup double sum of a matvec workgroup (NW waves; pairwise tree over waves)
template <int NW = kMVWaves>
__device__ double block_sum_d(double v, double* red) {
    v = wave_sum_d(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) r[w] = red[w];
#pragma unroll
    for (int o = 1; o < NW; o <<= 1)
#pragma unroll
        for (int w = 0; w + o < NW; w += 2 * o) r[w] = r[w] + r[w + o];
    return r[0];
}

// ----------------------------------------------------------------------------------
// Prologue: [RMSNorm] + activation quantization into LDS.
// Thread t handles 16-element sub-blocks sb = t + 256k; the 16 lanes of one DPP row
// hold the 16 sub-blocks of one 256-element Q8_K block, two adjacent lanes one Q8_0
// block.  Bit-exact with ggml:
//   rms_norm: sum += (double)(x*x); mean = (float)(sum/n); scale = 1/sqrtf(mean+eps);
//             y = (x*scale)*w                          (ggml_compute_forward_rms_norm + mul)
//   q8_K:     first max |y| (signed) -> iscale = -127/max; q = min(127, nearest_int(iscale*y));
//             bsums per 16; d = 1/iscale; all-zero block -> d = 0, q = 0 (quantize_row_q8_K_ref)
//   q8_0:     d = amax/127 (stored f16), q = roundf(y * (d ? 1/d : 0))   (quantize_row_q8_0_ref)
// ----------------------------------------------------------------------------------
// Quantize one 16-element sub-block (values already normed) into the LDS image.
//   X86 = 1 (the x86 association mode, "x86 numerics" below): K-quant records hold the
//   block in NATURAL order (part 2c + k, half h = elements 64c + 32h + 16k .. +15), the
//   weights' x86 layout (common.h); q8_0 is upstream's AVX2 quantize_row_q8_0:
//   id = 127/amax, q = round-half-even(y * id) (oracle x86_quantize_row_q8_0).
template <int ACT, int X86 = 0>
__device__ __forceinline__ void quant_sub(const Lds& L, int cols, int sb, const float (&v)[16]) {
    int q[16];
    if constexpr (ACT == 0) {
        // max |y| of the Q8_K block (order-free), then the SIGNED value ggml keeps: the
        // first element (lowest index) whose |y| equals it ('if (ax > amax)' scan).  Key =
        // (index within the block) * 2 + sign, minimised over the 16 lanes of the block.
        float am = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[j]));
        am = fmaxf(am, xor_partner<1>(am));
        am = fmaxf(am, xor_partner<2>(am));
        am = fmaxf(am, xor_partner<4>(am));
        am = fmaxf(am, xor_partner<8>(am));
        int key = 0x7fffffff;
#pragma unroll
        for (int j = 15; j >= 0; --j)
            key = fabsf(v[j]) == am ? (((sb & 15) * 16 + j) << 1) | (v[j] < 0.f ? 1 : 0) : key;
        key = min(key, xor_partner_i<1>(key));
        key = min(key, xor_partner_i<2>(key));
        key = min(key, xor_partner_i<4>(key));
        key = min(key, xor_partner_i<8>(key));
        const float mv = (key & 1) ? -am : am;
        float dval = 0.f;
        int bsum = 0;
        if (am == 0.f) {
#pragma unroll
            for (int j = 0; j < 16; ++j) q[j] = 0;
        } else {
            const float iscale = -127.f / mv;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int t = llmi_nearest_int(iscale * v[j]);
                q[j] = t < 127 ? t : 127;
                bsum += q[j];
            }
            dval = 1.0f / iscale;
        }
        // sub-block sb = unit u, 16-element piece s = 4c + 2h + half of chunk c, half
        // h (LO / HI): elements tt = 16 half + j of the half sit at part 2c + l/4, byte
        // 4 (l%4) + i with l = tt%8 = j%8, i = tt/8 = 2 half + j/8 (residue order), so
        // q[j] and q[j+8] are one 16-bit store
        const int s = sb & 15;
        uint8_t* rec = L.act + (size_t)(sb >> 4) * kRec;
        if constexpr (X86) {  // s = 4c + 2h + k: part 2c + k, half h, bytes 0..15 in order
            u32x4 pk;
#pragma unroll
            for (int w = 0; w < 4; ++w)
                pk[w] = (uint32_t)(q[4 * w] & 0xff) | ((uint32_t)(q[4 * w + 1] & 0xff) << 8) |
                        ((uint32_t)(q[4 * w + 2] & 0xff) << 16) | ((uint32_t)(q[4 * w + 3] & 0xff) << 24);
            *(u32x4*)(rec + 64 * (s >> 2) + 32 * (s & 1) + 16 * ((s >> 1) & 1)) = pk;
        } else {
            uint8_t* base = rec + 64 * (s >> 2) + 16 * ((s >> 1) & 1) + 2 * (s & 1);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                *(uint16_t*)(base + 32 * (j >> 2) + 4 * (j & 3)) = (uint16_t)((q[j] & 0xff) | ((q[j + 8] & 0xff) << 8));
        }
        *(int16_t*)(rec + kRecBs + 2 * s) = (int16_t)bsum;
        if (s == 0) *(float*)(rec + kRecD) = dval;
    } else {
        float am = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[j]));
        am = fmaxf(am, xor_partner<1>(am));
        const float d = am / 127;
        if constexpr (X86) {
            const float id = am != 0.f ? 127.f / am : 0.0f;
#pragma unroll
            for (int j = 0; j < 16; ++j) q[j] = (int)__builtin_rintf(v[j] * id);
        } else {
            const float id = d != 0.f ? 1.0f / d : 0.0f;
#pragma unroll
            for (int j = 0; j < 16; ++j) q[j] = (int)roundf(v[j] * id);
        }
        uint8_t* rec = L.act + (size_t)(sb >> 4) * kRec;
        if ((sb & 1) == 0) *(float*)(rec + kRecBs + 2 * (sb & 15)) = h2f(f2h(d));
        u32x4 pk;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            pk[w] = (uint32_t)(q[4 * w] & 0xff) | ((uint32_t)(q[4 * w + 1] & 0xff) << 8) |
                    ((uint32_t)(q[4 * w + 2] & 0xff) << 16) | ((uint32_t)(q[4 * w + 3] & 0xff) << 24);
        *(u32x4*)(rec + 16 * (sb & 15)) = pk;
    }
}

// Prologue in two halves so a caller can put the weight prefetch between them:
// issue() loads this thread's first NP sub-blocks of x (and norm w) into registers —
// UNCONDITIONALLY (indices clamped), so the load count is static and the first use
// waits with vmcnt(#weight loads issued after them) instead of vmcnt(0), i.e. the
// prologue never waits for the weight prefetch; finish() computes the norm,
// quantizes and writes LDS.  NP = ceil(cols / (16 * kMVThreads)) rounded up to 1/2/4
// (chosen at launch); sub-blocks beyond NP are loaded inside finish().
template <bool NORM, int NP>
struct ProRegs {
    float x[NP][16];
    float w[NORM ? NP : 1][16];
};
template <bool NORM, int NP, int NT = kMVThreads>
__device__ __forceinline__ void mv_prologue_issue(const MVArgs& A, ProRegs<NORM, NP>& R) {
    const int nsub = A.cols / 16;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int sb = min((int)threadIdx.x + i * NT, nsub - 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 xv = *(const float4*)(A.x + sb * 16 + 4 * k);
            R.x[i][4 * k + 0] = xv.x; R.x[i][4 * k + 1] = xv.y; R.x[i][4 * k + 2] = xv.z; R.x[i][4 * k + 3] = xv.w;
            if constexpr (NORM) {
                const float4 wv = *(const float4*)(A.nw + sb * 16 + 4 * k);
                R.w[i][4 * k + 0] = wv.x; R.w[i][4 * k + 1] = wv.y; R.w[i][4 * k + 2] = wv.z; R.w[i][4 * k + 3] = wv.w;
            }
        }
    }
}
template <bool NORM, int NP>
__device__ __forceinline__ void load_sub(const MVArgs& A, const ProRegs<NORM, NP>& R, int i, int sb, float (&v)[16],
                                         float (&w)[16]) {
    if (i < NP) {
#pragma unroll
        for (int ii = 0; ii < NP; ++ii)
            if (ii == i) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    v[j] = R.x[ii][j];
                    if constexpr (NORM) w[j] = R.w[ii][j];
                }
            }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 xv = *(const float4*)(A.x + sb * 16 + 4 * k);
            v[4 * k + 0] = xv.x; v[4 * k + 1] = xv.y; v[4 * k + 2] = xv.z; v[4 * k + 3] = xv.w;
            if constexpr (NORM) {
                const float4 wv = *(const float4*)(A.nw + sb * 16 + 4 * k);
                w[4 * k + 0] = wv.x; w[4 * k + 1] = wv.y; w[4 * k + 2] = wv.z; w[4 * k + 3] = wv.w;
            }
        }
    }
}
// RMSNorm scale of the row (1 without NORM): per-thread double sums over sub-blocks tid,
// tid + NT, ... then the block reduction (every caller the same order, so the same bits)
template <bool NORM, int NP, int NT = kMVThreads>
__device__ __forceinline__ float mv_norm_scale(const MVArgs& A, const Lds& L, const ProRegs<NORM, NP>& R) {
    const int tid = threadIdx.x, cols = A.cols;
    const int nsub = cols / 16;
    float scale = 1.0f;
    if constexpr (NORM) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NP; ++i)  // register-held sub-blocks (static indices)
            if (tid + i * NT < nsub) {
#pragma unroll
                for (int j = 0; j < 16; ++j) s += (double)(R.x[i][j] * R.x[i][j]);
            }
        for (int sb = tid + NP * NT; sb < nsub; sb += NT) {  // rest (cols > NP*16*threads)
            float v[16], w[16];
            load_sub<NORM, NP>(A, R, NP, sb, v, w);
#pragma unroll
            for (int j = 0; j < 16; ++j) s += (double)(v[j] * v[j]);
        }
        s = block_sum_d<NT / 64>(s, L.red);
        const float mean = (float)(s / (double)cols);
        scale = 1.0f / sqrtf(mean + A.eps);
    }
    return scale;
}
template <int ACT, bool NORM, int NP, int NT = kMVThreads, int X86 = 0>
__device__ __forceinline__ void mv_prologue_finish(const MVArgs& A, const Lds& L, const ProRegs<NORM, NP>& R) {
    const int tid = threadIdx.x, cols = A.cols;
    const int nsub = cols / 16;
    const float scale = mv_norm_scale<NORM, NP, NT>(A, L, R);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int sb = tid + i * NT;
        if (sb < nsub) {
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                v[j] = R.x[i][j];
                if constexpr (NORM) v[j] = (v[j] * scale) * R.w[i][j];
            }
            quant_sub<ACT, X86>(L, cols, sb, v);
        }
    }
    for (int sb = tid + NP * NT; sb < nsub; sb += NT) {
        float v[16], w[16];
        load_sub<NORM, NP>(A, R, NP, sb, v, w);
        if constexpr (NORM) {
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = (v[j] * scale) * w[j];
        }
        quant_sub<ACT, X86>(L, cols, sb, v);
    }
}
// Pre-quantized activation (MVArgs::xq): the LDS image is copied from global memory.
// NI 16-B pieces per thread, loaded unconditionally (clamped) like the x loads above.
template <int NI>
struct ImgRegs {
    u32x4 v[NI];
};
template <int NI, int NT = kMVThreads>
__device__ __forceinline__ void mv_img_issue(const MVArgs& A, ImgRegs<NI>& R) {
    const int n16 = (A.cols >> 8) * (kRec / 16);
#pragma unroll
    for (int i = 0; i < NI; ++i) R.v[i] = *(const u32x4*)(A.xq + 16 * min((int)threadIdx.x + i * NT, n16 - 1));
}
template <int NI, int NT = kMVThreads>
__device__ __forceinline__ void mv_img_finish(const MVArgs& A, const Lds& L, const ImgRegs<NI>& R) {
    const int n16 = (A.cols >> 8) * (kRec / 16);
#pragma unroll
    for (int i = 0; i < NI; ++i)
        if ((int)threadIdx.x + i * NT < n16) ((u32x4*)L.act)[threadIdx.x + i * NT] = R.v[i];
    for (int i = (int)threadIdx.x + NI * NT; i < n16; i += NT) ((u32x4*)L.act)[i] = *(const u32x4*)(A.xq + 16 * i);
}

template <int ACT, bool NORM, int X86 = 0>
__device__ __forceinline__ void mv_prologue(const MVArgs& A, const Lds& L) {
    ProRegs<NORM, 1> R;
    mv_prologue_issue<NORM, 1>(A, R);
    mv_prologue_finish<ACT, NORM, 1, kMVThreads, X86>(A, L, R);
}

// ----------------------------------------------------------------------------------
// One lane's 256-weight unit of one row: load (global) and ggml's generic block terms
// ----------------------------------------------------------------------------------
constexpr uint32_t M4 = 0x0F0F0F0Fu, M2 = 0x03030303u, M1 = 0x01010101u;

// upstream get_scale_min_k4 on the 12 scale bytes held as three words (branchless:
// j varies per lane, so both forms are computed and selected)
__device__ __forceinline__ void scale_min(int j, uint32_t s0, uint32_t s1, uint32_t s2, int& sc, int& m) {
    const int k = (j & 3) * 8;
    const uint32_t b0 = (s0 >> k) & 0xffu, b1 = (s1 >> k) & 0xffu, b2 = (s2 >> k) & 0xffu;
    const uint32_t sc_hi = (b2 & 0xFu) | ((b0 >> 6) << 4), m_hi = (b2 >> 4) | ((b1 >> 6) << 4);
    sc = (int)(j < 4 ? (b0 & 63u) : sc_hi);
    m = (int)(j < 4 ? (b1 & 63u) : m_hi);
}
// the eight 6-bit scales / mins of a K-quant header as bytes: sc_j = byte j%4 of
// (j < 4 ? sc.x : sc.y), likewise the mins (get_scale_min_k4 for all j at once)
__device__ __forceinline__ void scales_mins(uint32_t s0, uint32_t s1, uint32_t s2, u32x2& sc, u32x2& mn) {
    sc.x = s0 & 0x3F3F3F3Fu;
    mn.x = s1 & 0x3F3F3F3Fu;
    sc.y = (s2 & M4) | ((s0 >> 2) & 0x30303030u);
    mn.y = ((s2 >> 4) & M4) | ((s1 >> 2) & 0x30303030u);
}
// 4 bits -> the low bit of 4 bytes
__device__ __forceinline__ uint32_t spread4(uint32_t x) { return (x * 0x00204081u) & M1; }

struct PairSum {
    float a, b;
};

// LDS accesses of one wave handed between its own lanes: LDS executes a wave's
// instructions in order, so only the compiler must not move accesses across this point
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// Q6_K high bits are stored XOR 2 (common.h): v_perm maps them straight to the signed
// high part of q - 32 ({0x00, 0x10, 0xE0, 0xF0} for stored 0..3)
__device__ __forceinline__ uint32_t q6_hi_bytes(uint32_t sel) { return __builtin_amdgcn_perm(0xF0E01000u, 0xF0E01000u, sel); }

template <int T>
__host__ __device__ constexpr int unit_parts() { return T == T_Q8_0 ? 16 : 8; }
template <int T>
__host__ __device__ constexpr int unit_hparts() { return T == T_Q6_K ? 4 : T == T_Q5_K ? 2 : 1; }
// plane bytes per unit (row strides are U times these)
template <int T>
__host__ __device__ constexpr uint32_t unit_abytes() { return T == T_Q8_0 ? 256u : 128u; }

// byte offset of 16-B piece (row, part p, unit u) of an A / H plane with np parts per
// unit, rows in groups of 2^rgs (common.h ROW GROUPS)
__host__ __device__ __forceinline__ uint32_t piece_off(uint32_t row, uint32_t p, uint32_t u, uint32_t U, uint32_t np,
                                                       int rgs) {
    const uint32_t g = row >> rgs, r = row & ((1u << rgs) - 1u);
    return ((((g * np + p) << rgs) + r) * U + u) * 16u;
}

template <int T>
struct UnitW {
    u32x4 q[unit_parts<T>()];   // quant parts
    u32x4 s;                    // Q4_K/Q5_K header; Q6_K 16 scales; Q8_0 eight fp16 d
    u32x4 h[unit_hparts<T>()];  // Q5_K fifth bits (2 x 16 B); Q6_K 2-bit highs (4 x 16 B)
    uint32_t d;                 // Q6_K fp16 d
};

// Unit u of row `row` of a segment.  Loads are unconditional (callers clamp row and
// unit into the matrix and discard the terms of invalid lanes): straight-line code lets
// the compiler count vmcnt exactly, so the next unit's loads stay in flight while this
// one is reduced.  Offsets are 32-bit from the segment's (uniform) plane bases.
template <int T>
__device__ __forceinline__ UnitW<T> load_unit(const Seg& sg, uint32_t row, uint32_t u, uint32_t U) {
    UnitW<T> w;
    const uint32_t P = (U * 16) << sg.rgs, ru = row * U + u;
    const uint32_t oa = piece_off(row, 0, u, U, unit_parts<T>(), sg.rgs);
#pragma unroll
    for (int p = 0; p < unit_parts<T>(); ++p) w.q[p] = ldw(sg.a + oa + (uint32_t)p * P);
    if constexpr (T == T_Q8_0) {
        w.s = ldw(sg.d + ru * 16);
    } else {
        w.s = ldw(sg.s + ru * 16);
        if constexpr (T == T_Q5_K || T == T_Q6_K) {
            const uint32_t oh = piece_off(row, 0, u, U, unit_hparts<T>(), sg.rgs);
#pragma unroll
            for (int c = 0; c < unit_hparts<T>(); ++c) w.h[c] = ldw(sg.h + oh + (uint32_t)c * P);
        }
        if constexpr (T == T_Q6_K) w.d = *(const uint16_t*)(sg.d + ru * 2);
    }
    return w;
}

// ----------------------------------------------------------------------------------
// ggml's generic fp32 order (oracle/ggml_oracle.c vd_q4_K/vd_q5_K/vd_q6_K,
// vd_q8_0, restating upstream ggml_vec_dot_*_generic).  Per row:
//   K-quants: for each 256-block b in order
//       aux32[l] = sum over the block's elements e with e % 8 == l of scale(e)*q(e)*a(e)
//       sums[l] += (d_w(b) * d_a(b)) * (float)aux32[l]       (8 fp32 chains, l = 0..7)
//       sumf    -= (dmin_w(b) * d_a(b)) * (float)sumi(b)     (Q4_K/Q5_K; sumi = min terms)
//     then sumf += sums[0]; ... sumf += sums[7]
//   Q8_0:     sumf += (float)sumi(b) * (d_w(b) * d_a(b)) per 32-block b in order
// Integer sums are exact in any grouping; the fp32 operations run exactly in this order.
//
// Device mapping.  A lane owns one unit (= one K-quant block) of one row, so a block's
// integer sums never leave the lane:
//   unit_terms  the residue-order layout makes every sdot4 a same-residue dot:
//               aux32[l] = sum over chunks of sc_lo * dot(LO) + sc_hi * dot(HI); the
//               block's fp32 terms d*(float)aux32[l] and -(dmin*(float)sumi) (Q8_0: the
//               eight 32-block terms) go to the wave's fold buffer F[row][chain][unit]
//   fold        fold lane f = (row, chain) adds its chain's terms unit after unit (the
//               blocks in order) onto its running fp32 chain
//   final       sumf chain + sums[0..7] in order, one lane per row
// ----------------------------------------------------------------------------------
template <int T>
__host__ __device__ constexpr int unit_chains() { return T == T_Q8_0 ? 8 : 9; }  // terms per unit
template <int ACT>
__host__ __device__ constexpr int row_chains() { return ACT ? 1 : 9; }            // fp32 chains per row

// The unit's terms against activation record `rec` (kRec layout): K-quants tm[l] =
// d*(float)aux32[l] (l < 8), tm[8] = -(dmin*(float)sumi) (Q6_K: +0, there is no min
// chain and sumf starts at 0); Q8_0 tm[b] = (float)sumi_b * (d_w * d_a), b < 8.
template <int T>
__device__ __forceinline__ void unit_terms(const UnitW<T>& w, const uint8_t* rec, float (&tm)[9]) {
#if defined(LLMI_EXP_NOVALU)
    // experiment builds only: the unit's integer work replaced by an XOR of its words (loads
    // kept live, results garbage) -- what the launch costs without the per-weight VALU
    if constexpr (T == T_Q4_K) {
        uint32_t x = w.s.x ^ w.s.y ^ w.s.z ^ w.s.w;
#pragma unroll
        for (int p = 0; p < 8; ++p) x ^= w.q[p][0] ^ w.q[p][1] ^ w.q[p][2] ^ w.q[p][3];
        const float da = *(const float*)(rec + kRecD);
#pragma unroll
        for (int l = 0; l < 9; ++l) tm[l] = da * (float)(int)(x >> l);
        return;
    }
#endif
    if constexpr (T == T_Q4_K || T == T_Q5_K) {
        u32x2 sc, mn;
        scales_mins(w.s.y, w.s.z, w.s.w, sc, mn);
        int t[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) t[l] = 0;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int c = p >> 1, k = p & 1;
            // sub-blocks 2c (low nibbles) and 2c + 1 (high nibbles)
            const uint32_t sw = c < 2 ? sc.x : sc.y;
            const int slo = (int)((sw >> (16 * (c & 1))) & 0xffu), shi = (int)((sw >> (16 * (c & 1) + 8)) & 0xffu);
            const i32x4 alo = *(const i32x4*)(rec + 32 * p), ahi = *(const i32x4*)(rec + 32 * p + 16);
            uint32_t hlo = 0, hhi = 0;
            if constexpr (T == T_Q5_K) {  // fifth bits of chunk c: byte i, bit l of the lo / hi word
                hlo = w.h[c >> 1][2 * (c & 1)];
                hhi = w.h[c >> 1][2 * (c & 1) + 1];
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int l = 4 * k + m;
                uint32_t l4 = w.q[p][m] & M4, h4 = (w.q[p][m] >> 4) & M4;
                if constexpr (T == T_Q5_K) {
                    l4 |= (l <= 4 ? hlo << (4 - l) : hlo >> (l - 4)) & 0x10101010u;
                    h4 |= (l <= 4 ? hhi << (4 - l) : hhi >> (l - 4)) & 0x10101010u;
                }
                // |dot| <= 4*31*127, scales <= 63: exact 24-bit multiplies
                t[l] = __mul24(slo, dot4(l4, alo[m], 0)) + t[l];
                t[l] = __mul24(shi, dot4(h4, ahi[m], 0)) + t[l];
            }
        }
        // sumi = sum_j m_j * (bs[2j] + bs[2j+1]): int16 pairs against (m_j, m_j)
        const i32x4 b0 = *(const i32x4*)(rec + kRecBs), b1 = *(const i32x4*)(rec + kRecBs + 16);
        int sumi = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t sel = 0x0c000c00u | (uint32_t)(j & 3) * 0x00010001u;
            const uint32_t mm = __builtin_amdgcn_perm(0u, j < 4 ? mn.x : mn.y, sel);
            const int bp = j < 4 ? b0[j] : b1[j - 4];
            sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, bp), __builtin_bit_cast(short2_t, mm), sumi, false);
        }
        const float da = *(const float*)(rec + kRecD);
        const float d = h2f(w.s.x) * da, dm = h2f(w.s.x >> 16) * da;
#pragma unroll
        for (int l = 0; l < 8; ++l) tm[l] = d * (float)t[l];
        tm[8] = -(dm * (float)sumi);
    } else if constexpr (T == T_Q6_K) {
        int t[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) t[l] = 0;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int c = p >> 1, k = p & 1;
            // sub-blocks 4c + 2h + (i >= 2): bytes 0,1 of a dword are elements l, l+8,
            // bytes 2,3 are l+16, l+24 -> one masked sdot4 per sub-block
            const uint32_t s4 = w.s[c];
            const int c0 = (int)(int8_t)(s4 & 0xff), c1 = (int)(int8_t)((s4 >> 8) & 0xff),
                      c2 = (int)(int8_t)((s4 >> 16) & 0xff), c3 = (int)(int8_t)(s4 >> 24);
            const i32x4 alo = *(const i32x4*)(rec + 32 * p), ahi = *(const i32x4*)(rec + 32 * p + 16);
            const uint32_t hl = w.h[c][k], hh = w.h[c][2 + k];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t q = w.q[p][m];
                const uint32_t wl = (q & M4) | q6_hi_bytes((hl >> (2 * m)) & M2);
                const uint32_t wh = ((q >> 4) & M4) | q6_hi_bytes((hh >> (2 * m)) & M2);
                // |s| <= 2*32*127, |c| <= 128: exact in 24-bit multiplies
                int a = t[4 * k + m];
                a = __mul24(c0, dot4(wl, alo[m] & 0xffff, 0)) + a;
                a = __mul24(c1, dot4(wl, alo[m] & (int)0xffff0000u, 0)) + a;
                a = __mul24(c2, dot4(wh, ahi[m] & 0xffff, 0)) + a;
                a = __mul24(c3, dot4(wh, ahi[m] & (int)0xffff0000u, 0)) + a;
                t[4 * k + m] = a;
            }
        }
        const float d = h2f(w.d) * *(const float*)(rec + kRecD);
#pragma unroll
        for (int l = 0; l < 8; ++l) tm[l] = d * (float)t[l];
        tm[8] = 0.f;
    } else {
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const i32x4 a0 = *(const i32x4*)(rec + 32 * b), a1 = *(const i32x4*)(rec + 32 * b + 16);
            int si = 0;
#pragma unroll
            for (int m = 0; m < 4; ++m) si = dot4(w.q[2 * b][m], a0[m], si);
#pragma unroll
            for (int m = 0; m < 4; ++m) si = dot4(w.q[2 * b + 1][m], a1[m], si);
            const float dw = h2f(w.s[b >> 1] >> (16 * (b & 1))), da = *(const float*)(rec + kRecBs + 4 * b);
            tm[b] = (float)si * (dw * da);
        }
        tm[8] = 0.f;
    }
}

// Q6_K with the activation pre-masked (k_matvec's pipelined Q6_K path): a Q6_K dword holds
// bytes of two sub-blocks (elements l, l+8 | l+16, l+24), so each sdot4 needs the
// activation with the other sub-block's two bytes zeroed -- 128 v_and per unit in
// unit_terms<T_Q6_K>.  The workgroup builds both masked copies of its image once
// (q6_masks_build) and reads them instead: per unit 8 parts x {lo & 0x0000ffff,
// lo & 0xffff0000, hi & 0x0000ffff, hi & 0xffff0000} x 16 B.  Same integer sums, same
// fp32 terms: bit-identical.
// bytes of masked activation per unit: 8 parts x 64 B, padded to 33 x 16 B so that the 16
// lanes of a ds_read_b128 group (16 consecutive units) hit 16 distinct bank quads (an odd
// stride in 16-B units, as kRec's 19)
constexpr int kQ6MaskRec = 8 * 64 + 16;
template <int NT>
__device__ __forceinline__ void q6_masks_build(const Lds& L, int U, uint8_t* mbase) {
    for (int i = threadIdx.x; i < U * 64; i += NT) {  // dword i: unit i / 64, part (i % 64) / 8, word i % 8
        const int u = i >> 6, p = (i >> 3) & 7, wd = i & 7;  // wd < 4: LO words, else HI
        const uint32_t v = *(const uint32_t*)(L.act + (size_t)u * kRec + 32 * p + 4 * wd);
        uint8_t* m = mbase + (size_t)u * kQ6MaskRec + 64 * p + 32 * (wd >> 2) + 4 * (wd & 3);
        *(uint32_t*)m = v & 0x0000ffffu;
        *(uint32_t*)(m + 16) = v & 0xffff0000u;
    }
}
__device__ __forceinline__ void unit_terms_q6m(const UnitW<T_Q6_K>& w, const uint8_t* mrec, float da, float (&tm)[9]) {
    int t[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) t[l] = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const int c = p >> 1, k = p & 1;
        const uint32_t s4 = w.s[c];
        const int c0 = (int)(int8_t)(s4 & 0xff), c1 = (int)(int8_t)((s4 >> 8) & 0xff),
                  c2 = (int)(int8_t)((s4 >> 16) & 0xff), c3 = (int)(int8_t)(s4 >> 24);
        const i32x4 a0 = *(const i32x4*)(mrec + 64 * p), a1 = *(const i32x4*)(mrec + 64 * p + 16),
                    a2 = *(const i32x4*)(mrec + 64 * p + 32), a3 = *(const i32x4*)(mrec + 64 * p + 48);
        const uint32_t hl = w.h[c][k], hh = w.h[c][2 + k];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t q = w.q[p][m];
            const uint32_t wl = (q & M4) | q6_hi_bytes((hl >> (2 * m)) & M2);
            const uint32_t wh = ((q >> 4) & M4) | q6_hi_bytes((hh >> (2 * m)) & M2);
            int a = t[4 * k + m];
            a = __mul24(c0, dot4(wl, a0[m], 0)) + a;
            a = __mul24(c1, dot4(wl, a1[m], 0)) + a;
            a = __mul24(c2, dot4(wh, a2[m], 0)) + a;
            a = __mul24(c3, dot4(wh, a3[m], 0)) + a;
            t[4 * k + m] = a;
        }
    }
    const float d = h2f(w.d) * da;
#pragma unroll
    for (int l = 0; l < 8; ++l) tm[l] = d * (float)t[l];
    tm[8] = 0.f;
}

// ----------------------------------------------------------------------------------
// x86 numerics (model numerics LLMI_NUMERICS_X86): the association upstream's x86 AVX2
// kernels use [upstream ggml-cpu arch/x86/quants.c ggml_vec_dot_{q4_K,q5_K,q6_K}_q8_K,
// ggml_vec_dot_q8_0_q8_0; recalled, not vendored], as restated by the oracle's x86 mode
// (oracle/ggml_oracle.c x86_q4_K .. x86_q8_0).  Per row:
//   K-quants: per 256-block b, in order
//       sumi[k] = sum over the block's elements e with (e % 32) / 4 == k of scale(e)*q(e)*a(e)
//                 (the 8 int32 lanes of maddubs + madd over 32-byte vectors, k = 0..7)
//       acc[k]  = fma(d_a(b) * d_w(b), (float)sumi[k], acc[k])
//       Q4_K:  prod[k] = m[2k](bs[4k] + bs[4k+1]) + m[2k+1](bs[4k+2] + bs[4k+3]) (k < 4),
//              acc_m[k] = fma(-d_a(b) * dmin_w(b), (float)prod[k], acc_m[k])
//       Q5_K:  summs = fma(-d_a(b) * dmin_w(b), (float)sum_j m[j/2] bs[j], summs)
//     result  hsum_float_8(acc) [+ (acc_m[0] + acc_m[2]) + (acc_m[1] + acc_m[3])] [+ summs]
//   Q8_0:     per 32-block b: sumi[k] over bytes 4k..4k+3, acc[k] = fma(d_w*d_a, (float)sumi[k],
//             acc[k]); result hsum_float_8(acc)
// with hsum_float_8(a) = ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7)).  The weights'
// x86 layout (common.h) puts the 4 elements of one lane k of one 32-element vector in one
// dword, so the integer code is the generic one with l read as the lane; the fold runs
// the fma chains (d and the lane sums kept apart until the chain's fma).
// Fold buffer per wave (floats): K-quants S[R][12][Lr] | D[R][2][Lr] (d, -dmin) | G[R][12];
// Q8_0 S[R][8][CS] | D[R][CS] | G[R][8] with the chain (and d-row) stride CS = x86q_cs(Lr)
// = 8 Lr + 4 (Lr >= 8): fold lane f reads chain f at f CS, so the 16 lanes of a
// ds_read_b128 group start on 16 different 16-B bank slots (an 8 Lr stride put them all on
// one: 16-way, and the unit's 64 single-dword stores were 8-way).  The buffer is sized per
// geometry (fold_stride): the largest (Lr = 8, R = 8) takes 4352 + 544 + 64 floats, and
// wide rows far less (TinyLlama's ffn_down, Lr = 24: 3544), which keeps two 4-wave
// workgroups per CU where a fixed 4960 would not.
// ----------------------------------------------------------------------------------
// generic K-quants: S[R][9][CS] chains at stride CS = kq_cs(Lr) (Lr, or Lr + 4 when Lr / 4 is
// even, so the stride in 16-B slots is odd and a fold read group's 16 lanes meet 16 slots:
// Lr = 16 (Llama-3-8B's 4096 columns) had them on 4 slots, 4-way); R 9 CS <= 864.
__host__ __device__ constexpr int kq_cs(int lr) { return (lr / 4) % 2 == 0 ? lr + 4 : lr; }
constexpr int kFoldF = 864, kFoldFloats = kFoldF + 9 * 16;
constexpr int kX86KD = 12 * 64, kX86KG = kX86KD + 2 * 64, kX86KFloats = kX86KG + 12 * 16;
__host__ __device__ constexpr int x86q_cs(int lr) { return lr >= 8 ? 8 * lr + 4 : 8 * lr; }
__host__ __device__ constexpr int x86q_d(int R, int lr) { return R * 8 * x86q_cs(lr); }
__host__ __device__ constexpr int x86q_g(int R, int lr) { return x86q_d(R, lr) + R * x86q_cs(lr); }
constexpr int kX86QFloats = 4960;
static_assert(x86q_g(8, 8) + 8 * 8 <= kX86QFloats && x86q_g(16, 4) + 8 * 16 <= kX86QFloats &&
                  x86q_g(4, 16) + 8 * 4 <= kX86QFloats && x86q_g(2, 32) + 8 * 2 <= kX86QFloats &&
                  x86q_g(1, 64) + 8 <= kX86QFloats,
              "x86 Q8_0 fold buffer");
template <int ACT, int X86>
__host__ __device__ constexpr int fold_floats() { return X86 ? (ACT ? kX86QFloats : kX86KFloats) : kFoldFloats; }
template <int ACT>
__host__ __device__ constexpr int x86_chains() { return ACT ? 8 : 12; }
// floats of one wave's fold buffer at task geometry (R, Lr) -- a multiple of 4 (16-B aligned)
__host__ __device__ constexpr int fold_stride(int act, int x86, int R, int lr) {
    return x86 && act ? (x86q_g(R, lr) + 8 * R + 3) & ~3 : x86 ? kX86KFloats : kFoldFloats;
}
// the largest fold_stride a launch over `cols` columns can take (mv_geometry's Lr for both
// epilogue caps, R before any halving)
__host__ __device__ inline int fold_stride_cols(int act, int x86, int cols) {
    if (!(x86 && act)) return fold_stride(act, x86, 1, 4);
    const int U = cols >> 8;
    int f = 0;
    for (int lmax = 32; lmax <= 64; lmax += 32) {
        int lr = ((U < lmax ? U : lmax) + 3) & ~3;
        lr = lr < 4 ? 4 : lr > lmax ? lmax : lr;
        int R = 1;
        while (2 * R * lr <= 64) R *= 2;
        const int v = fold_stride(act, x86, R, lr);
        f = v > f ? v : f;
    }
    return f;
}

// upstream hsum_float_8 (AVX: lo128 + hi128, movehl + add, movehdup + add_ss)
__device__ __forceinline__ float x86_hsum8(const float* a) {
    const float t0 = a[0] + a[4], t1 = a[1] + a[5], t2 = a[2] + a[6], t3 = a[3] + a[7];
    return (t0 + t2) + (t1 + t3);
}

// the unit's x86 terms straight into the fold buffer (lane: row r, unit ul of the sub-item)
template <int T>
__device__ __forceinline__ void unit_store_x86(const UnitW<T>& w, const uint8_t* rec, float* F, int r, int ul, int lr,
                                               int R, bool valid) {
    if constexpr (T == T_Q8_0) {
        // per 32-block b: lanes k < 4 are dwords of part 2b, k >= 4 of part 2b + 1; the
        // unit's 8 terms of chain k are 8 consecutive floats: blocks 0-3 and 4-7 go out
        // as one 16-B store each (16 stores of 64 terms instead of 64 single dwords)
        const int cs = x86q_cs(lr);
        float* S = F + (size_t)r * 8 * cs + 8 * ul;
        float* D = F + x86q_d(R, lr) + (size_t)r * cs + 8 * ul;
        float db[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float s[4][8];
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) {
                const int b = 4 * h + bb;
                const i32x4 a0 = *(const i32x4*)(rec + 32 * b), a1 = *(const i32x4*)(rec + 32 * b + 16);
                const float dw = h2f(w.s[b >> 1] >> (16 * (b & 1))), da = *(const float*)(rec + kRecBs + 4 * b);
                db[b] = dw * da;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    s[bb][m] = (float)dot4(w.q[2 * b][m], a0[m], 0);
                    s[bb][4 + m] = (float)dot4(w.q[2 * b + 1][m], a1[m], 0);
                }
            }
            if (valid) {
#pragma unroll
                for (int k = 0; k < 8; ++k) *(float4*)(S + (size_t)k * cs + 4 * h) = make_float4(s[0][k], s[1][k], s[2][k], s[3][k]);
            }
        }
        if (valid) {
            *(float4*)D = make_float4(db[0], db[1], db[2], db[3]);
            *(float4*)(D + 4) = make_float4(db[4], db[5], db[6], db[7]);
        }
    } else {
        int t[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) t[l] = 0;
        float d, dm = 0.f;
        float ms[4] = {0.f, 0.f, 0.f, 0.f};
        const float da = *(const float*)(rec + kRecD);
        if constexpr (T == T_Q4_K || T == T_Q5_K) {
            u32x2 sc, mn;
            scales_mins(w.s.y, w.s.z, w.s.w, sc, mn);
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const int c = p >> 1, k = p & 1;
                const uint32_t sw = c < 2 ? sc.x : sc.y;
                const int slo = (int)((sw >> (16 * (c & 1))) & 0xffu), shi = (int)((sw >> (16 * (c & 1) + 8)) & 0xffu);
                const i32x4 alo = *(const i32x4*)(rec + 32 * p), ahi = *(const i32x4*)(rec + 32 * p + 16);
                uint32_t hlo = 0, hhi = 0;
                if constexpr (T == T_Q5_K) {
                    hlo = w.h[c >> 1][2 * (c & 1)];
                    hhi = w.h[c >> 1][2 * (c & 1) + 1];
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int l = 4 * k + m;
                    uint32_t l4 = w.q[p][m] & M4, h4 = (w.q[p][m] >> 4) & M4;
                    if constexpr (T == T_Q5_K) {
                        l4 |= (l <= 4 ? hlo << (4 - l) : hlo >> (l - 4)) & 0x10101010u;
                        h4 |= (l <= 4 ? hhi << (4 - l) : hhi >> (l - 4)) & 0x10101010u;
                    }
                    t[l] = __mul24(slo, dot4(l4, alo[m], 0)) + t[l];
                    t[l] = __mul24(shi, dot4(h4, ahi[m], 0)) + t[l];
                }
            }
            // bsum pairs (bs[2j], bs[2j+1]) against (m_j, m_j): prod[k] = pairs 2k, 2k+1
            const i32x4 b0 = *(const i32x4*)(rec + kRecBs), b1 = *(const i32x4*)(rec + kRecBs + 16);
            int pr[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t sel = 0x0c000c00u | (uint32_t)(j & 3) * 0x00010001u;
                const uint32_t mm = __builtin_amdgcn_perm(0u, j < 4 ? mn.x : mn.y, sel);
                const int bp = j < 4 ? b0[j] : b1[j - 4];
                pr[j >> 1] = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, bp), __builtin_bit_cast(short2_t, mm), pr[j >> 1], false);
            }
            d = da * h2f(w.s.x);
            dm = -da * h2f(w.s.x >> 16);
            if constexpr (T == T_Q4_K) {
#pragma unroll
                for (int k = 0; k < 4; ++k) ms[k] = (float)pr[k];
            } else {
                ms[0] = (float)(((pr[0] + pr[1]) + pr[2]) + pr[3]);
            }
        } else {  // Q6_K: a dword = 4 consecutive elements of one 16-element sub-block, one scale
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const int c = p >> 1, k = p & 1;
                const uint32_t s4 = w.s[c];
                const int clo = (int)(int8_t)((s4 >> (8 * k)) & 0xff), chi = (int)(int8_t)((s4 >> (8 * (2 + k))) & 0xff);
                const i32x4 alo = *(const i32x4*)(rec + 32 * p), ahi = *(const i32x4*)(rec + 32 * p + 16);
                const uint32_t hl = w.h[c][k], hh = w.h[c][2 + k];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const uint32_t q = w.q[p][m];
                    const uint32_t wl = (q & M4) | q6_hi_bytes((hl >> (2 * m)) & M2);
                    const uint32_t wh = ((q >> 4) & M4) | q6_hi_bytes((hh >> (2 * m)) & M2);
                    int a = t[4 * k + m];
                    a = __mul24(clo, dot4(wl, alo[m], 0)) + a;
                    a = __mul24(chi, dot4(wh, ahi[m], 0)) + a;
                    t[4 * k + m] = a;
                }
            }
            d = da * h2f(w.d);
        }
        if (valid) {
            float* S = F + (size_t)r * 12 * lr + ul;
#pragma unroll
            for (int l = 0; l < 8; ++l) S[l * lr] = (float)t[l];
#pragma unroll
            for (int k = 0; k < 4; ++k) S[(8 + k) * lr] = ms[k];
            float* D = F + kX86KD + (size_t)r * 2 * lr + ul;
            D[0] = d;
            D[lr] = dm;
        }
    }
}

// The fold's chains in order with their LDS reads batched: 16 terms per batch, the next
// batch's four ds_read_b128 issued before the current batch's adds, so a chain waits one
// LDS latency per 16 terms instead of one per 4 (the per-4 loop waited on every read:
// 44 waits for a Q8_0 row of 5632 columns).  Reads run up to 15 floats past the chain's
// last term -- inside the wave's fold buffer (kFoldFloats >= 9 R Lr + 16) -- and those
// values are never added.  `a` sees exactly the adds / fmas of the plain loop.
template <class OP>
__device__ __forceinline__ float chain_batched(int len, float a, OP&& term) {
    constexpr int TB = OP::TB;  // terms per batch (16 floats of registers)
    float c[16], nx[16];
    term.load(0, c);
    int b = 0;
    for (; b + TB <= len; b += TB) {
        if (b + TB < len) term.load(b + TB, nx);  // (uniform: len is the wave's)
#pragma unroll
        for (int k = 0; k < TB; ++k) a = term.apply(a, c, k);
#pragma unroll
        for (int k = 0; k < 16; ++k) c[k] = nx[k];
    }
#pragma unroll
    for (int k = 0; k < TB - 1; ++k)
        if (b + k < len) a = term.apply(a, c, k);
    return a;
}
struct ChainAdd {  // a += q[i]
    static constexpr int TB = 16;
    const float* q;
    __device__ __forceinline__ void load(int b, float* v) const {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 x = *(const float4*)(q + b + 4 * k);
            v[4 * k] = x.x;
            v[4 * k + 1] = x.y;
            v[4 * k + 2] = x.z;
            v[4 * k + 3] = x.w;
        }
    }
    __device__ __forceinline__ float apply(float a, const float* v, int k) const { return a + v[k]; }
};
struct ChainFma {  // a = fma(d[i], s[i], a); v holds the batch's 8 (d, s) pairs
    static constexpr int TB = 8;
    const float* d;
    const float* s;
    __device__ __forceinline__ void load(int b, float* v) const {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const float4 x = *(const float4*)(d + b + 4 * k), y = *(const float4*)(s + b + 4 * k);
            v[8 * k] = x.x;
            v[8 * k + 1] = y.x;
            v[8 * k + 2] = x.y;
            v[8 * k + 3] = y.y;
            v[8 * k + 4] = x.z;
            v[8 * k + 5] = y.z;
            v[8 * k + 6] = x.w;
            v[8 * k + 7] = y.w;
        }
    }
    __device__ __forceinline__ float apply(float a, const float* v, int k) const { return __builtin_fmaf(v[2 * k], v[2 * k + 1], a); }
};

// Fold lane f = (row f / NC, chain f % NC) runs its fma chain over the sub-item's n units
// (Q8_0: 8 n blocks) in order; chains 0..7 take d, chains 8..11 (the min lanes) -dmin.
template <int ACT>
__device__ __forceinline__ void fold_sub_x86(float* F, int R, int lr, int n, bool last, float& acc) {
    constexpr int NC = x86_chains<ACT>();
    const int lane = threadIdx.x & 63, nf = R * NC;
    for (int f = lane; f < nf; f += 64) {
        const int r = f / NC, c = f - r * NC;
        float a;
        if constexpr (ACT) {
            const float* s = F + (size_t)(r * 8 + c) * x86q_cs(lr);
            const float* d = F + x86q_d(R, lr) + (size_t)r * x86q_cs(lr);
            a = chain_batched(8 * n, acc, ChainFma{d, s});
            if (last) F[x86q_g(R, lr) + f] = a;
        } else {
            const float* s = F + (size_t)(r * 12 + c) * lr;
            const float* d = F + kX86KD + (size_t)(r * 2 + (c >= 8 ? 1 : 0)) * lr;
            a = chain_batched(n, acc, ChainFma{d, s});
            if (last) F[kX86KG + f] = a;
        }
        if (last) a = 0.f;
        acc = a;
    }
}
// final value of row r of the task (after a wave_lds_sync)
template <int ACT>
__device__ __forceinline__ float row_final_x86(const float* F, int r, int type, int R, int lr) {
    if constexpr (ACT) {
        return x86_hsum8(F + x86q_g(R, lr) + 8 * r);
    } else {
        const float* g = F + kX86KG + 12 * r;
        const float h = x86_hsum8(g);
        if (type == T_Q4_K) return h + ((g[8] + g[10]) + (g[9] + g[11]));
        if (type == T_Q5_K) return h + g[8];
        return h;
    }
}

// upstream ggml_v_expf (AVX2/AVX-512: the ARM optimized-routines polynomial exp; every
// lane of a vector computes exactly this, the special-case blend included), and
// ggml_v_silu(x) = x / (1 + ggml_v_expf(-x))
__device__ __forceinline__ float x86_v_expf(float x) {
    const float r = 0x1.8p23f;
    const float z = __builtin_fmaf(x, 0x1.715476p+0f, r);
    const float n = z - r;
    const float b = __builtin_fmaf(-n, 0x1.7f7d1cp-20f, __builtin_fmaf(-n, 0x1.62e4p-1f, x));
    const uint32_t e = __float_as_uint(z) << 23;
    const float k = __uint_as_float(e + __float_as_uint(1.0f));
    const float u = b * b;
    const float j = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(0x1.0e4020p-7f, b, 0x1.573e2ep-5f), u,
                                                  __builtin_fmaf(0x1.555e66p-3f, b, 0x1.fffdb6p-2f)),
                                   u, 0x1.ffffecp-1f * b);
    if (!(fabsf(n) > 126.f)) return __builtin_fmaf(j, k, k);
    const uint32_t g = n <= 0.f ? 0x82000000u : 0u;
    const float s1 = __uint_as_float(g + 0x7f000000u), s2 = __uint_as_float(e - g);
    if (fabsf(n) > 192.f) return s1 * s1;
    return __builtin_fmaf(s2, j, s2) * s1;
}
__device__ __forceinline__ float x86_silu(float x) { return x / (1.0f + x86_v_expf(-x)); }

// ----------------------------------------------------------------------------------
// Row tasks.  A matvec launch's rows are cut into TASKS of R rows (gate/up launches: R
// gate rows then the same R up rows); lane L works on row r = L / Lr of the task, units
// L % Lr + Lr j (Lr lanes per row, a multiple of 4; R = 64 / Lr rounded down to a power
// of two).  A task is NJ = ceil(U / Lr) SUB-ITEMS (SwiGLU: 2 NJ, gate rows first), each
// within one segment, so its plane bases are uniform.  The host fills MVGeom.
// ----------------------------------------------------------------------------------
struct TaskGeo {
    int lr, R, nj, U;
};
__host__ __device__ inline TaskGeo task_geo(const MVArgs& A) {
    TaskGeo g;
    g.lr = A.lr;
    g.R = A.rpt;
    g.U = A.cols >> 8;
    g.nj = (g.U + g.lr - 1) / g.lr;
    return g;
}

// Fold buffer per wave: F[row][chain][Lr] terms + G[row][chain] chain results (kFoldF,
// kFoldFloats: above, with the x86 buffers).  Q8_0: row r's 8 Lr terms at r * (8 Lr + 4),
// so the fold lanes' 16-B reads start on different bank slots (R (8 Lr + 4) <= kFoldF).
__host__ __device__ constexpr int q80_rs(int lr) { return 8 * lr + 4; }

// Fold lane f (< R * chains) adds its chain's n terms of the sub-item (K-quants: chain f
// = (row f / 9, chain f % 9), Lr terms apart; Q8_0: chain = row f, 8 terms per unit) in
// unit order onto acc; on the task's last sub-item of the row set the chain result goes
// to G[f] and acc restarts.  Only NJ == 1 geometries have more than 64 chains (then no
// chain carries across sub-items).
template <int ACT>
__device__ __forceinline__ void fold_sub(float* F, int R, int lr, int n, bool last, float& acc) {
    constexpr int NC = row_chains<ACT>();
    const int lane = threadIdx.x & 63, nf = R * NC;
    const int len = ACT ? 8 * n : n, stride = ACT ? q80_rs(lr) : kq_cs(lr);
    for (int f = lane; f < nf; f += 64) {
        float a = chain_batched(len, acc, ChainAdd{F + f * stride});
        if (last) {
            F[kFoldF + f] = a;
            a = 0.f;
        }
        acc = a;
    }
}
// final value of row r of the task from G (after a wave_lds_sync)
template <int ACT>
__device__ __forceinline__ float row_final(const float* F, int r) {
    const float* g = F + kFoldF;
    if constexpr (ACT) {
        return g[r];
    } else {
        float v = g[9 * r + 8];
#pragma unroll
        for (int l = 0; l < 8; ++l) v += g[9 * r + l];
        return v;
    }
}
// the unit's terms into F (lane: row r, unit index ul of the sub-item)
template <int T>
__device__ __forceinline__ void store_terms(float* F, int r, int ul, int lr, const float (&tm)[9]) {
    if constexpr (T == T_Q8_0) {
        float* q = F + r * q80_rs(lr) + 8 * ul;
        *(float4*)q = make_float4(tm[0], tm[1], tm[2], tm[3]);
        *(float4*)(q + 4) = make_float4(tm[4], tm[5], tm[6], tm[7]);
    } else {
        const int cs = kq_cs(lr);
        float* q = F + r * 9 * cs + ul;
#pragma unroll
        for (int c = 0; c < 9; ++c) q[c * cs] = tm[c];
    }
}

// (the descriptor type is a template parameter: the persistent step reads its phase
// descriptors through the constant address space, step.hip)
template <class MA>
__device__ __forceinline__ Seg pick(const MA& A, int si) {
    Seg s;
    s.a = si == 0 ? A.seg[0].a : si == 1 ? A.seg[1].a : A.seg[2].a;
    s.h = si == 0 ? A.seg[0].h : si == 1 ? A.seg[1].h : A.seg[2].h;
    s.s = si == 0 ? A.seg[0].s : si == 1 ? A.seg[1].s : A.seg[2].s;
    s.d = si == 0 ? A.seg[0].d : si == 1 ? A.seg[1].d : A.seg[2].d;
    s.type = si == 0 ? A.seg[0].type : si == 1 ? A.seg[1].type : A.seg[2].type;
    s.rows = si == 0 ? A.seg[0].rows : si == 1 ? A.seg[1].rows : A.seg[2].rows;
    s.row0 = si == 0 ? A.seg[0].row0 : si == 1 ? A.seg[1].row0 : A.seg[2].row0;
    s.rgs = si == 0 ? A.seg[0].rgs : si == 1 ? A.seg[1].rgs : A.seg[2].rgs;
    return s;
}

// ----------------------------------------------------------------------------------
// Row-pair work items.  A wave streams its pairs p = w0, w0+G, ... (G = 4*gridDim.x);
// item j of a pair is piece P = lane + 64*j of both rows (NJ = ceil(pieces/64)).
// ----------------------------------------------------------------------------------
struct PairRef {
    Seg sa, sb;
    int ra, rb;
    int vb;      // (an int, not a bool: no padding bytes for SROA to keep in scratch)
    int type;  // common type of both rows, or -1 if they differ
};

template <int EPI, class MA>
__device__ __forceinline__ PairRef pair_ref(const MA& A, int p) {
    PairRef r;
    if constexpr (EPI == EPI_SWIGLU) {
        r.sa = pick(A, 0);
        r.sb = pick(A, 1);
        r.ra = r.rb = p;
        r.vb = true;
    } else {
        const int g = A.seg[0].row0 + 2 * p;
        int si = 0;
        if (A.nseg > 1 && g >= A.seg[1].row0) si = 1;
        if (A.nseg > 2 && g >= A.seg[2].row0) si = 2;
        r.sa = pick(A, si);
        r.sb = r.sa;
        r.ra = g - r.sa.row0;
        r.rb = r.ra + 1;
        r.vb = r.rb < r.sa.rows;
    }
    r.type = r.sa.type == r.sb.type ? r.sa.type : -1;
    return r;
}

// ordered key of (logit, row): larger logit wins, ties -> smaller row (first max wins,
// as upstream llama_sampler_greedy's strict '>' scan)
__device__ __forceinline__ unsigned long long argmax_key(float v, int row) {
    if (v == 0.f) v = 0.f;  // -0 == +0
    uint32_t u = __float_as_uint(v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (unsigned long long)(0xffffffffu - (uint32_t)row);
}

// Global accesses of data handed between the phases of ONE launch (the persistent step,
// step.hip): write-through `sc1` stores and `sc1` loads (relaxed agent-scope atomics),
// the hand-off form MI355X_MICROARCH.md §visibility validates without acquire fences.
// WT = false: plain accesses (separate launches hand over at kernel boundaries).
typedef unsigned int __attribute__((address_space(1))) gu32_t;
typedef unsigned short __attribute__((address_space(1))) gu16_t;
typedef unsigned long long __attribute__((address_space(1))) gu64_t;
template <bool WT>
__device__ __forceinline__ void st_f32(float* p, float v) {
    if constexpr (WT) __hip_atomic_store((gu32_t*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
template <bool WT>
__device__ __forceinline__ float ld_f32(const float* p) {
    if constexpr (WT) return __uint_as_float(__hip_atomic_load((const gu32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    else return *p;
}
template <bool WT>
__device__ __forceinline__ void st_u32(void* p, uint32_t v) {
    if constexpr (WT) __hip_atomic_store((gu32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *(uint32_t*)p = v;
}
template <bool WT>
__device__ __forceinline__ void st_u16(uint16_t* p, uint16_t v) {
    if constexpr (WT) __hip_atomic_store((gu16_t*)p, (unsigned short)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

// Epilogue of one finished pair (every lane holds both row sums; lane 0 writes).
// (ANY_LANE: the calling lane writes; the batched matvec runs one token per lane)
// PRE (the layer engine, leng.hip): the epilogue's one dependent load was issued early by
// the caller -- ADD: pre.x = the residual y[row a] (r.vb == 0); QKV: pre = the RoPE (cos,
// sin) of the pair -- so it does not wait behind the CU's weight stream at the task's end.
template <int EPI, bool WT = false, class MA, bool ANY_LANE = false, int X86 = 0, bool PRE = false>
__device__ __forceinline__ void epilogue(const MA& A, const PairRef& r, int p, PairSum v, int pos,
                                         unsigned long long& best, float2 pre = float2{0.f, 0.f}) {
    const int lane = threadIdx.x & 63;
    const float va = v.a, vb = v.b;
    if (!ANY_LANE && lane != 0) return;
    if constexpr (EPI == EPI_STORE) {
        st_f32<WT>(A.y + r.sa.row0 + r.ra, va);
        if (r.vb) st_f32<WT>(A.y + r.sa.row0 + r.rb, vb);
    } else if constexpr (EPI == EPI_ADD) {
        float* ya = A.y + r.sa.row0 + r.ra;
        st_f32<WT>(ya, (PRE ? pre.x : ld_f32<WT>(ya)) + va);
        if (r.vb) {
            float* yb = A.y + r.sa.row0 + r.rb;
            st_f32<WT>(yb, ld_f32<WT>(yb) + vb);
        }
    } else if constexpr (EPI == EPI_LOGITS) {
        A.y[r.ra] = va;
        unsigned long long k = argmax_key(va, r.ra);
        best = k > best ? k : best;
        if (r.vb) {
            A.y[r.rb] = vb;
            k = argmax_key(vb, r.rb);
            best = k > best ? k : best;
        }
    } else if constexpr (EPI == EPI_SWIGLU) {
        st_f32<WT>(A.y + p, (X86 ? x86_silu(va) : llmi_silu(va)) * vb);
    } else if constexpr (EPI == EPI_QKV) {
        // sa.row0 tells q (0), k (nq) or v (nq+nk); rows (ra, ra+1) are a RoPE pair
        const int hd = A.head_dim;
        const int h = r.ra / hd, d = r.ra - h * hd;
        if (r.sa.row0 < A.nq + A.nk) {
            float o0 = va, o1 = vb;
            if (d < A.n_rot) {  // ggml rope NORM mode on the adjacent pair (d, d+1)
                const float2 cs = PRE ? pre : *(const float2*)(A.rope + ((size_t)pos * (A.n_rot / 2) + d / 2) * 2);
                o0 = va * cs.x - vb * cs.y;
                o1 = va * cs.y + vb * cs.x;
            }
            if (r.sa.row0 == 0) {
                st_f32<WT>(A.y + r.ra, o0);
                st_f32<WT>(A.y + r.ra + 1, o1);
            } else {
                const uint32_t w = (uint32_t)f2h(o0) | ((uint32_t)f2h(o1) << 16);
                st_u32<WT>(A.kc + ((size_t)h * A.n_ctx + pos) * hd + d, w);
            }
        } else {
            st_u16<WT>(A.vc + ((size_t)h * hd + d) * A.n_ctx + pos, f2h(va));
            st_u16<WT>(A.vc + ((size_t)h * hd + d + 1) * A.n_ctx + pos, f2h(vb));
        }
    }
}

// Sub-item s of a task: its segment, the segment-local row of the task's row 0 and the
// unit block j (units Lr j .. Lr j + Lr - 1).  Uniform per wave.
struct Sub {
    int si, row0, j;
};
template <int EPI, class MA>
__device__ __forceinline__ Sub sub_of(const MA& A, const TaskGeo& g, int task, int s) {
    Sub b;
    if constexpr (EPI == EPI_SWIGLU) {  // gate rows (segment 0) for s < NJ, then the same up rows
        b.si = s >= g.nj ? 1 : 0;
        b.j = s - b.si * g.nj;
        b.row0 = task * g.R;
    } else {
        // (the starts pass through readfirstlane so that the select below stays a select
        // of values: folded into A.seg[si] it copies the kernel arguments to scratch)
        const int r0 = uniform(A.seg[0].row0), r1 = uniform(A.seg[1].row0), r2 = uniform(A.seg[2].row0);
        const int q = r0 + task * g.R;
        int si = 0;
        if (A.nseg > 1 && q >= r1) si = 1;
        if (A.nseg > 2 && q >= r2) si = 2;
        b.si = si;
        b.j = s;
        b.row0 = q - (si == 0 ? r0 : si == 1 ? r1 : r2);
    }
    return b;
}
// is every sub-item of the task of type T (the pipelined type)?
template <int EPI, int T, class MA>
__device__ __forceinline__ bool task_is(const MA& A, const TaskGeo& g, int task) {
    if constexpr (EPI == EPI_SWIGLU) return A.seg[0].type == T && A.seg[1].type == T;
    else return pick(A, sub_of<EPI>(A, g, task, 0).si).type == T;
}

// The lane's row / unit of a sub-item, clamped into the matrix (loads stay unconditional).
struct LaneUnit {
    uint32_t row, u;
    bool valid;
};
__device__ __forceinline__ LaneUnit lane_unit(const TaskGeo& g, const Sub& b, const Seg& sg, int r, int ul) {
    LaneUnit x;
    const int row = b.row0 + r, u = ul + g.lr * b.j;
    x.valid = r < g.R && row < sg.rows && u < g.U;
    x.row = (uint32_t)(row < sg.rows ? row : sg.rows - 1);
    x.u = (uint32_t)(u < g.U ? u : g.U - 1);
    return x;
}

// After the lanes' unit terms: store, fold, and on the row set's last sub-item the row
// results and the epilogue (lane r' < R handles row r' of the task).
// (X86: the lane's terms are already in F, unit_store_x86; tm is unused)
// (WT: write-through epilogue stores, for outputs handed to other workgroups of the same
// launch: the layer engine, leng.hip)
template <int ACT, int EPI, class MA, int X86 = 0, bool WT = false, bool PRE = false>
__device__ __forceinline__ void sub_finish(const MA& A, float* F, const TaskGeo& g, int s, const Sub& b, const Seg& sg,
                                           const float (&tm)[9], const LaneUnit& lu, int r, int ul, float& acc,
                                           float& vg, int pos, unsigned long long& best,
                                           float2 pre = float2{0.f, 0.f}) {
    if constexpr (!X86)
        if (lu.valid) store_terms<ACT ? T_Q8_0 : T_Q4_K>(F, r, ul, g.lr, tm);
    wave_lds_sync();
    const int n = min(g.lr, g.U - g.lr * b.j);
    const bool last = b.j == g.nj - 1;
    if constexpr (X86) fold_sub_x86<ACT>(F, g.R, g.lr, n, last, acc);
    else fold_sub<ACT>(F, g.R, g.lr, n, last, acc);
    auto final_of = [&](int rr) { return X86 ? row_final_x86<ACT>(F, rr, sg.type, g.R, g.lr) : row_final<ACT>(F, rr); };
    if (last) {
        wave_lds_sync();
        const int lane = threadIdx.x & 63;
        const int row = b.row0 + lane;
        if (lane < g.R && row < sg.rows) {
            const float v = final_of(lane);
            PairRef ref;
            ref.sa = ref.sb = sg;
            ref.ra = row;
            ref.rb = row + 1;
            ref.vb = 0;
            ref.type = sg.type;
            if constexpr (EPI == EPI_SWIGLU) {
                if (s < g.nj) vg = v;
                else epilogue<EPI, WT, MA, true, X86>(A, ref, row, PairSum{vg, v}, pos, best);
            } else if constexpr (EPI == EPI_QKV) {
                ref.vb = 1;  // RoPE pairs (row, row + 1): R and every segment start are even
                if ((lane & 1) == 0)
                    epilogue<EPI, WT, MA, true, X86, PRE>(A, ref, row, PairSum{v, final_of(lane + 1)}, pos, best, pre);
            } else {
                epilogue<EPI, WT, MA, true, X86, PRE>(A, ref, row, PairSum{v, 0.f}, pos, best, pre);
            }
        }
    }
    wave_lds_sync();  // the fold / final reads before the next sub-item's stores
}

// One task of any type, not pipelined (tasks whose type is not the kernel's primary type:
// the Q6_K attn_v rows of a Q4_K QKV launch, mixed-type gate/up).
template <int ACT, int EPI, class MA, int X86 = 0>
__device__ __forceinline__ void task_any(const MA& A, const Lds& L, float* F, const TaskGeo& g, int task, int r, int ul,
                                         int pos, unsigned long long& best) {
    const int S = EPI == EPI_SWIGLU ? 2 * g.nj : g.nj;
    float acc = 0.f, vg = 0.f;
    for (int s = 0; s < S; ++s) {
        const Sub b = sub_of<EPI>(A, g, task, s);
        const Seg sg = pick(A, b.si);
        const LaneUnit lu = lane_unit(g, b, sg, r, ul);
        const uint8_t* rec = L.act + (size_t)lu.u * kRec;
        float tm[9];
        if constexpr (X86) {
            if constexpr (ACT == 1) {
                unit_store_x86<T_Q8_0>(load_unit<T_Q8_0>(sg, lu.row, lu.u, g.U), rec, F, r, ul, g.lr, g.R, lu.valid);
            } else {
                switch (sg.type) {
                    case T_Q4_K: unit_store_x86<T_Q4_K>(load_unit<T_Q4_K>(sg, lu.row, lu.u, g.U), rec, F, r, ul, g.lr, g.R, lu.valid); break;
                    case T_Q5_K: unit_store_x86<T_Q5_K>(load_unit<T_Q5_K>(sg, lu.row, lu.u, g.U), rec, F, r, ul, g.lr, g.R, lu.valid); break;
                    default: unit_store_x86<T_Q6_K>(load_unit<T_Q6_K>(sg, lu.row, lu.u, g.U), rec, F, r, ul, g.lr, g.R, lu.valid); break;
                }
            }
        } else if constexpr (ACT == 1) {
            unit_terms<T_Q8_0>(load_unit<T_Q8_0>(sg, lu.row, lu.u, g.U), rec, tm);
        } else {
            switch (sg.type) {
                case T_Q4_K: unit_terms<T_Q4_K>(load_unit<T_Q4_K>(sg, lu.row, lu.u, g.U), rec, tm); break;
                case T_Q5_K: unit_terms<T_Q5_K>(load_unit<T_Q5_K>(sg, lu.row, lu.u, g.U), rec, tm); break;
                default: unit_terms<T_Q6_K>(load_unit<T_Q6_K>(sg, lu.row, lu.u, g.U), rec, tm); break;
            }
        }
        sub_finish<ACT, EPI, MA, X86>(A, F, g, s, b, sg, tm, lu, r, ul, acc, vg, pos, best);
    }
}

// get_rows: element e of row `row` dequantized from the device layout (bit-exact with
// upstream dequantize_row_*)
__device__ __forceinline__ float dequant_elem(const Seg& w, int row, int e, int cols) {
    const size_t U = (size_t)(cols >> 8), u = (size_t)(e >> 8), ru = (size_t)row * U + u;
    switch (w.type) {
        case T_F32: return ((const float*)w.a)[(size_t)row * cols + e];
        case T_F16: return h2f(((const uint16_t*)w.a)[(size_t)row * cols + e]);
        case T_Q4_K:
        case T_Q5_K:
        case T_Q6_K: {
            // residue order (common.h): element 64c + 32hi + l + 8i of the unit sits in
            // part 2c + l/4, byte 4 (l % 4) + i (low nibble: hi = 0, high nibble: hi = 1);
            // x86 order: element 64c + 32hi + 4l + i (l = 4k + m), the same part / byte / bits
            const int t = e & 255, c = t >> 6, hi = (t >> 5) & 1;
            const int l = w.x86 ? (t & 31) >> 2 : t & 7, i = w.x86 ? t & 3 : (t & 31) >> 3, k = l >> 2, m = l & 3;
            const uint8_t qb = w.a[piece_off(row, 2 * c + k, u, U, 8, w.rgs) + 4 * m + i];
            int q = hi ? (qb >> 4) : (qb & 0xF);
            if (w.type == T_Q6_K) {  // H part c: dword (2*hi + k), byte i, bits 2m: the 2 high bits XOR 2
                const uint8_t hb = w.h[piece_off(row, c, u, U, 4, w.rgs) + (2 * hi + k) * 4 + i];
                q |= (((hb >> (2 * m)) & 3) ^ 2) << 4;
                const float d = h2f(*(const uint16_t*)(w.d + ru * 2));
                const int sc = (int8_t)w.s[ru * 16 + (t >> 4)];
                return d * (float)sc * (float)(q - 32);
            }
            const uint32_t* s32 = (const uint32_t*)(w.s + ru * 16);
            int sc, mn;
            scale_min(2 * c + hi, s32[1], s32[2], s32[3], sc, mn);
            if (w.type == T_Q5_K) {  // H part c/2: chunk c's lo / hi word, byte i, bit l
                const uint8_t hb = w.h[piece_off(row, c >> 1, u, U, 2, w.rgs) + 8 * (c & 1) + 4 * hi + i];
                q += ((hb >> l) & 1) << 4;
            }
            const float d = h2f(s32[0]), dmin = h2f(s32[0] >> 16);
            const float d1 = d * (float)sc, m1 = dmin * (float)mn;
            return d1 * (float)q - m1;
        }
        case T_Q8_0: {
            const int t = e & 255;
            const uint8_t qb = w.a[piece_off(row, t >> 4, u, U, 16, w.rgs) + (t & 15)];
            return (float)(int8_t)qb * h2f(*(const uint16_t*)(w.d + ru * 16 + 2 * (t >> 5)));
        }
        default: return 0.f;
    }
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#define LLMI_MAX64_STEP(O)                                                                        \
    {                                                                                             \
        const uint32_t lo = xor_partner_u32<O>((uint32_t)v), hi = xor_partner_u32<O>((uint32_t)(v >> 32)); \
        const unsigned long long o = ((unsigned long long)hi << 32) | lo;                         \
        v = o > v ? o : v;                                                                        \
    }
    LLMI_MAX64_STEP(1) LLMI_MAX64_STEP(2) LLMI_MAX64_STEP(4) LLMI_MAX64_STEP(8) LLMI_MAX64_STEP(16) LLMI_MAX64_STEP(32)
#undef LLMI_MAX64_STEP
    return v;
}

#if defined(LLMI_EXP_TRACE)
// per-wave stamps of the attention kernels: trace[(k * 4096 + block) * 16 + wave * 4 + i]
#define LLMI_ATT_STAMP(K, I)                                                                      \
    if (a.trace && (threadIdx.x & 63) == 0)                                                       \
        a.trace[((size_t)(K) * 4096 + blockIdx.y * gridDim.x + blockIdx.x) * 64 + (threadIdx.x >> 6) * 4 + (I)] = \
            __builtin_amdgcn_s_memrealtime();
#else
#define LLMI_ATT_STAMP(K, I)
#endif

// Split attention v2, phase 1: grid (HK, kv_bound/32), 256 threads; thread (t, qd)
// dots 1/8 of K row t (D/8 dims) with the G f16-rounded query heads (G independent
// double chains of D/8), 8-lane butterfly; K loads issued before the position is
// known.  Also writes the tile's per-head score maximum (tmax) so phase 2 needs no
// pass over the scores to find the row maximum (max is exact in any order).
template <int D, int G>
__device__ __forceinline__ void attn_scores8_body(const AttnArgs& a) {
    LLMI_ATT_STAMP(0, 0)
    const int g = blockIdx.x, tile = blockIdx.y, t0 = tile * 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int DQ = D / 8;  // 16 (D=128) or 8 (D=64) dims per lane
    const int t = t0 + (tid >> 3), qd = tid & 7;
    const uint16_t* kr = a.kc + ((size_t)g * a.n_ctx + t) * D + qd * DQ;
    u32x4 kv[DQ / 8];
#pragma unroll
    for (int i = 0; i < DQ / 8; ++i) kv[i] = __builtin_nontemporal_load((const u32x4*)(kr + 8 * i));  // K read once
    // q rounded to f16 as upstream's KQ mul_mat does, held as double: every k*q product
    // of two f16 values is exact, so fma(k, q, acc) == acc + (double)(k * q)
    __shared__ __attribute__((aligned(16))) double qs[G][D];
    __shared__ float wmax[4][G];
    for (int i = tid; i < G * D; i += 256) qs[i / D][i % D] = (double)h2f(f2h(a.q[(size_t)g * G * D + i]));
    const int n_kv = a.st->pos + 1;
    __syncthreads();
    LLMI_ATT_STAMP(0, 1)
    if (t0 >= n_kv) return;
    double acc[G];
#pragma unroll
    for (int hh = 0; hh < G; ++hh) acc[hh] = 0.0;
#pragma unroll
    for (int i = 0; i < DQ / 8; ++i) {
        const int d = qd * DQ + 8 * i;
        double k[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            k[2 * j] = (double)h2f((uint16_t)kv[i][j]);
            k[2 * j + 1] = (double)h2f((uint16_t)(kv[i][j] >> 16));
        }
#pragma unroll
        for (int hh = 0; hh < G; ++hh)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[hh] = __builtin_fma(k[j], qs[hh][d + j], acc[hh]);
    }
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        acc[hh] += xor_partner_d<1>(acc[hh]);
        acc[hh] += xor_partner_d<2>(acc[hh]);
        acc[hh] += xor_partner_d<4>(acc[hh]);
        const float sc = (float)acc[hh] * a.scale;
        if (t < n_kv && qd == (hh & 7)) a.scores[(size_t)(g * G + hh) * a.n_ctx + t] = sc;
        // tile max: 8 positions per wave (lanes xor 8, 16, 32), then the 4 waves
        float m = t < n_kv ? sc : -INFINITY;
        m = fmaxf(m, xor_partner<8>(m));
        m = fmaxf(m, xor_partner<16>(m));
        m = fmaxf(m, xor_partner<32>(m));
        if (lane == 0) wmax[wave][hh] = m;
    }
    __syncthreads();
    if (tid < G)
        a.tmax[(size_t)(g * G + tid) * (a.n_ctx / 32) + tile] =
            fmaxf(fmaxf(wmax[0][tid], wmax[1][tid]), fmaxf(wmax[2][tid], wmax[3][tid]));
    LLMI_ATT_STAMP(0, 3)
}

// Split attention v2, phase 2: grid (HK, D/16), 512 threads.  Softmax of the group's G
// heads by 8/G waves each: row max from the tile maxima, e = expf(s - max) with a
// double sum (waves combined in fixed order), p = f16(e / sum) exactly as upstream's
// non-FA path, in LDS as f32 (scores -> e -> p in place); then PV for 16
// output dims: 32 lanes per dim, lane sl takes positions 4*sl + 128*k (8-B V loads, a
// 1024-position window in flight, issued before the position is known),
// fma(v, p, acc) in double (f16 x f16 products are exact; p read as conflict-free
// float4 per 4 positions), 32-lane butterfly.
template <int D, int G>
__device__ __forceinline__ void attn_pv16_body(const AttnArgs& a, int kvb) {
    LLMI_ATT_STAMP(1, 0)
    extern __shared__ __attribute__((aligned(16))) float spd[];  // [G][kvb]
    __shared__ float redm[8];
    __shared__ double reds[8];
    constexpr int WPH = 8 / G;  // waves per head
    const int g = blockIdx.x, dc = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int d = dc * 16 + (tid >> 5), sl = tid & 31;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    // 1. stage the G score rows (all kv_bound positions; those past n_kv are never used)
    const int n4 = kvb >> 2;
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        const float4* src = (const float4*)(a.scores + (size_t)(g * G + hh) * a.n_ctx);
        float4* dst = (float4*)(spd + hh * kvb);
        for (int j = tid; j < n4; j += 512) dst[j] = src[j];
    }
    // V window issued after the score staging (loads return in order: the staging
    // must not queue behind it), in flight during the softmax
    constexpr int NV = 8;  // 8-B V loads in flight per lane: a 1024-position window
    u32x2 vv[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) vv[k] = __builtin_nontemporal_load((const u32x2*)(vr + min(4 * sl + 128 * k, kvb - 4)));
    const int n_kv = a.st->pos + 1;
    const int hh = wave / WPH, wi = wave % WPH;
    {   // row max from the tile maxima (all kv_bound/32 tiles loaded without waiting for
        // the position; tiles past n_kv masked afterwards)
        const float* tm = a.tmax + (size_t)(g * G + hh) * (a.n_ctx / 32);
        const int nt_all = kvb >> 5;
        float mt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) mt[u] = tm[min(wi * 64 + lane + u * WPH * 64, nt_all - 1)];
        const int ntile = (n_kv + 31) >> 5;
        float m = -INFINITY;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (wi * 64 + lane + u * WPH * 64 < ntile) m = fmaxf(m, mt[u]);
        for (int i = wi * 64 + lane + 4 * WPH * 64; i < ntile; i += WPH * 64) m = fmaxf(m, tm[i]);
        m = wave_max(m);
        if (lane == 0) redm[wave] = m;
    }
    __syncthreads();
    LLMI_ATT_STAMP(1, 1)
    float mx = redm[hh * WPH];
#pragma unroll
    for (int i = 1; i < WPH; ++i) mx = fmaxf(mx, redm[hh * WPH + i]);
    // 2. e and the double sum, then p
    float* sp = spd + hh * kvb;
    double sum = 0.0;
    for (int t = wi * 64 + lane; t < n_kv; t += WPH * 64) {
        const float e = llmi_expf(sp[t] - mx);
        sp[t] = e;
        sum += (double)e;
    }
    sum = wave_sum_d(sum);
    if (lane == 0) reds[wave] = sum;
    __syncthreads();
    double tot = reds[hh * WPH];
#pragma unroll
    for (int i = 1; i < WPH; ++i) tot += reds[hh * WPH + i];
    const float inv = (float)(1.0 / tot);
    for (int t = wi * 64 + lane; t < n_kv; t += WPH * 64) sp[t] = h2f(f2h(sp[t] * inv));
    for (int t = n_kv + wi * 64 + lane; t < ((n_kv + 3) & ~3); t += WPH * 64) sp[t] = 0.f;
    __syncthreads();
    LLMI_ATT_STAMP(1, 2)
    // 3. PV
    double acc[G];
#pragma unroll
    for (int h = 0; h < G; ++h) acc[h] = 0.0;
    for (int t0 = 4 * sl;;) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int tb = t0 + 128 * k;
            if (tb < n_kv) {
                double v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float f = h2f((uint16_t)((j < 2 ? vv[k].x : vv[k].y) >> (16 * (j & 1))));
                    v[j] = tb + j < n_kv ? (double)f : 0.0;
                }
#pragma unroll
                for (int h = 0; h < G; ++h) {
                    const float4 p = *(const float4*)(spd + h * kvb + tb);
                    acc[h] = __builtin_fma(v[0], (double)p.x, acc[h]);
                    acc[h] = __builtin_fma(v[1], (double)p.y, acc[h]);
                    acc[h] = __builtin_fma(v[2], (double)p.z, acc[h]);
                    acc[h] = __builtin_fma(v[3], (double)p.w, acc[h]);
                }
            }
        }
        t0 += 128 * NV;
        if (t0 >= n_kv) break;
#pragma unroll
        for (int k = 0; k < NV; ++k) vv[k] = __builtin_nontemporal_load((const u32x2*)(vr + min(t0 + 128 * k, kvb - 4)));
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
        double v = acc[h];
        v += xor_partner_d<1>(v);
        v += xor_partner_d<2>(v);
        v += xor_partner_d<4>(v);
        v += xor_partner_d<8>(v);
        v += xor_partner_d<16>(v);
        if (sl == 0) a.out[(size_t)(g * G + h) * D + d] = (float)v;
    }
    LLMI_ATT_STAMP(1, 3)
}

// Long-context attention (path 7): every phase spread over position tiles so the K and V
// streams use the whole chip, in four launches (a softmax over a whole row cannot be
// formed piecewise bit-exactly: p = f16(e / sum) needs the row's max and sum first).
//   1. k_attn_scores8 (split path phase 1): scores of the G heads per 32-position tile,
//      K read once, plus per-tile maxima
//   2. k_attl_exp    grid (H, tiles of kLongTile): row max from the tile maxima, e =
//      expf(s - max) in place, the tile's double sum of e
//   3. k_attl_pv     grid (HK, tiles): row sum = the tile sums in fixed order, p =
//      f16(e * (float)(1 / sum)), PV of the tile's positions for all D dims of the G
//      heads (V read once), double partial per (head, tile, dim)
//   4. k_attl_sum    grid H: out = the partials summed over tiles in fixed order
// The double sums are exact in practice, as on every other path (tests compare with the
// oracle and the other paths bit for bit).
__device__ __forceinline__ double* attl_tsum(const AttnArgs& a, int n_head) {
    return (double*)(a.scores + attn_long_off(n_head, a.n_ctx));
}
__device__ __forceinline__ double* attl_part(const AttnArgs& a, int n_head) {
    return attl_tsum(a, n_head) + (size_t)n_head * ((a.n_ctx + kLongTile - 1) / kLongTile);
}

// phase 1 for long contexts: k_attn_scores8 with NP 32-position passes per workgroup (the
// q staging amortised over 32*NP positions, every K load issued at entry); same per-pass
// arithmetic, scores and tile maxima as attn_scores8_body
template <int D, int G, int NP>
__device__ __forceinline__ void attl_scores_body(const AttnArgs& a) {
    constexpr int DQ = D / 8;
    __shared__ __attribute__((aligned(16))) double qs[G][D];
    __shared__ float wmax[NP][4][G];
    const int g = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, qd = tid & 7;
    const int tb0 = blockIdx.y * 32 * NP;
    const int kvb = a.n_ctx;
    u32x4 kv[NP][DQ / 8];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int t = min(tb0 + 32 * p + (tid >> 3), kvb - 1);
        const uint16_t* kr = a.kc + ((size_t)g * a.n_ctx + t) * D + qd * DQ;
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i) kv[p][i] = __builtin_nontemporal_load((const u32x4*)(kr + 8 * i));
    }
    for (int i = tid; i < G * D; i += 256) qs[i / D][i % D] = (double)h2f(f2h(a.q[(size_t)g * G * D + i]));
    const int n_kv = a.st->pos + 1;
    __syncthreads();
    if (tb0 >= n_kv) return;  // uniform
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int t = tb0 + 32 * p + (tid >> 3);
        double acc[G];
#pragma unroll
        for (int hh = 0; hh < G; ++hh) acc[hh] = 0.0;
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i) {
            const int d = qd * DQ + 8 * i;
            double k[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                k[2 * j] = (double)h2f((uint16_t)kv[p][i][j]);
                k[2 * j + 1] = (double)h2f((uint16_t)(kv[p][i][j] >> 16));
            }
#pragma unroll
            for (int hh = 0; hh < G; ++hh)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[hh] = __builtin_fma(k[j], qs[hh][d + j], acc[hh]);
        }
#pragma unroll
        for (int hh = 0; hh < G; ++hh) {
            acc[hh] += xor_partner_d<1>(acc[hh]);
            acc[hh] += xor_partner_d<2>(acc[hh]);
            acc[hh] += xor_partner_d<4>(acc[hh]);
            const float sc = (float)acc[hh] * a.scale;
            if (t < n_kv && qd == (hh & 7)) a.scores[(size_t)(g * G + hh) * a.n_ctx + t] = sc;
            float m = t < n_kv ? sc : -INFINITY;
            m = fmaxf(m, xor_partner<8>(m));
            m = fmaxf(m, xor_partner<16>(m));
            m = fmaxf(m, xor_partner<32>(m));
            if (lane == 0) wmax[p][wave][hh] = m;
        }
    }
    __syncthreads();
    if (tid < NP * G) {
        const int p = tid / G, hh = tid % G;
        if (tb0 + 32 * p < n_kv)
            a.tmax[(size_t)(g * G + hh) * (a.n_ctx / 32) + (tb0 >> 5) + p] =
                fmaxf(fmaxf(wmax[p][0][hh], wmax[p][1][hh]), fmaxf(wmax[p][2][hh], wmax[p][3][hh]));
    }
}

__device__ __forceinline__ void attl_exp_body(const AttnArgs& a, int n_head, int kvb) {
    __shared__ float redm[4];
    __shared__ double reds[4];
    const int h = blockIdx.x, tile = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // loads before the position is known: this position's score, the head's tile maxima
    const int t = tile * kLongTile + tid;
    float* srow = a.scores + (size_t)h * a.n_ctx;
    const float s = srow[min(t, kvb - 1)];
    const float* tm = a.tmax + (size_t)h * (a.n_ctx / 32);
    const int ntm_all = kvb >> 5;
    constexpr int NM = 32768 / 32 / 256;  // tile maxima per thread up to a 32768-position bound
    float mt[NM];
#pragma unroll
    for (int k = 0; k < NM; ++k) mt[k] = tm[min(tid + 256 * k, ntm_all - 1)];
    const int n_kv = a.st->pos + 1;
    const int ntl = (a.n_ctx + kLongTile - 1) / kLongTile;
    double* tsum = attl_tsum(a, n_head) + (size_t)h * ntl;
    if (tile * kLongTile >= n_kv) {  // uniform: tiles past the position
        if (tid == 0) tsum[tile] = 0.0;
        return;
    }
    const int ntm = (n_kv + 31) >> 5;
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < NM; ++k)
        if (tid + 256 * k < ntm) m = fmaxf(m, mt[k]);
    for (int i = tid + 256 * NM; i < ntm; i += 256) m = fmaxf(m, tm[i]);
    m = wave_max(m);
    if (lane == 0) redm[wave] = m;
    __syncthreads();
    const float mx = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
    double sum = 0.0;
    if (t < n_kv) {
        const float e = llmi_expf(s - mx);
        srow[t] = e;
        sum = (double)e;
    }
    sum = wave_sum_d(sum);
    if (lane == 0) reds[wave] = sum;
    __syncthreads();
    if (tid == 0) tsum[tile] = ((reds[0] + reds[1]) + reds[2]) + reds[3];
}

template <int D, int G>
__device__ __forceinline__ void attl_pv_body(const AttnArgs& a, int n_head, int kvb) {
    constexpr int SL = 512 / D;                  // lanes per output dim (4 or 8)
    constexpr int NV = kLongTile / (8 * SL);     // 16-B V loads per lane (8 positions each)
    __shared__ __attribute__((aligned(16))) float sp[G][kLongTile];
    __shared__ float sinv[G];
    const int g = blockIdx.x, tile = blockIdx.y, t0 = tile * kLongTile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n_kv = a.st->pos + 1;
    if (t0 >= n_kv) return;  // uniform
    const int ntl = (a.n_ctx + kLongTile - 1) / kLongTile;
    // V rows of this tile first (independent of everything else)
    const int d = tid / SL, sl = tid % SL;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    u32x4 vv[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) vv[u] = __builtin_nontemporal_load((const u32x4*)(vr + min(t0 + 8 * sl + 8 * SL * u, kvb - 8)));
    // this tile's e values (k_attl_exp) of the G heads, also before the row sums
    constexpr int NE = (G * kLongTile + 511) / 512;
    float ev[NE];
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int i = min(tid + 512 * k, G * kLongTile - 1);
        ev[k] = a.scores[(size_t)(g * G + i / kLongTile) * a.n_ctx + min(t0 + i % kLongTile, kvb - 1)];
    }
    // row sums: wave hh < G adds its head's tile sums (lanes, then the fixed butterfly)
    const int ntv = (n_kv + kLongTile - 1) / kLongTile;
    if (wave < G) {
        const double* ts = attl_tsum(a, n_head) + (size_t)(g * G + wave) * ntl;
        constexpr int NS = 32768 / kLongTile / 64;  // tile sums per lane up to 32768 positions
        double tv[NS];
#pragma unroll
        for (int k = 0; k < NS; ++k) tv[k] = ts[min(lane + 64 * k, ntl - 1)];
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if (lane + 64 * k < ntv) s += tv[k];
        for (int i = lane + 64 * NS; i < ntv; i += 64) s += ts[i];
        s = wave_sum_d(s);
        if (lane == 0) sinv[wave] = (float)(1.0 / s);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int i = tid + 512 * k;
        if (i < G * kLongTile) {
            const int hh = i / kLongTile, t = t0 + i % kLongTile;
            sp[hh][i % kLongTile] = t < n_kv ? h2f(f2h(ev[k] * sinv[hh])) : 0.f;
        }
    }
    __syncthreads();
    double acc[G];
#pragma unroll
    for (int hh = 0; hh < G; ++hh) acc[hh] = 0.0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        const int tb = 8 * sl + 8 * SL * u;  // within the tile
        if (t0 + tb < n_kv) {
            double v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float f = h2f((uint16_t)(vv[u][j >> 1] >> (16 * (j & 1))));
                v[j] = t0 + tb + j < n_kv ? (double)f : 0.0;
            }
#pragma unroll
            for (int hh = 0; hh < G; ++hh) {
                const float4 p0 = *(const float4*)&sp[hh][tb], p1 = *(const float4*)&sp[hh][tb + 4];
                acc[hh] = __builtin_fma(v[0], (double)p0.x, acc[hh]);
                acc[hh] = __builtin_fma(v[1], (double)p0.y, acc[hh]);
                acc[hh] = __builtin_fma(v[2], (double)p0.z, acc[hh]);
                acc[hh] = __builtin_fma(v[3], (double)p0.w, acc[hh]);
                acc[hh] = __builtin_fma(v[4], (double)p1.x, acc[hh]);
                acc[hh] = __builtin_fma(v[5], (double)p1.y, acc[hh]);
                acc[hh] = __builtin_fma(v[6], (double)p1.z, acc[hh]);
                acc[hh] = __builtin_fma(v[7], (double)p1.w, acc[hh]);
            }
        }
    }
    double* part = attl_part(a, n_head);
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        double v = acc[hh];
        v += xor_partner_d<1>(v);
        v += xor_partner_d<2>(v);
        if constexpr (SL == 8) v += xor_partner_d<4>(v);
        if (sl == 0) part[((size_t)(g * G + hh) * ntl + tile) * D + d] = v;
    }
}

template <int D>
__device__ __forceinline__ void attl_sum_body(const AttnArgs& a, int n_head) {
    const int h = blockIdx.x, d = threadIdx.x;
    const int n_kv = a.st->pos + 1;
    const int ntl = (a.n_ctx + kLongTile - 1) / kLongTile, ntv = (n_kv + kLongTile - 1) / kLongTile;
    const double* part = attl_part(a, n_head) + (size_t)h * ntl * D + d;
    // batches of 16 loads in flight, summed in tile order
    double s = 0.0;
    for (int j0 = 0; j0 < ntv; j0 += 16) {
        double v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = part[(size_t)min(j0 + k, ntl - 1) * D];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (j0 + k < ntv) s += v[k];
    }
    a.out[(size_t)h * D + d] = (float)s;
}

// Dim-split one-launch attention (path 6, kv_bound <= 64*P <= 1024): H*S workgroups of
// 512 threads.  Workgroup b serves query head h of KV group g = b % HK and the DS = D/S
// output dims of slice b / H.  Each workgroup recomputes its head's scores and softmax
// in full (no cross-workgroup hand-off) and splits only the PV, so a head's K rows are
// read by S workgroups and its V rows once in total.  Placement: the G*S workgroups of a
// KV group have equal b % HK, i.e. one XCD under round-robin dispatch (HK = 8), so a K
// row comes from HBM once and from that XCD's L2 for the others (default cache policy
// on K and V for that reason).  Every global load is issued at entry, as in k_attn_r;
// numerics are k_attn_r's (exact f16 products summed in double, p = f16(e * (float)(1 /
// sum)), double PV); the per-position work and the PV lane split differ only in how the
// exact double sums are associated.
template <int D, int P, int S>
__device__ __forceinline__ void attn_d_body(const AttnArgs& a, int G, int HK, int kvb, int pf = 0, int rot_on = 0) {
    constexpr int DQ = D / 8;                    // score dims per lane
    constexpr int DS = D / S;                    // output dims of this workgroup
    constexpr int SLV = 512 / DS;                // PV lanes per output dim (<= 64)
    constexpr int NVL = (64 * P + 8 * SLV - 1) / (8 * SLV);  // 16-B V loads per lane
    static_assert(SLV <= 64 && (SLV & (SLV - 1)) == 0, "PV lanes of a dim stay in one wave");
    __shared__ __attribute__((aligned(16))) float sp[64 * P + 8];
    __shared__ float redm[8];
    __shared__ double reds[8];
    LLMI_ATT_STAMP(0, 0)
    const int b = blockIdx.x, H = HK * G;
    const int g = b % HK, h = g * G + (b / HK) % G, ds = b / H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int qd = tid & 7, pp = tid >> 3;
    // 1. every load up front: position, q slice, the K rows of all passes, the V slice.
    // pf (the default): the K passes / V loads past the position are skipped (uniform
    // branches on the position read first) instead of loading the whole KV bucket
    const int pos = a.st->pos;
    const int lim = pf ? pos + 1 : kvb;
    // rot_on (the default): the workgroups of one KV group (one XCD) start their K passes
    // at different positions, so the requests for a K row are spread over the issue window
    // and the later ones hit that XCD's L2 (3-8 % faster, profiles/r02/attn_dim_split.md);
    // register pass p holds positions 64 * pb(p) ...
    const int rot = rot_on ? (b / HK) % P : 0;
    auto pb = [&](int p) { return p + rot < P ? p + rot : p + rot - P; };
    float4 qv[DQ / 4];
#pragma unroll
    for (int i = 0; i < DQ / 4; ++i) qv[i] = *(const float4*)(a.q + (size_t)h * D + qd * DQ + 4 * i);
    u32x4 kv[P][DQ / 8];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int t = min(64 * pb(p) + pp, kvb - 1);
        const uint16_t* kr = a.kc + ((size_t)g * a.n_ctx + t) * D + qd * DQ;
        if (64 * pb(p) < lim) {
#pragma unroll
            for (int i = 0; i < DQ / 8; ++i) kv[p][i] = *(const u32x4*)(kr + 8 * i);
        } else {
#pragma unroll
            for (int i = 0; i < DQ / 8; ++i) kv[p][i] = u32x4{0u, 0u, 0u, 0u};
        }
    }
    const int d = ds * DS + tid / SLV, sl = tid % SLV;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    u32x4 vv[NVL];
#pragma unroll
    for (int u = 0; u < NVL; ++u) {
        if (8 * SLV * u < lim) vv[u] = *(const u32x4*)(vr + min(8 * sl + 8 * SLV * u, kvb - 8));
        else vv[u] = u32x4{0u, 0u, 0u, 0u};
    }
    const int n_kv = pos + 1;
    // 2. scores (q rounded to f16 as upstream's KQ mul_mat does; f16 x f16 products exact)
    double q[DQ];
#pragma unroll
    for (int i = 0; i < DQ / 4; ++i) {
        q[4 * i + 0] = (double)h2f(f2h(qv[i].x)); q[4 * i + 1] = (double)h2f(f2h(qv[i].y));
        q[4 * i + 2] = (double)h2f(f2h(qv[i].z)); q[4 * i + 3] = (double)h2f(f2h(qv[i].w));
    }
    float m = -INFINITY;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        if (64 * pb(p) >= lim) continue;  // uniform: passes past the position (pf only)
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                acc = __builtin_fma((double)h2f((uint16_t)kv[p][i][jj]), q[8 * i + 2 * jj], acc);
                acc = __builtin_fma((double)h2f((uint16_t)(kv[p][i][jj] >> 16)), q[8 * i + 2 * jj + 1], acc);
            }
        acc += xor_partner_d<1>(acc);
        acc += xor_partner_d<2>(acc);
        acc += xor_partner_d<4>(acc);
        const int t = 64 * pb(p) + pp;
        const float sc = (float)acc * a.scale;
        if (qd == 0) sp[t] = sc;
        if (t < n_kv) m = fmaxf(m, sc);
    }
    LLMI_ATT_STAMP(0, 1)
    m = wave_max(m);
    if (lane == 0) redm[wave] = m;
    __syncthreads();
    float mx = redm[0];
#pragma unroll
    for (int w = 1; w < 8; ++w) mx = fmaxf(mx, redm[w]);
    // 3. softmax: thread t owns positions t, t + 512
    constexpr int NE = (64 * P + 511) / 512;
    float e[NE];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int t = tid + 512 * k;
        e[k] = 0.f;
        if (t < n_kv && t < 64 * P) {
            e[k] = llmi_expf(sp[t] - mx);
            s += (double)e[k];
        }
    }
    s = wave_sum_d(s);
    if (lane == 0) reds[wave] = s;
    __syncthreads();
    double tot = reds[0];
#pragma unroll
    for (int w = 1; w < 8; ++w) tot += reds[w];
    const float inv = (float)(1.0 / tot);
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int t = tid + 512 * k;
        if (t < 64 * P) sp[t] = t < n_kv ? h2f(f2h(e[k] * inv)) : 0.f;
    }
    __syncthreads();
    LLMI_ATT_STAMP(0, 2)
    // 4. PV of this workgroup's DS dims: lane sl covers positions 8*sl + 8*SLV*u + j
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int u = 0; u < NVL; ++u) {
        const int tb = 8 * sl + 8 * SLV * u;
        if (tb < n_kv) {
            const float4 p0 = *(const float4*)(sp + tb), p1 = *(const float4*)(sp + tb + 4);
            const float pr[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float f = h2f((uint16_t)(vv[u][j >> 1] >> (16 * (j & 1))));
                const double v = tb + j < n_kv ? (double)f : 0.0;
                if (j & 1) acc1 = __builtin_fma(v, (double)pr[j], acc1);
                else acc0 = __builtin_fma(v, (double)pr[j], acc0);
            }
        }
    }
    double acc = acc0 + acc1;
    if constexpr (SLV >= 2) acc += xor_partner_d<1>(acc);
    if constexpr (SLV >= 4) acc += xor_partner_d<2>(acc);
    if constexpr (SLV >= 8) acc += xor_partner_d<4>(acc);
    if constexpr (SLV >= 16) acc += xor_partner_d<8>(acc);
    if constexpr (SLV >= 32) acc += xor_partner_d<16>(acc);
    if constexpr (SLV >= 64) acc += xor_partner_d<32>(acc);
    if (sl == 0) a.out[(size_t)h * D + d] = (float)acc;
    LLMI_ATT_STAMP(0, 3)
}

}  // namespace llmi
