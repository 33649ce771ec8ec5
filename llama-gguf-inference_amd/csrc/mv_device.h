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
// f16 ulp, tools/pf_diag9.py).
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
// steps in the order 1, 2, 4, 8, 16, 32; the oracle's device order models exactly that.
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
// LDS image of the quantized activation, in the weights' chunk-part order (common.h):
//   K-quants (block_q8_K): LO[k][ch], HI[k][ch]: 16 int8 each = activation of the
//     weights in the low / high nibbles of quant part k of chunk ch, in residue order:
//     byte 4m + i of part k = chunk element l + 8i (LO) / 32 + l + 8i (HI), l = 4k + m;
//     BS[4ch+i] = bsums in natural order; D[b] per 256-block.
//   Q8_0 (block_q8_0): LO[k][ch] (k < 4) = elements 64ch+16k..+15; D[b] per 32-block
//     (f16-rounded, as stored by quantize_row_q8_0).
// Lane L reads LO[k][L + 64j]: 16 consecutive 16-B slots per ds_read_b128 lane group,
// conflict-free.
// ----------------------------------------------------------------------------------
struct Lds {
    uint8_t* lo;
    uint8_t* hi;
    int16_t* bs;
    float* d;
    double* red;
};
__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }
// byte offsets of the regions; act 0 = q8_K (K-quant weights), 1 = q8_0
__host__ __device__ inline size_t lds_hi_off(int act, int cols) { return act ? (size_t)cols : (size_t)cols / 2; }
__host__ __device__ inline size_t lds_bs_off(int act, int cols) { return (size_t)cols; }
__host__ __device__ inline size_t lds_d_off(int act, int cols) { return a16((size_t)cols + (act ? 0 : (size_t)cols / 8)); }
__host__ __device__ inline size_t lds_red_off(int act, int cols) {
    return a16(lds_d_off(act, cols) + (size_t)(act ? cols / 32 : cols / 256) * 4);
}
// (mv_lds_bytes: defined in kernels.hip)

__device__ __forceinline__ Lds carve(uint8_t* smem, int act, int cols) {
    Lds l;
    l.lo = smem;
    l.hi = smem + lds_hi_off(act, cols);
    l.bs = (int16_t*)(smem + lds_bs_off(act, cols));
    l.d = (float*)(smem + lds_d_off(act, cols));
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
template <int ACT>
__device__ __forceinline__ void quant_sub(const Lds& L, int cols, int sb, const float (&v)[16]) {
    const int tid = threadIdx.x;
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
        // sub-block sb = chunk ch = sb/4, quarter qq = sb%4: half h = qq/2 (LO / HI image),
        // elements tt = 16*(qq%2) + j of the half.  Residue order (common.h): element tt of
        // a half sits at part k = l/4, byte 4*(l%4) + i with l = tt%8, i = tt/8, so q[j]
        // and q[j+8] (same l, i = 2*(qq%2) + 0/1) are one 16-bit store.
        const int nch = cols >> 6, ch = sb >> 2, qq = sb & 3;
        const int hoff = qq < 2 ? 0 : (int)(L.hi - L.lo);  // (no pointer select: it spills to scratch)
        uint8_t* base = L.lo + hoff + 16 * ch + 2 * (qq & 1);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            *(uint16_t*)(base + 16 * nch * (j >> 2) + 4 * (j & 3)) =
                (uint16_t)((q[j] & 0xff) | ((q[j + 8] & 0xff) << 8));
        L.bs[sb] = (int16_t)bsum;
        if ((tid & 15) == 0) L.d[sb >> 4] = dval;
    } else {
        float am = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[j]));
        am = fmaxf(am, xor_partner<1>(am));
        const float d = am / 127;
        const float id = d != 0.f ? 1.0f / d : 0.0f;
#pragma unroll
        for (int j = 0; j < 16; ++j) q[j] = (int)roundf(v[j] * id);
        if ((tid & 1) == 0) L.d[sb >> 1] = h2f(f2h(d));
        const int nch = cols >> 6;
        u32x4 pk;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            pk[w] = (uint32_t)(q[4 * w] & 0xff) | ((uint32_t)(q[4 * w + 1] & 0xff) << 8) |
                    ((uint32_t)(q[4 * w + 2] & 0xff) << 16) | ((uint32_t)(q[4 * w + 3] & 0xff) << 24);
        *(u32x4*)(L.lo + 16 * ((sb & 3) * nch + (sb >> 2))) = pk;
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
template <int ACT, bool NORM, int NP, int NT = kMVThreads>
__device__ __forceinline__ void mv_prologue_finish(const MVArgs& A, const Lds& L, const ProRegs<NORM, NP>& R) {
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
            quant_sub<ACT>(L, cols, sb, v);
        }
    }
    for (int sb = tid + NP * NT; sb < nsub; sb += NT) {
        float v[16], w[16];
        load_sub<NORM, NP>(A, R, NP, sb, v, w);
        if constexpr (NORM) {
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = (v[j] * scale) * w[j];
        }
        quant_sub<ACT>(L, cols, sb, v);
    }
}
template <int ACT, bool NORM>
__device__ __forceinline__ void mv_prologue(const MVArgs& A, const Lds& L) {
    ProRegs<NORM, 1> R;
    mv_prologue_issue<NORM, 1>(A, R);
    mv_prologue_finish<ACT, NORM, 1>(A, L, R);
}

// ----------------------------------------------------------------------------------
// Per-type 64-weight chunk: load (global) and integer dot against the LDS activation
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
// 4 bits -> the low bit of 4 bytes
__device__ __forceinline__ uint32_t spread4(uint32_t x) { return (x * 0x00204081u) & M1; }

template <int T>
__host__ __device__ constexpr int kparts() { return T == T_Q8_0 ? 4 : 2; }

// One chunk of one row in registers.
struct Raw {
    u32x4 q0, q1, q2, q3;  // quant parts (q2, q3: Q8_0 only)
    u32x4 hdr;             // Q4_K/Q5_K block header; Q6_K: 2-bit highs (4 dwords)
    u32x2 qh;              // Q5_K fifth bits (lo 32, hi 32)
    uint32_t e0;           // Q6_K chunk scales (4 x int8); Q8_0: the two fp16 d
    uint32_t e1;           // Q6_K fp16 d
};

// Row view: uniform per-row base pointers (SGPRs) so per-lane addressing is a small
// 32-bit offset: quant part k of chunk ch at qa + (k*nch + ch)*16.
struct RowPtr {
    const uint8_t* qa;  // A plane, this row
    const uint8_t* hb;  // H plane, this row
    const uint8_t* sb;  // S plane, this row
    const uint8_t* db;  // D plane, this row
};
template <int T>
__device__ __forceinline__ RowPtr row_ptr(const Seg& s, int row, int cols) {
    RowPtr r;
    const size_t nch = (size_t)(cols >> 6), nblk = (T == T_Q8_0) ? (size_t)(cols >> 5) : (size_t)(cols >> 8);
    r.qa = s.a + (size_t)row * nch * (T == T_Q8_0 ? 64 : 32);
    r.hb = s.h + (size_t)row * nch * (T == T_Q6_K ? 16 : 8);
    r.sb = s.s + (size_t)row * nblk * 16;
    r.db = s.d + (size_t)row * nblk * 2;
    return r;
}

template <int T>
__device__ __forceinline__ Raw load_chunk(const RowPtr& rp, int ch, int nch) {
    Raw r;
    const uint32_t o = (uint32_t)ch * 16, step = (uint32_t)nch * 16;
    r.q0 = ldw(rp.qa + o);
    r.q1 = ldw(rp.qa + o + step);
    if constexpr (T == T_Q4_K || T == T_Q5_K) {
        // the block header is shared by the 4 lanes of a block: default policy (nt loads
        // of duplicated addresses were fetched once per lane: +24 % FETCH_SIZE)
        r.hdr = *(const u32x4*)(rp.sb + (uint32_t)(ch >> 2) * 16);
        if constexpr (T == T_Q5_K) r.qh = ldw8(rp.hb + (uint32_t)ch * 8);
    } else if constexpr (T == T_Q6_K) {
        r.hdr = ldw(rp.hb + (uint32_t)ch * 16);
        r.e0 = ldw4(rp.sb + (uint32_t)ch * 4);
        r.e1 = *(const uint16_t*)(rp.db + (uint32_t)(ch >> 2) * 2);
    } else {
        r.q2 = ldw(rp.qa + o + 2 * step);
        r.q3 = ldw(rp.qa + o + 3 * step);
        r.e0 = ldw4(rp.db + (uint32_t)ch * 4);
    }
    return r;
}

struct Act {
    i32x4 a0, a1, a2, a3;  // K: lo part 0, lo part 1, hi part 0, hi part 1; Q8_0: parts 0..3
    int bs[4];
    float d0, d1;
};
template <int ACT>
__device__ __forceinline__ Act load_act(const Lds& L, int ch, int nch) {
    Act a;
    const int step = nch * 16;
    a.a0 = *(const i32x4*)(L.lo + 16 * ch);
    a.a1 = *(const i32x4*)(L.lo + 16 * ch + step);
    if constexpr (ACT == 0) {
        a.a2 = *(const i32x4*)(L.hi + 16 * ch);
        a.a3 = *(const i32x4*)(L.hi + 16 * ch + step);
        const uint2 bw = *(const uint2*)(L.bs + 4 * ch);
        a.bs[0] = (int16_t)(bw.x & 0xffff); a.bs[1] = (int16_t)(bw.x >> 16);
        a.bs[2] = (int16_t)(bw.y & 0xffff); a.bs[3] = (int16_t)(bw.y >> 16);
        a.d0 = L.d[ch >> 2];
    } else {
        a.a2 = *(const i32x4*)(L.lo + 16 * ch + 2 * step);
        a.a3 = *(const i32x4*)(L.lo + 16 * ch + 3 * step);
        const float2 dd = *(const float2*)(L.d + 2 * ch);
        a.d0 = dd.x;
        a.d1 = dd.y;
    }
    return a;
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
// Device mapping.  Lane L of a wave holds chunk L (+64 j) of the wave's two rows.
//   chunk_isum  the chunk's integer sums by residue l (the residue-order layout makes
//               every sdot4 a same-residue dot: t[l] = sc0*dot(lo) + sc1*dot(hi))
//   quad        the 4 chunks of block b are lanes 4b..4b+3; a reduce-scatter over the
//               quad leaves residues 2c, 2c+1 of the block's aux32 in lane c
//   item_terms  the block's fp32 terms d*(float)aux32[l] and -(dmin*(float)sumi) go to
//               the wave's LDS fold buffer F[row][chain][block]
//   fold_item   18 fold lanes (2 rows x 9 chains; Q8_0: 2 lanes, one chain) add the
//               item's terms block after block onto their running chain
//   fold_final  sumf chain + sums[0..7] in order, both rows, every lane
// ----------------------------------------------------------------------------------
struct PairSum {
    float a, b;
};
constexpr int kFoldRow = 144;                     // floats per row: 9 chains x 16 blocks (Q8_0: 128 blocks)
constexpr int kFoldFloats = 2 * kFoldRow + 32;   // + the chain results G[18] (padded)

// LDS accesses of one wave handed between its own lanes: LDS executes a wave's
// instructions in order, so only the compiler must not move accesses across this point
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

struct ISum {
    int t[8];   // K-quants: per-residue sums of the chunk; Q8_0: t[0], t[1] = its two 32-block sums
    int imin;   // Q4_K/Q5_K: min term of the chunk (m0*(bs0+bs1) + m1*(bs2+bs3)); else 0
};

// Q6_K high bits are stored XOR 2 (common.h): v_perm maps them straight to the signed
// high part of q - 32 ({0x00, 0x10, 0xE0, 0xF0} for stored 0..3)
__device__ __forceinline__ uint32_t q6_hi_bytes(uint32_t sel) { return __builtin_amdgcn_perm(0xF0E01000u, 0xF0E01000u, sel); }

template <int T>
__device__ __forceinline__ ISum chunk_isum(const Raw& r, const Act& a, int ch) {
    ISum s;
    s.imin = 0;
    if constexpr (T == T_Q4_K || T == T_Q5_K) {
        const int c = ch & 3;
        int sc0, m0, sc1, m1;
        scale_min(2 * c, r.hdr.y, r.hdr.z, r.hdr.w, sc0, m0);
        scale_min(2 * c + 1, r.hdr.y, r.hdr.z, r.hdr.w, sc1, m1);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const u32x4 q = k ? r.q1 : r.q0;
            const i32x4 al = k ? a.a1 : a.a0, ah = k ? a.a3 : a.a2;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                uint32_t l4 = q[m] & M4, h4 = (q[m] >> 4) & M4;
                if constexpr (T == T_Q5_K) {
                    l4 |= spread4((r.qh.x >> (16 * k + 4 * m)) & 0xFu) << 4;
                    h4 |= spread4((r.qh.y >> (16 * k + 4 * m)) & 0xFu) << 4;
                }
                // |dot| <= 4*31*127: 24-bit multiplies are exact
                s.t[4 * k + m] = __mul24(sc0, dot4(l4, al[m], 0)) + __mul24(sc1, dot4(h4, ah[m], 0));
            }
        }
        s.imin = m0 * (a.bs[0] + a.bs[1]) + m1 * (a.bs[2] + a.bs[3]);
    } else if constexpr (T == T_Q6_K) {
        // bytes 0,1 of a dword are elements l, l+8 (sub-block 4c + 2h), bytes 2,3 are
        // l+16, l+24 (sub-block 4c + 2h + 1): one masked sdot4 per sub-block
        const int c0 = (int)(int8_t)(r.e0 & 0xff), c1 = (int)(int8_t)((r.e0 >> 8) & 0xff),
                  c2 = (int)(int8_t)((r.e0 >> 16) & 0xff), c3 = (int)(int8_t)(r.e0 >> 24);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const u32x4 q = k ? r.q1 : r.q0;
            const i32x4 al = k ? a.a1 : a.a0, ah = k ? a.a3 : a.a2;
            const uint32_t hl = r.hdr[k], hh = r.hdr[2 + k];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t wl = (q[m] & M4) | q6_hi_bytes((hl >> (2 * m)) & M2);
                const uint32_t wh = ((q[m] >> 4) & M4) | q6_hi_bytes((hh >> (2 * m)) & M2);
                const int s0 = dot4(wl, al[m] & 0xffff, 0), s1 = dot4(wl, al[m] & (int)0xffff0000u, 0);
                const int s2 = dot4(wh, ah[m] & 0xffff, 0), s3 = dot4(wh, ah[m] & (int)0xffff0000u, 0);
                // |s| <= 2*32*127, |c| <= 128: exact in 24-bit multiplies
                s.t[4 * k + m] = __mul24(c0, s0) + __mul24(c1, s1) + __mul24(c2, s2) + __mul24(c3, s3);
            }
        }
    } else {
        int s0 = 0, s1 = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            s0 = dot4(r.q0[m], a.a0[m], s0);
            s0 = dot4(r.q1[m], a.a1[m], s0);
            s1 = dot4(r.q2[m], a.a2[m], s1);
            s1 = dot4(r.q3[m], a.a3[m], s1);
        }
        s.t[0] = s0;
        s.t[1] = s1;
    }
    return s;
}

// Quad reduce-scatter of the block's per-residue sums (lanes 4b..4b+3): lane c keeps
// residues 2c, 2c+1 (a0, a1); the min term is summed into every lane of the quad.
__device__ __forceinline__ void quad_scatter(ISum& s, int& a0, int& a1) {
    const bool b0 = (threadIdx.x & 1) != 0, b1 = (threadIdx.x & 2) != 0;
    // level 1 (lane ^ 1): keep residue pairs b0 and b0 + 2
    int k[4];
    {
        const int s0 = b0 ? s.t[0] : s.t[2], s1 = b0 ? s.t[1] : s.t[3];
        const int s2 = b0 ? s.t[4] : s.t[6], s3 = b0 ? s.t[5] : s.t[7];
        k[0] = (b0 ? s.t[2] : s.t[0]) + xor_partner_i<1>(s0);
        k[1] = (b0 ? s.t[3] : s.t[1]) + xor_partner_i<1>(s1);
        k[2] = (b0 ? s.t[6] : s.t[4]) + xor_partner_i<1>(s2);
        k[3] = (b0 ? s.t[7] : s.t[5]) + xor_partner_i<1>(s3);
    }
    // level 2 (lane ^ 2): keep pair b0 + 2*b1 = c
    const int r0 = b1 ? k[0] : k[2], r1 = b1 ? k[1] : k[3];
    a0 = (b1 ? k[2] : k[0]) + xor_partner_i<2>(r0);
    a1 = (b1 ? k[3] : k[1]) + xor_partner_i<2>(r1);
    s.imin += xor_partner_i<1>(s.imin);
    s.imin += xor_partner_i<2>(s.imin);
}

// The item's fp32 terms of one row into its fold buffer Fr (chain ch, block bi at
// Fr[ch * 16 + bi]; Q8_0: Fr[bi], 128 blocks).  Every lane calls it (cross-lane ops);
// `valid` (the chunk exists) guards only the stores — chunks past the row come in whole
// blocks (cols % 256 == 0).
template <int T>
__device__ __forceinline__ void item_terms(const Raw& r, const Act& a, int ch, bool valid, float* Fr) {
    ISum s = chunk_isum<T>(r, a, ch);
    const int lane = threadIdx.x & 63;
    if constexpr (T == T_Q8_0) {
        const float t0 = (float)s.t[0] * (h2f(r.e0) * a.d0), t1 = (float)s.t[1] * (h2f(r.e0 >> 16) * a.d1);
        if (valid) *(float2*)(Fr + 2 * lane) = make_float2(t0, t1);
    } else {
        int a0, a1;
        quad_scatter(s, a0, a1);
        const int c = lane & 3, bi = lane >> 2;
        const float d = (T == T_Q6_K ? h2f(r.e1) : h2f(r.hdr.x)) * a.d0;
        const float p0 = d * (float)a0, p1 = d * (float)a1;
        float nq = 0.f;
        if constexpr (T != T_Q6_K) nq = -((h2f(r.hdr.x >> 16) * a.d0) * (float)s.imin);
        if (valid) {
            Fr[(2 * c) * 16 + bi] = p0;
            Fr[(2 * c + 1) * 16 + bi] = p1;
            if (c == 0) Fr[8 * 16 + bi] = nq;  // Q6_K: no min chain (+0 terms, as sumf = 0)
        }
    }
}

// blocks of item j of a row of `cols` weights (K-quants: 16 per item, Q8_0: 128)
template <int ACT>
__device__ __forceinline__ int item_blocks(int cols, int j) {
    const int nb = ACT ? (cols >> 5) - 128 * j : (cols >> 8) - 16 * j;
    const int per = ACT ? 128 : 16;
    return nb < per ? nb : per;
}

// Fold lane f (< 18, Q8_0 < 2) adds chain f's terms of nb blocks in block order.
template <int ACT>
__device__ __forceinline__ void fold_item(const float* F, int nb, float& acc) {
    constexpr int NC = ACT ? 1 : 9, CS = ACT ? 128 : 16;
    const int lane = threadIdx.x & 63;
    if (lane < 2 * NC) {
        const int r = lane >= NC ? 1 : 0;
        const float* p = F + r * kFoldRow + (lane - r * NC) * CS;
        for (int b = 0; b < nb; b += 4) {
            const float4 v = *(const float4*)(p + b);
            acc += v.x;
            if (b + 1 < nb) acc += v.y;
            if (b + 2 < nb) acc += v.z;
            if (b + 3 < nb) acc += v.w;
        }
    }
}

// Both rows' final sums in every lane: sumf chain, then += sums[0..7] (K-quants).
template <int ACT>
__device__ __forceinline__ PairSum fold_final(float* F, float acc) {
    constexpr int NC = ACT ? 1 : 9;
    float* G = F + 2 * kFoldRow;
    const int lane = threadIdx.x & 63;
    wave_lds_sync();
    if (lane < 2 * NC) G[lane] = acc;
    wave_lds_sync();
    PairSum v;
    if constexpr (ACT) {
        v.a = G[0];
        v.b = G[1];
    } else {
        float sa = G[8], sb = G[17];
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            sa += G[l];
            sb += G[9 + l];
        }
        v.a = sa;
        v.b = sb;
    }
    wave_lds_sync();
    return v;
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

template <int T>
struct PairRaw {
    Raw a, b;
};
template <int T>
struct PairRows {
    RowPtr a, b;
};

template <int T>
__device__ __forceinline__ PairRows<T> pair_rows(const PairRef& r, int cols) {
    PairRows<T> pr;
    pr.a = row_ptr<T>(r.sa, r.ra, cols);
    pr.b = row_ptr<T>(r.sb, r.vb ? r.rb : r.ra, cols);
    return pr;
}

// Unconditional loads (the chunk index is clamped to a valid one; callers discard the
// contribution of out-of-range lanes): straight-line code lets the compiler count
// vmcnt exactly, so the next item's loads stay in flight while this one is reduced.
template <int T>
__device__ __forceinline__ PairRaw<T> load_item(const PairRows<T>& pr, int ch, int nch) {
    PairRaw<T> w;
    const int c = ch < nch ? ch : nch - 1;
    w.a = load_chunk<T>(pr.a, c, nch);
    w.b = load_chunk<T>(pr.b, c, nch);
    return w;
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
template <int EPI, bool WT = false, class MA, bool ANY_LANE = false>
__device__ __forceinline__ void epilogue(const MA& A, const PairRef& r, int p, PairSum v, int pos,
                                         unsigned long long& best) {
    const int lane = threadIdx.x & 63;
    const float va = v.a, vb = v.b;
    if (!ANY_LANE && lane != 0) return;
    if constexpr (EPI == EPI_STORE) {
        st_f32<WT>(A.y + r.sa.row0 + r.ra, va);
        if (r.vb) st_f32<WT>(A.y + r.sa.row0 + r.rb, vb);
    } else if constexpr (EPI == EPI_ADD) {
        float* ya = A.y + r.sa.row0 + r.ra;
        st_f32<WT>(ya, ld_f32<WT>(ya) + va);
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
        st_f32<WT>(A.y + p, llmi_silu(va) * vb);
    } else if constexpr (EPI == EPI_QKV) {
        // sa.row0 tells q (0), k (nq) or v (nq+nk); rows (ra, ra+1) are a RoPE pair
        const int hd = A.head_dim;
        const int h = r.ra / hd, d = r.ra - h * hd;
        if (r.sa.row0 < A.nq + A.nk) {
            float o0 = va, o1 = vb;
            if (d < A.n_rot) {  // ggml rope NORM mode on the adjacent pair (d, d+1)
                const float2 cs = *(const float2*)(A.rope + ((size_t)pos * (A.n_rot / 2) + d / 2) * 2);
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

// Non-pipelined fallback for pairs whose type is not the kernel's primary type (the
// Q6_K attn_v segment inside a Q4_K QKV launch, mixed-type gate/up pairs): the same
// terms and fold, one item at a time, each row in its own type.
template <int ACT, int T>
__device__ __forceinline__ void row_terms(const Seg& s, int row, int cols, int ch, const Act& act, float* Fr) {
    const int nch = cols >> 6;
    const RowPtr rp = row_ptr<T>(s, row, cols);
    const int chc = ch < nch ? ch : nch - 1;
    item_terms<T>(load_chunk<T>(rp, chc, nch), act, chc, ch < nch, Fr);
}
template <int ACT>
__device__ __forceinline__ void row_terms_any(int type, const Seg& s, int row, int cols, int ch, const Act& act,
                                              float* Fr) {
    if constexpr (ACT == 1) {
        row_terms<1, T_Q8_0>(s, row, cols, ch, act, Fr);
    } else {
        switch (type) {
            case T_Q4_K: row_terms<0, T_Q4_K>(s, row, cols, ch, act, Fr); break;
            case T_Q5_K: row_terms<0, T_Q5_K>(s, row, cols, ch, act, Fr); break;
            case T_Q6_K: row_terms<0, T_Q6_K>(s, row, cols, ch, act, Fr); break;
            default: break;
        }
    }
}
template <int ACT>
__device__ __forceinline__ PairSum pair_any(const PairRef& r, int cols, const Lds& L, float* F) {
    const int nch = cols >> 6, NJ = (nch + 63) >> 6;
    const int lane = threadIdx.x & 63;
    float acc = 0.f;
    for (int j = 0; j < NJ; ++j) {
        const int ch = lane + 64 * j, chc = ch < nch ? ch : nch - 1;
        const Act act = load_act<ACT>(L, chc, nch);
        row_terms_any<ACT>(r.sa.type, r.sa, r.ra, cols, ch, act, F);
        row_terms_any<ACT>(r.sb.type, r.sb, r.vb ? r.rb : r.ra, cols, ch, act, F + kFoldRow);
        wave_lds_sync();
        fold_item<ACT>(F, item_blocks<ACT>(cols, j), acc);
        wave_lds_sync();
    }
    return fold_final<ACT>(F, acc);
}

// get_rows: element e of row `row` dequantized from the device layout (bit-exact with
// upstream dequantize_row_*)
__device__ __forceinline__ float dequant_elem(const Seg& w, int row, int e, int cols) {
    switch (w.type) {
        case T_F32: return ((const float*)w.a)[(size_t)row * cols + e];
        case T_F16: return h2f(((const uint16_t*)w.a)[(size_t)row * cols + e]);
        case T_Q4_K:
        case T_Q5_K:
        case T_Q6_K: {
            // residue order (common.h): chunk element t = 32 hi + l + 8 i sits in part
            // k = l / 4, byte 4 (l % 4) + i (low nibble: hi = 0, high nibble: hi = 1)
            const int nch = cols >> 6, nbr = cols >> 8;
            const int ch = e >> 6, t = e & 63, hi = t >= 32, l = t & 7, i = (t & 31) >> 3, k = l >> 2, m = l & 3;
            const size_t gb = (size_t)row * nbr + (e >> 8);
            const uint8_t qb = w.a[(size_t)row * nch * 32 + (size_t)(k * nch + ch) * 16 + 4 * m + i];
            int q = hi ? (qb >> 4) : (qb & 0xF);
            if (w.type == T_Q6_K) {  // H dword (2*hi + k), byte i, bits 2m: the 2 high bits XOR 2
                const uint8_t hb = w.h[((size_t)row * nch + ch) * 16 + (2 * hi + k) * 4 + i];
                q |= (((hb >> (2 * m)) & 3) ^ 2) << 4;
                const float d = h2f(*(const uint16_t*)(w.d + gb * 2));
                const int sc = (int8_t)w.s[gb * 16 + ((e & 255) >> 4)];
                return d * (float)sc * (float)(q - 32);
            }
            const uint32_t* s32 = (const uint32_t*)(w.s + gb * 16);
            int sc, mn;
            scale_min(2 * (ch & 3) + hi, s32[1], s32[2], s32[3], sc, mn);
            if (w.type == T_Q5_K) q += ((ldw4(w.h + ((size_t)row * nch + ch) * 8 + 4 * hi) >> (4 * l + i)) & 1) << 4;
            const float d = h2f(s32[0]), dmin = h2f(s32[0] >> 16);
            const float d1 = d * (float)sc, m1 = dmin * (float)mn;
            return d1 * (float)q - m1;
        }
        case T_Q8_0: {
            const int nch = cols >> 6, ch = e >> 6, t = e & 63;
            const uint8_t qb = w.a[(size_t)row * nch * 64 + (size_t)((t >> 4) * nch + ch) * 16 + (t & 15)];
            return (float)(int8_t)qb * h2f(*(const uint16_t*)(w.d + ((size_t)row * (cols / 32) + e / 32) * 2));
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
