// kernels.hip — gfx950 (CDNA4, wave64) kernels of the GGUF K-quant decode step.
//
// The hot path of SURVEY.md §8(a): per token, every linear layer is a quantized
// matrix-vector product that streams the whole weight matrix from HBM once (rows
// a6-a9, ~100% of the bytes), wrapped by the small fused ops a5 (activation
// quantization), a10-a15.  Design:
//
//   k_matvec  one launch per fused weight group (QKV, O, gate+up, down, output head).
//     prologue  every workgroup re-derives the quantized activation in LDS from the
//               f32 input (L2/MALL-resident, 16-57 KB): optional RMSNorm (double sum, as
//               ggml_compute_forward_rms_norm) then quantize_row_q8_K_ref /
//               quantize_row_q8_0_ref, bit-exactly.  This replaces a separate
//               norm+quantize launch (a 1.2-1.9 us dependent-kernel boundary on MI355X).
//     body      a wave owns a PAIR of rows; lane L owns pieces L, L+64, ... of both rows
//               (a piece = 32 weights, common.h): 16-B loads that cover 1 KiB of
//               consecutive bytes per wave instruction, integer v_dot4c_i32_i8 against
//               the LDS activation (stored in the same piece order: conflict-free
//               ds_read_b128), exact int32 per-piece sums combined in fp32 as
//               ggml_vec_dot_*_q8_K does (d_w*d_a*isum - dmin_w*d_a*imin), then a
//               64-lane butterfly.  The next piece's weights are in flight while the
//               current one is reduced, and a wave's first piece is issued before the
//               prologue so HBM latency overlaps it.
//     epilogue  store / residual add / RoPE + f16 KV write / SwiGLU / logits + argmax.
//   k_attn_*   decode attention over the f16 KV cache with ggml's non-flash numerics.
//   k_embed    token selection (host token or previous argmax) + get_rows dequant.
//   k_repack_* one-time load-time layout transforms (common.h).
#include "kernels.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

namespace llmi {

// Launch-event hook (llmi_profile_kernels): while armed, the timed launches record
// `start` when the first kernel of the op begins and `stop` when the last one ends
// (hipExtLaunchKernelGGL), i.e. kernel execution time without dependent-launch gaps.
static thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
void set_launch_events(hipEvent_t start, hipEvent_t stop) {
    t_ev_start = start;
    t_ev_stop = stop;
}
template <typename K, typename... Args>
static void launch_k(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, bool first, bool last, Args... args) {
    hipEvent_t e0 = first ? t_ev_start : nullptr, e1 = last ? t_ev_stop : nullptr;
    if (e0 || e1) hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, s, e0, e1, 0, args...);
    else hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}


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
//     weights in the low / high nibbles of quant part k of chunk ch (chunk weights
//     16k..16k+15 and 32+16k..32+16k+15); BS[4ch+i] = bsums in natural order;
//     D[b] per 256-block.
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
size_t mv_lds_bytes(int act, int cols) { return lds_red_off(act, cols) + kMVWaves * sizeof(double); }

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
    uint8_t* dst;
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
        // sub-block sb = chunk ch = sb/4, quarter qq = sb%4: lo part k=qq (qq<2), hi part k=qq-2
        const int nch = cols >> 6, ch = sb >> 2, qq = sb & 3;
        const int hoff = qq < 2 ? 0 : (int)(L.hi - L.lo);  // (no pointer select: it spills to scratch)
        dst = L.lo + hoff + 16 * ((qq & 1) * nch + ch);
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
        dst = L.lo + 16 * ((sb & 3) * nch + (sb >> 2));
    }
    u32x4 pk;
#pragma unroll
    for (int w = 0; w < 4; ++w)
        pk[w] = (uint32_t)(q[4 * w] & 0xff) | ((uint32_t)(q[4 * w + 1] & 0xff) << 8) |
                ((uint32_t)(q[4 * w + 2] & 0xff) << 16) | ((uint32_t)(q[4 * w + 3] & 0xff) << 24);
    *(u32x4*)dst = pk;
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

// ggml_vec_dot_<T>_q8_K restricted to one 64-weight chunk; exact int32 sums, fp32
// combine exactly as ggml's per-block formula (d_w*d_a*isum - dmin_w*d_a*imin).
template <int T>
__device__ __forceinline__ float dot_chunk(const Raw& r, const Act& a, int ch) {
    if constexpr (T == T_Q4_K || T == T_Q5_K) {
        const int c = ch & 3;
        int sc0, m0, sc1, m1;
        scale_min(2 * c, r.hdr.y, r.hdr.z, r.hdr.w, sc0, m0);
        scale_min(2 * c + 1, r.hdr.y, r.hdr.z, r.hdr.w, sc1, m1);
        int lo = 0, hi = 0;
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
                lo = dot4(l4, al[m], lo);
                hi = dot4(h4, ah[m], hi);
            }
        }
        const int isum = sc0 * lo + sc1 * hi;
        const int imin = m0 * (a.bs[0] + a.bs[1]) + m1 * (a.bs[2] + a.bs[3]);
        const float d = h2f(r.hdr.x), dmin = h2f(r.hdr.x >> 16);
        return (d * a.d0) * (float)isum - (dmin * a.d0) * (float)imin;
    } else if constexpr (T == T_Q6_K) {
        int dm[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const u32x4 q = k ? r.q1 : r.q0;
            const i32x4 al = k ? a.a1 : a.a0, ah = k ? a.a3 : a.a2;
            const uint32_t hl = r.hdr[k], hh = r.hdr[2 + k];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t ulo = (q[m] & M4) | (((hl >> (2 * m)) & M2) << 4);
                const uint32_t uhi = ((q[m] >> 4) & M4) | (((hh >> (2 * m)) & M2) << 4);
                dm[k] = dot4(ulo, al[m], dm[k]);
                dm[2 + k] = dot4(uhi, ah[m], dm[2 + k]);
            }
        }
        int isum = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m) isum += (int)(int8_t)(r.e0 >> (8 * m)) * (dm[m] - 32 * a.bs[m]);
        return (h2f(r.e1) * a.d0) * (float)isum;
    } else {
        int s0 = 0, s1 = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            s0 = dot4(r.q0[m], a.a0[m], s0);
            s0 = dot4(r.q1[m], a.a1[m], s0);
            s1 = dot4(r.q2[m], a.a2[m], s1);
            s1 = dot4(r.q3[m], a.a3[m], s1);
        }
        return (float)s0 * (h2f(r.e0) * a.d0) + (float)s1 * (h2f(r.e0 >> 16) * a.d1);
    }
}

__device__ __forceinline__ Seg pick(const MVArgs& A, int si) {
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
    bool vb;
    int type;  // common type of both rows, or -1 if they differ
};

template <int EPI>
__device__ __forceinline__ PairRef pair_ref(const MVArgs& A, int p) {
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

// Row sums of a pair: one 64-lane butterfly per row (steps 1,2,4,8,16,32; DPP and
// permlane swaps, no LDS), the oracle's device order models this tree exactly.
struct PairSum {
    float a, b;
};
__device__ __forceinline__ PairSum reduce_pair(float acc_a, float acc_b) {
    return {wave_sum(acc_a), wave_sum(acc_b)};
}

// ordered key of (logit, row): larger logit wins, ties -> smaller row (first max wins,
// as upstream llama_sampler_greedy's strict '>' scan)
__device__ __forceinline__ unsigned long long argmax_key(float v, int row) {
    if (v == 0.f) v = 0.f;  // -0 == +0
    uint32_t u = __float_as_uint(v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (unsigned long long)(0xffffffffu - (uint32_t)row);
}

// Epilogue of one finished pair (every lane holds both row sums; lane 0 writes).
template <int EPI>
__device__ __forceinline__ void epilogue(const MVArgs& A, const PairRef& r, int p, PairSum v, int pos,
                                         unsigned long long& best) {
    const int lane = threadIdx.x & 63;
    const float va = v.a, vb = v.b;
    if (lane != 0) return;
    if constexpr (EPI == EPI_STORE) {
        A.y[r.sa.row0 + r.ra] = va;
        if (r.vb) A.y[r.sa.row0 + r.rb] = vb;
    } else if constexpr (EPI == EPI_ADD) {
        A.y[r.sa.row0 + r.ra] += va;
        if (r.vb) A.y[r.sa.row0 + r.rb] += vb;
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
        A.y[p] = llmi_silu(va) * vb;
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
                A.y[r.ra] = o0;
                A.y[r.ra + 1] = o1;
            } else {
                const uint32_t w = (uint32_t)f2h(o0) | ((uint32_t)f2h(o1) << 16);
                *(uint32_t*)(A.kc + ((size_t)h * A.n_ctx + pos) * hd + d) = w;
            }
        } else {
            A.vc[((size_t)h * hd + d) * A.n_ctx + pos] = f2h(va);
            A.vc[((size_t)h * hd + d + 1) * A.n_ctx + pos] = f2h(vb);
        }
    }
}

// Non-pipelined fallback for pairs whose type is not the kernel's primary type (the
// Q6_K attn_v segment inside a Q4_K QKV launch, mixed-type gate/up pairs).
template <int ACT, int T>
__device__ __forceinline__ float generic_row(const Seg& s, int row, int cols, const Lds& L) {
    const int nch = cols >> 6;
    const RowPtr rp = row_ptr<T>(s, row, cols);
    float acc = 0.f;
    for (int ch = threadIdx.x & 63; ch < nch; ch += 64) {
        const Raw w = load_chunk<T>(rp, ch, nch);
        acc += dot_chunk<T>(w, load_act<ACT>(L, ch, nch), ch);
    }
    return acc;
}
template <int ACT>
__device__ __forceinline__ float generic_row_any(int type, const Seg& s, int row, int cols, const Lds& L) {
    if constexpr (ACT == 1) {
        return generic_row<1, T_Q8_0>(s, row, cols, L);
    } else {
        switch (type) {
            case T_Q4_K: return generic_row<0, T_Q4_K>(s, row, cols, L);
            case T_Q5_K: return generic_row<0, T_Q5_K>(s, row, cols, L);
            case T_Q6_K: return generic_row<0, T_Q6_K>(s, row, cols, L);
            default: return 0.f;
        }
    }
}

// The matvec of the pair range [pbeg, pend) by waves starting at pair p0 with stride G
// (one type group of a launch); returns the wave's LOGITS argmax key.
template <int ACT, bool NORM, int EPI, int T, int NP>
__device__ __forceinline__ unsigned long long mv_body(const MVArgs& A, const Lds& L, int p0, int G, int pbeg, int pend) {
    int pos = 0;
    if constexpr (EPI == EPI_QKV) pos = A.st->pos;
    unsigned long long best = 0;
    const int lane = threadIdx.x & 63;
    const int nch = A.cols >> 6, NJ = (nch + 63) >> 6;

#if defined(LLMI_EXP_TRACE)
    const int wave = threadIdx.x >> 6;
    const unsigned long long tr0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long tr1 = 0, tr2 = 0, tr_x = 0, tr_q = 0;
    int tr_items = 0;
#endif
    int p = p0;
    PairRef r;
    PairRows<T> rows;
    bool pipe = false;
    ProRegs<NORM, NP> R;
    mv_prologue_issue<NORM, NP>(A, R);  // activation loads first ...
    // Single-round launches (every wave owns at most one pair: QKV, attn_output) issue
    // their weights only once the activation has arrived: the activation loads then do
    // not queue behind the chip-wide weight burst, and the weight latency overlaps the
    // quantization instead (4096x4096: 5.2 -> 4.7 us).  Multi-round launches keep the
    // weights in flight from the start.
    if (pend - pbeg <= G || A.xfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    r = pair_ref<EPI>(A, p < pend ? p : pend - 1);
    pipe = p < pend && r.type == T;
    rows = pair_rows<T>(r, A.cols);
    // ... then the first weights, in flight during the prologue.  Issued on every path
    // (a wave without a pipelined pair reads a dummy chunk inside x: every plane offset
    // of one chunk stays below cols*4 bytes) so the prologue's first wait counts only
    // the activation loads.
    {
        const uint8_t* xb = (const uint8_t*)A.x;
        const RowPtr dummy{xb, xb, xb, xb};
        if (!pipe) rows.a = rows.b = dummy;
    }
    PairRaw<T> cur = load_item<T>(rows, lane, nch);
#if defined(LLMI_EXP_TRACE)
    // stamp once this wave's activation registers have arrived (forces the wait here)
    asm volatile("" ::"v"(R.x[0][0]), "v"(R.x[0][15]));
    tr_x = __builtin_amdgcn_s_memrealtime();
#endif
#if !defined(LLMI_EXP_NOPRO)
    mv_prologue_finish<ACT, NORM, NP>(A, L, R);
#if defined(LLMI_EXP_TRACE)
    tr_q = __builtin_amdgcn_s_memrealtime();
#endif
#else
    if (R.x[0][0] == 1234.5f) L.d[0] = R.x[0][1];
#endif
    __syncthreads();
#if defined(LLMI_EXP_TRACE)
    tr1 = __builtin_amdgcn_s_memrealtime();
#endif

    if (pipe) {
        int j = 0;
        float acc_a = 0.f, acc_b = 0.f;
        for (;;) {
            // next work item: (p, j+1) or (p+G, 0); uniform control flow
            int pn = p, jn = j + 1;
            PairRef rn = r;
            PairRows<T> rowsn = rows;
            if (jn == NJ) {
                jn = 0;
                pn = p + G;
                if (pn < pend) {
                    rn = pair_ref<EPI>(A, pn);
                    rowsn = pair_rows<T>(rn, A.cols);
                }
            }
            const bool has_next = pn < pend && rn.type == T;
            // always issue the prefetch (a valid re-load of the current item if none)
            const PairRaw<T> nxt = load_item<T>(has_next ? rowsn : rows, lane + 64 * (has_next ? jn : j), nch);
            const int ch = lane + 64 * j;
            const int chc = ch < nch ? ch : nch - 1;
            const Act act = load_act<ACT>(L, chc, nch);
#if defined(LLMI_EXP_NODOT)
            const float va = (float)(cur.a.q0.x ^ cur.a.q1.y ^ cur.a.hdr.x), vb = (float)(cur.b.q0.x ^ cur.b.q1.y ^ cur.b.hdr.x);
            (void)act;
#else
            const float va = dot_chunk<T>(cur.a, act, chc), vb = dot_chunk<T>(cur.b, act, chc);
#endif
            acc_a += ch < nch ? va : 0.f;
            acc_b += ch < nch ? vb : 0.f;
            if (j == NJ - 1) {
                epilogue<EPI>(A, r, p, reduce_pair(acc_a, acc_b), pos, best);
                acc_a = acc_b = 0.f;
#if defined(LLMI_EXP_TRACE)
                if (tr_items++ == 0) tr2 = __builtin_amdgcn_s_memrealtime();
#endif
            }
            if (!has_next) {
                p = pn;
                break;
            }
            cur = nxt;
            p = pn;
            j = jn;
            r = rn;
            rows = rowsn;
        }
    }
    // remaining pairs of other types (or all pairs if the first was not of type T)
    for (; p < pend; p += G) {
        r = pair_ref<EPI>(A, p);
        const float acc_a = generic_row_any<ACT>(r.sa.type, r.sa, r.ra, A.cols, L);
        const float acc_b = r.vb ? generic_row_any<ACT>(r.sb.type, r.sb, r.rb, A.cols, L) : 0.f;
        epilogue<EPI>(A, r, p, reduce_pair(acc_a, acc_b), pos, best);
    }
#if defined(LLMI_EXP_TRACE)
    if (A.trace && lane == 0) {
        unsigned hw = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        unsigned long long* t = A.trace + ((size_t)blockIdx.x * kMVWaves + wave) * 8;
        t[0] = tr0; t[1] = tr1; t[2] = tr2; t[3] = __builtin_amdgcn_s_memrealtime();
        t[4] = hw; t[5] = ((unsigned long long)xcc << 32) | (unsigned)tr_items;
        t[6] = tr_x; t[7] = tr_q;
    }
#endif
    return best;
}

// A launch whose segments form two type groups (QKV with a Q6_K or Q5_K attn_v) is
// split by workgroup: workgroups [0, split_wgs) run the pairs of type T, the rest the
// pairs of type T2, each group pipelined in its own type (no divergence in a workgroup).
template <int ACT, bool NORM, int EPI, int T, int NP, int T2 = T>
__global__ __launch_bounds__(kMVThreads) void k_matvec(MVArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Lds L = carve(smem, ACT, A.cols);
    const int wave = uniform((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    unsigned long long best;
    if constexpr (T2 == T) {
        best = mv_body<ACT, NORM, EPI, T, NP>(A, L, blockIdx.x * kMVWaves + wave, gridDim.x * kMVWaves, 0, A.npairs);
    } else {
        if ((int)blockIdx.x < A.split_wgs)
            best = mv_body<ACT, NORM, EPI, T, NP>(A, L, blockIdx.x * kMVWaves + wave, A.split_wgs * kMVWaves, 0,
                                                  A.split_pairs);
        else
            best = mv_body<ACT, NORM, EPI, T2, NP>(A, L, A.split_pairs + (blockIdx.x - A.split_wgs) * kMVWaves + wave,
                                                   (gridDim.x - A.split_wgs) * kMVWaves, A.split_pairs, A.npairs);
    }
    if constexpr (EPI == EPI_LOGITS) {
        // workgroup max of the waves' keys, then one atomic into this workgroup's slot
        const int cur_pos = A.st->pos;
        unsigned long long* red = (unsigned long long*)L.red;
        __syncthreads();
        if (lane == 0) red[wave] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long b = red[0];
#pragma unroll
            for (int w = 1; w < kMVWaves; ++w) b = red[w] > b ? red[w] : b;
            if (b) atomicMax(&A.argmax[(cur_pos & 1) * kArgSlots + blockIdx.x % kArgSlots], b);
            if (blockIdx.x == 0) A.st->pos_next = cur_pos + 1;
        }
    }
}

// K-split matvec for rows longer than one 64-chunk item (NJ = ceil(cols/4096) >= 2:
// ffn_down, 70B-wide inputs).  A workgroup's 4 waves form 4/KS pair slots of KS waves;
// the waves of a slot split the pair's items (wave sub takes items sub, sub+KS, ...),
// so every item of the first pair is in flight during the prologue, instead of one
// item per wave with the rest fetched serially after it.  Per-lane item values go to
// LDS; the slot's wave 0 adds them in item order starting from 0.f — exactly the
// single-wave loop's `acc += item value` sequence, so the fp32 association (the
// oracle's device order) is unchanged — then runs the butterfly and the epilogue.
// LDS part buffer double-buffered by round: one barrier per round.
constexpr int kKSThreads = 1024, kKSWaves = kKSThreads / 64;  // one workgroup per CU
template <int KS>
__host__ __device__ inline size_t ks_part_bytes(int cols) {
    const int nj = ((cols >> 6) + 63) >> 6;
    return (size_t)2 * (kKSWaves / KS) * nj * 128 * sizeof(float);
}
__host__ __device__ inline size_t ks_part_off(int act, int cols) { return a16(lds_red_off(act, cols) + kKSWaves * sizeof(double)); }

template <int ACT, bool NORM, int EPI, int T, int NP, int KS>
__global__ __launch_bounds__(kKSThreads) void k_matvec_ks(MVArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Lds L = carve(smem, ACT, A.cols);
    float* part = (float*)(smem + ks_part_off(ACT, A.cols));  // [2][PPW][NJ][2][64]
    constexpr int PPW = kKSWaves / KS;
    const int wave = uniform((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int slot = wave / KS, sub = wave % KS;
    const int nch = A.cols >> 6, NJ = (nch + 63) >> 6;
    const int stride = gridDim.x * PPW;
    const int rounds = (A.npairs + stride - 1) / stride;
    int pos = 0;
    if constexpr (EPI == EPI_QKV) pos = A.st->pos;
    unsigned long long best = 0;
    const uint8_t* xb = (const uint8_t*)A.x;
    const RowPtr dummy{xb, xb, xb, xb};

    ProRegs<NORM, NP> R;
    mv_prologue_issue<NORM, NP, kKSThreads>(A, R);  // activation loads first, then this wave's first item
    if (A.xfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int pr = blockIdx.x * PPW + slot;   // this slot's pair in the current round
    PairRows<T> rows = pair_rows<T>(pair_ref<EPI>(A, pr < A.npairs ? pr : A.npairs - 1), A.cols);
    if (!(pr < A.npairs && sub < NJ)) rows.a = rows.b = dummy;
    PairRaw<T> cur = load_item<T>(rows, lane + 64 * (sub < NJ ? sub : 0), nch);
    mv_prologue_finish<ACT, NORM, NP, kKSThreads>(A, L, R);
    __syncthreads();

    int buf = 0;
    for (int rd = 0; rd < rounds; ++rd, pr += stride) {
        const bool have = pr < A.npairs;
        float* pb = part + (size_t)(buf * PPW + slot) * NJ * 128;
        for (int j = sub; j < NJ; j += KS) {
            // the wave's next item: (pr, j+KS) or (pr+stride, sub); loads always issued
            int jn = j + KS, prn = pr;
            PairRows<T> rowsn = rows;
            if (jn >= NJ) {
                jn = sub;
                prn = pr + stride;
                rowsn = pair_rows<T>(pair_ref<EPI>(A, prn < A.npairs ? prn : A.npairs - 1), A.cols);
                if (prn >= A.npairs) rowsn.a = rowsn.b = dummy;
            }
            const PairRaw<T> nxt = load_item<T>(rowsn, lane + 64 * jn, nch);
            if (have) {
                const int ch = lane + 64 * j;
                const int chc = ch < nch ? ch : nch - 1;
                const Act act = load_act<ACT>(L, chc, nch);
                const float va = dot_chunk<T>(cur.a, act, chc), vb = dot_chunk<T>(cur.b, act, chc);
                pb[j * 128 + lane] = ch < nch ? va : 0.f;
                pb[j * 128 + 64 + lane] = ch < nch ? vb : 0.f;
            }
            cur = nxt;
            rows = rowsn;
        }
        __syncthreads();
        if (sub == 0 && have) {
            float acc_a = 0.f, acc_b = 0.f;
            for (int j = 0; j < NJ; ++j) {
                acc_a += pb[j * 128 + lane];
                acc_b += pb[j * 128 + 64 + lane];
            }
            epilogue<EPI>(A, pair_ref<EPI>(A, pr), pr, reduce_pair(acc_a, acc_b), pos, best);
        }
        buf ^= 1;
    }
    if constexpr (EPI == EPI_LOGITS) {
        const int cur_pos = A.st->pos;
        unsigned long long* red = (unsigned long long*)L.red;
        __syncthreads();
        if (lane == 0) red[wave] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long b = red[0];
#pragma unroll
            for (int w = 1; w < kKSWaves; ++w) b = red[w] > b ? red[w] : b;
            if (b) atomicMax(&A.argmax[(cur_pos & 1) * kArgSlots + blockIdx.x % kArgSlots], b);
            if (blockIdx.x == 0) A.st->pos_next = cur_pos + 1;
        }
    }
}

// The prologue's quantized activation written out in ggml block form (test hook).
template <int ACT>
__global__ __launch_bounds__(kMVThreads) void k_quant_dump(MVArgs A, uint8_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Lds L = carve(smem, ACT, A.cols);
    if (A.nw) mv_prologue<ACT, true>(A, L);
    else mv_prologue<ACT, false>(A, L);
    __syncthreads();
    const int cols = A.cols;
    const int nch = cols >> 6;
    for (int e = threadIdx.x; e < cols; e += blockDim.x) {
        const int ch = e >> 6, t = e & 63;
        if (ACT == 0) {
            const int k = (t & 31) >> 4;
            const int8_t qv = (int8_t)((t < 32 ? L.lo : L.hi)[16 * (k * nch + ch) + (t & 15)]);
            out[(size_t)(e >> 8) * 292 + 4 + (e & 255)] = (uint8_t)qv;
        } else {
            out[(size_t)(e >> 5) * 34 + 2 + (e & 31)] = L.lo[16 * ((t >> 4) * nch + ch) + (t & 15)];
        }
    }
    if (ACT == 0) {
        for (int b = threadIdx.x; b < cols / 256; b += blockDim.x) *(float*)(out + (size_t)b * 292) = L.d[b];
        for (int sb = threadIdx.x; sb < cols / 16; sb += blockDim.x)
            *(int16_t*)(out + (size_t)(sb >> 4) * 292 + 260 + 2 * (sb & 15)) = L.bs[sb];
    } else {
        for (int b = threadIdx.x; b < cols / 32; b += blockDim.x) *(uint16_t*)(out + (size_t)b * 34) = f2h(L.d[b]);
    }
}

// ----------------------------------------------------------------------------------
// Attention, ggml non-flash path:
//   kq[t] = sum_d f16(q_d) * K[t][d]        (ggml_vec_dot_f16, exact products, double sum)
//   w[t]  = kq[t] * (1/sqrt(D)); M = max w; e = exp(w-M); S = sum (double) e
//   p[t]  = f16(e * (float)(1/S));  out[d] = sum_t V[t][d] * p[t]    (double sum)
// scores: grid (HK, ceil(kv_bound/64)); workgroup = one kv head x 64 positions, its
//         K tile staged through LDS (rows padded by 16 B: conflict-free ds_read_b128).
// pv:     grid (HK, D/16); workgroup = one kv head x 16 dims for all GQA heads, reading
//         the transposed V cache [HK][D][n_ctx] with coalesced 128-B rows.
// ----------------------------------------------------------------------------------
template <int D, int G>
__global__ __launch_bounds__(256) void k_attn_scores(AttnArgs a) {
    const int g = blockIdx.x, chunk = blockIdx.y;
    const int n_kv = a.st->pos + 1;
    const int t0 = chunk * 64;
    if (t0 >= n_kv) return;
    const int nt = min(64, n_kv - t0);
    __shared__ float qs[G][D];
    __shared__ __attribute__((aligned(16))) uint16_t ks[64][D + 8];
    for (int i = threadIdx.x; i < G * D; i += 256) qs[i / D][i % D] = h2f(f2h(a.q[(size_t)g * G * D + i]));
    constexpr int PPR = D * 2 / 16;  // 16-B pieces per K row
    const uint16_t* kb = a.kc + ((size_t)g * a.n_ctx + t0) * D;
    for (int i = threadIdx.x; i < nt * PPR; i += 256) {
        const int r = i / PPR, pc = i % PPR;
        *(u32x4*)&ks[r][pc * 8] = *(const u32x4*)(kb + (size_t)r * D + pc * 8);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane < nt) {
        for (int hh = wave; hh < G; hh += 4) {
            double acc = 0.0;
#pragma unroll 4
            for (int d = 0; d < D; d += 8) {
                const u32x4 kv = *(const u32x4*)&ks[lane][d];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc += (double)(h2f(kv[j]) * qs[hh][d + 2 * j]);
                    acc += (double)(h2f(kv[j] >> 16) * qs[hh][d + 2 * j + 1]);
                }
            }
            a.scores[(size_t)(g * G + hh) * a.n_ctx + t0 + lane] = (float)acc * a.scale;
        }
    }
}

template <int D, int G>
__global__ __launch_bounds__(256) void k_attn_pv(AttnArgs a) {
    const int g = blockIdx.x, dc = blockIdx.y;
    const int n_kv = a.st->pos + 1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ float sM[G], sInv[G];
    __shared__ float sp[G][256];
    __shared__ double red[4];
    __shared__ float redf[4];
    for (int hh = 0; hh < G; ++hh) {
        const float* w = a.scores + (size_t)(g * G + hh) * a.n_ctx;
        float mx = -INFINITY;
        for (int t = tid; t < n_kv; t += 256) mx = fmaxf(mx, w[t]);
        mx = wave_max(mx);
        if (lane == 0) redf[wave] = mx;
        __syncthreads();
        mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
        double s = 0.0;
        for (int t = tid; t < n_kv; t += 256) s += (double)llmi_expf(w[t] - mx);
        s = wave_sum_d(s);
        if (lane == 0) red[wave] = s;
        __syncthreads();
        if (tid == 0) {
            sM[hh] = mx;
            sInv[hh] = (float)(1.0 / ((red[0] + red[1]) + (red[2] + red[3])));
        }
        __syncthreads();
    }
    const int d0 = dc * 16 + wave * 4;
    double acc[G][4];
#pragma unroll
    for (int hh = 0; hh < G; ++hh)
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) acc[hh][dd] = 0.0;
    const uint16_t* vb = a.vc + ((size_t)g * D + d0) * a.n_ctx;
    for (int tc = 0; tc < n_kv; tc += 256) {
        __syncthreads();
        const int t = tc + tid;
#pragma unroll
        for (int hh = 0; hh < G; ++hh) {
            float p = 0.f;
            if (t < n_kv) {
                const float e = llmi_expf(a.scores[(size_t)(g * G + hh) * a.n_ctx + t] - sM[hh]);
                p = h2f(f2h(e * sInv[hh]));
            }
            sp[hh][tid] = p;
        }
        __syncthreads();
        const int nt = min(256, n_kv - tc);
        for (int j = lane; j < nt; j += 64) {
#pragma unroll
            for (int dd = 0; dd < 4; ++dd) {
                const float v = h2f(vb[(size_t)dd * a.n_ctx + tc + j]);
#pragma unroll
                for (int hh = 0; hh < G; ++hh) acc[hh][dd] += (double)(v * sp[hh][j]);
            }
        }
    }
#pragma unroll
    for (int hh = 0; hh < G; ++hh)
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
            const double s = wave_sum_d(acc[hh][dd]);
            if (lane == 0) a.out[(size_t)(g * G + hh) * D + d0 + dd] = (float)s;
        }
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
// Split attention, phase 1: grid (HK, kv_bound/64), 256 threads; thread (t, qd) dots
// quarter qd of K row t with the G f16-rounded query heads of its group (G independent
// double chains of D/4), then a 4-lane butterfly; K rows are read straight from HBM,
// 4 lanes x (D/2) B per row.  Rows < kv_bound are always inside the cache, so the K
// loads are issued before the position is known (no dependent-load chain).
template <int D, int G>
__global__ __launch_bounds__(256) void k_attn_scores4(AttnArgs a) {
    LLMI_ATT_STAMP(0, 0)
    const int g = blockIdx.x, t0 = blockIdx.y * 64;
    const int tid = threadIdx.x;
    constexpr int DQ = D / 4;
    const int t = t0 + (tid >> 2), qd = tid & 3;
    const uint16_t* kr = a.kc + ((size_t)g * a.n_ctx + t) * D + qd * DQ;
    u32x4 kv[DQ / 8];
#pragma unroll
    for (int i = 0; i < DQ / 8; ++i) kv[i] = *(const u32x4*)(kr + 8 * i);
    __shared__ __attribute__((aligned(16))) float qs[G][D];
    for (int i = tid; i < G * D; i += 256) qs[i / D][i % D] = h2f(f2h(a.q[(size_t)g * G * D + i]));
    const int n_kv = a.st->pos + 1;
    __syncthreads();
    LLMI_ATT_STAMP(0, 1)
    if (t0 >= n_kv) return;
#if defined(LLMI_EXP_TRACE)
    asm volatile("" ::"v"(kv[0].x));
    LLMI_ATT_STAMP(0, 2)
#endif
    double acc[G];
#pragma unroll
    for (int hh = 0; hh < G; ++hh) acc[hh] = 0.0;
#pragma unroll
    for (int i = 0; i < DQ / 8; ++i) {
        const int d = qd * DQ + 8 * i;
        float k[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            k[2 * j] = h2f((uint16_t)kv[i][j]);
            k[2 * j + 1] = h2f((uint16_t)(kv[i][j] >> 16));
        }
#pragma unroll
        for (int hh = 0; hh < G; ++hh) {
            const float4 qa = *(const float4*)&qs[hh][d], qb = *(const float4*)&qs[hh][d + 4];
            acc[hh] += (double)(k[0] * qa.x); acc[hh] += (double)(k[1] * qa.y);
            acc[hh] += (double)(k[2] * qa.z); acc[hh] += (double)(k[3] * qa.w);
            acc[hh] += (double)(k[4] * qb.x); acc[hh] += (double)(k[5] * qb.y);
            acc[hh] += (double)(k[6] * qb.z); acc[hh] += (double)(k[7] * qb.w);
        }
    }
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        acc[hh] += xor_partner_d<1>(acc[hh]);
        acc[hh] += xor_partner_d<2>(acc[hh]);
        if (t < n_kv && qd == (hh & 3)) a.scores[(size_t)(g * G + hh) * a.n_ctx + t] = (float)acc[hh] * a.scale;
    }
    LLMI_ATT_STAMP(0, 3)
}

// Split attention, phase 2: grid (HK, D/8), 256 threads.  Every workgroup recomputes
// the softmax of its G heads from the scores (one wave per head: max, e = expf(s - max)
// kept in LDS, double sum, p = f16(e / sum) exactly as the fused kernel), then
// accumulates 8 output dims: 32 lanes per dim, 8 positions (16 B of the transposed V
// row) per lane and step, 4 steps of loads in flight, G double accumulators, 32-lane
// butterfly.  Score and first V loads are issued before the position is known.
template <int D, int G>
__global__ __launch_bounds__(256) void k_attn_pv_split(AttnArgs a, int kvb) {
    LLMI_ATT_STAMP(1, 0)
    extern __shared__ __attribute__((aligned(16))) float spv[];  // [G][kvb]
    const int g = blockIdx.x, dc = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int d = dc * 8 + (tid >> 5), sl = tid & 31;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    u32x4 vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) vv[u] = *(const u32x4*)(vr + min(8 * sl + 256 * u, kvb - 8));
    // 1. stage the G score rows (all kv_bound positions; those past n_kv are never used)
    const int n4 = kvb >> 2;
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        const float4* src = (const float4*)(a.scores + (size_t)(g * G + hh) * a.n_ctx);
        float4* dst = (float4*)(spv + hh * kvb);
        for (int j0 = tid; j0 < n4; j0 += 1024) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = src[min(j0 + 256 * u, n4 - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j0 + 256 * u < n4) dst[j0 + 256 * u] = v[u];
        }
    }
    const int n_kv = a.st->pos + 1;
    __syncthreads();
    LLMI_ATT_STAMP(1, 1)
    // 2. softmax, one wave per head; p = 0 past n_kv (up to the next multiple of 8)
    for (int hh = wave; hh < G; hh += 4) {
        float* sp = spv + hh * kvb;
        float mx = -INFINITY;
        for (int t = lane; t < n_kv; t += 64) mx = fmaxf(mx, sp[t]);
        mx = wave_max(mx);
        double sum = 0.0;
        for (int t = lane; t < n_kv; t += 64) {
            const float e = llmi_expf(sp[t] - mx);
            sp[t] = e;
            sum += (double)e;
        }
        sum = wave_sum_d(sum);
        const float inv = (float)(1.0 / sum);
        for (int t = lane; t < n_kv; t += 64) sp[t] = h2f(f2h(sp[t] * inv));
        for (int t = n_kv + lane; t < ((n_kv + 7) & ~7); t += 64) sp[t] = 0.f;
    }
    __syncthreads();
    LLMI_ATT_STAMP(1, 2)
    // 3. PV (V past n_kv may be anything: masked to 0 so 0 * NaN never happens)
    double acc[G];
#pragma unroll
    for (int hh = 0; hh < G; ++hh) acc[hh] = 0.0;
    for (int t0 = 8 * sl;;) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int tb = t0 + 256 * u;
            if (tb < n_kv) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float f = h2f((uint16_t)(vv[u][j >> 1] >> (16 * (j & 1))));
                    v[j] = tb + j < n_kv ? f : 0.f;
                }
#pragma unroll
                for (int hh = 0; hh < G; ++hh) {
                    const float4 pa = *(const float4*)&spv[hh * kvb + tb], pb = *(const float4*)&spv[hh * kvb + tb + 4];
                    acc[hh] += (double)(v[0] * pa.x); acc[hh] += (double)(v[1] * pa.y);
                    acc[hh] += (double)(v[2] * pa.z); acc[hh] += (double)(v[3] * pa.w);
                    acc[hh] += (double)(v[4] * pb.x); acc[hh] += (double)(v[5] * pb.y);
                    acc[hh] += (double)(v[6] * pb.z); acc[hh] += (double)(v[7] * pb.w);
                }
            }
        }
        t0 += 1024;
        if (t0 >= n_kv) break;
#pragma unroll
        for (int u = 0; u < 4; ++u) vv[u] = *(const u32x4*)(vr + min(t0 + 256 * u, kvb - 8));
    }
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        double v = acc[hh];
        v += xor_partner_d<1>(v);
        v += xor_partner_d<2>(v);
        v += xor_partner_d<4>(v);
        v += xor_partner_d<8>(v);
        v += xor_partner_d<16>(v);
        if (sl == 0) a.out[(size_t)(g * G + hh) * D + d] = (float)v;
    }
    LLMI_ATT_STAMP(1, 3)
}

// Split attention v2, phase 1: grid (HK, kv_bound/32), 256 threads; thread (t, qd)
// dots 1/8 of K row t (D/8 dims) with the G f16-rounded query heads (G independent
// double chains of D/8), 8-lane butterfly; K loads issued before the position is
// known.  Also writes the tile's per-head score maximum (tmax) so phase 2 needs no
// pass over the scores to find the row maximum (max is exact in any order).
template <int D, int G>
__global__ __launch_bounds__(256) void k_attn_scores8(AttnArgs a) {
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
__global__ __launch_bounds__(512) void k_attn_pv16(AttnArgs a, int kvb) {
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

// One-launch exchange attention for short contexts (kv_bound <= kXAttnMaxKV): grid
// (HK, D/16), 512 threads.  Workgroup (g, j) computes the scores of position tile j
// (64*NP positions; 8 lanes x D/8 dims per position, exact f16 products in double as
// k_attn_scores8) and publishes them as 8-byte {tag, score} granules (one relaxed
// agent-scope store each: the data is the flag, no fence; MI355X_MICROARCH.md
// "R2 granules").  Every workgroup of the group then sweeps all G x n_kv granules of
// its group until their tags match this step's (tag = step seq * 256 + layer + 1, read
// from device state at run time, so graph replays never see a previous step's
// granules), and runs k_attn_pv16's softmax and PV for its 16 output dims.  One
// launch and one hand-off replace the scores -> PV kernel boundary; K and V loads are
// issued before the position is known.  Every spin is bounded: a timed-out wait writes
// NaN outputs and sets *a.fault instead of hanging the GPU.
constexpr int kXSpinLimit = 1 << 22;
typedef unsigned long long __attribute__((address_space(1))) gu64;
template <int D, int G, int NP>
__global__ __launch_bounds__(512) void k_attn_x(AttnArgs a, int kvb) {
    LLMI_ATT_STAMP(0, 0)
    extern __shared__ __attribute__((aligned(16))) float spx[];  // [G][kvb] probabilities
    __shared__ __attribute__((aligned(16))) double qs[G][D];
    __shared__ float redm[8];
    __shared__ double reds[8];
    __shared__ int s_fault;
    constexpr int WPH = 8 / G;             // waves per head (softmax)
    constexpr int DQ = D / 8;              // dims per lane in the scores
    constexpr int NS = kXAttnMaxKV / (WPH * 64);  // max positions per lane in the softmax
    const int g = blockIdx.x, j = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // 1. step state and q first (they gate everything), then this tile's K rows (NP
    // passes of 64 positions), then this workgroup's V window: loads complete in issue
    // order, so nothing early waits behind the K/V stream
    const int pos = a.st->pos;
    const uint32_t seq = a.st->seq;
    float qv[(G * D + 511) / 512];
#pragma unroll
    for (int k = 0; k < (G * D + 511) / 512; ++k) qv[k] = a.q[(size_t)g * G * D + min(tid + 512 * k, G * D - 1)];
    const int qd = tid & 7;
    const int tile0 = j * 64 * NP;
    u32x4 kv[NP][DQ / 8];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int t = min(tile0 + p * 64 + (tid >> 3), kvb - 1);
        const uint16_t* kr = a.kc + ((size_t)g * a.n_ctx + t) * D + qd * DQ;
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i) kv[p][i] = __builtin_nontemporal_load((const u32x4*)(kr + 8 * i));
    }
    const int d = j * 16 + (tid >> 5), sl = tid & 31;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    constexpr int NV = 8;  // 8-B V loads in flight per lane: a 1024-position window
    u32x2 vv[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) vv[k] = __builtin_nontemporal_load((const u32x2*)(vr + min(4 * sl + 128 * k, kvb - 4)));
#pragma unroll
    for (int k = 0; k < (G * D + 511) / 512; ++k)
        if (tid + 512 * k < G * D) qs[(tid + 512 * k) / D][(tid + 512 * k) % D] = (double)h2f(f2h(qv[k]));
    if (tid == 0) s_fault = 0;
    const int n_kv = pos + 1;
    const uint32_t tag = seq * 256u + (uint32_t)a.layer + 1u;
    const uint32_t want = tag + (uint32_t)a.tag_skew;  // test option: 1 = a hand-off that never completes
    __syncthreads();
    LLMI_ATT_STAMP(0, 1)
    // 2. scores of the tile -> granules
    gu64* gr = (gu64*)a.gran + (size_t)g * G * kXAttnMaxKV;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int t = tile0 + p * 64 + (tid >> 3);
        if (tile0 + p * 64 >= n_kv) break;  // uniform
        double acc[G];
#pragma unroll
        for (int hh = 0; hh < G; ++hh) acc[hh] = 0.0;
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i) {
            const int d0 = qd * DQ + 8 * i;
            double k[8];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                k[2 * jj] = (double)h2f((uint16_t)kv[p][i][jj]);
                k[2 * jj + 1] = (double)h2f((uint16_t)(kv[p][i][jj] >> 16));
            }
#pragma unroll
            for (int hh = 0; hh < G; ++hh)
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) acc[hh] = __builtin_fma(k[jj], qs[hh][d0 + jj], acc[hh]);
        }
#pragma unroll
        for (int hh = 0; hh < G; ++hh) {
            acc[hh] += xor_partner_d<1>(acc[hh]);
            acc[hh] += xor_partner_d<2>(acc[hh]);
            acc[hh] += xor_partner_d<4>(acc[hh]);
            if (t < n_kv && qd == (hh & 7)) {
                const float sc = (float)acc[hh] * a.scale;
                __hip_atomic_store(gr + (size_t)hh * kXAttnMaxKV + t,
                                   ((unsigned long long)tag << 32) | __float_as_uint(sc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    LLMI_ATT_STAMP(0, 2)
    // 3. sweep: lane (head hh, wave wi of the head) owns positions wi*64 + lane + k*WPH*64,
    // the softmax's own mapping, so the scores stay in registers.  All of a lane's
    // granule loads are issued together; only stragglers are re-read (bounded spin).
    const int hh = wave / WPH, wi = wave % WPH;
    const gu64* gh = gr + (size_t)hh * kXAttnMaxKV;
    float sv[NS];
    {
        unsigned long long x[NS];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const int t = wi * 64 + lane + k * WPH * 64;
            x[k] = t < n_kv ? __hip_atomic_load(gh + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : ((unsigned long long)tag << 32);
        }
        for (int spins = 0;; ++spins) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < NS; ++k) ok &= (uint32_t)(x[k] >> 32) == want;
            if (__all(ok)) break;
            if (spins >= a.spin_limit) {
                s_fault = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                const int t = wi * 64 + lane + k * WPH * 64;
                if ((uint32_t)(x[k] >> 32) != want && t < n_kv)
                    x[k] = __hip_atomic_load(gh + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int k = 0; k < NS; ++k) sv[k] = __uint_as_float((uint32_t)x[k]);
    }
    LLMI_ATT_STAMP(0, 3)
    // 4. softmax as k_attn_pv16: row max (exact in any order), e = expf(s - max) with a
    // double sum (waves combined in fixed order), p = f16(e / sum) into LDS
    {
        float m = -INFINITY;
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if (wi * 64 + lane + k * WPH * 64 < n_kv) m = fmaxf(m, sv[k]);
        m = wave_max(m);
        if (lane == 0) redm[wave] = m;
    }
    __syncthreads();
    float mx = redm[hh * WPH];
#pragma unroll
    for (int i = 1; i < WPH; ++i) mx = fmaxf(mx, redm[hh * WPH + i]);
    double sum = 0.0;
#pragma unroll
    for (int k = 0; k < NS; ++k)
        if (wi * 64 + lane + k * WPH * 64 < n_kv) {
            sv[k] = llmi_expf(sv[k] - mx);
            sum += (double)sv[k];
        }
    sum = wave_sum_d(sum);
    if (lane == 0) reds[wave] = sum;
    __syncthreads();
    double tot = reds[hh * WPH];
#pragma unroll
    for (int i = 1; i < WPH; ++i) tot += reds[hh * WPH + i];
    const float inv = (float)(1.0 / tot);
    float* sp = spx + hh * kvb;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const int t = wi * 64 + lane + k * WPH * 64;
        if (t < n_kv) sp[t] = h2f(f2h(sv[k] * inv));
        else if (t < ((n_kv + 3) & ~3)) sp[t] = 0.f;
    }
    __syncthreads();
    LLMI_ATT_STAMP(1, 0)
    // 5. PV for dims [16j, 16j+16): as k_attn_pv16
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
                for (int jj = 0; jj < 4; ++jj) {
                    const float f = h2f((uint16_t)((jj < 2 ? vv[k].x : vv[k].y) >> (16 * (jj & 1))));
                    v[jj] = tb + jj < n_kv ? (double)f : 0.0;
                }
#pragma unroll
                for (int h = 0; h < G; ++h) {
                    const float4 p = *(const float4*)(spx + h * kvb + tb);
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
    LLMI_ATT_STAMP(1, 1)
    const bool fault = s_fault != 0;
#pragma unroll
    for (int h = 0; h < G; ++h) {
        double v = acc[h];
        v += xor_partner_d<1>(v);
        v += xor_partner_d<2>(v);
        v += xor_partner_d<4>(v);
        v += xor_partner_d<8>(v);
        v += xor_partner_d<16>(v);
        if (sl == 0) a.out[(size_t)(g * G + h) * D + d] = fault ? __uint_as_float(0x7fc00000u) : (float)v;
    }
    if (fault && tid == 0) atomicOr(a.fault, 1u);
}

// Fused single-launch attention for KV lengths that fit in LDS (kv_bound <= 8192):
// one 1024-thread workgroup per query head; scores, softmax statistics and the
// f16-rounded probabilities stay in LDS, so the only global traffic is one K and one V
// read per head (the G heads of a KV group are dealt to one XCD: blockIdx % HK = group,
// so 3 of 4 K/V reads hit that XCD's L2).  Same numerics as the two-kernel path above.
template <int D>
__global__ __launch_bounds__(1024) void k_attn_fused(AttnArgs a, int G, int HK) {
    extern __shared__ __attribute__((aligned(16))) float sp_lds[];
    __shared__ float qs[D];
    __shared__ double redd[16];
    __shared__ float redf[16];
    const int b = blockIdx.x;
    const int g = b % HK, h = g * G + b / HK;
    const int n_kv = a.st->pos + 1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < D) qs[tid] = h2f(f2h(a.q[(size_t)h * D + tid]));
    __syncthreads();
    // scores: one position per thread, K row read straight from HBM/L2 (16 x 16 B)
    const uint16_t* kb = a.kc + (size_t)g * a.n_ctx * D;
    float mx = -INFINITY;
    for (int t = tid; t < n_kv; t += 1024) {
        const uint16_t* kr = kb + (size_t)t * D;
        double acc = 0.0;
#pragma unroll 4
        for (int d = 0; d < D; d += 8) {
            const u32x4 kv = *(const u32x4*)(kr + d);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc += (double)(h2f(kv[j]) * qs[d + 2 * j]);
                acc += (double)(h2f(kv[j] >> 16) * qs[d + 2 * j + 1]);
            }
        }
        const float w = (float)acc * a.scale;
        sp_lds[t] = w;
        mx = fmaxf(mx, w);
    }
    mx = wave_max(mx);
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    mx = redf[0];
#pragma unroll
    for (int w = 1; w < 16; ++w) mx = fmaxf(mx, redf[w]);
    double s = 0.0;
    for (int t = tid; t < n_kv; t += 1024) s += (double)llmi_expf(sp_lds[t] - mx);
    s = wave_sum_d(s);
    if (lane == 0) redd[wave] = s;
    __syncthreads();
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) tot += redd[w];
    const float inv = (float)(1.0 / tot);
    for (int t = tid; t < n_kv; t += 1024) sp_lds[t] = h2f(f2h(llmi_expf(sp_lds[t] - mx) * inv));
    __syncthreads();
    // PV over the transposed V cache: SL threads per output dim, 8 positions (16 B) each
    constexpr int SL = 1024 / D;
    const int d = tid / SL, sl = tid % SL;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    double acc = 0.0;
    for (int t0 = 8 * sl; t0 < n_kv; t0 += 32 * SL) {  // 4 loads in flight, addresses clamped into the row
        u32x4 vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) vv[u] = *(const u32x4*)(vr + min(t0 + 8 * SL * u, a.n_ctx - 8));
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = t0 + 8 * SL * u + 2 * j;
                if (t < n_kv) acc += (double)(h2f(vv[u][j]) * sp_lds[t]);
                if (t + 1 < n_kv) acc += (double)(h2f(vv[u][j] >> 16) * sp_lds[t + 1]);
            }
    }
    acc += xor_partner_d<1>(acc);
    acc += xor_partner_d<2>(acc);
    acc += xor_partner_d<4>(acc);
    if constexpr (SL >= 16) acc += xor_partner_d<8>(acc);
    static_assert(SL == 8 || SL == 16, "head_dim 64 or 128");
    if (sl == 0) a.out[(size_t)h * D + d] = (float)acc;
}

// ----------------------------------------------------------------------------------
// Step entry: choose the token, advance pos, dequantize its embedding row
// (upstream ggml_get_rows + dequantize_row_*; bit-exact).
// Reads the piece-planar device layout (common.h).
// ----------------------------------------------------------------------------------
__device__ float dequant_elem(const Seg& w, int row, int e, int cols) {
    switch (w.type) {
        case T_F32: return ((const float*)w.a)[(size_t)row * cols + e];
        case T_F16: return h2f(((const uint16_t*)w.a)[(size_t)row * cols + e]);
        case T_Q4_K:
        case T_Q5_K:
        case T_Q6_K: {
            const int nch = cols >> 6, nbr = cols >> 8;
            const int ch = e >> 6, t = e & 63, hi = t >= 32, l = t & 31, k = l >> 4, i = l & 15;
            const size_t gb = (size_t)row * nbr + (e >> 8);
            const uint8_t qb = w.a[(size_t)row * nch * 32 + (size_t)(k * nch + ch) * 16 + i];
            int q = hi ? (qb >> 4) : (qb & 0xF);
            if (w.type == T_Q6_K) {  // H dword (2*hi + k), byte i&3, bits 2*(i>>2)
                const uint8_t hb = w.h[((size_t)row * nch + ch) * 16 + (2 * hi + k) * 4 + (i & 3)];
                q |= ((hb >> (2 * (i >> 2))) & 3) << 4;
                const float d = h2f(*(const uint16_t*)(w.d + gb * 2));
                const int sc = (int8_t)w.s[gb * 16 + ((e & 255) >> 4)];
                return d * (float)sc * (float)(q - 32);
            }
            const uint32_t* s32 = (const uint32_t*)(w.s + gb * 16);
            int sc, m;
            scale_min(2 * (ch & 3) + hi, s32[1], s32[2], s32[3], sc, m);
            if (w.type == T_Q5_K) q += ((ldw4(w.h + ((size_t)row * nch + ch) * 8 + 4 * hi) >> l) & 1) << 4;
            const float d = h2f(s32[0]), dmin = h2f(s32[0] >> 16);
            const float d1 = d * (float)sc, m1 = dmin * (float)m;
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

__global__ __launch_bounds__(256) void k_embed(EmbArgs a) {
    StepState* st = a.st;
    const int pos = st->pos_next;
    __shared__ int s_tok;
    if (threadIdx.x < 64) {  // wave 0: max over the previous step's argmax slots
        static_assert(kArgSlots == 64, "one slot per lane");
        const unsigned long long k = wave_max_u64(st->key[(pos + 1) & 1][threadIdx.x]);
        if (threadIdx.x == 0) {
            int tok = st->token_in_pos == pos ? st->token_in : (int)(0xffffffffu - (uint32_t)(k & 0xffffffffull));
            if (tok < 0 || tok >= a.vocab) tok = 0;
            s_tok = tok;
        }
    }
    __syncthreads();
    const int tok = s_tok;
    if (blockIdx.x == 0) {
        if (threadIdx.x < kArgSlots) st->key[pos & 1][threadIdx.x] = 0;
        if (threadIdx.x == 0) {
            st->pos = pos;
            st->token = tok;
            st->seq = st->seq + 1u;  // tags of this step's in-launch hand-offs (k_attn_x)
            if (pos >= 0 && pos < a.n_ctx) a.hist[pos] = tok;
        }
    }
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e < a.cols) a.x[e] = dequant_elem(a.w, tok, e, a.cols);
}

__global__ void k_state_tick(StepState* st) { st->seq = st->seq + 1u; }

hipError_t launch_state_tick(StepState* st, hipStream_t s) {
    hipLaunchKernelGGL(k_state_tick, dim3(1), dim3(1), 0, s, st);
    return hipGetLastError();
}

__global__ void k_state_set(StepState* st, int token_in, int pos_next) {
    st->token_in = token_in;
    st->token_in_pos = pos_next;
    st->pos_next = pos_next;
}

// ----------------------------------------------------------------------------------
// Load-time repack of GGUF blocks into the chunk-planar layout (common.h).
// One thread per (block, chunk c in 0..3); nbr = blocks per row.
// ----------------------------------------------------------------------------------
__global__ void k_repack_kq(int type, const uint8_t* raw, uint8_t* A, uint8_t* H, uint8_t* S, uint8_t* Dp, int64_t nblk,
                            int nbr) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = gid >> 2;
    const int c = (int)(gid & 3);
    if (b >= nblk) return;
    const int64_t row = b / nbr, bi = b % nbr, nch = (int64_t)nbr * 4, ch = bi * 4 + c;
    uint8_t* arow = A + row * nch * 32;
    if (type == T_Q4_K || type == T_Q5_K) {
        const int bb = type == T_Q4_K ? 144 : 176;
        const uint8_t* x = raw + b * bb;
        const uint8_t* qs = x + (type == T_Q4_K ? 16 : 48);
        for (int k = 0; k < 2; ++k)
            for (int i = 0; i < 16; ++i) arow[(k * nch + ch) * 16 + i] = qs[32 * c + 16 * k + i];
        if (c == 0)
            for (int i = 0; i < 16; ++i) S[b * 16 + i] = x[i];
        if (type == T_Q5_K) {  // bit l of the lo word: qh[l] bit 2c; hi word: bit 2c+1
            const uint8_t* qh = x + 16;
            uint32_t lo = 0, hi = 0;
            for (int l = 0; l < 32; ++l) {
                lo |= (uint32_t)((qh[l] >> (2 * c)) & 1) << l;
                hi |= (uint32_t)((qh[l] >> (2 * c + 1)) & 1) << l;
            }
            uint8_t* h = H + (row * nch + ch) * 8;
            for (int k = 0; k < 4; ++k) { h[k] = (uint8_t)(lo >> (8 * k)); h[4 + k] = (uint8_t)(hi >> (8 * k)); }
        }
    } else {  // Q6_K
        const uint8_t* x = raw + b * 210;
        const uint8_t* ql = x;
        const uint8_t* qh = x + 128;
        auto u6 = [&](int w) -> int {  // 6-bit unsigned value of weight w of the block
            const int n = w >> 7, rr = w & 127, quad = rr >> 5, l = rr & 31;
            const uint8_t qlb = ql[64 * n + l + 32 * (quad & 1)];
            const int lo = (quad >> 1) ? (qlb >> 4) : (qlb & 0xF);
            const int hi = (qh[32 * n + l] >> (2 * quad)) & 3;
            return lo | (hi << 4);
        };
        for (int k = 0; k < 2; ++k)
            for (int i = 0; i < 16; ++i) {
                const int t = 16 * k + i;
                arow[(k * nch + ch) * 16 + i] = (uint8_t)((u6(64 * c + t) & 15) | ((u6(64 * c + 32 + t) & 15) << 4));
            }
        // H dword g = 2*hi + k: byte j bits [2m, 2m+1] = high2 of chunk weight 32*hi + 16k + 4m + j
        uint8_t* h = H + (row * nch + ch) * 16;
        for (int g = 0; g < 4; ++g)
            for (int j = 0; j < 4; ++j) {
                uint8_t v = 0;
                for (int m = 0; m < 4; ++m) v |= (uint8_t)((u6(64 * c + 32 * (g >> 1) + 16 * (g & 1) + 4 * m + j) >> 4) << (2 * m));
                h[4 * g + j] = v;
            }
        for (int i = 0; i < 4; ++i) S[b * 16 + 4 * c + i] = x[192 + 4 * c + i];
        if (c == 0) { Dp[b * 2] = x[208]; Dp[b * 2 + 1] = x[209]; }
    }
}

// Q8_0: one thread per 64-weight chunk (two blocks)
__global__ void k_repack_q80(const uint8_t* raw, uint8_t* A, uint8_t* Dp, int64_t nchunk, int nch_row) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nchunk) return;
    const int64_t row = g / nch_row, ch = g % nch_row;
    uint8_t* arow = A + row * nch_row * 64;
    for (int half = 0; half < 2; ++half) {
        const uint8_t* x = raw + (g * 2 + half) * 34;
        for (int k = 0; k < 2; ++k)
            for (int i = 0; i < 16; ++i) arow[((2 * half + k) * nch_row + ch) * 16 + i] = x[2 + 16 * k + i];
        Dp[(g * 2 + half) * 2] = x[0];
        Dp[(g * 2 + half) * 2 + 1] = x[1];
    }
}

// Streaming-read reference (achievable HBM rate for a perfectly coalesced 16-B/lane
// read of the same bytes): each thread sums dwords of grid-strided 16-B pieces.
__global__ __launch_bounds__(256) void k_stream_read(const u32x4* p, size_t n16, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const u32x4 v = ldw((const uint8_t*)(p + i));
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

hipError_t launch_stream_read(const void* p, size_t bytes, unsigned* out, int blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_stream_read, dim3(blocks), dim3(256), 0, s, (const u32x4*)p, bytes / 16, out);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------
// Grid of a matvec launch: never more workgroups than can be resident at once (the
// kernel is grid-strided over row pairs; a second dispatch round would be a tail of
// idle CUs).  Residency per CU comes from the occupancy query for the instantiation
// and its LDS, cached per (kernel, LDS bytes, device).
template <typename K>
static dim3 resident_grid(K kernel, dim3 grid, size_t lds, int threads = kMVThreads) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, size_t, int>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple((const void*)kernel, lds, dev * 4096 + threads);
    int cap = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) {
            cap = it->second;
        } else {
            int occ = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, threads, lds) != hipSuccess || occ <= 0) occ = 1;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 1;
            cap = occ * cus;
            cache.emplace(key, cap);
        }
    }
    if ((int)grid.x > cap) grid.x = cap;
    return grid;
}

template <int ACT, bool NORM, int T, int EPI, int NP>
static hipError_t mv_launch(const MVArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    auto k = k_matvec<ACT, NORM, EPI, T, NP>;
    launch_k(k, resident_grid(k, grid, lds), dim3(kMVThreads), lds, s, true, true, a);
    return hipGetLastError();
}

// Two type groups (pairs [0, split) of type T, [split, npairs) of type T2): the
// resident grid is dealt to the groups in proportion to their pairs (>= 1 each).
template <int ACT, bool NORM, int T, int T2, int EPI, int NP>
static hipError_t mv_launch2(const MVArgs& a0, int split_pairs, dim3 grid, size_t lds, hipStream_t s) {
    auto k = k_matvec<ACT, NORM, EPI, T, NP, T2>;
    const dim3 g = resident_grid(k, grid, lds);
    MVArgs a = a0;
    a.split_pairs = split_pairs;
    int w1 = (int)(((long long)g.x * split_pairs + a.npairs / 2) / a.npairs);
    w1 = w1 < 1 ? 1 : w1 > (int)g.x - 1 ? (int)g.x - 1 : w1;
    a.split_wgs = w1;
    launch_k(k, g, dim3(kMVThreads), lds, s, true, true, a);
    return hipGetLastError();
}

// prologue sub-blocks per thread held in registers: 1, 2 or 4
static int prologue_np(int cols) {
    const int per = (cols / 16 + kMVThreads - 1) / kMVThreads;
    return per <= 1 ? 1 : per <= 2 ? 2 : 4;
}

template <int ACT, bool NORM, int T, int EPI, int NP, int KS>
static hipError_t mv_launch_ks(const MVArgs& a, int max_blocks, hipStream_t s) {
    auto k = k_matvec_ks<ACT, NORM, EPI, T, NP, KS>;
    const size_t lds = ks_part_off(ACT, a.cols) + ks_part_bytes<KS>(a.cols);
    constexpr int PPW = kKSWaves / KS;
    int blocks = (a.npairs + PPW - 1) / PPW;
    if (blocks > max_blocks) blocks = max_blocks;
    launch_k(k, resident_grid(k, dim3(blocks), lds, kKSThreads), dim3(kKSThreads), lds, s, true, true, a);
    return hipGetLastError();
}

static thread_local int g_mv_max_blocks = 1024;  // set by launch_matvec

// K-split is taken for rows of >= 2 items when every segment has the pipelined type
static bool use_ks(const MVArgs& a, int T) {
    if (((a.cols >> 6) + 63) >> 6 < 2) return false;
    for (int i = 0; i < a.nseg; ++i)
        if (a.seg[i].type != T) return false;
    return true;
}

template <int ACT, bool NORM, int T, int EPI>
static hipError_t mv_launch_np(const MVArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    if (use_ks(a, T)) {  // one 1024-thread workgroup per CU: NP from 1024 threads
        const int nj = ((a.cols >> 6) + 63) >> 6;
        const int per = (a.cols / 16 + kKSThreads - 1) / kKSThreads;
        const int mb = g_mv_max_blocks;
        // K-split width (waves per pair slot), measured (profiles/r01/ks_sweep.md):
        //   rows of >= 6 items (70B ffn_down, 28672 columns): KS = 1 when its part buffer
        //     fits LDS — one pair per wave, no per-round barrier wait (30.7 -> 29.0 us);
        //   otherwise KS = 2 (8B ffn_down Q4_K 10.3 -> 9.8 us against KS = 4).
        // LLMI_KS = 2 / 4 forces that width (A/B hook; 4 only for rows of >= 4 items).
        static const int ks_env = [] {
            const char* e = getenv("LLMI_KS");
            return e ? atoi(e) : 0;
        }();
        if (ks_env == 4 && nj >= 4) {
            if (per <= 1) return mv_launch_ks<ACT, NORM, T, EPI, 1, 4>(a, mb, s);
            return mv_launch_ks<ACT, NORM, T, EPI, 2, 4>(a, mb, s);
        }
        if (ks_env == 0 && nj >= 6 && per > 1 && ks_part_off(ACT, a.cols) + ks_part_bytes<1>(a.cols) <= 160 * 1024)
            return mv_launch_ks<ACT, NORM, T, EPI, 2, 1>(a, mb, s);
        if (per <= 1) return mv_launch_ks<ACT, NORM, T, EPI, 1, 2>(a, mb, s);
        return mv_launch_ks<ACT, NORM, T, EPI, 2, 2>(a, mb, s);
    }
    switch (prologue_np(a.cols)) {
        case 1: return mv_launch<ACT, NORM, T, EPI, 1>(a, grid, lds, s);
        case 2: return mv_launch<ACT, NORM, T, EPI, 2>(a, grid, lds, s);
        default: return mv_launch<ACT, NORM, T, EPI, 4>(a, grid, lds, s);
    }
}

// Instantiated (ACT, NORM, EPI) combinations: STORE and ADD with or without the fused
// RMSNorm; QKV, SWIGLU and LOGITS always take a normalised input.
template <int ACT, bool NORM, int T>
static hipError_t mv_dispatch_epi(const MVArgs& a, int epi, dim3 grid, size_t lds, hipStream_t s) {
    switch (epi) {
        case EPI_STORE: return mv_launch_np<ACT, NORM, T, EPI_STORE>(a, grid, lds, s);
        case EPI_ADD: return mv_launch_np<ACT, NORM, T, EPI_ADD>(a, grid, lds, s);
        default: break;
    }
    if constexpr (NORM) {
        switch (epi) {
            case EPI_QKV: return mv_launch_np<ACT, NORM, T, EPI_QKV>(a, grid, lds, s);
            case EPI_SWIGLU: return mv_launch_np<ACT, NORM, T, EPI_SWIGLU>(a, grid, lds, s);
            case EPI_LOGITS: return mv_launch_np<ACT, NORM, T, EPI_LOGITS>(a, grid, lds, s);
            default: break;
        }
    }
    return hipErrorInvalidValue;
}

// QKV whose segments form two contiguous type groups split at an even row: both groups
// pipelined (k_matvec's T2 path).  Returns hipErrorNotSupported when not applicable.
template <bool NORM>
static hipError_t mv_dispatch_qkv2(const MVArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    if (a.nseg < 2 || grid.x < 2) return hipErrorNotSupported;
    int t1 = a.seg[0].type, t2 = -1, split_row = -1;
    for (int i = 1; i < a.nseg; ++i) {
        if (a.seg[i].type == (t2 < 0 ? t1 : t2)) continue;
        if (t2 >= 0) return hipErrorNotSupported;  // a third group
        t2 = a.seg[i].type;
        split_row = a.seg[i].row0 - a.seg[0].row0;
    }
    if (t2 < 0 || (split_row & 1) || prologue_np(a.cols) != 1) return hipErrorNotSupported;
    const int sp = split_row / 2;
#define LLMI_QKV2(A_, B_)                                                                            \
    if (t1 == A_ && t2 == B_) return mv_launch2<0, NORM, A_, B_, EPI_QKV, 1>(a, sp, grid, lds, s);
    if constexpr (NORM) {
        LLMI_QKV2(T_Q4_K, T_Q6_K) LLMI_QKV2(T_Q4_K, T_Q5_K) LLMI_QKV2(T_Q5_K, T_Q6_K)
    }
#undef LLMI_QKV2
    return hipErrorNotSupported;
}

template <bool NORM>
static hipError_t mv_dispatch_type(const MVArgs& a, int epi, dim3 grid, size_t lds, hipStream_t s) {
    static const bool qkv2 = !getenv("LLMI_NO_QKV2");  // A/B switch for measurements
    if (epi == EPI_QKV && qkv2) {
        const hipError_t e = mv_dispatch_qkv2<NORM>(a, grid, lds, s);
        if (e != hipErrorNotSupported) return e;
    }
    // primary (pipelined) type = the type owning the most rows of the launch
    int best = a.seg[0].type, best_rows = 0;
    for (int i = 0; i < a.nseg; ++i) {
        int rows = 0;
        for (int k = 0; k < a.nseg; ++k)
            if (a.seg[k].type == a.seg[i].type) rows += a.seg[k].rows;
        if (rows > best_rows) { best_rows = rows; best = a.seg[i].type; }
    }
    switch (best) {
        case T_Q4_K: return mv_dispatch_epi<0, NORM, T_Q4_K>(a, epi, grid, lds, s);
        case T_Q5_K: return mv_dispatch_epi<0, NORM, T_Q5_K>(a, epi, grid, lds, s);
        case T_Q6_K: return mv_dispatch_epi<0, NORM, T_Q6_K>(a, epi, grid, lds, s);
        case T_Q8_0: return mv_dispatch_epi<1, NORM, T_Q8_0>(a, epi, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_matvec(const MVArgs& a, int epi, int max_blocks, hipStream_t s) {
    g_mv_max_blocks = max_blocks;
    if (a.nseg < 1 || a.cols <= 0 || a.cols % 256 || a.npairs <= 0) return hipErrorInvalidValue;
    const int act = act_kind(a.seg[0].type);
    for (int i = 1; i < a.nseg; ++i)
        if (act_kind(a.seg[i].type) != act) return hipErrorInvalidValue;
    const size_t lds = mv_lds_bytes(act, a.cols);
    int blocks = (a.npairs + kMVWaves - 1) / kMVWaves;
    if (blocks > max_blocks) blocks = max_blocks;
#if defined(LLMI_EXPERIMENTS)
    static const int exp_blocks = [] {  // experiment builds: fixed grid for launch sweeps
        const char* e = getenv("LLMI_MV_BLOCKS");
        return e ? atoi(e) : 0;
    }();
    if (exp_blocks > 0 && exp_blocks < blocks) blocks = exp_blocks;
#endif
#if defined(LLMI_EXP_BALANCE)
    {  // experiment: equal pairs per wave (fewer workgroups when that divides better)
        const int waves = blocks * kMVWaves, per = (a.npairs + waves - 1) / waves;
        blocks = ((a.npairs + per - 1) / per + kMVWaves - 1) / kMVWaves;
    }
#endif
    const dim3 grid(blocks);
    return a.nw ? mv_dispatch_type<true>(a, epi, grid, lds, s) : mv_dispatch_type<false>(a, epi, grid, lds, s);
}

hipError_t launch_quant_dump(const MVArgs& a, int act, void* out, hipStream_t s) {
    if (a.cols <= 0 || a.cols % 256) return hipErrorInvalidValue;
    const size_t lds = mv_lds_bytes(act, a.cols);
    if (act == 0) hipLaunchKernelGGL((k_quant_dump<0>), dim3(1), dim3(kMVThreads), lds, s, a, (uint8_t*)out);
    else hipLaunchKernelGGL((k_quant_dump<1>), dim3(1), dim3(kMVThreads), lds, s, a, (uint8_t*)out);
    return hipGetLastError();
}

template <int D>
static hipError_t attn_dispatch_g(const AttnArgs& a, int g, int hk, int kv_bound, hipStream_t s) {
    const dim3 gs(hk, (kv_bound + 63) / 64), gp(hk, D / 16);
    switch (g) {
#define LLMI_ATT(G)                                                                   \
    case G:                                                                           \
        launch_k(k_attn_scores<D, G>, gs, dim3(256), 0, s, true, false, a);          \
        launch_k(k_attn_pv<D, G>, gp, dim3(256), 0, s, false, true, a);              \
        break;
        LLMI_ATT(1) LLMI_ATT(2) LLMI_ATT(4) LLMI_ATT(8)
#undef LLMI_ATT
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int D>
static hipError_t attn_split_g(const AttnArgs& a, int g, int hk, int kv_bound, hipStream_t s) {
    const dim3 gs(hk, (kv_bound + 31) / 32), gp(hk, D / 16);
    const size_t lds = (size_t)g * kv_bound * 4;
    switch (g) {
#define LLMI_ATT(G)                                                                    \
    case G:                                                                            \
        launch_k(k_attn_scores8<D, G>, gs, dim3(256), 0, s, true, false, a);          \
        launch_k(k_attn_pv16<D, G>, gp, dim3(512), lds, s, false, true, a, kv_bound);  \
        break;
        LLMI_ATT(1) LLMI_ATT(2) LLMI_ATT(4) LLMI_ATT(8)
#undef LLMI_ATT
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// exchange attention: K tile passes for a KV bound (tiles of 64*NP positions cover
// kv_bound with D/16 workgroups per group); 0 = not applicable
static int attn_x_np(int head_dim, int kv_bound) {
    const int nw = head_dim / 16;
    const int np = (kv_bound + nw * 64 - 1) / (nw * 64);
    if (kv_bound > kXAttnMaxKV) return 0;
    return np <= 1 ? 1 : np <= 2 ? 2 : np <= 4 ? 4 : 0;
}

template <int D>
static hipError_t attn_x_g(const AttnArgs& a, int g, int hk, int kv_bound, hipStream_t s) {
    const int np = attn_x_np(D, kv_bound);
    const dim3 grid(hk, D / 16);
    const size_t lds = (size_t)g * kv_bound * 4;
#define LLMI_ATTX(G, NPV) \
    if (g == G && np == NPV) { launch_k(k_attn_x<D, G, NPV>, grid, dim3(512), lds, s, true, true, a, kv_bound); return hipGetLastError(); }
#define LLMI_ATTX_G(G) LLMI_ATTX(G, 1) LLMI_ATTX(G, 2) LLMI_ATTX(G, 4)
    LLMI_ATTX_G(1) LLMI_ATTX_G(2) LLMI_ATTX_G(4) LLMI_ATTX_G(8)
#undef LLMI_ATTX_G
#undef LLMI_ATTX
    return hipErrorInvalidValue;
}

// Test options (llmi_test_option; never read from the environment): paths that give
// bit-identical results, or limits lowered so a test reaches a fallback / fault path.
int g_pf_attn_simple = 0;               // batched-prefill attention: one head per workgroup
int g_pf_max_kv = kPfAttnMaxKV;         // longest KV the batched-prefill attention takes
int g_xspin_limit = kXSpinLimit;        // k_attn_x bounded-wait polls before it faults
int g_xtag_skew = 0;                    // k_attn_x consumers expect tag + skew (1: never matches)
int pf_max_kv() { return g_pf_max_kv; }

static int g_attn_mode = 0;  // 0 auto, 1 fused, 2 split, 3 two-kernel, 4 exchange (experiments: LLMI_ATTN_MODE)
void set_attn_mode(int mode) { g_attn_mode = mode; }
int attn_path(int n_head, int n_head_kv, int kv_bound, int head_dim) {
    const int g = n_head / n_head_kv;
    const bool split_ok = (size_t)g * kv_bound * 4 <= kSplitAttnMaxLds;
    const bool fused_ok = kv_bound <= kFusedAttnMaxKV;
    (void)n_head;
    if (g_attn_mode == 4 && g <= 8 && kv_bound <= kXAttnMaxKV) return 4;
    if (g_attn_mode == 1 && fused_ok) return 1;
    if (g_attn_mode == 2 && split_ok) return 2;
    if (g_attn_mode == 3) return 3;
    // auto, from the crossovers measured by tools/attnbench.py (graph-free launches, us;
    // profiles/r01/attn_modes.md):
    //   G=4, D=128 (8B, Mistral): fused <= 256 (8.1 vs 8.4 exchange), exchange <= 512,
    //                             split beyond (640: 10.8 vs 12.9 exchange)
    //   G=8, D=128 (70B): fused <= 640 (128: 8.1 vs 16.3 exchange), split beyond
    //   G=8, D=64 (TinyLlama): fused <= 2048 (128: 6.2 vs 9.7; 1280: 15.9 vs 20.9)
    if (g_attn_mode == 0) {
        if (g == 8 && fused_ok && kv_bound <= (head_dim == 64 ? 2048 : 640)) return 1;
        if (g == 4 && fused_ok && kv_bound <= 256) return 1;
        if (g == 4 && split_ok && kv_bound > 512) return 2;
        if (g <= 8 && kv_bound <= kXAttnMaxKV) return 4;
    }
    return split_ok ? 2 : fused_ok ? 1 : 3;
}

hipError_t launch_attention(const AttnArgs& a0, int n_head, int n_head_kv, int head_dim, int kv_bound, hipStream_t s) {
    if (n_head_kv <= 0 || n_head % n_head_kv) return hipErrorInvalidValue;
    AttnArgs a = a0;
    a.spin_limit = g_xspin_limit;
    a.tag_skew = g_xtag_skew;
    const int g = n_head / n_head_kv;
    int path = attn_path(n_head, n_head_kv, kv_bound, head_dim);
    if (path == 4 && (!a.gran || !a.fault || a.layer < 0 || a.layer > 254))
        path = attn_path(n_head, n_head_kv, kXAttnMaxKV + 256, head_dim);
    if (path == 4) {
        if (head_dim == 128 && attn_x_np(128, kv_bound)) return attn_x_g<128>(a, g, n_head_kv, kv_bound, s);
        if (head_dim == 64 && attn_x_np(64, kv_bound)) return attn_x_g<64>(a, g, n_head_kv, kv_bound, s);
        return hipErrorInvalidValue;
    }
    if (path == 2) {
        if (head_dim == 128) return attn_split_g<128>(a, g, n_head_kv, kv_bound, s);
        if (head_dim == 64) return attn_split_g<64>(a, g, n_head_kv, kv_bound, s);
        return hipErrorInvalidValue;
    }
    if (path == 1) {
        const size_t lds = (size_t)kv_bound * 4;
        if (head_dim == 128) launch_k(k_attn_fused<128>, dim3(n_head), dim3(1024), lds, s, true, true, a, g, n_head_kv);
        else if (head_dim == 64) launch_k(k_attn_fused<64>, dim3(n_head), dim3(1024), lds, s, true, true, a, g, n_head_kv);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (head_dim == 128) return attn_dispatch_g<128>(a, g, n_head_kv, kv_bound, s);
    if (head_dim == 64) return attn_dispatch_g<64>(a, g, n_head_kv, kv_bound, s);
    return hipErrorInvalidValue;
}

hipError_t launch_embed(const EmbArgs& a, hipStream_t s) {
    launch_k(k_embed, dim3((a.cols + 255) / 256), dim3(256), 0, s, true, true, a);
    return hipGetLastError();
}

hipError_t launch_state_set(StepState* st, int token_in, int pos_next, hipStream_t s) {
    hipLaunchKernelGGL(k_state_set, dim3(1), dim3(1), 0, s, st, token_in, pos_next);
    return hipGetLastError();
}

hipError_t launch_repack(int type, const void* raw, uint8_t* a, uint8_t* h, uint8_t* sp, uint8_t* d, int64_t nblk,
                         int64_t cols, hipStream_t s) {
    if (nblk <= 0) return hipSuccess;
    if (cols % 256) return hipErrorInvalidValue;
    if (type == T_Q4_K || type == T_Q5_K || type == T_Q6_K) {
        const int64_t thr = nblk * 4;
        hipLaunchKernelGGL(k_repack_kq, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s, type, (const uint8_t*)raw, a,
                           h, sp, d, nblk, (int)(cols / 256));
    } else if (type == T_Q8_0) {
        const int64_t nchunk = nblk / 2;
        hipLaunchKernelGGL(k_repack_q80, dim3((unsigned)((nchunk + 255) / 256)), dim3(256), 0, s, (const uint8_t*)raw, a, d,
                           nchunk, (int)(cols / 64));
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// batched prefill (MFMA): same translation unit, shares the device helpers above
#include "prefill.hip.inc"

}  // namespace llmi
