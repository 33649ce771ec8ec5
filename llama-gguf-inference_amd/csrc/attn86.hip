// attn86.hip — decode and prefill attention in the x86 association mode (model numerics
// LLMI_NUMERICS_X86; mv_device.h "x86 numerics").
//
// Upstream's non-flash CPU attention [upstream ggml-cpu ops.cpp mul_mat + soft_max,
// vec.h ggml_vec_dot_f16 / ggml_vec_soft_max_f32, simd-mappings.h; recalled, not
// vendored] on an x86 AVX2+F16C build, as the oracle's x86 mode restates it
// (oracle/ggml_oracle.c x86_dot_f16f, attn_head with OR_X86_F16DOT | OR_X86_VEXP):
//   kq[t]  = dot_f16(K[t], f16(q)): element i accumulates into lane (i % 32) of 4 x 8 fp32
//            fma chains (i in order), reduced acc0 + acc2, acc1 + acc3, then those two,
//            then lo4 + hi4 and two hadds: ((t0 + t1) + (t2 + t3))
//   w[t]   = kq[t] * (1 / sqrt(D)); M = max w
//   e[t]   = ggml_v_expf(w[t] - M); S = double sum over 8-position chunks of the chunk's
//            fp32 hsum_float_8 (the row padded to 32 with masked zeros)
//   p[t]   = f16(e[t] * (float)(1 / S))
//   out[d] = dot_f16(V[d][.], p) over the positions padded to 32 (p = 0, V = 0 past n_kv),
//            the same 4 x 8-lane association over positions.
// The fp32 chains are exact sequences (one lane per chain); only the double sum of chunk
// sums is reordered (a lane tree, absorbed by double as on every other path).
//
//   decode:  k_a86_h, one launch up to kA86MaxKV positions: (head, 16-dim slice) per
//            workgroup, every workgroup of a head takes the head's scores and softmax
//            (LDS) and its slice of PV; beyond: k_a86_scores (KV group x 64-position tile)
//            -> k_a86_softmax (one workgroup per head, p in place of the scores) -> k_a86_pv
//            (KV group x 16 dims)
//   prefill: k_pf_a86 (KV group x query token), scores and p in LDS
#include "kernels.h"
#include "launch_util.h"
#include "mv_device.h"

namespace llmi {

// the 32 fp32 chains of ggml_vec_dot_f16 (x86), reduced as upstream's GGML_F16_VEC_REDUCE
__device__ __forceinline__ float x86_f16dot_reduce(const float (&acc)[32]) {
    float c[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) c[l] = (acc[l] + acc[16 + l]) + (acc[8 + l] + acc[24 + l]);
    const float t0 = c[0] + c[4], t1 = c[1] + c[5], t2 = c[2] + c[6], t3 = c[3] + c[7];
    return (t0 + t1) + (t2 + t3);
}
// the same reduction over 32 lanes (lane c holds chain c) of a 32-lane group; lane c = 0 of
// the group gets the result
__device__ __forceinline__ float x86_f16dot_reduce_lanes(float v) {
    v = v + __shfl_xor(v, 16, 64);
    v = v + __shfl_xor(v, 8, 64);
    v = v + __shfl_xor(v, 4, 64);
    const float a = v + __shfl_xor(v, 1, 64);  // lane 0: t0 + t1, lane 2: t2 + t3
    return a + __shfl_xor(a, 2, 64);
}

// ---- decode ------------------------------------------------------------------------
template <int D, int G>
__global__ __launch_bounds__(256) void k_a86_scores(AttnArgs a) {
    const int g = blockIdx.x, t0 = blockIdx.y * 64;
    const int n_kv = a.st->pos + 1;
    if (t0 >= n_kv) return;
    const int nt = min(64, n_kv - t0);
    __shared__ float qs[G][D];
    __shared__ __attribute__((aligned(16))) uint16_t ks[64][D + 8];
    const int tid = threadIdx.x;
    for (int i = tid; i < G * D; i += 256) qs[i / D][i % D] = h2f(f2h(a.q[(size_t)g * G * D + i]));
    constexpr int PPR = D * 2 / 16;
    const uint16_t* kb = a.kc + ((size_t)g * a.n_ctx + t0) * D;
    for (int i = tid; i < nt * PPR; i += 256) *(u32x4*)&ks[i / PPR][(i % PPR) * 8] = *(const u32x4*)(kb + (size_t)(i / PPR) * D + (i % PPR) * 8);
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6;
    if (lane >= nt) return;
    for (int hh = wave; hh < G; hh += 4) {
        float acc[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) acc[i] = 0.f;
#pragma unroll
        for (int d0 = 0; d0 < D; d0 += 8) {
            const u32x4 kv = *(const u32x4*)&ks[lane][d0];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = d0 + j;
                acc[i & 31] = __builtin_fmaf(h2f(kv[j >> 1] >> (16 * (j & 1))), qs[hh][i], acc[i & 31]);
            }
        }
        a.scores[(size_t)(g * G + hh) * a.n_ctx + t0 + lane] = x86_f16dot_reduce(acc) * a.scale;
    }
}

// softmax of one head over its scores row (in place -> p, padded with zeros to 32)
__global__ __launch_bounds__(256) void k_a86_softmax(AttnArgs a) {
    const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n_kv = a.st->pos + 1, np = (n_kv + 31) & ~31;
    float* w = a.scores + (size_t)h * a.n_ctx;
    __shared__ float redm[4];
    __shared__ double reds[4];
    float m = -INFINITY;
    for (int t = tid; t < n_kv; t += 256) m = fmaxf(m, w[t]);
    m = wave_max(m);
    if (lane == 0) redm[wave] = m;
    __syncthreads();
    const float mx = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
    // chunk c = positions 8c .. 8c+7 (masked positions: exactly 0, as v_expf(-inf))
    double sum = 0.0;
    for (int c = tid; 8 * c < n_kv; c += 256) {
        float e[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) e[l] = 8 * c + l < n_kv ? x86_v_expf(w[8 * c + l] - mx) : 0.f;
        sum += (double)x86_hsum8(e);
    }
    sum = wave_sum_d(sum);
    if (lane == 0) reds[wave] = sum;
    __syncthreads();
    const float inv = (float)(1.0 / ((reds[0] + reds[1]) + (reds[2] + reds[3])));
    // p over the thread's own chunks (e taken again: no thread reads another's writes)
    for (int c = tid; 8 * c < np; c += 256) {
        float p[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const int t = 8 * c + l;
            p[l] = t < n_kv ? h2f(f2h(x86_v_expf(w[t] - mx) * inv)) : 0.f;
        }
        *(float4*)(w + 8 * c) = make_float4(p[0], p[1], p[2], p[3]);
        *(float4*)(w + 8 * c + 4) = make_float4(p[4], p[5], p[6], p[7]);
    }
}

// PV: thread (dim d of 16, chain c of 32): chain c runs positions c, c + 32, ... < np
template <int D, int G>
__global__ __launch_bounds__(512) void k_a86_pv(AttnArgs a) {
    const int g = blockIdx.x, tid = threadIdx.x, c = tid & 31, d = blockIdx.y * 16 + (tid >> 5);
    const int n_kv = a.st->pos + 1, np = (n_kv + 31) & ~31;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    const float* p = a.scores + (size_t)g * G * a.n_ctx;
    float acc[G];
#pragma unroll
    for (int hh = 0; hh < G; ++hh) acc[hh] = 0.f;
    constexpr int U = 4;  // positions of a chain loaded ahead
    for (int t0 = c; t0 < np; t0 += 32 * U) {
        float v[U], pv[U][G];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = t0 + 32 * u;
            const int tc = min(t, a.n_ctx - 1);
            v[u] = t < n_kv ? h2f(vr[tc]) : 0.f;
#pragma unroll
            for (int hh = 0; hh < G; ++hh) pv[u][hh] = p[(size_t)hh * a.n_ctx + tc];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + 32 * u < np)
#pragma unroll
                for (int hh = 0; hh < G; ++hh) acc[hh] = __builtin_fmaf(v[u], pv[u][hh], acc[hh]);
    }
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        const float r = x86_f16dot_reduce_lanes(acc[hh]);
        if (c == 0) a.out[(size_t)(g * G + hh) * D + d] = r;
    }
}

// One launch: workgroup (head h, slice of DS dims), 512 threads, H x D/DS workgroups.
// The V slice is loaded first (registers, then LDS: it does not depend on the scores).
// Scores: a quad of lanes per position, lane q of the quad running the 8 chains
// 8q .. 8q+7 of the f16 dot (chain c over elements c, c + 32, ...), its 32 q values in
// registers; the 4 x 8-lane reduction of x86_f16dot_reduce is two quad DPP steps (xor 2:
// acc[l] + acc[16 + l], xor 1: + (acc[8 + l] + acc[24 + l]) of the partner) and the
// t0..t3 tree in the lane.  A wave takes 16 positions per pass (4 rows x 64 B per load:
// coalesced), U such rows per quad loaded at once (one pass covers 128 U positions: U
// from the KV bucket, at most 8).  Max, chunk sums and p as
// k_a86_softmax.  PV: 32 lanes per dim, lane c running chain c over positions c, c + 32,
// ... < np, reduced by x86_f16dot_reduce_lanes.
constexpr int kA86MaxKV = 2048, kA86Threads = 512;
__device__ __forceinline__ float a86_quad_reduce(float (&acc)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += xor_partner<2>(acc[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += xor_partner<1>(acc[j]);
    const float t0 = acc[0] + acc[4], t1 = acc[1] + acc[5], t2 = acc[2] + acc[6], t3 = acc[3] + acc[7];
    return (t0 + t1) + (t2 + t3);
}
#if defined(LLMI_EXP_TRACE)
#define A86_STAMP(I) if (threadIdx.x == 0 && a.trace) a.trace[blockIdx.x * 8 + (I)] = __builtin_amdgcn_s_memrealtime();
#else
#define A86_STAMP(I)
#endif
template <int D, int DS, int U>
__device__ __forceinline__ void a86_h_body(const AttnArgs& a, int n_head, int gq, int kvb, int stop) {
    // V staging registers sized for this pass class's largest KV bound (U: 128 U positions
    // per pass up to 512, else up to kA86MaxKV)
    constexpr int KVMAX = U >= 8 ? kA86MaxKV : 128 * U;
    constexpr int NT = kA86Threads, NW = NT / 64, VP = (DS * KVMAX / 8 + NT - 1) / NT, NE = D / 32;
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    const int vst = kvb + 8;                                  // V row stride (f16): rows off one bank quad
    float* wl = (float*)sm;                                   // [kvb]: scores, then p
    uint16_t* vs = (uint16_t*)(wl + kvb);                     // [DS][vst]
    __shared__ float redm[NW];
    __shared__ double reds[NW];
    const int h = blockIdx.x % n_head, d0 = (blockIdx.x / n_head) * DS, g = h / gq;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, qg = lane & 3;
    A86_STAMP(0)
    const int n_kv = a.st->pos + 1, np = (n_kv + 31) & ~31;
    const int prow = np >> 3;
    const uint16_t* vb = a.vc + ((size_t)g * D + d0) * a.n_ctx;
    u32x4 vr[VP];
#pragma unroll
    for (int k = 0; k < VP; ++k) {
        const int i = tid + k * NT;
        if (i < DS * prow) vr[k] = *(const u32x4*)(vb + (size_t)(i / prow) * a.n_ctx + (i % prow) * 8);
    }
    // the first pass's K rows, issued before q is waited on (their latencies overlap) where
    // the registers allow (head_dim 128 at 1024 positions per pass would spill)
    constexpr bool kHoist = U * NE <= 16;
    const uint16_t* K = a.kc + (size_t)g * a.n_ctx * D + 8 * qg;
    // a pass: U positions per quad, wave w takes positions pass * 128 U + 128 u + 16 w + lane / 4
    const int pw = wave * 16 + (lane >> 2);
    u32x4 kr[U][NE];
    if constexpr (kHoist)
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = min(NW * 16 * u + pw, n_kv - 1);
#pragma unroll
        for (int e = 0; e < NE; ++e) kr[u][e] = *(const u32x4*)(K + (size_t)t * D + 32 * e);
    }
    // this lane's q values: q[8 qg + 32 e + j], f16-rounded
    float qv[NE][8];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const float4 qa = *(const float4*)(a.q + (size_t)h * D + 8 * qg + 32 * e);
        const float4 qb = *(const float4*)(a.q + (size_t)h * D + 8 * qg + 32 * e + 4);
        const float qf[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) qv[e][j] = h2f(f2h(qf[j]));
    }
    A86_STAMP(1)
    if (stop == 1) return;
    float m = -INFINITY;
    for (int t0 = 0; t0 < n_kv; t0 += NW * 16 * U) {
        if (!kHoist || t0 > 0) {  // (uniform) the later passes
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = min(t0 + NW * 16 * u + pw, n_kv - 1);
#pragma unroll
                for (int e = 0; e < NE; ++e) kr[u][e] = *(const u32x4*)(K + (size_t)t * D + 32 * e);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = t0 + NW * 16 * u + pw;
            float acc[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
            for (int e = 0; e < NE; ++e)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    acc[j] = __builtin_fmaf(h2f(kr[u][e][j >> 1] >> (16 * (j & 1))), qv[e][j], acc[j]);
            const float w = a86_quad_reduce(acc) * a.scale;
            if (t < n_kv) {
                if (qg == 0) wl[t] = w;
                m = fmaxf(m, w);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < VP; ++k) {
        const int i = tid + k * NT;
        if (i < DS * prow) *(u32x4*)(vs + (size_t)(i / prow) * vst + (i % prow) * 8) = vr[k];
    }
    m = wave_max(m);
    if (lane == 0) redm[wave] = m;
    __syncthreads();
    A86_STAMP(2)
    if (stop == 2) return;
    float mx = redm[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) mx = fmaxf(mx, redm[w]);
    // one exp per thread (position t, kept in wl[t] for p), the 8-position chunk sums of
    // the AVX2 code, ((e0 + e4) + (e2 + e6)) + ((e1 + e5) + (e3 + e7)), across each 8-lane
    // group by DPP: lane 4 + i takes e_i by row_shr:4 (t_i = e_i + e_{i+4} in lanes 4..7; the
    // xor-4 helper's half-mirror would pair e_i with e_{7-i}), then quad xor 2 and xor 1;
    // the chunk sums (lane 4 of each group) into the double total
    double sum = 0.0;
    const int n8 = (n_kv + 7) & ~7;
    for (int t = tid; t < n8; t += NT) {
        const float e = t < n_kv ? x86_v_expf(wl[t] - mx) : 0.f;
        wl[t] = e;
        const float t4 = e + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(e), 0x114, 0xF, 0xF, false));
        const float t2 = t4 + xor_partner<2>(t4);
        const float c = t2 + xor_partner<1>(t2);
        if ((lane & 7) == 4) sum += (double)c;
    }
    sum = wave_sum_d(sum);
    if (lane == 0) reds[wave] = sum;
    __syncthreads();
    A86_STAMP(3)
    if (stop == 3) return;
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += reds[w];
    const float inv = (float)(1.0 / tot);
    for (int t = tid; t < np; t += NT) wl[t] = t < n_kv ? h2f(f2h(wl[t] * inv)) : 0.f;  // wl[t] = e (own thread)
    __syncthreads();
    A86_STAMP(4)
    if (stop == 4) return;
    // PV: 32 lanes per dim, lane c = chain c (positions c, c + 32, ...), 16 dims per pass
    const int c = lane & 31;
    for (int dl = tid >> 5; dl < DS; dl += NT / 32) {
        float acc = 0.f;
#pragma unroll 4
        for (int q = c; q < np; q += 32) {
            const float v = q < n_kv ? h2f(vs[dl * vst + q]) : 0.f;
            acc = __builtin_fmaf(v, wl[q], acc);
        }
        const float r = x86_f16dot_reduce_lanes(acc);
        if (c == 0) a.out[(size_t)h * D + d0 + dl] = r;
    }
    A86_STAMP(5)
}
template <int D, int DS, int U>
__global__ __launch_bounds__(kA86Threads) void k_a86_h(AttnArgs a, int n_head, int gq, int kvb, int stop) {
    a86_h_body<D, DS, U>(a, n_head, gq, kvb, stop);
}
// batched decode (batch.hip launch_battention): batch slot = blockIdx.y, its own sequence's
// caches, q, output and position (kvb: the batch's common KV bound)
template <int D, int DS, int U>
__global__ __launch_bounds__(kA86Threads) void k_ba86_h(BAttnArgs b, int n_head, int gq, int kvb) {
    a86_h_body<D, DS, U>(b.a[blockIdx.y], n_head, gq, kvb, 0);
}

template <int D, int G>
static hipError_t a86_launch(const AttnArgs& a, int n_head, int hk, int kv_bound, hipStream_t s, int mode) {
    if (mode != 3 && kv_bound <= kA86MaxKV) {
#if defined(LLMI_EXPERIMENTS)
        static const int stop = getenv("LLMI_EXP_A86_STOP") ? atoi(getenv("LLMI_EXP_A86_STOP")) : 0;
#else
        constexpr int stop = 0;
#endif
        constexpr int DS = 16;
        const size_t lds = (size_t)kv_bound * 4 + (size_t)DS * (kv_bound + 8) * 2;
        const dim3 grid(n_head * (D / DS));
        if (kv_bound <= 128) launch_k(k_a86_h<D, DS, 1>, grid, dim3(kA86Threads), lds, s, true, true, a, n_head, G, kv_bound, stop);
        else if (kv_bound <= 256) launch_k(k_a86_h<D, DS, 2>, grid, dim3(kA86Threads), lds, s, true, true, a, n_head, G, kv_bound, stop);
        else if (kv_bound <= 512) launch_k(k_a86_h<D, DS, 4>, grid, dim3(kA86Threads), lds, s, true, true, a, n_head, G, kv_bound, stop);
        else launch_k(k_a86_h<D, DS, 8>, grid, dim3(kA86Threads), lds, s, true, true, a, n_head, G, kv_bound, stop);
        return hipGetLastError();
    }
    launch_k(k_a86_scores<D, G>, dim3(hk, (kv_bound + 63) / 64), dim3(256), 0, s, true, false, a);
    launch_k(k_a86_softmax, dim3(n_head), dim3(256), 0, s, false, false, a);
    launch_k(k_a86_pv<D, G>, dim3(hk, D / 16), dim3(512), 0, s, false, true, a);
    return hipGetLastError();
}

// 32-dim slices (half the workgroups of the single-sequence launch: nt heads' worth of
// workgroups already fill the chip, and each slice recomputes its head's scores)
template <int D>
static hipError_t ba86_launch(const BAttnArgs& b, int nt, int n_head, int G, int kv_bound, hipStream_t s) {
    constexpr int DS = 32;
    const size_t lds = (size_t)kv_bound * 4 + (size_t)DS * (kv_bound + 8) * 2;
    const dim3 grid(n_head * (D / DS), nt);
    if (kv_bound <= 128) launch_k(k_ba86_h<D, DS, 1>, grid, dim3(kA86Threads), lds, s, true, true, b, n_head, G, kv_bound);
    else if (kv_bound <= 256) launch_k(k_ba86_h<D, DS, 2>, grid, dim3(kA86Threads), lds, s, true, true, b, n_head, G, kv_bound);
    else if (kv_bound <= 512) launch_k(k_ba86_h<D, DS, 4>, grid, dim3(kA86Threads), lds, s, true, true, b, n_head, G, kv_bound);
    else launch_k(k_ba86_h<D, DS, 8>, grid, dim3(kA86Threads), lds, s, true, true, b, n_head, G, kv_bound);
    return hipGetLastError();
}
// the batched step's x86 attention: one launch for every slot up to kA86MaxKV positions, past
// it the three-launch form per slot
hipError_t launch_battention_x86(const BAttnArgs& b, int nt, int n_head, int n_head_kv, int head_dim, int kv_bound,
                                 hipStream_t s) {
    if (nt < 1 || nt > kMaxBatch || n_head_kv <= 0 || n_head % n_head_kv) return hipErrorInvalidValue;
    if (head_dim != 128 && head_dim != 64) return hipErrorInvalidValue;
    if (kv_bound > kA86MaxKV) {
        for (int t = 0; t < nt; ++t) {
            const hipError_t e = launch_attention_x86(b.a[t], n_head, n_head_kv, head_dim, kv_bound, s, 0);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const int G = n_head / n_head_kv;
    return head_dim == 128 ? ba86_launch<128>(b, nt, n_head, G, kv_bound, s) : ba86_launch<64>(b, nt, n_head, G, kv_bound, s);
}

hipError_t launch_attention_x86(const AttnArgs& a, int n_head, int n_head_kv, int head_dim, int kv_bound, hipStream_t s,
                                int mode) {
    if (n_head_kv <= 0 || n_head % n_head_kv) return hipErrorInvalidValue;
    const int g = n_head / n_head_kv;
#define LLMI_A86(D_, G_) \
    if (head_dim == D_ && g == G_) return a86_launch<D_, G_>(a, n_head, n_head_kv, kv_bound, s, mode);
    LLMI_A86(128, 1) LLMI_A86(128, 2) LLMI_A86(128, 4) LLMI_A86(128, 8)
    LLMI_A86(64, 1) LLMI_A86(64, 2) LLMI_A86(64, 4) LLMI_A86(64, 8)
#undef LLMI_A86
    return hipErrorInvalidValue;
}

// ---- prefill -----------------------------------------------------------------------
// k_pf_a86: grid (HK, T), 256 threads: query token t (position pos0 + t) for the G heads of
// KV group g, scores and p in LDS ([G][ldw], ldw = max_kv rounded up to 32); the same
// operations as the decode kernels above.
template <int D, int G>
__global__ __launch_bounds__(256) void k_pf_a86(PfAttn a) {
    extern __shared__ __attribute__((aligned(16))) float wl[];  // [G][ldw]
    __shared__ float qs[G][D];
    __shared__ float redm[4][G];
    __shared__ double reds[4][G];
    const int g = blockIdx.x, t = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ldw = (a.max_kv + 31) & ~31;
    const int n_kv = a.pos0 + t + 1, np = (n_kv + 31) & ~31;
    for (int i = tid; i < G * D; i += 256) qs[i / D][i % D] = h2f(f2h(a.q[(size_t)t * a.ldq + (size_t)g * G * D + i]));
    __syncthreads();
    const uint16_t* K = a.kc + (size_t)g * a.n_ctx * D;
    float mx[G];
#pragma unroll
    for (int hh = 0; hh < G; ++hh) mx[hh] = -INFINITY;
    for (int p = tid; p < n_kv; p += 256) {
        u32x4 kr[D / 8];
#pragma unroll
        for (int k = 0; k < D / 8; ++k) kr[k] = *(const u32x4*)(K + (size_t)p * D + 8 * k);
#pragma unroll
        for (int hh = 0; hh < G; ++hh) {
            float acc[32];
#pragma unroll
            for (int i = 0; i < 32; ++i) acc[i] = 0.f;
#pragma unroll
            for (int i = 0; i < D; ++i)
                acc[i & 31] = __builtin_fmaf(h2f(kr[i >> 3][(i & 7) >> 1] >> (16 * (i & 1))), qs[hh][i], acc[i & 31]);
            const float w = x86_f16dot_reduce(acc) * a.scale;
            wl[hh * ldw + p] = w;
            mx[hh] = fmaxf(mx[hh], w);
        }
    }
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        const float m = wave_max(mx[hh]);
        if (lane == 0) redm[wave][hh] = m;
    }
    __syncthreads();
#pragma unroll
    for (int hh = 0; hh < G; ++hh) mx[hh] = fmaxf(fmaxf(redm[0][hh], redm[1][hh]), fmaxf(redm[2][hh], redm[3][hh]));
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        double sum = 0.0;
        for (int c = tid; 8 * c < n_kv; c += 256) {
            float e[8];
#pragma unroll
            for (int l = 0; l < 8; ++l) e[l] = 8 * c + l < n_kv ? x86_v_expf(wl[hh * ldw + 8 * c + l] - mx[hh]) : 0.f;
            sum += (double)x86_hsum8(e);
        }
        sum = wave_sum_d(sum);
        if (lane == 0) reds[wave][hh] = sum;
    }
    __syncthreads();  // also: every score written before any p replaces it
#pragma unroll
    for (int hh = 0; hh < G; ++hh) {
        const float inv = (float)(1.0 / ((reds[0][hh] + reds[1][hh]) + (reds[2][hh] + reds[3][hh])));
        for (int c = tid; 8 * c < np; c += 256)
#pragma unroll
            for (int l = 0; l < 8; ++l) {
                const int q = 8 * c + l;
                wl[hh * ldw + q] = q < n_kv ? h2f(f2h(x86_v_expf(wl[hh * ldw + q] - mx[hh]) * inv)) : 0.f;
            }
    }
    __syncthreads();
    // PV: thread (chain c, dim group dg): dims dg + 8 k, G heads
    const int c = tid & 31, dg = tid >> 5;
    constexpr int ND = D / 8;
    const uint16_t* V = a.vc + (size_t)g * D * a.n_ctx;
    float acc[ND][G];
#pragma unroll
    for (int k = 0; k < ND; ++k)
#pragma unroll
        for (int hh = 0; hh < G; ++hh) acc[k][hh] = 0.f;
    for (int q = c; q < np; q += 32) {
        float pv[G];
#pragma unroll
        for (int hh = 0; hh < G; ++hh) pv[hh] = wl[hh * ldw + q];
        const int qc = min(q, a.n_ctx - 1);
#pragma unroll
        for (int k = 0; k < ND; ++k) {
            const float v = q < n_kv ? h2f(V[(size_t)(dg + 8 * k) * a.n_ctx + qc]) : 0.f;
#pragma unroll
            for (int hh = 0; hh < G; ++hh) acc[k][hh] = __builtin_fmaf(v, pv[hh], acc[k][hh]);
        }
    }
#pragma unroll
    for (int k = 0; k < ND; ++k)
#pragma unroll
        for (int hh = 0; hh < G; ++hh) {
            const float r = x86_f16dot_reduce_lanes(acc[k][hh]);
            if (c == 0) a.out[(size_t)t * a.ldq + (size_t)(g * G + hh) * D + dg + 8 * k] = r;
        }
}

// longest KV the prefill kernel's LDS score rows take (the rest of a prompt: decode steps)
int pf_attn_x86_max_kv(int n_head, int n_head_kv, int head_dim) {
    (void)head_dim;
    const int g = n_head / n_head_kv;
    const size_t static_lds = (size_t)g * head_dim * 4 + 4 * g * 12 + 64;
    return (int)(((160u * 1024u - static_lds) / (4u * (size_t)g)) & ~(size_t)31);
}

hipError_t launch_pf_attn_x86(const PfAttn& a, int n_head, int n_head_kv, int head_dim, int T, hipStream_t s) {
    if (n_head_kv <= 0 || n_head % n_head_kv || T <= 0) return hipErrorInvalidValue;
    const int g = n_head / n_head_kv;
    if (a.max_kv > pf_attn_x86_max_kv(n_head, n_head_kv, head_dim)) return hipErrorInvalidValue;
    // (gfx950 takes up to 160 KiB of dynamic LDS as is; the attribute call is refused,
    // prefill.hip.inc launch_pf_attn)
    const size_t lds = (size_t)g * ((a.max_kv + 31) & ~31) * 4;
#define LLMI_PA86(D_, G_)                                                                     \
    if (head_dim == D_ && g == G_) {                                                          \
        launch_k(k_pf_a86<D_, G_>, dim3(n_head_kv, T), dim3(256), lds, s, true, true, a);     \
        return hipGetLastError();                                                             \
    }
    LLMI_PA86(128, 1) LLMI_PA86(128, 2) LLMI_PA86(128, 4) LLMI_PA86(128, 8)
    LLMI_PA86(64, 1) LLMI_PA86(64, 2) LLMI_PA86(64, 4) LLMI_PA86(64, 8)
#undef LLMI_PA86
    return hipErrorInvalidValue;
}

}  // namespace llmi
