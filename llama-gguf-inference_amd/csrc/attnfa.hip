// attnfa.hip — decode attention in the flash-attention numerics (model numerics bit
// LLMI_NUMERICS_FA).
//
// Upstream's CPU ggml_compute_forward_flash_attn_ext_f16 for one query row with f16 K/V
// [ggml-cpu ops.cpp "one_chunk"; upstream, recalled, not vendored] — what llama-server's
// `-fa auto` (start.sh passes no --flash-attn) runs on the reference's CPU path — as the
// oracle restates it (oracle/ggml_oracle.c attn_head_fa):
//   s[t]   = dot_f16(K[t], f16(q)) * scale + 0          (generic: double sum in element
//            order; X86: the 4 x 8-lane fp32 fma chains of the AVX2+F16C build)
//   per t in order: if s[t] > M { ms = expf(M - s[t]); M = s[t]; VKQ = f16(f32(VKQ) * ms) }
//                   else        { vs = expf(s[t] - M) }
//                   VKQ = f16(f32(VKQ) + f32(V[t]) * vs)   (X86: one fp32 fma)
//                   S = S * ms + vs                        (X86: fma)
//   out = f32(VKQ) * (S == 0 ? 0 : 1 / S)
// with glibc's expf (llmi_expf_glibc, FMA build; pinned to a real glibc by
// tests/test_oracle_math.py).
//
// The per-position f16 rounding of VKQ makes the recurrence sequential in t, so the
// kernel (one 256-thread workgroup per query head) takes it apart:
//   1. scores, one thread per position, into LDS
//   2. the running max is a prefix max (exact in any association): a block scan; every
//      position's factors then depend only on (s[t], max of s[0..t-1]) and are computed in
//      parallel: new max -> ms = expf(Mold - s), vs = 1; else ms = 1, vs = expf(s - Mold)
//   3. thread d runs dim d's recurrence over t (scaling by ms = 1 is exact, so the scale
//      step runs unconditionally), V streamed 8 positions per 16-B load; every thread runs
//      the S recurrence beside it
// Exact against the oracle for every association (nothing is reordered but the max).
#include "kernels.h"
#include "launch_util.h"
#include "mv_device.h"

namespace llmi {

namespace {

template <int D, int X86>
__device__ __forceinline__ void attn_fa_body(const AttnArgs& a, int G) {
    extern __shared__ __attribute__((aligned(16))) float fa_lds[];
    float* sc = fa_lds;               // [kFaMaxKV] scores, then vs
    float* msv = fa_lds + kFaMaxKV;   // [kFaMaxKV] ms
    __shared__ float qs[D];
    __shared__ float cmax[256];
    const int h = blockIdx.x, g = h / G, tid = threadIdx.x;
    const int n_kv = a.st->pos + 1;
    for (int d = tid; d < D; d += 256) qs[d] = h2f(f2h(a.q[(size_t)h * D + d]));
    __syncthreads();
    // 1. scores
    const uint16_t* kb = a.kc + (size_t)g * a.n_ctx * D;
    for (int t = tid; t < n_kv; t += 256) {
        const uint16_t* kr = kb + (size_t)t * D;
        float s;
        if constexpr (X86) {
            float acc[32];
#pragma unroll
            for (int i = 0; i < 32; ++i) acc[i] = 0.f;
#pragma unroll
            for (int d0 = 0; d0 < D; d0 += 8) {
                const u32x4 kv = *(const u32x4*)(kr + d0);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int i = d0 + j;
                    acc[i & 31] = __builtin_fmaf(h2f((uint16_t)(kv[j >> 1] >> (16 * (j & 1)))), qs[i], acc[i & 31]);
                }
            }
            float c[8];
#pragma unroll
            for (int l = 0; l < 8; ++l) c[l] = (acc[l] + acc[16 + l]) + (acc[8 + l] + acc[24 + l]);
            const float t0 = c[0] + c[4], t1 = c[1] + c[5], t2 = c[2] + c[6], t3 = c[3] + c[7];
            s = (float)(double)((t0 + t1) + (t2 + t3));
        } else {
            double sum = 0.0;
#pragma unroll
            for (int d0 = 0; d0 < D; d0 += 8) {
                const u32x4 kv = *(const u32x4*)(kr + d0);
#pragma unroll
                for (int j = 0; j < 8; ++j) sum += (double)(h2f((uint16_t)(kv[j >> 1] >> (16 * (j & 1)))) * qs[d0 + j]);
            }
            s = (float)sum;
        }
        s = s * a.scale;
        sc[t] = s + 0.0f;  // + slope * mask (0 for every position the query sees)
    }
    __syncthreads();
    // 2. exclusive prefix max over t: thread tid owns positions [tid * C, tid * C + C)
    const int C = (n_kv + 255) / 256, lo = tid * C, hi = min(n_kv, lo + C);
    float m = -INFINITY;
    for (int t = lo; t < hi; ++t) m = fmaxf(m, sc[t]);
    cmax[tid] = m;
    __syncthreads();
    float prev = -INFINITY;
    for (int j = 0; j < tid; ++j) prev = fmaxf(prev, cmax[j]);
    for (int t = lo; t < hi; ++t) {
        const float s = sc[t];
        float ms = 1.0f, vs = 1.0f;
        if (s > prev) {
            ms = llmi_expf_glibc(prev - s, 1);
            prev = s;
        } else {
            vs = llmi_expf_glibc(s - prev, 1);
        }
        msv[t] = ms;
        sc[t] = vs;
    }
    __syncthreads();
    // 3. dim d's recurrence, V row of dim d streamed 8 positions per load (transposed V)
    if (tid >= D) return;
    const uint16_t* vr = a.vc + ((size_t)g * D + tid) * a.n_ctx;
    uint16_t y = 0;
    float S = 0.0f;
    const int nb = (n_kv + 7) / 8;
    u32x4 cur = *(const u32x4*)vr;
    for (int b = 0; b < nb; ++b) {
        const u32x4 nxt = *(const u32x4*)(vr + 8 * min(b + 1, nb - 1));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = 8 * b + j;
            if (t < n_kv) {
                const float ms = msv[t], vs = sc[t];
                const float v = h2f((uint16_t)(cur[j >> 1] >> (16 * (j & 1))));
                y = f2h(h2f(y) * ms);
                if constexpr (X86) {
                    y = f2h(__builtin_fmaf(v, vs, h2f(y)));
                    S = __builtin_fmaf(S, ms, vs);
                } else {
                    y = f2h(h2f(y) + v * vs);
                    S = S * ms + vs;
                }
            }
        }
        cur = nxt;
    }
    const float S_inv = S == 0.0f ? 0.0f : 1.0f / S;
    a.out[(size_t)h * D + tid] = h2f(y) * S_inv;
}
template <int D, int X86>
__global__ __launch_bounds__(256) void k_attn_fa(AttnArgs a, int G) { attn_fa_body<D, X86>(a, G); }
// batched decode: batch slot = blockIdx.y (its own sequence's caches, q, output, position)
template <int D, int X86>
__global__ __launch_bounds__(256) void k_battn_fa(BAttnArgs b, int G) { attn_fa_body<D, X86>(b.a[blockIdx.y], G); }

}  // namespace

hipError_t launch_battention_fa(const BAttnArgs& b, int nt, int n_head, int n_head_kv, int head_dim, int kv_bound,
                                hipStream_t s) {
    const AttnArgs& a = b.a[0];
    if (nt < 1 || nt > kMaxBatch || n_head_kv <= 0 || n_head % n_head_kv || kv_bound > kFaMaxKV || kv_bound > a.n_ctx ||
        a.n_ctx % 8)
        return hipErrorNotSupported;
    const int G = n_head / n_head_kv, x86 = a.num ? 1 : 0;
    const size_t lds = (size_t)2 * kFaMaxKV * 4;
#define LLMI_BFA(D_, X_) \
    if (head_dim == D_ && x86 == X_) { launch_k(k_battn_fa<D_, X_>, dim3(n_head, nt), dim3(256), lds, s, true, true, b, G); return hipGetLastError(); }
    LLMI_BFA(128, 0) LLMI_BFA(128, 1) LLMI_BFA(64, 0) LLMI_BFA(64, 1)
#undef LLMI_BFA
    return hipErrorNotSupported;
}

hipError_t launch_attention_fa(const AttnArgs& a, int n_head, int n_head_kv, int head_dim, int kv_bound, hipStream_t s) {
    if (n_head_kv <= 0 || n_head % n_head_kv || kv_bound > kFaMaxKV || kv_bound > a.n_ctx || a.n_ctx % 8)
        return hipErrorNotSupported;
    const int G = n_head / n_head_kv, x86 = a.num ? 1 : 0;
    const size_t lds = (size_t)2 * kFaMaxKV * 4;
#define LLMI_FA(D_, X_) \
    if (head_dim == D_ && x86 == X_) { launch_k(k_attn_fa<D_, X_>, dim3(n_head), dim3(256), lds, s, true, true, a, G); return hipGetLastError(); }
    LLMI_FA(128, 0) LLMI_FA(128, 1) LLMI_FA(64, 0) LLMI_FA(64, 1)
#undef LLMI_FA
    return hipErrorNotSupported;
}

}  // namespace llmi
