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
#include "mv_device.h"
#include "pf_device.h"
#include "launch_util.h"

#include <algorithm>
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
hipEvent_t launch_event(bool stop) { return stop ? t_ev_stop : t_ev_start; }

// LDS of a matvec workgroup: the activation image, the prologue's reduction slots, then
// one fold buffer (mv_device.h kFoldFloats) per wave
size_t mv_lds_bytes(int act, int cols) { return fold_off(act, cols, kMVWaves) + (size_t)kMVWaves * kFoldFloats * 4; }


// The prologue's quantized activation written out in ggml block form (test hook).
template <int ACT, int X86>
__global__ __launch_bounds__(kMVThreads) void k_quant_dump(MVArgs A, uint8_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Lds L = carve(smem, ACT, A.cols);
    if (A.nw) mv_prologue<ACT, true, X86>(A, L);
    else mv_prologue<ACT, false, X86>(A, L);
    __syncthreads();
    const int cols = A.cols;
    for (int e = threadIdx.x; e < cols; e += blockDim.x) {
        const uint8_t* rec = L.act + (size_t)(e >> 8) * kRec;
        const int t = e & 255;
        if (ACT == 0) {  // residue order: element 64c + 32h + l + 8i at part 2c + l/4, half h, byte 4 (l % 4) + i
                         // (x86: element 64c + 32h + 4l + i)
            const int c = t >> 6, h = (t >> 5) & 1, l = X86 ? (t & 31) >> 2 : t & 7, i = X86 ? t & 3 : (t & 31) >> 3;
            out[(size_t)(e >> 8) * 292 + 4 + t] = rec[32 * (2 * c + (l >> 2)) + 16 * h + 4 * (l & 3) + i];
        } else {
            out[(size_t)(e >> 5) * 34 + 2 + (e & 31)] = rec[t];
        }
    }
    if (ACT == 0) {
        for (int b = threadIdx.x; b < cols / 256; b += blockDim.x)
            *(float*)(out + (size_t)b * 292) = *(const float*)(L.act + (size_t)b * kRec + kRecD);
        for (int sb = threadIdx.x; sb < cols / 16; sb += blockDim.x)
            *(int16_t*)(out + (size_t)(sb >> 4) * 292 + 260 + 2 * (sb & 15)) =
                *(const int16_t*)(L.act + (size_t)(sb >> 4) * kRec + kRecBs + 2 * (sb & 15));
    } else {
        for (int b = threadIdx.x; b < cols / 32; b += blockDim.x)
            *(uint16_t*)(out + (size_t)b * 34) = f2h(*(const float*)(L.act + (size_t)(b >> 3) * kRec + kRecBs + 4 * (b & 7)));
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

// Split attention v2 (bodies in mv_device.h: attn_scores8_body / attn_pv16_body, shared
// with the batched decode's per-sequence launches in batch.hip).
template <int D, int G>
__global__ __launch_bounds__(256) void k_attn_scores8(AttnArgs a) { attn_scores8_body<D, G>(a); }
template <int D, int G>
__global__ __launch_bounds__(512) void k_attn_pv16(AttnArgs a, int kvb) { attn_pv16_body<D, G>(a, kvb); }

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
    LLMI_ATT_STAMP(0, 0)
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
    LLMI_ATT_STAMP(0, 1)
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
    LLMI_ATT_STAMP(0, 2)
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
    LLMI_ATT_STAMP(0, 3)
}

// Register-prefetched one-launch attention for short contexts (kv_bound <= 64*P <= 512):
// one 512-thread workgroup per query head.  Every global load of the launch — the step
// position, the head's q slice, all kv_bound K rows and the V window — is issued at
// entry (addresses clamped into the bucket, never gated on the position), so one memory
// latency covers the launch; the rest is the dependent compute chain:
//   scores  8 lanes x D/8 dims per position (exact f16 products summed in double, 3-step
//           butterfly), P passes of 64 positions; scores to LDS, row max per wave
//   softmax e = expf(s - max), double sum over the workgroup (fixed order), p =
//           f16(e * (float)(1/sum)) in LDS as f32 — the formulas of k_attn_fused
//   PV      512/D lanes per output dim, double fma of exact f16 products, butterfly.
// Same numerics as the other paths (the double sums are exact in practice; the paths
// are checked bit-identical against each other and the oracle).
template <int D, int P>
__global__ __launch_bounds__(512) void k_attn_r(AttnArgs a, int G, int kvb) {
    constexpr int DQ = D / 8;          // score dims per lane
    constexpr int SLV = 512 / D;       // PV lanes per output dim (4 or 8)
    constexpr int NVL = 64 * P / (8 * SLV);  // 16-B V loads per lane (8 positions each)
    __shared__ __attribute__((aligned(16))) float sp[64 * P + 8];
    __shared__ float redm[8];
    __shared__ double reds[8];
    LLMI_ATT_STAMP(0, 0)
    const int h = blockIdx.x, g = h / G;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int qd = tid & 7, pp = tid >> 3;
    // 1. every load up front: position, q slice, K rows of all passes, V window
    const int pos = a.st->pos;
    float4 qv[DQ / 4];
#pragma unroll
    for (int i = 0; i < DQ / 4; ++i) qv[i] = *(const float4*)(a.q + (size_t)h * D + qd * DQ + 4 * i);
    u32x4 kv[P][DQ / 8];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int t = min(64 * p + pp, kvb - 1);
        const uint16_t* kr = a.kc + ((size_t)g * a.n_ctx + t) * D + qd * DQ;
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i) kv[p][i] = __builtin_nontemporal_load((const u32x4*)(kr + 8 * i));
    }
    const int d = tid / SLV, sl = tid % SLV;
    const uint16_t* vr = a.vc + ((size_t)g * D + d) * a.n_ctx;
    u32x4 vv[NVL];
#pragma unroll
    for (int u = 0; u < NVL; ++u) vv[u] = __builtin_nontemporal_load((const u32x4*)(vr + min(8 * sl + 8 * SLV * u, kvb - 8)));
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
        const int t = 64 * p + pp;
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
    // 3. softmax: thread t owns position t (64*P <= 512 positions)
    float e = 0.f;
    double s = 0.0;
    if (tid < n_kv && tid < 64 * P) {
        e = llmi_expf(sp[tid] - mx);
        s = (double)e;
    }
    s = wave_sum_d(s);
    if (lane == 0) reds[wave] = s;
    __syncthreads();
    double tot = reds[0];
#pragma unroll
    for (int w = 1; w < 8; ++w) tot += reds[w];
    const float inv = (float)(1.0 / tot);
    if (tid < 64 * P) sp[tid] = tid < n_kv ? h2f(f2h(e * inv)) : 0.f;
    __syncthreads();
    LLMI_ATT_STAMP(0, 2)
    // 4. PV: lane sl covers positions 8*sl + 8*SLV*u + j; two double chains
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
    acc += xor_partner_d<1>(acc);
    acc += xor_partner_d<2>(acc);
    if constexpr (SLV == 8) acc += xor_partner_d<4>(acc);
    if (sl == 0) a.out[(size_t)h * D + d] = (float)acc;
    LLMI_ATT_STAMP(0, 3)
}

// Long-context attention (path 7): bodies in mv_device.h (shared with batch.hip)
template <int D, int G, int NP>
__global__ __launch_bounds__(256) void k_attl_scores(AttnArgs a) { attl_scores_body<D, G, NP>(a); }
__global__ __launch_bounds__(256) void k_attl_exp(AttnArgs a, int n_head, int kvb) { attl_exp_body(a, n_head, kvb); }
template <int D, int G>
__global__ __launch_bounds__(512) void k_attl_pv(AttnArgs a, int n_head, int kvb) { attl_pv_body<D, G>(a, n_head, kvb); }
template <int D>
__global__ __launch_bounds__(D) void k_attl_sum(AttnArgs a, int n_head) { attl_sum_body<D>(a, n_head); }

// Dim-split one-launch attention (path 6): body in mv_device.h (shared with batch.hip)
template <int D, int P, int S>
__global__ __launch_bounds__(512) void k_attn_d(AttnArgs a, int G, int HK, int kvb, int pf) {
    attn_d_body<D, P, S>(a, G, HK, kvb, pf & 1, (pf >> 1) & 1);
}

// ----------------------------------------------------------------------------------
// Step entry: choose the token, advance pos, dequantize its embedding row
// (upstream ggml_get_rows + dequantize_row_*; bit-exact).
// Reads the piece-planar device layout (common.h).
// ----------------------------------------------------------------------------------
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

// get_rows of the last step's token (st->token, set by k_embed) with k_embed's dequant:
// the per-op check of SURVEY.md §8a row a10 (llmi_debug_tap 0)
__global__ __launch_bounds__(256) void k_embed_row(Seg w, int cols, int vocab, const StepState* st, float* out) {
    int tok = st->token;
    if (tok < 0 || tok >= vocab) tok = 0;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e < cols) out[e] = dequant_elem(w, tok, e, cols);
}
hipError_t launch_embed_row(const EmbArgs& a, const StepState* st, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_embed_row, dim3((a.cols + 255) / 256), dim3(256), 0, s, a.w, a.cols, a.vocab, st, out);
    return hipGetLastError();
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
// Load-time repack of GGUF blocks into the unit-major layout (common.h).
// One thread per (block, chunk c in 0..3); nbr = blocks (units) per row.
// ----------------------------------------------------------------------------------
// x86 = 1: the x86-numerics byte order (common.h): part 2c + k = native bytes, i.e. byte
// 4m + i of part 2c + k holds chunk elements t = 16k + 4m + i (low nibble) and 32 + t
__global__ void k_repack_kq(int type, const uint8_t* raw, uint8_t* A, uint8_t* H, uint8_t* S, uint8_t* Dp, int64_t nblk,
                            int nbr, int rgs, int x86) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = gid >> 2;
    const int c = (int)(gid & 3);
    if (b >= nblk) return;
    const int64_t row = b / nbr, u = b % nbr, U = nbr;
    // piece (row, part p, unit u) at A + piece_off(row, p, u, U, 8, rgs) (common.h ROW GROUPS)
    auto apiece = [&](int p) { return A + piece_off((uint32_t)row, (uint32_t)p, (uint32_t)u, (uint32_t)U, 8, rgs); };
    // residue order: byte 4m + i of part 2c + k holds chunk elements t = l + 8i (low
    // nibble) and 32 + t (high nibble), l = 4k + m
    if (type == T_Q4_K || type == T_Q5_K) {
        const int bb = type == T_Q4_K ? 144 : 176;
        const uint8_t* x = raw + b * bb;
        const uint8_t* qs = x + (type == T_Q4_K ? 16 : 48);
        // chunk element of (l = 4k + m, byte i): residue order l + 8i, x86 order 4l + i
        auto el = [&](int l, int i) { return x86 ? 4 * l + i : l + 8 * i; };
        for (int k = 0; k < 2; ++k)
            for (int m = 0; m < 4; ++m)
                for (int i = 0; i < 4; ++i) apiece(2 * c + k)[4 * m + i] = qs[32 * c + el(4 * k + m, i)];
        if (c == 0)
            for (int i = 0; i < 16; ++i) S[b * 16 + i] = x[i];
        if (type == T_Q5_K) {  // byte i, bit l of the lo word: qh[el(l, i)] bit 2c; hi word: bit 2c+1
            const uint8_t* qh = x + 16;
            uint8_t* h = H + piece_off((uint32_t)row, (uint32_t)(c >> 1), (uint32_t)u, (uint32_t)U, 2, rgs) + 8 * (c & 1);
            for (int i = 0; i < 4; ++i) {
                uint8_t lo = 0, hi = 0;
                for (int l = 0; l < 8; ++l) {
                    lo |= (uint8_t)(((qh[el(l, i)] >> (2 * c)) & 1) << l);
                    hi |= (uint8_t)(((qh[el(l, i)] >> (2 * c + 1)) & 1) << l);
                }
                h[i] = lo;
                h[4 + i] = hi;
            }
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
        auto el = [&](int l, int i) { return x86 ? 4 * l + i : l + 8 * i; };
        for (int k = 0; k < 2; ++k)
            for (int m = 0; m < 4; ++m)
                for (int i = 0; i < 4; ++i) {
                    const int t = el(4 * k + m, i);
                    apiece(2 * c + k)[4 * m + i] =
                        (uint8_t)((u6(64 * c + t) & 15) | ((u6(64 * c + 32 + t) & 15) << 4));
                }
        // H part c, dword g = 2*hi + k: byte i bits [2m, 2m+1] = (high 2 bits of chunk
        // element 32*hi + el(4k + m, i)) XOR 2, which v_perm turns into the high part of q - 32
        uint8_t* h = H + piece_off((uint32_t)row, (uint32_t)c, (uint32_t)u, (uint32_t)U, 4, rgs);
        for (int g = 0; g < 4; ++g)
            for (int i = 0; i < 4; ++i) {
                uint8_t v = 0;
                for (int m = 0; m < 4; ++m)
                    v |= (uint8_t)(((u6(64 * c + 32 * (g >> 1) + el(4 * (g & 1) + m, i)) >> 4) ^ 2) << (2 * m));
                h[4 * g + i] = v;
            }
        for (int i = 0; i < 4; ++i) S[b * 16 + 4 * c + i] = x[192 + 4 * c + i];
        if (c == 0) { Dp[b * 2] = x[208]; Dp[b * 2 + 1] = x[209]; }
    }
}

// Q8_0: one thread per 32-block; unit u = 8 blocks, block b of the unit in parts 2b, 2b+1
__global__ void k_repack_q80(const uint8_t* raw, uint8_t* A, uint8_t* Dp, int64_t nblk, int nb_row, int rgs) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nblk) return;
    const int64_t row = g / nb_row, bi = g % nb_row, U = nb_row / 8, u = bi >> 3, b = bi & 7;
    const uint8_t* x = raw + g * 34;
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < 16; ++i)
            A[piece_off((uint32_t)row, (uint32_t)(2 * b + h), (uint32_t)u, (uint32_t)U, 16, rgs) + i] = x[2 + 16 * h + i];
    Dp[(row * U + u) * 16 + 2 * b] = x[0];
    Dp[(row * U + u) * 16 + 2 * b + 1] = x[1];
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

// Arena hash (replica check): H = sum over 8-byte words i (mod 2^64) of
// mix64(word_i ^ (i * phi)), mix64 = splitmix64's finalizer; the last partial word is
// zero-padded.  A sum of per-position terms is independent of the order the grid visits
// the words in, so every replica of the same bytes gets the same value on any device
// (tests/test_fanout_check.py restates it in numpy).
__device__ __forceinline__ unsigned long long hash_mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void k_arena_hash(const uint8_t* p, size_t bytes, unsigned long long* out) {
    const size_t nw = bytes >> 3, n16 = bytes >> 4;
    unsigned long long acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const u32x4 v = ldw(p + i * 16);
        const unsigned long long w0 = ((unsigned long long)v.y << 32) | v.x, w1 = ((unsigned long long)v.w << 32) | v.z;
        acc += hash_mix64(w0 ^ ((2 * i) * 0x9E3779B97F4A7C15ull));
        acc += hash_mix64(w1 ^ ((2 * i + 1) * 0x9E3779B97F4A7C15ull));
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the word past the last 16-B piece, and the tail
        for (size_t i = 2 * n16; i * 8 < bytes; ++i) {
            unsigned long long w = 0;
            for (size_t b = 0; b < 8 && i * 8 + b < bytes; ++b) w |= (unsigned long long)p[i * 8 + b] << (8 * b);
            acc += hash_mix64(w ^ (i * 0x9E3779B97F4A7C15ull));
        }
    }
    (void)nw;
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

hipError_t launch_arena_hash(const void* p, size_t bytes, unsigned long long* out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, 8, s);
    if (e != hipSuccess) return e;
    const size_t n16 = bytes >> 4;
    const int blocks = (int)std::max<size_t>(1, std::min<size_t>(4096, (n16 + 255) / 256));
    hipLaunchKernelGGL(k_arena_hash, dim3(blocks), dim3(256), 0, s, (const uint8_t*)p, bytes, out);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------
// QKV whose segments form two contiguous type groups split at a task boundary: both groups
// pipelined (k_matvec's T2 path).  Returns hipErrorNotSupported when not applicable.
template <bool NORM, int X86>
static hipError_t mv_dispatch_qkv2(const MVArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    if (a.nseg < 2 || grid.x < 2) return hipErrorNotSupported;
    int t1 = a.seg[0].type, t2 = -1, split_row = -1;
    for (int i = 1; i < a.nseg; ++i) {
        if (a.seg[i].type == (t2 < 0 ? t1 : t2)) continue;
        if (t2 >= 0) return hipErrorNotSupported;  // a third group
        t2 = a.seg[i].type;
        split_row = a.seg[i].row0 - a.seg[0].row0;
    }
    if (t2 < 0 || split_row % a.rpt || a.cols > 16 * kMVThreads) return hipErrorNotSupported;
    const int sp = split_row / a.rpt;
#define LLMI_QKV2(A_, B_)                                                                            \
    if (t1 == A_ && t2 == B_) return mv_qkv2_launch<NORM, A_, B_, X86>(a, sp, grid, lds, s);
    if constexpr (NORM) {
        LLMI_QKV2(T_Q4_K, T_Q6_K) LLMI_QKV2(T_Q4_K, T_Q5_K) LLMI_QKV2(T_Q5_K, T_Q6_K)
    }
#undef LLMI_QKV2
    return hipErrorNotSupported;
}

template <bool NORM, int X86>
static hipError_t mv_dispatch_type(const MVArgs& a, int epi, dim3 grid, size_t lds, hipStream_t s) {
    static const bool qkv2 = !getenv("LLMI_NO_QKV2");  // A/B switch for measurements
    if (epi == EPI_QKV && qkv2) {
        const hipError_t e = mv_dispatch_qkv2<NORM, X86>(a, grid, lds, s);
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
        case T_Q4_K: return mv_dispatch_epi<0, NORM, T_Q4_K, X86>(a, epi, grid, lds, s);
        case T_Q5_K: return mv_dispatch_epi<0, NORM, T_Q5_K, X86>(a, epi, grid, lds, s);
        case T_Q6_K: return mv_dispatch_epi<0, NORM, T_Q6_K, X86>(a, epi, grid, lds, s);
        case T_Q8_0: return mv_dispatch_epi<1, NORM, T_Q8_0, X86>(a, epi, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}

// Row-task geometry (mv_device.h "Row tasks"): Lr lanes per row = U rounded up to a
// multiple of 4, at most 64 (QKV: 32, so that a task holds RoPE pairs); R = 64 / Lr
// rounded down to a power of two, halved until every segment starts on a task boundary.
bool mv_geometry(MVArgs& a, int epi) {
    if (a.nseg < 1 || a.cols < 256 || a.cols % 256) return false;
    const int U = a.cols >> 8, lmax = epi == EPI_QKV ? 32 : 64;
    static const int lr_cap = [] {  // A/B knob: cap on lanes per row (more rows per task)
        const char* e = getenv("LLMI_MV_LR");
        return e ? atoi(e) : 64;
    }();
    int lr = (std::min(std::min(U, lmax), lr_cap) + 3) & ~3;
    lr = std::min(std::max(lr, 4), lmax);
    int R = 1;
    while (2 * R * lr <= 64) R *= 2;
    auto aligned = [&](int r) {
        for (int i = 1; i < a.nseg; ++i)
            if ((a.seg[i].row0 - a.seg[0].row0) % r) return false;
        return true;
    };
    if (epi != EPI_SWIGLU)
        while (R > 1 && !aligned(R)) R >>= 1;
    if (epi == EPI_QKV && R < 2) return false;
    int rows;
    if (epi == EPI_SWIGLU) {
        if (a.nseg != 2 || a.seg[0].rows != a.seg[1].rows) return false;
        rows = a.seg[0].rows;
    } else {
        rows = a.seg[a.nseg - 1].row0 + a.seg[a.nseg - 1].rows - a.seg[0].row0;
    }
    a.lr = lr;
    a.rpt = R;
    a.ntasks = (rows + R - 1) / R;
    return a.ntasks > 0;
}

// LLMI_MV_FW (A/B): 1 = each wave issues its second sub-item's weights only after its
// first sub-item's have landed, so the launch's first chip-wide round of requests is one
// sub-item per wave instead of two (every result is unchanged)
static int mv_fw() {
    static const int v = [] {
        const char* e = getenv("LLMI_MV_FW");
        return e ? atoi(e) : 0;
    }();
    return v;
}

hipError_t launch_matvec(const MVArgs& a0, int epi, int max_blocks, hipStream_t s) {
    if (a0.nseg < 1 || a0.cols <= 0 || a0.cols % 256) return hipErrorInvalidValue;
    MVArgs a = a0;
    a.fw = mv_fw();
    if (!mv_geometry(a, epi)) return hipErrorInvalidValue;
    const int act = act_kind(a.seg[0].type);
    for (int i = 1; i < a.nseg; ++i)
        if (act_kind(a.seg[i].type) != act) return hipErrorInvalidValue;
    const size_t lds = mv_lds_bytes(act, a.cols);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    int blocks = (a.ntasks + kMVWaves - 1) / kMVWaves;
    if (blocks > max_blocks) blocks = max_blocks;
#if defined(LLMI_EXPERIMENTS)
    static const int exp_blocks = [] {  // experiment builds: fixed grid for launch sweeps
        const char* e = getenv("LLMI_MV_BLOCKS");
        return e ? atoi(e) : 0;
    }();
    if (exp_blocks > 0 && exp_blocks < blocks) blocks = exp_blocks;
#endif
    const dim3 grid(blocks);
    // the weights' byte order must be the numerics' (common.h: x86 planes for x86 numerics)
    for (int i = 0; i < a.nseg; ++i)
        if ((a.seg[i].x86 != 0) != (a.num != 0)) return hipErrorInvalidValue;
    if (a.num) return a.nw ? mv_dispatch_type<true, 1>(a, epi, grid, lds, s) : mv_dispatch_type<false, 1>(a, epi, grid, lds, s);
    return a.nw ? mv_dispatch_type<true, 0>(a, epi, grid, lds, s) : mv_dispatch_type<false, 0>(a, epi, grid, lds, s);
}

hipError_t launch_quant_dump(const MVArgs& a, int act, void* out, hipStream_t s) {
    if (a.cols <= 0 || a.cols % 256) return hipErrorInvalidValue;
    const size_t lds = mv_lds_bytes(act, a.cols);
    if (a.num) {
        if (act == 0) hipLaunchKernelGGL((k_quant_dump<0, 1>), dim3(1), dim3(kMVThreads), lds, s, a, (uint8_t*)out);
        else hipLaunchKernelGGL((k_quant_dump<1, 1>), dim3(1), dim3(kMVThreads), lds, s, a, (uint8_t*)out);
    } else {
        if (act == 0) hipLaunchKernelGGL((k_quant_dump<0, 0>), dim3(1), dim3(kMVThreads), lds, s, a, (uint8_t*)out);
        else hipLaunchKernelGGL((k_quant_dump<1, 0>), dim3(1), dim3(kMVThreads), lds, s, a, (uint8_t*)out);
    }
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
int g_pf_fa_noalloc = 0;               // prefill: never allocate k_pf_fa's score scratch (its failure path)
#ifndef LLMI_PF_QUANT_BPC
#define LLMI_PF_QUANT_BPC 2
#endif
// k_pf_quant: 256-element blocks per workgroup when rows are split (0: never); LLMI_PF_QUANT_BPC (A/B)
int g_pf_quant_bpc = getenv("LLMI_PF_QUANT_BPC") ? atoi(getenv("LLMI_PF_QUANT_BPC")) : LLMI_PF_QUANT_BPC;
int g_pf_quant_split_below = 64;  // ... i.e. below this many rows (batched decode)
#ifndef LLMI_PF_XCD_MAP
#define LLMI_PF_XCD_MAP 1
#endif
int g_pf_xcd_map = LLMI_PF_XCD_MAP;  // k_pf_gemm: XCD-aware tile order
int g_pf_qkv_merge = 1;            // prefill: consecutive same-type q/k/v parts in one GEMM launch
int g_pf_gemm_ng = 2;                   // k_pf_gemm 32-token groups per workgroup (1 or 2)
int g_pf_fa_cfg = 440;                  // k_pf_fa configuration (prefill.hip.inc pf_fa_launch)
int g_pf_attn_fa = 1;                   // batched-prefill attention: tiled FP64-MFMA kernel when it applies
int g_pf_max_kv = kPfAttnMaxKV;         // longest KV the batched-prefill attention takes
int g_xspin_limit = kXSpinLimit;        // k_attn_x bounded-wait polls before it faults
int g_xtag_skew = 0;                    // k_attn_x consumers expect tag + skew (1: never matches)
int pf_max_kv() { return g_pf_max_kv; }

// dim slices of k_attn_d: about 256 workgroups (one per CU), 2..8, at least 8 dims each
static int g_attn_s = 0;  // LLMI_ATTN_S (A/B only): force 2, 4 or 8 slices
// k_attn_d reads the position before its K/V loads and skips those past it (default;
// LLMI_ATTN_PF=0 loads the whole KV bucket, A/B only): ties at bucket ends, up to 1.4 us
// faster mid-bucket (profiles/r02/attn_dim_split.md)
static int g_attn_pf = 3;
int attn_d_slices(int n_head, int head_dim) {
    const int s = g_attn_s ? g_attn_s : n_head >= 128 ? 2 : n_head >= 64 ? 4 : 8;
    return head_dim / s >= 8 ? s : head_dim / 8;
}

static int g_attn_mode = 0;  // 0 auto, 1 fused, 2 split, 3 two-kernel, 4 exchange (experiments: LLMI_ATTN_MODE)
void set_attn_mode(int mode) {
    g_attn_mode = mode;
    const char* e = getenv("LLMI_ATTN_S");
    const int v = e ? atoi(e) : 0;
    g_attn_s = (v == 2 || v == 4 || v == 8) ? v : 0;
    const char* f = getenv("LLMI_ATTN_PF");
    g_attn_pf = f ? atoi(f) : 1;
    const char* r = getenv("LLMI_ATTN_ROT");  // rotated K pass order (bit 1 of the word; default on)
    if (!r || atoi(r)) g_attn_pf |= 2;
}
int attn_path(int n_head, int n_head_kv, int kv_bound, int head_dim, int mode) {
    const int g = n_head / n_head_kv;
    const int m = mode < 0 ? g_attn_mode : mode;
    const bool split_ok = (size_t)g * kv_bound * 4 <= kSplitAttnMaxLds;
    const bool fused_ok = kv_bound <= kFusedAttnMaxKV;
    (void)n_head;
    if (m == 4 && g <= 8 && kv_bound <= kXAttnMaxKV) return 4;
    if (m == 5 && kv_bound <= kRegAttnMaxKV) return 5;
    if (m == 6 && kv_bound <= kDimAttnMaxKV) return 6;
    if (m == 7 && g <= 8) return 7;
    if (m == 1 && fused_ok) return 1;
    if (m == 2 && split_ok) return 2;
    if (m == 3) return 3;
    // auto, from the crossovers measured by tools/attnbench.py (graph-free launches, us;
    // profiles/r01/attn_modes.md):
    //   G=4, D=128 (8B, Mistral): fused <= 256 (8.1 vs 8.4 exchange), exchange <= 512,
    //                             split beyond (640: 10.8 vs 12.9 exchange)
    //   G=8, D=128 (70B): fused <= 640 (128: 8.1 vs 16.3 exchange), split beyond
    //   G=8, D=64 (TinyLlama): fused <= 2048 (128: 6.2 vs 9.7; 1280: 15.9 vs 20.9)
    //   G=8, D=64: register-prefetched k_attn_r <= 256 (5.5-5.9 vs 6.2-6.7 fused); for
    //              D=128 it loses to fused (one CU pulls 64 KB+ per head: per-CU bandwidth)
    //   k_attn_d (dim-split, scores recomputed per slice, round 2) beats all of the above
    //   up to 1024 positions on every shape (tools/attnbench.py, profiles/r02/attn_dim_split.md):
    //   G=4 D=128 128: 5.2 vs 8.1 fused, 512: 7.0 vs 10.0 exchange, 1024: 10.8 vs 12.7 split
    //   long-context four-launch path 7 (profiles/r02/attn_long.md): G=4 D=128 beyond 2048
    //   (4096: 25.4 vs 31.2 split, 16384: 62 vs 628 two-kernel), G=8 beyond 1024
    if (m == 0) {
        if (g <= 8 && kv_bound <= kDimAttnMaxKV && attn_d_slices(n_head, head_dim) >= 2) return 6;
        if (g == 8 && kv_bound > 1024) return 7;
        if (g <= 4 && kv_bound > 2048) return 7;
        if (g == 8 && head_dim == 64 && kv_bound <= 256) return 5;
        if (g == 8 && fused_ok && kv_bound <= (head_dim == 64 ? 2048 : 640)) return 1;
        if (g == 4 && fused_ok && kv_bound <= 256) return 1;
        if (g == 4 && split_ok && kv_bound > 512) return 2;
        if (g <= 8 && kv_bound <= kXAttnMaxKV) return 4;
    }
    return split_ok ? 2 : fused_ok ? 1 : 3;
}

hipError_t launch_attention(const AttnArgs& a0, int n_head, int n_head_kv, int head_dim, int kv_bound, hipStream_t s,
                            int mode) {
    if (n_head_kv <= 0 || n_head % n_head_kv) return hipErrorInvalidValue;
    if (a0.fa) return launch_attention_fa(a0, n_head, n_head_kv, head_dim, kv_bound, s);
    if (a0.num) return launch_attention_x86(a0, n_head, n_head_kv, head_dim, kv_bound, s, mode < 0 ? g_attn_mode : mode);
    AttnArgs a = a0;
    a.spin_limit = g_xspin_limit;
    a.tag_skew = g_xtag_skew;
    const int g = n_head / n_head_kv;
    int path = attn_path(n_head, n_head_kv, kv_bound, head_dim, mode);
    if (path == 4 && (!a.gran || !a.fault || a.layer < 0 || a.layer > 254))
        path = attn_path(n_head, n_head_kv, kXAttnMaxKV + 256, head_dim, mode);
    if (path == 5) {
        const int p = kv_bound <= 64 ? 1 : kv_bound <= 128 ? 2 : kv_bound <= 256 ? 4 : 8;
#define LLMI_ATTR(D_, P_) \
        if (head_dim == D_ && p == P_) { launch_k(k_attn_r<D_, P_>, dim3(n_head), dim3(512), 0, s, true, true, a, g, kv_bound); return hipGetLastError(); }
        LLMI_ATTR(128, 1) LLMI_ATTR(128, 2) LLMI_ATTR(128, 4) LLMI_ATTR(128, 8)
        LLMI_ATTR(64, 1) LLMI_ATTR(64, 2) LLMI_ATTR(64, 4) LLMI_ATTR(64, 8)
#undef LLMI_ATTR
        return hipErrorInvalidValue;
    }
    if (path == 7) {
        const int ntile = (kv_bound + kLongTile - 1) / kLongTile;
        const int np = kv_bound > 4096 ? 4 : 1;  // 32-position passes per scores workgroup
        const dim3 gs(n_head_kv, (kv_bound + 32 * np - 1) / (32 * np));
#define LLMI_ATTL(D_, G_)                                                                                   \
        if (head_dim == D_ && g == G_) {                                                                    \
            if (np == 4) launch_k(k_attl_scores<D_, G_, 4>, gs, dim3(256), 0, s, true, false, a);          \
            else launch_k(k_attl_scores<D_, G_, 1>, gs, dim3(256), 0, s, true, false, a);                  \
            launch_k(k_attl_exp, dim3(n_head, ntile), dim3(256), 0, s, false, false, a, n_head, kv_bound); \
            launch_k(k_attl_pv<D_, G_>, dim3(n_head_kv, ntile), dim3(512), 0, s, false, false, a, n_head, kv_bound); \
            launch_k(k_attl_sum<D_>, dim3(n_head), dim3(D_), 0, s, false, true, a, n_head);                \
            return hipGetLastError();                                                                       \
        }
        LLMI_ATTL(128, 1) LLMI_ATTL(128, 2) LLMI_ATTL(128, 4) LLMI_ATTL(128, 8)
        LLMI_ATTL(64, 1) LLMI_ATTL(64, 2) LLMI_ATTL(64, 4) LLMI_ATTL(64, 8)
#undef LLMI_ATTL
        return hipErrorInvalidValue;
    }
    if (path == 6) {
        const int p = kv_bound <= 64 ? 1 : kv_bound <= 128 ? 2 : kv_bound <= 256 ? 4 : kv_bound <= 512 ? 8
                    : kv_bound <= 768 ? 12 : 16;
        const int sdim = attn_d_slices(n_head, head_dim);
#define LLMI_ATTD(D_, P_, S_) \
        if (head_dim == D_ && p == P_ && sdim == S_) { launch_k(k_attn_d<D_, P_, S_>, dim3(n_head * S_), dim3(512), 0, s, true, true, a, g, n_head_kv, kv_bound, g_attn_pf); return hipGetLastError(); }
#define LLMI_ATTD_P(D_, S_) LLMI_ATTD(D_, 1, S_) LLMI_ATTD(D_, 2, S_) LLMI_ATTD(D_, 4, S_) LLMI_ATTD(D_, 8, S_) LLMI_ATTD(D_, 12, S_) LLMI_ATTD(D_, 16, S_)
        LLMI_ATTD_P(128, 2) LLMI_ATTD_P(128, 4) LLMI_ATTD_P(128, 8) LLMI_ATTD_P(64, 2) LLMI_ATTD_P(64, 4) LLMI_ATTD_P(64, 8)
#undef LLMI_ATTD_P
#undef LLMI_ATTD
        return hipErrorInvalidValue;
    }
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
                         int64_t cols, int rgs, int x86, hipStream_t s) {
    if (nblk <= 0) return hipSuccess;
    if (cols % 256) return hipErrorInvalidValue;
    if (type == T_Q4_K || type == T_Q5_K || type == T_Q6_K) {
        const int64_t thr = nblk * 4;
        hipLaunchKernelGGL(k_repack_kq, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s, type, (const uint8_t*)raw, a,
                           h, sp, d, nblk, (int)(cols / 256), rgs, x86);
    } else if (type == T_Q8_0) {
        hipLaunchKernelGGL(k_repack_q80, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, s, (const uint8_t*)raw, a, d,
                           nblk, (int)(cols / 32), rgs);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}


}  // namespace llmi
