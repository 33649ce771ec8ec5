// batch.hip — batched decode (continuous batching): up to
// kMaxBatch sequences advance one token per step, every weight byte streamed once for all
// of them.
//
// k_mvn is the matvec (kernels.hip k_matvec) with NT activation vectors: the prologue
// quantizes the NT inputs into NT LDS images exactly as the single-token prologue does
// (per-16 sub-block q8_K / q8_0, RMSNorm with a double sum); the main loop loads each
// lane's weight unit once and forms NT sets of block terms against it, each folded onto
// its token's chains in ggml's generic order (mv_device.h) — so every sequence's results
// are bit-identical to its own single-token decode.
//
// Attention runs the split kernels' bodies (mv_device.h) with a third grid dimension
// over the batch slots, each slot reading its own sequence's KV cache.
#include "kernels.h"
#include "mv_device.h"
#include "pf_device.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace llmi {

namespace {

constexpr int kBT = 512, kBW = kBT / 64;  // threads / waves per workgroup
// waves of a k_mvn workgroup that run row tasks: all 8, except for x86 Q8_0 rows, whose
// fold buffers (up to 19.8 KB per wave, mv_device.h fold_stride) fit the LDS for 4 waves
// beside the tokens' images; the other 4 waves take part in the prologue only
__host__ __device__ constexpr int mvn_work_waves(int act, int x86) { return act && x86 ? 4 : kBW; }

__host__ __device__ inline size_t img_bytes(int act, int cols) { return a16(lds_red_off(act, cols)); }

// per-token LDS image t at smem + t * img; the shared reduction scratch after the NT images
__device__ __forceinline__ Lds carve_t(uint8_t* smem, int act, int cols, int t, size_t img) {
    Lds L = carve(smem + (size_t)t * img, act, cols);
    return L;
}

// NT activation vectors (x + t * x_stride) -> NT LDS images: [RMSNorm] + quantization,
// bit-exact per token with the single-token prologue (the double sum of squares is exact
// in any association in practice, as for the K-split kernel's 1024-thread prologue).
// Work item i = tid + kBT k is (token i / nsub, sub-block i % nsub): the 16 lanes of a
// DPP row hold the 16 sub-blocks of one 256-element block of one token, as quant_sub needs.
template <int ACT, bool NORM, int NT, int X86 = 0>
__device__ __forceinline__ void bprologue(const MVArgs& A, uint8_t* smem, size_t img, double* red) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cols = A.cols, nsub = cols >> 4, nitem = NT * nsub;
    float scale[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) scale[t] = 1.0f;
    if constexpr (NORM) {
        double part[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) part[t] = 0.0;
        for (int i = tid; i < nitem; i += kBT) {
            const int t = i / nsub, sb = i - t * nsub;
            const float* xs = A.x + (size_t)t * A.x_stride + sb * 16;
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 v = *(const float4*)(xs + 4 * k);
                s += (double)(v.x * v.x); s += (double)(v.y * v.y); s += (double)(v.z * v.z); s += (double)(v.w * v.w);
            }
#pragma unroll
            for (int u = 0; u < NT; ++u)
                if (u == t) part[u] += s;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const double w = wave_sum_d(part[t]);
            if (lane == 0) red[t * kBW + wave] = w;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            double r[kBW];
#pragma unroll
            for (int w = 0; w < kBW; ++w) r[w] = red[t * kBW + w];
#pragma unroll
            for (int o = 1; o < kBW; o <<= 1)
#pragma unroll
                for (int w = 0; w + o < kBW; w += 2 * o) r[w] = r[w] + r[w + o];
            const float mean = (float)(r[0] / (double)cols);
            scale[t] = 1.0f / sqrtf(mean + A.eps);
        }
    }
    for (int i = tid; i < nitem; i += kBT) {
        const int t = i / nsub, sb = i - t * nsub;
        const float* xs = A.x + (size_t)t * A.x_stride + sb * 16;
        float v[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 xv = *(const float4*)(xs + 4 * k);
            v[4 * k] = xv.x; v[4 * k + 1] = xv.y; v[4 * k + 2] = xv.z; v[4 * k + 3] = xv.w;
        }
        if constexpr (NORM) {
            float sc = 1.0f;
#pragma unroll
            for (int u = 0; u < NT; ++u)
                if (u == t) sc = scale[u];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 w = *(const float4*)(A.nw + sb * 16 + 4 * k);
                v[4 * k + 0] = (v[4 * k + 0] * sc) * w.x;
                v[4 * k + 1] = (v[4 * k + 1] * sc) * w.y;
                v[4 * k + 2] = (v[4 * k + 2] * sc) * w.z;
                v[4 * k + 3] = (v[4 * k + 3] * sc) * w.w;
            }
        }
        quant_sub<ACT, X86>(carve_t(smem, ACT, cols, t, img), cols, sb, v);
    }
    __syncthreads();
}

// the per-token view of the launch's descriptor for the epilogue
__device__ __forceinline__ MVArgs token_view(const MVArgs& A, int t, int seq) {
    MVArgs B = A;
    B.y = A.y + (size_t)t * A.y_stride;
    B.kc = A.kc ? A.kc + (size_t)seq * A.kv_stride : nullptr;
    B.vc = A.vc ? A.vc + (size_t)seq * A.kv_stride : nullptr;
    return B;
}

}  // namespace

// X86 = 1: the x86 association (model numerics LLMI_NUMERICS_X86; mv_device.h "x86
// numerics"): x86 q8 images, the lane's per-4-byte-lane integer sums stored as fp32 fma
// chain terms (unit_store_x86), x86 fold and epilogues -- every token equal to its own
// single-sequence x86 decode (Q8_0: 4 working waves, mvn_work_waves).
template <int ACT, bool NORM, int EPI, int T, int NT, int X86 = 0>
__global__ __launch_bounds__(kBT) void k_mvn(MVArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const size_t img = img_bytes(ACT, A.cols);
    double* red = (double*)(smem + NT * img);
    const int lane = threadIdx.x & 63;
    const int wave = uniform((int)(threadIdx.x >> 6));
    constexpr int NWK = mvn_work_waves(ACT, X86);
    const TaskGeo g = task_geo(A);
    float* F = (float*)(smem + a16(NT * img + (size_t)kMaxBatch * kBW * 8)) + wave * fold_stride(ACT, X86, g.R, g.lr);
    const int S = EPI == EPI_SWIGLU ? 2 * g.nj : g.nj;
    const int r = lane / g.lr, ul = lane - r * g.lr;
    const int G = gridDim.x * NWK;
    unsigned long long best[NT];  // per token: the lane's LOGITS key
#pragma unroll
    for (int t = 0; t < NT; ++t) best[t] = 0;
    bprologue<ACT, NORM, NT, X86>(A, smem, img, red);

    // the tokens' positions and sequences, read once: a global load inside the loop would
    // wait (in-order vmcnt) behind the weight prefetch every sub-item
    int tpos[NT], tseq[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        tpos[t] = A.tpos ? A.tpos[t] : 0;
        tseq[t] = A.tseq ? A.tseq[t] : 0;
    }
    int task = wave < NWK ? blockIdx.x * NWK + wave : A.ntasks;  // (the others: prologue only)
    if (task < A.ntasks) {
        int s = 0;
        Sub b = sub_of<EPI>(A, g, task, 0);
        Seg sg = pick(A, b.si);
        LaneUnit lu = lane_unit(g, b, sg, r, ul);
        UnitW<T> cur = load_unit<T>(sg, lu.row, lu.u, g.U);
        float acc[NT], vg[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = vg[t] = 0.f;
        for (;;) {
            int tn = task, sn = s + 1;
            if (sn == S) {
                sn = 0;
                tn = task + G;
            }
            const bool has_next = tn < A.ntasks;
            Sub bn = b;
            Seg sgn = sg;
            if (has_next) {
                bn = sub_of<EPI>(A, g, tn, sn);
                sgn = pick(A, bn.si);
            }
            const LaneUnit lun = lane_unit(g, bn, sgn, r, ul);
            // past the last sub-item: one shared line per part (k_matvec's mv_body)
            const UnitW<T> nxt = load_unit<T>(sgn, has_next ? lun.row : 0u, has_next ? lun.u : 0u, g.U);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                float tm[9];
                if constexpr (X86) unit_store_x86<T>(cur, smem + (size_t)t * img + (size_t)lu.u * kRec, F, r, ul, g.lr, g.R, lu.valid);
                else unit_terms<T>(cur, smem + (size_t)t * img + (size_t)lu.u * kRec, tm);
                const MVArgs B = token_view(A, t, tseq[t]);
                sub_finish<ACT, EPI, MVArgs, X86>(B, F, g, s, b, sg, tm, lu, r, ul, acc[t], vg[t], tpos[t], best[t]);
            }
            if (!has_next) break;
            cur = nxt;
            task = tn;
            s = sn;
            b = bn;
            sg = sgn;
            lu = lun;
        }
    }
    if constexpr (EPI == EPI_LOGITS) {
        // per token: workgroup max of the lanes' keys, one atomic into the slot of its
        // sequence's StepState; workgroup 0 advances the sequence's next position
        unsigned long long* wred = (unsigned long long*)red;  // [kBW][NT]
        __syncthreads();
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const unsigned long long k = wave_max_u64(best[t]);
            if (lane == 0) wred[wave * NT + t] = k;
        }
        __syncthreads();
        if ((int)threadIdx.x < NT) {
            const int t = threadIdx.x;
            unsigned long long b = wred[t];
            for (int w = 1; w < kBW; ++w) b = wred[w * NT + t] > b ? wred[w * NT + t] : b;
            StepState* st = A.st + (A.tseq ? A.tseq[t] : 0);
            const int pt = A.tpos[t];
            if (b) atomicMax(&st->key[pt & 1][blockIdx.x % kArgSlots], b);
            if (blockIdx.x == 0) st->pos_next = pt + 1;
        }
    }
}

// batched step entry: per slot (blockIdx.y) the token (host-provided for this position,
// else the argmax of the sequence's previous step), the sequence state, the embedding row
__global__ __launch_bounds__(256) void k_bembed(BEmbArgs a) {
    const int s = blockIdx.y;
    const int seq = a.tseq[s];
    StepState* st = a.st + seq;
    const int pos = st->pos_next;
    __shared__ int s_tok;
    if (threadIdx.x < 64) {
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
            st->seq = st->seq + 1u;
            if (pos >= 0 && pos < a.n_ctx) a.hist[(size_t)seq * a.n_ctx + pos] = tok;
            a.tpos[s] = pos;
        }
    }
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e < a.cols) a.x[(size_t)s * a.cols + e] = dequant_elem(a.w, tok, e, a.cols);
}

template <int D, int G>
__global__ __launch_bounds__(256) void k_battn_scores8(BAttnArgs b) {
    const AttnArgs a = b.a[blockIdx.z];
    attn_scores8_body<D, G>(a);
}
template <int D, int G>
__global__ __launch_bounds__(512) void k_battn_pv16(BAttnArgs b, int kvb) {
    const AttnArgs a = b.a[blockIdx.z];
    attn_pv16_body<D, G>(a, kvb);
}


// ---- the batched matvec on the matrix cores ---------------------------------------------
// k_bmm: workgroup = one ROW TILE of 16 rows (SWIGLU: 16 gate rows and the same 16 up
// rows) for all nt <= 8 tokens, kBmW waves; the S unit stages of K are dealt round-robin
// over the waves (wave w: stages w, w + kBmW, ...).  Per stage a wave forms the exact
// integer sums of the prefill GEMM (pf_device.h; one v_mfma_f32_16x16x32_f16 per residue
// l, A = the tokens' q8 fragments from k_pf_quant, B = q * scale) and from them the fp32
// terms of ggml's generic order, (d_w d_a) aux32[l] and -((dmin_w d_a) sumi), for its
// (row, token) pairs (C layout: lane = row lane & 15, tokens 4 (lane >> 4) + i; lanes 32..63
// hold the padding tokens 8..15 and are dropped).  After each round of kBmW stages the
// terms go through LDS to the fold threads, one per (matrix, chain, lane quad), which add
// them stage after stage onto their chains — every chain sees the blocks in order, so a
// token's results equal its single-sequence decode (k_matvec) and the oracle bit for bit.
// The padded token rows of the MFMA are zero fragments (bm_load zeroes them; discarded).
constexpr int kBmW = 8, kBmT = kBmW * 64;
// chains per (row, token): generic 8 residues + sumf (Q6_K: no mins); x86 (X86 = 1, model
// numerics LLMI_NUMERICS_X86) the 8 AVX2 lanes + Q4_K's 4 min lanes / Q5_K's summs.  A
// round buffer holds bm_ns() term slots per (stage, matrix): generic 9, x86 one per chain.
template <int T, int X86>
__host__ __device__ constexpr int bm_nc() { return X86 ? (T == T_Q4_K ? 12 : T == T_Q5_K ? 9 : 8) : (T == T_Q6_K ? 8 : 9); }
template <int T, int X86>
__host__ __device__ constexpr int bm_ns() { return X86 ? bm_nc<T, X86>() : 9; }

template <int T, int NW>
struct BmStage {
    PfW<T> w[NW];
    h8 a[8];
    float da[4];
    h8 bs;  // sumi A fragment (K-quants with mins): the bsum pairs of token lane & 15
};

template <int T, int NW>
__device__ __forceinline__ void bm_load(BmStage<T, NW>& st, const RowPtr (&rp)[NW], const uint8_t* aq,
                                        const uint8_t* abf, const float* ad, int s, int S, int nt, int exp = 0,
                                        bool weights = true) {
    const int lane = threadIdx.x & 63, n = lane & 15, grp = lane >> 4;
    if (weights)
#pragma unroll
        for (int wi = 0; wi < NW; ++wi) st.w[wi] = pf_w_load<T>(rp[wi], s, S);
    // only the lanes of real tokens load (the padding rows' loads would repeat token 0's
    // fragments through the TA); the others keep zeros
    int ntl = nt;
#if defined(LLMI_EXPERIMENTS)
    if (exp & 2) ntl = 0;  // experiment: no activation loads
#endif
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        st.a[l] = h8{};
        if (n < ntl) st.a[l] = *(const h8*)(aq + pf_aq_off(n, s, 4 * l + grp, S));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int t = 4 * grp + i;
        st.da[i] = 0.f;
        if (t < ntl) {
            st.da[i] = ad[(size_t)t * S + s];
        }
    }
    if constexpr (T != T_Q6_K) st.bs = n < ntl ? *(const h8*)(abf + pf_abf_off(n, s, grp, S)) : h8{};
}

// the stage's terms tm[wi][chain][i] (token 4 grp + i, row lane & 15).  X86: the chains'
// integer sums as floats (the x86 weight planes and activation fragments make residue l's
// MFMA sum exactly x86 lane l's, as in k_pf_gemm), Q4_K's min lanes from masked sumi MFMAs;
// the fold multiplies by d_w d_a / -d_a dmin_w itself (dw[wi], dmw[wi] returned)
template <int T, int NW, int X86 = 0>
__device__ __forceinline__ void bm_terms(const BmStage<T, NW>& st, float (&tm)[NW][12][4], float (&dwo)[NW],
                                         float (&dmwo)[NW]) {
    const int lane = threadIdx.x & 63, grp = lane >> 4;
#pragma unroll
    for (int wi = 0; wi < NW; ++wi) {
        const PfW<T>& w = st.w[wi];
        h2 slo{}, shi{}, slo_o{}, shi_o{};
        h2 s6[8], s6o[8];
        float dw, dmw = 0.f;
        h8 bm{};  // sumi B fragment: (min, 64 min) of sub-blocks 2 grp, 2 grp + 1
        if constexpr (T == T_Q4_K || T == T_Q5_K) {
            int sc0, m0, sc1, m1;
            scale_min(2 * grp, w.hdr.y, w.hdr.z, w.hdr.w, sc0, m0);
            scale_min(2 * grp + 1, w.hdr.y, w.hdr.z, w.hdr.w, sc1, m1);
            slo = h2{(_Float16)(float)sc0, (_Float16)(float)sc0};
            shi = h2{(_Float16)(float)sc1, (_Float16)(float)sc1};
            slo_o = slo * h2{(_Float16)1024.f, (_Float16)1024.f};
            shi_o = shi * h2{(_Float16)1024.f, (_Float16)1024.f};
            dw = h2f(w.hdr.x);
            dmw = h2f(w.hdr.x >> 16);
            bm[0] = (_Float16)(float)m0;
            bm[1] = (_Float16)(float)(64 * m0);
            bm[2] = (_Float16)(float)m1;
            bm[3] = (_Float16)(float)(64 * m1);
        } else {  // Q6_K: sc = 16 sh + sl per sub-block 4 grp + k
            dw = h2f(w.d);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int sc = (int)(int8_t)(w.sc >> (8 * k));
                const int sh = sc >> 4, sl = sc & 15;
                const _Float16 fl = (_Float16)(float)sl, fh = (_Float16)(float)sh;
                s6[2 * k] = h2{fl, fl};
                s6[2 * k + 1] = h2{fh, fh};
                s6o[2 * k] = s6[2 * k] * h2{(_Float16)1056.f, (_Float16)1056.f};
                s6o[2 * k + 1] = s6[2 * k + 1] * h2{(_Float16)1056.f, (_Float16)1056.f};
            }
        }
        dwo[wi] = dw;
        dmwo[wi] = dmw;
        float d[4], dm[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            d[i] = X86 ? 1.0f : dw * st.da[i];
            dm[i] = dmw * st.da[i];
        }
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            h8 bf[2];
            pf_build_b<T, X86>(w, l, slo, shi, slo_o, shi_o, s6, s6o, bf);
            f4 acc = mfma16(st.a[l], bf[0], f4{0.f, 0.f, 0.f, 0.f});
            if constexpr (T == T_Q6_K) {
                const f4 acc_h = mfma16(st.a[l], bf[1], f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = acc_h[i] * 16.f + acc[i];  // exact (< 2^24)
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) tm[wi][l][i] = X86 ? acc[i] : d[i] * acc[i];
        }
        if constexpr (X86 && T == T_Q4_K) {  // prod[k] = lane group k's slice of the mins . bsum pairs
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f4 sm = mfma16(st.bs, grp == k ? bm : h8{}, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
                for (int i = 0; i < 4; ++i) tm[wi][8 + k][i] = sm[i];
            }
        } else if constexpr (X86 && T == T_Q5_K) {
            const f4 sm = mfma16(st.bs, bm, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int i = 0; i < 4; ++i) tm[wi][8][i] = sm[i];
        } else if constexpr (!X86) {
            // sumi = mins . bsum pairs on the MFMA (every product and partial sum an integer
            // < 2^24: exact, prefill.hip.inc k_pf_quant); the term -(dmin * d_a) * sumi
            f4 sm{0.f, 0.f, 0.f, 0.f};
            if constexpr (T != T_Q6_K) sm = mfma16(st.bs, bm, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int i = 0; i < 4; ++i) tm[wi][8][i] = T != T_Q6_K ? -(dm[i] * sm[i]) : 0.f;
        }
    }
}

// the tile's segment, segment-local row 0 and its lanes' row views (tile = 16 rows of the
// launch's concatenated segments; SWIGLU: 16 gate rows, the same up rows)
template <int T, int EPI, int NW>
__device__ __forceinline__ void bm_tile(const MVArgs& A, int tile, int& si, int& row0, RowPtr (&rp)[NW]) {
    si = 0;
    if constexpr (EPI == EPI_SWIGLU) {
        row0 = tile * 16;
    } else {
        const int r0 = uniform(A.seg[0].row0), r1 = uniform(A.seg[1].row0), r2 = uniform(A.seg[2].row0);
        const int q = r0 + tile * 16;
        if (A.nseg > 1 && q >= r1) si = 1;
        if (A.nseg > 2 && q >= r2) si = 2;
        row0 = q - (si == 0 ? r0 : si == 1 ? r1 : r2);
    }
#pragma unroll
    for (int wi = 0; wi < NW; ++wi)
        rp[wi] = row_ptr<T>(pick(A, EPI == EPI_SWIGLU ? wi : si), row0 + (int)(threadIdx.x & 15), A.cols);
#if defined(LLMI_EXPERIMENTS)
    if (A.prio_alt & 1)  // experiment: every lane reads row 0 of the tile (coalesced, L2 hits)
#pragma unroll
        for (int wi = 0; wi < NW; ++wi) rp[wi] = row_ptr<T>(pick(A, EPI == EPI_SWIGLU ? wi : si), row0, A.cols);
#endif
}

// wave 0 of a k_bmm / k_bmd workgroup: the tile's row values from its chain results G and the
// epilogue per token
template <int T, int EPI, int NW, int NC, int X86 = 0>
__device__ __forceinline__ void bm_epilogue(const MVArgs& A, const float4* G, int nt, int tile, int si, int row0) {
    constexpr int NS = bm_ns<T, X86>();
    const int t = threadIdx.x >> 3, n0 = 2 * (threadIdx.x & 7);
    unsigned long long best = 0;
    int seq = 0, pos = 0;
    if (t < nt) {
        seq = A.tseq ? A.tseq[t] : 0;
        pos = A.tpos ? A.tpos[t] : 0;
        const float* Gf = (const float*)G;
        float v[NW][2];
#pragma unroll
        for (int wi = 0; wi < NW; ++wi)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int L = n0 + h + 16 * (t >> 2), i = t & 3;
                auto g = [&](int c) { return Gf[((wi * NS + c) * 32 + L) * 4 + i]; };
                float x;
                if constexpr (X86) {  // hsum_float_8 of the lanes [+ min lanes (Q4_K) / summs (Q5_K)]
                    const float t0 = g(0) + g(4), t1 = g(1) + g(5), t2 = g(2) + g(6), t3 = g(3) + g(7);
                    x = (t0 + t2) + (t1 + t3);
                    if constexpr (T == T_Q4_K) x = x + ((g(8) + g(10)) + (g(9) + g(11)));
                    if constexpr (T == T_Q5_K) x = x + g(8);
                } else {
                    x = NC == 9 ? g(8) : 0.f;  // sumf, then + sums[0..7]
#pragma unroll
                    for (int l = 0; l < 8; ++l) x += g(l);
                }
                v[wi][h] = x;
            }
        const MVArgs B = token_view(A, t, seq);
        PairRef ref;
        ref.sa = ref.sb = pick(A, si);
        ref.ra = row0 + n0;
        ref.rb = ref.ra + 1;
        ref.vb = 1;
        ref.type = T;
        if constexpr (EPI == EPI_SWIGLU) {
            epilogue<EPI, false, MVArgs, true, X86>(B, ref, row0 + n0, PairSum{v[0][0], v[NW - 1][0]}, pos, best);
            epilogue<EPI, false, MVArgs, true, X86>(B, ref, row0 + n0 + 1, PairSum{v[0][1], v[NW - 1][1]}, pos, best);
        } else {
            epilogue<EPI, false, MVArgs, true, X86>(B, ref, ref.ra, PairSum{v[0][0], v[0][1]}, pos, best);
        }
    }
    if constexpr (EPI == EPI_LOGITS) {
        // per token: the max over its 8 threads (consecutive lanes), one atomic
        // into the slot of its sequence's StepState; tile 0 advances the position
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            const unsigned long long bo = __shfl_xor(best, o);
            best = bo > best ? bo : best;
        }
        if ((threadIdx.x & 7) == 0 && t < nt) {
            StepState* st = A.st + seq;
            if (best) atomicMax(&st->key[pos & 1][tile % kArgSlots], best);
            if (tile == 0) st->pos_next = pos + 1;
        }
    }
}

// Persistent: workgroup b runs tiles b, b + grid, ...; one ITERATION = one round of kBmW
// stages of one tile, the next iteration's loads (next round, or the next tile's first
// round) issued before this one's terms, so the next tile's weights are in flight during
// this tile's last fold and epilogue.  LDS: two round buffers of terms (parity of the
// iteration) and the chain results G of the tile just finished.
template <int T, int EPI>
__global__ __launch_bounds__(kBmT) void k_bmm(MVArgs A, const uint8_t* aq, const uint8_t* abf, const float* ad, int nt,
                                              int ntiles) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NW = EPI == EPI_SWIGLU ? 2 : 1;   // weight matrices (SWIGLU: gate, up)
    constexpr int NC = T == T_Q6_K ? 8 : 9;         // chains per (row, token)
    constexpr int kBuf = kBmW * NW * 9 * 32;        // float4 per round buffer
    float4* TmB = (float4*)smem;
    float4* G = TmB + 2 * kBuf;
    const int wave = uniform((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int S = A.cols >> 8, R = (S + kBmW - 1) / kBmW;
    int tile = blockIdx.x;
    if (tile >= ntiles) return;
    int si, row0;
    RowPtr rp[NW];
    bm_tile<T, EPI, NW>(A, tile, si, row0, rp);

    // fold items (matrix wi, chain c, lane quad L): threads tid and tid + kBmT
    constexpr int NI = NW * NC * 32;
    float4 fs[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    BmStage<T, NW> cur;
    bm_load<T, NW>(cur, rp, aq, abf, ad, wave < S ? wave : S - 1, S, nt, A.prio_alt);
    int rho = 0, it = 0;
    for (;;) {
        // the next iteration: (tile, rho + 1) or (tile + grid, 0); its loads now
        int tn = tile, rn = rho + 1;
        if (rn == R) {
            rn = 0;
            tn = tile + gridDim.x;
        }
        const bool has_next = tn < ntiles;
        int sin, row0n;
        RowPtr rpn[NW];
        bm_tile<T, EPI, NW>(A, has_next ? tn : tile, sin, row0n, rpn);  // unconditional (no scratch copies)
        const int s = rho * kBmW + wave, sn = rn * kBmW + wave;
        BmStage<T, NW> nxt;
        bm_load<T, NW>(nxt, rpn, aq, abf, ad, sn < S ? sn : S - 1, S, nt, A.prio_alt);
        float4* Tm = TmB + (it & 1) * kBuf;
        if (s < S) {
            float tm[NW][12][4], dw_[NW], dmw_[NW];
#if defined(LLMI_EXPERIMENTS)
            if (A.prio_alt & 4) {  // experiment: no terms (zeros)
#pragma unroll
                for (int wi = 0; wi < NW; ++wi)
#pragma unroll
                    for (int c = 0; c < 9; ++c)
#pragma unroll
                        for (int i = 0; i < 4; ++i) tm[wi][c][i] = cur.da[i] + (float)cur.w[wi].q0[i & 3];
            } else
#endif
            bm_terms<T, NW>(cur, tm, dw_, dmw_);
            if (lane < 32) {
#pragma unroll
                for (int wi = 0; wi < NW; ++wi)
#pragma unroll
                    for (int c = 0; c < NC; ++c)
                        Tm[((wave * NW + wi) * 9 + c) * 32 + lane] =
                            make_float4(tm[wi][c][0], tm[wi][c][1], tm[wi][c][2], tm[wi][c][3]);
            }
        }
        __syncthreads();
        const int nv = S - rho * kBmW < kBmW ? S - rho * kBmW : kBmW;
        const bool last = rho == R - 1;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int f = threadIdx.x + k * kBmT;
            if (f < NI) {
                const int wi = f / (NC * 32), c = (f / 32) % NC, L = f & 31;
                float4 a = fs[k];
                for (int w = 0; w < nv; ++w) {
                    const float4 v = Tm[((w * NW + wi) * 9 + c) * 32 + L];
                    a.x += v.x;
                    a.y += v.y;
                    a.z += v.z;
                    a.w += v.w;
                }
                if (last) {  // the tile's chain results; the chains restart for the next tile
                    G[(wi * 9 + c) * 32 + L] = a;
                    a = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                fs[k] = a;
            }
        }
        if (last) {
            __syncthreads();
            if (threadIdx.x < 64) bm_epilogue<T, EPI, NW, NC>(A, G, nt, tile, si, row0);
        }
        if (!has_next) break;
        cur = nxt;
        tile = tn;
        rho = rn;
        si = sin;
        row0 = row0n;
#pragma unroll
        for (int wi = 0; wi < NW; ++wi) rp[wi] = rpn[wi];
        ++it;
    }
}

// ---- k_bmd: k_bmm with the weights staged through LDS by DMA -----------------------------
// k_bmm's lanes read 16 B of 16 different rows per load (the MFMA's B layout), so every
// load touches 64 lines; at 8 sequences that access pattern, not the MFMA or the VALU, is
// what bounds it (LLMI_BMM_EXP=1, every lane reading row 0: 1272 -> 2030 tok/s).  k_bmd
// moves a whole round -- the kBmW consecutive units of every (matrix, row, plane part) of
// the tile, 128 contiguous bytes each -- with global_load_lds (1 KiB per wave instruction,
// no VGPRs) into one LDS buffer, and each wave takes its stage's parts from there.  Per
// round: weights out of LDS, barrier, next round's DMA + activations, terms, barrier
// (retires the DMA), fold.  The 16-B pieces of a segment are stored XOR-swizzled by row
// (slot = stage ^ (row & 7)) so the 16 rows of a read spread over the banks.  Same terms,
// same fold: bit-identical to k_bmm.
typedef __attribute__((address_space(3))) void* bmd_lds_vp;
typedef __attribute__((address_space(1))) void* bmd_glb_vp;
template <int T>
__host__ __device__ constexpr int bmd_nseg() { return T == T_Q4_K ? 9 : T == T_Q5_K ? 11 : 13; }
// bytes of a round's weight buffer
template <int T, int NW>
__host__ __device__ constexpr size_t bmd_wbytes() { return (size_t)NW * 16 * bmd_nseg<T>() * kBmW * 16; }
// plane base of segment `seg` of a row (unit u at + 16 u): A parts 0..7, then Q4_K the
// header; Q5_K the header and the two fifth-bit parts; Q6_K the four high-bit parts and the scales
template <int T>
__device__ __forceinline__ const uint8_t* bmd_seg_base(const RowPtr& rp, int seg) {
    if (seg < 8) return rp.qa + (uint32_t)seg * rp.ps;
    if constexpr (T == T_Q4_K) return rp.sb;
    else if constexpr (T == T_Q5_K) return seg == 8 ? rp.sb : rp.hb + (uint32_t)(seg - 9) * rp.ps;
    else return seg < 12 ? rp.hb + (uint32_t)(seg - 8) * rp.ps : rp.sb;
}
template <int T, int EPI, int NW>
__device__ __forceinline__ void bmd_dma(const MVArgs& A, int si, int row0, int rho, uint8_t* wb) {
    constexpr int NSEG = bmd_nseg<T>(), NPC = NW * 16 * NSEG * kBmW;  // 16-B pieces per round
    static_assert(NPC % 64 == 0, "whole DMA instructions");
    const int lane = threadIdx.x & 63, wave = uniform((int)(threadIdx.x >> 6));
    const int U = A.cols >> 8;
    for (int i = wave; i < NPC / 64; i += kBmW) {
        const int f = i * 64 + lane, q = f / kBmW, slot = f % kBmW;
        const int seg = q % NSEG, rr = q / NSEG, row = rr % 16, mat = rr / 16;
        const int u = min(rho * kBmW + (slot ^ (row & 7)), U - 1);
        const RowPtr rp = row_ptr<T>(pick(A, EPI == EPI_SWIGLU ? mat : si), row0 + row, A.cols);
        __builtin_amdgcn_global_load_lds((bmd_glb_vp)(bmd_seg_base<T>(rp, seg) + (uint32_t)u * 16),
                                         (bmd_lds_vp)(wb + (size_t)i * 1024), 16, 0, 0);
    }
}
// this wave's stage (slot `stg` of the round) of every matrix out of the round buffer (Q6_K's
// fp16 d, 2 B per unit, still from global memory)
template <int T, int NW>
__device__ __forceinline__ void bmd_w(BmStage<T, NW>& st, const uint8_t* wb, int stg, const RowPtr (&rp)[NW], int s) {
    constexpr int NSEG = bmd_nseg<T>();
    const int lane = threadIdx.x & 63, row = lane & 15, g = lane >> 4;
    const int slot = stg ^ (row & 7);
#pragma unroll
    for (int wi = 0; wi < NW; ++wi) {
        auto piece = [&](int seg) { return wb + ((((size_t)(wi * 16 + row) * NSEG + seg) * kBmW + slot) * 16); };
        PfW<T>& w = st.w[wi];
        w.q0 = *(const u32x4*)piece(2 * g);
        w.q1 = *(const u32x4*)piece(2 * g + 1);
        if constexpr (T == T_Q4_K || T == T_Q5_K) {
            w.hdr = *(const u32x4*)piece(8);
            if constexpr (T == T_Q5_K) w.qh = *(const u32x2*)(piece(9 + (g >> 1)) + 8 * (g & 1));
        } else {
            w.hdr = *(const u32x4*)piece(8 + g);
            w.sc = *(const uint32_t*)(piece(12) + 4 * g);
            w.d = *(const uint16_t*)(rp[wi].db + (uint32_t)s * 2);
        }
    }
}

// LDS of a k_bmd workgroup: the round's term slots, the tile's chain results G, (X86) the
// round's weight scales and activation d, the round's weight buffer
template <int T, int NW, int X86>
__host__ __device__ constexpr size_t bmd_lds() {
    return ((size_t)kBmW * NW * bm_ns<T, X86>() + (size_t)NW * bm_ns<T, X86>()) * 32 * 16 +
           (X86 ? (size_t)kBmW * NW * 16 * 8 + (size_t)kBmW * 8 * 4 : 0) + bmd_wbytes<T, NW>();
}

// the persistent tile loop of one k_bmd workgroup: tiles tile0, tile0 + stride, ... < ntiles.
// X86: the fold runs the x86 fma chains, a = fma(d, term, a) with d = d_w d_a (lanes) or
// -d_a dmin_w (Q4_K's min lanes, Q5_K's summs), d formed from the round's scales (Dw: per
// stage, matrix and row) and activation d (Da: per stage and token) exactly as the
// single-token fold's unit terms form it
template <int T, int EPI, int X86 = 0>
__device__ __forceinline__ void bmd_body(const MVArgs& A, const uint8_t* aq, const uint8_t* abf, const float* ad, int nt,
                                         int ntiles, int tile0, int stride, uint8_t* smem) {
    constexpr int NW = EPI == EPI_SWIGLU ? 2 : 1;
    constexpr int NC = bm_nc<T, X86>(), NS = bm_ns<T, X86>();
    constexpr int kBuf = kBmW * NW * NS * 32;        // float4 of a round's terms
    float4* Tm = (float4*)smem;
    float4* G = Tm + kBuf;
    float2* Dw = (float2*)(G + NW * NS * 32);        // X86: [stage][matrix][row] (d_w, dmin_w)
    float* Da = (float*)(Dw + (X86 ? kBmW * NW * 16 : 0));  // X86: [stage][token] d_a
    uint8_t* Wb = (uint8_t*)(Da + (X86 ? kBmW * 8 : 0));
    const int wave = uniform((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int S = A.cols >> 8, R = (S + kBmW - 1) / kBmW;
    int tile = tile0;
    if (tile >= ntiles) return;
    int si, row0;
    RowPtr rp[NW];
    bm_tile<T, EPI, NW>(A, tile, si, row0, rp);
    constexpr int NI = NW * NC * 32;
    static_assert(NI <= 2 * kBmT, "two fold items per thread");
    float4 fs[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    BmStage<T, NW> cur;
    bm_load<T, NW>(cur, rp, aq, abf, ad, wave < S ? wave : S - 1, S, nt, 0, false);
    bmd_dma<T, EPI, NW>(A, si, row0, 0, Wb);
    // explicit: a workgroup barrier alone need not wait for this wave's LDS-DMA writes
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // round 0 in LDS
    int rho = 0;
    for (;;) {
        const int s = rho * kBmW + wave;
        bmd_w<T, NW>(cur, Wb, wave, rp, s < S ? s : S - 1);
        int tn = tile, rn = rho + 1;
        if (rn == R) {
            rn = 0;
            tn = tile + stride;
        }
        const bool has_next = tn < ntiles;
        int sin, row0n;
        RowPtr rpn[NW];
        bm_tile<T, EPI, NW>(A, has_next ? tn : tile, sin, row0n, rpn);
        __syncthreads();  // every wave has its stage out of the round buffer
        if (has_next) bmd_dma<T, EPI, NW>(A, sin, row0n, rn, Wb);
        const int sn = rn * kBmW + wave;
        BmStage<T, NW> nxt;
        bm_load<T, NW>(nxt, rpn, aq, abf, ad, sn < S ? sn : S - 1, S, nt, 0, false);
        if (s < S) {
            float tm[NW][12][4], dw[NW], dmw[NW];
            bm_terms<T, NW, X86>(cur, tm, dw, dmw);
            if (lane < 32) {
#pragma unroll
                for (int wi = 0; wi < NW; ++wi)
#pragma unroll
                    for (int c = 0; c < NC; ++c)
                        Tm[((wave * NW + wi) * NS + c) * 32 + lane] =
                            make_float4(tm[wi][c][0], tm[wi][c][1], tm[wi][c][2], tm[wi][c][3]);
            }
            if constexpr (X86) {
                if (lane < 16)
#pragma unroll
                    for (int wi = 0; wi < NW; ++wi) Dw[(wave * NW + wi) * 16 + lane] = make_float2(dw[wi], dmw[wi]);
                if ((lane & 15) == 0 && lane < 32)
                    *(float4*)(Da + wave * 8 + 4 * (lane >> 4)) = make_float4(cur.da[0], cur.da[1], cur.da[2], cur.da[3]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next round's DMA has landed ...
        __syncthreads();  // ... in every wave; the terms in LDS
        const int nv = S - rho * kBmW < kBmW ? S - rho * kBmW : kBmW;
        const bool last = rho == R - 1;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int f = threadIdx.x + k * kBmT;
            if (f < NI) {
                const int wi = f / (NC * 32), c = (f / 32) % NC, L = f & 31;
                float4 a = fs[k];
                for (int w = 0; w < nv; ++w) {
                    const float4 v = Tm[((w * NW + wi) * NS + c) * 32 + L];
                    if constexpr (X86) {
                        const float2 sc = Dw[(w * NW + wi) * 16 + (L & 15)];
                        const float4 da = *(const float4*)(Da + w * 8 + 4 * (L >> 4));
                        const bool lanes = c < 8;  // the 8 lane chains: d_w d_a; else -d_a dmin_w
                        const float m = lanes ? sc.x : sc.y;
                        const float4 dd = lanes ? make_float4(m * da.x, m * da.y, m * da.z, m * da.w)
                                                : make_float4(-da.x * m, -da.y * m, -da.z * m, -da.w * m);
                        a.x = __builtin_fmaf(dd.x, v.x, a.x);
                        a.y = __builtin_fmaf(dd.y, v.y, a.y);
                        a.z = __builtin_fmaf(dd.z, v.z, a.z);
                        a.w = __builtin_fmaf(dd.w, v.w, a.w);
                    } else {
                        a.x += v.x;
                        a.y += v.y;
                        a.z += v.z;
                        a.w += v.w;
                    }
                }
                if (last) {
                    G[(wi * NS + c) * 32 + L] = a;
                    a = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                fs[k] = a;
            }
        }
        if (last) {
            __syncthreads();
            if (threadIdx.x < 64) bm_epilogue<T, EPI, NW, NC, X86>(A, G, nt, tile, si, row0);
        }
        if (!has_next) break;
        cur = nxt;
        tile = tn;
        rho = rn;
        si = sin;
        row0 = row0n;
#pragma unroll
        for (int wi = 0; wi < NW; ++wi) rp[wi] = rpn[wi];
    }
}
template <int T, int EPI, int X86 = 0>
__global__ __launch_bounds__(kBmT) void k_bmd(MVArgs A, const uint8_t* aq, const uint8_t* abf, const float* ad, int nt,
                                              int ntiles) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    bmd_body<T, EPI, X86>(A, aq, abf, ad, nt, ntiles, blockIdx.x, gridDim.x, smem);
}
// A QKV whose attn_v rows have another type (Llama-3 Q4_K_M: Q6_K in half the layers): both
// type groups in ONE launch, workgroups [0, w1) on the A1 tiles (type T), the rest on A2's
// (type T2) -- one launch instead of two, no second resident grid competing for the CUs
template <int T, int T2, int X86 = 0>
__global__ __launch_bounds__(kBmT) void k_bmd2(MVArgs A1, MVArgs A2, const uint8_t* aq, const uint8_t* abf, const float* ad,
                                               int nt, int ntiles1, int ntiles2, int w1) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if ((int)blockIdx.x < w1) bmd_body<T, EPI_QKV, X86>(A1, aq, abf, ad, nt, ntiles1, blockIdx.x, w1, smem);
    else bmd_body<T2, EPI_QKV, X86>(A2, aq, abf, ad, nt, ntiles2, blockIdx.x - w1, gridDim.x - w1, smem);
}

// ---- launchers -----------------------------------------------------------------------------
size_t mvn_lds_bytes(int act, int cols, int nt, int x86) {
    const size_t fold = x86 ? (act ? (size_t)kX86QFloats : (size_t)kX86KFloats) : (size_t)kFoldFloats;
    (void)fold;
    return a16((size_t)nt * img_bytes(act, cols) + (size_t)kMaxBatch * kBW * 8) +
           (size_t)mvn_work_waves(act, x86) * fold_stride_cols(act, x86, cols) * 4;
}

template <typename K>
static int mvn_grid(K kernel, int ntasks, size_t lds, int max_blocks, int nwk) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, size_t, int>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple((const void*)kernel, lds, dev);
    int cap = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) {
            cap = it->second;
        } else {
            if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            int occ = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, kBT, lds) != hipSuccess || occ <= 0) occ = 1;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 1;
            cap = std::min(occ, 2) * cus;  // as the single-token matvec: at most 2 workgroups per CU
            cache.emplace(key, cap);
        }
    }
    int blocks = (ntasks + nwk - 1) / nwk;
    blocks = std::min(blocks, std::min(cap, max_blocks));
    return std::max(blocks, 1);
}

template <int ACT, bool NORM, int EPI, int T, int NT, int X86>
static hipError_t mvn_launch(const MVArgs& a, int max_blocks, hipStream_t s) {
    auto k = k_mvn<ACT, NORM, EPI, T, NT, X86>;
    const size_t lds = mvn_lds_bytes(ACT, a.cols, NT, X86);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const int blocks = mvn_grid(k, a.ntasks, lds, max_blocks, mvn_work_waves(ACT, X86));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(kBT), lds, s, a);
    return hipGetLastError();
}

template <int ACT, bool NORM, int EPI, int T, int X86>
static hipError_t mvn_nt(const MVArgs& a, int nt, int mb, hipStream_t s) {
    switch (nt) {
        case 1: return mvn_launch<ACT, NORM, EPI, T, 1, X86>(a, mb, s);
        case 2: return mvn_launch<ACT, NORM, EPI, T, 2, X86>(a, mb, s);
        case 3: case 4: return mvn_launch<ACT, NORM, EPI, T, 4, X86>(a, mb, s);
        default: return mvn_launch<ACT, NORM, EPI, T, 8, X86>(a, mb, s);
    }
}

template <int ACT, int T, int X86>
static hipError_t mvn_epi(const MVArgs& a, int epi, int nt, int mb, hipStream_t s) {
    const bool norm = a.nw != nullptr;
    switch (epi) {
        case EPI_ADD: return norm ? hipErrorInvalidValue : mvn_nt<ACT, false, EPI_ADD, T, X86>(a, nt, mb, s);
        case EPI_STORE:
            return norm ? mvn_nt<ACT, true, EPI_STORE, T, X86>(a, nt, mb, s) : mvn_nt<ACT, false, EPI_STORE, T, X86>(a, nt, mb, s);
        case EPI_QKV: return mvn_nt<ACT, true, EPI_QKV, T, X86>(a, nt, mb, s);
        case EPI_SWIGLU: return mvn_nt<ACT, true, EPI_SWIGLU, T, X86>(a, nt, mb, s);
        case EPI_LOGITS: return mvn_nt<ACT, true, EPI_LOGITS, T, X86>(a, nt, mb, s);
        default: return hipErrorInvalidValue;
    }
}

static hipError_t mvn_type(const MVArgs& a, int epi, int nt, int max_blocks, hipStream_t s) {
    if (a.num) {  // x86 association
        switch (a.seg[0].type) {
            case T_Q4_K: return mvn_epi<0, T_Q4_K, 1>(a, epi, nt, max_blocks, s);
            case T_Q5_K: return mvn_epi<0, T_Q5_K, 1>(a, epi, nt, max_blocks, s);
            case T_Q6_K: return mvn_epi<0, T_Q6_K, 1>(a, epi, nt, max_blocks, s);
            case T_Q8_0: return mvn_epi<1, T_Q8_0, 1>(a, epi, nt, max_blocks, s);
            default: return hipErrorNotSupported;
        }
    }
    switch (a.seg[0].type) {
        case T_Q4_K: return mvn_epi<0, T_Q4_K, 0>(a, epi, nt, max_blocks, s);
        case T_Q5_K: return mvn_epi<0, T_Q5_K, 0>(a, epi, nt, max_blocks, s);
        case T_Q6_K: return mvn_epi<0, T_Q6_K, 0>(a, epi, nt, max_blocks, s);
        case T_Q8_0: return mvn_epi<1, T_Q8_0, 0>(a, epi, nt, max_blocks, s);
        default: return hipErrorInvalidValue;
    }
}

static int mvn_pad(int nt) { return nt <= 1 ? 1 : nt == 2 ? 2 : nt <= 4 ? 4 : 8; }

hipError_t launch_mvn(const MVArgs& a0, int epi, int nt, int max_blocks, hipStream_t s) {
    if (a0.nseg < 1 || a0.cols <= 0 || a0.cols % 256 || nt < 1 || nt > kMaxBatch) return hipErrorInvalidValue;
    MVArgs a = a0;
    if (!mv_geometry(a, epi)) return hipErrorInvalidValue;
    const int t = a.seg[0].type;
    for (int i = 1; i < a.nseg; ++i)
        if (a.seg[i].type != t) return hipErrorInvalidValue;  // callers group segments by type
    // the padded token count (3 -> 4, 5..7 -> 8) reads rows of the batch buffers past nt:
    // the caller keeps kMaxBatch rows allocated and finite.  Rows too long for NT LDS
    // images (70B ffn_down: 28672 columns, 32 KB per token) run as several launches of
    // fewer tokens each (each streams the weights again; results per token unchanged).
    const int act = t == T_Q8_0 ? 1 : 0, x86 = a.num ? 1 : 0;
    for (int i = 0; i < a.nseg; ++i)
        if ((a.seg[i].x86 != 0) != (x86 != 0)) return hipErrorInvalidValue;  // the planes' byte order
    int group = mvn_pad(nt);
    while (group > 1 && mvn_lds_bytes(act, a.cols, group, x86) > 160 * 1024) group >>= 1;
    if (mvn_lds_bytes(act, a.cols, group, x86) > 160 * 1024) return hipErrorInvalidValue;
    for (int t0 = 0; t0 < nt; t0 += group) {
        MVArgs b = a;
        const int n = nt - t0 < group ? nt - t0 : group;
        b.x += (size_t)t0 * a.x_stride;
        b.y += (size_t)t0 * a.y_stride;
        if (a.tpos) b.tpos += t0;
        if (a.tseq) b.tseq += t0;
        const hipError_t e = mvn_type(b, epi, n, max_blocks, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---- k_bmm launchers -------------------------------------------------------------------
static int g_bmm_env = getenv("LLMI_BMM") ? atoi(getenv("LLMI_BMM")) : 1;  // 0: k_mvn everywhere (A/B)

// fewest tokens for which the step takes the matrix-core kernel (its cost is nearly flat in
// nt; k_mvn's grows with nt and pads 3 to 4 and 5..7 tokens to 8).  8B bench, tok/s at
// 2 / 3 / 4 / 6 / 8 sequences: k_bmd from 2: 501 / 732 / 959 / 1410 / 1875; k_mvn below 5:
// 680 / 651 / 851 (profiles/r05/batch/).  LLMI_BMM_MIN overrides (A/B)
int bmm_min_tokens() {
    const char* e = getenv("LLMI_BMM_MIN");  // read per call (step capture): tests switch it
    return e ? atoi(e) : 3;
}

// LLMI_BMM_DMA (A/B): 1 k_bmd (weights through LDS by DMA, default), 0 k_bmm; read per
// launch (step capture), so tests can run both
static int bmm_dma() {
    const char* e = getenv("LLMI_BMM_DMA");
    return e ? atoi(e) : 1;
}

bool bmm_ok(const MVArgs& a, int epi) {
    if (!g_bmm_env || a.nseg < 1 || a.cols <= 0 || a.cols % 256) return false;
    if (a.num && !bmm_dma()) return false;  // the x86 fold is k_bmd's only
    for (int i = 0; i < a.nseg; ++i)
        if ((a.seg[i].x86 != 0) != (a.num != 0)) return false;  // the planes' byte order
    const int t = a.seg[0].type;
    if (!(t == T_Q4_K || t == T_Q5_K || t == T_Q6_K)) return false;
    if (epi == EPI_SWIGLU && (a.nseg != 2 || a.seg[0].rows != a.seg[1].rows)) return false;
    for (int i = 0; i < a.nseg; ++i) {
        if (a.seg[i].type != t || a.seg[i].rows % 16) return false;
        if (epi != EPI_SWIGLU && i > 0 && a.seg[i].row0 != a.seg[i - 1].row0 + a.seg[i - 1].rows) return false;
    }
    return epi == EPI_STORE || epi == EPI_ADD || epi == EPI_QKV || epi == EPI_SWIGLU || epi == EPI_LOGITS;
}

// Resident k_bmm workgroups on the CURRENT device, per (kernel, LDS bytes, device), with
// the dynamic-LDS attribute set once per device: in-process replicas run one scheduler
// thread per GPU, so the cache is keyed by device and guarded (as mvn_grid's).
static int bmm_cap(const void* k, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, size_t, int>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(k, lds, dev);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    if (lds > 64 * 1024) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int occ = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kBmT, lds) != hipSuccess || occ <= 0) occ = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 1;
    const int cap = occ * cus;
    cache.emplace(key, cap);
    return cap;
}


template <int T, int EPI, int X86>
static hipError_t bmm_launch(const MVArgs& a, const void* aq, const void* abf, const float* ad, int nt, hipStream_t s) {
    constexpr int NW = EPI == EPI_SWIGLU ? 2 : 1;
    const bool dma = X86 || bmm_dma() != 0;
    auto k = dma ? k_bmd<T, EPI, X86> : k_bmm<T, EPI>;
    const size_t lds = dma ? bmd_lds<T, NW, X86>() : (size_t)(2 * kBmW + 1) * NW * 9 * 32 * 16;
    // shape / occupancy rejections are hipErrorNotSupported: the caller then runs the two
    // type groups as separate launches (engine.cpp) instead of failing the step
    if (lds > 160 * 1024) return hipErrorNotSupported;
    const int cap = bmm_cap((const void*)k, lds);
    int rows = 0;
    if (EPI == EPI_SWIGLU) rows = a.seg[0].rows;
    else
        for (int i = 0; i < a.nseg; ++i) rows += a.seg[i].rows;
    const int ntiles = rows / 16;
    const int grid = ntiles < cap ? ntiles : cap;
#if defined(LLMI_EXPERIMENTS)
    MVArgs ax = a;
    ax.prio_alt = getenv("LLMI_BMM_EXP") ? atoi(getenv("LLMI_BMM_EXP")) : 0;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBmT), lds, s, ax, (const uint8_t*)aq, (const uint8_t*)abf, ad, nt, ntiles);
#else
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBmT), lds, s, a, (const uint8_t*)aq, (const uint8_t*)abf, ad, nt, ntiles);
#endif
    return hipGetLastError();
}

template <int T, int T2, int X86>
static hipError_t bmm2_launch(const MVArgs& a1, const MVArgs& a2, const void* aq, const void* abf, const float* ad, int nt,
                              hipStream_t s) {
    auto k = k_bmd2<T, T2, X86>;
    const size_t lds = std::max(bmd_lds<T, 1, X86>(), bmd_lds<T2, 1, X86>());
    // shape / occupancy rejections are hipErrorNotSupported: the caller then runs the two
    // type groups as separate launches (engine.cpp) instead of failing the step
    if (lds > 160 * 1024) return hipErrorNotSupported;
    const int cap = bmm_cap((const void*)k, lds);
    int r1 = 0, r2 = 0;
    for (int i = 0; i < a1.nseg; ++i) r1 += a1.seg[i].rows;
    for (int i = 0; i < a2.nseg; ++i) r2 += a2.seg[i].rows;
    const int nt1 = r1 / 16, nt2 = r2 / 16;
    if (nt1 < 1 || nt2 < 1 || cap < 2) return hipErrorNotSupported;
    // workgroups dealt by weight bytes, each group no more than its tiles
    const double b1 = (double)nt1 * block_bytes(T), b2 = (double)nt2 * block_bytes(T2);
    int w1 = (int)(cap * b1 / (b1 + b2) + 0.5);
    w1 = std::max(1, std::min(std::min(w1, cap - 1), nt1));
    const int w2 = std::max(1, std::min(cap - w1, nt2));
    hipLaunchKernelGGL(k, dim3(w1 + w2), dim3(kBmT), lds, s, a1, a2, (const uint8_t*)aq, (const uint8_t*)abf, ad, nt, nt1, nt2, w1);
    return hipGetLastError();
}
// LLMI_BMM2 (A/B): 1 mixed-type QKV in one k_bmd2 launch (default), 0 two launches
static int bmm2_on() {
    const char* e = getenv("LLMI_BMM2");
    return e ? atoi(e) : 1;
}
hipError_t launch_bmm_qkv2(const MVArgs& a1, const MVArgs& a2, int nt, const void* aq, const void* abf, const float* ad,
                           hipStream_t s) {
    if (nt < 1 || nt > kMaxBatch || !bmm2_on() || !bmm_dma() || !bmm_ok(a1, EPI_QKV) || !bmm_ok(a2, EPI_QKV) ||
        a1.cols != a2.cols)
        return hipErrorNotSupported;
    const int t1 = a1.seg[0].type, t2 = a2.seg[0].type;
    if (a1.num != a2.num) return hipErrorNotSupported;
    if (a1.num) {
        if (t1 == T_Q4_K && t2 == T_Q6_K) return bmm2_launch<T_Q4_K, T_Q6_K, 1>(a1, a2, aq, abf, ad, nt, s);
        if (t1 == T_Q4_K && t2 == T_Q5_K) return bmm2_launch<T_Q4_K, T_Q5_K, 1>(a1, a2, aq, abf, ad, nt, s);
        if (t1 == T_Q5_K && t2 == T_Q6_K) return bmm2_launch<T_Q5_K, T_Q6_K, 1>(a1, a2, aq, abf, ad, nt, s);
        return hipErrorNotSupported;
    }
    if (t1 == T_Q4_K && t2 == T_Q6_K) return bmm2_launch<T_Q4_K, T_Q6_K, 0>(a1, a2, aq, abf, ad, nt, s);
    if (t1 == T_Q4_K && t2 == T_Q5_K) return bmm2_launch<T_Q4_K, T_Q5_K, 0>(a1, a2, aq, abf, ad, nt, s);
    if (t1 == T_Q5_K && t2 == T_Q6_K) return bmm2_launch<T_Q5_K, T_Q6_K, 0>(a1, a2, aq, abf, ad, nt, s);
    return hipErrorNotSupported;
}

template <int T, int X86>
static hipError_t bmm_epi(const MVArgs& a, int epi, const void* aq, const void* abf, const float* ad, int nt, hipStream_t s) {
    switch (epi) {
        case EPI_STORE: return bmm_launch<T, EPI_STORE, X86>(a, aq, abf, ad, nt, s);
        case EPI_ADD: return bmm_launch<T, EPI_ADD, X86>(a, aq, abf, ad, nt, s);
        case EPI_QKV: return bmm_launch<T, EPI_QKV, X86>(a, aq, abf, ad, nt, s);
        case EPI_SWIGLU: return bmm_launch<T, EPI_SWIGLU, X86>(a, aq, abf, ad, nt, s);
        case EPI_LOGITS: return bmm_launch<T, EPI_LOGITS, X86>(a, aq, abf, ad, nt, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_bmm(const MVArgs& a, int epi, int nt, const void* aq, const void* abf, const float* ad, hipStream_t s) {
    if (nt < 1 || nt > kMaxBatch || !bmm_ok(a, epi)) return hipErrorInvalidValue;
    if (a.num) {
        switch (a.seg[0].type) {
            case T_Q4_K: return bmm_epi<T_Q4_K, 1>(a, epi, aq, abf, ad, nt, s);
            case T_Q5_K: return bmm_epi<T_Q5_K, 1>(a, epi, aq, abf, ad, nt, s);
            case T_Q6_K: return bmm_epi<T_Q6_K, 1>(a, epi, aq, abf, ad, nt, s);
            default: return hipErrorInvalidValue;
        }
    }
    switch (a.seg[0].type) {
        case T_Q4_K: return bmm_epi<T_Q4_K, 0>(a, epi, aq, abf, ad, nt, s);
        case T_Q5_K: return bmm_epi<T_Q5_K, 0>(a, epi, aq, abf, ad, nt, s);
        case T_Q6_K: return bmm_epi<T_Q6_K, 0>(a, epi, aq, abf, ad, nt, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_bembed(const BEmbArgs& a, hipStream_t s) {
    if (a.nt < 1 || a.nt > kMaxBatch) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_bembed, dim3((a.cols + 255) / 256, a.nt), dim3(256), 0, s, a);
    return hipGetLastError();
}

// the single-sequence dim-split and long-context attention bodies (mv_device.h) with the
// batch slot as the last grid dimension
template <int D, int P, int S>
__global__ __launch_bounds__(512) void k_battn_d(BAttnArgs b, int G, int HK, int kvb) {
    attn_d_body<D, P, S>(b.a[blockIdx.y], G, HK, kvb, 1, 1);
}
template <int D, int G, int NP>
__global__ __launch_bounds__(256) void k_battl_scores(BAttnArgs b) { attl_scores_body<D, G, NP>(b.a[blockIdx.z]); }
__global__ __launch_bounds__(256) void k_battl_exp(BAttnArgs b, int n_head, int kvb) { attl_exp_body(b.a[blockIdx.z], n_head, kvb); }
template <int D, int G>
__global__ __launch_bounds__(512) void k_battl_pv(BAttnArgs b, int n_head, int kvb) { attl_pv_body<D, G>(b.a[blockIdx.z], n_head, kvb); }
template <int D>
__global__ __launch_bounds__(D) void k_battl_sum(BAttnArgs b, int n_head) { attl_sum_body<D>(b.a[blockIdx.z], n_head); }

// batched attention path: dim split up to 1024 positions for up to 3 slots (8B bench:
// 2 slots 940 vs 897 tok/s split, 4: 1335 vs 1341, 8: 1746 vs 1823 with 8 dim slices —
// at 8 slots its redundant K reads cost more than the split path's second launch), and
// for any slot count up to 512 positions with 1-2 slices (battn_slices), split while its
// LDS fits up to 2048 (G <= 4) / 1024 positions, long-context beyond; LLMI_BATTN_MODE
// (A/B only) forces 2 split, 6 dim split or 7 long-context
// dim slices of the batched dim-split attention: the single-sequence choice (about 256
// workgroups) is H * S * slots workgroups here, each re-reading its head's K rows; up to
// 512 positions 2 slices for <= 4 slots and 1 beyond (8B, ~200 positions, 2/4/8 slots:
// 721/960/1878 tok/s split or 8 slices -> 731/992/1945 with 2, 727/987/1963 with 1,
// profiles/r05/batch/battn_slices.txt); LLMI_BATTN_S (A/B) forces 1, 2, 4 or 8
static int battn_slices(int n_head, int head_dim, int kv_bound, int nt) {
    if (const char* es = getenv("LLMI_BATTN_S")) {
        const int v = atoi(es);
        if ((v == 1 || v == 2 || v == 4 || v == 8) && head_dim / v >= 8) return v;
    }
    if (kv_bound <= 512 && nt >= 2) return nt > 4 ? 1 : 2;
    return attn_d_slices(n_head, head_dim);
}
static int battn_path(int g, int n_head, int head_dim, int kv_bound, int nt) {
    const char* e = getenv("LLMI_BATTN_MODE");
    const int forced = e ? atoi(e) : 0;
    const bool split_ok = (size_t)g * kv_bound * 4 <= kSplitAttnMaxLds;
    const bool dim_ok = g <= 8 && kv_bound <= kDimAttnMaxKV && attn_d_slices(n_head, head_dim) >= 2;
    if (forced == 2 && split_ok) return 2;
    if (forced == 6 && dim_ok) return 6;
    if (forced == 7 && g <= 8) return 7;
    if (dim_ok && (nt <= 3 || kv_bound <= 512)) return 6;
    if (split_ok && (g <= 4 ? kv_bound <= 2048 : kv_bound <= 1024)) return 2;
    if (dim_ok) return 6;
    return g <= 8 ? 7 : (split_ok ? 2 : 0);
}

hipError_t launch_battention(const BAttnArgs& b, int nt, int n_head, int n_head_kv, int head_dim, int kv_bound,
                             hipStream_t s) {
    if (nt < 1 || nt > kMaxBatch || n_head_kv <= 0 || n_head % n_head_kv) return hipErrorInvalidValue;
    // the model's numerics (every slot's): flash attention, x86 association, else generic
    if (b.a[0].fa) return launch_battention_fa(b, nt, n_head, n_head_kv, head_dim, kv_bound, s);
    if (b.a[0].num) return launch_battention_x86(b, nt, n_head, n_head_kv, head_dim, kv_bound, s);
    const int g = n_head / n_head_kv;
    const int path = battn_path(g, n_head, head_dim, kv_bound, nt);
    if (path == 6) {
        const int p = kv_bound <= 64 ? 1 : kv_bound <= 128 ? 2 : kv_bound <= 256 ? 4 : kv_bound <= 512 ? 8
                    : kv_bound <= 768 ? 12 : 16;
        const int sd = battn_slices(n_head, head_dim, kv_bound, nt);
#define LLMI_BATTD(D_, P_, S_) \
        if (head_dim == D_ && p == P_ && sd == S_) { hipLaunchKernelGGL((k_battn_d<D_, P_, S_>), dim3(n_head * S_, nt), dim3(512), 0, s, b, g, n_head_kv, kv_bound); return hipGetLastError(); }
#define LLMI_BATTD_P(D_, S_) LLMI_BATTD(D_, 1, S_) LLMI_BATTD(D_, 2, S_) LLMI_BATTD(D_, 4, S_) LLMI_BATTD(D_, 8, S_) LLMI_BATTD(D_, 12, S_) LLMI_BATTD(D_, 16, S_)
        LLMI_BATTD_P(128, 1) LLMI_BATTD_P(128, 2) LLMI_BATTD_P(128, 4) LLMI_BATTD_P(128, 8)
        LLMI_BATTD_P(64, 1) LLMI_BATTD_P(64, 2) LLMI_BATTD_P(64, 4) LLMI_BATTD_P(64, 8)
#undef LLMI_BATTD_P
#undef LLMI_BATTD
        return hipErrorInvalidValue;
    }
    if (path == 7) {
        const int ntile = (kv_bound + kLongTile - 1) / kLongTile;
        const int np = kv_bound > 4096 ? 4 : 1;
        const dim3 gs(n_head_kv, (kv_bound + 32 * np - 1) / (32 * np), nt);
#define LLMI_BATTL(D_, G_)                                                                                        \
        if (head_dim == D_ && g == G_) {                                                                          \
            if (np == 4) hipLaunchKernelGGL((k_battl_scores<D_, G_, 4>), gs, dim3(256), 0, s, b);                 \
            else hipLaunchKernelGGL((k_battl_scores<D_, G_, 1>), gs, dim3(256), 0, s, b);                         \
            hipLaunchKernelGGL(k_battl_exp, dim3(n_head, ntile, nt), dim3(256), 0, s, b, n_head, kv_bound);       \
            hipLaunchKernelGGL((k_battl_pv<D_, G_>), dim3(n_head_kv, ntile, nt), dim3(512), 0, s, b, n_head, kv_bound); \
            hipLaunchKernelGGL((k_battl_sum<D_>), dim3(n_head, 1, nt), dim3(D_), 0, s, b, n_head);               \
            return hipGetLastError();                                                                             \
        }
        LLMI_BATTL(128, 1) LLMI_BATTL(128, 2) LLMI_BATTL(128, 4) LLMI_BATTL(128, 8)
        LLMI_BATTL(64, 1) LLMI_BATTL(64, 2) LLMI_BATTL(64, 4) LLMI_BATTL(64, 8)
#undef LLMI_BATTL
        return hipErrorInvalidValue;
    }
    if (path != 2) return hipErrorInvalidValue;
    const size_t lds = (size_t)g * kv_bound * 4;
#define LLMI_BATT(D_, G_)                                                                                    \
    if (head_dim == D_ && g == G_) {                                                                         \
        hipLaunchKernelGGL((k_battn_scores8<D_, G_>), dim3(n_head_kv, (kv_bound + 31) / 32, nt), dim3(256), 0, s, b); \
        hipLaunchKernelGGL((k_battn_pv16<D_, G_>), dim3(n_head_kv, D_ / 16, nt), dim3(512), lds, s, b, kv_bound); \
        return hipGetLastError();                                                                            \
    }
    LLMI_BATT(128, 1) LLMI_BATT(128, 2) LLMI_BATT(128, 4) LLMI_BATT(128, 8)
    LLMI_BATT(64, 1) LLMI_BATT(64, 2) LLMI_BATT(64, 4) LLMI_BATT(64, 8)
#undef LLMI_BATT
    return hipErrorInvalidValue;
}

}  // namespace llmi
