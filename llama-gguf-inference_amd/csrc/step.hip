// step.hip — the persistent decode step: ONE launch per token.
//
// The per-op launches of kernels.hip cost a dependent-launch boundary (~1.2-1.5 us), a
// dispatch ramp (~0.5 us), and an exposed first-weight latency per op: ~190 launches x
// ~3-4 us of a 1.6 ms 8B step.  Here one workgroup per CU (1024 threads,
// 16 waves) runs every op of the token as a PHASE of one launch:
//
//   per layer:  QKV (+RoPE, f16 KV write) | attention scores | softmax + PV |
//               attn_output (+residual)   | gate/up (+SwiGLU) | down (+residual)
//   then:       output head (+argmax slots)
//
// separated by a grid barrier (8 counter shards by blockIdx % 8; every workgroup adds
// to its shard once its waves' write-through stores have drained, wave 0 polls the 8
// shards; tools/barrier_bench.hip: ~1.8 us).  Between a workgroup's arrival and its
// wait the 12 "streamer" waves (4-15) already issue the loads of their first weight
// item of the next phase, so each phase starts with its weights in flight while the 4
// "leader" waves (0-3, 256 threads) load and quantize the phase's activation into LDS
// exactly as the k_matvec prologue does.  Everything one phase writes for a later phase
// of the same launch is stored write-through (sc1) and read with sc1 loads (relaxed
// agent-scope atomics: MI355X_MICROARCH.md §visibility, row 1 of the valid hand-off
// forms), so no acquire/release fences are needed.
//
// Numerics are the per-op kernels' exactly (the same device functions, mv_device.h):
// each row pair is reduced by one wave in the matvec's device order, the activation is
// quantized bit-exactly as ggml does, attention is k_attn_scores8 + k_attn_pv16's math.
// Every wait is bounded; a wait that gives up sets the context fault word (bit 2), the
// launch drains, and the decode call returns -6.
#include "kernels.h"
#include "mv_device.h"

#include <map>
#include <mutex>
#include <tuple>

namespace llmi {

namespace {

constexpr int kST = 512, kSW = 8;        // threads / waves per workgroup; one workgroup per CU
constexpr int kLead = 256;               // leader threads (waves 0-3): the activation prologue
constexpr unsigned kBarSpin = 1u << 20;  // polls before a barrier wait gives up (~0.1-0.3 s)
constexpr int kCtl = 64;                 // LDS control block (bytes) ahead of the phase scratch

struct Ctl {
    int ok;      // last barrier passed
    int tok;     // this step's token
    int pad[2];
};

__device__ __forceinline__ unsigned ld_u32(const unsigned* p) {
    return __hip_atomic_load((const gu32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_u64(const void* p) {
    return __hip_atomic_load((const gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 B through two 8-B sc1 loads
__device__ __forceinline__ u32x4 ld_u128(const void* p) {
    const unsigned long long a = ld_u64(p), b = ld_u64((const char*)p + 8);
    u32x4 r;
    r.x = (uint32_t)a; r.y = (uint32_t)(a >> 32); r.z = (uint32_t)b; r.w = (uint32_t)(b >> 32);
    return r;
}

// ---- grid barrier, split so the next phase's weight loads go out between its halves --
#if defined(LLMI_EXP_TRACE)
// experiment builds: per workgroup and barrier, s_memrealtime at arrival and release
#define STEP_STAMP(a, idx, which)                                                                \
    if (a.trace && threadIdx.x == 0)                                                             \
        a.trace[((size_t)blockIdx.x * 512 + (idx)) * 2 + (which)] = __builtin_amdgcn_s_memrealtime();
#else
#define STEP_STAMP(a, idx, which)
#endif
__device__ __forceinline__ void bar_arrive(const StepArgs& a, unsigned phase) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's hand-off stores landed
    __syncthreads();                                   // ... and every other wave's
    STEP_STAMP(a, phase, 0)
    if (threadIdx.x == 0)
        __hip_atomic_fetch_add((gu32_t*)(a.bar + 16 * (blockIdx.x & 7)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool bar_wait(const StepArgs& a, unsigned phase, Ctl* ctl) {
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < 64) {
        const unsigned nwg = gridDim.x;
        const unsigned cnt = lane < 8 ? (nwg - lane + 7) / 8 : 0;  // workgroups b with b % 8 == lane
        const unsigned target = (phase + 1) * cnt;
        bool ok = true;
        for (unsigned s = 0;; ++s) {
            const unsigned v = lane < 8 ? ld_u32(a.bar + 16 * lane) : 0xffffffffu;
            if (__all(v >= target)) break;
            if ((s & 31) == 31 && ld_u32(a.fault) != 0) { ok = false; break; }  // another workgroup gave up
            if (s >= kBarSpin) { ok = false; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        if (lane == 0) {
            if (!ok) atomicOr(a.fault, 2u);
            ctl->ok = ok ? 1 : 0;
        }
    }
    __syncthreads();
    STEP_STAMP(a, phase, 1)
    return ctl->ok != 0;
}

// ---- activation prologue ---------------------------------------------------------------
// 16 consecutive activation values of sub-block sb of the hand-off vector (sc1 loads)
__device__ __forceinline__ void load_x16(const float* x, int sb, float (&v)[16]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const unsigned long long u = ld_u64(x + sb * 16 + 2 * k);
        v[2 * k] = __uint_as_float((uint32_t)u);
        v[2 * k + 1] = __uint_as_float((uint32_t)(u >> 32));
    }
}

// [RMSNorm] + q8_K / q8_0 quantization of `cols` values into the LDS image, leader
// threads only (sub-block sb = tid + 256 i: the k_matvec prologue's mapping and its
// double sum; waves 4-15 add 0.0 to the workgroup tree), bit-exact with ggml.
template <int ACT, bool NORM>
__device__ void eng_prologue(const float* x, const float* nw, float eps, int cols, const Lds& L) {
    const int tid = threadIdx.x;
    const int nsub = cols >> 4;
    float v0[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v0[j] = 0.f;
    float scale = 1.0f;
    if constexpr (NORM) {
        double s = 0.0;
        if (tid < kLead) {
            for (int sb = tid, i = 0; sb < nsub; sb += kLead, ++i) {
                float v[16];
                load_x16(x, sb, v);
#pragma unroll
                for (int j = 0; j < 16; ++j) s += (double)(v[j] * v[j]);
                if (i == 0) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) v0[j] = v[j];
                }
            }
        }
        s = block_sum_d<kSW>(s, L.red);
        const float mean = (float)(s / (double)cols);
        scale = 1.0f / sqrtf(mean + eps);
    }
    if (tid < kLead) {
        for (int sb = tid, i = 0; sb < nsub; sb += kLead, ++i) {
            float v[16];
            if (NORM && i == 0) {
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = v0[j];
            } else {
                load_x16(x, sb, v);
            }
            if constexpr (NORM) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 w = *(const float4*)(nw + sb * 16 + 4 * k);
                    v[4 * k + 0] = (v[4 * k + 0] * scale) * w.x;
                    v[4 * k + 1] = (v[4 * k + 1] * scale) * w.y;
                    v[4 * k + 2] = (v[4 * k + 2] * scale) * w.z;
                    v[4 * k + 3] = (v[4 * k + 3] * scale) * w.w;
                }
            }
            quant_sub<ACT>(L, cols, sb, v);
        }
    }
    __syncthreads();
}

// ---- the row pairs of one matvec phase ------------------------------------------------
template <int TO, int FROM>
__device__ __forceinline__ PairRaw<TO> as_raw(const PairRaw<FROM>& r) {
    PairRaw<TO> o;
    o.a = r.a;
    o.b = r.b;
    return o;
}

// pairs p = first, first + G, ... < pend of one weight type T, pipelined one item ahead
// (mv_body's loop); `cur` = the first item's loads already in flight when `have`.
template <int ACT, int EPI, int T, class MA>
__device__ __forceinline__ unsigned long long eng_pairs(const MA& A, const Lds& L, int p, int G, int pend, bool have,
                                        PairRaw<T> cur, int pos) {
    unsigned long long best = 0;
    if (p >= pend) return best;
    const int lane = threadIdx.x & 63;
    const int nch = A.cols >> 6, NJ = (nch + 63) >> 6;
    PairRef r = pair_ref<EPI>(A, p);
    PairRows<T> rows = pair_rows<T>(r, A.cols);
    if (!have) cur = load_item<T>(rows, lane, nch);
    // residual add: the pair's old y values are loaded when the pair starts (ahead of its
    // weight loads in the vmcnt queue), so the epilogue waits for nothing it prefetched
    float yoa = 0.f, yob = 0.f;
    if constexpr (EPI == EPI_ADD) {
        yoa = ld_f32<true>(A.y + r.sa.row0 + r.ra);
        yob = r.vb ? ld_f32<true>(A.y + r.sa.row0 + r.rb) : 0.f;
    }
    int j = 0;
    float acc_a = 0.f, acc_b = 0.f;
    for (;;) {
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
        const bool has_next = pn < pend;
        PairRaw<T> nxt{};
        if (has_next) nxt = load_item<T>(rowsn, lane + 64 * jn, nch);  // (no redundant re-load at the end)
        const int ch = lane + 64 * j;
        const int chc = ch < nch ? ch : nch - 1;
        const Act act = load_act<ACT>(L, chc, nch);
        const float va = dot_chunk<T>(cur.a, act, chc), vb = dot_chunk<T>(cur.b, act, chc);
        acc_a += ch < nch ? va : 0.f;
        acc_b += ch < nch ? vb : 0.f;
        if (j == NJ - 1) {
            const PairSum sum = reduce_pair(acc_a, acc_b);
            if constexpr (EPI == EPI_ADD) {
                if (lane == 0) {
                    st_f32<true>(A.y + r.sa.row0 + r.ra, yoa + sum.a);
                    if (r.vb) st_f32<true>(A.y + r.sa.row0 + r.rb, yob + sum.b);
                }
                if (has_next && jn == 0) {
                    yoa = ld_f32<true>(A.y + rn.sa.row0 + rn.ra);
                    yob = rn.vb ? ld_f32<true>(A.y + rn.sa.row0 + rn.rb) : 0.f;
                }
            } else {
                epilogue<EPI, true>(A, r, p, sum, pos, best);
            }
            acc_a = acc_b = 0.f;
        }
        if (!has_next) break;
        cur = nxt;
        p = pn;
        j = jn;
        r = rn;
        rows = rowsn;
    }
    return best;
}

// this wave's first pair in segment range [pbeg, pend): the smallest p >= pbeg, p == gw (mod G)
__device__ __forceinline__ int first_pair(int gw, int G, int pbeg) {
    return pbeg + (((gw - pbeg) % G) + G) % G;
}

// ---- phase descriptors built from the layer table ---------------------------------------
// segment type groups: a phase's segments [i0, i1) share one type (QKV: q+k and v may differ)
struct PhaseMV {
    MVArgs A;
    int epi = 0, act = 0;
    bool norm = false;
};

template <class MA>
__device__ __forceinline__ int seg_pairs_beg(const MA& A, int i) { return (A.seg[i].row0 - A.seg[0].row0) / 2; }
template <class MA>
__device__ __forceinline__ int seg_pairs_end(const MA& A, int i) {
    return (A.seg[i].row0 - A.seg[0].row0 + A.seg[i].rows + 1) / 2;
}

// issue this wave's first item of segment 0 (prefetch across the barrier)
template <int T, int EPI, class MA>
__device__ __forceinline__ PairRaw<T> first_item(const MA& A, int gw, bool& have) {
    PairRaw<T> w{};
    const int pend = EPI == EPI_SWIGLU ? A.npairs : seg_pairs_end(A, 0);
    have = gw < pend;
    if (have) {
        const PairRef r = pair_ref<EPI>(A, gw);
        w = load_item<T>(pair_rows<T>(r, A.cols), threadIdx.x & 63, A.cols >> 6);
    }
    return w;
}

// ---- attention phases (k_attn_scores8 / k_attn_pv16 math, items spread over the grid) --
// phase A: item (group g, 32-position tile); 4 items per workgroup (256 threads each).
template <int D, int G>
__device__ void eng_attn_scores(const StepArgs& a, int l, int n_kv, uint8_t* lds) {
    constexpr int IPW = kST / 256;  // items per workgroup pass
    const int tid = threadIdx.x, sg = tid >> 8, t256 = tid & 255, lane = tid & 63, wave = t256 >> 6;
    double* qs = (double*)lds + (size_t)sg * G * D;                        // [IPW][G][D]
    float* wmax = (float*)(lds + (size_t)IPW * G * D * 8) + (size_t)sg * 4 * G;  // [IPW][4][G]
    constexpr int DQ = D / 8;
    const int ntile = (n_kv + 31) >> 5;
    const int nitem = a.HK * ntile;
    const size_t kvl = (size_t)a.HK * a.n_ctx * D;
    const uint16_t* kc = a.kc + (size_t)l * kvl;
    for (int base = blockIdx.x * IPW; base < nitem; base += gridDim.x * IPW) {  // uniform per workgroup
        const int it = base + sg;
        const bool on = it < nitem;
        const int g = on ? it / ntile : 0, tile = on ? it % ntile : 0, t0 = tile * 32;
        const int t = t0 + (t256 >> 3), qd = t256 & 7;
        const int tc = t < n_kv ? t : n_kv - 1;
        u32x4 kv[DQ / 8];
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i) kv[i] = ld_u128(kc + ((size_t)g * a.n_ctx + tc) * D + qd * DQ + 8 * i);
        if (on)
            for (int i = t256; i < G * D; i += 256) qs[i] = (double)h2f(f2h(ld_f32<true>(a.q + (size_t)g * G * D + i)));
        __syncthreads();
        double k[DQ];
#pragma unroll
        for (int i = 0; i < DQ / 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                k[8 * i + 2 * j] = (double)h2f((uint16_t)kv[i][j]);
                k[8 * i + 2 * j + 1] = (double)h2f((uint16_t)(kv[i][j] >> 16));
            }
#pragma unroll 1
        for (int hh = 0; hh < G; ++hh) {  // one head at a time: DQ double FMAs, 8-lane butterfly
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < DQ; ++j) acc = __builtin_fma(k[j], qs[hh * D + qd * DQ + j], acc);
            acc += xor_partner_d<1>(acc);
            acc += xor_partner_d<2>(acc);
            acc += xor_partner_d<4>(acc);
            const float sc = (float)acc * a.scale;
            if (on && t < n_kv && qd == (hh & 7)) st_f32<true>(a.scores + (size_t)(g * G + hh) * a.n_ctx + t, sc);
            float m = t < n_kv ? sc : -INFINITY;
            m = fmaxf(m, xor_partner<8>(m));
            m = fmaxf(m, xor_partner<16>(m));
            m = fmaxf(m, xor_partner<32>(m));
            if (lane == 0) wmax[wave * G + hh] = m;
        }
        __syncthreads();
        if (on && t256 < G)
            st_f32<true>(a.tmax + (size_t)(g * G + t256) * (a.n_ctx / 32) + tile,
                         fmaxf(fmaxf(wmax[0 * G + t256], wmax[1 * G + t256]), fmaxf(wmax[2 * G + t256], wmax[3 * G + t256])));
        __syncthreads();
    }
}

// phase B: item (group g, 16 output dims): softmax of the group's G heads from the
// scores and tile maxima, p = f16(e / sum), PV (512 threads; one item per workgroup).
template <int D, int G>
__device__ void eng_attn_pv(const StepArgs& a, int l, int n_kv, uint8_t* lds) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kvb = a.kv_bound;
    float* spd = (float*)lds;                           // [G][kvb]
    float* redm = (float*)(lds + (size_t)G * kvb * 4);  // [8]
    double* reds = (double*)(redm + 8);                 // [8]
    constexpr int WPH = 8 / G;
    const int nitem = a.HK * (D / 16);
    const size_t kvl = (size_t)a.HK * a.n_ctx * D;
    const uint16_t* vcl = a.vc + (size_t)l * kvl;
    for (int it = blockIdx.x; it < nitem; it += gridDim.x) {  // uniform per workgroup
        const bool act = tid < 512;
        const int g = it / (D / 16), dc = it % (D / 16);
        const int d = dc * 16 + ((tid & 511) >> 5), sl = tid & 31;
        const uint16_t* vr = vcl + ((size_t)g * D + d) * a.n_ctx;
        if (act) {
            const int n4 = (n_kv + 3) >> 2;
            for (int hh = 0; hh < G; ++hh) {
                const float* src = a.scores + (size_t)(g * G + hh) * a.n_ctx;
                for (int j = tid; j < n4; j += 512) {
                    const u32x4 v = ld_u128(src + 4 * j);
                    *(u32x4*)(spd + hh * kvb + 4 * j) = v;
                }
            }
        }
        const int hh = wave / WPH, wi = wave % WPH;
        if (act) {  // row max from the tile maxima
            const float* tm = a.tmax + (size_t)(g * G + hh) * (a.n_ctx / 32);
            const int ntile = (n_kv + 31) >> 5;
            float m = -INFINITY;
            for (int i = wi * 64 + lane; i < ntile; i += WPH * 64) m = fmaxf(m, ld_f32<true>(tm + i));
            m = wave_max(m);
            if (lane == 0) redm[wave] = m;
        }
        __syncthreads();
        double sum = 0.0;
        float* sp = spd + hh * kvb;
        float mx = 0.f;
        if (act) {
            mx = redm[hh * WPH];
#pragma unroll
            for (int i = 1; i < WPH; ++i) mx = fmaxf(mx, redm[hh * WPH + i]);
            for (int t = wi * 64 + lane; t < n_kv; t += WPH * 64) {
                const float e = llmi_expf(sp[t] - mx);
                sp[t] = e;
                sum += (double)e;
            }
            sum = wave_sum_d(sum);
            if (lane == 0) reds[wave] = sum;
        }
        __syncthreads();
        if (act) {
            double tot = reds[hh * WPH];
#pragma unroll
            for (int i = 1; i < WPH; ++i) tot += reds[hh * WPH + i];
            const float inv = (float)(1.0 / tot);
            for (int t = wi * 64 + lane; t < n_kv; t += WPH * 64) sp[t] = h2f(f2h(sp[t] * inv));
            for (int t = n_kv + wi * 64 + lane; t < ((n_kv + 3) & ~3); t += WPH * 64) sp[t] = 0.f;
        }
        __syncthreads();
        if (act) {
            double acc[G];
#pragma unroll
            for (int h = 0; h < G; ++h) acc[h] = 0.0;
            constexpr int NV = 8;  // 8-B V loads in flight per lane: a 1024-position window
            for (int t0 = 4 * sl; t0 < n_kv; t0 += 128 * NV) {
                unsigned long long vv[NV];
#pragma unroll
                for (int k = 0; k < NV; ++k) vv[k] = ld_u64(vr + min(t0 + 128 * k, kvb - 4));
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                    const int tb = t0 + 128 * k;
                    if (tb < n_kv) {
                        double v[4];
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {
                            const float f = h2f((uint16_t)(vv[k] >> (16 * jj)));
                            v[jj] = tb + jj < n_kv ? (double)f : 0.0;
                        }
#pragma unroll
                        for (int h = 0; h < G; ++h) {
                            const float4 pp = *(const float4*)(spd + h * kvb + tb);
                            acc[h] = __builtin_fma(v[0], (double)pp.x, acc[h]);
                            acc[h] = __builtin_fma(v[1], (double)pp.y, acc[h]);
                            acc[h] = __builtin_fma(v[2], (double)pp.z, acc[h]);
                            acc[h] = __builtin_fma(v[3], (double)pp.w, acc[h]);
                        }
                    }
                }
            }
#pragma unroll
            for (int h = 0; h < G; ++h) {
                double v = acc[h];
                v += xor_partner_d<1>(v);
                v += xor_partner_d<2>(v);
                v += xor_partner_d<4>(v);
                v += xor_partner_d<8>(v);
                v += xor_partner_d<16>(v);
                if (sl == 0) st_f32<true>(a.att + (size_t)(g * G + h) * D + d, (float)v);
            }
        }
        __syncthreads();
    }
}

template <int D, int G>
__device__ __forceinline__ bool eng_attention_dg(const StepArgs& a, int l, int n_kv, uint8_t* lds, unsigned phase, Ctl* ctl) {
    eng_attn_scores<D, G>(a, l, n_kv, lds);
    bar_arrive(a, phase);
    if (!bar_wait(a, phase, ctl)) return false;
    eng_attn_pv<D, G>(a, l, n_kv, lds);
    return true;
}

// ---- one matvec phase whose first segment has weight type T --------------------------
// The streamer waves issue their first item's loads, THEN the workgroup waits at the
// barrier (if `wait`), then the leaders quantize the activation and every wave runs its
// pairs: segment 0 from the prefetched item, any further segment (QKV's attn_v of
// another type) in its own type.  Returns the wave's LOGITS argmax key.
template <int ACT, int EPI, int T, int T2, class MA>
__device__ __forceinline__ unsigned long long seg_pairs_t(const MA& A, const Lds& L, int i, int gw, int G, int pos) {
    const int pbeg = seg_pairs_beg(A, i), pend = seg_pairs_end(A, i);
    PairRaw<T2> none{};
    return eng_pairs<ACT, EPI, T2>(A, L, first_pair(gw, G, pbeg), G, pend, false, none, pos);
}

// The phase descriptor is read through the constant address space: scalar loads (lgkmcnt),
// held in SGPRs — with generic loads the compiler re-read fields with vector loads in the
// epilogues, and their vmcnt(0) waits drained the weight pipeline every pair.
typedef const __attribute__((address_space(4))) MVArgs ConstMV;

template <int EPI, int T>
__device__ __forceinline__ unsigned long long run_phase(const StepArgs& a, const MVArgs* Ap, bool norm,
                                        uint8_t* scratch, int gw, int G, bool streamer, bool wait, unsigned phase,
                                        Ctl* ctl, int pos) {
    constexpr int ACT = T == T_Q8_0 ? 1 : 0;
    ConstMV& A = *(ConstMV*)(uintptr_t)Ap;
    bool have = false;
    PairRaw<T> cur{};
    if (streamer) cur = first_item<T, EPI>(A, gw, have);
    if (wait && !bar_wait(a, phase, ctl)) return 0;  // the caller reads ctl->ok
    const Lds L = carve(scratch, ACT, A.cols);
    if (norm) eng_prologue<ACT, true>(A.x, A.nw, A.eps, A.cols, L);
    else eng_prologue<ACT, false>(A.x, A.nw, A.eps, A.cols, L);
    const int pend0 = EPI == EPI_SWIGLU ? A.npairs : seg_pairs_end(A, 0);
    unsigned long long best = eng_pairs<ACT, EPI, T>(A, L, gw, G, pend0, have, cur, pos);
    if constexpr (EPI == EPI_QKV) {
#pragma unroll
        for (int i = 1; i < 3; ++i) {  // constant segment indices: A stays in registers
            if (i >= A.nseg) break;
            unsigned long long b = 0;
            if constexpr (ACT == 1) {
                b = seg_pairs_t<1, EPI, T, T_Q8_0>(A, L, i, gw, G, pos);
            } else {
                switch (A.seg[i].type) {
                    case T_Q4_K: b = seg_pairs_t<0, EPI, T, T_Q4_K>(A, L, i, gw, G, pos); break;
                    case T_Q5_K: b = seg_pairs_t<0, EPI, T, T_Q5_K>(A, L, i, gw, G, pos); break;
                    case T_Q6_K: b = seg_pairs_t<0, EPI, T, T_Q6_K>(A, L, i, gw, G, pos); break;
                    default: break;
                }
            }
            best = b > best ? b : best;
        }
    }
    return best;
}

// dispatch on the phase's first weight type
template <int EPI>
__device__ __forceinline__ unsigned long long phase_any(const StepArgs& a, const MVArgs* Ap, bool norm,
                                                        uint8_t* scratch, int gw, int G, bool streamer,
                                                        bool wait, unsigned phase, Ctl* ctl, int pos) {
#ifdef STEP_ONLY_Q4K
    return run_phase<EPI, T_Q4_K>(a, Ap, norm, scratch, gw, G, streamer, wait, phase, ctl, pos);
#endif
    switch (((ConstMV*)(uintptr_t)Ap)->seg[0].type) {
        case T_Q4_K: return run_phase<EPI, T_Q4_K>(a, Ap, norm, scratch, gw, G, streamer, wait, phase, ctl, pos);
        case T_Q5_K: return run_phase<EPI, T_Q5_K>(a, Ap, norm, scratch, gw, G, streamer, wait, phase, ctl, pos);
        case T_Q6_K: return run_phase<EPI, T_Q6_K>(a, Ap, norm, scratch, gw, G, streamer, wait, phase, ctl, pos);
        default: return run_phase<EPI, T_Q8_0>(a, Ap, norm, scratch, gw, G, streamer, wait, phase, ctl, pos);
    }
}

}  // namespace

// The step's token selection, state update and embedding row run in k_embed, the
// launch before this one (its x is visible here through the kernel boundary).
template <int D, int GQ>
__global__ __launch_bounds__(kST) void k_step(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Ctl* ctl = (Ctl*)smem;
    uint8_t* scratch = smem + kCtl;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = uniform((int)(tid >> 6));
    const int G = (int)gridDim.x * kSW, gw = (int)blockIdx.x * kSW + wave;
    const bool streamer = wave >= kLead / 64;
    StepState* st = a.st;
    const int pos = st->pos;
    const int n_kv = pos + 1;
    // barrier 6 l + k closes phase k of layer l (QKV, scores, PV, O, gate/up, down); the
    // shard counters are cumulative over the launch: barrier b completes at (b + 1) x count
    ctl->ok = 1;
    __syncthreads();
    for (int l = 0; l < a.n_layer; ++l) {
        const unsigned b0 = 6u * (unsigned)l;
        // QKV + RoPE + f16 KV write (waits at the barrier that closed the previous down)
        (void)phase_any<EPI_QKV>(a, a.mv + 4 * l + 0, true, scratch, gw, G, streamer, l > 0, b0 - 1u, ctl, pos);
        if (!ctl->ok) return;
        bar_arrive(a, b0);
        if (!bar_wait(a, b0, ctl)) return;
        // attention: scores phase | barrier | softmax + PV phase
        if (!eng_attention_dg<D, GQ>(a, l, n_kv, scratch, b0 + 1u, ctl)) return;
        bar_arrive(a, b0 + 2u);
        // attn_output + residual
        (void)phase_any<EPI_ADD>(a, a.mv + 4 * l + 1, false, scratch, gw, G, streamer, true, b0 + 2u, ctl, pos);
        if (!ctl->ok) return;
        bar_arrive(a, b0 + 3u);
        // gate/up + SwiGLU
        (void)phase_any<EPI_SWIGLU>(a, a.mv + 4 * l + 2, true, scratch, gw, G, streamer, true, b0 + 3u, ctl, pos);
        if (!ctl->ok) return;
        bar_arrive(a, b0 + 4u);
        // down + residual
        (void)phase_any<EPI_ADD>(a, a.mv + 4 * l + 3, false, scratch, gw, G, streamer, true, b0 + 4u, ctl, pos);
        if (!ctl->ok) return;
        bar_arrive(a, b0 + 5u);
    }
    // output head + argmax: workgroup max of the waves' keys, one atomic per workgroup
    const unsigned long long best = phase_any<EPI_LOGITS>(a, a.mv + 4 * a.n_layer, true, scratch, gw, G, streamer, true,
                                                          6u * (unsigned)a.n_layer - 1u, ctl, pos);
    if (!ctl->ok) return;
    unsigned long long* red = (unsigned long long*)scratch;
    __syncthreads();
    if (lane == 0) red[wave] = best;
    __syncthreads();
    if (tid == 0) {
        unsigned long long b = red[0];
        for (int w = 1; w < kSW; ++w) b = red[w] > b ? red[w] : b;
        if (b) atomicMax(&st->key[pos & 1][blockIdx.x % kArgSlots], b);
        if (blockIdx.x == 0) st->pos_next = pos + 1;
    }
}

// ---- host side -----------------------------------------------------------------------------
static size_t step_lds(const StepArgs& a) {
    size_t m = 0;
    const int colss[3] = {a.E, a.H * a.D, a.F};
    for (int act = 0; act < 2; ++act)
        for (int c : colss) m = std::max(m, lds_red_off(act, c) + kSW * sizeof(double));
    const int G = a.HK > 0 ? a.H / a.HK : 1;
    m = std::max(m, (size_t)4 * G * a.D * 8 + 4 * 4 * G * 4);       // scores phase
    m = std::max(m, (size_t)G * a.kv_bound * 4 + 8 * 4 + 8 * 8);   // PV phase
    m = std::max(m, (size_t)kSW * 8);                                // argmax keys
    return kCtl + ((m + 15) & ~(size_t)15);
}

template <int D, int GQ>
static const void* step_kernel_t() { return (const void*)k_step<D, GQ>; }
static const void* step_kernel(const StepArgs& a) {
    const int g = a.HK > 0 ? a.H / a.HK : 0;
#define LLMI_SK(D_, G_) if (a.D == D_ && g == G_) return step_kernel_t<D_, G_>();
    LLMI_SK(128, 1) LLMI_SK(128, 2) LLMI_SK(128, 4) LLMI_SK(128, 8)
    LLMI_SK(64, 1) LLMI_SK(64, 2) LLMI_SK(64, 4) LLMI_SK(64, 8)
#undef LLMI_SK
    return nullptr;
}

bool step_supported(const StepArgs& a, int device, std::string* why) {
    auto no = [&](const char* w) {
        if (why) *why = w;
        return false;
    };
    const void* k = step_kernel(a);
    if (!k) return no("head_dim / GQA");
    if (a.E % 256 || a.F % 256 || (a.H * a.D) % 256) return no("widths");
    if (a.n_rot % 2 || a.n_rot > a.D) return no("n_rot");
    const size_t lds = step_lds(a);
    if (lds > 160 * 1024) return no("LDS (KV bound too long for the in-launch attention)");
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, size_t>, bool> cache;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_tuple(k, device, lds);
    auto it = cache.find(key);
    if (it == cache.end()) {
        bool ok = true;
        if (lds > 64 * 1024 && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            ok = false;
        int occ = 0;
        ok = ok && hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kST, lds) == hipSuccess && occ >= 1;
        it = cache.emplace(key, ok).first;
    }
    if (!it->second) return no("one workgroup per CU is not resident");
    return true;
}

hipError_t launch_step(const StepArgs& a, hipStream_t s) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return hipErrorInvalidDevice;
    const void* k = step_kernel(a);
    if (!k) return hipErrorInvalidValue;
    const size_t lds = step_lds(a);
    hipError_t e = hipMemsetAsync(a.bar, 0, kStepBarWords * 4, s);
    if (e != hipSuccess) return e;
    void* args[] = {(void*)&a};
    return hipLaunchKernel(k, dim3(cus), dim3(kST), args, lds, s);
}

}  // namespace llmi
