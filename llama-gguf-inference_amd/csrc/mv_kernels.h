// mv_kernels.h — the single-token quantized matvec kernel (k_matvec, 4- or 8-wave workgroups)
// and their launchers, compiled once per weight type in mv_q4k.hip / mv_q5k.hip /
// mv_q6k.hip / mv_q80.hip (explicit instantiations of mv_dispatch_epi and mv_qkv2_launch,
// declared in kernels.h).  Split by type so the instantiations build in parallel.
#pragma once
#include "kernels.h"
#include "launch_util.h"
#include "mv_device.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace llmi {

#ifndef LLMI_MV_PINGPONG
#define LLMI_MV_PINGPONG 1
#endif
#ifndef LLMI_Q6_MASKED
#define LLMI_Q6_MASKED 1
#endif
constexpr bool kQ6Masked = LLMI_Q6_MASKED != 0;
// LDS of a k_matvec launch of NW waves whose pipelined types are T / T2
__host__ inline size_t mv_lds_total(int act, int cols, int nw, int t, int t2, int x86 = 0) {
    const int ff = fold_stride_cols(act, x86, cols);
    const size_t base = fold_off(act, cols, nw) + (size_t)nw * ff * 4;
    return base + ((kQ6Masked && !x86 && (t == T_Q6_K || t2 == T_Q6_K)) ? (size_t)(cols >> 8) * kQ6MaskRec : 0);
}

static int g_split_by_pairs = getenv("LLMI_SPLIT_BY_PAIRS") ? atoi(getenv("LLMI_SPLIT_BY_PAIRS")) : 0;  // A/B only


// The matvec of the task range [tbeg, tend) by waves starting at task t0 with stride G
// (one type group of a launch); returns the wave's LOGITS argmax key.  Per sub-item:
// every lane's unit terms into the wave's fold buffer F, the fold lanes add them onto
// their chains; after a row set's last sub-item the row sums (ggml's generic order,
// mv_device.h) go to the epilogue.  The next sub-item's units are in flight meanwhile.
#if defined(LLMI_EXP_TRACE)
// per-wave stamps (tools/mvtrace.py): [block][wave][16] = {entry, prologue done, first
// sub-item done, exit, -, XCC << 32 | sub-items, x arrived, -, end of sub-items 2..9}
#define MV_STAMP(I, V)                                                                                    \
    if (A.trace && (threadIdx.x & 63) == 0)                                                               \
        A.trace[((size_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6)) * 16 + (I)] = (V);
#define MV_NOW __builtin_amdgcn_s_memrealtime()
#else
#define MV_STAMP(I, V)
#endif

template <int ACT, bool NORM, int EPI, int T, int NP, int NT = kMVThreads, int X86 = 0>
__device__ __forceinline__ unsigned long long mv_body(const MVArgs& A, const Lds& L, float* F, int t0, int G, int tbeg,
                                                      int tend) {
    int pos = 0;
    if constexpr (EPI == EPI_QKV) pos = A.st->pos;
    unsigned long long best = 0;
    const int lane = threadIdx.x & 63;
    const TaskGeo g = task_geo(A);
    const int S = EPI == EPI_SWIGLU ? 2 * g.nj : g.nj;
    const int r = lane / g.lr, ul = lane - r * g.lr;

    int task = t0;
    MV_STAMP(0, MV_NOW)
    [[maybe_unused]] int nsub_done = 0, nsub_alt = 0;
    ProRegs<NORM, NP> R;
    ImgRegs<2 * NP + 1> RI;
    const bool img = A.xq != nullptr;
    if (img) mv_img_issue<2 * NP + 1, NT>(A, RI);  // activation loads first ...
    else mv_prologue_issue<NORM, NP, NT>(A, R);
    // Single-round launches (every wave owns at most one task: QKV, attn_output) issue
    // their weights only once the activation has arrived: the activation loads then do
    // not queue behind the chip-wide weight burst, and the weight latency overlaps the
    // quantization instead.  Multi-round launches keep the weights in flight from the start.
    if ((tend - tbeg <= G && A.xfirst >= 0) || A.xfirst > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool pipe = task < tend && task_is<EPI, T>(A, g, task);
    Sub b = sub_of<EPI>(A, g, task < tend ? task : tend - 1, 0);
    Seg sg = pick(A, b.si);
    LaneUnit lu = lane_unit(g, b, sg, r, ul);
    // ... then the first units, in flight during the prologue (issued on every path: an
    // idle wave reads unit 0 of row 0, so the prologue's first wait counts only the activation)
    // (prefetch distance 2 -- three rotating register buffers in a 3x unrolled loop --
    // measured slower on every shape: gate+up 16.9 -> 21.2 us, 516 -> 433 tok/s)
    UnitW<T> cur = load_unit<T>(sg, pipe ? lu.row : 0u, pipe ? lu.u : 0u, g.U);
    if (img) mv_img_finish<2 * NP + 1, NT>(A, L, RI);
    else mv_prologue_finish<ACT, NORM, NP, NT, X86>(A, L, R);
    __syncthreads();
    // Q6_K: the masked activation copies (mv_device.h q6_masks_build), after the fold buffers
    [[maybe_unused]] uint8_t* q6m = nullptr;
    if constexpr (T == T_Q6_K && kQ6Masked && !X86) {
        q6m = (uint8_t*)L.act + fold_off(ACT, A.cols, NT / 64) + (size_t)(NT / 64) * kFoldFloats * 4;
        q6_masks_build<NT>(L, g.U, q6m);
        __syncthreads();
    }
    MV_STAMP(1, MV_NOW)

    if (pipe) {
        int s = 0;
        float acc = 0.f, vg = 0.f;
        bool first_sub = A.fw != 0;
        // One sub-item: prefetch the next one into `nxt`, reduce `cur`.  The loop runs it
        // twice per trip with the two register buffers' roles swapped (ping-pong), so no
        // `cur = nxt` copy of the 36-52 registers of a unit is made per sub-item (Q6_K:
        // ~130 v_mov of the ~885 VALU of a sub-item, and its matvecs are VALU-bound).
        auto step = [&](UnitW<T>& cur, UnitW<T>& nxt) -> bool {
            // next sub-item: (task, s+1) or (task+G, 0); uniform control flow
            int tn = task, sn = s + 1;
            Sub bn = b;
            Seg sgn = sg;
            bool has_next = true;
            if (sn == S) {
                sn = 0;
                tn = task + G;
                has_next = tn < tend && task_is<EPI, T>(A, g, tn);
            }
            if (has_next) {
                bn = sub_of<EPI>(A, g, tn, sn);
                sgn = pick(A, bn.si);
            }
            const LaneUnit lun = lane_unit(g, bn, sgn, r, ul);
            if (first_sub) {  // LLMI_MV_FW: the first sub-item lands before the second is requested
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                first_sub = false;
            }
            // always issue the prefetch (straight-line vmcnt counting); past the wave's last
            // sub-item every lane reads unit 0 of row 0 -- one line per part per wave instead
            // of a nontemporal re-read of the wave's 9-14 KB (FETCH_SIZE: +14 MB per gate+up)
            nxt = load_unit<T>(sgn, has_next ? lun.row : 0u, has_next ? lun.u : 0u, g.U);
            float tm[9];
            if constexpr (X86)
                unit_store_x86<T>(cur, L.act + (size_t)lu.u * kRec, F, r, ul, g.lr, g.R, lu.valid);
            else if constexpr (T == T_Q6_K && kQ6Masked)
                unit_terms_q6m(cur, q6m + (size_t)lu.u * kQ6MaskRec, *(const float*)(L.act + (size_t)lu.u * kRec + kRecD), tm);
            else
                unit_terms<T>(cur, L.act + (size_t)lu.u * kRec, tm);
            sub_finish<ACT, EPI, MVArgs, X86>(A, F, g, s, b, sg, tm, lu, r, ul, acc, vg, pos, best);
#if defined(LLMI_EXP_TRACE)
            ++nsub_done;
            if (nsub_done == 1) { MV_STAMP(2, MV_NOW) }
            else if (nsub_done <= 9) { MV_STAMP(6 + nsub_done, MV_NOW) }
#endif
            task = tn;
            if (!has_next) return false;
            s = sn;
            b = bn;
            sg = sgn;
            lu = lun;
            return true;
        };
#if LLMI_MV_PINGPONG
        UnitW<T> other;
        for (;;) {
            if (!step(cur, other)) break;
            if (!step(other, cur)) break;
        }
#else
        for (;;) {
            UnitW<T> nxt;
            if (!step(cur, nxt)) break;
            cur = nxt;
        }
#endif
    }
    // remaining tasks of other types (or all tasks if the first was not of type T)
    for (; task < tend; task += G) task_any<ACT, EPI, MVArgs, X86>(A, L, F, g, task, r, ul, pos, best);
    MV_STAMP(3, MV_NOW)
    MV_STAMP(5, ((unsigned long long)(__builtin_amdgcn_s_getreg(6164) & 15) << 32) | (unsigned)nsub_done)
    return best;
}

// A launch whose segments form two type groups (QKV with a Q6_K or Q5_K attn_v) is
// split by workgroup: workgroups [0, split_wgs) run the tasks of type T, the rest the
// tasks of type T2, each group pipelined in its own type (no divergence in a workgroup).
template <int ACT, bool NORM, int EPI, int T, int NP, int T2 = T, int NT = kMVThreads, int X86 = 0>
__global__ __launch_bounds__(NT) void k_matvec(MVArgs A) {
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Lds L = carve(smem, ACT, A.cols);
    const int wave = uniform((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    float* F = (float*)(smem + fold_off(ACT, A.cols, NW)) + wave * fold_stride(ACT, X86, A.rpt, A.lr);
    unsigned long long best;
    if constexpr (T2 == T) {
        // single type: optionally two task ranges, the larger one for the first dispatch
        // round of workgroups (mv_launch: the older of two co-resident workgroups wins
        // VALU arbitration and runs ~20 % faster per sub-item); one call site either way
        int t0 = blockIdx.x * NW + wave, G = gridDim.x * NW, tb = 0, te = A.ntasks;
        if (A.split_wgs > 0) {
            if ((int)blockIdx.x < A.split_wgs) {
                G = A.split_wgs * NW;
                te = A.split_tasks;
            } else {
                t0 = A.split_tasks + (blockIdx.x - A.split_wgs) * NW + wave;
                G = (gridDim.x - A.split_wgs) * NW;
                tb = A.split_tasks;
            }
        }
        best = mv_body<ACT, NORM, EPI, T, NP, NT, X86>(A, L, F, t0, G, tb, te);
    } else {
        if ((int)blockIdx.x < A.split_wgs)
            best = mv_body<ACT, NORM, EPI, T, NP, NT, X86>(A, L, F, blockIdx.x * NW + wave, A.split_wgs * NW, 0, A.split_tasks);
        else
            best = mv_body<ACT, NORM, EPI, T2, NP, NT, X86>(A, L, F, A.split_tasks + (blockIdx.x - A.split_wgs) * NW + wave,
                                                            (gridDim.x - A.split_wgs) * NW, A.split_tasks, A.ntasks);
    }
    if constexpr (EPI == EPI_LOGITS) {
        // workgroup max of the lanes' keys, then one atomic into this workgroup's slot
        const int cur_pos = A.st->pos;
        unsigned long long* red = (unsigned long long*)L.red;
        best = wave_max_u64(best);
        __syncthreads();
        if (lane == 0) red[wave] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long b = red[0];
#pragma unroll
            for (int w = 1; w < NW; ++w) b = red[w] > b ? red[w] : b;
            if (b) atomicMax(&A.argmax[(cur_pos & 1) * kArgSlots + blockIdx.x % kArgSlots], b);
            if (blockIdx.x == 0) A.st->pos_next = cur_pos + 1;
        }
    }
}

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

// Share of a long single-type launch's tasks given to the first dispatch round of
// workgroups when two workgroups share each CU (profiles/r03/matvec/old_young_workgroups.json:
// the older workgroup of a CU retires a sub-item in 3.91 us where the younger takes 4.90
// on the output head, 2.87 vs 3.40 on gate+up): the first round gets share / (1 + share)
// of the tasks.  LLMI_MV_OLD_SHARE (A/B; 1 = equal ranges, 0 = off) — which wave reduces
// a task never changes a result.
static inline double old_share() {
    static const double v = [] {
        const char* e = getenv("LLMI_MV_OLD_SHARE");
        return e ? atof(e) : 1.25;
    }();
    return v;
}
// Wide launches: ONE workgroup of 8 waves per CU instead of two of 4.  Every workgroup
// re-derives the activation image from the f32 input (the prologue), so the chip reads
// the activation once per workgroup: 512 x 57 KB = 29 MB beside ffn_down's 33 MB of
// weights at 14336 columns (profiles/r03/matvec trace: the first sub-item's weights land
// only ~6 us into the launch).  One workgroup per CU halves that traffic and shares the
// quantization over 512 threads.  LLMI_MV_WIDE = the fewest columns that go wide
// (0 = never); which wave reduces a row never changes a result.
static inline int wide_cols() {
    static const int v = [] {
        const char* e = getenv("LLMI_MV_WIDE");
        return e ? atoi(e) : 12288;  // ffn_down of the 8B / Mistral / 70B shapes
    }();
    return v;
}
// LLMI_MV_WIDE_EPI: bitmask of epilogues that may go wide (A/B; default ADD | SWIGLU | QKV)
static inline int wide_epis() {
    static const int v = [] {
        const char* e = getenv("LLMI_MV_WIDE_EPI");
        return e ? atoi(e) : (1 << EPI_ADD) | (1 << EPI_SWIGLU) | (1 << EPI_QKV);
    }();
    return v;
}
constexpr int kMVWide = 512;
template <int ACT, bool NORM, int T, int EPI, int NP, int X86>
static hipError_t mv_launch_wide(const MVArgs& a, hipStream_t s) {
    constexpr int NW = kMVWide / 64;
    const size_t lds = mv_lds_total(ACT, a.cols, NW, T, T, X86);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const int blocks = std::max(1, std::min(cu_count(), (a.ntasks + NW - 1) / NW));
    launch_k(k_matvec<ACT, NORM, EPI, T, NP, T, kMVWide, X86>, dim3(blocks), dim3(kMVWide), lds, s, true, true, a);
    return hipGetLastError();
}
template <int ACT, bool NORM, int T, int EPI, int X86>
static bool mv_try_wide(const MVArgs& a, hipStream_t s, hipError_t& e) {
    if constexpr ((EPI == EPI_ADD || EPI == EPI_SWIGLU || EPI == EPI_QKV || EPI == EPI_LOGITS) && !(X86 && ACT)) {
        const int wc = wide_cols();
        if (wc <= 0 || a.cols < wc || cu_count() <= 0 || !(wide_epis() >> EPI & 1)) return false;
        for (int i = 0; i < a.nseg; ++i)
            if (a.seg[i].type != T) return false;  // single-type launches only
        const int per = (a.cols / 16 + kMVWide - 1) / kMVWide;
        e = per <= 1 ? mv_launch_wide<ACT, NORM, T, EPI, 1, X86>(a, s)
            : per <= 2 ? mv_launch_wide<ACT, NORM, T, EPI, 2, X86>(a, s) : mv_launch_wide<ACT, NORM, T, EPI, 4, X86>(a, s);
        return true;
    } else {
        (void)a; (void)s; (void)e;
        return false;
    }
}
// Narrow launches: fewer tasks than the waves of one 4-wave workgroup per CU (TinyLlama's
// 2048-column QKV, O and gate+up: 256-704 tasks of 8 rows) run as one-wave workgroups, one
// task each, so they spread over up to ntasks CUs instead of ntasks / 4 (each workgroup
// still builds the whole activation image).  LLMI_MV_NARROW = 0 turns it off (A/B); which
// wave reduces a row never changes a result.
constexpr int kMVNarrow = 64;
static inline int narrow_on() {
    static const int v = getenv("LLMI_MV_NARROW") ? atoi(getenv("LLMI_MV_NARROW")) : 1;
    return v;
}
// tasks per CU below which a launch goes narrow (LLMI_MV_NARROW_TPC, A/B; default 4 = the
// waves of one 4-wave workgroup)
static inline int narrow_tpc() {
    static const int v = getenv("LLMI_MV_NARROW_TPC") ? atoi(getenv("LLMI_MV_NARROW_TPC")) : kMVWaves;
    return v;
}
template <int ACT, bool NORM, int T, int EPI, int NP, int X86>
static hipError_t mv_launch_narrow(const MVArgs& a0, hipStream_t s) {
    const size_t lds = mv_lds_total(ACT, a0.cols, 1, T, T, X86);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    auto k = k_matvec<ACT, NORM, EPI, T, NP, T, kMVNarrow, X86>;
    const dim3 g = resident_grid(k, dim3(a0.ntasks), lds, kMVNarrow);
    MVArgs a = a0;
    a.split_wgs = 0;
    launch_k(k, g, dim3(kMVNarrow), lds, s, true, true, a);
    return hipGetLastError();
}
template <int ACT, bool NORM, int T, int EPI, int X86>
static bool mv_try_narrow(const MVArgs& a, hipStream_t s, hipError_t& e) {
    if constexpr (EPI == EPI_ADD || EPI == EPI_SWIGLU || EPI == EPI_QKV || EPI == EPI_STORE) {
        const int cus = cu_count();
        if (!narrow_on() || cus <= 0 || a.ntasks >= cus * narrow_tpc()) return false;
        for (int i = 0; i < a.nseg; ++i)
            if (a.seg[i].type != T) return false;  // single-type launches only
        const int per = (a.cols / 16 + kMVNarrow - 1) / kMVNarrow;
        e = per <= 2 ? mv_launch_narrow<ACT, NORM, T, EPI, 2, X86>(a, s) : mv_launch_narrow<ACT, NORM, T, EPI, 4, X86>(a, s);
        return true;
    } else {
        (void)a; (void)s; (void)e;
        return false;
    }
}
template <int ACT, bool NORM, int T, int EPI, int NP, int X86>
static hipError_t mv_launch(const MVArgs& a0, dim3 grid, size_t lds_in, hipStream_t s) {
    const size_t lds = std::max(lds_in, mv_lds_total(ACT, a0.cols, kMVWaves, T, T, X86));
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    auto k = k_matvec<ACT, NORM, EPI, T, NP, T, kMVThreads, X86>;
    const dim3 g = resident_grid(k, grid, lds);
    MVArgs a = a0;
    a.split_wgs = 0;
    const double sh = old_share();
    const int cus = cu_count();
    // long launches only (>= 4 tasks per wave), and only when the grid is exactly two
    // dispatch rounds of one workgroup per CU
    if (sh > 0 && cus > 0 && (int)g.x == 2 * cus && a.ntasks >= 4 * (int)g.x * kMVWaves) {
        a.split_wgs = cus;
        a.split_tasks = (int)(a.ntasks * (sh / (1.0 + sh)) + 0.5);
    }
    launch_k(k, g, dim3(kMVThreads), lds, s, true, true, a);
    return hipGetLastError();
}

// Two type groups (tasks [0, split) of type T, [split, ntasks) of type T2): the
// resident grid is dealt to the groups so that the largest per-wave byte count (tasks per
// wave rounded up x bytes per task) is smallest, >= 1 workgroup each.  Which wave reduces
// a task never changes a result.
static inline int split_groups(int wgs, int p1, int p2, double b1, double b2) {
    int best = 1;
    double best_cost = 1e300;
    for (int w1 = 1; w1 < wgs; ++w1) {
        const int n1 = w1 * kMVWaves, n2 = (wgs - w1) * kMVWaves;
        const double c = std::max((double)((p1 + n1 - 1) / n1) * b1, (double)((p2 + n2 - 1) / n2) * b2);
        if (c < best_cost) { best_cost = c; best = w1; }
    }
    return best;
}
template <int ACT, bool NORM, int T, int T2, int EPI, int NP, int X86>
static hipError_t mv_launch2(const MVArgs& a0, int split_tasks, dim3 grid, size_t lds_in, hipStream_t s) {
    const size_t lds = std::max(lds_in, mv_lds_total(ACT, a0.cols, kMVWaves, T, T2, X86));
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    auto k = k_matvec<ACT, NORM, EPI, T, NP, T2, kMVThreads, X86>;
    const dim3 g = resident_grid(k, grid, lds);
    MVArgs a = a0;
    a.split_tasks = split_tasks;
    int w1;
    if (g_split_by_pairs) {  // A/B: deal by task count
        w1 = (int)(((long long)g.x * split_tasks + a.ntasks / 2) / a.ntasks);
        w1 = w1 < 1 ? 1 : w1 > (int)g.x - 1 ? (int)g.x - 1 : w1;
    } else {
        w1 = split_groups((int)g.x, split_tasks, a.ntasks - split_tasks, (double)tensor_bytes(T, a.rpt, a.cols),
                          (double)tensor_bytes(T2, a.rpt, a.cols));
    }
    a.split_wgs = w1;
    launch_k(k, g, dim3(kMVThreads), lds, s, true, true, a);
    return hipGetLastError();
}

// prologue sub-blocks per thread held in registers: 1, 2 or 4
static inline int prologue_np(int cols) {
    const int per = (cols / 16 + kMVThreads - 1) / kMVThreads;
    return per <= 1 ? 1 : per <= 2 ? 2 : 4;
}

template <int ACT, bool NORM, int T, int EPI, int X86>
static hipError_t mv_launch_np(const MVArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (mv_try_wide<ACT, NORM, T, EPI, X86>(a, s, e)) return e;
    if (mv_try_narrow<ACT, NORM, T, EPI, X86>(a, s, e)) return e;
    switch (prologue_np(a.cols)) {
        case 1: return mv_launch<ACT, NORM, T, EPI, 1, X86>(a, grid, lds, s);
        case 2: return mv_launch<ACT, NORM, T, EPI, 2, X86>(a, grid, lds, s);
        default: return mv_launch<ACT, NORM, T, EPI, 4, X86>(a, grid, lds, s);
    }
}

// Instantiated (ACT, NORM, EPI) combinations: STORE and ADD with or without the fused
// RMSNorm; QKV, SWIGLU and LOGITS always take a normalised input.
template <int ACT, bool NORM, int T, int X86>
hipError_t mv_dispatch_epi(const MVArgs& a, int epi, dim3 grid, size_t lds, hipStream_t s) {
    switch (epi) {
        case EPI_STORE: return mv_launch_np<ACT, NORM, T, EPI_STORE, X86>(a, grid, lds, s);
        case EPI_ADD: return mv_launch_np<ACT, NORM, T, EPI_ADD, X86>(a, grid, lds, s);
        default: break;
    }
    if constexpr (NORM) {
        switch (epi) {
            case EPI_QKV: return mv_launch_np<ACT, NORM, T, EPI_QKV, X86>(a, grid, lds, s);
            case EPI_SWIGLU: return mv_launch_np<ACT, NORM, T, EPI_SWIGLU, X86>(a, grid, lds, s);
            case EPI_LOGITS: return mv_launch_np<ACT, NORM, T, EPI_LOGITS, X86>(a, grid, lds, s);
            default: break;
        }
    }
    return hipErrorInvalidValue;
}

// QKV whose q/k and v segments are two type groups: workgroup-split launch (k_matvec's
// T2 path), called from kernels.hip mv_dispatch_qkv2.
template <bool NORM, int T, int T2, int X86>
hipError_t mv_qkv2_launch(const MVArgs& a, int split_tasks, dim3 grid, size_t lds, hipStream_t s) {
    return mv_launch2<0, NORM, T, T2, EPI_QKV, 1, X86>(a, split_tasks, grid, lds, s);
}

}  // namespace llmi
