// leng.hip — the layer engine: one persistent launch per decode layer runs attn_output,
// ffn_gate+up, ffn_down and the next layer's QKV (DESIGN.md §4 "Layer engine";
// cdna_hip_programming.md §5.6, MI355X_MICROARCH.md price rows engine-vs-launches,
// prefetch-credit, handoff-flag).  The reference side is the NGL=99 decode step that
// /root/reference/scripts/start.sh:473-494 launches (llm_build_llama's per-layer
// mul_mat chain, upstream).
//
// Why: a batch-1 decode launch is a chain of latencies (dispatch ramp, activation
// fetch + quantization, the first weights arriving behind the chip-wide burst, the tail
// of late XCDs), so four launches per layer cost ~2x their streaming
// time.  Weights do not depend on activations: here every CU's weight slices of all four
// matvecs stream into an LDS ring from the start of the launch, and the activation edges
// between the matvecs become in-launch hand-offs that the stream runs ahead of.
//
// Workgroup = 576 threads, one per CU (grid = CU count, every workgroup resident):
//   waves 0, 1  LOADERS: both walk the CU's sub-items of every op in order; loader l moves
//               the weights of every sub-item n with n % 2 == l global -> LDS ring by
//               LDS-DMA (one 1-KiB piece per wave instruction, lane L's 16 B of its unit),
//               keeps its last kLeDepth sub-items in flight and publishes how many of its
//               sub-items have landed (ctl.ready[l]); a loader never waits on an
//               activation, only on ring space (ctl.cons[], what each consumer still
//               needs).  One loader wave issued 16 GB/s per CU, two 27 (tools/lestream.py)
//   waves 2..8  CONSUMERS: per op, wait for the op's input edge, build the q8 activation
//               image in LDS (RMSNorm + quantize_row_q8_K / q8_0, bit-exact, mv_device.h),
//               then reduce their own tasks' sub-items straight from the ring with
//               k_matvec's unit-term / fold / epilogue code (unit_terms, sub_finish):
//               the numerics of every row are exactly the separate kernels' 
// Tasks (mv_geometry's R rows of one op) are dealt to CUs by task % gridDim.x and inside a
// CU to consumer waves round-robin (rotated per op for balance).
//
// Edges (op k's output -> op k+1's input; every CU needs the whole vector): the producer
// waves store their rows write-through (sc1), each drains its stores (vmcnt(0)) and adds
// to an LDS counter; the last wave of the workgroup adds 1 to the edge's global counter
// shard blockIdx % 8 (agent-scope atomic).  One consumer wave polls the 8 shards (relaxed
// sc1 loads, s_sleep), then sets an LDS word for the others; every load of a handed-off
// vector is an sc1 load.  This is MI355X_MICROARCH.md §visibility's "Valid forms" row 1
// (sc1 stores / counter / sc1 loads, one workgroup per CU) — no acquire fence.  The
// counters are zeroed by a memset node at the start of every step (engine.cpp).
// Every spin is bounded: a timed-out wait ORs a code into the context's fault word, sets
// ctl.dead and every wave of the workgroup leaves (the host reports the step as failed).
#include "kernels.h"
#include "launch_util.h"
#include "mv_device.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace llmi {

namespace {

constexpr int kLeNL = 2;                  // loader waves (waves 0 .. kLeNL-1)
#ifndef LLMI_LE_C
#define LLMI_LE_C 7
#endif
constexpr int kLeC = LLMI_LE_C;           // consumer waves (waves kLeNL .. kLeNL+kLeC-1); experiment builds: -DLLMI_LE_C=n
static_assert(kLeC >= 1 && kLeC <= 14, "16 wave slots");
constexpr int kLeT = (kLeNL + kLeC) * 64;  // threads per workgroup
constexpr int kLeMaxPieces = 136;
constexpr int kLeTraceWaves = 16;          // trace layout [block][16 waves][32 stamps]
constexpr unsigned kLeFaultRing = 0x100u, kLeFaultEdge = 0x200u, kLeFaultBar = 0x400u, kLeFaultSpace = 0x800u;

// LDS control block (16-B aligned, at offset 0 of the dynamic LDS)
struct LeCtl {
    unsigned ready[2]; // loader l: its sub-items landed (monotonic)
    unsigned dead;     // a bounded wait gave up: every wave leaves
    unsigned bar;      // consumer-barrier arrivals
    unsigned edge;     // highest op whose input edge the poller wave has seen
    unsigned cons[16]; // consumer wave w: first ring piece it still needs (monotonic)
    unsigned done[4];  // per op: consumer waves whose stores have drained
    unsigned quiet;    // LLMI_LE_EXP & 4: the workgroup is between an op's end and the next image
    double red[16];    // RMSNorm partial sums, one per consumer wave
};

// ring pieces (1 KiB = 64 lanes x 16 B) of one sub-item: the A-plane parts, then the H
// parts, the S plane (Q8_0: the D plane's 16 B), Q6_K's d (4 B per lane)
__host__ __device__ constexpr int le_pieces(int t) {
    return t == T_Q4_K ? 9 : t == T_Q5_K ? 11 : t == T_Q6_K ? 14 : 17;
}

__device__ __forceinline__ unsigned lds_ld(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// timeline stamps (llmi_engine_trace; null trace: one uniform branch each)
#define LE_STAMP(I, V)                                                                                      \
    if (A.trace && (threadIdx.x & 63) == 0)                                                                 \
        A.trace[((size_t)blockIdx.x * kLeTraceWaves + (threadIdx.x >> 6)) * 32 + (I)] = (V);
#define LE_NOW __builtin_amdgcn_s_memrealtime()

__device__ __forceinline__ void le_fault(const LeArgs& A, LeCtl* ctl, unsigned code) {
    if ((threadIdx.x & 63) == 0) atomicOr(A.fault, code);
    lds_st(&ctl->dead, 1u);
}

// wait until *w >= tgt (an LDS word another wave of this workgroup sets)
__device__ __forceinline__ bool le_spin_lds(const LeArgs& A, LeCtl* ctl, const unsigned* w, unsigned tgt, unsigned code) {
    for (int n = 0;; ++n) {
        if (lds_ld(w) >= tgt) break;
        if (lds_ld(&ctl->dead)) return false;
        if (n >= A.spin_limit) {
            le_fault(A, ctl, code);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // later LDS reads stay behind the match
    return true;
}

// barrier of the 7 consumer waves (the loader never joins one): LDS arrival counter
__device__ __forceinline__ bool le_cbar(const LeArgs& A, LeCtl* ctl, int& barn) {
    ++barn;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes are done
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(&ctl->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return le_spin_lds(A, ctl, &ctl->bar, (unsigned)barn * kLeC, kLeFaultBar);
}

// ---- loaders ---------------------------------------------------------------------
// LDS-DMA in inline asm (cdna_hip_programming.md §5.7 item 1): the compiler neither counts
// it nor waits for it; the loader's own s_waitcnt vmcnt(N) publishes landed sub-items.
// Always nontemporal: streamed weights one CU reads once (MI355X_MICROARCH.md nt-weights).
__device__ __forceinline__ void le_dma16(const uint8_t* src, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ void le_dma4(const uint8_t* src, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void le_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// sub-items a loader keeps in flight past its published ones, by the launch's smallest
// sub-item (pieces): ~30 pieces per loader wave (vmcnt counts at most 63)
__host__ __device__ constexpr int le_depth(int kmin) { return kmin >= 14 ? 2 : 3; }
// wait until at most le_depth(kmin) x kmin of this wave's pieces are in flight: every
// sub-item of this loader but its last le_depth(kmin) has landed
__device__ __forceinline__ void le_vm_lag(int kmin) {
    switch (kmin) {
        case 9: le_vmcnt<9 * le_depth(9)>(); break;
        case 11: le_vmcnt<11 * le_depth(11)>(); break;
        case 14: le_vmcnt<14 * le_depth(14)>(); break;
        default: le_vmcnt<17 * le_depth(17)>(); break;
    }
}

// walk state of a loader (all wave-uniform).  Both loaders walk every sub-item (so both
// know every sub-item's ring position); each issues its own.
struct LeLoad {
    unsigned pieces = 0;   // ring pieces of all sub-items walked (both loaders')
    unsigned sn = 0;       // sub-items walked
    unsigned mine = 0;     // this loader's sub-items issued
    unsigned pub = 0;      // this loader's sub-items published
    unsigned lowest = 0;   // last seen min over consumers of ctl.cons
    uint32_t ring = 0;     // LDS address of the ring (uniform)
    unsigned long long waits = 0, wait_ticks = 0;  // ring-full waits (traced launches)
    unsigned long long vm_ticks = 0;                // time in the lag's vmcnt waits (traced launches)
};

__device__ __forceinline__ void le_publish(LeCtl* ctl, LeLoad& L, unsigned v, int l) {
    if (v > L.pub) {
        L.pub = v;
        asm volatile("" ::: "memory");
        lds_st(&ctl->ready[l], v);
    }
}

// room in the ring for pieces [p0, p0 + k)?  Waits (publishing everything of its own in
// flight first) until every consumer has released what the new pieces overwrite.  (A
// variant that published its in-flight sub-items one at a time while waiting, never
// draining the stream, measured slower: DESIGN.md §4 "Layer engine".)
__device__ __forceinline__ bool le_space(const LeArgs& A, LeCtl* ctl, LeLoad& L, unsigned p0, int k, int l) {
    const unsigned long long end = (unsigned long long)p0 + (unsigned)k, NP = (unsigned)A.npieces;
    if (end <= (unsigned long long)L.lowest + NP) return true;
    const unsigned long long t0 = A.trace ? LE_NOW : 0ull;
    le_vmcnt<0>();
    le_publish(ctl, L, L.mine, l);
    for (int n = 0;; ++n) {
        unsigned m = 0xffffffffu;
#pragma unroll
        for (int w = 0; w < kLeC; ++w) m = min(m, lds_ld(&ctl->cons[w]));
        L.lowest = m;
        if (end <= (unsigned long long)m + NP) {
            if (A.trace) {
                L.waits += 1;
                L.wait_ticks += LE_NOW - t0;
            }
            return true;
        }
        if (lds_ld(&ctl->dead)) return false;
        if (n >= A.spin_limit) {
            le_fault(A, ctl, kLeFaultSpace);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// one sub-item's pieces at ring piece p0, lane = (row r, unit ul) of the task as in k_matvec
template <int T>
__device__ __forceinline__ void le_issue(const Seg& sg, const LaneUnit& lu, uint32_t U, uint32_t ring, unsigned p0,
                                         unsigned NP) {
    unsigned pw = __builtin_amdgcn_readfirstlane(p0 % NP);
    auto slot = [&](int q) -> uint32_t {  // uniform: scalar arithmetic
        unsigned p = pw + (unsigned)q;
        if (p >= NP) p -= NP;
        return ring + p * 1024u;
    };
    constexpr int NPART = unit_parts<T>();
    const uint32_t P = (U * 16u) << sg.rgs, ru = lu.row * U + lu.u;
    const uint8_t* a = sg.a + piece_off(lu.row, 0, lu.u, U, NPART, sg.rgs);
#pragma unroll
    for (int q = 0; q < NPART; ++q) le_dma16(a + (size_t)q * P, slot(q));
    if constexpr (T == T_Q8_0) {
        le_dma16(sg.d + ru * 16u, slot(NPART));
    } else {
        constexpr int NH = (T == T_Q5_K || T == T_Q6_K) ? unit_hparts<T>() : 0;
        if constexpr (NH > 0) {
            const uint8_t* h = sg.h + piece_off(lu.row, 0, lu.u, U, NH, sg.rgs);
#pragma unroll
            for (int c = 0; c < NH; ++c) le_dma16(h + (size_t)c * P, slot(NPART + c));
        }
        le_dma16(sg.s + ru * 16u, slot(NPART + NH));
        if constexpr (T == T_Q6_K) le_dma4(sg.d + ((ru * 2u) & ~3u), slot(NPART + NH + 1));
    }
}

// A segment of an op by a wave-uniform index, read straight from the kernel arguments
// (scalar loads at a dynamic offset: lgkmcnt only).  Copying the segments into a local
// array and selecting from it made the compiler keep a private copy of the arguments and
// load the selected fields from scratch once per sub-item; the vmcnt(0) before their use
// drained the loader's whole DMA stream (ISA, round 6).
__device__ __forceinline__ Seg le_pick(const MVArgs& M, int si) {
    si = __builtin_amdgcn_readfirstlane(si);
    return M.seg[si];
}

template <int EPI>
__device__ __forceinline__ int le_task_pieces(const MVArgs& M, const TaskGeo& g, int task) {
    if constexpr (EPI == EPI_SWIGLU) return g.nj * (le_pieces(M.seg[0].type) + le_pieces(M.seg[1].type));
    else return g.nj * le_pieces(le_pick(M, sub_of<EPI>(M, g, task, 0).si).type);
}

template <int OP, int ACT, int EPI>
__device__ __forceinline__ bool le_load_op(const LeArgs& A, LeCtl* ctl, LeLoad& L, int l) {
    if (OP >= A.nops) return true;
    const MVArgs& M = A.op[OP];
    const TaskGeo g = task_geo(M);
    const int lane = threadIdx.x & 63, r = lane / g.lr, ul = lane - r * g.lr;
    const int S = EPI == EPI_SWIGLU ? 2 * g.nj : g.nj;
    const unsigned NP = (unsigned)A.npieces;
    LE_STAMP(1 + 2 * OP, LE_NOW)
    int cur = -1;  // segment held in registers (reloaded only when the sub-item's changes)
    Seg sg;
    for (int task = blockIdx.x; task < M.ntasks; task += gridDim.x) {
        for (int s = 0; s < S; ++s) {
            const Sub b = sub_of<EPI>(M, g, task, s);
            if (b.si != cur) {
                sg = le_pick(M, b.si);
                cur = b.si;
            }
            const int k = le_pieces(sg.type);
            const unsigned p0 = L.pieces;
            const bool own = (L.sn & (kLeNL - 1)) == (unsigned)l;
            L.pieces += (unsigned)k;
            ++L.sn;
            if (!own) continue;
            if (!le_space(A, ctl, L, p0, k, l)) return false;
            if (A.exp & 4) {  // experiment: no new weight DMA while the workgroup gathers an edge
                for (int n = 0; lds_ld(&ctl->quiet) && n < A.spin_limit; ++n) __builtin_amdgcn_s_sleep(1);
            }
            const LaneUnit lu = lane_unit(g, b, sg, r, ul);
            if constexpr (ACT == 1) {
                le_issue<T_Q8_0>(sg, lu, (uint32_t)g.U, L.ring, p0, NP);
            } else {
                switch (sg.type) {
                    case T_Q4_K: le_issue<T_Q4_K>(sg, lu, (uint32_t)g.U, L.ring, p0, NP); break;
                    case T_Q5_K: le_issue<T_Q5_K>(sg, lu, (uint32_t)g.U, L.ring, p0, NP); break;
                    default: le_issue<T_Q6_K>(sg, lu, (uint32_t)g.U, L.ring, p0, NP); break;
                }
            }
            ++L.mine;
            const unsigned long long tv = A.trace ? LE_NOW : 0ull;
            le_vm_lag(A.kmin);
            if (A.trace) L.vm_ticks += LE_NOW - tv;
            const unsigned depth = (unsigned)le_depth(A.kmin);
            if (L.mine > depth) le_publish(ctl, L, L.mine - depth, l);
        }
    }
    LE_STAMP(2 + 2 * OP, LE_NOW)
    LE_STAMP(14 + 2 * OP, L.vm_ticks)
    LE_STAMP(15 + 2 * OP, L.wait_ticks)
    return true;
}

template <int ACT>
__device__ __forceinline__ void le_loader(const LeArgs& A, LeCtl* ctl, uint8_t* ring, int l) {
    LeLoad L;
    L.ring = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)ring);
    bool ok = le_load_op<0, ACT, EPI_ADD>(A, ctl, L, l) && le_load_op<1, ACT, EPI_SWIGLU>(A, ctl, L, l) &&
              le_load_op<2, ACT, EPI_ADD>(A, ctl, L, l) && le_load_op<3, ACT, EPI_QKV>(A, ctl, L, l);
    le_vmcnt<0>();  // no LDS-DMA may land after the workgroup's LDS is released
    if (ok) le_publish(ctl, L, L.mine, l);
    LE_STAMP(9, LE_NOW)
    LE_STAMP(10, L.waits)
    LE_STAMP(11, L.wait_ticks)
    LE_STAMP(12, L.mine)
    LE_STAMP(13, ((unsigned long long)(__builtin_amdgcn_s_getreg(6164) & 15)))
}

// ---- consumers ---------------------------------------------------------------------
template <int T>
__device__ __forceinline__ UnitW<T> le_ring_unit(const uint8_t* ring, unsigned pw, int NP, int lane, uint32_t ru) {
    UnitW<T> w;
    auto piece = [&](int q) -> const uint8_t* {
        unsigned p = pw + (unsigned)q;
        if (p >= (unsigned)NP) p -= (unsigned)NP;
        return ring + (size_t)p * 1024;
    };
    constexpr int NPART = unit_parts<T>();
#pragma unroll
    for (int q = 0; q < NPART; ++q) w.q[q] = *(const u32x4*)(piece(q) + 16 * lane);
    if constexpr (T == T_Q8_0) {
        w.s = *(const u32x4*)(piece(NPART) + 16 * lane);
    } else {
        constexpr int NH = (T == T_Q5_K || T == T_Q6_K) ? unit_hparts<T>() : 0;
        if constexpr (NH > 0) {
#pragma unroll
            for (int c = 0; c < NH; ++c) w.h[c] = *(const u32x4*)(piece(NPART + c) + 16 * lane);
        }
        w.s = *(const u32x4*)(piece(NPART + NH) + 16 * lane);
        if constexpr (T == T_Q6_K) w.d = *(const uint32_t*)(piece(NPART + NH + 1) + 4 * lane) >> (16 * (ru & 1u));
    }
    return w;
}

// the activation image of an op: all 7 consumer waves, the input read with sc1 loads
// (it may have been written by another CU in this launch); the RMSNorm double sum is
// per-thread partials -> wave butterfly -> a fixed tree over the 7 waves, exact under
// any association as in k_matvec's prologue
typedef unsigned long long __attribute__((address_space(1))) le_gu64;
template <int ACT, bool NORM, int X86>
__device__ __forceinline__ bool le_image(const LeArgs& A, const MVArgs& M, uint8_t* img, LeCtl* ctl, int cw, int& barn) {
    constexpr int NTc = kLeC * 64, NR = 4;
    const int ct = (int)threadIdx.x - 64 * kLeNL, cols = M.cols, nsub = cols >> 4;
    const int lane = threadIdx.x & 63;
    Lds L;
    L.act = img;
    L.red = nullptr;
    float v[NR][16];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int sb = ct + NTc * i;
#pragma unroll
        for (int j = 0; j < 16; ++j) v[i][j] = 0.f;
        if (sb < nsub) {
            const le_gu64* src = (const le_gu64*)(M.x + (size_t)sb * 16);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const unsigned long long u = __hip_atomic_load(src + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v[i][2 * m] = __uint_as_float((uint32_t)u);
                v[i][2 * m + 1] = __uint_as_float((uint32_t)(u >> 32));
            }
        }
    }
    float scale = 1.0f;
    if constexpr (NORM) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NR; ++i)
            if (ct + NTc * i < nsub) {
#pragma unroll
                for (int j = 0; j < 16; ++j) s += (double)(v[i][j] * v[i][j]);
            }
        s = wave_sum_d(s);
        if (lane == 0) ctl->red[cw] = s;
        if (!le_cbar(A, ctl, barn)) return false;
        double r[kLeC];
#pragma unroll
        for (int w = 0; w < kLeC; ++w) r[w] = ctl->red[w];
        double t;
        if constexpr (kLeC == 7) {
            t = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + r[6]);
        } else {
            t = r[0];
#pragma unroll
            for (int w = 1; w < kLeC; ++w) t += r[w];
        }
        const float mean = (float)(t / (double)cols);
        scale = 1.0f / sqrtf(mean + M.eps);
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int sb = ct + NTc * i;
        if (sb < nsub) {
            float y[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) y[j] = v[i][j];
            if constexpr (NORM) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 wv = *(const float4*)(M.nw + sb * 16 + 4 * k);
                    y[4 * k] = (y[4 * k] * scale) * wv.x;
                    y[4 * k + 1] = (y[4 * k + 1] * scale) * wv.y;
                    y[4 * k + 2] = (y[4 * k + 2] * scale) * wv.z;
                    y[4 * k + 3] = (y[4 * k + 3] * scale) * wv.w;
                }
            }
            quant_sub<ACT, X86>(L, cols, sb, y);
        }
    }
    return le_cbar(A, ctl, barn);
}

// op OP's input edge: op OP-1's output from every CU
template <int OP>
__device__ __forceinline__ bool le_edge(const LeArgs& A, LeCtl* ctl, int cw) {
    if (cw == 0) {
        const int lane = threadIdx.x & 63, j = lane & 7, NB = gridDim.x;
        const unsigned tgt = (unsigned)(NB / 8 + (j < (NB & 7) ? 1 : 0));
        const gu32_t* c = (const gu32_t*)(A.cnt + (size_t)j * A.cnt_stride + (OP - 1) * 16);
        for (int n = 0;; ++n) {
            const unsigned v = lane < 8 ? __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0xffffffffu;
            if (__all(v >= tgt)) {
                LE_STAMP(27 + OP, (unsigned long long)n + 1)
                break;
            }
            if (lds_ld(&ctl->dead)) return false;
            if (n >= (A.spin_limit >> 3)) {  // a global poll takes ~8x an LDS poll
                le_fault(A, ctl, kLeFaultEdge);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("" ::: "memory");
        lds_st(&ctl->edge, (unsigned)OP);
        return true;
    }
    return le_spin_lds(A, ctl, &ctl->edge, (unsigned)OP, kLeFaultEdge);
}

template <int T, int ACT, int EPI, bool WT, int X86>
__device__ __forceinline__ void le_sub(const MVArgs& M, LeCtl* ctl, const uint8_t* ring, unsigned pw, int NP,
                                       const uint8_t* img, float* F, const TaskGeo& g, int s, const Sub& sb, const Seg& sg,
                                       int r, int ul, unsigned bend, int cw, float& acc, float& vg, int pos, float2 pre) {
    const int lane = threadIdx.x & 63;
    const LaneUnit lu = lane_unit(g, sb, sg, r, ul);
    const UnitW<T> w = le_ring_unit<T>(ring, pw, NP, lane, lu.row * (uint32_t)g.U + lu.u);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the pieces are in registers ...
    lds_st(&ctl->cons[cw], bend);                      // ... and free for the loader
    float tm[9];
    if constexpr (X86) unit_store_x86<T>(w, img + (size_t)lu.u * kRec, F, r, ul, g.lr, g.R, lu.valid);
    else unit_terms<T>(w, img + (size_t)lu.u * kRec, tm);
    unsigned long long best = 0;
    sub_finish<ACT, EPI, MVArgs, X86, WT, EPI == EPI_ADD || EPI == EPI_QKV>(M, F, g, s, sb, sg, tm, lu, r, ul, acc, vg,
                                                                           pos, best, pre);
}

// ring position of the consumers' walk (identical in every consumer wave)
struct LeWalk {
    unsigned base = 0;  // first piece of the current op
    unsigned sn = 0;    // first sub-item of the current op (loader (sn % kLeNL) issues it)
    int rot = 0;        // task-to-wave rotation of the current op
    int barn = 0;       // consumer barriers passed
};

template <int OP, int ACT, int EPI, bool NORM, bool WT, int X86>
__device__ __forceinline__ bool le_cons_op(const LeArgs& A, LeCtl* ctl, uint8_t* ring, uint8_t* img, float* F, int cw,
                                           LeWalk& W) {
    if (OP >= A.nops) return true;
    const MVArgs& M = A.op[OP];
    const TaskGeo g = task_geo(M);
    const int lane = threadIdx.x & 63, r = lane / g.lr, ul = lane - r * g.lr;
    const int S = EPI == EPI_SWIGLU ? 2 * g.nj : g.nj;
    const int NB = gridDim.x, NP = A.npieces;
    // 0. tell the loader where this wave's first sub-item of the op starts (or that it
    //    needs nothing of this op): the stream runs ahead across the edge below
    {
        unsigned b = W.base;
        int i = 0;
        for (int task = blockIdx.x; task < M.ntasks; task += NB, ++i) {
            if ((i + W.rot) % kLeC == cw) break;
            b += (unsigned)le_task_pieces<EPI>(M, g, task);
        }
        lds_st(&ctl->cons[cw], b);
    }
    // 1. input edge (op 0's input comes from the previous launch)
    if constexpr (OP > 0)
        if (!(A.exp & 2) && !le_edge<OP>(A, ctl, cw)) return false;
    LE_STAMP(1 + 4 * OP, LE_NOW)
    // 2. activation image
    if (!(A.exp & 2) && !le_image<ACT, NORM, X86>(A, M, img, ctl, cw, W.barn)) return false;
    if ((A.exp & 4) && cw == 0) lds_st(&ctl->quiet, 0u);
    LE_STAMP(2 + 4 * OP, LE_NOW)
    bool first_sub = true;
    unsigned long long ring_ticks = 0;
    // 3. this wave's tasks, straight from the ring
    int pos = 0;
    if constexpr (EPI == EPI_QKV) pos = M.st->pos;
    unsigned b = W.base, sn = W.sn;
    unsigned pw = W.base % (unsigned)NP;
    int i = 0;
    for (int task = blockIdx.x; task < M.ntasks; task += NB, ++i) {
        if ((i + W.rot) % kLeC != cw) {
            const unsigned n = (unsigned)le_task_pieces<EPI>(M, g, task);
            b += n;
            pw = (pw + n) % (unsigned)NP;
            sn += (unsigned)S;
            continue;
        }
        float acc = 0.f, vg = 0.f;
        // the epilogue's dependent load (residual / RoPE pair) issued now, before the ring
        // wait and the reduction, instead of behind the weight stream at the task's end
        float2 pre = float2{0.f, 0.f};
        if constexpr (EPI == EPI_ADD || EPI == EPI_QKV) {
            const Sub b0 = sub_of<EPI>(M, g, task, 0);
            const Seg s0 = le_pick(M, b0.si);
            const int row = b0.row0 + lane;
            if (lane < g.R && row < s0.rows) {
                if constexpr (EPI == EPI_ADD) {
                    pre.x = ld_f32<true>(M.y + s0.row0 + row);
                } else {
                    const int hd = M.head_dim, d = row - (row / hd) * hd;
                    if ((lane & 1) == 0 && s0.row0 < M.nq + M.nk && d < M.n_rot)
                        pre = *(const float2*)(M.rope + ((size_t)pos * (M.n_rot / 2) + d / 2) * 2);
                }
            }
        }
        for (int s = 0; s < S; ++s) {
            const Sub sb = sub_of<EPI>(M, g, task, s);
            const Seg sg = le_pick(M, sb.si);
            const unsigned k = (unsigned)le_pieces(sg.type);
            lds_st(&ctl->cons[cw], b);
            const unsigned long long tw = A.trace ? LE_NOW : 0ull;
            if (!le_spin_lds(A, ctl, &ctl->ready[sn & (kLeNL - 1)], sn / kLeNL + 1, kLeFaultRing)) return false;
            if (A.trace) {
                const unsigned long long tn = LE_NOW;
                ring_ticks += tn - tw;
                if (first_sub) { LE_STAMP(3 + 4 * OP, tn) }
                first_sub = false;
            }
            if (A.exp & 1) {  // experiment: release the pieces unread (results garbage)
                lds_st(&ctl->cons[cw], b + k);
            } else if constexpr (ACT == 1) {
                le_sub<T_Q8_0, ACT, EPI, WT, X86>(M, ctl, ring, pw, NP, img, F, g, s, sb, sg, r, ul, b + k, cw, acc, vg, pos, pre);
            } else {
                switch (sg.type) {
                    case T_Q4_K: le_sub<T_Q4_K, ACT, EPI, WT, X86>(M, ctl, ring, pw, NP, img, F, g, s, sb, sg, r, ul, b + k, cw, acc, vg, pos, pre); break;
                    case T_Q5_K: le_sub<T_Q5_K, ACT, EPI, WT, X86>(M, ctl, ring, pw, NP, img, F, g, s, sb, sg, r, ul, b + k, cw, acc, vg, pos, pre); break;
                    default: le_sub<T_Q6_K, ACT, EPI, WT, X86>(M, ctl, ring, pw, NP, img, F, g, s, sb, sg, r, ul, b + k, cw, acc, vg, pos, pre); break;
                }
            }
            b += k;
            pw = (pw + k) % (unsigned)NP;
            ++sn;
        }
    }
    lds_st(&ctl->cons[cw], b);
    LE_STAMP(4 + 4 * OP, LE_NOW)
    LE_STAMP(20 + OP, ring_ticks)
    W.base = b;
    W.sn = sn;
    W.rot = (W.rot + i) % kLeC;
    // 4. hand the op's output on: every wave drains its write-through stores, the last
    //    wave of the workgroup adds to the edge counter (the last op's output is read by
    //    the next launch)
    if (OP + 1 < A.nops) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        LE_STAMP(24 + OP, LE_NOW)
        if (lane == 0) {
            const unsigned old = __hip_atomic_fetch_add(&ctl->done[OP], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == kLeC - 1) {
                if (A.exp & 4) lds_st(&ctl->quiet, 1u);
                __hip_atomic_fetch_add((gu32_t*)(A.cnt + (size_t)(blockIdx.x & 7) * A.cnt_stride + OP * 16), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    return true;
}

template <int ACT, int X86>
__global__ __launch_bounds__(kLeT, 1) void k_leng(LeArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    LeCtl* ctl = (LeCtl*)smem;
    uint8_t* ring = smem + A.ring_off;
    const int wave = uniform((int)(threadIdx.x >> 6));
    // a fault of an earlier launch (this step's outputs are already invalid): leave at once,
    // so a failed hand-off costs one bounded wait per step, not one per layer
    if (__hip_atomic_load(A.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    LE_STAMP(0, LE_NOW)
    if (threadIdx.x < sizeof(LeCtl) / 4) ((unsigned*)smem)[threadIdx.x] = 0u;
    __syncthreads();  // the only full-workgroup barrier
    if (wave < kLeNL) {
        le_loader<ACT>(A, ctl, ring, wave);
        return;
    }
    const int cw = wave - kLeNL;
    float* F = (float*)(smem + A.fold_off) + (size_t)cw * fold_floats<ACT, X86>();
    uint8_t* img0 = smem + A.img_off0;
    uint8_t* img1 = smem + A.img_off1;
    LeWalk W;
    if (!le_cons_op<0, ACT, EPI_ADD, false, true, X86>(A, ctl, ring, img0, F, cw, W)) return;
    if (!le_cons_op<1, ACT, EPI_SWIGLU, true, true, X86>(A, ctl, ring, img1, F, cw, W)) return;
    if (!le_cons_op<2, ACT, EPI_ADD, false, true, X86>(A, ctl, ring, img0, F, cw, W)) return;
    if (!le_cons_op<3, ACT, EPI_QKV, true, false, X86>(A, ctl, ring, img1, F, cw, W)) return;
    lds_st(&ctl->cons[cw], 0xffffffffu);
    LE_STAMP(17, LE_NOW)
}

}  // namespace

// Edge counters: 8 shards (one per XCD under round-robin dispatch: blockIdx % 8), each a
// block [layers][kLeOps][16 words] (64 B per counter); the shards of one counter lie
// le_counter_stride() words apart (>= 8 KiB) so their 32 arrivals each and the 256
// pollers' loads spread over memory channels instead of serialising on one or two lines
// (MI355X_MICROARCH.md fanin: ~12 ns per atomic on one counter).
size_t le_counter_stride(int n_layer) { return (size_t)std::max(n_layer, 32) * kLeOps * 16; }
size_t le_counter_bytes(int n_layer) { return 8 * le_counter_stride(n_layer) * 4; }

// the engine's op order and epilogues: attn_output + residual, gate/up + SwiGLU, down +
// residual, the next layer's QKV + RoPE + KV write
static const int kLeEpi[kLeOps] = {EPI_ADD, EPI_SWIGLU, EPI_ADD, EPI_QKV};

int g_le_on = [] {  // LLMI_ENGINE: 1 layer engine, 0 separate launches (the default until it is faster)
    const char* e = getenv("LLMI_ENGINE");
    return e ? atoi(e) : 0;
}();
int g_le_spin = 1 << 20;
int g_le_exp = [] {  // LLMI_LE_EXP (experiments): 1 consumers skip the math, 2 skip edges + images (both: results
                     // garbage), 4 loaders issue nothing while the workgroup gathers an edge (results exact)
    const char* e = getenv("LLMI_LE_EXP");
    return e ? atoi(e) : 0;
}();
bool le_wanted() { return g_le_on != 0; }

static hipError_t le_kernel(int act, int x86, const void** k) {
    *k = act ? (x86 ? (const void*)k_leng<1, 1> : (const void*)k_leng<1, 0>)
             : (x86 ? (const void*)k_leng<0, 1> : (const void*)k_leng<0, 0>);
    return hipSuccess;
}

hipError_t layer_engine_prepare(LeArgs& a) {
    if (a.nops < 1 || a.nops > kLeOps || !a.cnt || !a.fault) return hipErrorInvalidValue;
    int act = -1, maxp = 0, kmin = 99;
    size_t img[2] = {0, 0};
    const int x86 = a.op[0].num ? 1 : 0;
    for (int k = 0; k < a.nops; ++k) {
        MVArgs& m = a.op[k];
        if (m.cols < 256 || m.cols % 256 || m.cols > 16 * 4 * kLeC * 64) return hipErrorNotSupported;
        if (!mv_geometry(m, kLeEpi[k])) return hipErrorNotSupported;
        if ((m.num ? 1 : 0) != x86) return hipErrorInvalidValue;
        for (int i = 0; i < m.nseg; ++i) {
            const int t = m.seg[i].type;
            if (t != T_Q4_K && t != T_Q5_K && t != T_Q6_K && t != T_Q8_0) return hipErrorNotSupported;
            if (act >= 0 && act_kind(t) != act) return hipErrorNotSupported;
            act = act_kind(t);
            if ((m.seg[i].x86 != 0) != (x86 != 0)) return hipErrorInvalidValue;
            maxp = std::max(maxp, le_pieces(t));
            kmin = std::min(kmin, le_pieces(t));
        }
        img[k & 1] = std::max(img[k & 1], (size_t)(m.cols >> 8) * kRec);
    }
    if (x86 && act == 1) return hipErrorNotSupported;  // 7 x 18.5 KB of Q8_0 x86 fold buffers
    const size_t fold = (size_t)kLeC * (x86 ? (size_t)fold_floats<0, 1>() : (size_t)kFoldFloats) * 4;
    size_t off = a16(sizeof(LeCtl));
    a.img_off0 = (int)off;
    off = a16(off + img[0]);
    a.img_off1 = (int)off;
    off = a16(off + img[1]);
    a.fold_off = (int)off;
    off = a16(off + fold);
    a.ring_off = (int)off;
    const int np = std::min(kLeMaxPieces, (int)((160 * 1024 - (int)off) / 1024));
    if (np < 2 * kLeNL * maxp) return hipErrorNotSupported;
    a.npieces = np;
    a.act = act;
    if (a.spin_limit <= 0) a.spin_limit = g_le_spin;
    a.exp = g_le_exp;
    a.kmin = kmin;
    if (cu_count() < 8) return hipErrorNotSupported;
    // every workgroup must be resident at once (persistent grid): one per CU by LDS, and
    // the occupancy query must admit one (cached per kernel, LDS bytes and device)
    const void* kern = nullptr;
    le_kernel(act, x86, &kern);
    const size_t lds = (size_t)a.ring_off + (size_t)np * 1024;
    static std::mutex mu;
    static std::map<std::tuple<const void*, size_t, int>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(kern, lds, dev);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it == cache.end()) {
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kLeT, lds) != hipSuccess) occ = 0;
        it = cache.emplace(key, occ).first;
    }
    return it->second >= 1 ? hipSuccess : hipErrorNotSupported;
}

hipError_t launch_layer_engine(const LeArgs& a, hipStream_t s) {
    if (a.npieces <= 0 || a.act < 0) return hipErrorInvalidValue;  // layer_engine_prepare first
    const size_t lds = (size_t)a.ring_off + (size_t)a.npieces * 1024;
    const int x86 = a.op[0].num ? 1 : 0;
    const dim3 grid(cu_count()), block(kLeT);
    if (a.act) {
        if (x86) launch_k(k_leng<1, 1>, grid, block, lds, s, true, true, a);
        else launch_k(k_leng<1, 0>, grid, block, lds, s, true, true, a);
    } else {
        if (x86) launch_k(k_leng<0, 1>, grid, block, lds, s, true, true, a);
        else launch_k(k_leng<0, 0>, grid, block, lds, s, true, true, a);
    }
    return hipGetLastError();
}

}  // namespace llmi

// ---- LDS-DMA stream microbenchmark (llmi_le_stream_bench; DESIGN.md §4 "Layer engine") ----
namespace llmi {
namespace {
// every CU streams its contiguous share of `src` in 1-KiB pieces (lane L: bytes 16 L..)
//   mode 0: one loader wave, asm LDS-DMA with M0 saved / restored (the engine's le_dma16, always nt)
//   mode 1: one loader wave, __builtin_amdgcn_global_load_lds (compiler-managed M0)
//   mode 2 / 3: two / four loader waves (asm), pieces dealt round-robin
//   mode 4: eight waves of plain 16-B loads into registers, 8 in flight per wave (k_matvec's form)
template <int MODE>
__global__ __launch_bounds__(512, 1) void k_le_stream(const uint8_t* src, size_t per_cu, unsigned* sink, int nt) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = uniform((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const uint8_t* base = src + per_cu * blockIdx.x;
    const unsigned npc = (unsigned)(per_cu >> 10);
    if constexpr (MODE == 4) {
        u32x4 acc = {0u, 0u, 0u, 0u};
        for (unsigned p = (unsigned)wave; p < npc; p += 8 * 8) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const unsigned q = min(p + 8u * k, npc - 1);
                v[k] = __builtin_nontemporal_load((const u32x4*)(base + (size_t)q * 1024 + 16 * lane));
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= v[k];
        }
        if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = 1u;
        return;
    }
    constexpr int NL = MODE == 2 ? 2 : MODE == 3 ? 4 : 1;
    if (wave >= NL) return;
    const uint32_t ring = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)smem;
    unsigned slot = (unsigned)wave;
    int n = 0;
    for (unsigned p = (unsigned)wave; p < npc; p += NL) {
        const uint8_t* g = base + (size_t)p * 1024 + 16 * lane;
        const uint32_t l = __builtin_amdgcn_readfirstlane(ring + slot * 1024u);
        if constexpr (MODE == 1) {
            if (nt)
                __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                                 (void __attribute__((address_space(3)))*)(size_t)l, 16, 0, 2);
            else
                __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                                 (void __attribute__((address_space(3)))*)(size_t)l, 16, 0, 0);
        } else {
            le_dma16(g, l);
        }
        slot += NL;
        if (slot >= 128) slot -= 128;
        if (++n == 8) {
            n = 0;
            le_vmcnt<40>();
        }
    }
    le_vmcnt<0>();
}
}  // namespace

// bytes streamed per second (GB/s) of `iters` launches over `bytes` of device memory
double le_stream_bench(const void* src, size_t bytes, int mode, int iters, int nt) {
    const int cus = cu_count();
    if (cus <= 0 || iters <= 0) return -1;
    const size_t per_cu = (bytes / cus) & ~(size_t)1023;
    unsigned* sink = nullptr;
    if (hipMalloc(&sink, 16) != hipSuccess) return -1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&] {
        const uint8_t* s = (const uint8_t*)src;
        switch (mode) {
            case 0: hipLaunchKernelGGL(k_le_stream<0>, dim3(cus), dim3(512), 128 * 1024, 0, s, per_cu, sink, nt); break;
            case 1: hipLaunchKernelGGL(k_le_stream<1>, dim3(cus), dim3(512), 128 * 1024, 0, s, per_cu, sink, nt); break;
            case 2: hipLaunchKernelGGL(k_le_stream<2>, dim3(cus), dim3(512), 128 * 1024, 0, s, per_cu, sink, nt); break;
            case 3: hipLaunchKernelGGL(k_le_stream<3>, dim3(cus), dim3(512), 128 * 1024, 0, s, per_cu, sink, nt); break;
            default: hipLaunchKernelGGL(k_le_stream<4>, dim3(cus), dim3(512), 128 * 1024, 0, s, per_cu, sink, nt); break;
        }
    };
    run();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) run();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(sink);
    return ms > 0 ? (double)per_cu * cus * iters / (ms * 1e-3) / 1e9 : -1;
}
}  // namespace llmi
