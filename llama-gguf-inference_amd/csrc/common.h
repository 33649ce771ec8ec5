// common.h — shared host/device definitions of the llmi decode path.
//
// Device weight layouts (DESIGN.md §Data layout in HBM).  Every quantized matrix is
// repacked once at load into a UNIT-MAJOR planar form.  A UNIT is 256 consecutive
// weights of a row (a K-quant block, or eight Q8_0 blocks); a row of `cols` weights has
// U = cols / 256 units.  Each unit's quant bytes are split into 16-B PARTS p, stored
// part-major per row:
//     A[row][p][unit][16 B]   (8 parts for K-quants, 16 for Q8_0)
// so lanes that hold consecutive units of a row read consecutive 16-B pieces (the
// matvec gives lane L unit L of its row, kernels.hip).  Per-unit headers / high bits
// live in their own planes, unit-major as well.  Byte counts equal GGUF exactly (the
// repack moves bytes, it never widens them):
//   Q4_K  A: qs 128 B/unit   S: header {d, dmin, scales[12]} 16 B/unit
//   Q5_K  A: qs 128 B/unit   H: [row][2][unit][16 B] fifth bits   S: header 16 B/unit
//   Q6_K  A: ql 128 B/unit   H: [row][4][unit][16 B] 2-bit highs (XOR 2)
//         S: scales 16 B/unit (native order)   D: fp16 d 2 B/unit
//   Q8_0  A: qs 256 B/unit (part p = 32-block p/2, half p%2)   D: 8 fp16 d = 16 B/unit
//   F32/F16 plain (A).
// K-quant parts are in RESIDUE ORDER: part p = 2c + k of chunk c (64 weights: low
// nibbles = weights 64c + t, high nibbles = 64c + 32 + t of native qs[32c + t]), byte
// 4m + i = native byte t = l + 8i with l = 4k + m: one dword holds the 8 weights of
// residue class l (element index mod 8) of the chunk — the grouping ggml's generic dot
// sums by (aux32[l], mv_device.h).  Q5_K fifth bits: 8 B per chunk (lo word: low-nibble
// weights, hi word: high-nibble weights; bit 4l + i as above), chunks 2h, 2h+1 in H
// part h.  Q6_K high bits: 16 B per chunk in H part c: dword 2*hi + k, byte i, bits 2m
// (XOR 2, so v_perm maps them to the signed high part of q - 32).
#pragma once

#include <cstddef>
#include <cstdint>

#include "../../include/llmi_synth.h"

namespace llmi {

enum : int {
    T_F32 = LLMI_T_F32, T_F16 = LLMI_T_F16, T_Q8_0 = LLMI_T_Q8_0,
    T_Q4_K = LLMI_T_Q4_K, T_Q5_K = LLMI_T_Q5_K, T_Q6_K = LLMI_T_Q6_K
};

inline int block_elems(int t) {
    switch (t) {
        case T_F32: case T_F16: return 1;
        case T_Q8_0: return 32;
        case T_Q4_K: case T_Q5_K: case T_Q6_K: return 256;
        default: return 0;
    }
}
inline int block_bytes(int t) {
    switch (t) {
        case T_F32: return 4; case T_F16: return 2; case T_Q8_0: return 34;
        case T_Q4_K: return 144; case T_Q5_K: return 176; case T_Q6_K: return 210;
        default: return 0;
    }
}
inline bool is_kquant(int t) { return t == T_Q4_K || t == T_Q5_K || t == T_Q6_K; }
inline bool type_supported(int t) { return block_bytes(t) != 0; }
inline const char* type_name(int t) {
    switch (t) {
        case T_F32: return "f32"; case T_F16: return "f16"; case T_Q8_0: return "q8_0";
        case T_Q4_K: return "q4_K"; case T_Q5_K: return "q5_K"; case T_Q6_K: return "q6_K";
        default: return "?";
    }
}
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
// bytes of a tensor in GGUF (== algorithmic bytes of its device layout)
inline size_t tensor_bytes(int t, int64_t rows, int64_t cols) {
    return (size_t)rows * (size_t)(cols / block_elems(t)) * (size_t)block_bytes(t);
}

// ROW GROUPS.  Rows are stored in groups of RG = 2^rgs consecutive rows; inside a group
// every part of the A and H planes holds the RG rows back to back, so 16-B piece
// (row, part p, unit u) of a plane with np parts per unit sits at
//     (((g np + p) RG + r) U + u) * 16      g = row / RG, r = row % RG
// (piece_off, mv_device.h).  RG is the matvec's rows per task at this width (kernels.hip
// mv_geometry: Lr = U lanes per row, R = 64 / Lr rows), so one wave load instruction of a
// task (R rows x U units of part p) reads R * U * 16 = 1 KiB of consecutive bytes, where
// the plain row-major form (RG = 1) gives R separate runs of U * 16 B.  The S and D planes
// are row-major per unit, which is already contiguous over a group.
inline int layout_rgs(int type, int64_t rows, int64_t cols) {
    if (!(type == T_Q4_K || type == T_Q5_K || type == T_Q6_K || type == T_Q8_0) || cols % 256) return 0;
    const int64_t U = cols / 256;
    int64_t lr = ((U < 64 ? U : 64) + 3) & ~(int64_t)3;
    if (lr < 4) lr = 4;
    int R = 1, s = 0;
    while (2 * R * lr <= 64) { R *= 2; ++s; }
    while (s > 0 && rows % R) { R >>= 1; --s; }
    return s;
}

// Placement of one matrix inside the device arena.
struct DevMat {
    int type = -1;
    int rgs = 0;                               // log2 of the row group (layout_rgs)
    int64_t rows = 0, cols = 0;
    size_t off_a = 0, off_h = 0, off_s = 0, off_d = 0;  // plane offsets (arena-relative)
    size_t bytes = 0;                          // algorithmic bytes
};

// plane layout of a matrix starting at arena offset `base`; returns end offset
inline size_t plan_planes(DevMat& m, size_t base) {
    const size_t nblk = (size_t)m.rows * (size_t)(m.cols / block_elems(m.type));
    m.bytes = tensor_bytes(m.type, m.rows, m.cols);
    m.rgs = layout_rgs(m.type, m.rows, m.cols);
    m.off_a = align_up(base, 256);
    m.off_h = m.off_s = m.off_d = m.off_a;
    switch (m.type) {
        case T_Q4_K:
            m.off_s = align_up(m.off_a + nblk * 128, 256);
            return m.off_s + nblk * 16;
        case T_Q5_K:
            m.off_h = align_up(m.off_a + nblk * 128, 256);
            m.off_s = align_up(m.off_h + nblk * 32, 256);
            return m.off_s + nblk * 16;
        case T_Q6_K:
            m.off_h = align_up(m.off_a + nblk * 128, 256);
            m.off_s = align_up(m.off_h + nblk * 64, 256);
            m.off_d = align_up(m.off_s + nblk * 16, 256);
            return m.off_d + nblk * 2;
        case T_Q8_0:
            m.off_d = align_up(m.off_a + nblk * 32, 256);
            return m.off_d + nblk * 2;
        default:
            return m.off_a + m.bytes;
    }
}
inline bool needs_repack(int t) { return t == T_Q4_K || t == T_Q5_K || t == T_Q6_K || t == T_Q8_0; }

// On-device decode state (one per context).  Step s at position p:
//   k_embed (every workgroup): p = pos_next; token = (token_in_pos == p) ? token_in
//           : argmax of key[(p-1)&1]; workgroup 0 publishes pos/token/hist[p] and
//           clears key[p&1];
//   logits kernel: each workgroup reduces its rows' argmax and atomicMax-es it into
//           slot blockIdx % kArgSlots of key[p&1] (spreading the atomics over 64
//           addresses: same-address atomics serialise at ~10 ns each); its workgroup 0
//           sets pos_next = p+1.  Consumers take the max over the slots.
// Every field is written by exactly one workgroup and never read by another workgroup
// of the same launch, so no intra-kernel synchronisation is needed.
struct StepState {
    int32_t token_in;        // host-provided token ...
    int32_t token_in_pos;    // ... valid for the step at this position (else greedy feedback)
    int32_t pos_next;        // position of the next step
    int32_t pos;             // position of the current step (written by k_embed)
    int32_t token;           // token of the current step
    uint32_t seq;            // step sequence number (k_embed increments; in-launch hand-off tags)
    unsigned long long key[2][64];  // per-parity argmax key slots: (ordered logit << 32) | (0xffffffff - row)
};
constexpr int kArgSlots = 64;
inline int key_token(const unsigned long long* slots) {  // host: token of a parity's slots
    unsigned long long k = 0;
    for (int i = 0; i < kArgSlots; ++i) k = slots[i] > k ? slots[i] : k;
    return (int)(0xffffffffu - (uint32_t)(k & 0xffffffffull));
}

}  // namespace llmi
