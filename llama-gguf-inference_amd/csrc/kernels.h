// kernels.h — launch interface of the gfx950 decode kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "common.h"

namespace llmi {

#ifndef LLMI_MV_THREADS
#define LLMI_MV_THREADS 256
#endif
constexpr int kMVThreads = LLMI_MV_THREADS;  // matvec workgroup; each wave owns one row task at a time
constexpr int kMVWaves = kMVThreads / 64;
constexpr int kFusedAttnMaxKV = 8192;  // fused one-launch attention up to this KV bound (LDS scores)
constexpr size_t kSplitAttnMaxLds = 128 * 1024;  // split attention: G * kv_bound f32 probabilities in LDS
constexpr int kXAttnMaxKV = 1024;
constexpr int kDimAttnMaxKV = 1024;  // dim-split one-launch attention (k_attn_d) up to this KV bound
constexpr int kRegAttnMaxKV = 512;  // register-prefetched one-launch attention (k_attn_r) up to this KV bound  // one-launch exchange attention (k_attn_x) up to this KV bound
constexpr int kPfAttnMaxKV = 32768;  // batched-prefill attention: scores of one head in LDS
// test options (llmi_test_option in capi.cpp): bit-identical path selection and lowered limits
extern int g_pf_fa_noalloc, g_pf_gemm_ng, g_pf_qkv_merge, g_pf_xcd_map, g_pf_quant_bpc, g_pf_quant_split_below, g_pf_attn_simple, g_pf_attn_fa, g_pf_fa_cfg, g_pf_max_kv, g_xspin_limit, g_xtag_skew;
int pf_max_kv();  // llama_decode hands prompt runs reaching past this KV length to decode steps
// scratch floats an attention context needs: scores [H][n_ctx] + tile maxima [H][n_ctx/32]
// + k_attn_x's 8-byte {tag, score} granules [H][kXAttnMaxKV] + a fault word
__host__ __device__ inline size_t attn_gran_off(int n_head, int n_ctx) {
    return ((size_t)n_head * n_ctx + (size_t)n_head * (n_ctx / 32 + 1) + 3) & ~(size_t)3;
}
// + the long-context path's (k_attl_*) per-256-position tile sums [H][n_ctx/256] and PV
// partials [H][n_ctx/256][<= 128 dims], both double
constexpr int kLongTile = 256;
__host__ __device__ inline size_t attn_long_off(int n_head, int n_ctx) { return attn_gran_off(n_head, n_ctx) + 2 * (size_t)n_head * kXAttnMaxKV + 4; }
inline size_t attn_scratch_floats(int n_head, int n_ctx) {
    return attn_long_off(n_head, n_ctx) + 2 * (size_t)n_head * ((n_ctx + kLongTile - 1) / kLongTile) * 129;
}

enum Epi : int { EPI_STORE = 0, EPI_ADD = 1, EPI_QKV = 2, EPI_SWIGLU = 3, EPI_LOGITS = 4,
                 EPI_SWIGLU_UP = 5 };  // prefill: y = silu(y) * up (gate/up of different types)

// One weight matrix of a fused matvec launch.
struct Seg {
    const uint8_t* a = nullptr;  // plane A: quants in piece order
    const uint8_t* h = nullptr;  // plane H: Q5_K fifth bits / Q6_K 2-bit highs
    const uint8_t* s = nullptr;  // plane S: Q4_K/Q5_K headers, Q6_K scales
    const uint8_t* d = nullptr;  // plane D: Q6_K / Q8_0 fp16 d
    int type = -1;
    int rows = 0;
    int row0 = 0;                // first row of this segment in the launch's output space
    int rgs = 0;                 // log2 of the row group of the A / H planes (common.h)
    int x86 = 0;                 // 1: the x86-numerics byte order of the A / H planes (common.h)
};

struct MVArgs {
    Seg seg[3];
    int nseg = 0;
    int cols = 0;
    int npairs = 0;              // row pairs (SWIGLU: gate/up pairs) — sizes the launch
    const float* x = nullptr;    // f32[cols] input
    const float* nw = nullptr;   // RMSNorm weight (nullptr: quantize x as is)
    const uint8_t* xq = nullptr; // pre-quantized activation image [cols/256][kRec] (mv_device.h):
                                 // when set, the prologue copies it into LDS instead of
                                 // normalising and quantizing x
    float eps = 0.f;
    float* y = nullptr;          // STORE/ADD/LOGITS: f32[rows]; SWIGLU: h; QKV: q
    // QKV epilogue: RoPE + f16 KV-cache write
    uint16_t* kc = nullptr;      // layer K cache [HK][n_ctx][D]
    uint16_t* vc = nullptr;      // layer V cache, transposed [HK][D][n_ctx]
    const float* rope = nullptr; // [n_ctx][n_rot/2][cos,sin]
    StepState* st = nullptr;     // QKV reads pos; LOGITS reads pos and advances pos_next
    int head_dim = 0, n_rot = 0, n_ctx = 0, nq = 0, nk = 0;
    unsigned long long* argmax = nullptr;  // LOGITS
    unsigned long long* trace = nullptr;   // LLMI_EXP_TRACE builds: per-wave s_memrealtime stamps
    // row tasks (mv_device.h; set by launch_matvec / launch_mvn from the segments)
    int lr = 0;                            // lanes per row (a multiple of 4)
    int rpt = 0;                           // rows per task R (SwiGLU: gate/up pairs)
    int ntasks = 0;
    int split_tasks = 0;                   // two-type launches: tasks of the first type group ...
    int split_wgs = 0;                     // ... and the workgroups that run them
    int xfirst = 0;                        // experiment: 1 multi-round launches also wait for x before weights, -1 none does
    int fw = 0;                            // 1: a wave's second sub-item is issued only once its first has landed (LLMI_MV_FW)
    int prio_alt = 0;                      // experiment builds: alternate s_setprio per sub-item (blocks >= prio_alt: other phase)
    // batched decode (batch.hip, k_mvn): token t of the batch is one decode step of
    // sequence tseq[t] at position tpos[t]; x / y rows are x_stride / y_stride floats
    // apart; the sequence's KV cache is kv_stride elements past the first one; LOGITS
    // uses the sequence's StepState (st + tseq[t]) for its argmax slots
    int x_stride = 0, y_stride = 0;
    const int* tpos = nullptr;
    const int* tseq = nullptr;
    size_t kv_stride = 0;
    int num = 0;                 // numerics: 0 ggml's generic order, 1 upstream's x86 association (mv_device.h)
};

// Layer engine (leng.hip): one persistent launch per decode layer runs up to kLeOps
// matvecs in stream order -- attn_output + residual (EPI_ADD), ffn_gate+up + SwiGLU
// (EPI_SWIGLU), ffn_down + residual (EPI_ADD), the next layer's QKV (EPI_QKV) -- with the
// weights streamed into an LDS ring ahead of the activation hand-offs between them.
constexpr int kLeOps = 4;
struct LeArgs {
    MVArgs op[kLeOps];           // set like launch_matvec's (geometry filled by the launcher)
    int nops = 0;                // 3 (last layer: no next QKV) or 4
    unsigned* cnt = nullptr;     // this layer's edge counters: shard j of op k at cnt[j * cnt_stride + 16 k], zero at launch
    size_t cnt_stride = 0;       // words between shards (le_counter_stride)
    unsigned* fault = nullptr;   // context fault word: a bounded in-kernel wait gave up
    int spin_limit = 0;          // polls before a wait gives up (0: default)
    int kmin = 9;                // smallest sub-item of the launch in ring pieces
    // LDS carve (set by the launcher)
    int npieces = 0, img_off0 = 0, img_off1 = 0, fold_off = 0, ring_off = 0, act = -1;
    int exp = 0;                 // LLMI_LE_EXP experiments (results garbage): 1 no math, 2 no edges / images
    unsigned long long* trace = nullptr;  // llmi_engine_trace: [block][16 waves][32] s_memrealtime stamps
};
// bytes of the edge counters of n_layer layers (one memset per step zeroes them)
size_t le_counter_bytes(int n_layer);
size_t le_counter_stride(int n_layer);  // words
// fills the geometry and LDS carve; hipErrorNotSupported: shapes / types / LDS / residency
// the engine does not take (the caller runs the layer as separate launches)
hipError_t layer_engine_prepare(LeArgs& a);
hipError_t launch_layer_engine(const LeArgs& a, hipStream_t s);  // a prepared
double le_stream_bench(const void* src, size_t bytes, int mode, int iters, int nt);  // GB/s (tools/lestream.py)
bool le_wanted();                 // LLMI_ENGINE (default 1) / test option "engine"
extern int g_le_on, g_le_spin;    // test options: engine on/off, spin limit

struct AttnArgs {
    const float* q = nullptr;      // f32[H*D] (roped)
    const uint16_t* kc = nullptr;  // layer base
    const uint16_t* vc = nullptr;
    float* scores = nullptr;       // f32[H][n_ctx]
    float* tmax = nullptr;         // f32[H][n_ctx/32]: per-32-position tile max of the scores
    float* out = nullptr;          // f32[H*D]
    const StepState* st = nullptr;
    int n_ctx = 0;
    float scale = 0.f;
    int layer = 0;                        // k_attn_x: hand-off tag = step seq * 256 + layer + 1
    unsigned long long* gran = nullptr;   // k_attn_x: [H][kXAttnMaxKV] {tag, score} granules
    unsigned* fault = nullptr;            // k_attn_x: set when a bounded wait timed out
    int spin_limit = 1 << 22;             // k_attn_x: polls before a wait gives up (set at launch)
    int tag_skew = 0;                     // test option: consumers expect tag + skew
    unsigned long long* trace = nullptr;  // LLMI_EXP_TRACE builds: [kernel][block][wave][4] stamps
    int num = 0;                          // numerics (MVArgs::num): 1 = the x86 attention kernels (attn86.hip)
    int fa = 0;                           // 1: flash-attention numerics (attnfa.hip; num picks its association)
};

// Batched decode (batch.hip): up to kMaxBatch sequences advance one token per step.
constexpr int kMaxBatch = 8;
struct BAttnArgs {
    AttnArgs a[kMaxBatch];  // per batch slot (its sequence's caches, q, scratch, state)
};
struct BEmbArgs {
    Seg w;
    int cols = 0, vocab = 0, n_ctx = 0, nt = 0;
    float* x = nullptr;           // [nt][cols]
    StepState* st = nullptr;      // per sequence
    int32_t* hist = nullptr;      // [seq][n_ctx]
    const int* tseq = nullptr;    // slot -> sequence
    int* tpos = nullptr;          // slot -> position of this step (written)
};
hipError_t launch_bembed(const BEmbArgs& a, hipStream_t s);
hipError_t launch_mvn(const MVArgs& a, int epi, int nt, int max_blocks, hipStream_t s);
// batched matvec on the matrix cores (batch.hip k_bmm): K-quant segments whose rows are
// multiples of 16; the nt tokens' activations quantized by launch_pf_quant into (aq,
// abs, ad) first.  bmm_ok: whether launch_bmm takes these segments (else launch_mvn).
bool bmm_ok(const MVArgs& a, int epi);
int bmm_min_tokens();
// (abf: k_pf_quant's bsum fragments; the dmin chain's sumi runs on the MFMA)
hipError_t launch_bmm(const MVArgs& a, int epi, int nt, const void* aq, const void* abf, const float* ad, hipStream_t s);
// a QKV of two type groups (a1: q/k rows, a2: the attn_v rows) in one k_bmd2 launch over the
// same quantized activations; hipErrorNotSupported when the pair does not qualify
hipError_t launch_bmm_qkv2(const MVArgs& a1, const MVArgs& a2, int nt, const void* aq, const void* abf, const float* ad,
                           hipStream_t s);
hipError_t launch_battention(const BAttnArgs& b, int nt, int n_head, int n_head_kv, int head_dim, int kv_bound,
                             hipStream_t s);
size_t mvn_lds_bytes(int act, int cols, int nt, int x86 = 0);

struct EmbArgs {
    Seg w;                          // token_embd in device layout
    int cols = 0;
    int vocab = 0;
    float* x = nullptr;
    StepState* st = nullptr;
    int32_t* hist = nullptr;        // token history [n_ctx]
    int n_ctx = 0;
};

// Batched prefill (prefill.hip.inc): one launch per linear layer over T prompt tokens.
struct PfGemm {
    Seg w, w2;                 // weights (SWIGLU: w = gate, w2 = up)
    int rows = 0, cols = 0;
    int T = 0;                 // tokens (activation rows are padded to a multiple of 64)
    int xcd_map = 0;           // set by the launcher: XCD-aware tile order, token-group chunk (k_pf_gemm; 0 off)
    const void* aq = nullptr;     // f16 MFMA fragments of the q8 activations (prefill.hip.inc pf_aq_off), Tpad x cols x 2 B
    const int16_t* abs = nullptr; // [Tpad][cols/32] bsum pairs (q8_K)
    const float* ad = nullptr;    // [Tpad][cols/256] (q8_K) or [Tpad][cols/32] (q8_0) d
    const void* abf = nullptr;    // K-quants: the bsum pairs as sumi MFMA fragments (prefill.hip.inc pf_abf_off)
    float* y = nullptr;        // STORE / ADD / SWIGLU / QKV q: [T][ldy]
    int ldy = 0;
    int part = 0;              // QKV: 0 q (RoPE, f32 to y), 1 k (RoPE, f16 cache), 2 v (f16 cache)
    // QKV over consecutive same-type parts in one launch: rows [0, r1) are part `part` of w,
    // [r1, r2) part + 1 of wk, [r2, rows) part + 2 of wv (r1 = 0: one part); r1, r2
    // multiples of 64 (workgroup rows)
    Seg wk, wv;
    int r1 = 0, r2 = 0;
    uint16_t* kc = nullptr;    // layer K cache [HK][n_ctx][D]
    uint16_t* vc = nullptr;    // layer V cache [HK][D][n_ctx]
    const float* rope = nullptr;
    int pos0 = 0, head_dim = 0, n_rot = 0, n_ctx = 0;
    int exp = 0;               // experiment builds (LLMI_PF_EXP): 1 every lane reads its wave's first row
};
struct PfAttn {
    const float* q = nullptr;  // [T][ldq] roped q
    float* out = nullptr;      // [T][ldq]
    int ldq = 0;
    const uint16_t* kc = nullptr, *vc = nullptr;  // layer caches
    int n_ctx = 0, pos0 = 0, gqa = 1, max_kv = 0;  // max_kv >= pos0 + T (LDS score space)
    float scale = 0.f;
    float* wsc = nullptr;      // k_pf_fa score scratch (pf_fa_scratch_bytes), null: LDS kernels only
    size_t wsc_bytes = 0;
    int num = 0;               // numerics (MVArgs::num): 1 = k_pf_a86 (attn86.hip)
};
// score scratch k_pf_fa wants for ubatches of T tokens over n_ctx positions (0: the
// head shape has no tiled kernel); launches are chunked to fit a smaller scratch
size_t pf_fa_scratch_bytes(int n_head, int n_head_kv, int head_dim, int T, int n_ctx);
constexpr size_t kPfFaScratchCap = (size_t)1 << 30;
bool pf_gemm_ok(int type, int rows, int cols);
hipError_t launch_pf_embed(const Seg& w, int cols, int vocab, const int32_t* toks, float* X, int T, int32_t* hist,
                           int pos0, int n_ctx, hipStream_t s);
hipError_t launch_pf_quant(const float* x, int ldx, const float* nw, float eps, int cols, int act, int T, void* aq,
                           int16_t* abs, float* ad, void* abf, hipStream_t s, int x86 = 0);
hipError_t launch_pf_gemm(const PfGemm& g, int epi, hipStream_t s);
// path: -1 the process setting (pf_attn_fa / pf_attn_simple test options), 0 the tiled
// FP64-MFMA kernel only (hipErrorNotSupported when it does not apply or the scratch is
// short: never a silent fallback), 1 the LDS kernels (grouped, then one head per
// workgroup), 2 one head per workgroup
hipError_t launch_pf_attn(const PfAttn& a, int n_head, int head_dim, int T, hipStream_t s, int path = -1);

// activation kind of a weight type: 0 = block_q8_K (K-quants), 1 = block_q8_0
__host__ __device__ inline int act_kind(int t) { return t == T_Q8_0 ? 1 : 0; }
// row-task geometry of a matvec launch (lr, rpt, ntasks); false if the segments cannot
// be cut into tasks (a QKV segment boundary that is not on an even row)
bool mv_geometry(MVArgs& a, int epi);
size_t mv_lds_bytes(int act, int cols);
// per-type matvec launchers (mv_kernels.h; instantiated in mv_q4k/q5k/q6k/q80.hip)
template <int ACT, bool NORM, int T, int X86>
hipError_t mv_dispatch_epi(const MVArgs& a, int epi, dim3 grid, size_t lds, hipStream_t s);
template <bool NORM, int T, int T2, int X86>
hipError_t mv_qkv2_launch(const MVArgs& a, int split_tasks, dim3 grid, size_t lds, hipStream_t s);

// All launches are asynchronous on `stream` and graph-capturable (no allocation, no sync).
hipError_t launch_matvec(const MVArgs& a, int epi, int max_blocks, hipStream_t stream);
// attention path for a KV bound: 1 fused (one WG per head), 2 split (scores + PV over
// (group, 16-dim slice) workgroups), 3 two-kernel long-context path, 4 one-launch
// exchange (k_attn_x: scores tiles + granule hand-off + PV, kv_bound <= kXAttnMaxKV)
// mode: -1 the process setting (set_attn_mode, LLMI_ATTN_MODE at model load), 0 auto,
// 1..7 one path (A/B and test hooks; a path whose limits the shape passes falls back)
int attn_path(int n_head, int n_head_kv, int kv_bound, int head_dim, int mode = -1);
int attn_d_slices(int n_head, int head_dim);
// arm (or with nullptrs disarm) per-op kernel timing events for this thread's launches
void set_launch_events(hipEvent_t start, hipEvent_t stop);
void set_attn_mode(int mode);
// flash-attention numerics decode attention (attnfa.hip): up to kFaMaxKV positions
constexpr int kFaMaxKV = 8192;
hipError_t launch_attention_fa(const AttnArgs& a, int n_head, int n_head_kv, int head_dim, int kv_bound, hipStream_t s);
// the batched step's flash-attention / x86 attention: every batch slot in one launch
hipError_t launch_battention_fa(const BAttnArgs& b, int nt, int n_head, int n_head_kv, int head_dim, int kv_bound,
                                hipStream_t s);
hipError_t launch_battention_x86(const BAttnArgs& b, int nt, int n_head, int n_head_kv, int head_dim, int kv_bound,
                                 hipStream_t s);
hipError_t launch_attention(const AttnArgs& a, int n_head, int n_head_kv, int head_dim, int kv_bound, hipStream_t stream,
                            int mode = -1);
hipError_t launch_embed(const EmbArgs& a, hipStream_t stream);
// the last step's embedding row again (debug tap 0)
hipError_t launch_embed_row(const EmbArgs& a, const StepState* st, float* out, hipStream_t stream);
hipError_t launch_repack(int type, const void* raw, uint8_t* a, uint8_t* h, uint8_t* s, uint8_t* d, int64_t nblk, int64_t cols, int rgs,
                         int x86, hipStream_t stream);
// x86 numerics attention (attn86.hip): upstream's non-flash CPU attention in its x86 AVX2
// association (f16 dots in 4 x 8 fp32 fma lanes, ggml_v_expf softmax with per-8 sums)
// mode 3: the three-launch path at every context (tests); else one launch up to 2048 positions
hipError_t launch_attention_x86(const AttnArgs& a, int n_head, int n_head_kv, int head_dim, int kv_bound, hipStream_t s,
                                int mode = 0);
hipError_t launch_pf_attn_x86(const PfAttn& a, int n_head, int n_head_kv, int head_dim, int T, hipStream_t s);
int pf_attn_x86_max_kv(int n_head, int n_head_kv, int head_dim);
// writes the prologue's quantized activation in ggml block form (test hook)
hipError_t launch_quant_dump(const MVArgs& a, int act, void* out, hipStream_t stream);
hipError_t launch_stream_read(const void* p, size_t bytes, unsigned* out, int blocks, hipStream_t stream);
// order-independent 64-bit hash of `bytes` of device memory into *out (device), kernels.hip
hipError_t launch_arena_hash(const void* p, size_t bytes, unsigned long long* out, hipStream_t stream);
hipError_t launch_state_set(StepState* st, int token_in, int pos_next, hipStream_t stream);
hipError_t launch_state_tick(StepState* st, hipStream_t stream);  // seq += 1 (microbenchmarks)

}  // namespace llmi
