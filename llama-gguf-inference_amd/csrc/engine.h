// engine.h — model (device weight arena) and context (KV cache, scratch, step graphs).
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include <functional>

#include "common.h"
#include "gguf.h"
#include "kernels.h"
#include "tokenizer.h"

namespace llmi {

struct HParams {
    int n_embd = 0, n_layer = 0, n_head = 0, n_head_kv = 0, head_dim = 0, n_ff = 0, n_vocab = 0;
    int n_rot = 0, n_ctx_train = 0, file_type = 0;
    float eps = 1e-5f, rope_base = 10000.f;
};

struct Layer {
    DevMat attn_norm, wq, wk, wv, wo, ffn_norm, wg, wu, wd;
};

// Model numerics: the fp32 association every kernel reproduces.
//   0 ggml's generic scalar order (the oracle's default)
//   1 upstream's x86 AVX2 association (the oracle's or_set_x86_mode(X86_ALL)): the weight
//     planes in the x86 byte order (common.h), fma chains per 4-byte lane, the x86
//     attention (attn86.hip), ggml_v_expf softmax / SiLU, round-half-even q8_0
//   + NUMERICS_FA (bit 1 of llama_model_params.numerics): decode attention in ggml's CPU
//     flash-attention numerics (attnfa.hip) in the association of bit 0; such a model
//     runs prompts as decode steps and batched sequences one after another
enum : int { NUMERICS_GENERIC = 0, NUMERICS_X86 = 1, NUMERICS_FA = 2 };

struct Model {
    int device = 0;
    int numerics = NUMERICS_GENERIC;      // fixed at load: the weight planes' byte order depends on it
    int fa = 0;                           // 1: flash-attention numerics (NUMERICS_FA)
    std::string path, desc;
    std::shared_ptr<GgufFile> file;
    HParams hp;
    DevMat tok_embd, out_norm, output, rope_freqs;
    bool has_rope_freqs = false;
    std::vector<Layer> layers;
    uint8_t* arena = nullptr;
    size_t arena_bytes = 0;
    bool owns_arena = true;
    std::vector<std::string> vocab;
    std::shared_ptr<Tokenizer> tok;      // llama_tokenize / llama_token_to_piece (tokenizer.h)
    int bos = -1, eos = -1;
    std::vector<float> rope_freq_host;  // rope_freqs.weight, if present
    double upload_s = 0;                 // chunked pinned upload + repack time (model_load)
    ~Model();
};

// Kernel-class timing (llmi_profile_kernels): step_enqueue with a Prof attached only
// enqueues the launches of class `only` (all classes if -1), records their algorithmic
// bytes per class and, when `timed`, arms an event pair (kernel start / end) on each.
enum KClass : int { K_EMBED = 0, K_QKV, K_ATTN, K_ATTN_OUT, K_FFN_GATE_UP, K_FFN_DOWN, K_OUTPUT, K_LAYER, K_NCLASS };
// (K_LAYER: one layer-engine launch, leng.hip = attn_output + gate/up + down + next QKV)
struct Prof {
    int only = -1;               // class filter (-1: every class)
    bool timed = false;          // arm an event pair around every filtered launch
    int launches[K_NCLASS] = {};    // launches enqueued per class
    double bytes[K_NCLASS] = {};    // their fixed algorithmic bytes ...
    double per_kv[K_NCLASS] = {};   // ... + per_kv * n_kv (attention: K and V rows read)
    std::vector<hipEvent_t> ev;  // 2 per timed launch
    std::vector<int> ev_cls;     // class of each timed launch
    size_t used = 0;
    bool want(int k) const { return only < 0 || only == k; }
    void add(int k, double b, double b_per_kv = 0.0) {
        if (!want(k)) return;
        ++launches[k]; bytes[k] += b; per_kv[k] += b_per_kv;
    }
    bool arm(int k);             // next event pair -> set_launch_events
    static void disarm();
    double elapsed_us(int k, int* n) const;  // sum over class k's recorded pairs (after a sync)
    ~Prof();
};

struct Context {
    Model* m = nullptr;
    int device = 0;                         // m->device, kept so teardown never reads *m
    // sequences (llama_context_params.n_seq_max): each has its own KV cache, StepState
    // and token history; kc/vc/st/hist below point at the CURRENT sequence's (cur_seq),
    // kc0/vc0/st0/hist0 at sequence 0 of the arrays.  With n_seq > 1 one extra (dummy)
    // sequence backs the padded slots of a batched step.
    int n_seq = 1, cur_seq = 0;
    size_t kv_seq_elems = 0;                // K (or V) cache elements per sequence
    uint16_t *kc0 = nullptr, *vc0 = nullptr;
    StepState* st0 = nullptr;
    int32_t* hist0 = nullptr;
    std::vector<int> seq_past;              // per sequence: positions decoded
    int n_ctx = 0;
    bool use_graphs = true;
    hipStream_t stream = nullptr;
    int max_blocks = 1024;
    // device
    float *x = nullptr, *q = nullptr, *att = nullptr, *h = nullptr, *logits = nullptr, *scores = nullptr;
    float* rope = nullptr;
    uint16_t *kc = nullptr, *vc = nullptr;
    StepState* st = nullptr;
    int32_t* hist = nullptr;
    // host
    std::vector<float> logits_host;         // [n_outputs][n_vocab]
    std::vector<int> out_rows;              // batch index -> row in logits_host, -1 none
    std::vector<unsigned long long> out_keys;  // per output: argmax key
    int n_outputs = 0;
    int n_past = 0;
    std::map<int, hipGraphExec_t> graphs;   // by KV bucket * 256 + sequence
    // batched decode (batch.hip): kMaxBatch rows each, allocated on first use
    float *bx = nullptr, *bq = nullptr, *batt = nullptr, *bh = nullptr, *blogits = nullptr, *bscores = nullptr;
    int *btpos = nullptr, *btseq = nullptr;
    void* baq = nullptr;           // k_bmm: the step's quantized activations (pf_quant layout, 32 token rows)
    int16_t* babs = nullptr;
    float* bad = nullptr;
    void* babf = nullptr;          // k_bmm: the step's bsum pairs as sumi MFMA fragments (pf_abf_off)
    std::vector<int> btseq_host;            // the slot -> sequence map btseq holds
    std::map<std::string, hipGraphExec_t> bgraphs;  // by (slots, sequences, KV bucket)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    unsigned* fault_dev = nullptr;          // device fault word: a bounded in-kernel wait gave up
    unsigned* fault_host = nullptr;         // pinned copy, read back with every decode call
    unsigned* le_cnt = nullptr;             // layer-engine edge counters (le_counter_bytes), zeroed per step
    unsigned long long* le_trace = nullptr; // llmi_engine_trace: stamps of layer le_trace_layer's launch
    int le_trace_layer = -1;
    double last_bytes = 0, last_us = 0;
    Prof* prof = nullptr;                   // non-null only inside llmi_profile_kernels
    // batched prefill scratch (allocated on first use; ubatches of <= pf_cap tokens)
    int pf_cap = 0;
    int32_t* pf_tok = nullptr;
    float *pf_x = nullptr, *pf_q = nullptr, *pf_att = nullptr, *pf_h = nullptr;
    void* pf_aq = nullptr;         // f16 MFMA fragments of the ubatch's activations
    int16_t* pf_abs = nullptr;
    float* pf_ad = nullptr;
    void* pf_abf = nullptr;        // K-quants: bsum pairs as k_pf_gemm's sumi MFMA fragments
    float* pf_wsc = nullptr;       // k_pf_fa score scratch (pf_fa_scratch_bytes; null: LDS attention kernels)
    size_t pf_wsc_bytes = 0;
    ~Context();
};

// all return false and set err on failure
// Upload progress hook (replica fan-out pipelined behind the H2D): called
// after each tensor's chunks are enqueued on the upload stream `us` with the end of the
// arena prefix that is complete once `us` reaches that point (tensors are planned in
// upload order, so the prefix grows monotonically); false aborts the load.
using UploadHook = std::function<bool(size_t prefix_end, hipStream_t us)>;
bool model_load(const std::string& path, int device, bool vocab_only, bool no_upload, Model& m, std::string& err,
                const UploadHook* hook = nullptr, int numerics = NUMERICS_GENERIC);
// the upload half of model_load (after a load with no_upload)
bool model_upload(Model& m, std::string& err, const UploadHook* hook = nullptr);
// a matrix of the arena as a matvec segment (rows start at row0 of the launch)
Seg seg_of(const Model& m, const DevMat& d, int row0);

// Fan-out pieces of an arena: [k * chunk, min((k + 1) * chunk, arena_bytes)).  Piece k is
// issued after the first upload event whose prefix covers its end; ready[k] = index of
// that event in prefix_ends (ascending).  Returns the number of pieces.
size_t fanout_plan(size_t arena_bytes, size_t chunk, const std::vector<size_t>& prefix_ends, std::vector<int>& ready);
constexpr size_t kFanoutChunk = 256u << 20;  // 256 MB broadcasts behind the upload
bool context_init(Model* m, int n_ctx, bool use_graphs, int n_seq, Context& c, std::string& err);
// point the single-sequence paths (step_run, prefill_enqueue, state) at sequence s
void context_select_seq(Context& c, int s);
// clear one sequence's KV cache, history and state
void context_clear_seq(Context& c, int s);
// one batched decode step of nt sequences seqs[0..nt) (their StepStates hold token and
// position), replayed from a graph per (slots, sequences, KV bucket of max_pos)
bool bstep_run(Context& c, int nt, const int* seqs, int max_pos, std::string& err);
// enqueue one decode step for a state already set (token_in/pos_next); kv_bound >= pos+1
bool step_enqueue(Context& c, int kv_bound, std::string& err);
// run one step via the cached graph of its KV bucket (or eagerly)
bool step_run(Context& c, int pos, std::string& err);
double bytes_per_token(const Model& m, int n_kv);
// batched prefill: can the model's layers run through the MFMA prefill path?
bool prefill_supported(const Model& m);
bool bstep_supported(const Model& m);  // batched steps in this model's numerics (engine.cpp)
// positions the batched prefill's attention reaches: the context when the tiled kernel
// (k_pf_fa) takes the model's heads, else the LDS kernels' pf_max_kv()
int prefill_max_kv(Context& c);
// run tokens [0, n) at positions pos0.. through every layer as batched launches (KV
// cache written, no logits); enqueued on c.stream, no synchronisation
bool prefill_enqueue(Context& c, const int32_t* tokens, int n, int pos0, std::string& err);
void context_clear(Context& c);
// enqueue the device fault word's read-back (before the call's stream sync) ...
void context_fault_readback(Context& c);
// ... and after the sync: false (err set, word re-armed) if an in-kernel wait gave up
bool context_fault_ok(Context& c, std::string& err);
size_t model_tensor_bytes(const Model& m);
// arena layout of a model for another device (replica); no upload
bool model_clone_layout(const Model& src, int device, Model& dst, std::string& err);

std::string hip_err(hipError_t e);
// matvec grid cap = CUs x wg_per_cu() workgroups (env LLMI_WG_PER_CU, read when a context
// is created; default 2: measured best on every config, profiles/r01/wg_sweep.md)
int wg_per_cu();
int64_t synth_write_gguf(const std::string& path, const std::string& preset, uint64_t seed, int n_layer, int n_vocab,
                         int n_threads, std::string& err);

}  // namespace llmi
