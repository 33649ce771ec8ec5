// capi.cpp — extern "C" drop-in surface (include/llmi.h).  Each function restates
// the upstream llama.h entry point of the same name; no C++ exception
// crosses this boundary, errors go to the thread-local llmi_last_error().
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/llmi.h"
#include "engine.h"

using namespace llmi;

struct llama_model {
    Model m;
};
struct llama_vocab {
    const Model* m;                      // null for llmi_vocab_load_from_file handles
    const Tokenizer* tok;
    std::unique_ptr<Tokenizer> owned;
};
struct llama_context {
    Context c;
    llama_model* owner;
    uint8_t* outs = nullptr;        // device copies of flagged logits rows [cap][n_vocab]
    int outs_cap = 0;
    std::vector<char> host_valid;   // per output row: logits_host filled
    unsigned long long* keys_pinned = nullptr;  // per output row argmax key (pinned host)
    int keys_cap = 0;
};

namespace {
thread_local std::string g_err;
void set_err(const std::string& e) { g_err = e; }
#define API_TRY try {
#define API_CATCH(ret)                                   \
    }                                                    \
    catch (const std::bad_alloc&) {                      \
        set_err("out of host memory");                   \
        return ret;                                      \
    }                                                    \
    catch (...) {                                        \
        set_err("internal error");                       \
        return ret;                                      \
    }

llama_vocab* vocab_handle(const llama_model* m) {
    static thread_local std::vector<std::unique_ptr<llama_vocab>> pool;
    for (auto& v : pool)
        if (v->m == &m->m) return v.get();
    auto v = std::make_unique<llama_vocab>();
    v->m = &m->m;
    v->tok = m->m.tok.get();
    pool.push_back(std::move(v));
    return pool.back().get();
}

bool ensure_outs(llama_context* ctx, int n) {
    const int V = ctx->c.m->hp.n_vocab;
    if (n <= ctx->outs_cap) return true;
    if (ctx->outs) (void)hipFree(ctx->outs);
    ctx->outs = nullptr;
    ctx->outs_cap = 0;
    if (hipMalloc(&ctx->outs, (size_t)n * V * 4) != hipSuccess) { set_err("hipMalloc logits outputs"); return false; }
    ctx->outs_cap = n;
    if (n > ctx->keys_cap) {
        if (ctx->keys_pinned) (void)hipHostFree(ctx->keys_pinned);
        ctx->keys_pinned = nullptr;
        if (hipHostMalloc((void**)&ctx->keys_pinned, (size_t)n * 8 * kArgSlots, hipHostMallocDefault) != hipSuccess) {
            set_err("hipHostMalloc");
            return false;
        }
        ctx->keys_cap = n;
    }
    return true;
}
}  // namespace

extern "C" {

const char* llmi_last_error(void) { return g_err.c_str(); }

int32_t llmi_model_numerics(const struct llama_model* model) {
    return model ? model->m.numerics | (model->m.fa ? NUMERICS_FA : 0) : -1;
}

void llama_backend_init(void) { (void)hipInit(0); }
void llama_backend_free(void) {}

struct llama_model_params llama_model_default_params(void) {
    struct llama_model_params p;
    p.n_gpu_layers = 999;
    p.main_gpu = 0;
    p.vocab_only = false;
    p.use_mmap = true;
    p.no_upload = false;
    p.numerics = LLMI_NUMERICS_GENERIC;
    return p;
}

struct llama_context_params llama_context_default_params(void) {
    struct llama_context_params p;
    p.n_ctx = 4096;
    p.n_batch = 2048;
    p.n_ubatch = 512;
    p.n_seq_max = 1;
    p.n_threads = 0;
    p.use_graphs = true;
    return p;
}

int32_t llmi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

struct llama_model* llama_model_load_from_file(const char* path, struct llama_model_params params) {
    API_TRY
    if (!path) { set_err("null path"); return nullptr; }
    if (params.n_gpu_layers == 0 && !params.vocab_only) {
        set_err("n_gpu_layers=0 requests the CPU path; llmi is GPU-only (the NGL=0 path is the reference's "
                "llama.cpp CPU server, Dockerfile.cpu:84-89)");
        return nullptr;
    }
    if (!params.vocab_only) {
        const int n = llmi_device_count();
        if (n <= 0) { set_err("no HIP device visible"); return nullptr; }
        if (params.main_gpu < 0 || params.main_gpu >= n) { set_err("main_gpu out of range"); return nullptr; }
    }
    auto* m = new llama_model();
    std::string err;
    if (!model_load(path, params.main_gpu, params.vocab_only, params.no_upload, m->m, err, nullptr, params.numerics)) {
        set_err(err);
        delete m;
        return nullptr;
    }
    return m;
    API_CATCH(nullptr)
}

void llama_model_free(struct llama_model* model) { delete model; }

struct llama_context* llama_init_from_model(struct llama_model* model, struct llama_context_params params) {
    API_TRY
    if (!model || !model->m.arena) { set_err("model has no device weights"); return nullptr; }
    auto* ctx = new llama_context();
    ctx->owner = model;
    std::string err;
    if (!context_init(&model->m, (int)params.n_ctx, params.use_graphs, (int)std::max<uint32_t>(1u, params.n_seq_max), ctx->c, err)) {
        set_err(err);
        delete ctx;
        return nullptr;
    }
    return ctx;
    API_CATCH(nullptr)
}

void llama_free(struct llama_context* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->c.device);  // never reads the model: it may be freed already
    if (ctx->outs) (void)hipFree(ctx->outs);
    if (ctx->keys_pinned) (void)hipHostFree(ctx->keys_pinned);
    delete ctx;
}

struct llama_batch llama_batch_get_one(llama_token* tokens, int32_t n_tokens) {
    struct llama_batch b;
    std::memset(&b, 0, sizeof b);
    b.n_tokens = n_tokens;
    b.token = tokens;
    return b;
}

struct llama_batch llama_batch_init(int32_t n_tokens, int32_t embd, int32_t n_seq_max) {
    struct llama_batch b;
    std::memset(&b, 0, sizeof b);
    if (n_tokens <= 0) return b;
    if (embd) b.embd = (float*)calloc((size_t)n_tokens * embd, sizeof(float));
    else b.token = (llama_token*)calloc((size_t)n_tokens, sizeof(llama_token));
    b.pos = (llama_pos*)calloc((size_t)n_tokens, sizeof(llama_pos));
    b.n_seq_id = (int32_t*)calloc((size_t)n_tokens, sizeof(int32_t));
    b.seq_id = (llama_seq_id**)calloc((size_t)n_tokens + 1, sizeof(llama_seq_id*));
    for (int i = 0; i < n_tokens; ++i) b.seq_id[i] = (llama_seq_id*)calloc((size_t)std::max(1, n_seq_max), sizeof(llama_seq_id));
    b.logits = (int8_t*)calloc((size_t)n_tokens, 1);
    return b;
}

void llama_batch_free(struct llama_batch b) {
    free(b.token);
    free(b.embd);
    free(b.pos);
    free(b.n_seq_id);
    if (b.seq_id) {
        for (int i = 0; b.seq_id[i]; ++i) free(b.seq_id[i]);
        free(b.seq_id);
    }
    free(b.logits);
}

// shortest prompt run taken by the batched prefill path (shorter runs: decode steps)
static constexpr int kPrefillMin = 2;

static int seq_past_of(const Context& c, int s) { return s == c.cur_seq ? c.n_past : c.seq_past[(size_t)s]; }
static void set_seq_past(Context& c, int s, int v) {
    if (s == c.cur_seq) c.n_past = v;
    else c.seq_past[(size_t)s] = v;
}

static void copy_out(llama_context* ctx, int r, const float* logits_dev, const StepState* st, int pos) {
    Context& c = ctx->c;
    const size_t V = (size_t)c.m->hp.n_vocab;
    (void)hipMemcpyAsync(ctx->outs + (size_t)r * V * 4, logits_dev, V * 4, hipMemcpyDeviceToDevice, c.stream);
    (void)hipMemcpyAsync(ctx->keys_pinned + (size_t)r * kArgSlots, &st->key[pos & 1][0], 8 * kArgSlots, hipMemcpyDeviceToHost,
                         c.stream);
}

// One sequence's tokens (batch indices idx, positions pos) through the single-sequence
// path: the batched prefill of the leading run of consecutive, logit-less tokens (leaving
// at least the last token to a decode step), then decode steps.
// LLMI_NO_PREFILL=1 runs every token as a decode step.
static bool run_seq(llama_context* ctx, const llama_batch& batch, int seq, const std::vector<int>& idx,
                    const std::vector<int>& pos, const std::vector<int>& rows, double& bytes, std::string& err) {
    Context& c = ctx->c;
    context_select_seq(c, seq);
    const int n = (int)idx.size();
    int i0 = 0;
    const char* no_pf_env = getenv("LLMI_NO_PREFILL");
    const bool no_pf = no_pf_env && atoi(no_pf_env) != 0;
    const int p0 = pos[0];
    int run = 0;
    while (run < n - 1 && rows[(size_t)idx[(size_t)run]] < 0 && pos[(size_t)run] == p0 + run) ++run;
    // a run reaching past prefill_max_kv() positions (the LDS-resident attention kernels'
    // limit where the tiled one does not apply) goes through decode steps from there on
    if (!no_pf && run >= kPrefillMin && prefill_supported(*c.m)) {
        const int pf_lim = prefill_max_kv(c);
        if (p0 + run > pf_lim) run = std::max(0, pf_lim - p0);
    }
    if (!no_pf && run >= kPrefillMin && prefill_supported(*c.m)) {
        std::vector<int32_t> toks((size_t)run);
        for (int i = 0; i < run; ++i) toks[(size_t)i] = batch.token[idx[(size_t)i]];
        if (!prefill_enqueue(c, toks.data(), run, p0, err)) return false;
        for (int i = 0; i < run; ++i) bytes += bytes_per_token(*c.m, p0 + i + 1);
        i0 = run;
    }
    for (int i = i0; i < n; ++i) {
        const int p = pos[(size_t)i];
        if (launch_state_set(c.st, batch.token[idx[(size_t)i]], p, c.stream) != hipSuccess || !step_run(c, p, err)) {
            if (err.empty()) err = "launch failed";
            return false;
        }
        bytes += bytes_per_token(*c.m, p + 1);
        const int r = rows[(size_t)idx[(size_t)i]];
        if (r >= 0) copy_out(ctx, r, c.logits, c.st, p);
    }
    return true;
}

int32_t llama_decode(struct llama_context* ctx, struct llama_batch batch) {
    API_TRY
    if (!ctx) { set_err("null context"); return -1; }
    Context& c = ctx->c;
    const HParams& hp = c.m->hp;
    if (batch.n_tokens <= 0 || !batch.token) { set_err("llama_decode: empty batch or no tokens"); return -1; }
    if (batch.embd) { set_err("llama_decode: embedding input is not supported"); return -1; }
    const int n = batch.n_tokens;
    std::vector<int> rows((size_t)n, -1);
    int n_out = 0;
    for (int i = 0; i < n; ++i)
        if (batch.logits ? batch.logits[i] != 0 : i == n - 1) rows[(size_t)i] = n_out++;
    // tokens by sequence (llama_batch.seq_id[i][0]; no seq_id: sequence 0), in batch order
    std::vector<std::vector<int>> by_seq((size_t)c.n_seq), pos_of((size_t)c.n_seq);
    for (int i = 0; i < n; ++i) {
        const int tok = batch.token[i];
        if (tok < 0 || tok >= hp.n_vocab) { set_err("llama_decode: token id out of range"); return -1; }
        int s = 0;
        if (batch.seq_id && batch.n_seq_id) {
            if (batch.n_seq_id[i] > 1) { set_err("llama_decode: a token shared by several sequences is not supported"); return -1; }
            if (batch.n_seq_id[i] == 1) s = batch.seq_id[i][0];
        }
        if (s < 0 || s >= c.n_seq) { set_err("llama_decode: seq_id out of range (n_seq_max)"); return -1; }
        const int pos = batch.pos ? batch.pos[i] : seq_past_of(c, s) + (int)by_seq[(size_t)s].size();
        if (pos < 0) { set_err("llama_decode: negative position"); return -1; }
        if (pos >= c.n_ctx) { set_err("llama_decode: no KV slot (position >= n_ctx)"); return 1; }
        by_seq[(size_t)s].push_back(i);
        pos_of[(size_t)s].push_back(pos);
    }
    if (hipSetDevice(c.m->device) != hipSuccess) { set_err("hipSetDevice"); return -2; }
    (void)hipGetLastError();  // launch wrappers report hipGetLastError: drop an unrelated stale one
    if (n_out > 0 && !ensure_outs(ctx, n_out)) return -2;
    c.out_rows = rows;
    c.n_outputs = n_out;
    ctx->host_valid.assign((size_t)n_out, 0);
    c.logits_host.resize((size_t)std::max(1, n_out) * hp.n_vocab);
    std::string err;
    double bytes = 0;
    hipEventRecord(c.ev0, c.stream);
    // sequences with one token each advance together through batched steps (batch.hip,
    // up to kMaxBatch per step); the others run one sequence at a time
    std::vector<int> singles;
    for (int s = 0; s < c.n_seq; ++s)
        if (by_seq[(size_t)s].size() == 1) singles.push_back(s);
    if (singles.size() < 2) singles.clear();
    for (size_t g = 0; g < singles.size(); g += kMaxBatch) {
        const int nt = (int)std::min<size_t>(kMaxBatch, singles.size() - g);
        const int* seqs = singles.data() + g;
        int max_pos = 0;
        for (int k = 0; k < nt; ++k) {
            const int s = seqs[k], p = pos_of[(size_t)s][0];
            max_pos = std::max(max_pos, p);
            if (launch_state_set(c.st0 + s, batch.token[by_seq[(size_t)s][0]], p, c.stream) != hipSuccess) {
                set_err("llama_decode: state set failed");
                return -3;
            }
        }
        if (!bstep_run(c, nt, seqs, max_pos, err)) {
            // not batchable here (context beyond the batched attention's LDS bound, mixed
            // gate/up types): these sequences take the single-sequence path below
            err.clear();
            singles.resize(g);
            break;
        }
        for (int k = 0; k < nt; ++k) {
            const int s = seqs[k], p = pos_of[(size_t)s][0];
            bytes += bytes_per_token(*c.m, p + 1) / nt;  // weights once for the group, KV per sequence
            const int r = rows[(size_t)by_seq[(size_t)s][0]];
            if (r >= 0) copy_out(ctx, r, c.blogits + (size_t)k * hp.n_vocab, c.st0 + s, p);
        }
    }
    for (int s = 0; s < c.n_seq; ++s) {
        if (by_seq[(size_t)s].empty() || std::find(singles.begin(), singles.end(), s) != singles.end()) continue;
        if (!run_seq(ctx, batch, s, by_seq[(size_t)s], pos_of[(size_t)s], rows, bytes, err)) {
            set_err("llama_decode: " + err);
            return -3;
        }
    }
    hipEventRecord(c.ev1, c.stream);
    context_fault_readback(c);
    hipError_t e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) { set_err("llama_decode: " + hip_err(e)); return -4; }
    if (!context_fault_ok(c, err)) { set_err("llama_decode: " + err); return -6; }
    float ms = 0.f;
    hipEventElapsedTime(&ms, c.ev0, c.ev1);
    c.last_us = ms * 1e3;
    c.last_bytes = bytes;
    for (int s = 0; s < c.n_seq; ++s) {
        if (by_seq[(size_t)s].empty()) continue;
        int last = seq_past_of(c, s) - 1;
        for (int p : pos_of[(size_t)s]) last = std::max(last, p);
        set_seq_past(c, s, last + 1);
    }
    return 0;
    API_CATCH(-5)
}

int llama_eval(struct llama_context* ctx, llama_token* tokens, int32_t n_tokens, int32_t n_past) {
    if (!ctx || !tokens || n_tokens <= 0) { set_err("llama_eval: bad arguments"); return 1; }
    std::vector<llama_pos> pos((size_t)n_tokens);
    for (int i = 0; i < n_tokens; ++i) pos[(size_t)i] = n_past + i;
    struct llama_batch b = llama_batch_get_one(tokens, n_tokens);
    b.pos = pos.data();
    return llama_decode(ctx, b) == 0 ? 0 : 1;
}

static int out_row(llama_context* ctx, int32_t i) {
    Context& c = ctx->c;
    if (c.n_outputs <= 0) return -1;
    if (i < 0) return c.n_outputs - 1;
    if (i >= (int)c.out_rows.size()) return -1;
    return c.out_rows[(size_t)i];
}

float* llama_get_logits_ith(struct llama_context* ctx, int32_t i) {
    API_TRY
    if (!ctx) return nullptr;
    const int r = out_row(ctx, i);
    if (r < 0) { set_err("llama_get_logits_ith: no logits for this batch index"); return nullptr; }
    Context& c = ctx->c;
    const size_t V = (size_t)c.m->hp.n_vocab;
    if (!ctx->host_valid[(size_t)r]) {
        (void)hipSetDevice(c.m->device);
        if (hipMemcpy(c.logits_host.data() + (size_t)r * V, ctx->outs + (size_t)r * V * 4, V * 4,
                      hipMemcpyDeviceToHost) != hipSuccess) {
            set_err("logits copy failed");
            return nullptr;
        }
        ctx->host_valid[(size_t)r] = 1;
    }
    return c.logits_host.data() + (size_t)r * V;
    API_CATCH(nullptr)
}

float* llama_get_logits(struct llama_context* ctx) {
    if (!ctx || ctx->c.n_outputs <= 0) { set_err("llama_get_logits: no outputs"); return nullptr; }
    for (int r = 0; r < ctx->c.n_outputs; ++r) {
        // materialise every output row
        int idx = -1;
        for (size_t k = 0; k < ctx->c.out_rows.size(); ++k)
            if (ctx->c.out_rows[k] == r) idx = (int)k;
        if (idx >= 0 && !llama_get_logits_ith(ctx, idx)) return nullptr;
    }
    return ctx->c.logits_host.data();
}

llama_token llmi_greedy_ith(struct llama_context* ctx, int32_t i) {
    if (!ctx) return -1;
    const int r = out_row(ctx, i);
    if (r < 0) { set_err("llmi_greedy_ith: no logits for this batch index"); return -1; }
    return (llama_token)key_token(ctx->keys_pinned + (size_t)r * kArgSlots);
}

int32_t llmi_generate_greedy(struct llama_context* ctx, llama_token first, int32_t pos0, int32_t n_gen, llama_token* out) {
    API_TRY
    if (!ctx || !out || n_gen <= 0) { set_err("llmi_generate_greedy: bad arguments"); return -1; }
    Context& c = ctx->c;
    const HParams& hp = c.m->hp;
    if (first < 0 || first >= hp.n_vocab) { set_err("llmi_generate_greedy: token out of range"); return -1; }
    if (pos0 < 0 || pos0 + n_gen > c.n_ctx) { set_err("llmi_generate_greedy: exceeds n_ctx"); return 1; }
    (void)hipSetDevice(c.m->device);
    (void)hipGetLastError();
    std::string err;
    double bytes = 0;
    if (launch_state_set(c.st, first, pos0, c.stream) != hipSuccess) { set_err("state set failed"); return -3; }
    hipEventRecord(c.ev0, c.stream);
    for (int k = 0; k < n_gen; ++k) {
        if (!step_run(c, pos0 + k, err)) { set_err("llmi_generate_greedy: " + err); return -3; }
        bytes += bytes_per_token(*c.m, pos0 + k + 1);
    }
    hipEventRecord(c.ev1, c.stream);
    std::vector<int32_t> h((size_t)n_gen);
    unsigned long long keys[kArgSlots];
    if (n_gen > 1)
        (void)hipMemcpyAsync(h.data(), c.hist + pos0 + 1, (size_t)(n_gen - 1) * 4, hipMemcpyDeviceToHost, c.stream);
    (void)hipMemcpyAsync(keys, &c.st->key[(pos0 + n_gen - 1) & 1][0], sizeof(keys), hipMemcpyDeviceToHost, c.stream);
    context_fault_readback(c);
    hipError_t e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) { set_err("llmi_generate_greedy: " + hip_err(e)); return -4; }
    if (!context_fault_ok(c, err)) { set_err("llmi_generate_greedy: " + err); return -6; }
    for (int k = 0; k + 1 < n_gen; ++k) out[k] = h[(size_t)k];
    out[n_gen - 1] = (llama_token)key_token(keys);
    float ms = 0.f;
    hipEventElapsedTime(&ms, c.ev0, c.ev1);
    c.last_us = ms * 1e3;
    c.last_bytes = bytes;
    c.n_past = pos0 + n_gen;
    c.n_outputs = 0;
    return n_gen;
    API_CATCH(-5)
}

int32_t llmi_generate_greedy_batch(struct llama_context* ctx, int32_t n, const int32_t* seqs, const llama_token* first,
                                   const int32_t* pos0, int32_t n_gen, llama_token* out) {
    API_TRY
    if (!ctx || n <= 0 || n > kMaxBatch || !seqs || !first || !pos0 || !out || n_gen <= 0) {
        set_err("llmi_generate_greedy_batch: bad arguments (1..8 sequences)");
        return -1;
    }
    Context& c = ctx->c;
    const HParams& hp = c.m->hp;
    int max_end = 0;
    for (int k = 0; k < n; ++k) {
        if (seqs[k] < 0 || seqs[k] >= c.n_seq) { set_err("llmi_generate_greedy_batch: seq out of range (n_seq_max)"); return -1; }
        for (int j = 0; j < k; ++j)
            if (seqs[j] == seqs[k]) { set_err("llmi_generate_greedy_batch: repeated sequence"); return -1; }
        if (first[k] < 0 || first[k] >= hp.n_vocab) { set_err("llmi_generate_greedy_batch: token out of range"); return -1; }
        if (pos0[k] < 0 || pos0[k] + n_gen > c.n_ctx) { set_err("llmi_generate_greedy_batch: exceeds n_ctx"); return 1; }
        max_end = std::max(max_end, pos0[k] + n_gen);
    }
    if (n == 1) {  // one sequence: the single-sequence step (k_matvec path, its own graphs)
        context_select_seq(c, seqs[0]);
        return llmi_generate_greedy(ctx, first[0], pos0[0], n_gen, out);
    }
    if (!bstep_supported(*c.m)) {  // (every numerics has a batched step since round 6; kept for a model that has none)
        for (int k = 0; k < n; ++k) {
            context_select_seq(c, seqs[k]);
            const int32_t r = llmi_generate_greedy(ctx, first[k], pos0[k], n_gen, out + (size_t)k * n_gen);
            if (r != n_gen) return r;
        }
        return n_gen;
    }
    (void)hipSetDevice(c.m->device);
    (void)hipGetLastError();
    std::string err;
    double bytes = 0;
    for (int k = 0; k < n; ++k)
        if (launch_state_set(c.st0 + seqs[k], first[k], pos0[k], c.stream) != hipSuccess) { set_err("state set failed"); return -3; }
    hipEventRecord(c.ev0, c.stream);
    for (int j = 0; j < n_gen; ++j) {
        int max_pos = 0;
        for (int k = 0; k < n; ++k) {
            max_pos = std::max(max_pos, pos0[k] + j);
            bytes += bytes_per_token(*c.m, pos0[k] + j + 1) / n;
        }
        if (!bstep_run(c, n, seqs, max_pos, err)) { set_err("llmi_generate_greedy_batch: " + err); return -3; }
    }
    hipEventRecord(c.ev1, c.stream);
    std::vector<int32_t> h((size_t)n * n_gen);
    std::vector<unsigned long long> keys((size_t)n * kArgSlots);
    for (int k = 0; k < n; ++k) {
        const int32_t* hist = c.hist0 + (size_t)seqs[k] * c.n_ctx;
        if (n_gen > 1)
            (void)hipMemcpyAsync(h.data() + (size_t)k * n_gen, hist + pos0[k] + 1, (size_t)(n_gen - 1) * 4, hipMemcpyDeviceToHost,
                                 c.stream);
        (void)hipMemcpyAsync(keys.data() + (size_t)k * kArgSlots, &c.st0[seqs[k]].key[(pos0[k] + n_gen - 1) & 1][0],
                             8 * kArgSlots, hipMemcpyDeviceToHost, c.stream);
    }
    context_fault_readback(c);
    hipError_t e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) { set_err("llmi_generate_greedy_batch: " + hip_err(e)); return -4; }
    if (!context_fault_ok(c, err)) { set_err("llmi_generate_greedy_batch: " + err); return -6; }
    for (int k = 0; k < n; ++k) {
        for (int j = 0; j + 1 < n_gen; ++j) out[(size_t)k * n_gen + j] = h[(size_t)k * n_gen + j];
        out[(size_t)k * n_gen + n_gen - 1] = (llama_token)key_token(keys.data() + (size_t)k * kArgSlots);
        set_seq_past(c, seqs[k], pos0[k] + n_gen);
    }
    float ms = 0.f;
    hipEventElapsedTime(&ms, c.ev0, c.ev1);
    c.last_us = ms * 1e3;
    c.last_bytes = bytes;
    c.n_outputs = 0;
    (void)max_end;
    return n_gen;
    API_CATCH(-5)
}

bool llama_kv_self_seq_rm(struct llama_context* ctx, llama_seq_id seq_id, llama_pos p0, llama_pos p1) {
    if (!ctx) return false;
    Context& c = ctx->c;
    if (seq_id >= c.n_seq) return false;
    if (p1 >= 0) { set_err("llama_kv_self_seq_rm: only tail removal [p0, inf) is supported"); return false; }
    const int lo = seq_id < 0 ? 0 : seq_id, hi = seq_id < 0 ? c.n_seq : seq_id + 1;
    (void)hipSetDevice(c.device);
    for (int s = lo; s < hi; ++s) {
        if (p0 <= 0) {
            context_clear_seq(c, s);
        } else {
            // positions >= p0 are rewritten before any step attends to them (a step at
            // position p reads KV rows [0, p]): truncation is a bookkeeping change
            set_seq_past(c, s, std::min(seq_past_of(c, s), (int)p0));
        }
    }
    return true;
}

int32_t llmi_seq_pos_max(const struct llama_context* ctx, llama_seq_id seq_id) {
    if (!ctx || seq_id < 0 || seq_id >= ctx->c.n_seq) return -1;
    return seq_past_of(ctx->c, seq_id) - 1;
}

int32_t llmi_profile_kernels(struct llama_context* ctx, llama_token first, int32_t pos0, int32_t n_steps, double* us,
                             double* bytes, int32_t* launches) {
    API_TRY
    if (!ctx || n_steps <= 0 || !us || !bytes || !launches) { set_err("llmi_profile_kernels: bad arguments"); return -1; }
    Context& c = ctx->c;
    if (first < 0 || first >= c.m->hp.n_vocab || pos0 < 0 || pos0 >= c.n_ctx) {
        set_err("llmi_profile_kernels: token/position out of range");
        return -1;
    }
    (void)hipSetDevice(c.m->device);
    // In situ: n_steps whole decode steps at position pos0 (the decode graph's exact
    // kernels, grids and arguments, in their order), launched one by one with EVERY
    // kernel armed with an event pair that the runtime records when it starts and ends
    // (hipExtLaunchKernelGGL): each kernel's execution time in its real place in the
    // step (caches as its predecessor leaves them), without launch gaps.  One warm step
    // first.  No tokens are consumed: the state is reset to (first, pos0) afterwards.
    const int kv_bound = std::min(c.n_ctx, (pos0 / 256 + 1) * 256);
    std::string err;
    int rc = 0;
    {
        Prof warm;
        if (launch_state_set(c.st, first, pos0, c.stream) != hipSuccess) { set_err("state set failed"); return -3; }
        c.prof = &warm;
        bool ok = step_enqueue(c, kv_bound, err);
        Prof pk;
        pk.timed = true;
        for (int r = 0; ok && r < n_steps; ++r) {
            if (launch_state_set(c.st, first, pos0, c.stream) != hipSuccess) { ok = false; break; }
            c.prof = &pk;
            ok = step_enqueue(c, kv_bound, err);
        }
        c.prof = nullptr;
        if (!ok || hipStreamSynchronize(c.stream) != hipSuccess) {
            set_err("llmi_profile_kernels: " + (err.empty() ? std::string("launch failed") : err));
            rc = -4;
        }
        for (int k = 0; rc == 0 && k < K_NCLASS; ++k) {
            int used = 0;
            const double t = pk.elapsed_us(k, &used);
            const int n = std::max(1, pk.launches[k]);
            us[k] = used ? t / (double)used : 0.0;
            bytes[k] = (pk.bytes[k] + pk.per_kv[k] * (double)(pos0 + 1)) / n;
            launches[k] = pk.launches[k] / n_steps;
        }
    }
    if (launch_state_set(c.st, first, pos0, c.stream) != hipSuccess || hipStreamSynchronize(c.stream) != hipSuccess) {
        if (rc == 0) { set_err("llmi_profile_kernels: state reset failed"); rc = -4; }
    }
    c.n_past = pos0;
    return rc;
    API_CATCH(-5)
}


int32_t llmi_engine_trace(struct llama_context* ctx, llama_token first, int32_t pos0, int32_t layer, uint64_t* out,
                          int64_t n_out) {
    API_TRY
    if (!ctx || !out) { set_err("llmi_engine_trace: bad arguments"); return -1; }
    Context& c = ctx->c;
    if (first < 0 || first >= c.m->hp.n_vocab || pos0 < 0 || pos0 >= c.n_ctx || layer < 0 || layer >= c.m->hp.n_layer) {
        set_err("llmi_engine_trace: token/position/layer out of range");
        return -1;
    }
    (void)hipSetDevice(c.m->device);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.m->device);
    const size_t n = (size_t)cus * 16 * 32;
    if ((size_t)n_out < n) { set_err("llmi_engine_trace: out holds fewer than CUs x 512 stamps"); return -1; }
    // one eager warm step, then one traced step at (first, pos0); the state is reset after
    const int kv_bound = std::min(c.n_ctx, (pos0 / 256 + 1) * 256);
    std::string err;
    int rc = 0;
    if (!c.le_trace && hipMalloc(&c.le_trace, n * 8) != hipSuccess) { set_err("llmi_engine_trace: hipMalloc"); return -3; }
    (void)hipMemsetAsync(c.le_trace, 0, n * 8, c.stream);
    bool ok = launch_state_set(c.st, first, pos0, c.stream) == hipSuccess && step_enqueue(c, kv_bound, err);
    c.le_trace_layer = layer;
    ok = ok && launch_state_set(c.st, first, pos0, c.stream) == hipSuccess && step_enqueue(c, kv_bound, err);
    c.le_trace_layer = -1;
    if (!ok || hipMemcpyAsync(out, c.le_trace, n * 8, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
        hipStreamSynchronize(c.stream) != hipSuccess) {
        set_err("llmi_engine_trace: " + (err.empty() ? std::string("launch failed") : err));
        rc = -4;
    }
    if (launch_state_set(c.st, first, pos0, c.stream) != hipSuccess || hipStreamSynchronize(c.stream) != hipSuccess)
        if (rc == 0) { set_err("llmi_engine_trace: state reset failed"); rc = -4; }
    c.n_past = pos0;
    return rc == 0 ? cus : rc;
    API_CATCH(-5)
}

double llmi_le_stream_bench(const void* src, int64_t bytes, int32_t mode, int32_t iters, int32_t nt) {
    return le_stream_bench(src, (size_t)bytes, mode, iters, nt);
}

// numerics of this thread's kernel-level entry points (llmi_test_option "numerics")
static thread_local int t_hook_numerics = 0;

int32_t llmi_test_option(const char* name, int32_t value) {
    if (!name) return -1;
    int* opt = nullptr;
    if (!strcmp(name, "numerics")) {
        const int old = t_hook_numerics;
        if (value >= 0 && value <= (NUMERICS_X86 | NUMERICS_FA)) t_hook_numerics = value;
        else if (value >= 0) { set_err("llmi_test_option: numerics must be 0..3"); return -1; }
        return old;
    }
    if (!strcmp(name, "pf_attn_simple")) opt = &g_pf_attn_simple;
    else if (!strcmp(name, "pf_fa_noalloc")) opt = &g_pf_fa_noalloc;
    else if (!strcmp(name, "pf_attn_fa")) opt = &g_pf_attn_fa;
    else if (!strcmp(name, "pf_gemm_ng")) opt = &g_pf_gemm_ng;
    else if (!strcmp(name, "pf_qkv_merge")) opt = &g_pf_qkv_merge;
    else if (!strcmp(name, "pf_xcd_map")) opt = &g_pf_xcd_map;
    else if (!strcmp(name, "pf_quant_bpc")) opt = &g_pf_quant_bpc;
    else if (!strcmp(name, "pf_quant_split_below")) opt = &g_pf_quant_split_below;
    else if (!strcmp(name, "pf_fa_cfg")) opt = &g_pf_fa_cfg;
    else if (!strcmp(name, "pf_max_kv")) opt = &g_pf_max_kv;
    else if (!strcmp(name, "xspin_limit")) opt = &g_xspin_limit;
    else if (!strcmp(name, "xtag_skew")) opt = &g_xtag_skew;
    else if (!strcmp(name, "engine")) opt = &g_le_on;      // layer engine on/off (contexts made after)
    else if (!strcmp(name, "le_spin")) opt = &g_le_spin;   // layer engine's bounded-wait polls
    if (!opt) { set_err("llmi_test_option: unknown option"); return -1; }
    const int old = *opt;
    if (value >= 0) *opt = value;
    return old;
}

void llmi_last_step_stats(struct llama_context* ctx, double* bytes, double* usec) {
    if (!ctx) return;
    if (bytes) *bytes = ctx->c.last_bytes;
    if (usec) *usec = ctx->c.last_us;
}

int32_t llmi_debug_tap(struct llama_context* ctx, int32_t which, float* out) {
    if (!ctx || !out) { set_err("llmi_debug_tap: bad arguments"); return -1; }
    Context& c = ctx->c;
    const HParams& hp = c.m->hp;
    (void)hipSetDevice(c.m->device);
    if (which == 7 || which == 8) {  // last layer's K ([HK][n_ctx][D]) or V ([HK][D][n_ctx]) cache, raw f16
        const size_t kvl = (size_t)hp.n_head_kv * c.n_ctx * hp.head_dim;
        const uint16_t* base = (which == 7 ? c.kc : c.vc) + (size_t)(hp.n_layer - 1) * kvl;
        hipError_t e = hipMemcpyAsync(out, base, kvl * 2, hipMemcpyDeviceToHost, c.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
        if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
        return 0;
    }
    if (which >= 11 && which <= 15) {  // batched-step buffers, kMaxBatch rows each
        const float* b = which == 11 ? c.bx : which == 12 ? c.bq : which == 13 ? c.batt : which == 14 ? c.bh : c.blogits;
        const size_t per = which == 11 ? hp.n_embd : which == 14 ? hp.n_ff : which == 15 ? hp.n_vocab
                                                                                     : (size_t)hp.n_head * hp.head_dim;
        if (!b) { set_err("llmi_debug_tap: no batched step ran"); return -1; }
        hipError_t e = hipMemcpy(out, b, per * kMaxBatch * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
        return 0;
    }
    if (which == 0) {  // the last step's embedding row (get_rows), recomputed by k_embed's dequant
        float* tmp = nullptr;
        if (hipMalloc(&tmp, (size_t)hp.n_embd * 4) != hipSuccess) { set_err("out of device memory"); return -2; }
        EmbArgs ea;
        ea.w = seg_of(*c.m, c.m->tok_embd, 0);
        ea.cols = hp.n_embd;
        ea.vocab = hp.n_vocab;
        hipError_t e = launch_embed_row(ea, c.st, tmp, c.stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out, tmp, (size_t)hp.n_embd * 4, hipMemcpyDeviceToHost, c.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
        (void)hipFree(tmp);
        if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
        return 0;
    }
    const float* src = which == 1 ? c.x : which == 2 ? c.q : which == 3 ? c.att : which == 4 ? c.h : nullptr;
    const size_t n = which == 1 ? hp.n_embd : which == 4 ? hp.n_ff : (size_t)hp.n_head * hp.head_dim;
    if (!src) { set_err("llmi_debug_tap: unknown tap"); return -1; }
    (void)hipSetDevice(c.m->device);
    hipError_t e = hipMemcpyAsync(out, src, n * 4, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
    return 0;
}

double llmi_model_upload_s(const struct llama_model* model) { return model ? model->m.upload_s : -1.0; }

int32_t llmi_prefill_supported(const struct llama_model* model) {
    return model && prefill_supported(model->m) ? 1 : 0;
}

double llmi_bytes_per_token(const struct llama_model* model, int32_t n_kv) {
    return model ? bytes_per_token(model->m, n_kv) : 0.0;
}

int32_t llmi_model_arena(const struct llama_model* model, void** dev_ptr, uint64_t* bytes) {
    if (!model) return -1;
    if (dev_ptr) *dev_ptr = model->m.arena;
    if (bytes) *bytes = model->m.arena_bytes;
    return 0;
}

// synchronous hash of device memory on `device` (launch_arena_hash, kernels.hip)
static bool device_hash(int device, const void* p, size_t bytes, uint64_t* out, std::string& err) {
    if (hipSetDevice(device) != hipSuccess) { err = "hipSetDevice"; return false; }
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 8) != hipSuccess) { err = "hipMalloc (hash)"; return false; }
    hipError_t e = launch_arena_hash(p, bytes, d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d, 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) { err = std::string("arena hash: ") + hipGetErrorString(e); return false; }
    return true;
}

int32_t llmi_model_arena_hash(const struct llama_model* model, uint64_t* out) {
    API_TRY
    if (!model || !out || !model->m.arena) { set_err("llmi_model_arena_hash: bad arguments"); return -1; }
    std::string err;
    if (!device_hash(model->m.device, model->m.arena, model->m.arena_bytes, out, err)) { set_err(err); return -2; }
    return 0;
    API_CATCH(-5)
}

int32_t llmi_device_hash(const void* dev_ptr, uint64_t bytes, uint64_t* out) {
    API_TRY
    if (!dev_ptr || !out) { set_err("llmi_device_hash: bad arguments"); return -1; }
    hipPointerAttribute_t at{};
    int dev = 0;
    if (hipPointerGetAttributes(&at, dev_ptr) == hipSuccess && at.device >= 0) dev = at.device;
    else (void)hipGetDevice(&dev);
    std::string err;
    if (!device_hash(dev, dev_ptr, (size_t)bytes, out, err)) { set_err(err); return -2; }
    return 0;
    API_CATCH(-5)
}

// ---- replica fan-out ------------------------------------------------
// The arena goes out in kFanoutChunk (256 MB) pieces on real streams.  When the source is
// still uploading (llmi_model_load_fanout / llmi_model_load_replicated), piece k is issued
// as soon as the upload stream has completed the arena prefix that covers it (an event on
// the upload stream, waited on by the broadcast streams), so the xGMI broadcast runs
// behind the host-to-device copy instead of after it.  engine.cpp fanout_plan states the
// schedule; tests/test_fanout_plan.py checks it.
namespace {
struct Fanout {
    // one rank per entry: (device, arena, comm, stream); entry 0 is the root
    std::vector<int> dev;
    std::vector<uint8_t*> buf;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> st;
    size_t bytes = 0, next = 0;  // arena bytes; first piece not yet issued
    std::vector<hipEvent_t> evs;
    bool ok = true;        // every step so far succeeded
    bool nccl_ok = true;   // no ncclBroadcast failed: pieces must still be issued (the other
                           // ranks wait in their matching broadcasts), whatever else failed

    ~Fanout() {
        for (size_t r = 0; r < st.size(); ++r) {
            (void)hipSetDevice(dev[r]);
            if (st[r]) (void)hipStreamSynchronize(st[r]);
        }
        for (size_t r = 0; r < comm.size(); ++r)
            if (comm[r]) ncclCommDestroy(comm[r]);
        for (size_t r = 0; r < st.size(); ++r) {
            (void)hipSetDevice(dev[r]);
            if (st[r]) (void)hipStreamDestroy(st[r]);
        }
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
    bool make_streams() {
        st.assign(dev.size(), nullptr);
        for (size_t r = 0; r < dev.size(); ++r) {
            if (hipSetDevice(dev[r]) != hipSuccess) return false;
            if (hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking) != hipSuccess) return false;
        }
        return true;
    }
    // issue every piece that ends at or before `prefix` (all of them if prefix >= bytes);
    // `wait`: an event on the root's upload stream the broadcast streams wait on first
    bool issue(size_t prefix, hipEvent_t wait) {
        bool waited = false;
        while (nccl_ok && next * kFanoutChunk < bytes) {
            const size_t off = next * kFanoutChunk, len = std::min(kFanoutChunk, bytes - off);
            if (off + len > prefix) break;
            if (wait && !waited) {
                for (size_t r = 0; r < dev.size(); ++r) {
                    (void)hipSetDevice(dev[r]);
                    if (hipStreamWaitEvent(st[r], wait, 0) != hipSuccess) {
                        ok = false;  // the piece still goes out, after the upload reached it
                        (void)hipEventSynchronize(wait);
                    }
                }
                waited = true;
            }
            ncclResult_t nr = dev.size() > 1 ? ncclGroupStart() : ncclSuccess;
            for (size_t r = 0; r < dev.size() && nr == ncclSuccess; ++r) {
                (void)hipSetDevice(dev[r]);
                nr = ncclBroadcast(buf[r] + off, buf[r] + off, len, ncclUint8, 0, comm[r], st[r]);
            }
            if (dev.size() > 1) {
                const ncclResult_t ne = ncclGroupEnd();
                if (nr == ncclSuccess) nr = ne;
            }
            if (nr != ncclSuccess) ok = nccl_ok = false;
            ++next;
        }
        return ok;
    }
    bool finish() {
        issue(bytes, nullptr);
        for (size_t r = 0; r < dev.size(); ++r) {
            (void)hipSetDevice(dev[r]);
            if (hipStreamSynchronize(st[r]) != hipSuccess) ok = false;
        }
        return ok;
    }
    // After finish(): the root's {status, arena hash} goes to every rank of the
    // communicator (one more broadcast, so every rank leaves the fan-out together), and
    // each rank compares its own arena's hash with the root's.  root_ok: the caller's own
    // view of the root's load (upload + pieces).  Returns whether THIS process's ranks
    // hold the root's bytes; err says why not.  (a rank used to return
    // success with a partly written arena when the root's upload failed.)
    bool verify(bool root_ok, std::string& err) {
        if (comm.empty()) return root_ok;
        const size_t n = dev.size();
        std::vector<uint64_t> own(n, 0);
        bool hashed = true;
        for (size_t r = 0; r < n; ++r) {
            std::string e;
            if (!device_hash(dev[r], buf[r], bytes, &own[r], e)) { hashed = false; err = e; }
        }
        std::vector<unsigned long long*> w(n, nullptr);
        bool alloc = true;
        for (size_t r = 0; r < n; ++r) {
            (void)hipSetDevice(dev[r]);
            if (hipMalloc(&w[r], 16) != hipSuccess) alloc = false;
        }
        // the root's words: status (0 ok), its arena hash; other ranks' buffers are overwritten
        const bool is_root = rank0;
        uint64_t msg[2] = {(root_ok && hashed) ? 0ull : 1ull, own[0]};
        for (size_t r = 0; r < n && alloc; ++r) {
            (void)hipSetDevice(dev[r]);
            if (hipMemcpy(w[r], msg, 16, hipMemcpyHostToDevice) != hipSuccess) alloc = false;
        }
        bool ok_all = alloc;
        if (alloc) {
            ncclResult_t nr = n > 1 ? ncclGroupStart() : ncclSuccess;
            for (size_t r = 0; r < n && nr == ncclSuccess; ++r) {
                (void)hipSetDevice(dev[r]);
                nr = ncclBroadcast(w[r], w[r], 16, ncclUint8, 0, comm[r], st[r]);
            }
            if (n > 1) {
                const ncclResult_t ne = ncclGroupEnd();
                if (nr == ncclSuccess) nr = ne;
            }
            if (nr != ncclSuccess) { ok_all = false; err = "status broadcast failed"; }
            for (size_t r = 0; r < n && ok_all; ++r) {
                (void)hipSetDevice(dev[r]);
                uint64_t got[2] = {1, 0};
                if (hipStreamSynchronize(st[r]) != hipSuccess ||
                    hipMemcpy(got, w[r], 16, hipMemcpyDeviceToHost) != hipSuccess) {
                    ok_all = false;
                    err = "status read back failed";
                } else if (got[0] != 0) {
                    ok_all = false;
                    if (err.empty()) err = is_root && r == 0 ? "the upload failed" : "the root rank's upload failed";
                } else if (!hashed || got[1] != own[r]) {
                    ok_all = false;
                    if (err.empty()) err = "arena hash of rank-local replica differs from the root's";
                }
            }
        } else if (err.empty()) {
            err = "status buffers";
        }
        for (size_t r = 0; r < n; ++r) {
            (void)hipSetDevice(dev[r]);
            if (w[r]) (void)hipFree(w[r]);
        }
        (void)hipSetDevice(dev[0]);
        return ok_all;
    }
    bool rank0 = true;  // entry 0 is the communicator's root (in-process fan-outs, rank 0)
    // the model_load hook of the root: record the prefix on the upload stream, issue what it covers
    UploadHook hook() {
        return [this](size_t prefix_end, hipStream_t us) -> bool {
            hipEvent_t e = nullptr;
            (void)hipSetDevice(dev[0]);
            bool local = hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
            if (local) {
                evs.push_back(e);
                local = hipEventRecord(e, us) == hipSuccess;
            }
            if (!local) {  // no event to order the pieces behind the upload: wait for it here
                ok = false;
                (void)hipStreamSynchronize(us);
            }
            issue(prefix_end, local ? e : nullptr);
            (void)hipSetDevice(dev[0]);
            return ok;  // false aborts the upload; finish() still issues every remaining piece
        };
    }
};

bool check_replica_devices(int src, const int32_t* devices, int32_t n, const char* who) {
    const int nd = llmi_device_count();
    std::vector<int> seen{src};
    for (int i = 0; i < n; ++i) {
        if (devices[i] < 0 || devices[i] >= nd) { set_err(std::string(who) + ": device index out of range"); return false; }
        if (std::find(seen.begin(), seen.end(), devices[i]) != seen.end()) {
            set_err(std::string(who) + ": device " + std::to_string(devices[i]) +
                    " listed twice (or the source model's own device)");
            return false;
        }
        seen.push_back(devices[i]);
    }
    return true;
}

// in-process replicas: layouts on `devices`, one communicator over {src, devices...}
bool replica_setup(const Model& src, const int32_t* devices, int32_t n, std::vector<llama_model*>& reps, Fanout& F,
                   std::string& err) {
    reps.assign((size_t)n, nullptr);
    for (int i = 0; i < n; ++i) {
        reps[(size_t)i] = new llama_model();
        if (!model_clone_layout(src, devices[i], reps[(size_t)i]->m, err)) return false;
    }
    F.dev.push_back(src.device);
    F.buf.push_back(src.arena);
    for (int i = 0; i < n; ++i) {
        F.dev.push_back(devices[i]);
        F.buf.push_back(reps[(size_t)i]->m.arena);
    }
    F.bytes = src.arena_bytes;
    F.comm.assign(F.dev.size(), nullptr);
    if (ncclCommInitAll(F.comm.data(), (int)F.dev.size(), F.dev.data()) != ncclSuccess) {
        F.comm.clear();
        err = "ncclCommInitAll failed";
        return false;
    }
    if (!F.make_streams()) { err = "replica streams"; return false; }
    return true;
}
}  // namespace

int32_t llmi_replicate(struct llama_model* model, const int32_t* devices, int32_t n, struct llama_model** out) {
    API_TRY
    if (!model || !devices || n <= 0 || !out) { set_err("llmi_replicate: bad arguments"); return -1; }
    // one RCCL rank per device: a device listed twice (or the source's own device) would
    // put two ranks of the communicator on one GPU
    if (!check_replica_devices(model->m.device, devices, n, "llmi_replicate")) return -1;
    std::vector<llama_model*> reps;
    std::string err;
    int rc = 0;
    {
        Fanout F;
        if (!replica_setup(model->m, devices, n, reps, F, err)) rc = -2;
        else if (!F.finish()) { err = "ncclBroadcast failed"; rc = -4; (void)F.verify(false, err); }
        else if (!F.verify(true, err)) rc = -6;
    }
    if (rc) {
        set_err("llmi_replicate: " + err);
        for (auto* r : reps) delete r;
        return rc;
    }
    for (int i = 0; i < n; ++i) out[i] = reps[(size_t)i];
    return 0;
    API_CATCH(-5)
}

struct llama_model* llmi_model_load_replicated(const char* path, struct llama_model_params params, const int32_t* devices,
                                               int32_t n, struct llama_model** out) {
    API_TRY
    if (!path || (n > 0 && (!devices || !out)) || n < 0 || params.vocab_only || params.no_upload) {
        set_err("llmi_model_load_replicated: bad arguments");
        return nullptr;
    }
    if (params.n_gpu_layers == 0) {
        set_err("llmi_model_load_replicated: n_gpu_layers=0 requests the CPU path; llmi is GPU-only");
        return nullptr;
    }
    const int nd = llmi_device_count();
    if (nd <= 0) { set_err("no HIP device visible"); return nullptr; }
    if (params.main_gpu < 0 || params.main_gpu >= nd) { set_err("main_gpu out of range"); return nullptr; }
    if (!check_replica_devices(params.main_gpu, devices, n, "llmi_model_load_replicated")) return nullptr;
    auto* m = new llama_model();
    std::string err;
    // the layout first (no upload), then the replicas and the communicator, then the
    // upload with the pieces going out behind it
    if (!model_load(path, params.main_gpu, false, true, m->m, err, nullptr, params.numerics)) {
        set_err(err);
        delete m;
        return nullptr;
    }
    std::vector<llama_model*> reps;
    bool ok = true;
    {
        Fanout F;
        if (n > 0) ok = replica_setup(m->m, devices, n, reps, F, err);
        if (ok) {
            const UploadHook h = F.hook();
            ok = model_upload(m->m, err, n > 0 ? &h : nullptr);
            if (n > 0) {
                // every piece and the status go out even after a failed upload (every
                // replica learns it), then each replica's hash is checked against the root's
                const bool pieces = F.finish();
                if (ok && !pieces) { err = "ncclBroadcast failed"; ok = false; }
                std::string verr;
                if (!F.verify(ok, verr) && ok) { err = verr; ok = false; }
            }
        }
    }
    if (!ok) {
        set_err("llmi_model_load_replicated: " + err);
        for (auto* r : reps) delete r;
        delete m;
        return nullptr;
    }
    for (int i = 0; i < n; ++i) out[i] = reps[(size_t)i];
    return m;
    API_CATCH(nullptr)
}

int32_t llmi_rccl_unique_id(uint8_t* out, int32_t n) {
    if (!out || n < (int32_t)sizeof(ncclUniqueId)) { set_err("llmi_rccl_unique_id: buffer too small"); return -1; }
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) { set_err("ncclGetUniqueId failed"); return -2; }
    std::memcpy(out, &id, sizeof id);
    return 0;
}

namespace {
bool proc_fanout_init(Fanout& F, const Model& m, const uint8_t* uid, int32_t nranks, int32_t rank) {
    (void)hipSetDevice(m.device);
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    F.dev = {m.device};
    F.buf = {m.arena};
    F.bytes = m.arena_bytes;
    F.comm.assign(1, nullptr);
    if (ncclCommInitRank(&F.comm[0], nranks, id, rank) != ncclSuccess) {
        F.comm.clear();
        set_err("ncclCommInitRank failed");
        return false;
    }
    if (!F.make_streams()) { set_err("fan-out stream"); return false; }
    return true;
}
}  // namespace

int32_t llmi_model_fanout(struct llama_model* model, const uint8_t* uid, int32_t nranks, int32_t rank) {
    API_TRY
    if (!model || !uid || nranks <= 0 || rank < 0 || rank >= nranks || !model->m.arena) {
        set_err("llmi_model_fanout: bad arguments");
        return -1;
    }
    if (nranks == 1) return 0;
    Fanout F;
    if (!proc_fanout_init(F, model->m, uid, nranks, rank)) return -2;
    F.rank0 = rank == 0;
    const bool pieces = F.finish();
    std::string err;
    if (!F.verify(pieces || rank != 0, err)) { set_err("llmi_model_fanout: " + err); return pieces ? -6 : -3; }
    if (!pieces) { set_err("llmi_model_fanout: broadcast failed"); return -3; }
    return 0;
    API_CATCH(-5)
}

struct llama_model* llmi_model_load_fanout(const char* path, struct llama_model_params params, const uint8_t* uid,
                                           int32_t nranks, int32_t rank) {
    API_TRY
    if (!path || !uid || nranks <= 0 || rank < 0 || rank >= nranks || params.vocab_only) {
        set_err("llmi_model_load_fanout: bad arguments");
        return nullptr;
    }
    if (params.n_gpu_layers == 0) {
        set_err("llmi_model_load_fanout: n_gpu_layers=0 requests the CPU path; llmi is GPU-only");
        return nullptr;
    }
    const int nd = llmi_device_count();
    if (nd <= 0) { set_err("no HIP device visible"); return nullptr; }
    if (params.main_gpu < 0 || params.main_gpu >= nd) { set_err("main_gpu out of range"); return nullptr; }
    auto* m = new llama_model();
    std::string err;
    if (!model_load(path, params.main_gpu, false, true, m->m, err, nullptr, params.numerics)) {
        set_err(err);
        delete m;
        return nullptr;
    }
    bool ok = true;
    if (nranks > 1) {
        Fanout F;
        ok = proc_fanout_init(F, m->m, uid, nranks, rank);
        F.rank0 = rank == 0;
        if (ok && rank == 0) {
            const UploadHook h = F.hook();
            ok = model_upload(m->m, err, &h);
            if (!ok) set_err(err);
        }
        // every piece is issued even after a failed upload: the other ranks are blocked in
        // their matching broadcasts and would otherwise never return
        if (!F.comm.empty()) {
            const bool pieces = F.finish();
            if (!pieces && ok) { set_err("llmi_model_load_fanout: broadcast failed"); ok = false; }
            // then the root's status + arena hash: a rank whose root failed (or whose
            // replica differs) returns NULL instead of a partly written arena
            std::string verr;
            if (!F.verify(rank == 0 ? ok : true, verr) && ok) {
                set_err("llmi_model_load_fanout: " + verr);
                ok = false;
            }
        }
    } else {
        ok = model_upload(m->m, err, nullptr);
        if (!ok) set_err(err);
    }
    if (!ok) {
        delete m;
        return nullptr;
    }
    return m;
    API_CATCH(nullptr)
}

int32_t llmi_fanout_plan(uint64_t arena_bytes, uint64_t chunk, const uint64_t* prefix_ends, int32_t n_prefix,
                         int32_t* ready, int32_t max_pieces) {
    if (n_prefix < 0 || (n_prefix > 0 && !prefix_ends) || max_pieces < 0 || (max_pieces > 0 && !ready)) return -1;
    API_TRY
    std::vector<size_t> pe(prefix_ends, prefix_ends + n_prefix);
    std::vector<int> rd;
    const size_t n = fanout_plan((size_t)arena_bytes, (size_t)chunk, pe, rd);
    for (size_t k = 0; k < n && (int32_t)k < max_pieces; ++k) ready[k] = rd[k];
    return (int32_t)n;
    API_CATCH(-5)
}

const struct llama_vocab* llama_model_get_vocab(const struct llama_model* model) {
    return model ? vocab_handle(model) : nullptr;
}
int32_t llama_vocab_n_tokens(const struct llama_vocab* v) {
    return !v ? 0 : v->m ? v->m->hp.n_vocab : (int32_t)v->tok->tokens.size();
}
llama_token llama_vocab_bos(const struct llama_vocab* v) { return v ? v->tok->bos : -1; }
llama_token llama_vocab_eos(const struct llama_vocab* v) { return v ? v->tok->eos : -1; }
const char* llama_vocab_get_text(const struct llama_vocab* v, llama_token t) {
    if (!v || t < 0 || t >= (int)v->tok->tokens.size()) return nullptr;
    return v->tok->tokens[(size_t)t].c_str();
}
bool llama_vocab_get_add_bos(const struct llama_vocab* v) { return v && v->tok->add_bos; }

// upstream llama_tokenize: the count, or -(count) when n_tokens_max is too small
int32_t llama_tokenize(const struct llama_vocab* v, const char* text, int32_t text_len, llama_token* tokens,
                       int32_t n_tokens_max, bool add_special, bool parse_special) {
    if (!v || (!text && text_len > 0) || text_len < 0) {
        set_err("llama_tokenize: bad arguments");
        return INT32_MIN;
    }
    try {
        const std::vector<int32_t> ids = v->tok->tokenize(std::string(text ? text : "", (size_t)text_len), add_special,
                                                          parse_special);
        if ((int64_t)ids.size() > (int64_t)INT32_MAX) {
            set_err("llama_tokenize: too many tokens");
            return INT32_MIN;
        }
        const int32_t n = (int32_t)ids.size();
        if (n > n_tokens_max) return -n;
        for (int32_t i = 0; i < n; ++i) tokens[i] = ids[(size_t)i];
        return n;
    } catch (const std::exception& e) {
        set_err(std::string("llama_tokenize: ") + e.what());
        return INT32_MIN;
    }
}

// upstream llama_token_to_piece: bytes written (no NUL), or -(bytes needed); up to
// lstrip leading spaces are skipped; special renders CONTROL tokens as their text
int32_t llama_token_to_piece(const struct llama_vocab* v, llama_token token, char* buf, int32_t length, int32_t lstrip,
                             bool special) {
    if (!v) return 0;
    API_TRY
    std::string p = v->tok->piece(token, special);
    size_t k = 0;
    while (lstrip > 0 && k < p.size() && p[k] == ' ') {
        ++k;
        --lstrip;
    }
    const int32_t n = (int32_t)(p.size() - k);
    if (n > length) return -n;
    if (n > 0) memcpy(buf, p.data() + k, (size_t)n);
    return n;
    API_CATCH(INT32_MIN)
}

// upstream llama_detokenize: the pieces concatenated; remove_special drops a leading BOS
// (when the vocabulary adds one) and a trailing EOS (when it adds one: add_eos_token);
// unparse_special renders CONTROL text.
// Bytes written, or -(bytes needed).
int32_t llama_detokenize(const struct llama_vocab* v, const llama_token* tokens, int32_t n_tokens, char* text,
                         int32_t text_len_max, bool remove_special, bool unparse_special) {
    if (!v || n_tokens < 0 || (!tokens && n_tokens > 0)) return INT32_MIN;
    API_TRY
    int32_t b = 0, e = n_tokens;
    if (remove_special && e > b && v->tok->add_bos && tokens[b] == v->tok->bos) ++b;
    if (remove_special && e > b && v->tok->add_eos && tokens[e - 1] == v->tok->eos) --e;
    std::string out;
    for (int32_t i = b; i < e; ++i) out += v->tok->piece(tokens[i], unparse_special);
    if ((int64_t)out.size() > (int64_t)text_len_max) return -(int32_t)out.size();
    if (!out.empty()) memcpy(text, out.data(), out.size());
    return (int32_t)out.size();
    API_CATCH(INT32_MIN)
}

// a tokenizer-only handle from a GGUF's metadata (no tensors needed)
struct llama_vocab* llmi_vocab_load_from_file(const char* path) {
    API_TRY
    GgufFile f;
    std::string err;
    if (!path || !f.open(path, err)) {
        set_err(err.empty() ? "llmi_vocab_load_from_file: no path" : err);
        return nullptr;
    }
    const GgufTensor* te = f.tensor("token_embd.weight");
    auto v = std::make_unique<llama_vocab>();
    v->m = nullptr;
    v->owned = Tokenizer::from_gguf(f, te ? (int)te->ne[1] : 0);
    v->tok = v->owned.get();
    return v.release();
    API_CATCH(nullptr)
}
void llmi_vocab_free(struct llama_vocab* v) {
    if (v && v->owned) delete v;
}
int32_t llama_model_n_embd(const struct llama_model* m) { return m ? m->m.hp.n_embd : 0; }
int32_t llama_model_n_layer(const struct llama_model* m) { return m ? m->m.hp.n_layer : 0; }
int32_t llama_model_n_head(const struct llama_model* m) { return m ? m->m.hp.n_head : 0; }
int32_t llama_model_n_head_kv(const struct llama_model* m) { return m ? m->m.hp.n_head_kv : 0; }
int32_t llama_model_n_ctx_train(const struct llama_model* m) { return m ? m->m.hp.n_ctx_train : 0; }
uint64_t llama_model_size(const struct llama_model* m) { return m ? (uint64_t)model_tensor_bytes(m->m) : 0; }
int32_t llama_model_desc(const struct llama_model* m, char* buf, size_t n) {
    if (!m) return -1;
    return snprintf(buf, n, "%s", m->m.desc.c_str());
}
uint32_t llama_n_ctx(const struct llama_context* ctx) { return ctx ? (uint32_t)ctx->c.n_ctx : 0; }
void llama_kv_self_clear(struct llama_context* ctx) {
    if (ctx) context_clear(ctx->c);
}

int64_t llmi_synth_write_gguf(const char* path, const char* preset, uint64_t seed, int32_t n_layer, int32_t n_vocab,
                              int32_t n_threads) {
    API_TRY
    if (!path || !preset) { set_err("null argument"); return -1; }
    std::string err;
    int64_t r = synth_write_gguf(path, preset, seed, n_layer, n_vocab, n_threads, err);
    if (r < 0) set_err(err);
    return r;
    API_CATCH(-1)
}

// ---------------- kernel-level entry points (tests / microbenchmarks) ----------------
static Seg seg_at(int32_t type, const void* w, int64_t rows, int64_t cols) {
    DevMat dm;
    dm.type = type;
    dm.rows = rows;
    dm.cols = cols;
    plan_planes(dm, 0);
    Seg s;
    s.a = (const uint8_t*)w + dm.off_a;
    s.h = (const uint8_t*)w + dm.off_h;
    s.s = (const uint8_t*)w + dm.off_s;
    s.d = (const uint8_t*)w + dm.off_d;
    s.type = type;
    s.rows = (int)rows;
    s.row0 = 0;
    s.rgs = dm.rgs;
    s.x86 = (t_hook_numerics & NUMERICS_X86) != 0;
    return s;
}

int64_t llmi_device_layout_bytes(int32_t type, int64_t rows, int64_t cols) {
    if (!type_supported(type) || cols % block_elems(type)) return -1;
    DevMat dm;
    dm.type = type; dm.rows = rows; dm.cols = cols;
    return (int64_t)plan_planes(dm, 0);
}

int32_t llmi_repack(int32_t type, const void* raw, void* w, int64_t rows, int64_t cols) {
    if (!type_supported(type) || cols % block_elems(type)) { set_err("bad type/shape"); return -1; }
    DevMat dm;
    dm.type = type; dm.rows = rows; dm.cols = cols;
    plan_planes(dm, 0);
    hipError_t e;
    if (needs_repack(type)) {
        e = launch_repack(type, raw, (uint8_t*)w + dm.off_a, (uint8_t*)w + dm.off_h, (uint8_t*)w + dm.off_s,
                          (uint8_t*)w + dm.off_d, rows * (cols / block_elems(type)), cols, dm.rgs,
                          (t_hook_numerics & NUMERICS_X86) != 0, nullptr);
    } else {
        e = hipMemcpy(w, raw, dm.bytes, hipMemcpyDeviceToDevice);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
    return 0;
}

int32_t llmi_matvec(int32_t type, const void* w, int64_t rows, int64_t cols, const float* x, const float* nw, float eps,
                    float* y, int32_t mode) {
    if (!(type == T_Q4_K || type == T_Q5_K || type == T_Q6_K || type == T_Q8_0) || cols % 256 || rows <= 0) {
        set_err("llmi_matvec: unsupported type/shape");
        return -1;
    }
    MVArgs a;
    a.seg[0] = seg_at(type, w, rows, cols);
    a.nseg = 1;
    a.cols = (int)cols;
    a.npairs = (int)((rows + 1) / 2);
    a.x = x; a.nw = nw; a.eps = eps; a.y = y;
    a.num = t_hook_numerics & NUMERICS_X86;
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, dev);
    hipError_t e = launch_matvec(a, mode == 1 ? EPI_ADD : EPI_STORE, std::max(64, prop.multiProcessorCount * wg_per_cu()), nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
    return 0;
}

int32_t llmi_pf_gemm(int32_t type, const void* w, int64_t rows, int64_t cols, const float* x, const float* nw, float eps,
                     int32_t n_tok, float* y, double* usec) {
    if (!pf_gemm_ok(type, (int)rows, (int)cols) || n_tok <= 0) { set_err("llmi_pf_gemm: unsupported type/shape"); return -1; }
    const int x86 = (t_hook_numerics & NUMERICS_X86) != 0;
    const int tpad = (n_tok + 63) / 64 * 64;
    void* aq = nullptr;
    int16_t* abs = nullptr;
    float* ad = nullptr;
    void* abf = nullptr;
    hipError_t e = hipMalloc(&aq, (size_t)tpad * cols * 2);
    if (e == hipSuccess) e = hipMalloc(&abf, (size_t)tpad * (cols / 256) * 64);
    if (e == hipSuccess) e = hipMemset(abf, 0, (size_t)tpad * (cols / 256) * 64);
    if (e == hipSuccess) e = hipMalloc(&abs, (size_t)tpad * (cols / 16) * 2);
    if (e == hipSuccess) e = hipMalloc(&ad, (size_t)tpad * (cols / 32) * 4);
    if (e == hipSuccess) e = hipMemset(aq, 0, (size_t)tpad * cols * 2);
    if (e == hipSuccess) e = hipMemset(abs, 0, (size_t)tpad * (cols / 16) * 2);
    if (e == hipSuccess) e = hipMemset(ad, 0, (size_t)tpad * (cols / 32) * 4);
    if (e == hipSuccess) e = launch_pf_quant(x, (int)cols, nw, eps, (int)cols, act_kind(type), n_tok, aq, abs, ad, abf, nullptr, x86);
    PfGemm g;
    g.w = seg_at(type, w, rows, cols); g.rows = (int)rows; g.cols = (int)cols; g.T = n_tok;
    g.aq = aq; g.abs = abs; g.ad = ad; g.abf = abf; g.y = y; g.ldy = (int)rows;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (e == hipSuccess && usec) { (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventRecord(e0, nullptr); }
    if (e == hipSuccess) e = launch_pf_gemm(g, EPI_STORE, nullptr);
    if (e == hipSuccess && usec) {
        (void)hipEventRecord(e1, nullptr);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        *usec = ms * 1e3;
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(aq); (void)hipFree(abs); (void)hipFree(ad); (void)hipFree(abf);
    if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
    return 0;
}

int32_t llmi_quantize_act(int32_t type, int64_t cols, const float* x, const float* nw, float eps, void* out) {
    if (cols % 256) { set_err("cols must be a multiple of 256"); return -1; }
    MVArgs a;
    a.cols = (int)cols; a.x = x; a.nw = nw; a.eps = eps;
    a.num = t_hook_numerics & NUMERICS_X86;
    hipError_t e = launch_quant_dump(a, act_kind(type), out, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) { set_err(hip_err(e)); return -2; }
    return 0;
}

double llmi_bench_matvec_ex(int32_t type, const void* w, int32_t n_mats, int64_t rows, int64_t cols, const float* x, float* y,
                            int32_t reps, int32_t mode) {
    const int64_t lb = llmi_device_layout_bytes(type, rows, cols);
    if (lb <= 0 || n_mats <= 0 || reps <= 0) { set_err("bad arguments"); return -1.0; }
    const size_t stride = align_up((size_t)lb, 4096);
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, dev);
    const int mb = std::max(64, prop.multiProcessorCount * wg_per_cu());
    float* nw = nullptr;
    StepState* st = nullptr;
    // mode bit 5: gate+up SwiGLU launch (rows = both halves; RMSNorm on), bit 6: residual-add
    // epilogue (ffn_down / attn_output)
    const bool swiglu = mode & 32, add = mode & 64;
    const bool norm = (mode & 1) || swiglu, logits = mode & 2, img = mode & 8;
    if (norm) {
        std::vector<float> ones((size_t)cols, 1.0f);
        if (hipMalloc(&nw, (size_t)cols * 4) != hipSuccess) { set_err("out of device memory"); return -1.0; }
        (void)hipMemcpy(nw, ones.data(), (size_t)cols * 4, hipMemcpyHostToDevice);
    }
    if (logits) {
        if (hipMalloc(&st, sizeof(StepState)) != hipSuccess) { (void)hipFree(nw); set_err("out of device memory"); return -1.0; }
        (void)hipMemset(st, 0, sizeof(StepState));
    }
    MVArgs a;
    a.nseg = 1; a.cols = (int)cols; a.npairs = (int)((rows + 1) / 2); a.x = x; a.y = y;
    a.nw = nw; a.eps = 1e-5f; a.xfirst = (mode & 4) ? 1 : (mode & 256) ? -1 : 0;  // mode bit 2: weights after x, bit 8: never
    if (mode & 16) a.prio_alt = prop.multiProcessorCount;  // mode bit 4 (experiment builds): alternating priority
    if (logits) { a.st = st; a.argmax = &st->key[0][0]; }
    uint8_t* xq = nullptr;  // mode bit 3: timing with a pre-quantized activation image (zeros)
    if (img) {
        if (hipMalloc(&xq, (size_t)(cols / 256) * 304) != hipSuccess) { set_err("out of device memory"); return -1.0; }
        (void)hipMemset(xq, 0, (size_t)(cols / 256) * 304);
        a.xq = xq;
    }
    const int epi = logits ? EPI_LOGITS : swiglu ? EPI_SWIGLU : add ? EPI_ADD : EPI_STORE;
    const size_t half = swiglu ? (size_t)llmi_device_layout_bytes(type, rows / 2, cols) : 0;
    // one graph of n_mats launches (one per weight copy), replayed: no host launch cost
    hipStream_t s = nullptr;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipGraph_t g = nullptr;
    hipGraphExec_t ex = nullptr;
    bool ok = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess;
    // mode bit 7: every launch reads copy 0 (its weights L2/MALL-hot from the launch before)
    const size_t wstride = (mode & 128) ? 0 : stride;
    for (int k = 0; ok && k < n_mats; ++k) {
        if (swiglu) {
            a.nseg = 2;
            a.seg[0] = seg_at(type, (const uint8_t*)w + wstride * k, rows / 2, cols);
            a.seg[1] = seg_at(type, (const uint8_t*)w + wstride * k + half, rows / 2, cols);
        } else {
            a.seg[0] = seg_at(type, (const uint8_t*)w + wstride * k, rows, cols);
        }
        ok = launch_matvec(a, epi, mb, s) == hipSuccess;
    }
    ok = (hipStreamEndCapture(s, &g) == hipSuccess) && ok && hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess;
    double res = -1.0;
    const int nrep = std::max(1, reps / n_mats);
    if (ok) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipGraphLaunch(ex, s);  // warm-up (code, TLB)
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < nrep; ++r) (void)hipGraphLaunch(ex, s);
        (void)hipEventRecord(e1, s);
        float ms = 0.f;
        if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess)
            res = (double)ms * 1e3 / ((double)nrep * n_mats);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    } else {
        set_err("llmi_bench_matvec: capture/launch failed");
    }
    if (ex) (void)hipGraphExecDestroy(ex);
    if (g) (void)hipGraphDestroy(g);
    (void)hipStreamDestroy(s);
    (void)hipFree(nw);
    (void)hipFree(st);
    (void)hipFree(xq);
    return res;
}

double llmi_bench_matvec(int32_t type, const void* w, int32_t n_mats, int64_t rows, int64_t cols, const float* x, float* y,
                         int32_t reps) {
    return llmi_bench_matvec_ex(type, w, n_mats, rows, cols, x, y, reps, 0);
}

double llmi_bench_stream(const void* dev, int32_t n_bufs, uint64_t stride, uint64_t bytes, int32_t reps, int32_t blocks) {
    unsigned* out = nullptr;
    if (hipMalloc(&out, 16) != hipSuccess) return -1.0;
    for (int k = 0; k < n_bufs; ++k) (void)launch_stream_read((const uint8_t*)dev + stride * k, bytes, out, blocks, nullptr);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; ++r) (void)launch_stream_read((const uint8_t*)dev + stride * (r % n_bufs), bytes, out, blocks, nullptr);
    hipEventRecord(e1, nullptr);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    (void)hipFree(out);
    return (double)ms * 1e3 / reps;
}

}  // extern "C"

// Attention microbenchmark (kernel level, no model): n_layers distinct KV caches of
// n_ctx = round256(n_kv) positions (>= 512 MB in total, so replays stream them from HBM
// like a decode step does), one launch per layer captured into a graph, `reps` graph
// replays timed between two events.  Returns microseconds per launch (incl. the
// dependent-launch gap), < 0 on error.  mode: attention path (0 auto, 1 fused, 2 split, 3 two-kernel).
int32_t llmi_attention(int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t n_kv, int32_t n_ctx, const float* q,
                       const uint16_t* kc, const uint16_t* vc, float* out, int32_t mode) {
    if (n_head <= 0 || n_head_kv <= 0 || n_head % n_head_kv || (head_dim != 64 && head_dim != 128) || n_kv <= 0 ||
        n_ctx < n_kv || n_ctx % 256 || !q || !kc || !vc || !out) {
        set_err("llmi_attention: bad arguments");
        return -1;
    }
    API_TRY
    float* scores = nullptr;
    StepState* st = nullptr;
    if (hipMalloc(&scores, attn_scratch_floats(n_head, n_ctx) * 4) != hipSuccess || hipMalloc(&st, sizeof(StepState)) != hipSuccess) {
        (void)hipFree(scores);
        set_err("llmi_attention: out of device memory");
        return -2;
    }
    StepState hs{};
    hs.pos = n_kv - 1;
    hs.pos_next = n_kv;
    hs.seq = 1;
    (void)hipMemcpy(st, &hs, sizeof(hs), hipMemcpyHostToDevice);
    (void)hipMemset(scores, 0, attn_scratch_floats(n_head, n_ctx) * 4);
    AttnArgs a;
    a.q = q; a.kc = kc; a.vc = vc; a.scores = scores; a.out = out; a.st = st; a.n_ctx = n_ctx;
    a.scale = 1.0f / sqrtf((float)head_dim);
    a.tmax = scores + (size_t)n_head * n_ctx;
    a.gran = (unsigned long long*)(scores + attn_gran_off(n_head, n_ctx));
    a.fault = (unsigned*)(scores + attn_gran_off(n_head, n_ctx) + 2 * (size_t)n_head * kXAttnMaxKV);
    a.num = t_hook_numerics & NUMERICS_X86;
    a.fa = (t_hook_numerics & NUMERICS_FA) ? 1 : 0;
    const int kv_bound = std::min(n_ctx, (n_kv + 255) / 256 * 256);
    hipError_t e = launch_attention(a, n_head, n_head_kv, head_dim, kv_bound, nullptr, mode);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    (void)hipFree(scores);
    (void)hipFree(st);
    if (e != hipSuccess) { set_err(std::string("llmi_attention: ") + hip_err(e)); return -3; }
    return 0;
    API_CATCH(-5)
}

double llmi_pf_attention(int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t T, int32_t pos0, int32_t n_ctx,
                         const float* q, const uint16_t* kc, const uint16_t* vc, float* out, int32_t mode,
                         int64_t scratch_bytes) {
    if (n_head <= 0 || n_head_kv <= 0 || n_head % n_head_kv || (head_dim != 64 && head_dim != 128) || T <= 0 ||
        pos0 < 0 || n_ctx % 256 || pos0 + T > n_ctx || pos0 + T > kPfAttnMaxKV || mode < 0 || mode > 2 || !q || !kc ||
        !vc || !out) {
        set_err("llmi_pf_attention: bad arguments");
        return -1;
    }
    API_TRY
    PfAttn at;
    at.q = q; at.out = out; at.ldq = n_head * head_dim; at.kc = kc; at.vc = vc;
    at.n_ctx = n_ctx; at.pos0 = pos0; at.gqa = n_head / n_head_kv; at.max_kv = pos0 + T;
    at.scale = 1.0f / sqrtf((float)head_dim);
    float* wsc = nullptr;
    if (mode == 0) {
        size_t bytes = pf_fa_scratch_bytes(n_head, n_head_kv, head_dim, std::max(T, 512), n_ctx);
        if (!bytes) { set_err("llmi_pf_attention: no tiled kernel for this head shape"); return -1; }
        if (scratch_bytes > 0) bytes = (size_t)scratch_bytes;
        if (hipMalloc(&wsc, bytes) != hipSuccess) { set_err("llmi_pf_attention: out of device memory"); return -2; }
        at.wsc = wsc; at.wsc_bytes = bytes;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, nullptr);
    hipError_t e = launch_pf_attn(at, n_head, head_dim, T, nullptr, mode);
    (void)hipEventRecord(e1, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    float ms = 0.f;
    if (e == hipSuccess) (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(wsc);
    if (e != hipSuccess) { set_err(std::string("llmi_pf_attention: ") + hip_err(e)); return -3; }
    return (double)ms * 1e3;
    API_CATCH(-5)
}

double llmi_bench_attention(int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t n_kv, int32_t mode, int32_t reps,
                            uint64_t* trace_dev) {
    if (n_head <= 0 || n_head_kv <= 0 || n_head % n_head_kv || (head_dim != 64 && head_dim != 128) || n_kv <= 0 || reps <= 0) {
        set_err("llmi_bench_attention: bad arguments");
        return -1.0;
    }
    const int n_ctx = (n_kv + 255) / 256 * 256;
    const size_t kv_layer = (size_t)n_head_kv * n_ctx * head_dim;  // elements per layer, K or V
    const int nl = (int)std::max<size_t>(2, (size_t)(512u << 20) / (kv_layer * 4) + 1);
    uint16_t *kc = nullptr, *vc = nullptr;
    float *q = nullptr, *scores = nullptr, *out = nullptr;
    StepState* st = nullptr;
    auto cleanup = [&] {
        (void)hipFree(kc); (void)hipFree(vc); (void)hipFree(q); (void)hipFree(scores); (void)hipFree(out); (void)hipFree(st);
    };
    if (hipMalloc(&kc, kv_layer * nl * 2) != hipSuccess || hipMalloc(&vc, kv_layer * nl * 2) != hipSuccess ||
        hipMalloc(&q, (size_t)n_head * head_dim * 4) != hipSuccess ||
        hipMalloc(&scores, attn_scratch_floats(n_head, n_ctx) * 4) != hipSuccess ||
        hipMalloc(&out, (size_t)n_head * head_dim * 4) != hipSuccess || hipMalloc(&st, sizeof(StepState)) != hipSuccess) {
        cleanup();
        set_err("llmi_bench_attention: out of device memory");
        return -1.0;
    }
    (void)hipMemset(kc, 0x3c, kv_layer * nl * 2);  // f16 0x3c3c ~ 1.06
    (void)hipMemset(vc, 0x3c, kv_layer * nl * 2);
    (void)hipMemset(q, 0, (size_t)n_head * head_dim * 4);
    StepState hs{};
    hs.pos = n_kv - 1;
    hs.pos_next = n_kv;
    (void)hipMemcpy(st, &hs, sizeof(hs), hipMemcpyHostToDevice);
    hipStream_t s = nullptr;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int kv_bound = std::min(n_ctx, (n_kv + 255) / 256 * 256);
    AttnArgs a;
    a.q = q; a.scores = scores; a.out = out; a.st = st; a.n_ctx = n_ctx; a.scale = 1.0f / sqrtf((float)head_dim);
    a.num = t_hook_numerics & NUMERICS_X86;
    a.tmax = scores + (size_t)n_head * n_ctx;
    a.gran = (unsigned long long*)(scores + attn_gran_off(n_head, n_ctx));
    a.fault = (unsigned*)(scores + attn_gran_off(n_head, n_ctx) + 2 * (size_t)n_head * kXAttnMaxKV);
    (void)hipMemset(scores, 0, attn_scratch_floats(n_head, n_ctx) * 4);
    if (trace_dev) {  // one traced eager launch on a cold layer (LLMI_EXP_TRACE builds)
        for (int l = 0; l + 1 < nl; ++l) {
            a.kc = kc + (size_t)l * kv_layer;
            a.vc = vc + (size_t)l * kv_layer;
            a.layer = l % 255;
            (void)launch_attention(a, n_head, n_head_kv, head_dim, kv_bound, s, mode);
        }
        a.kc = kc + (size_t)(nl - 1) * kv_layer;
        a.vc = vc + (size_t)(nl - 1) * kv_layer;
        a.layer = (nl - 1) % 255;
        a.trace = (unsigned long long*)trace_dev;
        const bool okt = launch_attention(a, n_head, n_head_kv, head_dim, kv_bound, s, mode) == hipSuccess &&
                         hipStreamSynchronize(s) == hipSuccess;
        (void)hipStreamDestroy(s);
        cleanup();
        return okt ? 0.0 : -1.0;
    }
    hipGraph_t g = nullptr;
    hipGraphExec_t ex = nullptr;
    bool ok = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess;
    // a new step sequence number per replay: k_attn_x's hand-off tags never repeat
    ok = ok && launch_state_tick(st, s) == hipSuccess;
    for (int l = 0; ok && l < nl; ++l) {
        a.kc = kc + (size_t)l * kv_layer;
        a.vc = vc + (size_t)l * kv_layer;
        a.layer = l % 255;
        ok = launch_attention(a, n_head, n_head_kv, head_dim, kv_bound, s, mode) == hipSuccess;
    }
    ok = (hipStreamEndCapture(s, &g) == hipSuccess) && ok && hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess;
    double res = -1.0;
    if (ok) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipGraphLaunch(ex, s);
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ex, s);
        (void)hipEventRecord(e1, s);
        float ms = 0.f;
        if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess)
            res = (double)ms * 1e3 / ((double)reps * nl);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    } else {
        set_err("llmi_bench_attention: capture/launch failed");
    }
    if (ex) (void)hipGraphExecDestroy(ex);
    if (g) (void)hipGraphDestroy(g);
    (void)hipStreamDestroy(s);
    cleanup();
    return res;
}

// Experiment hook (LLMI_EXP_TRACE builds): one STORE matvec launch with per-wave
// s_memrealtime stamps {entry, after prologue, first pair done, exit, HW_ID, XCC<<32|pairs}
// written to trace_dev[grid*waves*6]; returns the grid size, < 0 on error.
int32_t llmi_trace_matvec(int32_t type, const void* w, int64_t rows, int64_t cols, const float* x, float* y, int32_t mode,
                          uint64_t* trace_dev) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, dev);
    const int mb = std::max(64, prop.multiProcessorCount * wg_per_cu());
    MVArgs a;
    a.nseg = 1; a.cols = (int)cols; a.npairs = (int)((rows + 1) / 2); a.x = x; a.y = y;
    a.seg[0] = seg_at(type, w, rows, cols);
    a.trace = (unsigned long long*)trace_dev;
    if (mode & 256) a.xfirst = -1;  // mode bit 8: weights issued before the activation arrives
    uint8_t* xq = nullptr;  // mode bit 3: pre-quantized activation image (zeros)
    if ((mode & 8) && hipMalloc(&xq, (size_t)(cols / 256) * 304) == hipSuccess) {
        (void)hipMemset(xq, 0, (size_t)(cols / 256) * 304);
        a.xq = xq;
    }
    const bool ok = launch_matvec(a, EPI_STORE, mb, nullptr) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
    (void)hipFree(xq);
    if (!ok) {
        set_err("llmi_trace_matvec: launch failed");
        return -1;
    }
    return std::min(mb, (a.npairs + kMVWaves - 1) / kMVWaves);
}
