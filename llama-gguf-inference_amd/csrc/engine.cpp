// engine.cpp — GGUF model -> HBM arena, decode context, per-step kernel schedule.
//
// Replaces the parts of upstream libllama that sit on the decode path:
// llama_model_loader (a4), the llm_build_llama graph for one token (a5-a15) and the
// f16 KV cache (a16).  One decode step is 2 + 6*n_layer kernel launches, captured once
// per 256-position KV bucket into a HIP graph and replayed; the next token is fed back
// on the device (argmax key -> k_embed), so greedy generation needs no host round trip.
#include "engine.h"

#include <chrono>
#include <cstring>
#include <thread>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace llmi {

std::string hip_err(hipError_t e) { return std::string(hipGetErrorString(e)); }

int wg_per_cu() {  // read per call (context creation): tests vary it within a process
    const char* e = getenv("LLMI_WG_PER_CU");
    const int n = e ? atoi(e) : 0;
    return n > 0 ? n : 2;
}

#define HIPC(expr)                                                         \
    do {                                                                   \
        hipError_t e_ = (expr);                                            \
        if (e_ != hipSuccess) {                                            \
            err = std::string(#expr) + ": " + hip_err(e_);                 \
            return false;                                                  \
        }                                                                  \
    } while (0)

Model::~Model() {
    if (arena && owns_arena) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        (void)hipFree(arena);
        (void)hipSetDevice(cur);
    }
}

Context::~Context() {
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (m) (void)hipSetDevice(device);
    for (auto& g : graphs) (void)hipGraphExecDestroy(g.second);
    for (auto& g : bgraphs) (void)hipGraphExecDestroy(g.second);
    void* bufs[] = {x, q, att, h, logits, scores, rope, kc0, vc0, st0, hist0, pf_tok, pf_x, pf_q, pf_att, pf_h, pf_aq, pf_abs, pf_ad, pf_abf, pf_wsc,
                    bx, bq, batt, bh, blogits, bscores, btpos, btseq, baq, babs, bad, babf, le_cnt, le_trace};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (fault_host) (void)hipHostFree(fault_host);
    if (stream) (void)hipStreamDestroy(stream);
    (void)hipSetDevice(cur);
}

namespace {

bool map_mat(const GgufFile& f, const std::string& name, DevMat& m, std::string& err, bool required = true) {
    const GgufTensor* t = f.tensor(name);
    if (!t) {
        if (required) err = "missing tensor " + name;
        return false;
    }
    m.type = t->type;
    m.cols = t->ne[0];
    m.rows = t->ne[1] * t->ne[2] * t->ne[3];
    return true;
}

}  // namespace

size_t model_tensor_bytes(const Model& m) {
    size_t b = m.tok_embd.bytes + m.out_norm.bytes + (m.output.off_a == m.tok_embd.off_a ? 0 : m.output.bytes);
    for (const Layer& L : m.layers)
        b += L.attn_norm.bytes + L.wq.bytes + L.wk.bytes + L.wv.bytes + L.wo.bytes + L.ffn_norm.bytes + L.wg.bytes +
             L.wu.bytes + L.wd.bytes;
    return b;
}

double bytes_per_token(const Model& m, int n_kv) {
    const HParams& hp = m.hp;
    double b = (double)m.output.bytes + (double)m.out_norm.bytes + (double)m.tok_embd.bytes / hp.n_vocab;
    for (const Layer& L : m.layers)
        b += (double)(L.attn_norm.bytes + L.wq.bytes + L.wk.bytes + L.wv.bytes + L.wo.bytes + L.ffn_norm.bytes +
                      L.wg.bytes + L.wu.bytes + L.wd.bytes);
    const double kv_row = 2.0 * hp.n_head_kv * hp.head_dim * 2.0;  // K+V f16 per layer per position
    b += hp.n_layer * kv_row * (double)n_kv;                       // KV read
    b += hp.n_layer * kv_row;                                      // KV write of the new token
    return b;
}

// end of a matrix's planes in the arena (plan_planes)
static size_t region_end(const DevMat& m) {
    const size_t nblk = (size_t)m.rows * (size_t)(m.cols / block_elems(m.type));
    switch (m.type) {
        case T_Q4_K: case T_Q5_K: return m.off_s + nblk * 16;
        case T_Q6_K: case T_Q8_0: return m.off_d + nblk * 2;
        default: return m.off_a + m.bytes;
    }
}

size_t fanout_plan(size_t arena_bytes, size_t chunk, const std::vector<size_t>& prefix_ends, std::vector<int>& ready) {
    ready.clear();
    if (chunk == 0 || arena_bytes == 0) return 0;
    const size_t n = (arena_bytes + chunk - 1) / chunk;
    size_t e = 0;
    for (size_t k = 0; k < n; ++k) {
        const size_t end = std::min((k + 1) * chunk, arena_bytes);
        while (e < prefix_ends.size() && prefix_ends[e] < end) ++e;
        ready.push_back(e < prefix_ends.size() ? (int)e : (int)prefix_ends.size() - 1);
    }
    return n;
}

bool model_load(const std::string& path, int device, bool vocab_only, bool no_upload, Model& M, std::string& err,
                const UploadHook* hook, int numerics) {
    M.path = path;
    M.device = device;
    if (numerics < 0 || numerics > (NUMERICS_X86 | NUMERICS_FA)) { err = "unknown numerics " + std::to_string(numerics); return false; }
    M.numerics = numerics & NUMERICS_X86;
    M.fa = (numerics & NUMERICS_FA) ? 1 : 0;
    M.file = std::make_shared<GgufFile>();
    GgufFile& f = *M.file;
    if (!f.open(path, err)) return false;
    const std::string arch = f.str("general.architecture", "");
    if (arch != "llama") { err = "unsupported architecture '" + arch + "' (llmi decodes the llama family)"; return false; }
    HParams& hp = M.hp;
    hp.n_embd = (int)f.num("llama.embedding_length", 0);
    hp.n_layer = (int)f.num("llama.block_count", 0);
    hp.n_head = (int)f.num("llama.attention.head_count", 0);
    hp.n_head_kv = (int)f.num("llama.attention.head_count_kv", hp.n_head);
    hp.n_ff = (int)f.num("llama.feed_forward_length", 0);
    hp.n_ctx_train = (int)f.num("llama.context_length", 4096);
    hp.eps = (float)f.num("llama.attention.layer_norm_rms_epsilon", 1e-5);
    hp.rope_base = (float)f.num("llama.rope.freq_base", 10000.0);
    hp.file_type = (int)f.num("general.file_type", 0);
    if (hp.n_embd <= 0 || hp.n_layer <= 0 || hp.n_head <= 0 || hp.n_head_kv <= 0) {
        err = "missing llama.* hyperparameters";
        return false;
    }
    hp.head_dim = hp.n_embd / hp.n_head;
    hp.n_rot = (int)f.num("llama.rope.dimension_count", hp.head_dim);
    if (const GgufKV* tk = f.kv("tokenizer.ggml.tokens")) M.vocab = tk->arr_str;
    M.bos = (int)f.num("tokenizer.ggml.bos_token_id", -1);
    M.eos = (int)f.num("tokenizer.ggml.eos_token_id", -1);
    if (!map_mat(f, "token_embd.weight", M.tok_embd, err)) return false;
    if (!map_mat(f, "output_norm.weight", M.out_norm, err)) return false;
    bool tied = !map_mat(f, "output.weight", M.output, err, false);
    hp.n_vocab = (int)M.tok_embd.rows;
    if (M.vocab.empty()) {
        M.vocab.resize((size_t)hp.n_vocab);
    }
    M.tok = Tokenizer::from_gguf(f, hp.n_vocab);
    M.layers.resize((size_t)hp.n_layer);
    for (int l = 0; l < hp.n_layer; ++l) {
        Layer& L = M.layers[(size_t)l];
        const std::string p = "blk." + std::to_string(l) + ".";
        if (!map_mat(f, p + "attn_norm.weight", L.attn_norm, err) || !map_mat(f, p + "attn_q.weight", L.wq, err) ||
            !map_mat(f, p + "attn_k.weight", L.wk, err) || !map_mat(f, p + "attn_v.weight", L.wv, err) ||
            !map_mat(f, p + "attn_output.weight", L.wo, err) || !map_mat(f, p + "ffn_norm.weight", L.ffn_norm, err) ||
            !map_mat(f, p + "ffn_gate.weight", L.wg, err) || !map_mat(f, p + "ffn_up.weight", L.wu, err) ||
            !map_mat(f, p + "ffn_down.weight", L.wd, err))
            return false;
    }
    if (hp.n_ff <= 0) hp.n_ff = (int)M.layers[0].wg.rows;
    // shape checks: everything the kernels assume
    const int E = hp.n_embd, D = hp.head_dim, nq = hp.n_head * D, nk = hp.n_head_kv * D;
    if (D != 64 && D != 128) { err = "head_dim " + std::to_string(D) + " unsupported (64 or 128)"; return false; }
    const int gqa = hp.n_head / hp.n_head_kv;
    if (hp.n_head % hp.n_head_kv || (gqa != 1 && gqa != 2 && gqa != 4 && gqa != 8)) {
        err = "GQA ratio unsupported";
        return false;
    }
    if (hp.n_rot > D || hp.n_rot % 2) { err = "bad rope.dimension_count"; return false; }
    if (E % 256 || hp.n_ff % 256) { err = "n_embd and n_ff must be multiples of 256"; return false; }
    auto chk = [&](const DevMat& m, int64_t rows, int64_t cols, const char* nm, bool quant) {
        if (m.rows != rows || m.cols != cols) { err = std::string(nm) + ": unexpected shape"; return false; }
        if (quant && !(m.type == T_Q4_K || m.type == T_Q5_K || m.type == T_Q6_K || m.type == T_Q8_0)) {
            err = std::string(nm) + ": weight type " + type_name(m.type) + " not supported on the decode path";
            return false;
        }
        if (!quant && m.type != T_F32) { err = std::string(nm) + ": norm weight must be f32"; return false; }
        return true;
    };
    if (!chk(M.out_norm, 1, E, "output_norm", false)) return false;
    if (M.tok_embd.cols != E) { err = "token_embd: unexpected shape"; return false; }
    if (!tied && !chk(M.output, hp.n_vocab, E, "output", true)) return false;
    for (const Layer& L : M.layers) {
        if (!chk(L.attn_norm, 1, E, "attn_norm", false) || !chk(L.ffn_norm, 1, E, "ffn_norm", false) ||
            !chk(L.wq, nq, E, "attn_q", true) || !chk(L.wk, nk, E, "attn_k", true) || !chk(L.wv, nk, E, "attn_v", true) ||
            !chk(L.wo, E, nq, "attn_output", true) || !chk(L.wg, hp.n_ff, E, "ffn_gate", true) ||
            !chk(L.wu, hp.n_ff, E, "ffn_up", true) || !chk(L.wd, E, hp.n_ff, "ffn_down", true))
            return false;
        if (act_kind(L.wg.type) != act_kind(L.wu.type)) { err = "ffn_gate/ffn_up mix Q8_0 with K-quants"; return false; }
    }
    if (const GgufTensor* rf = f.tensor("rope_freqs.weight")) {
        if (rf->type != T_F32 || rf->ne[0] * 2 < hp.n_rot) { err = "bad rope_freqs.weight"; return false; }
        M.rope_freq_host.assign((const float*)rf->data, (const float*)rf->data + rf->ne[0]);
        M.has_rope_freqs = true;
    }
    // ---- arena plan ----
    size_t off = 0;
    auto plan = [&](DevMat& m) { off = plan_planes(m, off); };
    plan(M.tok_embd);
    plan(M.out_norm);
    if (tied) M.output = M.tok_embd;
    else plan(M.output);
    for (Layer& L : M.layers) {
        plan(L.attn_norm); plan(L.wq); plan(L.wk); plan(L.wv); plan(L.wo);
        plan(L.ffn_norm); plan(L.wg); plan(L.wu); plan(L.wd);
    }
    M.arena_bytes = align_up(off, 4096);
    char desc[256];
    snprintf(desc, sizeof desc, "llama %dL E%d H%d/%d FF%d V%d ftype %d (%.2f GB)", hp.n_layer, E, hp.n_head,
             hp.n_head_kv, hp.n_ff, hp.n_vocab, hp.file_type, (double)model_tensor_bytes(M) / 1e9);
    M.desc = desc;
    if (vocab_only) return true;
    HIPC(hipSetDevice(device));
    HIPC(hipMalloc(&M.arena, M.arena_bytes));
    M.owns_arena = true;
    if (no_upload) return true;
    return model_upload(M, err, hook);
}

// The chunked H2D + on-device repack of every tensor into the planned arena (the model's
// GGUF stays mapped in M.file).  `hook` (replica fan-out) sees the arena prefix grow.
bool model_upload(Model& M, std::string& err, const UploadHook* hook) {
    if (!M.file || !M.arena) { err = "model_upload: no layout"; return false; }
    GgufFile& f = *M.file;
    const HParams& hp = M.hp;
    const bool tied = f.tensor("output.weight") == nullptr;
    if (hipSetDevice(M.device) != hipSuccess) { err = "hipSetDevice"; return false; }
    (void)hipGetLastError();  // launch_repack reports hipGetLastError: start from a clean slate
    // ---- upload: H2D + on-device repack of the unaligned block types ----
    struct Item { const GgufTensor* t; DevMat* m; };
    std::vector<Item> items;
    auto add = [&](const std::string& name, DevMat* m) { items.push_back({f.tensor(name), m}); };
    add("token_embd.weight", &M.tok_embd);
    add("output_norm.weight", &M.out_norm);
    if (!tied) add("output.weight", &M.output);
    for (int l = 0; l < hp.n_layer; ++l) {
        Layer& L = M.layers[(size_t)l];
        const std::string p = "blk." + std::to_string(l) + ".";
        add(p + "attn_norm.weight", &L.attn_norm); add(p + "attn_q.weight", &L.wq); add(p + "attn_k.weight", &L.wk);
        add(p + "attn_v.weight", &L.wv); add(p + "attn_output.weight", &L.wo); add(p + "ffn_norm.weight", &L.ffn_norm);
        add(p + "ffn_gate.weight", &L.wg); add(p + "ffn_up.weight", &L.wu); add(p + "ffn_down.weight", &L.wd);
    }
    // Chunked, double-buffered upload: host threads copy a chunk of whole rows from the
    // mmap into a pinned buffer (page faults of a cold file taken in parallel) while the
    // previous chunk's DMA and on-device repack run on the upload stream.
    constexpr size_t kChunk = 64u << 20;
    uint8_t* pin[2] = {nullptr, nullptr};
    uint8_t* dstage[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    hipStream_t us = nullptr;
    bool ok = true;
    auto cleanup = [&]() {
        if (us) (void)hipStreamSynchronize(us);
        for (int k = 0; k < 2; ++k) {
            if (pin[k]) (void)hipHostFree(pin[k]);
            if (dstage[k]) (void)hipFree(dstage[k]);
            if (ev[k]) (void)hipEventDestroy(ev[k]);
        }
        if (us) (void)hipStreamDestroy(us);
    };
    hipError_t e = hipStreamCreateWithFlags(&us, hipStreamNonBlocking);
    for (int k = 0; k < 2 && e == hipSuccess; ++k) {
        e = hipHostMalloc((void**)&pin[k], kChunk, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc(&dstage[k], kChunk);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        err = "upload buffers: " + hip_err(e);
        cleanup();
        return false;
    }
    const unsigned nthr = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    auto host_copy = [&](uint8_t* dst, const uint8_t* src, size_t n) {
        if (n < (4u << 20) || nthr == 1) { memcpy(dst, src, n); return; }
        std::vector<std::thread> th;
        const size_t per = (n + nthr - 1) / nthr;
        for (unsigned t = 0; t < nthr; ++t) {
            const size_t o = t * per;
            if (o >= n) break;
            th.emplace_back([=] { memcpy(dst + o, src + o, std::min(per, n - o)); });
        }
        for (auto& x : th) x.join();
    };
    int slot = 0;
    auto next_slot = [&]() -> hipError_t {
        if (used[slot]) {
            hipError_t e2 = hipEventSynchronize(ev[slot]);
            if (e2 != hipSuccess) return e2;
        }
        return hipSuccess;
    };
    const auto t_up = std::chrono::steady_clock::now();
    for (const Item& it : items) {
        const DevMat& m = *it.m;
        const uint8_t* src = (const uint8_t*)it.t->data;
        e = hipSuccess;
        if (needs_repack(m.type)) {
            const int64_t bpr = m.cols / block_elems(m.type);  // blocks per row
            const size_t row_raw = (size_t)bpr * block_bytes(m.type);
            // chunks of whole row groups (common.h): a multiple of 64 rows
            const int64_t rows_per = std::max<int64_t>(64, (int64_t)(kChunk / row_raw) / 64 * 64);
            const size_t pa = m.type == T_Q8_0 ? 32 : 128, ph = m.type == T_Q5_K ? 32 : m.type == T_Q6_K ? 64 : 0,
                         ps = m.type == T_Q8_0 ? 0 : 16, pd = (m.type == T_Q6_K || m.type == T_Q8_0) ? 2 : 0;
            for (int64_t r0 = 0; r0 < m.rows && e == hipSuccess; r0 += rows_per) {
                const int64_t nr = std::min(rows_per, m.rows - r0);
                const size_t n = (size_t)nr * row_raw;
                const size_t b0 = (size_t)r0 * bpr;
                e = next_slot();
                if (e != hipSuccess) break;
                host_copy(pin[slot], src + (size_t)r0 * row_raw, n);
                e = hipMemcpyAsync(dstage[slot], pin[slot], n, hipMemcpyHostToDevice, us);
                if (e == hipSuccess)
                    e = launch_repack(m.type, dstage[slot], M.arena + m.off_a + b0 * pa, M.arena + m.off_h + b0 * ph,
                                      M.arena + m.off_s + b0 * ps, M.arena + m.off_d + b0 * pd, nr * bpr, m.cols, m.rgs,
                                      M.numerics == NUMERICS_X86, us);
                if (e == hipSuccess) e = hipEventRecord(ev[slot], us);
                used[slot] = true;
                slot ^= 1;
            }
        } else {
            for (size_t o = 0; o < it.t->nbytes && e == hipSuccess; o += kChunk) {
                const size_t n = std::min(kChunk, it.t->nbytes - o);
                e = next_slot();
                if (e != hipSuccess) break;
                host_copy(pin[slot], src + o, n);
                e = hipMemcpyAsync(M.arena + m.off_a + o, pin[slot], n, hipMemcpyHostToDevice, us);
                if (e == hipSuccess) e = hipEventRecord(ev[slot], us);
                used[slot] = true;
                slot ^= 1;
            }
        }
        if (e != hipSuccess) { err = "upload of " + it.t->name + ": " + hip_err(e); ok = false; break; }
        if (hook) {
            const size_t end = &it == &items.back() ? M.arena_bytes : region_end(m);
            if (!(*hook)(end, us)) { err = "upload: fan-out failed"; ok = false; break; }
        }
    }
    if (ok) {
        e = hipStreamSynchronize(us);
        if (e != hipSuccess) { err = "upload: " + hip_err(e); ok = false; }
    }
    M.upload_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_up).count();
    cleanup();
    return ok;
}

bool model_clone_layout(const Model& src, int device, Model& dst, std::string& err) {
    dst.device = device;
    dst.numerics = src.numerics;
    dst.fa = src.fa;
    dst.path = src.path;
    dst.desc = src.desc;
    dst.file = src.file;
    dst.hp = src.hp;
    dst.tok_embd = src.tok_embd; dst.out_norm = src.out_norm; dst.output = src.output;
    dst.layers = src.layers;
    dst.vocab = src.vocab; dst.tok = src.tok; dst.bos = src.bos; dst.eos = src.eos;
    dst.rope_freq_host = src.rope_freq_host; dst.has_rope_freqs = src.has_rope_freqs;
    dst.arena_bytes = src.arena_bytes;
    HIPC(hipSetDevice(device));
    HIPC(hipMalloc(&dst.arena, dst.arena_bytes));
    dst.owns_arena = true;
    return true;
}

bool context_init(Model* m, int n_ctx, bool use_graphs, int n_seq, Context& c, std::string& err) {
    const HParams& hp = m->hp;
    c.m = m;
    c.device = m->device;
    c.n_ctx = n_ctx > 0 ? n_ctx : std::min(hp.n_ctx_train > 0 ? hp.n_ctx_train : 4096, 4096);
    // padded like upstream llama.cpp's KV cache (multiple of 256): the attention kernels
    // read V rows in 16-B (8-position) pieces and K in 64-position tiles
    c.n_ctx = (c.n_ctx + 255) / 256 * 256;
    {
        const char* e = getenv("LLMI_ATTN_MODE");
        set_attn_mode(e ? atoi(e) : 0);
    }
    c.use_graphs = use_graphs;
    HIPC(hipSetDevice(m->device));
    hipDeviceProp_t prop;
    HIPC(hipGetDeviceProperties(&prop, m->device));
    c.max_blocks = std::max(64, prop.multiProcessorCount * wg_per_cu());
    HIPC(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    HIPC(hipEventCreate(&c.ev0));
    HIPC(hipEventCreate(&c.ev1));
    const size_t E = (size_t)hp.n_embd, QD = (size_t)hp.n_head * hp.head_dim;
    const size_t kv_elems = (size_t)hp.n_layer * hp.n_head_kv * (size_t)c.n_ctx * hp.head_dim;
    HIPC(hipMalloc(&c.x, E * 4));
    HIPC(hipMalloc(&c.q, QD * 4));
    HIPC(hipMalloc(&c.att, QD * 4));
    HIPC(hipMalloc(&c.h, (size_t)hp.n_ff * 4));
    HIPC(hipMalloc(&c.logits, (size_t)hp.n_vocab * 4));
    HIPC(hipMalloc(&c.scores, attn_scratch_floats(hp.n_head, c.n_ctx) * 4));
    c.fault_dev = (unsigned*)(c.scores + attn_gran_off(hp.n_head, c.n_ctx) + 2 * (size_t)hp.n_head * kXAttnMaxKV);
    HIPC(hipHostMalloc((void**)&c.fault_host, 16, hipHostMallocDefault));
    HIPC(hipMalloc(&c.le_cnt, le_counter_bytes(hp.n_layer)));
    *c.fault_host = 0;
    if (n_seq < 1 || n_seq > 64) { err = "n_seq_max must be in [1, 64]"; return false; }
    c.n_seq = n_seq;
    c.kv_seq_elems = kv_elems;
    const int nalloc = n_seq > 1 ? n_seq + 1 : 1;  // + the dummy sequence of padded batch slots
    HIPC(hipMalloc(&c.kc0, kv_elems * 2 * nalloc));
    HIPC(hipMalloc(&c.vc0, kv_elems * 2 * nalloc));
    HIPC(hipMalloc(&c.st0, sizeof(StepState) * nalloc));
    HIPC(hipMalloc(&c.hist0, (size_t)c.n_ctx * 4 * nalloc));
    c.seq_past.assign((size_t)n_seq, 0);
    c.kc = c.kc0; c.vc = c.vc0; c.st = c.st0; c.hist = c.hist0; c.cur_seq = 0;
    // RoPE table [pos][n_rot/2][cos,sin]: ggml_rope_cache_init's iterative theta, computed
    // on the host with libm cosf/sinf exactly as the CPU path does
    const int half = hp.n_rot / 2;
    std::vector<float> tab((size_t)c.n_ctx * half * 2);
    const float theta_scale = powf(hp.rope_base, -2.0f / (float)hp.n_rot);
    for (int p = 0; p < c.n_ctx; ++p) {
        float theta = (float)p;
        for (int i = 0; i < half; ++i) {
            const float ff = m->has_rope_freqs ? m->rope_freq_host[(size_t)i] : 1.0f;
            const float th = 1.0f * (theta / ff);
            tab[((size_t)p * half + i) * 2 + 0] = cosf(th) * 1.0f;
            tab[((size_t)p * half + i) * 2 + 1] = sinf(th) * 1.0f;
            theta *= theta_scale;
        }
    }
    HIPC(hipMalloc(&c.rope, tab.size() * 4));
    HIPC(hipMemcpy(c.rope, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    context_clear(c);
    HIPC(hipStreamSynchronize(c.stream));
    return true;
}

void context_select_seq(Context& c, int s) {
    if (s < 0 || s >= std::max(1, c.n_seq + (c.n_seq > 1 ? 1 : 0))) return;
    if (s != c.cur_seq && c.cur_seq < (int)c.seq_past.size()) c.seq_past[(size_t)c.cur_seq] = c.n_past;
    c.cur_seq = s;
    c.kc = c.kc0 + (size_t)s * c.kv_seq_elems;
    c.vc = c.vc0 + (size_t)s * c.kv_seq_elems;
    c.st = c.st0 + s;
    c.hist = c.hist0 + (size_t)s * c.n_ctx;
    if (s < (int)c.seq_past.size()) c.n_past = c.seq_past[(size_t)s];
}

void context_clear_seq(Context& c, int s) {
    (void)hipSetDevice(c.device);
    (void)hipMemsetAsync(c.kc0 + (size_t)s * c.kv_seq_elems, 0, c.kv_seq_elems * 2, c.stream);
    (void)hipMemsetAsync(c.vc0 + (size_t)s * c.kv_seq_elems, 0, c.kv_seq_elems * 2, c.stream);
    (void)hipMemsetAsync(c.hist0 + (size_t)s * c.n_ctx, 0, (size_t)c.n_ctx * 4, c.stream);
    StepState s0{};
    s0.token_in = -1;
    s0.token_in_pos = -1;
    (void)hipMemcpyAsync(c.st0 + s, &s0, sizeof s0, hipMemcpyHostToDevice, c.stream);
    (void)hipStreamSynchronize(c.stream);
    if (s < (int)c.seq_past.size()) c.seq_past[(size_t)s] = 0;
    if (s == c.cur_seq) c.n_past = 0;
}

void context_clear(Context& c) {
    const HParams& hp = c.m->hp;
    const int nalloc = c.n_seq > 1 ? c.n_seq + 1 : 1;
    const size_t kv_elems = (size_t)hp.n_layer * hp.n_head_kv * (size_t)c.n_ctx * hp.head_dim * nalloc;
    (void)hipSetDevice(c.m->device);
    (void)hipMemsetAsync(c.kc0, 0, kv_elems * 2, c.stream);
    (void)hipMemsetAsync(c.vc0, 0, kv_elems * 2, c.stream);
    (void)hipMemsetAsync(c.hist0, 0, (size_t)c.n_ctx * 4 * nalloc, c.stream);
    for (int s = 1; s < nalloc; ++s) {
        StepState s1{};
        s1.token_in = -1;
        s1.token_in_pos = -1;
        (void)hipMemcpyAsync(c.st0 + s, &s1, sizeof s1, hipMemcpyHostToDevice, c.stream);
    }
    std::fill(c.seq_past.begin(), c.seq_past.end(), 0);
    // attention scratch incl. k_attn_x's granules: the step sequence restarts at 0 below,
    // so no granule of an earlier sequence may keep a tag the new one will use
    (void)hipMemsetAsync(c.scores, 0, attn_scratch_floats(hp.n_head, c.n_ctx) * 4, c.stream);
    StepState s0{};
    s0.token_in = -1;
    s0.token_in_pos = -1;
    (void)hipMemcpyAsync(c.st0, &s0, sizeof s0, hipMemcpyHostToDevice, c.stream);
    (void)hipStreamSynchronize(c.stream);
    c.n_past = 0;
}

void context_fault_readback(Context& c) {
    (void)hipMemcpyAsync(c.fault_host, c.fault_dev, 4, hipMemcpyDeviceToHost, c.stream);
}

bool context_fault_ok(Context& c, std::string& err) {
    if (*c.fault_host == 0) return true;
    err = "an in-kernel bounded wait gave up (device fault word " + std::to_string(*c.fault_host) +
          ": bit 0 attention hand-off, 0x100.. layer engine ring / edge / barrier / ring space); this call's "
          "outputs are invalid";
    *c.fault_host = 0;
    (void)hipMemsetAsync(c.fault_dev, 0, 4, c.stream);
    (void)hipStreamSynchronize(c.stream);
    return false;
}

bool Prof::arm(int k) {
    if (!timed) return true;
    while (ev.size() < 2 * (used + 1)) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return false;
        ev.push_back(e);
    }
    if (ev_cls.size() < used + 1) ev_cls.resize(used + 1);
    ev_cls[used] = k;
    set_launch_events(ev[2 * used], ev[2 * used + 1]);
    ++used;
    return true;
}
void Prof::disarm() { set_launch_events(nullptr, nullptr); }
double Prof::elapsed_us(int k, int* n) const {
    double t = 0;
    int cnt = 0;
    for (size_t i = 0; i < used; ++i) {
        if (ev_cls[i] != k) continue;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) == hipSuccess) { t += ms * 1e3; ++cnt; }
    }
    if (n) *n = cnt;
    return t;
}
Prof::~Prof() {
    disarm();
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
}

Seg seg_of(const Model& m, const DevMat& d, int row0) {
    Seg s;
    s.a = m.arena + d.off_a;
    s.h = m.arena + d.off_h;
    s.s = m.arena + d.off_s;
    s.d = m.arena + d.off_d;
    s.type = d.type;
    s.rows = (int)d.rows;
    s.row0 = row0;
    s.rgs = d.rgs;
    s.x86 = m.numerics == NUMERICS_X86;
    return s;
}

namespace {
}  // namespace

#if defined(LLMI_EXPERIMENTS)
// LLMI_EXP_XQ (step_enqueue): a zero q8 image, allocated before any capture
static const int exp_xq = [] {
    const char* e = getenv("LLMI_EXP_XQ");
    return e ? atoi(e) : 0;
}();
static uint8_t* g_exp_img = nullptr;
static bool exp_prepare(const Model& m) {
    if (!exp_xq || g_exp_img) return true;
    const size_t nb = (size_t)(std::max<int64_t>(m.hp.n_ff, m.hp.n_vocab > 0 ? m.hp.n_embd * 2 : 0) / 256 + 1) * 304;
    return hipMalloc(&g_exp_img, nb) == hipSuccess && hipMemset(g_exp_img, 0, nb) == hipSuccess &&
           hipDeviceSynchronize() == hipSuccess;
}
#endif

bool step_enqueue(Context& c, int kv_bound, std::string& err) {
    const Model& m = *c.m;
    const HParams& hp = m.hp;
    const int E = hp.n_embd, D = hp.head_dim, nq = hp.n_head * D, nk = hp.n_head_kv * D;
    const size_t kv_layer = (size_t)hp.n_head_kv * c.n_ctx * D;
    EmbArgs ea;
    ea.w = seg_of(m, m.tok_embd, 0);
    ea.cols = E; ea.vocab = hp.n_vocab; ea.x = c.x; ea.st = c.st; ea.hist = c.hist; ea.n_ctx = c.n_ctx;
    Prof* P = c.prof;
    const double kvpos = (double)hp.n_head_kv * D * 2.0;  // bytes of K (or V) per layer per position
#if defined(LLMI_EXPERIMENTS)
    // experiment builds only (make EXTRA=-DLLMI_EXPERIMENTS; results garbage, never in
    // the product library): LLMI_EXP_SKIP = bitmask of kernel classes left out of the
    // step, LLMI_EXP_XFIRST = multi-round launches also wait for x before the weights
    static const int exp_skip = [] {
        const char* e = getenv("LLMI_EXP_SKIP");
        return e ? atoi(e) : 0;
    }();
    static const int exp_xfirst = [] {
        const char* e = getenv("LLMI_EXP_XFIRST");
        return e ? atoi(e) : 0;
    }();
    // LLMI_EXP_XQ = bitmask (1 QKV, 2 attn_output, 4 gate+up, 8 down, 16 output) of launches
    // fed a zero q8 image instead of their prologue: the upper bound of a free image
    if (exp_xq && !g_exp_img) { err = "exp_img not allocated"; return false; }
    auto xq_for = [&](int bit) -> const uint8_t* { return (exp_xq >> bit & 1) ? g_exp_img : nullptr; };
#else
    constexpr int exp_skip = 0, exp_xfirst = 0;
    auto xq_for = [](int) -> const uint8_t* { return nullptr; };
#endif
    auto want = [P](int k) { return !(exp_skip >> k & 1) && (!P || P->want(k)); };
    // a filtered launch, armed with an event pair when the profiler asks for timing
#define LLMI_RUN(K, EXPR)                                  \
    do {                                                   \
        if (want(K)) {                                     \
            if (P && !P->arm(K)) {                         \
                err = "hipEventCreate failed";             \
                return false;                              \
            }                                              \
            hipError_t e_ = (EXPR);                        \
            if (P) Prof::disarm();                         \
            if (e_ != hipSuccess) {                        \
                err = std::string(#EXPR) + ": " + hip_err(e_); \
                return false;                              \
            }                                              \
        }                                                  \
    } while (0)
    // layer engine (leng.hip): one persistent launch per layer for attn_output, gate/up,
    // down and the next layer's QKV when the shapes qualify (LLMI_ENGINE=0: separate
    // launches); its edge counters are zeroed once per step
    const bool use_le = le_wanted() && c.le_cnt && !exp_skip && !exp_xfirst && !xq_for(0) && !xq_for(1) && !xq_for(2) &&
                        !xq_for(3);
    if (use_le && hipMemsetAsync(c.le_cnt, 0, le_counter_bytes(hp.n_layer), c.stream) != hipSuccess) {
        err = "hipMemsetAsync(le_cnt) failed";
        return false;
    }
    LLMI_RUN(K_EMBED, launch_embed(ea, c.stream));
    if (P) P->add(K_EMBED, (double)m.tok_embd.bytes / hp.n_vocab + E * 4.0);
    const int num = m.numerics;
    // QKV + RoPE + KV write of layer l, grouped by activation kind: n launches' args
    auto qkv_groups = [&](int l, MVArgs (&out)[3], double (&bytes)[3]) -> int {
        const Layer& L = m.layers[(size_t)l];
        MVArgs a; a.xfirst = exp_xfirst >> 0 & 1; a.num = num; a.xq = xq_for(0);
        a.cols = E; a.x = c.x; a.nw = (const float*)(m.arena + L.attn_norm.off_a); a.eps = hp.eps; a.y = c.q;
        a.kc = c.kc + l * kv_layer; a.vc = c.vc + l * kv_layer; a.rope = c.rope; a.st = c.st;
        a.head_dim = D; a.n_rot = hp.n_rot; a.n_ctx = c.n_ctx; a.nq = nq; a.nk = nk;
        const Seg qkv[3] = {seg_of(m, L.wq, 0), seg_of(m, L.wk, nq), seg_of(m, L.wv, nq + nk)};
        int i = 0, n = 0;
        while (i < 3) {
            int j = i;
            a.nseg = 0;
            int rows = 0;
            while (j < 3 && act_kind(qkv[j].type) == act_kind(qkv[i].type)) { a.seg[a.nseg++] = qkv[j]; rows += qkv[j].rows; ++j; }
            a.npairs = rows / 2;
            double b = 8.0 * E;
            for (int k = i; k < j; ++k) {
                const DevMat& dm = k == 0 ? L.wq : k == 1 ? L.wk : L.wv;
                b += (double)dm.bytes + (k == 0 ? 4.0 * nq : 2.0 * nk);
            }
            out[n] = a;
            bytes[n++] = b;
            i = j;
        }
        return n;
    };
    bool qkv_done = false;  // layer l's QKV already ran inside layer l-1's engine launch
    for (int l = 0; l < hp.n_layer; ++l) {
        const Layer& L = m.layers[(size_t)l];
        if (!qkv_done) {
            MVArgs qg[3];
            double qb[3];
            const int nqg = qkv_groups(l, qg, qb);
            for (int i = 0; i < nqg; ++i) {
                LLMI_RUN(K_QKV, launch_matvec(qg[i], EPI_QKV, c.max_blocks, c.stream));
                if (P) P->add(K_QKV, qb[i]);
            }
        }
        qkv_done = false;
        // --- attention ---
        AttnArgs at;
        at.q = c.q; at.kc = c.kc + l * kv_layer; at.vc = c.vc + l * kv_layer; at.scores = c.scores; at.out = c.att; at.st = c.st;
        at.tmax = c.scores + (size_t)hp.n_head * c.n_ctx;
        at.n_ctx = c.n_ctx; at.scale = 1.0f / sqrtf((float)D);
        at.layer = l;
        at.gran = (unsigned long long*)(c.scores + attn_gran_off(hp.n_head, c.n_ctx));
        at.fault = c.fault_dev;
        at.num = num;
        at.fa = m.fa;
        LLMI_RUN(K_ATTN, launch_attention(at, hp.n_head, hp.n_head_kv, D, kv_bound, c.stream));
        if (P) P->add(K_ATTN, 8.0 * nq, 2.0 * kvpos);
        // --- output projection + residual ---
        MVArgs o; o.xfirst = exp_xfirst >> 1 & 1; o.num = num; o.xq = xq_for(1);
        o.seg[0] = seg_of(m, L.wo, 0); o.nseg = 1; o.cols = nq; o.x = c.att; o.y = c.x; o.npairs = (E + 1) / 2;
        const double o_bytes = (double)L.wo.bytes + 4.0 * nq + 8.0 * E;
        // --- gate/up + SwiGLU ---
        MVArgs gu; gu.xfirst = exp_xfirst >> 2 & 1; gu.num = num; gu.xq = xq_for(2);
        gu.seg[0] = seg_of(m, L.wg, 0); gu.seg[1] = seg_of(m, L.wu, 0); gu.nseg = 2;
        gu.cols = E; gu.x = c.x; gu.nw = (const float*)(m.arena + L.ffn_norm.off_a); gu.eps = hp.eps;
        gu.y = c.h; gu.npairs = hp.n_ff;
        const double gu_bytes = (double)(L.wg.bytes + L.wu.bytes) + 8.0 * E + 4.0 * hp.n_ff;
        // --- down + residual ---
        MVArgs dn; dn.xfirst = exp_xfirst >> 3 & 1; dn.num = num; dn.xq = xq_for(3);
        dn.seg[0] = seg_of(m, L.wd, 0); dn.nseg = 1; dn.cols = hp.n_ff; dn.x = c.h; dn.y = c.x; dn.npairs = (E + 1) / 2;
        const double dn_bytes = (double)L.wd.bytes + 4.0 * hp.n_ff + 8.0 * E;
        bool engine_ran = false;
        if (use_le && want(K_LAYER)) {
            LeArgs la;
            la.op[0] = o; la.op[1] = gu; la.op[2] = dn; la.nops = 3;
            double lb = o_bytes + gu_bytes + dn_bytes;
            if (l + 1 < hp.n_layer) {
                MVArgs qn[3];
                double qb[3];
                if (qkv_groups(l + 1, qn, qb) == 1) { la.op[3] = qn[0]; la.nops = 4; lb += qb[0]; }
            }
            la.cnt = c.le_cnt + (size_t)l * kLeOps * 16;
            la.cnt_stride = le_counter_stride(hp.n_layer);
            la.fault = c.fault_dev;
            if (l == c.le_trace_layer) la.trace = c.le_trace;
            const hipError_t ep = layer_engine_prepare(la);
            if (ep == hipSuccess) {
                LLMI_RUN(K_LAYER, launch_layer_engine(la, c.stream));
                if (P) P->add(K_LAYER, lb);
                engine_ran = true;
                qkv_done = la.nops == 4;
            } else if (ep != hipErrorNotSupported) {
                err = "layer_engine_prepare: " + hip_err(ep);
                return false;
            }
        }
        if (!engine_ran) {
            LLMI_RUN(K_ATTN_OUT, launch_matvec(o, EPI_ADD, c.max_blocks, c.stream));
            if (P) P->add(K_ATTN_OUT, o_bytes);
            LLMI_RUN(K_FFN_GATE_UP, launch_matvec(gu, EPI_SWIGLU, c.max_blocks, c.stream));
            if (P) P->add(K_FFN_GATE_UP, gu_bytes);
            LLMI_RUN(K_FFN_DOWN, launch_matvec(dn, EPI_ADD, c.max_blocks, c.stream));
            if (P) P->add(K_FFN_DOWN, dn_bytes);
        }
    }
    MVArgs lo;
    lo.num = m.numerics; lo.xq = xq_for(4);
    lo.seg[0] = seg_of(m, m.output, 0); lo.nseg = 1; lo.cols = E; lo.x = c.x;
    lo.nw = (const float*)(m.arena + m.out_norm.off_a); lo.eps = hp.eps; lo.y = c.logits;
    lo.npairs = (hp.n_vocab + 1) / 2; lo.argmax = &c.st->key[0][0]; lo.st = c.st;
    LLMI_RUN(K_OUTPUT, launch_matvec(lo, EPI_LOGITS, c.max_blocks, c.stream));
    if (P) P->add(K_OUTPUT, (double)m.output.bytes + 8.0 * E + 4.0 * hp.n_vocab);
#undef LLMI_RUN
    return true;
}

bool step_run(Context& c, int pos, std::string& err) {
#if defined(LLMI_EXPERIMENTS)
    if (!exp_prepare(*c.m)) { err = "exp_img"; return false; }
#endif
    const int bucket = pos / 256;
    const int kv_bound = std::min(c.n_ctx, (bucket + 1) * 256);
    if (!c.use_graphs) return step_enqueue(c, kv_bound, err);
    const int gkey = bucket * 256 + c.cur_seq;
    auto it = c.graphs.find(gkey);
    if (it == c.graphs.end()) {
        hipGraph_t g = nullptr;
        HIPC(hipStreamBeginCapture(c.stream, hipStreamCaptureModeThreadLocal));
        std::string e2;
        const bool ok = step_enqueue(c, kv_bound, e2);
        hipError_t ec = hipStreamEndCapture(c.stream, &g);
        if (!ok) { err = "capture: " + e2; if (g) (void)hipGraphDestroy(g); return false; }
        if (ec != hipSuccess) { err = "hipStreamEndCapture: " + hip_err(ec); return false; }
        hipGraphExec_t ex = nullptr;
        hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ei != hipSuccess) { err = "hipGraphInstantiate: " + hip_err(ei); return false; }
        it = c.graphs.emplace(gkey, ex).first;
    }
    HIPC(hipGraphLaunch(it->second, c.stream));
    return true;
}

// ---------------------------------------------------------------------------------
// Batched decode (batch.hip): nt sequences advance one token per
// step; every launch streams its weights once for all of them.  Per step: k_bembed, then
// per layer QKV (k_mvn, segments grouped by weight type), the split attention over a
// third grid dimension of slots, attn_output, gate/up, down; the output head (k_mvn
// LOGITS) leaves each sequence's argmax in its own StepState slots.
// ---------------------------------------------------------------------------------
static bool balloc(Context& c, std::string& err) {
    if (c.bx) return true;
    const HParams& hp = c.m->hp;
    const size_t B = kMaxBatch, E = hp.n_embd, QD = (size_t)hp.n_head * hp.head_dim, F = hp.n_ff, V = hp.n_vocab;
    HIPC(hipMalloc(&c.bx, B * E * 4));
    HIPC(hipMalloc(&c.bq, B * QD * 4));
    HIPC(hipMalloc(&c.batt, B * QD * 4));
    HIPC(hipMalloc(&c.bh, B * F * 4));
    HIPC(hipMalloc(&c.blogits, B * V * 4));
    HIPC(hipMalloc(&c.bscores, B * attn_scratch_floats(hp.n_head, c.n_ctx) * 4));
    HIPC(hipMalloc(&c.btpos, B * 4));
    HIPC(hipMalloc(&c.btseq, B * 4));
    const size_t maxc = std::max({(size_t)E, QD, F});
    HIPC(hipMalloc(&c.baq, 32 * maxc * 2));
    HIPC(hipMalloc(&c.babs, B * (maxc / 16) * 2));
    HIPC(hipMalloc(&c.bad, B * (maxc / 32) * 4));
    HIPC(hipMemsetAsync(c.baq, 0, 32 * maxc * 2, c.stream));
    HIPC(hipMalloc(&c.babf, 32 * (maxc / 256) * 64));
    HIPC(hipMemsetAsync(c.babf, 0, 32 * (maxc / 256) * 64, c.stream));
    // padded slots read these rows: finite (zeros); their positions 0.  On the context
    // stream (a null-stream memset is not ordered with it: it could land after the slot
    // map upload that follows and point every slot at sequence 0)
    HIPC(hipMemsetAsync(c.bx, 0, B * E * 4, c.stream));
    HIPC(hipMemsetAsync(c.batt, 0, B * QD * 4, c.stream));
    HIPC(hipMemsetAsync(c.bh, 0, B * F * 4, c.stream));
    HIPC(hipMemsetAsync(c.btpos, 0, B * 4, c.stream));
    HIPC(hipMemsetAsync(c.btseq, 0, B * 4, c.stream));
    HIPC(hipStreamSynchronize(c.stream));
    return true;
}

static bool bstep_enqueue(Context& c, int nt, const int* seqs, int kv_bound, std::string& err) {
    const Model& m = *c.m;
    const HParams& hp = m.hp;
    const int E = hp.n_embd, D = hp.head_dim, QD = hp.n_head * D, nk = hp.n_head_kv * D, F = hp.n_ff, V = hp.n_vocab;
    const size_t kv_layer = (size_t)hp.n_head_kv * c.n_ctx * D;
#define BC(expr)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) { err = std::string(#expr) + ": " + hip_err(e_); return false; } \
    } while (0)
    BEmbArgs ea;
    ea.w = seg_of(m, m.tok_embd, 0); ea.cols = E; ea.vocab = V; ea.n_ctx = c.n_ctx; ea.nt = nt;
    ea.x = c.bx; ea.st = c.st0; ea.hist = c.hist0; ea.tseq = c.btseq; ea.tpos = c.btpos;
    BC(launch_bembed(ea, c.stream));
    MVArgs base;
    base.tpos = c.btpos; base.tseq = c.btseq; base.kv_stride = c.kv_seq_elems; base.st = c.st0;
    base.num = m.numerics;
    const bool x86 = m.numerics == NUMERICS_X86;
    // one matvec of the step: k_bmd / k_bmm (matrix cores; x86 numerics: k_bmd's x86 fold)
    // after quantizing the nt inputs, where its segments qualify, else k_mvn (x86: its x86
    // form); `quantized` skips the quantization for a launch that reads the same input as
    // the previous one
    bool qkv_quant = false;
    auto bmv = [&](const MVArgs& a, int epi, bool& quantized) -> hipError_t {
        if (nt < bmm_min_tokens() || !bmm_ok(a, epi)) return launch_mvn(a, epi, nt, c.max_blocks, c.stream);
        if (!quantized) {
            const hipError_t e = launch_pf_quant(a.x, a.x_stride, a.nw, a.eps, a.cols, 0, nt, c.baq, c.babs, c.bad, c.babf,
                                                 c.stream, x86 ? 1 : 0);
            if (e != hipSuccess) return e;
            quantized = true;
        }
        return launch_bmm(a, epi, nt, c.baq, c.babf, c.bad, c.stream);
    };
    for (int l = 0; l < hp.n_layer; ++l) {
        const Layer& L = m.layers[(size_t)l];
        qkv_quant = false;
        // QKV + RoPE + f16 KV write: one launch per run of same-type segments, or both type
        // groups in one k_bmd2 launch (launch_bmm_qkv2) on the matrix cores
        const Seg qkv[3] = {seg_of(m, L.wq, 0), seg_of(m, L.wk, QD), seg_of(m, L.wv, QD + nk)};
        MVArgs grp[3];
        int ng = 0;
        for (int i = 0; i < 3;) {
            int j = i;
            MVArgs a = base;
            a.nseg = 0;
            int rows = 0;
            while (j < 3 && qkv[j].type == qkv[i].type) { a.seg[a.nseg++] = qkv[j]; rows += qkv[j].rows; ++j; }
            a.cols = E; a.x = c.bx; a.x_stride = E; a.nw = (const float*)(m.arena + L.attn_norm.off_a); a.eps = hp.eps;
            a.y = c.bq; a.y_stride = QD; a.kc = c.kc0 + l * kv_layer; a.vc = c.vc0 + l * kv_layer; a.rope = c.rope;
            a.head_dim = D; a.n_rot = hp.n_rot; a.n_ctx = c.n_ctx; a.nq = QD; a.nk = nk; a.npairs = rows / 2;
            grp[ng++] = a;
            i = j;
        }
        bool done = false;
        if (ng == 2 && nt >= bmm_min_tokens() && bmm_ok(grp[0], EPI_QKV) && bmm_ok(grp[1], EPI_QKV)) {
            BC(launch_pf_quant(c.bx, E, grp[0].nw, hp.eps, E, 0, nt, c.baq, c.babs, c.bad, c.babf, c.stream, x86 ? 1 : 0));
            qkv_quant = true;
            const hipError_t e2 = launch_bmm_qkv2(grp[0], grp[1], nt, c.baq, c.babf, c.bad, c.stream);
            if (e2 != hipErrorNotSupported) {
                BC(e2);
                done = true;
            }
        }
        if (!done)
            for (int gi = 0; gi < ng; ++gi) BC(bmv(grp[gi], EPI_QKV, qkv_quant));
        BAttnArgs ba;
        const size_t scr = attn_scratch_floats(hp.n_head, c.n_ctx);
        for (int s = 0; s < nt; ++s) {
            AttnArgs& at = ba.a[s];
            const size_t sq = (size_t)seqs[s] * c.kv_seq_elems;
            at.q = c.bq + (size_t)s * QD; at.kc = c.kc0 + sq + l * kv_layer; at.vc = c.vc0 + sq + l * kv_layer;
            at.scores = c.bscores + (size_t)s * scr; at.tmax = at.scores + (size_t)hp.n_head * c.n_ctx;
            at.out = c.batt + (size_t)s * QD; at.st = c.st0 + seqs[s]; at.n_ctx = c.n_ctx;
            at.scale = 1.0f / sqrtf((float)D); at.layer = l;
            at.num = m.numerics;
            at.fa = m.fa;
        }
        // every slot in one launch (generic, x86 and flash-attention kernels alike)
        BC(launch_battention(ba, nt, hp.n_head, hp.n_head_kv, D, kv_bound, c.stream));
        MVArgs o = base;
        o.seg[0] = seg_of(m, L.wo, 0); o.nseg = 1; o.cols = QD; o.x = c.batt; o.x_stride = QD; o.y = c.bx; o.y_stride = E;
        o.npairs = (E + 1) / 2;
        { bool q = false; BC(bmv(o, EPI_ADD, q)); }
        MVArgs gu = base;
        gu.seg[0] = seg_of(m, L.wg, 0); gu.seg[1] = seg_of(m, L.wu, 0); gu.nseg = 2; gu.cols = E; gu.x = c.bx; gu.x_stride = E;
        gu.nw = (const float*)(m.arena + L.ffn_norm.off_a); gu.eps = hp.eps; gu.y = c.bh; gu.y_stride = F; gu.npairs = F;
        { bool q = false; BC(bmv(gu, EPI_SWIGLU, q)); }
        MVArgs dn = base;
        dn.seg[0] = seg_of(m, L.wd, 0); dn.nseg = 1; dn.cols = F; dn.x = c.bh; dn.x_stride = F; dn.y = c.bx; dn.y_stride = E;
        dn.npairs = (E + 1) / 2;
        { bool q = false; BC(bmv(dn, EPI_ADD, q)); }
    }
    MVArgs lo = base;
    lo.seg[0] = seg_of(m, m.output, 0); lo.nseg = 1; lo.cols = E; lo.x = c.bx; lo.x_stride = E;
    lo.nw = (const float*)(m.arena + m.out_norm.off_a); lo.eps = hp.eps; lo.y = c.blogits; lo.y_stride = V;
    lo.npairs = (V + 1) / 2;
    { bool q = false; BC(bmv(lo, EPI_LOGITS, q)); }
#undef BC
    return true;
}

// the batched step in this model's numerics: every numerics and weight type (generic and
// x86 K-quant rows on the matrix cores from 3 tokens, the rest through k_mvn; x86 Q8_0
// rows with 4 working waves per workgroup, batch.hip mvn_work_waves).  A layer whose
// ffn_gate and ffn_up differ in type has no batched step in any numerics (bstep_run's
// error; llama_decode then steps such sequences one at a time)
bool bstep_supported(const Model& m) {
    (void)m;
    return true;
}

bool bstep_run(Context& c, int nt, const int* seqs, int max_pos, std::string& err) {
    const HParams& hp = c.m->hp;
    if (nt < 1 || nt > kMaxBatch || c.n_seq < 2) { err = "batched step: 1..8 slots of a context with n_seq_max >= 2"; return false; }
    if (!bstep_supported(*c.m)) { err = "batched step: not supported for this model"; return false; }
    for (const Layer& L : c.m->layers)
        if (L.wg.type != L.wu.type) { err = "batched step: ffn_gate / ffn_up of different types"; return false; }
    if (!balloc(c, err)) return false;
    const int bucket = max_pos / 256;
    const int kv_bound = std::min(c.n_ctx, (bucket + 1) * 256);
    if (hp.n_head / hp.n_head_kv > 8 && (size_t)(hp.n_head / hp.n_head_kv) * kv_bound * 4 > kSplitAttnMaxLds) {
        err = "batched step: context too long for GQA groups of more than 8 heads";
        return false;
    }
    // slot -> sequence map (padded slots -> the dummy sequence n_seq)
    std::vector<int> map((size_t)kMaxBatch, c.n_seq);
    for (int s = 0; s < nt; ++s) map[(size_t)s] = seqs[s];
    if (map != c.btseq_host) {
        HIPC(hipMemcpyAsync(c.btseq, map.data(), kMaxBatch * 4, hipMemcpyHostToDevice, c.stream));
        HIPC(hipStreamSynchronize(c.stream));
        c.btseq_host = map;
    }
    if (!c.use_graphs) return bstep_enqueue(c, nt, seqs, kv_bound, err);
    std::string key = std::to_string(bucket) + ":" + std::to_string(nt);
    for (int s = 0; s < nt; ++s) key += "," + std::to_string(seqs[s]);
    auto it = c.bgraphs.find(key);
    if (it == c.bgraphs.end()) {
        hipGraph_t g = nullptr;
        HIPC(hipStreamBeginCapture(c.stream, hipStreamCaptureModeThreadLocal));
        std::string e2;
        const bool ok = bstep_enqueue(c, nt, seqs, kv_bound, e2);
        hipError_t ec = hipStreamEndCapture(c.stream, &g);
        if (!ok) { err = "capture: " + e2; if (g) (void)hipGraphDestroy(g); return false; }
        if (ec != hipSuccess) { err = "hipStreamEndCapture: " + hip_err(ec); return false; }
        hipGraphExec_t ex = nullptr;
        hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ei != hipSuccess) { err = "hipGraphInstantiate: " + hip_err(ei); return false; }
        it = c.bgraphs.emplace(key, ex).first;
    }
    HIPC(hipGraphLaunch(it->second, c.stream));
    return true;
}

// ---------------------------------------------------------------------------------
// Batched prefill: the prompt's tokens go through every layer as
// one launch per op over all of them (prefill.hip.inc): embed -> per layer [norm+quant,
// q/k/v GEMMs (RoPE, KV write), causal attention, quant, attn_output GEMM (+residual),
// norm+quant, gate/up GEMM (SwiGLU), quant, down GEMM (+residual)].  Results equal T
// decode steps bit for bit (both follow ggml's generic order); the caller runs
// the prompt's last token as an ordinary decode step for its logits.
// ---------------------------------------------------------------------------------
bool prefill_supported(const Model& m) {
    const HParams& hp = m.hp;
    if (m.fa) return false;  // flash-attention numerics: prompts as decode steps (attnfa.hip is decode-only)
    if (hp.head_dim != 128 && hp.head_dim != 64) return false;
    if (hp.n_rot % 2 || hp.n_rot > hp.head_dim) return false;
    for (const Layer& L : m.layers) {
        const DevMat* ms[] = {&L.wq, &L.wk, &L.wv, &L.wo, &L.wg, &L.wu, &L.wd};
        for (const DevMat* d : ms) {
            if (!pf_gemm_ok(d->type, (int)d->rows, (int)d->cols)) return false;
        }
        if (act_kind(L.wg.type) != act_kind(L.wu.type)) return false;
    }
    return true;
}

static bool prefill_alloc(Context& c, std::string& err) {
    if (c.pf_cap) return true;
    const HParams& hp = c.m->hp;
    // ubatch (llama.cpp's default n_ubatch 512; LLMI_PF_UBATCH, a multiple of 64 up to
    // 4096, for A/B), a multiple of 64 (k_pf_gemm's token groups)
    int cap = 512;
    if (const char* e = getenv("LLMI_PF_UBATCH")) {
        const int v = atoi(e);
        if (v >= 64 && v <= 4096 && v % 64 == 0) cap = v;
    }
    const size_t E = hp.n_embd, QD = (size_t)hp.n_head * hp.head_dim, F = hp.n_ff;
    const size_t maxc = std::max({E, QD, F});
    HIPC(hipMalloc(&c.pf_tok, cap * 4));
    HIPC(hipMalloc(&c.pf_x, cap * E * 4));
    HIPC(hipMalloc(&c.pf_q, cap * QD * 4));
    HIPC(hipMalloc(&c.pf_att, cap * QD * 4));
    HIPC(hipMalloc(&c.pf_h, cap * F * 4));
    HIPC(hipMalloc(&c.pf_aq, cap * maxc * 2));
    HIPC(hipMalloc(&c.pf_abs, cap * (maxc / 16) * 2));
    HIPC(hipMalloc(&c.pf_ad, cap * (maxc / 32) * 4));
    HIPC(hipMalloc(&c.pf_abf, cap * (maxc / 256) * 64));
    // padded token rows of the activation buffers are read (never stored): keep them finite
    HIPC(hipMemsetAsync(c.pf_aq, 0, cap * maxc * 2, c.stream));
    HIPC(hipMemsetAsync(c.pf_abs, 0, cap * (maxc / 16) * 2, c.stream));
    HIPC(hipMemsetAsync(c.pf_ad, 0, cap * (maxc / 32) * 4, c.stream));
    HIPC(hipMemsetAsync(c.pf_abf, 0, cap * (maxc / 256) * 64, c.stream));
    // the tiled attention's score rows (<= kPfFaScratchCap, launches chunked to fit); a
    // failed allocation leaves the LDS kernels in charge
    const size_t wsc = pf_fa_scratch_bytes(hp.n_head, hp.n_head_kv, hp.head_dim, cap, c.n_ctx);
    if (wsc && !g_pf_fa_noalloc && hipMalloc(&c.pf_wsc, wsc) == hipSuccess) c.pf_wsc_bytes = wsc;
    else { c.pf_wsc = nullptr; (void)hipGetLastError(); }
    c.pf_cap = cap;
    return true;
}

int prefill_max_kv(Context& c) {
    const HParams& hp = c.m->hp;
    const int lim = pf_max_kv();
    if (c.m->numerics == NUMERICS_X86)  // k_pf_a86 keeps the G heads' scores in LDS
        return std::min(lim, pf_attn_x86_max_kv(hp.n_head, hp.n_head_kv, hp.head_dim));
    // the whole context only where the tiled kernel can run: its score scratch must exist
    // (allocated here, before the limit is chosen; a failed allocation leaves the LDS
    // kernels' limit)
    std::string err;
    if (lim == kPfAttnMaxKV && g_pf_attn_fa && !g_pf_attn_simple && prefill_alloc(c, err) && c.pf_wsc)
        return c.n_ctx;
    return lim;
}

bool prefill_enqueue(Context& c, const int32_t* tokens, int n, int pos0, std::string& err) {
    const Model& m = *c.m;
    const HParams& hp = m.hp;
    if (!prefill_supported(m)) { err = "prefill: model shapes not supported by the batched path"; return false; }
    if (pos0 < 0 || pos0 + n > c.n_ctx) { err = "prefill: positions out of the context"; return false; }
    if (!prefill_alloc(c, err)) return false;
    const int E = hp.n_embd, D = hp.head_dim, nq = hp.n_head * D, nk = hp.n_head_kv * D, F = hp.n_ff;
    const size_t kv_layer = (size_t)hp.n_head_kv * c.n_ctx * D;
    const int x86 = m.numerics == NUMERICS_X86;
#define PFC(expr)                                                              \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) { err = std::string(#expr) + ": " + hip_err(e_); return false; } \
    } while (0)
    for (int b0 = 0; b0 < n; b0 += c.pf_cap) {
        const int T = std::min(c.pf_cap, n - b0), p0 = pos0 + b0;
        PFC(hipMemcpyAsync(c.pf_tok, tokens + b0, (size_t)T * 4, hipMemcpyHostToDevice, c.stream));
        PFC(launch_pf_embed(seg_of(m, m.tok_embd, 0), E, hp.n_vocab, c.pf_tok, c.pf_x, T, c.hist, p0, c.n_ctx, c.stream));
        for (int l = 0; l < hp.n_layer; ++l) {
            const Layer& L = m.layers[(size_t)l];
            PfGemm g;
            g.T = T; g.aq = c.pf_aq; g.abs = c.pf_abs; g.ad = c.pf_ad; g.abf = c.pf_abf;
            g.kc = c.kc + l * kv_layer; g.vc = c.vc + l * kv_layer; g.rope = c.rope;
            g.pos0 = p0; g.head_dim = D; g.n_rot = hp.n_rot; g.n_ctx = c.n_ctx;
            // q, k, v (each quantized for its own activation kind)
            const DevMat* qkv[3] = {&L.wq, &L.wk, &L.wv};
            int quant_kind = -1;
            // consecutive same-type parts (rows multiples of 64) share one launch
            for (int part = 0; part < 3;) {
                const DevMat& W = *qkv[part];
                if (act_kind(W.type) != quant_kind) {
                    quant_kind = act_kind(W.type);
                    PFC(launch_pf_quant(c.pf_x, E, (const float*)(m.arena + L.attn_norm.off_a), hp.eps, E, quant_kind, T,
                                        c.pf_aq, c.pf_abs, c.pf_ad, c.pf_abf, c.stream, x86));
                }
                int end = part + 1;
                while (g_pf_qkv_merge && end < 3 && qkv[end]->type == W.type && qkv[end - 1]->rows % 64 == 0) ++end;
                g.w = seg_of(m, W, 0); g.rows = (int)W.rows; g.cols = E; g.part = part; g.r1 = g.r2 = 0;
                if (end > part + 1) {
                    g.wk = seg_of(m, *qkv[part + 1], 0);
                    g.r1 = (int)W.rows;
                    g.r2 = g.r1 + (int)qkv[part + 1]->rows;
                    g.rows = g.r2;
                    if (end > part + 2) {
                        g.wv = seg_of(m, *qkv[part + 2], 0);
                        g.rows += (int)qkv[part + 2]->rows;
                    }
                }
                g.y = c.pf_q; g.ldy = nq;
                PFC(launch_pf_gemm(g, EPI_QKV, c.stream));
                part = end;
            }
            g.r1 = g.r2 = 0;
            (void)nk;
            PfAttn at;
            at.q = c.pf_q; at.out = c.pf_att; at.ldq = nq; at.kc = g.kc; at.vc = g.vc;
            at.n_ctx = c.n_ctx; at.pos0 = p0; at.gqa = hp.n_head / hp.n_head_kv; at.max_kv = p0 + T;
            at.scale = 1.0f / sqrtf((float)D);
            at.wsc = c.pf_wsc; at.wsc_bytes = c.pf_wsc_bytes;
            at.num = x86;
            PFC(launch_pf_attn(at, hp.n_head, D, T, c.stream));
            // attn_output + residual
            PFC(launch_pf_quant(c.pf_att, nq, nullptr, 0.f, nq, act_kind(L.wo.type), T, c.pf_aq, c.pf_abs, c.pf_ad, c.pf_abf, c.stream, x86));
            g.w = seg_of(m, L.wo, 0); g.rows = (int)L.wo.rows; g.cols = nq; g.y = c.pf_x; g.ldy = E;
            PFC(launch_pf_gemm(g, EPI_ADD, c.stream));
            // gate/up + SwiGLU
            PFC(launch_pf_quant(c.pf_x, E, (const float*)(m.arena + L.ffn_norm.off_a), hp.eps, E, act_kind(L.wg.type), T,
                                c.pf_aq, c.pf_abs, c.pf_ad, c.pf_abf, c.stream, x86));
            g.w = seg_of(m, L.wg, 0); g.w2 = seg_of(m, L.wu, 0); g.rows = (int)L.wg.rows; g.cols = E; g.y = c.pf_h; g.ldy = F;
            {  // gate into h, then h = silu(h) * up (two launches: a fused gate+up launch
               // spills past 256 VGPRs and measured slower: Mistral 2048 TTFT 229 vs 225
               // ms, 8B 180 vs 165, profiles/r04/prefill/swiglu_fused_vs_two.txt)
                if (act_kind(L.wu.type) != act_kind(L.wg.type)) {
                    err = "prefill: ffn_gate/ffn_up of different activation kinds";
                    return false;
                }
                PFC(launch_pf_gemm(g, EPI_STORE, c.stream));
                g.w = seg_of(m, L.wu, 0);
                PFC(launch_pf_gemm(g, EPI_SWIGLU_UP, c.stream));
            }
            // down + residual
            PFC(launch_pf_quant(c.pf_h, F, nullptr, 0.f, F, act_kind(L.wd.type), T, c.pf_aq, c.pf_abs, c.pf_ad, c.pf_abf, c.stream, x86));
            g.w = seg_of(m, L.wd, 0); g.rows = (int)L.wd.rows; g.cols = F; g.y = c.pf_x; g.ldy = E;
            PFC(launch_pf_gemm(g, EPI_ADD, c.stream));
        }
    }
#undef PFC
    return true;
}

}  // namespace llmi
