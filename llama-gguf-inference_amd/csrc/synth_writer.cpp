// synth_writer.cpp — synthetic GGUF v3 files with the exact shapes and quantization
// type tables of the BASELINE.json configs (SURVEY.md §8d "Synthetic inputs").
//
// No real checkpoints exist offline; decode performance is shape-determined, so the
// benchmark and parity models are written here.  Block contents come from
// include/llmi_synth.h (pure function of seed/tensor/block), written with pwrite from
// several threads so a 4.9 GB Llama-3-8B-shaped file takes seconds.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "gguf.h"

namespace llmi {

namespace {

struct Preset {
    std::string name;
    int E, L, H, HK, FF, V, ctx;
    float rope_base, eps;
    int file_type;
    bool spm;  // SentencePiece-style vocab (TinyLlama/Mistral) vs Llama-3 BPE ids
};

// upstream llama_tensor_get_type use_more_bits(): first/last eighth + every third layer
bool more_bits(int i, int n) { return i < n / 8 || i >= 7 * n / 8 || (i - n / 8) % 3 == 2; }

struct TSpec {
    std::string name;
    int type;
    int64_t ne0, ne1;  // ne0 = row length (in features), ne1 = rows
    bool norm;
};

bool get_preset(const std::string& p, Preset& out) {
    if (p == "llama3-8b-q4km") out = {p, 4096, 32, 32, 8, 14336, 128256, 8192, 500000.f, 1e-5f, 15, false};
    else if (p == "llama3-70b-q4km") out = {p, 8192, 80, 64, 8, 28672, 128256, 8192, 500000.f, 1e-5f, 15, false};
    else if (p == "tinyllama-q8_0") out = {p, 2048, 22, 32, 4, 5632, 32000, 2048, 10000.f, 1e-5f, 7, true};
    else if (p == "mistral7b-q6k") out = {p, 4096, 32, 32, 8, 14336, 32000, 32768, 1000000.f, 1e-5f, 18, true};
    else if (p == "mistral7b-q5km") out = {p, 4096, 32, 32, 8, 14336, 32000, 32768, 1000000.f, 1e-5f, 17, true};
    else if (p == "tiny-mixed") out = {p, 256, 2, 4, 2, 512, 1000, 512, 10000.f, 1e-5f, 1, true};
    else if (p == "tiny-mixed-d128") out = {p, 512, 2, 4, 2, 768, 777, 512, 500000.f, 1e-5f, 1, false};
    else return false;
    return true;
}

// quantization type table of each preset (SURVEY.md §8 "Q4_K_M mix")
std::vector<TSpec> tensor_table(const Preset& P) {
    std::vector<TSpec> t;
    const int64_t E = P.E, F = P.FF, V = P.V, HD = P.E / P.H, KV = (int64_t)P.HK * HD;
    int emb = T_Q4_K, out = T_Q6_K;
    if (P.name == "tinyllama-q8_0") emb = out = T_Q8_0;
    if (P.name == "mistral7b-q6k") emb = out = T_Q6_K;
    if (P.name == "mistral7b-q5km") emb = T_Q5_K;
    if (P.name == "tiny-mixed") { emb = T_Q6_K; out = T_Q8_0; }
    if (P.name == "tiny-mixed-d128") { emb = T_Q8_0; out = T_Q5_K; }
    t.push_back({"token_embd.weight", emb, E, V, false});
    for (int l = 0; l < P.L; ++l) {
        int q = T_Q4_K, k = T_Q4_K, v = T_Q4_K, o = T_Q4_K, g = T_Q4_K, u = T_Q4_K, d = T_Q4_K;
        const bool mb = more_bits(l, P.L);
        if (P.name == "llama3-8b-q4km") { v = d = mb ? T_Q6_K : T_Q4_K; }
        else if (P.name == "llama3-70b-q4km") { v = mb ? T_Q6_K : T_Q5_K; d = mb ? T_Q6_K : T_Q4_K; }
        else if (P.name == "tinyllama-q8_0") { q = k = v = o = g = u = d = T_Q8_0; }
        else if (P.name == "mistral7b-q6k") { q = k = v = o = g = u = d = T_Q6_K; }
        else if (P.name == "mistral7b-q5km") { q = k = o = g = u = T_Q5_K; v = d = mb ? T_Q6_K : T_Q5_K; }
        else if (P.name == "tiny-mixed") {
            if (l == 0) { q = T_Q4_K; k = T_Q5_K; v = T_Q6_K; o = T_Q5_K; g = T_Q6_K; u = T_Q4_K; d = T_Q5_K; }
            else { q = k = v = T_Q8_0; o = T_Q6_K; g = u = T_Q8_0; d = T_Q4_K; }
        } else if (P.name == "tiny-mixed-d128") {
            if (l == 0) { q = T_Q6_K; k = T_Q4_K; v = T_Q5_K; o = T_Q8_0; g = T_Q5_K; u = T_Q5_K; d = T_Q6_K; }
            else { q = k = v = T_Q4_K; o = T_Q4_K; g = u = T_Q6_K; d = T_Q8_0; }
        }
        auto nm = [&](const char* s) { return "blk." + std::to_string(l) + "." + s + ".weight"; };
        t.push_back({nm("attn_norm"), T_F32, E, 1, true});
        t.push_back({nm("attn_q"), q, E, E, false});
        t.push_back({nm("attn_k"), k, E, KV, false});
        t.push_back({nm("attn_v"), v, E, KV, false});
        t.push_back({nm("attn_output"), o, E, E, false});
        t.push_back({nm("ffn_norm"), T_F32, E, 1, true});
        t.push_back({nm("ffn_gate"), g, E, F, false});
        t.push_back({nm("ffn_up"), u, E, F, false});
        t.push_back({nm("ffn_down"), d, F, E, false});
    }
    t.push_back({"output_norm.weight", T_F32, E, 1, true});
    t.push_back({"output.weight", out, E, V, false});
    return t;
}

struct Buf {
    std::vector<uint8_t> b;
    void u(uint64_t v, int n) { for (int i = 0; i < n; ++i) b.push_back((uint8_t)(v >> (8 * i))); }
    void s(const std::string& x) { u(x.size(), 8); b.insert(b.end(), x.begin(), x.end()); }
    void f(float x) { uint32_t w; std::memcpy(&w, &x, 4); u(w, 4); }
    void kv_u32(const std::string& k, uint32_t v) { s(k); u(G_U32, 4); u(v, 4); }
    void kv_f32(const std::string& k, float v) { s(k); u(G_F32, 4); f(v); }
    void kv_str(const std::string& k, const std::string& v) { s(k); u(G_STR, 4); s(v); }
};

// fill [b0, b1) blocks of tensor `ti` into dst
void gen_range(const TSpec& T, uint64_t seed, uint64_t ti, uint64_t b0, uint64_t b1, uint8_t* dst) {
    const int bb = block_bytes(T.type);
    for (uint64_t b = b0; b < b1; ++b) {
        uint8_t* o = dst + (b - b0) * bb;
        if (T.type == T_F32) {
            float v = llmi_synth_f32(seed, ti, b, T.norm ? 1 : 0);
            std::memcpy(o, &v, 4);
        } else if (T.type == T_F16) {
            uint16_t h = llmi_f2h(llmi_synth_f32(seed, ti, b, 0));
            std::memcpy(o, &h, 2);
        } else {
            llmi_synth_block(T.type, seed, ti, b, o);
        }
    }
}

}  // namespace

int64_t synth_write_gguf(const std::string& path, const std::string& preset, uint64_t seed,
                         int n_layer, int n_vocab, int n_threads, std::string& err) {
    Preset P;
    if (!get_preset(preset, P)) { err = "unknown synthetic preset " + preset; return -1; }
    if (n_layer > 0) P.L = n_layer;
    if (n_vocab > 0) P.V = n_vocab;
    std::vector<TSpec> T = tensor_table(P);
    Buf h;
    h.u(0x46554747u, 4);
    h.u(3, 4);
    h.u(T.size(), 8);
    const int n_kv = 18;
    h.u(n_kv, 8);
    h.kv_str("general.architecture", "llama");
    h.kv_str("general.name", "llmi-synthetic-" + P.name);
    h.kv_u32("general.file_type", (uint32_t)P.file_type);
    h.kv_u32("general.alignment", 32);
    h.kv_u32("llama.context_length", (uint32_t)P.ctx);
    h.kv_u32("llama.embedding_length", (uint32_t)P.E);
    h.kv_u32("llama.block_count", (uint32_t)P.L);
    h.kv_u32("llama.feed_forward_length", (uint32_t)P.FF);
    h.kv_u32("llama.attention.head_count", (uint32_t)P.H);
    h.kv_u32("llama.attention.head_count_kv", (uint32_t)P.HK);
    h.kv_f32("llama.attention.layer_norm_rms_epsilon", P.eps);
    h.kv_f32("llama.rope.freq_base", P.rope_base);
    h.kv_u32("llama.rope.dimension_count", (uint32_t)(P.E / P.H));
    h.kv_u32("llama.vocab_size", (uint32_t)P.V);
    h.kv_str("tokenizer.ggml.model", P.spm ? "llama" : "gpt2");
    // synthetic vocabulary: every ordinary token is a space-prefixed word, so the text of
    // n generated tokens has n whitespace-separated words (scripts/benchmark.py:120-125)
    const int bos = P.spm ? 1 : (P.V > 128009 ? 128000 : P.V - 2), eos = P.spm ? 2 : (P.V > 128009 ? 128009 : P.V - 1);
    h.s("tokenizer.ggml.tokens");
    h.u(G_ARR, 4);
    h.u(G_STR, 4);
    h.u((uint64_t)P.V, 8);
    for (int i = 0; i < P.V; ++i) {
        if (i == bos) h.s(P.spm ? "<s>" : "<|begin_of_text|>");
        else if (i == eos) h.s(P.spm ? "</s>" : "<|eot_id|>");
        else if (P.spm && i == 0) h.s("<unk>");
        else h.s(" w" + std::to_string(i));
    }
    h.s("tokenizer.ggml.bos_token_id"); h.u(G_U32, 4); h.u((uint32_t)bos, 4);
    h.s("tokenizer.ggml.eos_token_id"); h.u(G_U32, 4); h.u((uint32_t)eos, 4);
    // 18 kvs: 15 scalars/strings above + tokens + bos + eos
    std::vector<uint64_t> offs(T.size());
    uint64_t off = 0;
    for (size_t i = 0; i < T.size(); ++i) {
        offs[i] = off;
        off = align_up(off + tensor_bytes(T[i].type, T[i].ne1, T[i].ne0), 32);
        h.s(T[i].name);
        const bool one_d = T[i].ne1 == 1;
        h.u(one_d ? 1 : 2, 4);
        h.u((uint64_t)T[i].ne0, 8);
        if (!one_d) h.u((uint64_t)T[i].ne1, 8);
        h.u((uint64_t)T[i].type, 4);
        h.u(offs[i], 8);
    }
    const size_t data_start = align_up(h.b.size(), 32);
    h.b.resize(data_start, 0);
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) { err = "cannot create " + path; return -1; }
    bool ok = ::pwrite(fd, h.b.data(), h.b.size(), 0) == (ssize_t)h.b.size();
    const size_t total = data_start + off;
    ok = ok && ::ftruncate(fd, (off_t)total) == 0;
    if (n_threads <= 0) n_threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    // work items: (tensor, block range) pieces of <= 8 MiB
    struct Piece { size_t ti; uint64_t b0, b1; };
    std::vector<Piece> pieces;
    for (size_t i = 0; i < T.size(); ++i) {
        const uint64_t nb = (uint64_t)T[i].ne1 * (uint64_t)(T[i].ne0 / block_elems(T[i].type));
        const uint64_t per = std::max<uint64_t>(1, (8u << 20) / block_bytes(T[i].type));
        for (uint64_t b = 0; b < nb; b += per) pieces.push_back({i, b, std::min(nb, b + per)});
    }
    std::atomic<size_t> next{0};
    std::atomic<bool> fail{false};
    auto worker = [&]() {
        std::vector<uint8_t> buf;
        for (;;) {
            size_t k = next.fetch_add(1);
            if (k >= pieces.size() || fail.load()) break;
            const Piece& p = pieces[k];
            const TSpec& t = T[p.ti];
            const size_t bb = (size_t)block_bytes(t.type);
            buf.resize((size_t)(p.b1 - p.b0) * bb);
            gen_range(t, seed, p.ti, p.b0, p.b1, buf.data());
            const off_t at = (off_t)(data_start + offs[p.ti] + p.b0 * bb);
            if (::pwrite(fd, buf.data(), buf.size(), at) != (ssize_t)buf.size()) fail = true;
        }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < n_threads; ++i) th.emplace_back(worker);
    for (auto& x : th) x.join();
    ok = ok && !fail.load();
    ::close(fd);
    if (!ok) { err = "write failed for " + path; return -1; }
    return (int64_t)total;
}

}  // namespace llmi
