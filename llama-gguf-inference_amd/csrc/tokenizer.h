// tokenizer.h — text <-> token ids from a GGUF's tokenizer metadata (llama_tokenize /
// llama_token_to_piece of the C ABI, include/llmi.h).
//
// The reference's llama-server tokenizes with llama.cpp's vocabulary code (upstream
// llama-vocab.cpp, not vendored; reached through scripts/gateway.py:699-804).  This is
// the native form of llmi/tokenizer.py — the same algorithms, the same results on every
// input (tests/test_tokenizer_native.py checks them against each other):
//   tokenizer.ggml.model "llama" with scores  -> SPM (score-ordered merges, byte fallback)
//   tokenizer.ggml.model "gpt2" with merges   -> byte-level BPE (llama3 / gpt-2 pre-tokenizer)
//   otherwise                                 -> greedy longest match over the token texts
// with llama.cpp's special-token partition and token types.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace llmi {

class GgufFile;

enum TokType : int { TT_NORMAL = 1, TT_UNKNOWN = 2, TT_CONTROL = 3, TT_USER_DEFINED = 4, TT_UNUSED = 5, TT_BYTE = 6 };

class Tokenizer {
public:
    enum Kind { SPM, BPE, GREEDY };
    // from a GGUF's metadata; n_vocab_fallback names tokens "<tok_i>" when the file has none
    static std::unique_ptr<Tokenizer> from_gguf(const GgufFile& f, int n_vocab_fallback);
    // from arrays (scores / merges / types may be empty)
    static std::unique_ptr<Tokenizer> build(const std::string& model, const std::string& pre,
                                            std::vector<std::string> tokens, std::vector<float> scores,
                                            std::vector<int> types, const std::vector<std::string>& merges, int bos,
                                            int eos, bool add_bos, bool add_space_prefix);

    std::vector<int32_t> tokenize(const std::string& utf8, bool add_special, bool parse_special) const;
    // the bytes a token renders as (special: CONTROL tokens render their text)
    std::string piece(int32_t id, bool special) const;

    Kind kind = GREEDY;
    std::vector<std::string> tokens;
    std::vector<int> types;
    int bos = -1, eos = -1;
    bool add_bos = true;
    bool add_eos = false;  // tokenizer.ggml.add_eos_token (llama_detokenize's remove_special)

private:
    void init_common();
    std::vector<int32_t> encode_fragment(const std::u32string& text, bool first) const;
    std::vector<int32_t> spm(const std::u32string& text, bool first) const;
    std::vector<int32_t> bpe(const std::u32string& text) const;
    std::vector<int32_t> greedy(const std::u32string& text) const;
    void bpe_word(const std::string& bytes, std::vector<int32_t>& out) const;

    std::vector<float> scores_;
    bool add_space_prefix_ = true;
    bool llama3_pre_ = false;
    int unk_ = 0;
    std::unordered_map<std::string, int> by_text_;
    std::vector<std::pair<std::u32string, int>> specials_;  // longest first
    int byte_ids_[256];
    std::unordered_map<std::string, int> ranks_;            // "a\xff" "b" -> merge rank
    std::vector<std::u32string> surface_;                   // greedy
    std::unordered_map<std::u32string, int> by_surface_;
    size_t max_surface_ = 1;
};

}  // namespace llmi
