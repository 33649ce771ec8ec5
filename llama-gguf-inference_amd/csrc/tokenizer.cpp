// tokenizer.cpp — native restatement of llmi/tokenizer.py (see tokenizer.h).  Every
// branch below names the Python function it follows; the two are checked against each
// other on the same vocabularies and texts (tests/test_tokenizer_native.py).
#include "tokenizer.h"

#include <algorithm>
#include <queue>

#include "gguf.h"
#include "unicode_tables.h"

namespace llmi {

namespace {

// ---- UTF-8 <-> code points (invalid bytes decode to U+FFFD one byte at a time) ----
std::u32string utf8_decode(const std::string& s) {
    std::u32string out;
    out.reserve(s.size());
    size_t i = 0;
    const size_t n = s.size();
    while (i < n) {
        const unsigned char c = (unsigned char)s[i];
        int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        char32_t cp = len == 1 ? c : len == 2 ? (c & 0x1F) : len == 3 ? (c & 0x0F) : (c & 0x07);
        bool ok = len > 0 && i + len <= n;
        for (int k = 1; ok && k < len; ++k) {
            const unsigned char d = (unsigned char)s[i + k];
            if ((d & 0xC0) != 0x80) ok = false;
            else cp = (cp << 6) | (d & 0x3F);
        }
        if (ok && ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
                   (cp >= 0xD800 && cp <= 0xDFFF)))
            ok = false;
        if (!ok) {
            out.push_back(0xFFFD);
            ++i;
            continue;
        }
        out.push_back(cp);
        i += (size_t)len;
    }
    return out;
}
void utf8_append(std::string& out, char32_t cp) {
    if (cp < 0x80) {
        out.push_back((char)cp);
    } else if (cp < 0x800) {
        out.push_back((char)(0xC0 | (cp >> 6)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
        out.push_back((char)(0xE0 | (cp >> 12)));
        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
        out.push_back((char)(0xF0 | (cp >> 18)));
        out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
    }
}
std::string utf8_encode(const std::u32string& s) {
    std::string out;
    out.reserve(s.size());
    for (char32_t c : s) utf8_append(out, c);
    return out;
}

// ---- character classes of the pre-tokenizer regexes (unicode_tables.h) ----
bool in_ranges(const uint32_t (*r)[2], int n, char32_t cp) {
    int lo = 0, hi = n - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) / 2;
        if (cp < r[mid][0]) hi = mid - 1;
        else if (cp > r[mid][1]) lo = mid + 1;
        else return true;
    }
    return false;
}
bool is_L(char32_t c) { return in_ranges(k_uni_letter, k_uni_letter_n, c); }
bool is_N(char32_t c) { return in_ranges(k_uni_number, k_uni_number_n, c); }
bool is_S(char32_t c) { return in_ranges(k_uni_space, k_uni_space_n, c); }
bool is_other(char32_t c) { return !is_S(c) && !is_L(c) && !is_N(c); }
bool is_crlf(char32_t c) { return c == U'\r' || c == U'\n'; }
char32_t lower_ascii(char32_t c) { return c >= U'A' && c <= U'Z' ? c + 32 : c; }

// end of the whitespace alternatives of both regexes at i (t[i] is \s):
//   \s*[\r\n]+ (llama3 only) | \s+(?!\S) | \s+
size_t match_space(const std::u32string& t, size_t i, bool crlf_alt) {
    const size_t n = t.size();
    size_t j = i;
    while (j < n && is_S(t[j])) ++j;
    if (crlf_alt) {  // greedy \s* backs off to the last CR/LF of the run
        for (size_t k = j; k > i; --k)
            if (is_crlf(t[k - 1])) return k;
    }
    if (j == n) return j;           // \s+(?!\S) at the end of the text
    if (j - i >= 2) return j - 1;   // \s+(?!\S): leave the last space for the next word
    return j;                       // \s+
}

// llmi/tokenizer.py _PRE_LLAMA3 (llama.cpp LLAMA_VOCAB_PRE_TYPE_LLAMA3): end of the
// match at i, alternatives in the regex's order
size_t match_llama3(const std::u32string& t, size_t i) {
    const size_t n = t.size();
    const char32_t c = t[i];
    if (c == U'\'' && i + 1 < n) {  // '[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD]
        const char32_t a = lower_ascii(t[i + 1]);
        if (a == U's' || a == U't' || a == U'm' || a == U'd') return i + 2;
        if (i + 2 < n) {
            const char32_t b = lower_ascii(t[i + 2]);
            if ((a == U'r' && b == U'e') || (a == U'v' && b == U'e') || (a == U'l' && b == U'l')) return i + 3;
        }
    }
    // [^\r\n\p{L}\p{N}]?\p{L}+
    if (!is_crlf(c) && !is_L(c) && !is_N(c) && i + 1 < n && is_L(t[i + 1])) {
        size_t j = i + 1;
        while (j < n && is_L(t[j])) ++j;
        return j;
    }
    if (is_L(c)) {
        size_t j = i;
        while (j < n && is_L(t[j])) ++j;
        return j;
    }
    if (is_N(c)) {  // \p{N}{1,3}
        size_t j = i;
        while (j < n && j < i + 3 && is_N(t[j])) ++j;
        return j;
    }
    // ' ?[^\s\p{L}\p{N}]+[\r\n]*'
    size_t k = i;
    if (c == U' ' && i + 1 < n && is_other(t[i + 1])) k = i + 1;
    if (is_other(t[k])) {
        size_t j = k;
        while (j < n && is_other(t[j])) ++j;
        while (j < n && is_crlf(t[j])) ++j;
        return j;
    }
    return match_space(t, i, true);  // t[i] is \s here
}

// llmi/tokenizer.py _PRE_GPT2: 's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
size_t match_gpt2(const std::u32string& t, size_t i) {
    const size_t n = t.size();
    const char32_t c = t[i];
    if (c == U'\'' && i + 1 < n) {
        const char32_t a = t[i + 1];
        if (a == U's' || a == U't' || a == U'm' || a == U'd') return i + 2;
        if (i + 2 < n) {
            const char32_t b = t[i + 2];
            if ((a == U'r' && b == U'e') || (a == U'v' && b == U'e') || (a == U'l' && b == U'l')) return i + 3;
        }
    }
    bool (*cls[3])(char32_t) = {is_L, is_N, is_other};
    for (auto f : cls) {
        size_t k = i;
        if (c == U' ' && i + 1 < n && f(t[i + 1])) k = i + 1;
        if (f(t[k])) {
            size_t j = k;
            while (j < n && f(t[j])) ++j;
            return j;
        }
    }
    return match_space(t, i, false);
}

// GPT-2's reversible byte <-> printable unicode map (llmi/tokenizer.py _bytes_to_unicode)
struct ByteMap {
    char32_t b2u[256];
    std::unordered_map<char32_t, int> u2b;
    ByteMap() {
        bool used[256] = {};
        auto mark = [&](int a, int b) {
            for (int x = a; x <= b; ++x) {
                used[x] = true;
                b2u[x] = (char32_t)x;
            }
        };
        mark('!', '~');
        mark(0xA1, 0xAC);
        mark(0xAE, 0xFF);
        int k = 0;
        for (int x = 0; x < 256; ++x)
            if (!used[x]) b2u[x] = (char32_t)(256 + k++);
        for (int x = 0; x < 256; ++x) u2b[b2u[x]] = x;
    }
};
const ByteMap& byte_map() {
    static const ByteMap m;
    return m;
}

int byte_token_value(const std::string& t) {  // "<0xXX>" -> XX, else -1
    if (t.size() != 6 || t.compare(0, 3, "<0x") != 0 || t[5] != '>') return -1;
    auto hex = [](char ch) { return ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10
                                                                     : ch >= 'A' && ch <= 'F' ? ch - 'A' + 10 : -1; };
    const int h = hex(t[3]), l = hex(t[4]);
    return h < 0 || l < 0 ? -1 : h * 16 + l;
}

const std::string kSpmSpace = "\xe2\x96\x81";  // U+2581

std::string replace_all(std::string s, const std::string& from, const std::string& to) {
    size_t p = 0;
    while ((p = s.find(from, p)) != std::string::npos) {
        s.replace(p, from.size(), to);
        p += to.size();
    }
    return s;
}

}  // namespace

std::unique_ptr<Tokenizer> Tokenizer::build(const std::string& model, const std::string& pre, std::vector<std::string> tokens,
                                            std::vector<float> scores, std::vector<int> types,
                                            const std::vector<std::string>& merges, int bos, int eos, bool add_bos,
                                            bool add_space_prefix) {
    auto tk = std::make_unique<Tokenizer>();
    tk->tokens = std::move(tokens);
    tk->bos = bos;
    tk->eos = eos;
    tk->add_bos = add_bos;
    tk->add_space_prefix_ = add_space_prefix;
    const size_t n = tk->tokens.size();
    if (types.size() != n) {  // Tokenizer._infer_type
        types.assign(n, TT_NORMAL);
        for (size_t i = 0; i < n; ++i) {
            const std::string& t = tk->tokens[i];
            if (byte_token_value(t) >= 0) types[i] = TT_BYTE;
            else if ((int)i == bos || (int)i == eos ||
                     (t.size() > 2 && t.front() == '<' && t.back() == '>' && t.find(' ') == std::string::npos &&
                      utf8_decode(t).size() > 2))
                types[i] = TT_CONTROL;
        }
    }
    tk->types = std::move(types);
    if (model == "llama" && !scores.empty() && scores.size() == n) {
        tk->kind = SPM;
        tk->scores_ = std::move(scores);
    } else if (model == "gpt2" && !merges.empty()) {
        tk->kind = BPE;
        for (size_t r = 0; r < merges.size(); ++r) {  // a, _, b = m.partition(" ")
            const std::string& m = merges[r];
            const size_t sp = m.find(' ');
            const std::string a = sp == std::string::npos ? m : m.substr(0, sp);
            const std::string b = sp == std::string::npos ? std::string() : m.substr(sp + 1);
            tk->ranks_.emplace(a + '\xff' + b, (int)r);
        }
        static const char* llama3[] = {"llama-bpe", "llama3", "llama-v3", "smaug-bpe", "falcon3", "pixtral", "tekken"};
        for (const char* p : llama3)
            if (pre == p) tk->llama3_pre_ = true;
    } else {
        tk->kind = GREEDY;
    }
    tk->init_common();
    return tk;
}

void Tokenizer::init_common() {
    const size_t n = tokens.size();
    for (size_t i = 0; i < n; ++i) by_text_.emplace(tokens[i], (int)i);
    for (size_t i = 0; i < n; ++i)
        if ((types[i] == TT_CONTROL || types[i] == TT_USER_DEFINED) && !tokens[i].empty())
            specials_.emplace_back(utf8_decode(tokens[i]), by_text_[tokens[i]]);
    std::stable_sort(specials_.begin(), specials_.end(),
                     [](const auto& a, const auto& b) { return a.first.size() > b.first.size(); });
    for (int& b : byte_ids_) b = -1;
    for (size_t i = 0; i < n; ++i) {
        const int b = byte_token_value(tokens[i]);
        if (b >= 0 && types[i] == TT_BYTE && byte_ids_[b] < 0) byte_ids_[b] = (int)i;
    }
    unk_ = 0;
    for (size_t i = 0; i < n; ++i)
        if (types[i] == TT_UNKNOWN) {
            unk_ = (int)i;
            break;
        }
    if (kind == GREEDY) {  // GreedyTokenizer._surface
        surface_.resize(n);
        for (size_t i = 0; i < n; ++i) {
            const std::string& t = tokens[i];
            if (types[i] == TT_BYTE) {
                const int b = byte_token_value(t);
                surface_[i] = std::u32string(1, (char32_t)(b < 0 ? 0 : b));
            } else if (types[i] == TT_CONTROL || types[i] == TT_UNUSED) {
                surface_[i].clear();
            } else {
                std::string s = replace_all(t, kSpmSpace, " ");
                s = replace_all(s, "\xc4\xa0", " ");   // U+0120 (GPT-2 space)
                s = replace_all(s, "\xc4\x8a", "\n");  // U+010A (GPT-2 newline)
                surface_[i] = utf8_decode(s);
            }
        }
        max_surface_ = 1;
        for (size_t i = 0; i < n; ++i)
            if (!surface_[i].empty() && (types[i] == TT_NORMAL || types[i] == TT_USER_DEFINED)) {
                by_surface_.emplace(surface_[i], (int)i);
                max_surface_ = std::max(max_surface_, surface_[i].size());
            }
    }
}

std::unique_ptr<Tokenizer> Tokenizer::from_gguf(const GgufFile& f, int n_vocab_fallback) {
    std::vector<std::string> tokens;
    if (const GgufKV* kv = f.kv("tokenizer.ggml.tokens")) tokens = kv->arr_str;
    const bool synthetic = tokens.empty();
    if (synthetic) {
        tokens.resize((size_t)std::max(0, n_vocab_fallback));
        for (size_t i = 0; i < tokens.size(); ++i) tokens[i] = "<tok_" + std::to_string(i) + ">";
    }
    std::vector<float> scores;
    if (const GgufKV* kv = f.kv("tokenizer.ggml.scores"))
        for (double d : kv->arr_num) scores.push_back((float)d);
    std::vector<int> types;
    if (const GgufKV* kv = f.kv("tokenizer.ggml.token_type"))
        for (double d : kv->arr_num) types.push_back((int)d);
    // placeholder pieces of a GGUF without a vocabulary are UNUSED, not CONTROL: they never
    // enter the special-token partition (a scan over n_vocab specials per tokenize call)
    if (synthetic) types.assign(tokens.size(), TT_UNUSED);
    std::vector<std::string> merges;
    if (const GgufKV* kv = f.kv("tokenizer.ggml.merges")) merges = kv->arr_str;
    auto tk = build(f.str("tokenizer.ggml.model", "llama"), f.str("tokenizer.ggml.pre", "default"), std::move(tokens),
                    std::move(scores), std::move(types), merges, (int)f.num("tokenizer.ggml.bos_token_id", -1),
                    (int)f.num("tokenizer.ggml.eos_token_id", -1), f.num("tokenizer.ggml.add_bos_token", 1) != 0,
                    f.num("tokenizer.ggml.add_space_prefix", 1) != 0);
    tk->add_eos = f.num("tokenizer.ggml.add_eos_token", 0) != 0;
    return tk;
}

// Tokenizer.tokenize: special-token partition, then each text fragment encoded
std::vector<int32_t> Tokenizer::tokenize(const std::string& utf8, bool add_special, bool parse_special) const {
    std::vector<int32_t> out;
    if (add_special && add_bos && bos >= 0) out.push_back(bos);
    struct Frag {
        std::u32string text;
        int id;  // >= 0: a special token
    };
    std::vector<Frag> frags{{utf8_decode(utf8), -1}};
    if (parse_special) {  // Tokenizer._partition: longest special first, str.split semantics
        for (const auto& sp : specials_) {
            std::vector<Frag> next;
            for (Frag& fr : frags) {
                if (fr.id >= 0 || fr.text.find(sp.first) == std::u32string::npos) {
                    next.push_back(std::move(fr));
                    continue;
                }
                size_t p = 0;
                for (;;) {
                    const size_t q = fr.text.find(sp.first, p);
                    const size_t e = q == std::u32string::npos ? fr.text.size() : q;
                    if (e > p) next.push_back({fr.text.substr(p, e - p), -1});
                    if (q == std::u32string::npos) break;
                    next.push_back({std::u32string(), sp.second});
                    p = q + sp.first.size();
                }
            }
            frags.swap(next);
        }
    }
    bool prev_special = true;  // llama.cpp is_prev_special: SPM space prefix
    for (const Frag& fr : frags) {
        if (fr.id >= 0) {
            out.push_back(fr.id);
            prev_special = true;
        } else {
            const auto ids = encode_fragment(fr.text, prev_special);
            out.insert(out.end(), ids.begin(), ids.end());
            prev_special = false;
        }
    }
    return out;
}

std::vector<int32_t> Tokenizer::encode_fragment(const std::u32string& text, bool first) const {
    switch (kind) {
        case SPM: return spm(text, first);
        case BPE: return bpe(text);
        default: return greedy(text);
    }
}

// SpmTokenizer._encode_fragment: score-ordered bigram merges over UTF-8 characters
std::vector<int32_t> Tokenizer::spm(const std::u32string& in, bool first) const {
    std::u32string text = first && add_space_prefix_ ? U" " + in : in;
    for (char32_t& c : text)
        if (c == U' ') c = 0x2581;
    const int n = (int)text.size();
    std::vector<int32_t> out;
    if (n == 0) return out;
    std::vector<std::u32string> sym((size_t)n);
    std::vector<int> prev((size_t)n), nxt((size_t)n);
    std::vector<char> alive((size_t)n, 1);
    for (int i = 0; i < n; ++i) {
        sym[(size_t)i] = std::u32string(1, text[(size_t)i]);
        prev[(size_t)i] = i - 1;
        nxt[(size_t)i] = i + 1 < n ? i + 1 : -1;
    }
    struct Big {
        double neg;  // -score: the heap pops the highest score, then the leftmost
        int l, r;
        std::u32string s;
        bool operator>(const Big& o) const {
            if (neg != o.neg) return neg > o.neg;
            if (l != o.l) return l > o.l;
            if (r != o.r) return r > o.r;
            return s > o.s;
        }
    };
    std::priority_queue<Big, std::vector<Big>, std::greater<Big>> heap;
    std::unordered_map<std::u32string, std::pair<std::u32string, std::u32string>> rev;
    auto add = [&](int l, int r) {
        if (l < 0 || r < 0) return;
        std::u32string s = sym[(size_t)l] + sym[(size_t)r];
        auto it = by_text_.find(utf8_encode(s));
        if (it == by_text_.end()) return;
        rev[s] = {sym[(size_t)l], sym[(size_t)r]};
        heap.push({-(double)scores_[(size_t)it->second], l, r, std::move(s)});
    };
    for (int i = 0; i + 1 < n; ++i) add(i, i + 1);
    while (!heap.empty()) {
        Big b = heap.top();
        heap.pop();
        const size_t l = (size_t)b.l, r = (size_t)b.r;
        if (!alive[l] || !alive[r] || nxt[l] != b.r || sym[l] + sym[r] != b.s) continue;  // outdated
        sym[l] = b.s;
        alive[r] = 0;
        nxt[l] = nxt[r];
        if (nxt[r] >= 0) prev[(size_t)nxt[r]] = b.l;
        add(prev[l], b.l);
        add(b.l, nxt[l]);
    }
    // resegment: a symbol that is no token splits back along its merge history, then bytes
    for (int i = 0; i >= 0; i = nxt[(size_t)i]) {
        if (!alive[(size_t)i]) continue;
        std::vector<std::u32string> work{sym[(size_t)i]};
        while (!work.empty()) {
            std::u32string s = std::move(work.back());
            work.pop_back();
            const std::string u = utf8_encode(s);
            auto it = by_text_.find(u);
            if (it != by_text_.end()) {
                out.push_back(it->second);
                continue;
            }
            auto rm = rev.find(s);
            if (rm != rev.end()) {
                work.push_back(rm->second.second);  // right after left
                work.push_back(rm->second.first);
                continue;
            }
            for (unsigned char c : u) out.push_back(byte_ids_[c] >= 0 ? byte_ids_[c] : unk_);
        }
    }
    return out;
}

// BpeTokenizer._bpe: lowest-rank adjacent merge until none applies
void Tokenizer::bpe_word(const std::string& bytes, std::vector<int32_t>& out) const {
    const ByteMap& bm = byte_map();
    std::vector<std::string> parts;
    parts.reserve(bytes.size());
    for (unsigned char c : bytes) {
        std::string p;
        utf8_append(p, bm.b2u[c]);
        parts.push_back(std::move(p));
    }
    while (parts.size() > 1) {
        int best = -1;
        size_t bi = 0;
        for (size_t i = 0; i + 1 < parts.size(); ++i) {
            auto it = ranks_.find(parts[i] + '\xff' + parts[i + 1]);
            if (it != ranks_.end() && (best < 0 || it->second < best)) {
                best = it->second;
                bi = i;
            }
        }
        if (best < 0) break;
        parts[bi] += parts[bi + 1];
        parts.erase(parts.begin() + (long)bi + 1);
    }
    for (const std::string& p : parts) {
        auto it = by_text_.find(p);
        if (it != by_text_.end()) {
            out.push_back(it->second);
            continue;
        }
        for (char32_t c : utf8_decode(p)) {  // unknown piece: its characters one by one
            std::string one;
            utf8_append(one, c);
            auto jt = by_text_.find(one);
            if (jt != by_text_.end()) out.push_back(jt->second);
        }
    }
}

std::vector<int32_t> Tokenizer::bpe(const std::u32string& text) const {
    std::vector<int32_t> out;
    size_t i = 0;
    while (i < text.size()) {
        const size_t j = llama3_pre_ ? match_llama3(text, i) : match_gpt2(text, i);
        bpe_word(utf8_encode(text.substr(i, j - i)), out);
        i = j;
    }
    return out;
}

// GreedyTokenizer._encode_fragment: longest surface match, unmatched characters skipped
std::vector<int32_t> Tokenizer::greedy(const std::u32string& text) const {
    std::vector<int32_t> out;
    size_t i = 0;
    while (i < text.size()) {
        bool hit = false;
        for (size_t n = std::min(max_surface_, text.size() - i); n > 0; --n) {
            auto it = by_surface_.find(text.substr(i, n));
            if (it != by_surface_.end()) {
                out.push_back(it->second);
                i += n;
                hit = true;
                break;
            }
        }
        if (!hit) ++i;
    }
    return out;
}

// SpmTokenizer.piece / BpeTokenizer.piece / GreedyTokenizer.piece; `special` renders
// CONTROL tokens as their text (llama_token_to_piece's special flag)
std::string Tokenizer::piece(int32_t id, bool special) const {
    if (id < 0 || (size_t)id >= tokens.size()) return std::string();
    const std::string& t = tokens[(size_t)id];
    const int ty = types[(size_t)id];
    if (special && ty == TT_CONTROL) return t;
    if (kind == GREEDY) return utf8_encode(surface_[(size_t)id]);
    if (ty == TT_USER_DEFINED) return t;
    if (ty == TT_BYTE) {
        const int b = byte_token_value(t);
        return b < 0 ? std::string() : std::string(1, (char)b);
    }
    if (kind == SPM) {
        if (ty == TT_NORMAL) return replace_all(t, kSpmSpace, " ");
        if (ty == TT_UNKNOWN) return "\xe2\x96\x85";  // U+2585
        return std::string();
    }
    if (ty == TT_NORMAL) {  // byte-level: printable unicode back to bytes ('?' if unmapped)
        const ByteMap& bm = byte_map();
        std::string out;
        for (char32_t c : utf8_decode(t)) {
            auto it = bm.u2b.find(c);
            out.push_back(it == bm.u2b.end() ? '?' : (char)it->second);
        }
        return out;
    }
    return std::string();
}

}  // namespace llmi
