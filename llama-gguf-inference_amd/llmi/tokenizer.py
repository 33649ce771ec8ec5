"""Text <-> token ids from a GGUF's own tokenizer metadata.

The reference's llama-server tokenizes prompts and renders chat templates with
llama.cpp's vocabulary code (upstream `llama-vocab.cpp`, not vendored in
/root/reference; the gateway only proxies text, scripts/gateway.py:699-804).  This module
restates that behaviour host-side, reading everything from the GGUF header:

  tokenizer.ggml.model        "llama" -> SPM (llm_tokenizer_spm), "gpt2" -> byte-level BPE
  tokenizer.ggml.pre          BPE pre-tokenizer regex ("llama-bpe"/"llama3" or gpt-2 default)
  tokenizer.ggml.tokens / scores / token_type / merges
  tokenizer.ggml.bos_token_id / eos_token_id / add_bos_token / add_space_prefix
  tokenizer.chat_template     Jinja2 template (rendered sandboxed, as HF/minja do)

Algorithms (restated from the published llama.cpp / SentencePiece / GPT-2 behaviour):
  special-token partition: control and user-defined token texts found in the input
      split it first and map to their ids (parse_special = true, as llama-server's
      prompt tokenization)
  SPM: ' ' -> U+2581, a space prefixed to the first fragment; symbols = UTF-8 characters;
      repeatedly merge the adjacent pair whose concatenation is a vocabulary token of
      highest score (ties: leftmost); a final symbol that is not a token is split back
      along its merge history, then byte-fallback <0xXX> tokens
  BPE: pre-tokenizer regex, bytes -> GPT-2 printable unicode, merge the adjacent pair of
      lowest merge rank until none applies, unknown pieces byte by byte
  detokenize: NORMAL pieces (SPM: U+2581 -> ' '; BPE: unicode -> bytes), BYTE tokens as
      their byte, CONTROL/UNKNOWN/UNUSED rendered empty; UTF-8 assembled across tokens

Vocabularies without scores (SPM) or merges (BPE) — the synthetic GGUFs of the bench —
fall back to greedy longest match over the token texts.  Parity against llama.cpp on
real vocabularies is unpinned (llama.cpp is absent here); tests pin the algorithms on
hand-built vocabularies with known segmentations and cross-check the BPE against the
`tokenizers` library when it is importable (tests/test_tokenizer.py).
"""
from __future__ import annotations

import heapq
import struct
from typing import Iterable, Optional

# llama.cpp token types (tokenizer.ggml.token_type)
NORMAL, UNKNOWN, CONTROL, USER_DEFINED, UNUSED, BYTE = 1, 2, 3, 4, 5, 6

# ---------------------------------------------------------------------------------------
# GGUF header (metadata only; the tensor table and data are never read here)
# ---------------------------------------------------------------------------------------
_SCALAR = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q", 12: "<d"}
_STR, _ARR = 8, 9


def read_gguf_meta(path: str, prefixes: tuple = ("tokenizer.", "general.")) -> dict:
    """Key/value metadata of a GGUF v2/v3 file whose key starts with one of `prefixes`
    (others are skipped without decoding their arrays)."""
    with open(path, "rb") as f:
        data = f.read(16 << 20)  # the header of real models fits (vocab + merges < 16 MB)
        o = 0

        def need(n):
            nonlocal data
            while o + n > len(data):
                more = f.read(16 << 20)
                if not more:
                    raise ValueError("truncated GGUF header")
                data += more

        def take(fmt):
            nonlocal o
            n = struct.calcsize(fmt)
            need(n)
            v = struct.unpack_from(fmt, data, o)[0]
            o += n
            return v

        def string(decode=True):
            nonlocal o
            n = take("<Q")
            need(n)
            s = data[o:o + n]
            o += n
            return s.decode("utf-8", "replace") if decode else None

        def value(t, keep):
            nonlocal o
            if t in _SCALAR:
                return take(_SCALAR[t])
            if t == _STR:
                return string(keep)
            if t == _ARR:
                et, n = take("<I"), take("<Q")
                if et in _SCALAR and not keep:
                    sz = struct.calcsize(_SCALAR[et]) * n
                    need(sz)
                    o += sz
                    return None
                if keep:
                    return [value(et, True) for _ in range(n)]
                for _ in range(n):
                    value(et, False)
                return None
            raise ValueError(f"bad GGUF value type {t}")

        if take("<4s") != b"GGUF":
            raise ValueError("not a GGUF file")
        ver = take("<I")
        if ver not in (2, 3):
            raise ValueError(f"unsupported GGUF version {ver}")
        take("<Q")  # tensors
        n_kv = take("<Q")
        meta = {}
        for _ in range(n_kv):
            k = string()
            t = take("<I")
            keep = k.startswith(prefixes)
            v = value(t, keep)
            if keep:
                meta[k] = v
        return meta


# ---------------------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------------------
def _bytes_to_unicode() -> dict:
    """GPT-2's reversible byte -> printable unicode map (byte-level BPE)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


_B2U = _bytes_to_unicode()
_U2B = {u: b for b, u in _B2U.items()}

# pre-tokenizer regexes (llama.cpp LLAMA_VOCAB_PRE_TYPE_LLAMA3 and the GPT-2 default)
_PRE_LLAMA3 = (r"(?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
               r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
_PRE_GPT2 = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"
_LLAMA3_PRE_NAMES = {"llama-bpe", "llama3", "llama-v3", "smaug-bpe", "falcon3", "pixtral", "tekken"}


def _byte_token_value(piece: str) -> Optional[int]:
    if len(piece) == 6 and piece.startswith("<0x") and piece.endswith(">"):
        try:
            return int(piece[3:5], 16)
        except ValueError:
            return None
    return None


class Tokenizer:
    """Common surface: tokenize(text, add_special, parse_special) -> ids; piece(id) ->
    bytes; detokenize(ids) -> str; a StreamDecoder for incremental text."""

    kind = "base"

    def __init__(self, tokens: list[str], types: Optional[list[int]], bos: int, eos: int, add_bos: bool):
        self.tokens = tokens
        self.n_vocab = len(tokens)
        self.bos, self.eos, self.add_bos = bos, eos, add_bos
        if types is None or len(types) != len(tokens):
            types = [self._infer_type(i, t) for i, t in enumerate(tokens)]
        self.types = types
        self.by_text: dict[str, int] = {}
        for i, t in enumerate(tokens):
            self.by_text.setdefault(t, i)
        # special tokens matched literally in input text, longest first
        self.specials = sorted((t for i, t in enumerate(tokens) if types[i] in (CONTROL, USER_DEFINED) and t),
                               key=len, reverse=True)
        self.byte_ids = {}
        for i, t in enumerate(tokens):
            b = _byte_token_value(t)
            if b is not None and types[i] == BYTE:
                self.byte_ids.setdefault(b, i)

    def _infer_type(self, i: int, t: str) -> int:
        if _byte_token_value(t) is not None:
            return BYTE
        if i in (self.bos, self.eos) or (t.startswith("<") and t.endswith(">") and len(t) > 2 and " " not in t):
            return CONTROL
        return NORMAL

    # ---- special-token partition (llama.cpp tokenizer_st_partition)
    def _partition(self, text: str, parse_special: bool) -> list:
        frags: list = [text]
        if not parse_special:
            return frags
        for sp in self.specials:
            tid = self.by_text[sp]
            out = []
            for fr in frags:
                if not isinstance(fr, str) or sp not in fr:
                    out.append(fr)
                    continue
                parts = fr.split(sp)
                for k, p in enumerate(parts):
                    if p:
                        out.append(p)
                    if k + 1 < len(parts):
                        out.append(tid)
            frags = out
        return frags

    def tokenize(self, text: str, add_special: bool = True, parse_special: bool = True) -> list[int]:
        out: list[int] = []
        if add_special and self.add_bos and self.bos >= 0:
            out.append(self.bos)
        # llama.cpp's is_prev_special: a fragment that starts the text or follows a special
        # token gets the SPM space prefix
        prev_special = True
        for fr in self._partition(text, parse_special):
            if isinstance(fr, int):
                out.append(fr)
                prev_special = True
            else:
                out += self._encode_fragment(fr, prev_special)
                prev_special = False
        return out

    def _encode_fragment(self, text: str, first: bool) -> list[int]:
        raise NotImplementedError

    def piece(self, tid: int) -> bytes:
        raise NotImplementedError

    def detokenize(self, ids: Iterable[int]) -> str:
        return b"".join(self.piece(i) for i in ids).decode("utf-8", "replace")

    def stream(self) -> "StreamDecoder":
        return StreamDecoder(self)


class StreamDecoder:
    """Incremental detokenization: bytes of an incomplete UTF-8 sequence are held back
    until the token that completes them (llama-server's validate_utf8 behaviour)."""

    def __init__(self, tok: Tokenizer):
        self.tok = tok
        self.buf = b""

    def push(self, tid: int) -> str:
        self.buf += self.tok.piece(tid)
        n = len(self.buf)
        # longest prefix that does not end inside a multi-byte sequence
        k = n
        for back in range(1, min(4, n) + 1):
            c = self.buf[n - back]
            if c & 0xC0 == 0x80:
                continue
            need = 1 if c < 0x80 else 2 if c >> 5 == 6 else 3 if c >> 4 == 14 else 4 if c >> 3 == 30 else 1
            if need > back:
                k = n - back
            break
        s, self.buf = self.buf[:k], self.buf[k:]
        return s.decode("utf-8", "replace")

    def flush(self) -> str:
        s, self.buf = self.buf, b""
        return s.decode("utf-8", "replace")


# ---------------------------------------------------------------------------------------
# SPM (llama.cpp llm_tokenizer_spm)
# ---------------------------------------------------------------------------------------
class SpmTokenizer(Tokenizer):
    kind = "spm"

    def __init__(self, tokens, scores, types, bos, eos, add_bos=True, add_space_prefix=True):
        super().__init__(tokens, types, bos, eos, add_bos)
        self.scores = scores
        self.add_space_prefix = add_space_prefix
        self.unk = next((i for i, t in enumerate(self.types) if t == UNKNOWN), 0)

    def _encode_fragment(self, text: str, first: bool) -> list[int]:
        if first and self.add_space_prefix:
            text = " " + text
        text = text.replace(" ", "▁")
        # symbols: UTF-8 characters in a doubly linked list
        sym = list(text)
        n = len(sym)
        if n == 0:
            return []
        prev = list(range(-1, n - 1))
        nxt = list(range(1, n + 1))
        nxt[-1] = -1
        alive = [True] * n
        rev_merge: dict[str, tuple] = {}
        heap: list = []

        def add_bigram(l, r):
            if l < 0 or r < 0:
                return
            s = sym[l] + sym[r]
            tid = self.by_text.get(s)
            if tid is None:
                return
            # priority: higher score first, then leftmost
            heapq.heappush(heap, (-self.scores[tid], l, r, s))
            rev_merge[s] = (sym[l], sym[r])

        for i in range(n - 1):
            add_bigram(i, i + 1)
        while heap:
            _, l, r, s = heapq.heappop(heap)
            if not alive[l] or not alive[r] or nxt[l] != r or sym[l] + sym[r] != s:
                continue  # outdated bigram
            sym[l] = s
            alive[r] = False
            nxt[l] = nxt[r]
            if nxt[r] >= 0:
                prev[nxt[r]] = l
            add_bigram(prev[l], l)
            add_bigram(l, nxt[l])
        out: list[int] = []

        def resegment(s: str):
            tid = self.by_text.get(s)
            if tid is not None:
                out.append(tid)
                return
            parts = rev_merge.get(s)
            if parts is not None:
                resegment(parts[0])
                resegment(parts[1])
                return
            for b in s.encode("utf-8"):  # byte fallback
                out.append(self.byte_ids.get(b, self.unk))

        i = 0
        while i >= 0:
            if alive[i]:
                resegment(sym[i])
            i = nxt[i]
        return out

    def piece(self, tid: int) -> bytes:
        if not 0 <= tid < self.n_vocab:
            return b""
        t, ty = self.tokens[tid], self.types[tid]
        if ty == NORMAL:
            return t.replace("▁", " ").encode("utf-8")
        if ty == BYTE:
            b = _byte_token_value(t)
            return bytes([b]) if b is not None else b""
        if ty == USER_DEFINED:
            return t.encode("utf-8")
        if ty == UNKNOWN:
            return "▅".encode("utf-8")
        return b""  # CONTROL / UNUSED


# ---------------------------------------------------------------------------------------
# byte-level BPE (llama.cpp llm_tokenizer_bpe)
# ---------------------------------------------------------------------------------------
class BpeTokenizer(Tokenizer):
    kind = "bpe"

    def __init__(self, tokens, merges, types, bos, eos, add_bos=True, pre: str = "default"):
        super().__init__(tokens, types, bos, eos, add_bos)
        import regex  # \p{L} / \p{N} classes

        self.ranks: dict[tuple, int] = {}
        for r, m in enumerate(merges):
            a, _, b = m.partition(" ")
            self.ranks.setdefault((a, b), r)
        self.pre = pre
        self.rx = regex.compile(_PRE_LLAMA3 if pre in _LLAMA3_PRE_NAMES else _PRE_GPT2)
        self._cache: dict[str, list[int]] = {}

    def _bpe(self, word: str) -> list[int]:
        hit = self._cache.get(word)
        if hit is not None:
            return hit
        parts = list(word)
        while len(parts) > 1:
            best, bi = None, -1
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if best is None:
                break
            parts[bi:bi + 2] = [parts[bi] + parts[bi + 1]]
        out: list[int] = []
        for p in parts:
            tid = self.by_text.get(p)
            if tid is not None:
                out.append(tid)
            else:  # unknown piece: its characters one by one
                out += [self.by_text[c] for c in p if c in self.by_text]
        if len(self._cache) < 65536:
            self._cache[word] = out
        return out

    def _encode_fragment(self, text: str, first: bool) -> list[int]:
        out: list[int] = []
        for w in self.rx.findall(text):
            out += self._bpe("".join(_B2U[b] for b in w.encode("utf-8")))
        return out

    def piece(self, tid: int) -> bytes:
        if not 0 <= tid < self.n_vocab:
            return b""
        t, ty = self.tokens[tid], self.types[tid]
        if ty == NORMAL:
            return bytes(_U2B[c] if c in _U2B else 0x3F for c in t)
        if ty == USER_DEFINED:
            return t.encode("utf-8")
        if ty == BYTE:
            b = _byte_token_value(t)
            return bytes([b]) if b is not None else b""
        return b""  # CONTROL / UNKNOWN / UNUSED


# ---------------------------------------------------------------------------------------
# greedy longest match (vocabularies without scores / merges: the synthetic GGUFs)
# ---------------------------------------------------------------------------------------
class GreedyTokenizer(Tokenizer):
    kind = "greedy"

    def __init__(self, tokens, types, bos, eos, add_bos=True):
        super().__init__(tokens, types, bos, eos, add_bos)
        self.surface = [self._surface(i) for i in range(self.n_vocab)]
        self.by_surface: dict[str, int] = {}
        for i, s in enumerate(self.surface):
            if s and self.types[i] in (NORMAL, USER_DEFINED):
                self.by_surface.setdefault(s, i)
        self.max_len = max((len(s) for s in self.by_surface), default=1)

    def _surface(self, i: int) -> str:
        t = self.tokens[i]
        if self.types[i] == BYTE:
            return chr(_byte_token_value(t) or 0)
        if self.types[i] in (CONTROL, UNUSED):
            return ""
        return t.replace("▁", " ").replace("Ġ", " ").replace("Ċ", "\n")

    def _encode_fragment(self, text: str, first: bool) -> list[int]:
        out, i = [], 0
        while i < len(text):
            for n in range(min(self.max_len, len(text) - i), 0, -1):
                t = self.by_surface.get(text[i:i + n])
                if t is not None:
                    out.append(t)
                    i += n
                    break
            else:
                i += 1  # no piece covers this character: skipped
        return out

    def piece(self, tid: int) -> bytes:
        return self.surface[tid].encode("utf-8") if 0 <= tid < self.n_vocab else b""


def make_tokenizer(meta: dict, tokens: Optional[list[str]] = None, bos: int = -1, eos: int = -1) -> Tokenizer:
    """The tokenizer a GGUF's metadata describes (see module docstring)."""
    tokens = tokens if tokens is not None else meta.get("tokenizer.ggml.tokens") or []
    model = meta.get("tokenizer.ggml.model", "llama")
    types = meta.get("tokenizer.ggml.token_type")
    bos = int(meta.get("tokenizer.ggml.bos_token_id", bos))
    eos = int(meta.get("tokenizer.ggml.eos_token_id", eos))
    scores = meta.get("tokenizer.ggml.scores")
    merges = meta.get("tokenizer.ggml.merges")
    add_bos = bool(meta.get("tokenizer.ggml.add_bos_token", True))
    if model == "llama" and scores and len(scores) == len(tokens):
        return SpmTokenizer(tokens, scores, types, bos, eos, add_bos,
                            bool(meta.get("tokenizer.ggml.add_space_prefix", True)))
    if model == "gpt2" and merges:
        return BpeTokenizer(tokens, merges, types, bos, eos, add_bos, meta.get("tokenizer.ggml.pre", "default"))
    return GreedyTokenizer(tokens, types, bos, eos, add_bos)


# ---------------------------------------------------------------------------------------
# chat template (tokenizer.chat_template, Jinja2, sandboxed)
# ---------------------------------------------------------------------------------------
CHATML = ("{% for message in messages %}{{ '<|im_start|>' + message['role'] + '\n' + message['content'] + "
          "'<|im_end|>' + '\n' }}{% endfor %}{% if add_generation_prompt %}{{ '<|im_start|>assistant\n' }}{% endif %}")


class TemplateError(ValueError):
    pass


def render_chat(template: Optional[str], messages: list[dict], bos_text: str = "", eos_text: str = "",
                add_generation_prompt: bool = True) -> str:
    """Render `messages` with the GGUF's chat template (llama.cpp's default, chatml, when
    the file carries none).  Sandboxed Jinja2 with HF's trim_blocks/lstrip_blocks."""
    from jinja2.sandbox import ImmutableSandboxedEnvironment

    def raise_exception(msg):
        raise TemplateError(msg)

    env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
    env.globals["raise_exception"] = raise_exception
    try:
        t = env.from_string(template or CHATML)
        return t.render(messages=messages, add_generation_prompt=add_generation_prompt, bos_token=bos_text,
                        eos_token=eos_text)
    except TemplateError:
        raise
    except Exception as e:  # malformed template / messages
        raise TemplateError(f"chat template: {e}") from e
