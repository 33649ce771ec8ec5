"""The C ABI's tokenizer (llama_tokenize / llama_token_to_piece / llama_detokenize,
csrc/tokenizer.cpp) against the host tokenizer it restates (llmi/tokenizer.py, itself
pinned by tests/test_tokenizer.py on hand-built segmentations and the `tokenizers`
library): the same GGUF metadata through both, the same ids and bytes on every text.
CPU only (tokenization never touches the device)."""
from __future__ import annotations

import os
import struct
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import llmi  # noqa: E402
from llmi import tokenizer as T  # noqa: E402

import test_tokenizer as TT  # noqa: E402  (the hand-built vocabularies)


def _write_meta_gguf(path: str, kv: dict) -> None:
    """A tensorless GGUF v3 holding only metadata (strings, ints, floats, bools, arrays)."""

    def s(x: str) -> bytes:
        b = x.encode("utf-8")
        return struct.pack("<Q", len(b)) + b

    def val(v):
        if isinstance(v, bool):
            return struct.pack("<I", 7) + struct.pack("<?", v)
        if isinstance(v, int):
            return struct.pack("<I", 5) + struct.pack("<i", v)
        if isinstance(v, float):
            return struct.pack("<I", 6) + struct.pack("<f", v)
        if isinstance(v, str):
            return struct.pack("<I", 8) + s(v)
        if isinstance(v, tuple):  # (element type, list)
            et, items = v
            body = b"".join(s(x) if et == 8 else struct.pack({5: "<i", 6: "<f"}[et], x) for x in items)
            return struct.pack("<I", 9) + struct.pack("<IQ", et, len(items)) + body
        raise TypeError(v)

    out = b"GGUF" + struct.pack("<IQQ", 3, 0, len(kv))
    for k, v in kv.items():
        out += s(k) + val(v)
    with open(path, "wb") as f:
        f.write(out)


def _gguf_of(tk: T.Tokenizer, path: str, **extra) -> None:
    kv = {"general.architecture": "llama", "tokenizer.ggml.tokens": (8, tk.tokens),
          "tokenizer.ggml.token_type": (5, list(tk.types)), "tokenizer.ggml.bos_token_id": tk.bos,
          "tokenizer.ggml.eos_token_id": tk.eos, "tokenizer.ggml.add_bos_token": tk.add_bos}
    if tk.kind == "spm":
        kv["tokenizer.ggml.model"] = "llama"
        kv["tokenizer.ggml.scores"] = (6, [float(x) for x in tk.scores])
        kv["tokenizer.ggml.add_space_prefix"] = tk.add_space_prefix
    elif tk.kind == "bpe":
        kv["tokenizer.ggml.model"] = "gpt2"
        kv["tokenizer.ggml.pre"] = tk.pre
        kv["tokenizer.ggml.merges"] = (8, extra["merges"])
    _write_meta_gguf(path, kv)


TEXTS = ["hello world", "world", "hé", "[INST]hello</s>", "</s>", "", " ", "  leading", "trailing  ", "a\n\nb",
         "The quick brown fox jumps over the lazy dog. 12345 6789!", "Hello, world! It's a test: don't panic; we'll",
         "Ünïcödé text — with dashes, émojis 🙂 and\nnew lines\n\n  indented   spaces.",
         "def f(x):\n    return x ** 2  # comment\n", "don't we'll THEY'RE 'Ve 'x", "\t\ttabs\t and \r\n crlf \r\r",
         "数字 123456789 ١٢٣ Ⅻ", "<|begin_of_text|>Hello<|eot_id|> x <|eot_id|>", "!!! ??? ... ---", "a  b   c    d",
         "'s'S'll'LL'd", "x\n \n  y", " \n", "🙂🙂 🙂"]


def _check(path: str, py: T.Tokenizer):
    nv = llmi.Vocab.from_file(path)
    try:
        assert nv.n_tokens == py.n_vocab and nv.bos == py.bos and nv.eos == py.eos
        for text in TEXTS:
            for add_special in (True, False):
                for parse_special in (True, False):
                    want = py.tokenize(text, add_special=add_special, parse_special=parse_special)
                    got = nv.tokenize(text, add_special=add_special, parse_special=parse_special)
                    assert got == want, (text, add_special, parse_special, got, want)
        for tid in range(py.n_vocab):
            assert nv.piece(tid) == py.piece(tid), tid
        ids = py.tokenize(TEXTS[12], add_special=False)
        assert nv.detokenize(ids) == b"".join(py.piece(i) for i in ids)
    finally:
        nv.close()


def test_native_spm_matches_host(tmp_path):
    py = TT._spm()
    p = str(tmp_path / "spm.gguf")
    _gguf_of(py, p)
    _check(p, py)
    nv = llmi.Vocab.from_file(p)
    # the hand-pinned segmentations of tests/test_tokenizer.py, natively
    assert [py.tokens[i] for i in nv.tokenize("hello world")] == ["<s>", "▁hello", "▁world"]
    assert [py.tokens[i] for i in nv.tokenize("hé", add_special=False)] == ["▁h", "<0xC3>", "<0xA9>"]
    # special flag: CONTROL tokens render their text only when asked
    assert nv.piece(py.bos) == b"" and nv.piece(py.bos, special=True) == b"<s>"
    assert nv.piece(nv.tokenize("hello", add_special=False)[0], lstrip=1) == b"hello"
    ids = nv.tokenize("hello world")
    assert nv.detokenize(ids, remove_special=True) == b" hello world"
    nv.close()


def test_native_bpe_matches_host(tmp_path):
    pytest.importorskip("tokenizers")
    hf, py = TT._bpe_pair(TT.CORPUS)
    import json

    merges = [m if isinstance(m, str) else " ".join(m) for m in json.loads(hf.to_str())["model"]["merges"]]
    p = str(tmp_path / "bpe.gguf")
    _gguf_of(py, p, merges=merges)
    _check(p, py)
    # and against the tokenizers library directly
    nv = llmi.Vocab.from_file(p)
    for text in TEXTS:
        assert nv.tokenize(text, add_special=False) == hf.encode(text, add_special_tokens=False).ids
    nv.close()


def test_native_gpt2_pretokenizer_matches_host(tmp_path):
    """The gpt-2 default pre-tokenizer (tokenizer.ggml.pre absent / 'default')."""
    pytest.importorskip("tokenizers")
    hf, llama3 = TT._bpe_pair(TT.CORPUS)
    import json

    merges = [m if isinstance(m, str) else " ".join(m) for m in json.loads(hf.to_str())["model"]["merges"]]
    py = T.BpeTokenizer(llama3.tokens, merges, llama3.types, llama3.bos, llama3.eos, add_bos=True, pre="default")
    p = str(tmp_path / "gpt2.gguf")
    _gguf_of(py, p, merges=merges)
    _check(p, py)


def test_native_greedy_synthetic_vocab(tmp_path):
    p = str(tmp_path / "t.gguf")
    llmi.write_synthetic_gguf(p, "tiny-mixed", seed=1)
    py = T.make_tokenizer(T.read_gguf_meta(p))
    assert py.kind == "greedy"
    _check(p, py)
    nv = llmi.Vocab.from_file(p)
    assert nv.tokenize(" w5 w17 w999") == [1, 5, 17, 999]
    nv.close()


def test_tokenize_buffer_protocol(tmp_path):
    """Upstream return conventions: -(count) when the buffer is too small."""
    import ctypes as C

    py = TT._spm()
    p = str(tmp_path / "spm.gguf")
    _gguf_of(py, p)
    nv = llmi.Vocab.from_file(p)
    L = llmi.lib()
    buf = (C.c_int32 * 1)()
    assert L.llama_tokenize(nv._h, b"hello world", 11, buf, 1, True, True) == -3
    cbuf = C.create_string_buffer(2)
    tid = nv.tokenize("hello", add_special=False)[0]
    assert L.llama_token_to_piece(nv._h, tid, cbuf, 2, 0, False) == -len(" hello")
    assert L.llmi_vocab_load_from_file(str(tmp_path / "missing.gguf").encode()) is None
    nv.close()
