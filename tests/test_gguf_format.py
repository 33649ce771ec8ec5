"""The synthetic GGUF writer (csrc/synth_writer.cpp) checked with an independent
pure-Python reader (tests/gguf_reader.py): header, KV table, tensor infos, alignment,
offsets, byte counts and the Llama-3-8B Q4_K_M type table of SURVEY.md §8."""
from __future__ import annotations

import numpy as np
import pytest

import llmi
from gguf_reader import GGML_TYPES, read_gguf

Q4_K, Q5_K, Q6_K, Q8_0, F32 = 12, 13, 14, 8, 0


def _write(tmp_path, preset, **kw):
    p = str(tmp_path / f"{preset}.gguf")
    llmi.write_synthetic_gguf(p, preset, seed=3, **kw)
    return read_gguf(p)


def test_header_and_layout(tmp_path):
    g = _write(tmp_path, "tiny-mixed-d128")
    assert g["version"] == 3 and g["alignment"] == 32 and g["data_start"] % 32 == 0
    kv = g["kv"]
    assert kv["general.architecture"] == "llama"
    E, L = kv["llama.embedding_length"], kv["llama.block_count"]
    H, HK = kv["llama.attention.head_count"], kv["llama.attention.head_count_kv"]
    assert (E, L, H, HK) == (512, 2, 4, 2)
    assert len(kv["tokenizer.ggml.tokens"]) == kv["llama.vocab_size"] == 777
    names = [t["name"] for t in g["tensors"]]
    assert names[0] == "token_embd.weight" and names[-1] == "output.weight" and "output_norm.weight" in names
    end = 0
    for t in g["tensors"]:
        assert t["offset"] % 32 == 0 and t["offset"] >= end
        end = t["offset"] + t["nbytes"]
        assert len(t["data"]) == t["nbytes"]
    assert g["data_start"] + end <= g["file_size"]


def test_llama3_8b_q4km_type_table(tmp_path):
    """Exact Q4_K_M table (token_embd Q4_K, output Q6_K, attn_v/ffn_down Q6_K in the
    use_more_bits layers {0-3, 6, 9, ..., 27, 28-31} of 32) at full width; depth and
    vocab reduced only where the writer is asked to (here: all 32 layers, vocab 512)."""
    g = _write(tmp_path, "llama3-8b-q4km", n_vocab=512)
    by = {t["name"]: t for t in g["tensors"]}
    assert by["token_embd.weight"]["type"] == Q4_K and by["output.weight"]["type"] == Q6_K
    more = {0, 1, 2, 3, 6, 9, 12, 15, 18, 21, 24, 27, 28, 29, 30, 31}
    for i in range(32):
        want = Q6_K if i in more else Q4_K
        assert by[f"blk.{i}.attn_v.weight"]["type"] == want, i
        assert by[f"blk.{i}.ffn_down.weight"]["type"] == want, i
        for n in ("attn_q", "attn_k", "attn_output", "ffn_gate", "ffn_up"):
            assert by[f"blk.{i}.{n}.weight"]["type"] == Q4_K
        assert by[f"blk.{i}.attn_norm.weight"]["type"] == F32
    assert by["blk.0.ffn_gate.weight"]["ne"] == [4096, 14336]
    assert by["blk.0.attn_k.weight"]["ne"] == [4096, 1024]
    layer_bytes = sum(t["nbytes"] for n, t in by.items() if n.startswith("blk."))
    assert abs(layer_bytes - 4186.4e6) / 4186.4e6 < 2e-3  # layers 4186.4 MB


@pytest.mark.parametrize("preset,qt", [("tinyllama-q8_0", Q8_0), ("mistral7b-q6k", Q6_K)])
def test_uniform_presets(tmp_path, preset, qt):
    g = _write(tmp_path, preset, n_layer=1, n_vocab=256)
    for t in g["tensors"]:
        if len(t["ne"]) == 2 and t["name"] != "token_embd.weight":
            assert t["type"] == qt, t["name"]


def test_block_statistics_q4k(tmp_path):
    """Random-init blocks are drawn so dequantized weights have std ~0.02, mean ~0."""
    import pyoracle as po

    g = _write(tmp_path, "tiny-mixed")
    t = next(t for t in g["tensors"] if t["type"] == Q4_K and len(t["ne"]) == 2)
    n = t["ne"][0] * t["ne"][1]
    w = po.dequantize(Q4_K, np.frombuffer(t["data"], np.uint8), n)
    assert abs(float(w.mean())) < 5e-3 and 0.01 < float(w.std()) < 0.04


def _patch_first_tensor_dims(src: str, dst: str, ne0: int, ne1: int) -> None:
    """Rewrite ne[0], ne[1] of the token_embd tensor info (u64 name len + name + u32
    n_dims + u64 ne[]) in a copy of a GGUF file."""
    import struct

    raw = bytearray(open(src, "rb").read())
    name = b"token_embd.weight"
    i = raw.find(struct.pack("<Q", len(name)) + name)
    assert i > 0
    p = i + 8 + len(name) + 4
    raw[p:p + 16] = struct.pack("<qq", ne0, ne1)
    open(dst, "wb").write(bytes(raw))


@pytest.mark.parametrize("ne0,ne1,msg", [(256, -5, "negative dimension"),
                                         (1 << 40, 1 << 40, "overflows"),
                                         (256, 1 << 50, "past end of file")])
def test_malformed_tensor_dims_rejected(tmp_path, ne0, ne1, msg):
    """Negative dims, element counts past INT64_MAX and sizes past the end of the file
    are rejected by the loader (as upstream gguf_init_from_file does) instead of
    wrapping the byte count and reading outside the mmap (vocab_only: no GPU needed)."""
    src = str(tmp_path / "ok.gguf")
    llmi.write_synthetic_gguf(src, "tiny-mixed", seed=1)
    bad = str(tmp_path / "bad.gguf")
    _patch_first_tensor_dims(src, bad, ne0, ne1)
    llmi.Model(src, vocab_only=True).close()
    with pytest.raises(llmi.LlmiError, match=msg):
        llmi.Model(bad, vocab_only=True)
