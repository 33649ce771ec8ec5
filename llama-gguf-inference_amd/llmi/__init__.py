"""llmi — MI355X-native GGUF decode path (Python host side over the libllmi.so C ABI).

Mirrors the llama.cpp decode surface the reference's llama-server drives
(SURVEY.md §8b): a Model is `llama_model_load_from_file`, a Context is
`llama_init_from_model`, `Context.decode` is `llama_decode` with the same return
codes, `Context.logits` is `llama_get_logits_ith`.  All compute runs in the HIP
library; nothing here computes numerics.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from ._lib import LlmiLibraryError, last_error, lib, llama_context_params, llama_model_params  # noqa: F401

# ggml type ids
F32, F16, Q8_0, Q4_K, Q5_K, Q6_K, Q8_K = 0, 1, 8, 12, 13, 14, 15
# model numerics (llama_model_params.numerics): ggml's generic scalar order, or upstream's
# x86 AVX2 association (the reference's NGL=0 build)
NUMERICS_GENERIC, NUMERICS_X86, NUMERICS_FA = 0, 1, 2  # NUMERICS_FA is OR-ed into either (llmi.h)
PRESETS = (
    "llama3-8b-q4km", "llama3-70b-q4km", "tinyllama-q8_0", "mistral7b-q6k", "mistral7b-q5km",
    "tiny-mixed", "tiny-mixed-d128",
)


class LlmiError(RuntimeError):
    pass


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    if lib().llmi_rccl_unique_id(buf, 128) != 0:
        raise LlmiError(last_error())
    return buf.raw


def test_option(name: str, value: int = -1) -> int:
    """llmi_test_option: set a test-only option (value < 0: query); returns the old value."""
    r = int(lib().llmi_test_option(name.encode(), int(value)))
    if r < 0:
        raise LlmiError(last_error())
    return r


def device_count() -> int:
    return int(lib().llmi_device_count())


def fanout_plan(arena_bytes: int, chunk: int, prefix_ends: Sequence[int]) -> list[int]:
    """The replica fan-out schedule (engine.cpp fanout_plan): for each chunk-sized piece of
    the arena, the index of the first upload prefix that covers it.  Host only."""
    n = len(prefix_ends)
    pe = (C.c_uint64 * max(1, n))(*prefix_ends)
    cap = (arena_bytes + chunk - 1) // chunk if chunk else 0
    rd = (C.c_int32 * max(1, cap))()
    k = lib().llmi_fanout_plan(int(arena_bytes), int(chunk), pe, n, rd, int(cap))
    if k < 0:
        raise LlmiError("llmi_fanout_plan: bad arguments")
    return [int(rd[i]) for i in range(k)]


def write_synthetic_gguf(path: str, preset: str, seed: int = 3, n_layer: int = 0, n_vocab: int = 0,
                         n_threads: int = 0) -> int:
    """Write a synthetic GGUF with the exact shapes/type table of `preset`."""
    n = lib().llmi_synth_write_gguf(path.encode(), preset.encode(), seed, n_layer, n_vocab, n_threads)
    if n < 0:
        raise LlmiError(last_error())
    return int(n)


class Vocab:
    """The native tokenizer (llama_tokenize / llama_token_to_piece / llama_detokenize of
    the C ABI, csrc/tokenizer.cpp).  From a model (Model.vocab) or, tokenizer only, from
    any GGUF's metadata (Vocab.from_file)."""

    def __init__(self, handle, owned: bool = False, keep=None):
        if not handle:
            raise LlmiError(f"vocab: {last_error()}")
        self._h, self._owned, self._keep = handle, owned, keep

    @classmethod
    def from_file(cls, path: str) -> "Vocab":
        return cls(lib().llmi_vocab_load_from_file(path.encode()), owned=True)

    @property
    def n_tokens(self) -> int:
        return lib().llama_vocab_n_tokens(self._h)

    @property
    def bos(self) -> int:
        return lib().llama_vocab_bos(self._h)

    @property
    def eos(self) -> int:
        return lib().llama_vocab_eos(self._h)

    def tokenize(self, text: str, add_special: bool = True, parse_special: bool = True) -> list[int]:
        L = lib()
        b = text.encode("utf-8")
        cap = len(b) + 8
        while True:
            buf = (C.c_int32 * cap)()
            n = L.llama_tokenize(self._h, b, len(b), buf, cap, add_special, parse_special)
            if n == -(2 ** 31):
                raise LlmiError(f"llama_tokenize: {last_error()}")
            if n >= 0:
                return list(buf[:n])
            cap = -n

    def piece(self, tid: int, special: bool = False, lstrip: int = 0) -> bytes:
        L = lib()
        buf = C.create_string_buffer(64)
        n = L.llama_token_to_piece(self._h, int(tid), buf, 64, lstrip, special)
        if n < 0:
            buf = C.create_string_buffer(-n)
            n = L.llama_token_to_piece(self._h, int(tid), buf, -n, lstrip, special)
        return buf.raw[:n]

    def detokenize(self, ids: Sequence[int], remove_special: bool = False, unparse_special: bool = False) -> bytes:
        L = lib()
        arr = (C.c_int32 * max(1, len(ids)))(*ids)
        cap = 16 * len(ids) + 16
        buf = C.create_string_buffer(cap)
        n = L.llama_detokenize(self._h, arr, len(ids), buf, cap, remove_special, unparse_special)
        if n < 0:
            buf = C.create_string_buffer(-n)
            n = L.llama_detokenize(self._h, arr, len(ids), buf, -n, remove_special, unparse_special)
        return buf.raw[:n]

    def close(self) -> None:
        if self._owned and self._h:
            lib().llmi_vocab_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass



def device_hash(ptr: int, nbytes: int) -> int:
    """llmi_device_hash: the arena hash of any device memory (test hook)."""
    h = C.c_uint64()
    if lib().llmi_device_hash(C.c_void_p(ptr), int(nbytes), C.byref(h)) != 0:
        raise LlmiError(last_error())
    return int(h.value)

class Model:
    """llama_model_load_from_file: GGUF -> HBM arena on `main_gpu`."""

    def __init__(self, path: str, n_gpu_layers: int = 999, main_gpu: int = 0, vocab_only: bool = False,
                 no_upload: bool = False, numerics: int = NUMERICS_GENERIC):
        L = lib()
        p = L.llama_model_default_params()
        p.n_gpu_layers = n_gpu_layers
        p.main_gpu = main_gpu
        p.vocab_only = vocab_only
        p.no_upload = no_upload
        p.numerics = numerics
        self._h = L.llama_model_load_from_file(path.encode(), p)
        if not self._h:
            raise LlmiError(last_error())
        self.path = path
        self.device = main_gpu
        v = L.llama_model_get_vocab(self._h)
        self._vocab = v
        self.n_vocab = L.llama_vocab_n_tokens(v)
        self.bos = L.llama_vocab_bos(v)
        self.eos = L.llama_vocab_eos(v)
        self.n_embd = L.llama_model_n_embd(self._h)
        self.n_layer = L.llama_model_n_layer(self._h)
        self.n_head = L.llama_model_n_head(self._h)
        self.n_head_kv = L.llama_model_n_head_kv(self._h)
        self.n_ctx_train = L.llama_model_n_ctx_train(self._h)
        self.size = int(L.llama_model_size(self._h))
        buf = C.create_string_buffer(256)
        L.llama_model_desc(self._h, buf, 256)
        self.desc = buf.value.decode()
        self.numerics = int(L.llmi_model_numerics(self._h))

    @classmethod
    def load_fanout(cls, path: str, main_gpu: int, uid: bytes, nranks: int, rank: int,
                    numerics: int = NUMERICS_GENERIC) -> "Model":
        """Load with the replica fan-out pipelined behind the upload (llmi_model_load_fanout,
        SURVEY.md §8e): every rank calls it with the same RCCL unique id; rank 0 uploads the
        GGUF, the others receive the arena in 256 MB pieces over xGMI."""
        L = lib()
        p = L.llama_model_default_params()
        p.main_gpu = main_gpu
        p.numerics = numerics
        h = L.llmi_model_load_fanout(path.encode(), p, uid, int(nranks), int(rank))
        if not h:
            raise LlmiError(last_error())
        return cls._from_handle(h, path, main_gpu)

    @classmethod
    def load_replicated(cls, path: str, main_gpu: int, devices: Sequence[int], n_gpu_layers: int = 999,
                        numerics: int = NUMERICS_GENERIC) -> tuple["Model", list["Model"]]:
        """One process: the model on main_gpu and a replica on each of `devices`, the RCCL
        broadcast pipelined behind the upload (llmi_model_load_replicated)."""
        L = lib()
        p = L.llama_model_default_params()
        p.main_gpu = main_gpu
        p.n_gpu_layers = n_gpu_layers
        p.numerics = numerics
        n = len(devices)
        devs = (C.c_int32 * max(1, n))(*devices)
        out = (C.c_void_p * max(1, n))()
        h = L.llmi_model_load_replicated(path.encode(), p, devs, n, out)
        if not h:
            raise LlmiError(last_error())
        return cls._from_handle(h, path, main_gpu), [cls._from_handle(out[i], path, devices[i]) for i in range(n)]

    @classmethod
    def _from_handle(cls, h, path: str, device: int) -> "Model":
        self = cls.__new__(cls)
        L = lib()
        self._h = h
        self.path = path
        self.device = device
        v = L.llama_model_get_vocab(h)
        self._vocab = v
        self.n_vocab = L.llama_vocab_n_tokens(v)
        self.bos, self.eos = L.llama_vocab_bos(v), L.llama_vocab_eos(v)
        self.n_embd, self.n_layer = L.llama_model_n_embd(h), L.llama_model_n_layer(h)
        self.n_head, self.n_head_kv = L.llama_model_n_head(h), L.llama_model_n_head_kv(h)
        self.n_ctx_train = L.llama_model_n_ctx_train(h)
        self.size = int(L.llama_model_size(h))
        self.desc = ""
        self.numerics = int(L.llmi_model_numerics(h))
        return self

    @property
    def vocab(self) -> Vocab:
        """The model's native tokenizer (owned by the model)."""
        return Vocab(self._vocab, owned=False, keep=self)

    def token_text(self, t: int) -> str:
        s = lib().llama_vocab_get_text(self._vocab, int(t))
        return s.decode("utf-8", "replace") if s is not None else ""

    @property
    def upload_s(self) -> float:
        """Seconds of the weight upload (chunked pinned H2D + on-device repack)."""
        return float(lib().llmi_model_upload_s(self._h))

    def bytes_per_token(self, n_kv: int) -> float:
        return float(lib().llmi_bytes_per_token(self._h, int(n_kv)))

    @property
    def prefill_supported(self) -> bool:
        """Whether llama_decode prefills prompts with the batched MFMA path."""
        return bool(lib().llmi_prefill_supported(self._h))

    def arena(self) -> tuple[int, int]:
        p, n = C.c_void_p(), C.c_uint64()
        lib().llmi_model_arena(self._h, C.byref(p), C.byref(n))
        return int(p.value or 0), int(n.value)

    def arena_hash(self) -> int:
        """Order-independent 64-bit hash of the device arena (llmi_model_arena_hash): equal
        on every replica of the same weights (the fan-out's replica check)."""
        h = C.c_uint64()
        if lib().llmi_model_arena_hash(self._h, C.byref(h)) != 0:
            raise LlmiError(last_error())
        return int(h.value)

    def replicate(self, devices: Sequence[int]) -> list["Model"]:
        """In-process RCCL broadcast of the arena to `devices`."""
        n = len(devices)
        devs = (C.c_int32 * n)(*devices)
        out = (C.c_void_p * n)()
        if lib().llmi_replicate(self._h, devs, n, out) != 0:
            raise LlmiError(last_error())
        return [Model._from_handle(out[i], self.path, devices[i]) for i in range(n)]

    def fanout(self, uid: bytes, nranks: int, rank: int) -> None:
        """Multi-process replica fan-out: RCCL broadcast of rank 0's arena."""
        if lib().llmi_model_fanout(self._h, uid, int(nranks), int(rank)) != 0:
            raise LlmiError(last_error())

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().llama_model_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """llama_init_from_model: KV cache + scratch + step graphs on the model's device."""

    def __init__(self, model: Model, n_ctx: int = 0, use_graphs: bool = True, n_seq: int = 1):
        L = lib()
        p = L.llama_context_default_params()
        p.n_ctx = n_ctx
        p.use_graphs = use_graphs
        p.n_seq_max = n_seq
        self.n_seq = n_seq
        self._h = L.llama_init_from_model(model._h, p)
        if not self._h:
            raise LlmiError(last_error())
        self.model = model
        self.n_ctx = int(L.llama_n_ctx(self._h))

    def decode(self, tokens: Sequence[int], pos: Optional[Sequence[int]] = None, logits_all: bool = False,
               seq: Optional[Sequence[int]] = None) -> int:
        """llama_decode: returns 0 ok, 1 no KV slot, <0 error (same codes as upstream).
        seq: per-token sequence id (llama_batch.seq_id[i][0]); None = sequence 0."""
        n = len(tokens)
        toks = (C.c_int32 * n)(*tokens)
        b = lib().llama_batch_get_one(toks, n)
        keep = [toks]
        if seq is not None:
            ids = [(C.c_int32 * 1)(int(s)) for s in seq]
            ptrs = (C.POINTER(C.c_int32) * n)(*[C.cast(a, C.POINTER(C.c_int32)) for a in ids])
            nsi = (C.c_int32 * n)(*([1] * n))
            b.seq_id = C.cast(ptrs, C.POINTER(C.POINTER(C.c_int32)))
            b.n_seq_id = C.cast(nsi, C.POINTER(C.c_int32))
            keep += [ids, ptrs, nsi]
        if pos is not None:
            pa = (C.c_int32 * n)(*pos)
            b.pos = C.cast(pa, C.POINTER(C.c_int32))
            keep.append(pa)
        if logits_all:
            la = (C.c_int8 * n)(*([1] * n))
            b.logits = C.cast(la, C.POINTER(C.c_int8))
            keep.append(la)
        rc = int(lib().llama_decode(self._h, b))
        del keep
        return rc

    def eval(self, tokens: Sequence[int], n_past: int) -> int:
        n = len(tokens)
        toks = (C.c_int32 * n)(*tokens)
        return int(lib().llama_eval(self._h, toks, n, n_past))

    def logits(self, i: int = -1) -> np.ndarray:
        p = lib().llama_get_logits_ith(self._h, i)
        if not p:
            raise LlmiError(last_error())
        return np.ctypeslib.as_array(p, shape=(self.model.n_vocab,)).copy()

    def tap(self, which: int, n: int) -> np.ndarray:
        """llmi_debug_tap of the last decode step (the oracle's or_tap numbering): 0
        embedding row, 1 residual x after the last layer, 2 roped q, 3 attention output,
        4 SwiGLU output (the last layer's); 7 / 8 the last layer's raw f16 K / V cache.
        n = element count (f32; u16 for 7 / 8)."""
        out = np.empty(n, dtype=np.uint16 if which in (7, 8) else np.float32)
        if lib().llmi_debug_tap(self._h, int(which), out.ctypes.data_as(C.c_void_p)) != 0:
            raise LlmiError(last_error())
        return out

    def greedy(self, i: int = -1) -> int:
        t = int(lib().llmi_greedy_ith(self._h, i))
        if t < 0:
            raise LlmiError(last_error())
        return t

    def generate_greedy(self, first: int, pos0: int, n: int) -> list[int]:
        out = (C.c_int32 * n)()
        r = lib().llmi_generate_greedy(self._h, int(first), int(pos0), int(n), out)
        if r != n:
            raise LlmiError(f"llmi_generate_greedy returned {r}: {last_error()}")
        return list(out)

    def generate_greedy_batch(self, seqs: Sequence[int], first: Sequence[int], pos0: Sequence[int], n: int) -> list[list[int]]:
        """llmi_generate_greedy_batch: sequences seqs advance together, one batched step
        per token (continuous batching); returns each sequence's n tokens."""
        k = len(seqs)
        sa, fa, pa = (C.c_int32 * k)(*seqs), (C.c_int32 * k)(*first), (C.c_int32 * k)(*pos0)
        out = (C.c_int32 * (k * n))()
        r = lib().llmi_generate_greedy_batch(self._h, k, sa, fa, pa, int(n), out)
        if r != n:
            raise LlmiError(f"llmi_generate_greedy_batch returned {r}: {last_error()}")
        return [list(out[i * n:(i + 1) * n]) for i in range(k)]

    def seq_rm(self, seq: int, p0: int = 0, p1: int = -1) -> bool:
        """llama_kv_self_seq_rm (tail removal)."""
        return bool(lib().llama_kv_self_seq_rm(self._h, int(seq), int(p0), int(p1)))

    def seq_pos_max(self, seq: int) -> int:
        return int(lib().llmi_seq_pos_max(self._h, int(seq)))

    def stats(self) -> tuple[float, float]:
        b, u = C.c_double(), C.c_double()
        lib().llmi_last_step_stats(self._h, C.byref(b), C.byref(u))
        return b.value, u.value

    KERNEL_CLASSES = ("embed", "qkv", "attention", "attn_output", "ffn_gate_up", "ffn_down", "output", "layer")

    def profile_kernels(self, first: int, pos0: int, n_steps: int) -> dict:
        """Per-kernel-class mean kernel execution time / algorithmic bytes per launch:
        each class's launches of n_steps steps at pos0, every launch bracketed by HIP
        events recorded at kernel start/end (llmi_profile_kernels).  Consumes no tokens."""
        n = len(self.KERNEL_CLASSES)
        us, by, nl = (C.c_double * n)(), (C.c_double * n)(), (C.c_int32 * n)()
        if lib().llmi_profile_kernels(self._h, int(first), int(pos0), int(n_steps), us, by, nl) != 0:
            raise LlmiError(last_error())
        return {k: {"us": us[i], "bytes": by[i], "launches_per_step": nl[i],
                    "GBps": (by[i] / (us[i] * 1e-6) / 1e9) if us[i] > 0 else 0.0}
                for i, k in enumerate(self.KERNEL_CLASSES)}

    def engine_trace(self, first: int, pos0: int, layer: int) -> np.ndarray:
        """llmi_engine_trace: s_memrealtime stamps (10 ns ticks) of layer `layer`'s layer-engine
        launch in one eager step at pos0, shaped [CUs][16 wave slots][32] (tools/letrace.py)."""
        n = 256 * 16 * 32 * 4
        out = (C.c_uint64 * n)()
        g = int(lib().llmi_engine_trace(self._h, int(first), int(pos0), int(layer), out, n))
        if g < 0:
            raise LlmiError(last_error())
        return np.ctypeslib.as_array(out)[: g * 16 * 32].reshape(g, 16, 32).copy()

    def kv_clear(self) -> None:
        lib().llama_kv_self_clear(self._h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().llama_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
