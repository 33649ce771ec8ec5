"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/ggml_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this, as
the checker.  PARITY UNPINNED by the reference (see ggml_oracle.h / SURVEY.md §8c).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_GENERIC = os.path.join(HERE, "build", "libggml_oracle.so")
LIB_SIMD = os.path.join(HERE, "build", "libggml_oracle_simd.so")
# LLMI_ORACLE=simd selects the -O3 -march=x86-64-v3 build of the same source (bit-identical
# results, tests/test_oracle_simd.py); default: the -O2 generic build
LIB = LIB_SIMD if os.environ.get("LLMI_ORACLE") == "simd" else LIB_GENERIC

F32, F16, Q8_0, Q4_K, Q5_K, Q6_K, Q8_K = 0, 1, 8, 12, 13, 14, 15
BLOCK_ELEMS = {F32: 1, F16: 1, Q8_0: 32, Q4_K: 256, Q5_K: 256, Q6_K: 256, Q8_K: 256}
BLOCK_BYTES = {F32: 4, F16: 2, Q8_0: 34, Q4_K: 144, Q5_K: 176, Q6_K: 210, Q8_K: 292}

_lib = None


def prefer_simd() -> None:
    """Use the -O3 -march=x86-64-v3 build (bit-identical, faster) if the library is not
    loaded yet in this process (the GPU tests call this; CPU tests keep the -O2 build)."""
    global LIB
    if _lib is None and os.path.exists(LIB_SIMD):
        LIB = LIB_SIMD


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def set_fast_dots(on) -> int:
    """CPU-baseline timing only: vectorised dots (not the generic order the parity checks
    use).  on: True / 1 = AVX2 (the baseline's default: faster than the AVX-512BW forms on
    the GPU boxes' Zen 5 host, profiles/r06/cpu_baseline/avx512_ab.txt); 2 = AVX-512BW where
    the host has them.  Returns the mode in effect (2, 1, or 0 = off / no AVX2 build)."""
    mode = 0 if not on else (2 if on == 2 else 1)
    return int(lib().or_set_fast_dots(mode))


# x86 association flags (ggml_oracle.c "x86 association mode"): parity MEASUREMENT only
X86_DOTS, X86_Q80, X86_F16DOT, X86_VEXP, X86_LIBM, X86_NOFMA, X86_FA = 1, 2, 4, 8, 16, 32, 64
X86_ALL = X86_DOTS | X86_Q80 | X86_F16DOT | X86_VEXP  # upstream's AVX2 build as restated


def set_x86_mode(flags: int) -> None:
    """Switch the oracle (process-global) onto upstream's x86 association; 0 = generic."""
    lib().or_set_x86_mode(int(flags))


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    L = C.CDLL(LIB)
    P = C.c_void_p
    sig = {
        "or_type_size": (C.c_size_t, [C.c_int]),
        "or_block_size": (C.c_int, [C.c_int]),
        "or_vec_dot_type": (C.c_int, [C.c_int]),
        "or_fp16_to_fp32": (C.c_float, [C.c_uint16]),
        "or_fp32_to_fp16": (C.c_uint16, [C.c_float]),
        "or_expf": (C.c_float, [C.c_float]),
        "or_expf_glibc_check": (C.c_int64, [C.c_float, C.c_float, C.c_int, C.c_int, C.POINTER(C.c_float)]),
        "or_dequantize_row": (C.c_int, [C.c_int, P, P, C.c_int64]),
        "or_quantize_row_q8_K": (None, [P, P, C.c_int64]),
        "or_quantize_row_q8_0": (None, [P, P, C.c_int64]),
        "or_vec_dot": (C.c_float, [C.c_int, C.c_int, P, P]),
        "or_matvec": (C.c_int, [C.c_int, P, C.c_int64, C.c_int64, P, P, C.c_int]),
        "or_rms_norm_mul": (None, [P, P, P, C.c_int, C.c_float]),
        "or_model_load": (P, [C.c_char_p, C.c_int]),
        "or_model_free": (None, [P]),
        "or_model_localize": (C.c_int64, [P, C.c_int]),
        "or_last_error": (C.c_char_p, []),
        "or_model_info": (None, [P, P]),
        "or_decode": (C.c_int, [P, C.c_int32, C.c_int32, P, C.c_int]),
        "or_kv_clear": (None, [P]),
        "or_prefill": (C.c_int, [P, P, C.c_int, C.c_int32, C.c_int]),
        "or_host_stream_gbps": (C.c_double, [C.c_size_t, C.c_int, C.c_int]),
        "or_tap": (C.c_int, [P, C.c_int, P]),
        "or_bytes_per_token": (C.c_double, [P, C.c_int]),
        "or_set_fast_dots": (C.c_int, [C.c_int]),
        "or_set_x86_mode": (C.c_int, [C.c_int]),
        "or_quantize_act": (C.c_int, [C.c_int, P, P, C.c_int64]),
        "or_get_x86_mode": (C.c_int, []),
    }
    for k, (r, a) in sig.items():
        f = getattr(L, k)
        f.restype = r
        f.argtypes = a
    _lib = L
    return L


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def nthreads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def physical_cores() -> int:
    """Physical cores of this host (unique (package, core) pairs in /proc/cpuinfo)."""
    pairs, phys, core = set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("physical id"):
                    phys = ln.split(":")[1].strip()
                elif ln.startswith("core id"):
                    core = ln.split(":")[1].strip()
                elif not ln.strip():
                    if core is not None:
                        pairs.add((phys, core))
                    phys = core = None
    except OSError:
        pass
    return len(pairs) or (os.cpu_count() or 1)


def host_stream_gbps(nbytes: int = 1 << 30, reps: int = 3, threads: int = 0) -> float:
    return float(lib().or_host_stream_gbps(int(nbytes), int(reps), threads or nthreads()))


def dequantize(type_: int, raw: np.ndarray, n: int) -> np.ndarray:
    raw = np.ascontiguousarray(raw, dtype=np.uint8)
    out = np.empty(n, dtype=np.float32)
    assert lib().or_dequantize_row(type_, _p(raw), _p(out), n) == 0
    return out


def quantize_q8_K(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.zeros(x.size // 256 * 292, dtype=np.uint8)
    lib().or_quantize_row_q8_K(_p(x), _p(out), x.size)
    return out


def quantize_q8_0(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.zeros(x.size // 32 * 34, dtype=np.uint8)
    lib().or_quantize_row_q8_0(_p(x), _p(out), x.size)
    return out


def quantize_act(wtype: int, x: np.ndarray, x86: int | None = None) -> np.ndarray:
    """The activation conversion of a matvec with weight type wtype; x86: the oracle's
    association flags for the call (X86_Q80: upstream's x86 round-half-even q8_0; None:
    the current mode)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = x.size // 32 * 34 if wtype == Q8_0 else x.size // 256 * 292
    out = np.zeros(n, dtype=np.uint8)
    with x86_mode(x86):
        assert lib().or_quantize_act(wtype, _p(x), _p(out), x.size) == 0
    return out


class x86_mode:
    """Context manager: the oracle's (process-global) association flags for a block."""

    def __init__(self, flags: int | None):
        self.flags = flags  # None: leave the current mode

    def __enter__(self):
        self.old = int(lib().or_get_x86_mode())
        if self.flags is not None:
            lib().or_set_x86_mode(int(self.flags))
        return self

    def __exit__(self, *exc):
        lib().or_set_x86_mode(self.old)
        return False


def rms_norm_mul(x: np.ndarray, w: np.ndarray, eps: float) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    w = np.ascontiguousarray(w, dtype=np.float32)
    y = np.empty_like(x)
    lib().or_rms_norm_mul(_p(x), _p(w), _p(y), x.size, eps)
    return y


def matvec(type_: int, W: np.ndarray, rows: int, cols: int, x: np.ndarray, threads: int = 0,
           x86: int | None = None) -> np.ndarray:
    W = np.ascontiguousarray(W, dtype=np.uint8)
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty(rows, dtype=np.float32)
    with x86_mode(x86):
        assert lib().or_matvec(type_, _p(W), rows, cols, _p(x), _p(y), threads or nthreads()) == 0
    return y


def expf(x: float) -> float:
    return float(lib().or_expf(x))


class OracleModel:
    """Whole-model decode (llm_build_llama order) on the CPU, f16 KV cache."""

    def __init__(self, path: str, n_ctx: int = 512, threads: int = 0, x86: int = 0):
        """x86: association flags applied around this model's calls (0 = the generic order
        the parity checks use; nonzero only for the x86 distance measurement)."""
        L = lib()
        self.x86 = int(x86)
        self._h = L.or_model_load(path.encode(), n_ctx)
        if not self._h:
            raise RuntimeError("oracle load failed: " + L.or_last_error().decode())
        info = np.zeros(10, dtype=np.int64)
        L.or_model_info(self._h, _p(info))
        (self.n_embd, self.n_layer, self.n_head, self.n_head_kv, self.n_ff, self.n_vocab,
         self.n_rot, self.n_ctx, self.head_dim, self.file_type) = (int(v) for v in info)
        self.threads = threads or nthreads()

    def localize(self) -> int:
        """Copy the decode matrices into anonymous memory, each row first-touched by the
        OpenMP thread (of self.threads) that reads it (NUMA placement; numerics unchanged)."""
        n = int(lib().or_model_localize(self._h, self.threads))
        if n < 0:
            raise RuntimeError("or_model_localize: out of memory")
        return n

    def decode(self, token: int, pos: int, logits: bool = True) -> np.ndarray | None:
        """One decode step; logits=False skips the output head (prompt tokens)."""
        out = np.empty(self.n_vocab, dtype=np.float32) if logits else None
        with x86_mode(self.x86):  # the mode is process-global: restored after the call
            rc = lib().or_decode(self._h, int(token), int(pos), _p(out) if logits else None, self.threads)
        if rc != 0:
            raise RuntimeError(f"or_decode rc={rc}: " + lib().or_last_error().decode())
        return out

    def prefill(self, tokens, pos0: int = 0) -> None:
        """T decode steps at pos0.. with no logits (or_prefill: the same operations per
        token, loops reordered so each weight row is unpacked once)."""
        toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32))
        with x86_mode(self.x86):
            rc = lib().or_prefill(self._h, _p(toks), int(toks.size), int(pos0), self.threads)
        if rc != 0:
            raise RuntimeError(f"or_prefill rc={rc}: " + lib().or_last_error().decode())

    def tap(self, which: int) -> np.ndarray:
        """or_tap: 0 embedding row, 1 final hidden (pre-norm), 2 roped q, 3 attention
        output, 4 SwiGLU output, 5 roped k, 6 v (last layer of the last step); 7 / 8 the
        last layer's raw f16 K / V cache [n_ctx][n_head_kv * head_dim]."""
        kvd = self.n_head_kv * self.head_dim
        n = {0: self.n_embd, 1: self.n_embd, 2: self.n_head * self.head_dim, 3: self.n_head * self.head_dim,
             4: self.n_ff, 5: kvd, 6: kvd}.get(which)
        if which in (7, 8):
            out = np.empty(self.n_ctx * kvd, dtype=np.uint16)
        elif n is None:
            raise ValueError(f"tap {which}")
        else:
            out = np.empty(n, dtype=np.float32)
        assert lib().or_tap(self._h, which, _p(out)) == 0
        return out

    def kv_clear(self) -> None:
        lib().or_kv_clear(self._h)

    def bytes_per_token(self, ctx: int) -> float:
        return float(lib().or_bytes_per_token(self._h, ctx))

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().or_model_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
