"""ctypes binding of libllmi.so (include/llmi.h).

This is exactly the binding a caller of the reference's decode path would add
(INTEGRATION.md): plain C types, opaque handles, no torch in any signature.
The product path has no fallback: if the HIP library is missing, loading fails
loudly (LlmiLibraryError) instead of degrading to a CPU implementation.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LLMI_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libllmi.so")


class LlmiLibraryError(RuntimeError):
    pass


class llama_model_params(C.Structure):
    _fields_ = [
        ("n_gpu_layers", C.c_int32),
        ("main_gpu", C.c_int32),
        ("vocab_only", C.c_bool),
        ("use_mmap", C.c_bool),
        ("no_upload", C.c_bool),
        ("numerics", C.c_int32),
    ]


class llama_context_params(C.Structure):
    _fields_ = [
        ("n_ctx", C.c_uint32),
        ("n_batch", C.c_uint32),
        ("n_ubatch", C.c_uint32),
        ("n_seq_max", C.c_uint32),
        ("n_threads", C.c_int32),
        ("use_graphs", C.c_bool),
    ]


class llama_batch(C.Structure):
    _fields_ = [
        ("n_tokens", C.c_int32),
        ("token", C.POINTER(C.c_int32)),
        ("embd", C.POINTER(C.c_float)),
        ("pos", C.POINTER(C.c_int32)),
        ("n_seq_id", C.POINTER(C.c_int32)),
        ("seq_id", C.POINTER(C.POINTER(C.c_int32))),
        ("logits", C.POINTER(C.c_int8)),
    ]


# name -> (restype, argtypes); every entry point declared in include/llmi.h
_P = C.c_void_p
SIGNATURES = {
    "llama_backend_init": (None, []),
    "llama_backend_free": (None, []),
    "llama_model_default_params": (llama_model_params, []),
    "llama_context_default_params": (llama_context_params, []),
    "llama_model_load_from_file": (_P, [C.c_char_p, llama_model_params]),
    "llama_model_free": (None, [_P]),
    "llama_init_from_model": (_P, [_P, llama_context_params]),
    "llama_free": (None, [_P]),
    "llama_batch_get_one": (llama_batch, [C.POINTER(C.c_int32), C.c_int32]),
    "llama_batch_init": (llama_batch, [C.c_int32, C.c_int32, C.c_int32]),
    "llama_batch_free": (None, [llama_batch]),
    "llama_decode": (C.c_int32, [_P, llama_batch]),
    "llama_eval": (C.c_int, [_P, C.POINTER(C.c_int32), C.c_int32, C.c_int32]),
    "llama_get_logits": (C.POINTER(C.c_float), [_P]),
    "llama_get_logits_ith": (C.POINTER(C.c_float), [_P, C.c_int32]),
    "llama_model_get_vocab": (_P, [_P]),
    "llama_vocab_n_tokens": (C.c_int32, [_P]),
    "llama_vocab_bos": (C.c_int32, [_P]),
    "llama_vocab_eos": (C.c_int32, [_P]),
    "llama_vocab_get_text": (C.c_char_p, [_P, C.c_int32]),
    "llama_vocab_get_add_bos": (C.c_bool, [_P]),
    "llama_tokenize": (C.c_int32, [_P, C.c_char_p, C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.c_bool, C.c_bool]),
    "llama_token_to_piece": (C.c_int32, [_P, C.c_int32, C.c_char_p, C.c_int32, C.c_int32, C.c_bool]),
    "llama_detokenize": (C.c_int32, [_P, C.POINTER(C.c_int32), C.c_int32, C.c_char_p, C.c_int32, C.c_bool, C.c_bool]),
    "llmi_vocab_load_from_file": (_P, [C.c_char_p]),
    "llmi_vocab_free": (None, [_P]),
    "llama_model_n_embd": (C.c_int32, [_P]),
    "llama_model_n_layer": (C.c_int32, [_P]),
    "llama_model_n_head": (C.c_int32, [_P]),
    "llama_model_n_head_kv": (C.c_int32, [_P]),
    "llama_model_n_ctx_train": (C.c_int32, [_P]),
    "llama_model_size": (C.c_uint64, [_P]),
    "llama_model_desc": (C.c_int32, [_P, C.c_char_p, C.c_size_t]),
    "llama_n_ctx": (C.c_uint32, [_P]),
    "llama_kv_self_clear": (None, [_P]),
    "llmi_last_error": (C.c_char_p, []),
    "llmi_model_numerics": (C.c_int32, [_P]),
    "llmi_device_count": (C.c_int32, []),
    "llmi_greedy_ith": (C.c_int32, [_P, C.c_int32]),
    "llmi_generate_greedy": (C.c_int32, [_P, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]),
    "llmi_generate_greedy_batch": (C.c_int32, [_P, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                               C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_int32)]),
    "llama_kv_self_seq_rm": (C.c_bool, [_P, C.c_int32, C.c_int32, C.c_int32]),
    "llmi_seq_pos_max": (C.c_int32, [_P, C.c_int32]),
    "llmi_model_upload_s": (C.c_double, [_P]),
    "llmi_last_step_stats": (None, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "llmi_test_option": (C.c_int32, [C.c_char_p, C.c_int32]),
    "llmi_le_stream_bench": (C.c_double, [_P, C.c_int64, C.c_int32, C.c_int32, C.c_int32]),
    "llmi_engine_trace": (C.c_int32, [_P, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_uint64), C.c_int64]),
    "llmi_bytes_per_token": (C.c_double, [_P, C.c_int32]),
    "llmi_profile_kernels": (C.c_int32, [_P, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_double),
                                         C.POINTER(C.c_double), C.POINTER(C.c_int32)]),
    "llmi_prefill_supported": (C.c_int32, [_P]),
    "llmi_debug_tap": (C.c_int32, [_P, C.c_int32, _P]),
    "llmi_pf_gemm": (C.c_int32, [C.c_int32, _P, C.c_int64, C.c_int64, _P, _P, C.c_float, C.c_int32, _P,
                                 C.POINTER(C.c_double)]),
    "llmi_model_arena": (C.c_int32, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "llmi_model_arena_hash": (C.c_int32, [_P, C.POINTER(C.c_uint64)]),
    "llmi_device_hash": (C.c_int32, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    "llmi_attention": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P, C.c_int32]),
    "llmi_pf_attention": (C.c_double, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P,
                                       _P, C.c_int32, C.c_int64]),
    "llmi_replicate": (C.c_int32, [_P, C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_void_p)]),
    "llmi_rccl_unique_id": (C.c_int32, [C.c_char_p, C.c_int32]),
    "llmi_model_fanout": (C.c_int32, [_P, C.c_char_p, C.c_int32, C.c_int32]),
    "llmi_model_load_fanout": (_P, [C.c_char_p, llama_model_params, C.c_char_p, C.c_int32, C.c_int32]),
    "llmi_model_load_replicated": (_P, [C.c_char_p, llama_model_params, C.POINTER(C.c_int32), C.c_int32,
                                        C.POINTER(C.c_void_p)]),
    "llmi_fanout_plan": (C.c_int32, [C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64), C.c_int32,
                                     C.POINTER(C.c_int32), C.c_int32]),
    "llmi_synth_write_gguf": (C.c_int64, [C.c_char_p, C.c_char_p, C.c_uint64, C.c_int32, C.c_int32, C.c_int32]),
    "llmi_device_layout_bytes": (C.c_int64, [C.c_int32, C.c_int64, C.c_int64]),
    "llmi_repack": (C.c_int32, [C.c_int32, _P, _P, C.c_int64, C.c_int64]),
    "llmi_matvec": (C.c_int32, [C.c_int32, _P, C.c_int64, C.c_int64, _P, _P, C.c_float, _P, C.c_int32]),
    "llmi_quantize_act": (C.c_int32, [C.c_int32, C.c_int64, _P, _P, C.c_float, _P]),
    "llmi_bench_stream": (C.c_double, [_P, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32, C.c_int32]),
    "llmi_bench_matvec": (C.c_double, [C.c_int32, _P, C.c_int32, C.c_int64, C.c_int64, _P, _P, C.c_int32]),
    "llmi_bench_matvec_ex": (C.c_double, [C.c_int32, _P, C.c_int32, C.c_int64, C.c_int64, _P, _P, C.c_int32, C.c_int32]),
    "llmi_trace_matvec": (C.c_int32, [C.c_int32, _P, C.c_int64, C.c_int64, _P, _P, C.c_int32, _P]),
    "llmi_bench_attention": (C.c_double, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libllmi.so (built by `make -C llama-gguf-inference_amd`); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (same soname
    # libamdhip64.so.7).  If torch is installed, load it first so libllmi binds to the
    # already-loaded runtime instead of pulling in a second copy (two runtimes in one
    # process make torch's device init fail: "No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise LlmiLibraryError(
            f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the product has no CPU fallback)"
        )
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error() -> str:
    e = lib().llmi_last_error()
    return e.decode() if e else ""
