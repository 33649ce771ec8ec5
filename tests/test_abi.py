"""The C-ABI library (include/llmi.h) without a GPU: it loads, exports every function
the headers declare, the ctypes signature table covers exactly that set, and the
no-GPU error paths fail loudly (no CPU fallback)."""
from __future__ import annotations

import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "llmi.h")
LIB = os.path.join(ROOT, "llama-gguf-inference_amd", "lib", "libllmi.so")


def declared_functions() -> set[str]:
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = set()
    for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(([^;{}]*)\)\s*;", src):
        name = m.group(1)
        if name in ("if", "while", "for", "return", "sizeof"):
            continue
        names.add(name)
    return names


def exported_symbols() -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_every_declared_function_is_exported():
    decl = declared_functions()
    assert len(decl) > 40
    missing = decl - exported_symbols()
    assert not missing, f"declared but not exported: {sorted(missing)}"


def test_only_abi_symbols_exported():
    """-fvisibility=hidden: the library's dynamic text symbols are the ABI, nothing else."""
    extra = {s for s in exported_symbols() if not s.startswith(("llama_", "llmi_"))}
    assert not extra, sorted(extra)[:20]


def test_ctypes_table_matches_header():
    from llmi._lib import SIGNATURES

    assert set(SIGNATURES) == declared_functions()


def test_library_loads_and_reports_errors_without_gpu():
    import ctypes as C

    from llmi._lib import lib

    L = lib()
    assert L.llmi_device_count() >= 0
    # a missing model file is an error, never a CPU fallback
    p = L.llama_model_default_params()
    assert L.llama_model_load_from_file(b"/nonexistent.gguf", p) is None
    assert L.llmi_last_error()
    assert C.sizeof(C.c_void_p) == 8


def test_n_gpu_layers_zero_is_refused(tmp_path):
    """NGL=0 asks for the CPU path: this build has none (the oracle is test-only)."""
    import llmi

    path = str(tmp_path / "t.gguf")
    llmi.write_synthetic_gguf(path, "tiny-mixed", seed=1)
    with pytest.raises(llmi.LlmiError, match="n_gpu_layers=0"):
        llmi.Model(path, n_gpu_layers=0)
