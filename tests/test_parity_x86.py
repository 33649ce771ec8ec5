"""The oracle's x86 association mode (oracle/ggml_oracle.c): the
MEASUREMENT of the GPU's distance from the reference's NGL=0 numerics, never a check of
the product.  The GPU is bit-identical to the generic order (tests/test_gpu_long.py), so
generic-vs-x86 on the oracle is the GPU-vs-NGL=0 distance; tools/parity_x86.py runs it
at the configs' widths into profiles/r04/parity_x86.jsonl.  Here, at small sizes:

- the recalled ggml_v_expf polynomial is a faithful exp (<= 2 ulp over the softmax and
  SiLU domains; a misremembered constant would be off by thousands of ulp);
- the lane-emulated x86 dots (portable C) equal the AVX2-intrinsic timing dots bit for
  bit where the build has AVX2 -- two independent writings of the same association;
- x86 and generic dots agree to fp32 rounding (relative 1e-5), and are not bit-identical;
- the report tool's trajectory runs and mode 0 against mode 0 is exactly 0.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np
import pytest

import pyoracle as po
from helpers import Q4_K, Q5_K, Q6_K, Q8_0, random_blocks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture
def lib():
    L = po.lib()
    yield L
    L.or_set_x86_mode(0)


def test_v_expf_is_a_faithful_exp(lib):
    xs = np.concatenate([np.linspace(-87.0, 0.0, 60001), np.linspace(0.0, 80.0, 20001)]).astype(np.float32)
    lib.or_set_x86_mode(po.X86_VEXP)
    got = np.array([lib.or_expf(float(x)) for x in xs], dtype=np.float64)
    ref = np.exp(xs.astype(np.float64))
    ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert (np.abs(got - ref) / ulp).max() <= 2.0


@pytest.mark.parametrize("qt", [Q4_K, Q5_K, Q6_K, Q8_0])
def test_x86_dots_match_generic_to_rounding(lib, qt):
    rng = np.random.default_rng(100 + qt)
    rows, cols = 96, 4096
    w = random_blocks(qt, rows, cols, rng)
    x = rng.standard_normal(cols).astype(np.float32)
    y0 = po.matvec(qt, w, rows, cols, x, threads=2)
    lib.or_set_x86_mode(po.X86_DOTS)
    y1 = po.matvec(qt, w, rows, cols, x, threads=2)
    lib.or_set_x86_mode(0)
    scale = np.abs(y0).max()
    assert np.abs(y1 - y0).max() <= 1e-5 * scale
    assert not np.array_equal(y0, y1), "x86 association should not coincide with the generic order"


@pytest.mark.parametrize("qt", [Q4_K, Q5_K, Q6_K, Q8_0])
def test_lane_emulation_equals_avx2_intrinsics(qt):
    """libggml_oracle_simd.so: or_set_fast_dots (AVX2 intrinsics) == x86 mode (scalar lanes)."""
    if not os.path.exists(po.LIB_SIMD):
        po.build()
    L = C.CDLL(po.LIB_SIMD)
    L.or_matvec.restype = C.c_int
    L.or_matvec.argtypes = [C.c_int, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int]
    L.or_set_fast_dots.restype = C.c_int
    L.or_set_fast_dots.argtypes = [C.c_int]
    L.or_set_x86_mode.restype = C.c_int
    L.or_set_x86_mode.argtypes = [C.c_int]
    if not L.or_set_fast_dots(1):
        pytest.skip("oracle build without AVX2")
    rng = np.random.default_rng(7 + qt)
    rows, cols = 64, 4096
    w = np.ascontiguousarray(random_blocks(qt, rows, cols, rng))
    x = rng.standard_normal(cols).astype(np.float32)
    ya = np.empty(rows, np.float32)
    yb = np.empty(rows, np.float32)
    P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    try:
        assert L.or_matvec(qt, P(w), rows, cols, P(x), P(ya), 2) == 0
        L.or_set_fast_dots(0)
        L.or_set_x86_mode(po.X86_DOTS | po.X86_Q80)
        assert L.or_matvec(qt, P(w), rows, cols, P(x), P(yb), 2) == 0
    finally:
        L.or_set_fast_dots(0)
        L.or_set_x86_mode(0)
    if qt == Q8_0:  # the timing dots quantize with the generic q8_0 (ref) routine
        L.or_set_fast_dots(1)
        L.or_set_x86_mode(po.X86_Q80)
        try:
            assert L.or_matvec(qt, P(w), rows, cols, P(x), P(ya), 2) == 0
        finally:
            L.or_set_fast_dots(0)
            L.or_set_x86_mode(0)
    assert np.array_equal(ya, yb)


def test_report_tool_runs(tmp_path, lib):
    import parity_x86 as px

    path = os.path.join(ROOT, "tests", "golden", "tiny-mixed.gguf")
    same = px.run(path, n_prompt=4, n_gen=3, flags=0, threads=2, n_vocab_prompt=200)
    assert same["worst_abs_diff"] == 0.0 and same["frac_within_1e-3"] == 1.0
    assert same["first_id_divergence"] is None
    rep = px.run(path, n_prompt=4, n_gen=3, flags=po.X86_ALL, threads=2, n_vocab_prompt=200)
    for k in ("steps", "frac_within_1e-3", "worst_abs_diff", "median_abs_diff", "first_id_divergence",
              "id_mismatch_steps"):
        assert k in rep
    assert rep["steps"] == 4 and rep["worst_abs_diff"] > 0.0
