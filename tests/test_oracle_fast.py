"""The CPU baseline's AVX2 dot products (oracle/ggml_oracle.c or_set_fast_dots — bench.py
cpu_baseline timing only, never a parity reference) compute the same dot products as the
generic-order restatement up to fp32 association: relative agreement ~1e-5, not bit
equality.  Also: the switch is off by default and a no-AVX2 build reports it."""
import ctypes as C

import numpy as np
import pytest

import pyoracle as po
from helpers import Q4_K, Q5_K, Q6_K, Q8_0, random_blocks


@pytest.fixture(scope="module")
def simd():
    """The AVX2 build loaded on its own (other tests may already hold the generic build
    as pyoracle's library): or_matvec + or_set_fast_dots of libggml_oracle_simd.so."""
    import os
    if not os.path.exists(po.LIB_SIMD):
        po.build()
    L = C.CDLL(po.LIB_SIMD)
    L.or_matvec.restype = C.c_int
    L.or_matvec.argtypes = [C.c_int, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int]
    L.or_set_fast_dots.restype = C.c_int
    L.or_set_fast_dots.argtypes = [C.c_int]
    yield L
    L.or_set_fast_dots(0)


@pytest.mark.parametrize("mode", [1, 2], ids=["avx2", "avx512bw"])
@pytest.mark.parametrize("qt", [Q4_K, Q5_K, Q6_K, Q8_0])
def test_fast_dots_match_generic(simd, qt, mode):
    got = simd.or_set_fast_dots(mode)
    simd.or_set_fast_dots(0)
    if not got:
        pytest.skip("oracle build without AVX2")
    if got != mode:
        pytest.skip("host without AVX-512BW")
    rng = np.random.default_rng(qt)
    rows, cols = 64, 4096 + (32 if qt == Q8_0 else 0)  # Q8_0: an odd block count (the 2-block loop's tail)
    w = random_blocks(qt, rows, cols, rng)
    x = rng.standard_normal(cols).astype(np.float32)
    y0 = np.empty(rows, np.float32)
    y1 = np.empty(rows, np.float32)
    P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    assert simd.or_matvec(qt, P(w), rows, cols, P(x), P(y0), 4) == 0
    assert simd.or_set_fast_dots(mode) == mode
    try:
        assert simd.or_matvec(qt, P(w), rows, cols, P(x), P(y1), 4) == 0
    finally:
        simd.or_set_fast_dots(0)
    scale = np.abs(y0).max()
    assert np.abs(y1 - y0).max() <= 1e-5 * scale + 1e-6, (np.abs(y1 - y0).max(), scale)
    # off again: bit-identical to the generic order
    assert simd.or_matvec(qt, P(w), rows, cols, P(x), P(y1), 4) == 0
    assert np.array_equal(y0, y1)


def test_localized_weights_decode_identically(tmp_path):
    """or_model_localize (the CPU baseline's NUMA placement: decode matrices copied into
    rows first-touched by their reading thread) moves bytes only: logits bit-identical."""
    import llmi

    p = str(tmp_path / "t.gguf")
    llmi.write_synthetic_gguf(p, "tiny-mixed", seed=5)
    a = po.OracleModel(p, n_ctx=64, threads=3)
    b = po.OracleModel(p, n_ctx=64, threads=3)
    assert b.localize() > 0 and b.localize() == 0  # once
    for pos, t in enumerate([1, 7, 42, 300, 5]):
        assert np.array_equal(a.decode(t, pos), b.decode(t, pos))
    a.close(), b.close()
