"""The oracle's fast paths are the same function as its reference paths, bit for bit.

- libggml_oracle_simd.so (-O3 -march=x86-64-v3) == libggml_oracle.so (-O2): whole-model
  logits on a tiny mixed-type model (run in subprocesses: the library is chosen when
  pyoracle is imported).
- or_prefill (rows unpacked once, vd_generic_unpacked) leaves the same state as T
  or_decode steps (or_vec_dot per row and token).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as po
from helpers import QTYPES, random_blocks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1] + "/oracle", sys.argv[1] + "/llama-gguf-inference_amd"]
import pyoracle as po
om = po.OracleModel(sys.argv[2], n_ctx=64, threads=4)
out = [om.decode(t, p) for p, t in enumerate([1, 42, 7, 300, 5, 99])]
np.save(sys.argv[4], np.stack(out))
"""


def test_simd_build_bit_identical(tmp_path):
    import llmi

    path = str(tmp_path / "tiny.gguf")
    llmi.write_synthetic_gguf(path, "tiny-mixed-d128", seed=1)
    res = []
    for which in ("generic", "simd"):
        out = str(tmp_path / f"{which}.npy")
        env = dict(os.environ, LLMI_ORACLE=which)
        subprocess.run([sys.executable, "-c", _SCRIPT, ROOT, path, "0", out], check=True, env=env, timeout=300)
        res.append(np.load(out))
    assert np.array_equal(res[0], res[1])


@pytest.mark.parametrize("preset", ["tiny-mixed", "tiny-mixed-d128"])
def test_oracle_prefill_equals_decode_steps(tmp_path, preset):
    """or_prefill (loops reordered, weight rows unpacked once) leaves the same KV cache
    and state as T or_decode steps: the next step's logits are bit-identical."""
    import llmi

    path = str(tmp_path / f"{preset}.gguf")
    llmi.write_synthetic_gguf(path, preset, seed=1)
    rng = np.random.default_rng(3)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 70)]
    a = po.OracleModel(path, n_ctx=128, threads=4)
    for p, t in enumerate(prompt):
        a.decode(t, p, logits=False)
    la = a.decode(5, len(prompt))
    b = po.OracleModel(path, n_ctx=128, threads=4)
    b.prefill(prompt[:40])
    b.prefill(prompt[40:], pos0=40)
    lb = b.decode(5, len(prompt))
    assert np.array_equal(la, lb)
    assert np.array_equal(a.tap(3)[:64], b.tap(3)[:64])
