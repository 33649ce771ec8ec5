"""CPU checks against the committed fixtures of tests/golden/ (make_golden.py).

- closed-form single blocks: the oracle's dequantization of hand-built Q4_K/Q5_K/Q6_K/
  Q8_0 blocks equals the values written down from the block format (Appendix A of
  SURVEY.md; upstream dequantize_row_*), bit for bit;
- the synthetic GGUF writer reproduces the committed tiny-mixed.gguf byte for byte;
- the oracle reproduces the committed 16-step greedy run (full logits) bit for bit.
The oracle's agreement with llama.cpp itself is unpinned (no llama.cpp source, binary
or fixture exists in the reference); see DESIGN.md §Oracle."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

import pyoracle as po

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TYPES = {"q4_K": 12, "q5_K": 13, "q6_K": 14, "q8_0": 8}


@pytest.mark.parametrize("name", sorted(TYPES))
def test_closed_form_blocks(name):
    z = np.load(os.path.join(HERE, "blocks.npz"))
    blk, y = z[f"{name}_block"], z[f"{name}_y"]
    n = 32 if name == "q8_0" else 256
    got = po.dequantize(TYPES[name], blk, n)
    assert np.array_equal(got, y), f"{name}: max |d| {np.abs(got - y).max()}"


def test_writer_reproduces_fixture(tmp_path):
    import llmi

    p = str(tmp_path / "t.gguf")
    llmi.write_synthetic_gguf(p, "tiny-mixed", seed=1)
    a = hashlib.sha256(open(p, "rb").read()).hexdigest()
    b = hashlib.sha256(open(os.path.join(HERE, "tiny-mixed.gguf"), "rb").read()).hexdigest()
    assert a == b


def test_oracle_reproduces_greedy16():
    z = np.load(os.path.join(HERE, "greedy16.npz"))
    prompt = [int(t) for t in z["prompt"]]
    want_lg, want_ids = z["logits"], z["ids"]
    om = po.OracleModel(os.path.join(HERE, "tiny-mixed.gguf"), n_ctx=64, threads=2)
    cur, pos, ids = prompt[0], 0, []
    for step in range(want_lg.shape[0]):
        lg = om.decode(cur, pos)
        assert np.array_equal(lg, want_lg[step]), f"step {step}: max |d| {np.abs(lg - want_lg[step]).max()}"
        pos += 1
        if pos < len(prompt):
            cur = prompt[pos]
        else:
            cur = int(np.argmax(lg))
            ids.append(cur)
    om.close()
    assert ids == [int(i) for i in want_ids]
