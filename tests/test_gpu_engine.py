"""The layer engine (leng.hip: one persistent launch per layer for attn_output, ffn_gate+up,
ffn_down and the next layer's QKV, weights streamed into an LDS ring ahead of in-launch
hand-offs) against the CPU oracle and against the separate launches it replaces.

The bar is the decode step's: logits BIT-IDENTICAL to the oracle at every step, greedy
ids identical (the engine runs k_matvec's unit-term / fold / epilogue code on the same
rows; only the weights' path into registers and the edges between the matvecs differ).
"""
from __future__ import annotations

import numpy as np
import pytest

import llmi
from test_gpu_decode import run_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def engine_on():
    """Every test here runs with the layer engine on (contexts made inside the test)."""
    old = llmi.test_option("engine", 1)
    yield
    llmi.test_option("engine", old)


def engine_launches(c: llmi.Context, first: int, pos: int) -> int:
    prof = c.profile_kernels(first, pos, 1)
    return prof["layer"]["launches_per_step"]


@pytest.mark.parametrize("preset,n_layer,n_vocab", [("llama3-8b-q4km", 3, 0), ("tinyllama-q8_0", 3, 0),
                                                    ("mistral7b-q5km", 2, 0), ("mistral7b-q6k", 2, 0),
                                                    ("llama3-70b-q4km", 2, 32000)])
def test_engine_parity_real_widths(gpu, synth_dir, preset, n_layer, n_vocab):
    """Every layer of these shapes runs in the engine (profile: one 'layer' launch per
    layer) and every step's logits equal the oracle's bit for bit."""
    path = str(synth_dir / f"{preset}-L{n_layer}e.gguf")
    llmi.write_synthetic_gguf(path, preset, seed=5, n_layer=n_layer, n_vocab=n_vocab)
    prompt = [1, 100, 2000, 31000, 7, 9]
    worst, g, o, margins, m, c = run_parity(path, prompt, 6, n_ctx=64, exact=True)
    assert g == o
    assert engine_launches(c, g[-1], len(prompt) + 5) == n_layer


@pytest.mark.parametrize("preset", ["llama3-8b-q4km", "tinyllama-q8_0"])
def test_engine_equals_separate_launches(gpu, synth_dir, preset):
    """64 greedy tokens from a 32-token prompt: engine on and off give the same tokens and
    the same final logits (x86 numerics too, where the engine takes K-quant layers)."""
    path = str(synth_dir / f"{preset}-L2eq.gguf")
    llmi.write_synthetic_gguf(path, preset, seed=7, n_layer=2)
    rng = np.random.default_rng(3)
    prompt = [1] + [int(t) for t in rng.integers(3, 30000, 31)]
    outs = {}
    for num in (llmi.NUMERICS_GENERIC, llmi.NUMERICS_X86):
        for on in (1, 0):
            old = llmi.test_option("engine", on)
            try:
                m = llmi.Model(path, numerics=num)
                c = llmi.Context(m, n_ctx=256)
                assert c.decode(prompt) == 0
                first = c.greedy(-1)
                toks = c.generate_greedy(first, len(prompt), 64)
                assert c.decode([toks[-1]], pos=[len(prompt) + 64]) == 0
                outs[(num, on)] = (toks, c.logits(-1).copy())
                c.close()
                m.close()
            finally:
                llmi.test_option("engine", old)
        a, b = outs[(num, 1)], outs[(num, 0)]
        assert a[0] == b[0], f"numerics {num}: engine tokens differ from separate launches"
        assert np.array_equal(a[1], b[1]), f"numerics {num}: engine logits differ"


def test_engine_bounded_wait_fault_is_reported(gpu, synth_dir):
    """A hand-off that cannot complete in its poll budget (le_spin = 1) ends the step with
    an error (fault word), never a hang; with the budget restored the context decodes
    again and matches a fresh context."""
    path = str(synth_dir / "llama3-8b-q4km-L2f.gguf")
    llmi.write_synthetic_gguf(path, "llama3-8b-q4km", seed=9, n_layer=2)
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=64, use_graphs=False)
    old = llmi.test_option("le_spin", 1)
    try:
        with pytest.raises(llmi.LlmiError, match="bounded wait"):
            for p in range(4):
                if c.decode([1 + p], pos=[p]) != 0:
                    raise llmi.LlmiError(llmi.last_error())
    finally:
        llmi.test_option("le_spin", old)
    c.kv_clear()
    assert c.decode([1, 2, 3]) == 0
    ref = llmi.Context(m, n_ctx=64)
    assert ref.decode([1, 2, 3]) == 0
    assert np.array_equal(c.logits(-1), ref.logits(-1))
