"""Batched MFMA prefill (prefill.hip.inc) through the C ABI.

The prompt's leading tokens run through every layer as one launch per op over all of
them: q8 activations x quantized weights on v_mfma_f32_16x16x32_f16 (exact integer sums
per residue class), combined in fp32 exactly as the matvec does, in ggml's generic
order.  The bar is therefore BIT-IDENTITY with T decode steps, which are
themselves bit-identical to the oracle's generic order (test_gpu_decode.py):
- last-token logits of a batched prompt == the oracle's (generic order), bit for bit;
- the KV cache the prefill wrote: greedy continuation identical, logits bit-identical;
- prefill vs decode-step prompt processing (LLMI_NO_PREFILL=1) bit-identical at the
  real widths (8B / TinyLlama / Mistral / 70B, 2 layers), across the 512-token ubatch
  boundary and at a ragged (non-multiple-of-32) prompt length.
"""
from __future__ import annotations

import numpy as np
import pytest

import llmi
import pyoracle as po

pytestmark = pytest.mark.gpu


def _oracle_prompt_logits(path, prompt, n_ctx, n_gen):
    """Oracle (ggml's generic order): logits after the prompt and greedy continuation logits."""
    om = po.OracleModel(path, n_ctx=n_ctx)
    out = []
    lo = None
    for pos, t in enumerate(prompt):
        lo = om.decode(t, pos)
    out.append(lo)
    pos = len(prompt)
    for _ in range(n_gen):
        t = int(np.argmax(lo))
        lo = om.decode(t, pos)
        out.append(lo)
        pos += 1
    return out


def _gpu_prompt_logits(path, prompt, n_ctx, n_gen, monkeypatch=None, no_prefill=False):
    if monkeypatch is not None:
        if no_prefill:
            monkeypatch.setenv("LLMI_NO_PREFILL", "1")
        else:
            monkeypatch.delenv("LLMI_NO_PREFILL", raising=False)
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=n_ctx)
    assert c.decode(prompt) == 0
    out = [c.logits(-1)]
    pos = len(prompt)
    for _ in range(n_gen):
        t = c.greedy(-1)
        assert t == int(np.argmax(out[-1]))
        assert c.decode([t], pos=[pos]) == 0
        out.append(c.logits(-1))
        pos += 1
    return m, out


# (tiny-mixed-d128, 37/70) are the prompts on which a compiler-fused f32->f16 rounding
# (v_fma_mixlo_f16) once made the decode path leave the oracle.
PAST_DIVERGENCE_CASES = {("tiny-mixed-d128", 37), ("tiny-mixed-d128", 70)}


@pytest.mark.parametrize("preset,n_prompt", [("tiny-mixed", 2), ("tiny-mixed", 37), ("tiny-mixed", 70),
                                             ("tiny-mixed-d128", 2), ("tiny-mixed-d128", 20),
                                             ("tiny-mixed-d128", 37),
                                             ("tiny-mixed-d128", 70)])
def test_prefill_vs_oracle_tiny(gpu, tiny_models, monkeypatch, preset, n_prompt):
    """Every quant type (Q4_K/Q5_K/Q6_K/Q8_0, gate/up of different types), head_dim 64
    and 128, GQA 2: prompt logits and 6 continuation steps bit-identical to the oracle."""
    path = tiny_models[preset]
    rng = np.random.default_rng(11 + n_prompt)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, n_prompt - 1)]
    m, got = _gpu_prompt_logits(path, prompt, 128, 6, monkeypatch)
    assert m.prefill_supported
    want = _oracle_prompt_logits(path, prompt, 128, 6)
    for k, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, w), f"step {k}: max |d| {np.abs(g - w).max():.3g}"


@pytest.mark.parametrize("preset,n_prompt", sorted(PAST_DIVERGENCE_CASES))
def test_prefill_vs_steps_at_known_divergence(gpu, tiny_models, monkeypatch, preset, n_prompt):
    path = tiny_models[preset]
    rng = np.random.default_rng(11 + n_prompt)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, n_prompt - 1)]
    _, a = _gpu_prompt_logits(path, prompt, 128, 6, monkeypatch, no_prefill=False)
    _, b = _gpu_prompt_logits(path, prompt, 128, 6, monkeypatch, no_prefill=True)
    for k, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), f"step {k}: max |d| {np.abs(x - y).max():.3g}"


@pytest.mark.parametrize("preset,n_vocab,n_prompt", [("llama3-8b-q4km", 0, 131), ("tinyllama-q8_0", 0, 96),
                                                     ("mistral7b-q5km", 0, 64), ("mistral7b-q6k", 0, 33),
                                                     ("llama3-70b-q4km", 32000, 40)])
def test_prefill_vs_steps_real_widths(gpu, synth_dir, monkeypatch, preset, n_vocab, n_prompt):
    """Exact model widths (2 layers): the batched prefill equals decode-step prompt
    processing bit for bit (prompt logits and 4 continuation steps)."""
    path = str(synth_dir / f"{preset}-L2.gguf")
    llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=2, n_vocab=n_vocab)
    rng = np.random.default_rng(4)
    prompt = [1] + [int(t) for t in rng.integers(3, 30000, n_prompt - 1)]
    m, a = _gpu_prompt_logits(path, prompt, 256, 4, monkeypatch, no_prefill=False)
    assert m.prefill_supported
    _, b = _gpu_prompt_logits(path, prompt, 256, 4, monkeypatch, no_prefill=True)
    for k, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), f"step {k}: max |d| {np.abs(x - y).max():.3g}"


def test_prefill_ubatch_boundary(gpu, tiny_models, monkeypatch):
    """A 600-token prompt spans two 512-token ubatches (the second attends to the
    first's KV rows): bit-identical to decode steps, with the one-head-per-workgroup
    prefill attention (test option pf_attn_simple) against the split decode path (mode
    2).  The grouped prefill attention and every decode path are covered at the same
    lengths by test_long_context_vs_oracle / test_attention_variants_agree_long_context
    (the former disagreement was the compiler-fused f16 rounding)."""
    path = tiny_models["tiny-mixed-d128"]
    rng = np.random.default_rng(9)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 599)]
    monkeypatch.setenv("LLMI_ATTN_MODE", "2")
    llmi.test_option("pf_attn_simple", 1)
    try:
        _, a = _gpu_prompt_logits(path, prompt, 768, 3, monkeypatch, no_prefill=False)
    finally:
        llmi.test_option("pf_attn_simple", 0)
    _, b = _gpu_prompt_logits(path, prompt, 768, 3, monkeypatch, no_prefill=True)
    monkeypatch.setenv("LLMI_ATTN_MODE", "0")
    for k, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), f"step {k}: max |d| {np.abs(x - y).max():.3g}"


@pytest.mark.parametrize("preset,n_prompt", [("tiny-mixed", 400), ("tiny-mixed-d128", 300)])
@pytest.mark.parametrize("no_prefill", [False, True])
def test_long_context_vs_oracle(gpu, tiny_models, monkeypatch, preset, n_prompt, no_prefill):
    """Hundreds of positions: the prompt (batched prefill, or one decode step per token)
    and 4 continuation steps bit-identical to the oracle (generic order)."""
    path = tiny_models[preset]
    rng = np.random.default_rng(5 + n_prompt)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, n_prompt - 1)]
    _, got = _gpu_prompt_logits(path, prompt, 512, 4, monkeypatch, no_prefill=no_prefill)
    want = _oracle_prompt_logits(path, prompt, 512, 4)
    for k, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, w), f"step {k}: max |d| {np.abs(g - w).max():.3g}"


def test_attention_variants_agree_long_context(gpu, tiny_models, monkeypatch):
    path = tiny_models["tiny-mixed"]
    rng = np.random.default_rng(9)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 499)]
    res = []
    for mode in ("2", "4", "6", "7"):
        monkeypatch.setenv("LLMI_ATTN_MODE", mode)
        _, a = _gpu_prompt_logits(path, prompt, 768, 0, monkeypatch, no_prefill=True)
        res.append(a[0])
    monkeypatch.setenv("LLMI_ATTN_MODE", "0")
    assert np.array_equal(res[0], res[1])
    assert np.array_equal(res[0], res[2])
    assert np.array_equal(res[0], res[3])


def test_prefill_continues_after_past(gpu, tiny_models, monkeypatch):
    """A second multi-token batch at n_past > 0 (chat turn) prefills from the existing
    cache: equal to decode steps."""
    path = tiny_models["tiny-mixed"]
    res = []
    for no_pf in (False, True):
        if no_pf:
            monkeypatch.setenv("LLMI_NO_PREFILL", "1")
        else:
            monkeypatch.delenv("LLMI_NO_PREFILL", raising=False)
        m = llmi.Model(path)
        c = llmi.Context(m, n_ctx=256)
        assert c.decode([1, 5, 9, 33, 400]) == 0
        assert c.decode([7, 8, 9, 10, 11, 12, 13, 14, 15]) == 0
        res.append(c.logits(-1))
    assert np.array_equal(res[0], res[1])


# ---- kernel level: the prefill GEMM against per-token matvecs (bit-exact) ----------
from helpers import Q4_K, Q5_K, Q6_K, Q8_0, empty_dev, random_blocks, to_dev  # noqa: E402


def _p(t):
    import ctypes as C

    return C.c_void_p(t.data_ptr())


def _weights(qtype, rows, cols, rng):
    import torch
    from llmi._lib import lib

    L = lib()
    raw = random_blocks(qtype, rows, cols, rng)
    wd = empty_dev(L.llmi_device_layout_bytes(qtype, rows, cols))
    rd = to_dev(raw)
    torch.cuda.synchronize()
    assert L.llmi_repack(qtype, _p(rd), _p(wd), rows, cols) == 0
    return wd


@pytest.mark.parametrize("qtype", [Q4_K, Q5_K, Q6_K, Q8_0])
@pytest.mark.parametrize("rows,cols", [(32, 256), (96, 512), (128, 768), (160, 4096), (64, 14336)])
@pytest.mark.parametrize("n_tok", [1, 5, 33, 70])
@pytest.mark.parametrize("norm", [False, True])
@pytest.mark.parametrize("ng", [2, 1])
def test_pf_gemm_equals_matvec(gpu, qtype, rows, cols, n_tok, norm, ng):
    """k_pf_gemm (64-token workgroups, NG = 2, above 32 tokens; 32-token ones forced by
    the pf_gemm_ng option) against n_tok matvec launches, bit for bit."""
    import torch
    from llmi._lib import lib

    L = lib()
    if ng == 1 and (n_tok < 33 or cols > 768):
        pytest.skip("the 32-token workgroup variant is exercised on the ragged multi-group sizes")
    old = L.llmi_test_option(b"pf_gemm_ng", ng)
    try:
        _pf_gemm_case(L, qtype, rows, cols, n_tok, norm)
    finally:
        L.llmi_test_option(b"pf_gemm_ng", old)


def _pf_gemm_case(L, qtype, rows, cols, n_tok, norm):
    import torch

    rng = np.random.default_rng(rows + cols + n_tok + qtype)
    wd = _weights(qtype, rows, cols, rng)
    x = rng.standard_normal((n_tok, cols)).astype(np.float32)
    nw = rng.uniform(0.5, 1.5, cols).astype(np.float32) if norm else None
    xd = to_dev(x)
    nd = to_dev(nw) if norm else None
    y = torch.full((n_tok, rows), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    assert L.llmi_pf_gemm(qtype, _p(wd), rows, cols, _p(xd), _p(nd) if norm else None, 1e-5, n_tok, _p(y), None) == 0
    got = y.cpu().numpy()
    for t in range(n_tok):
        yt = torch.zeros(rows, dtype=torch.float32, device="cuda")
        xt = to_dev(x[t])
        torch.cuda.synchronize()
        assert L.llmi_matvec(qtype, _p(wd), rows, cols, _p(xt), _p(nd) if norm else None, 1e-5, _p(yt), 0) == 0
        want = yt.cpu().numpy()
        assert np.array_equal(got[t], want), f"token {t}: max |d| {np.abs(got[t] - want).max():.3g}"
