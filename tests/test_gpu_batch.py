"""Continuous batching (batch.hip): up to 8 sequences of one
context advance together, each batched step streaming every weight byte once for all
of them.  The bar is the same as for single-sequence decode: every sequence's logits and
greedy tokens are BIT-IDENTICAL to decoding that sequence alone (which in turn is
bit-identical to the generic-order oracle, tests/test_gpu_decode.py) — the batched
matvec forms each token's integer dots and fp32 reductions in the single-token order.

Covered: slot counts 1..8 (3, 5, 6, 7 run padded to 4 / 8 with a dummy sequence),
sequences at different positions (different KV lengths and RoPE angles in one step),
a step whose sequences straddle a 256-position KV bucket, llama_decode batches with
several seq_ids (single-token sequences batched, longer ones prefilled), sequence
removal and reuse, and the real widths (Llama-3-8B Q4_K_M, Mistral Q5_K_M / Q6_K,
TinyLlama Q8_0, Llama-3-70B Q4_K_M shapes at 2 layers; 70B's 28672-column ffn_down runs
as two 4-token launches, its LDS images of 8 tokens exceeding 160 KB).
"""
from __future__ import annotations

import numpy as np
import pytest

import llmi

pytestmark = pytest.mark.gpu


def _prompts(rng, k, lo=3, hi=700, min_len=2, max_len=40):
    return [[1] + [int(t) for t in rng.integers(lo, hi, int(rng.integers(min_len, max_len)))] for _ in range(k)]


def _single_reference(path, prompts, n_gen, n_ctx):
    """Each prompt alone: prefill + greedy on a one-sequence context."""
    m = llmi.Model(path)
    outs, logits = [], []
    for p in prompts:
        c = llmi.Context(m, n_ctx=n_ctx)
        assert c.decode(p) == 0
        logits.append(c.logits(-1))
        first = c.greedy(-1)
        outs.append([first] + c.generate_greedy(first, len(p), n_gen))
        c.close()
    return outs, logits


def _batched(path, prompts, n_gen, n_ctx, n_seq=8):
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=n_ctx, n_seq=n_seq)
    logits, firsts = [], []
    for s, p in enumerate(prompts):
        assert c.decode(p, seq=[s] * len(p)) == 0
        logits.append(c.logits(-1))
        firsts.append(c.greedy(-1))
    seqs = list(range(len(prompts)))
    gen = c.generate_greedy_batch(seqs, firsts, [len(p) for p in prompts], n_gen)
    return [[f] + g for f, g in zip(firsts, gen)], logits, c


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
def test_batched_greedy_matches_single(gpu, tiny_models, k):
    path = tiny_models["tiny-mixed-d128"]
    rng = np.random.default_rng(100 + k)
    prompts = _prompts(rng, k)
    want, want_lg = _single_reference(path, prompts, 20, 512)
    got, got_lg, _ = _batched(path, prompts, 20, 512)
    for s in range(k):
        assert np.array_equal(got_lg[s], want_lg[s]), f"seq {s}: prompt logits differ"
        assert got[s] == want[s], f"seq {s}: batched {got[s]} single {want[s]}"


def test_batched_straddles_kv_bucket(gpu, tiny_models):
    """Sequences at positions 250 and 10 in one step, stepping across position 256."""
    path = tiny_models["tiny-mixed-d128"]
    rng = np.random.default_rng(7)
    prompts = [[1] + [int(t) for t in rng.integers(3, 700, 249)], [1] + [int(t) for t in rng.integers(3, 700, 9)]]
    want, _ = _single_reference(path, prompts, 16, 512)
    got, _, _ = _batched(path, prompts, 16, 512)
    assert got == want


def test_llama_decode_multi_seq_batch(gpu, tiny_models):
    """One llama_decode batch holding a 1-token entry of 3 sequences (a batched step) and a
    12-token prompt of a 4th (prefill): logits of every entry equal the single-sequence ones."""
    path = tiny_models["tiny-mixed-d128"]
    rng = np.random.default_rng(21)
    pre = _prompts(rng, 3, min_len=4, max_len=20)
    tail = [int(t) for t in rng.integers(3, 700, 3)]
    fresh = [1] + [int(t) for t in rng.integers(3, 700, 11)]
    m = llmi.Model(path)
    ref = []
    for p, t in zip(pre, tail):
        c1 = llmi.Context(m, n_ctx=256)
        assert c1.decode(p + [t]) == 0
        ref.append(c1.logits(-1))
        c1.close()
    c1 = llmi.Context(m, n_ctx=256)
    assert c1.decode(fresh) == 0
    ref.append(c1.logits(-1))
    c1.close()

    c = llmi.Context(m, n_ctx=256, n_seq=4)
    for s, p in enumerate(pre):
        assert c.decode(p, seq=[s] * len(p)) == 0
    toks = tail + fresh
    seq = [0, 1, 2] + [3] * len(fresh)
    pos = [len(p) for p in pre] + list(range(len(fresh)))
    import ctypes as C

    n = len(toks)
    b = llmi.lib().llama_batch_init(n, 0, 1)
    try:
        b.n_tokens = n  # upstream llama_batch_init leaves n_tokens = 0 for the caller to set
        for i in range(n):
            b.token[i] = toks[i]
            b.pos[i] = pos[i]
            b.n_seq_id[i] = 1
            b.seq_id[i][0] = seq[i]
            b.logits[i] = 1 if i < 3 or i == n - 1 else 0
        assert llmi.lib().llama_decode(c._h, b) == 0, llmi.last_error()
    finally:
        llmi.lib().llama_batch_free(b)
    for i, r in zip([0, 1, 2, n - 1], ref):
        assert np.array_equal(c.logits(i), r), f"batch entry {i}"
    for s in range(4):
        assert c.seq_pos_max(s) == (len(pre[s]) if s < 3 else len(fresh) - 1)
    del C


def test_seq_rm_and_reuse(gpu, tiny_models):
    """Releasing a sequence (llama_kv_self_seq_rm) and decoding a new prompt in it gives the
    fresh-context result; truncation to p0 re-decodes from there identically."""
    path = tiny_models["tiny-mixed-d128"]
    rng = np.random.default_rng(5)
    a, b2 = _prompts(rng, 2, min_len=10, max_len=30)
    want, want_lg = _single_reference(path, [b2], 8, 256)
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=256, n_seq=2)
    assert c.decode(a, seq=[1] * len(a)) == 0
    assert c.seq_rm(1)
    assert c.seq_pos_max(1) == -1
    assert c.decode(b2, seq=[1] * len(b2)) == 0
    assert np.array_equal(c.logits(-1), want_lg[0])
    # truncate to 5 positions, re-decode the rest
    assert c.seq_rm(1, 5, -1)
    assert c.seq_pos_max(1) == 4
    assert c.decode(b2[5:], seq=[1] * (len(b2) - 5)) == 0
    assert np.array_equal(c.logits(-1), want_lg[0])
    assert not c.seq_rm(1, 2, 4), "interior removal is not supported and must say so"


def test_mixed_gate_up_types_fall_back(gpu, tiny_models):
    """tiny-mixed's layer 0 has ffn_gate Q6_K and ffn_up Q4_K: no batched step; llama_decode
    runs those sequences one at a time (same results), the batch API reports the error."""
    path = tiny_models["tiny-mixed"]
    rng = np.random.default_rng(9)
    prompts = _prompts(rng, 2)
    want, want_lg = _single_reference(path, prompts, 2, 256)
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=256, n_seq=2)
    for s, p in enumerate(prompts):
        assert c.decode(p, seq=[s] * len(p)) == 0
    t = [want[0][0], want[1][0]]
    assert c.decode(t, pos=[len(prompts[0]), len(prompts[1])], seq=[0, 1], logits_all=True) == 0
    assert c.greedy(0) == want[0][1] and c.greedy(1) == want[1][1]
    with pytest.raises(llmi.LlmiError):
        c.generate_greedy_batch([0, 1], t, [len(prompts[0]), len(prompts[1])], 2)


@pytest.mark.parametrize("preset,n_vocab", [("llama3-8b-q4km", 0), ("mistral7b-q5km", 0), ("mistral7b-q6k", 0),
                                            ("tinyllama-q8_0", 0), ("llama3-70b-q4km", 32000)])
def test_batched_real_widths(gpu, synth_dir, preset, n_vocab):
    path = str(synth_dir / f"{preset}-batch-L2.gguf")
    llmi.write_synthetic_gguf(path, preset, seed=11, n_layer=2, n_vocab=n_vocab)
    rng = np.random.default_rng(3)
    prompts = _prompts(rng, 8, hi=30000, max_len=24)
    want, want_lg = _single_reference(path, prompts, 12, 256)
    got, got_lg, _ = _batched(path, prompts, 12, 256)
    for s in range(8):
        assert np.array_equal(got_lg[s], want_lg[s]), f"seq {s}: prompt logits differ"
        assert got[s] == want[s], f"seq {s}"


@pytest.mark.parametrize("preset,k", [("llama3-8b-q4km", 2), ("llama3-8b-q4km", 5), ("mistral7b-q5km", 3),
                                       ("mistral7b-q6k", 8)])
@pytest.mark.parametrize("dma", ["1", "0"])  # k_bmd (weights staged through LDS by DMA) / k_bmm
def test_bmm_any_batch_size(gpu, synth_dir, monkeypatch, preset, k, dma):
    """The matrix-core batched matvec (batch.hip k_bmd, and k_bmm with LLMI_BMM_DMA=0) forced
    for every batch size (LLMI_BMM_MIN=1; by default it takes steps of 3 or more tokens): each
    sequence's tokens and logits equal its single-sequence decode at real widths, Q4_K / Q5_K /
    Q6_K."""
    monkeypatch.setenv("LLMI_BMM_MIN", "1")
    monkeypatch.setenv("LLMI_BMM_DMA", dma)
    path = str(synth_dir / f"{preset}-batch-L2.gguf")
    llmi.write_synthetic_gguf(path, preset, seed=11, n_layer=2)
    rng = np.random.default_rng(5 + k)
    prompts = _prompts(rng, k, hi=30000, max_len=24)
    want, want_lg = _single_reference(path, prompts, 10, 256)
    got, got_lg, _ = _batched(path, prompts, 10, 256, n_seq=k)
    for s in range(k):
        assert np.array_equal(got_lg[s], want_lg[s]), f"seq {s}: prompt logits differ"
        assert got[s] == want[s], f"seq {s}"


def test_batched_long_context_gqa8(gpu, synth_dir):
    """TinyLlama shapes (GQA 8) with one sequence past 4096 positions: the batched step's
    attention used to hold 8 heads x kv_bound scores in LDS and refused such batches; it
    now takes the long-context path (per-tile exp / PV partials) and every sequence's
    tokens and logits equal its single decode."""
    path = str(synth_dir / "tinyllama-q8_0-batch-L2.gguf")
    llmi.write_synthetic_gguf(path, "tinyllama-q8_0", seed=11, n_layer=2)
    rng = np.random.default_rng(8)
    prompts = [[1] + [int(t) for t in rng.integers(3, 30000, 4150)], [1] + [int(t) for t in rng.integers(3, 30000, 20)]]
    want, want_lg = _single_reference(path, prompts, 3, 4352)
    got, got_lg, _ = _batched(path, prompts, 3, 4352, n_seq=2)
    for s in range(2):
        assert np.array_equal(got_lg[s], want_lg[s]), f"seq {s}: prompt logits differ"
        assert got[s] == want[s], f"seq {s}: batched {got[s]} single {want[s]}"


@pytest.mark.parametrize("mode", ["2", "6", "7"])
def test_batched_attention_paths(gpu, tiny_models, monkeypatch, mode):
    """The batched step's attention forced to each path (LLMI_BATTN_MODE: 2 split, 6
    dim-split, 7 long-context), sequences straddling a KV bucket: tokens equal single
    decode."""
    monkeypatch.setenv("LLMI_BATTN_MODE", mode)
    for preset in ("tiny-mixed-d128",):  # (tiny-mixed: gate/up types differ, not batchable)
        path = tiny_models[preset]
        rng = np.random.default_rng(70 + int(mode))
        prompts = [[1] + [int(t) for t in rng.integers(3, 700, 249)], [1] + [int(t) for t in rng.integers(3, 700, 9)],
                   [1] + [int(t) for t in rng.integers(3, 700, 120)]]
        want, _ = _single_reference(path, prompts, 16, 512)
        got, _, _ = _batched(path, prompts, 16, 512)
        assert got == want, preset


@pytest.mark.parametrize("preset", ["tiny-mixed-d128", "tiny-mixed"])
def test_batched_steps_vs_oracle(gpu, tiny_models, preset):
    """The batched step against the oracle directly (ggml's generic fp32 order): 4 sequences at
    different positions advance one token per llama_decode call (one batched step; for
    tiny-mixed, whose layer 0 mixes gate/up types, the per-sequence fallback), and every
    sequence's logits equal the oracle's decode of that sequence, bit for bit."""
    import pyoracle as po

    path = tiny_models[preset]
    rng = np.random.default_rng(31)
    prompts = _prompts(rng, 4, min_len=3, max_len=30)
    oms = [po.OracleModel(path, n_ctx=256) for _ in prompts]
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=256, n_seq=4)
    cur, pos = [], []
    for s, p in enumerate(prompts):
        for k, t in enumerate(p[:-1]):
            oms[s].decode(t, k, logits=False)
        assert c.decode(p[:-1], seq=[s] * (len(p) - 1)) == 0
        cur.append(p[-1])
        pos.append(len(p) - 1)
    for step in range(6):
        assert c.decode(cur, pos=pos, seq=[0, 1, 2, 3], logits_all=True) == 0
        for s in range(4):
            want = oms[s].decode(cur[s], pos[s])
            got = c.logits(s)
            assert np.array_equal(got, want), f"step {step} seq {s}: max |d| {np.abs(got - want).max():.3g}"
            cur[s] = int(np.argmax(want))
            pos[s] += 1
    for om in oms:
        om.close()

