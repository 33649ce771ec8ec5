"""Long and full-width parity runs against the oracle (ggml's generic order), through the C ABI
and the HTTP front end — the BASELINE.json configs the shorter tests do not reach:

- C1: TinyLlama-1.1B Q8_0 (exact widths, all 22 layers), 16-token greedy decode driven
  through llmi.server over HTTP the way the reference gateway sends it, ids equal to the
  oracle's;
- C4: Mistral-7B widths (2 layers), a 2048-token prompt through the batched MFMA
  prefill (four 512-token ubatches), then decode steps — logits bit-identical to the
  oracle, once with the all-Q6_K table and once with the Q5_K_M table;
- >= 4096 positions: a tiny model's prompt of 4100 tokens, then decode steps on every
  attention path the dispatch can pick at that length (auto = split, fused, two-kernel);
- the prefill-length limit: a prompt reaching past the batched-prefill attention's KV
  limit continues as decode steps, bit-identical;
- the fault path: a bounded in-kernel wait that gives up makes llama_decode return -6
  instead of NaN logits;
- the north star's "within 1e-3 of the CPU path" on the configs' real trajectories (8B:
  128-token prompt -> 512 steps; 70B widths: 8 -> 128; TinyLlama; Mistral Q5_K_M), asserted
  bit-identical to the oracle (ggml's generic order) at every step and reported into
  $LLMI_REPORT_DIR/parity_generic.jsonl.
"""
from __future__ import annotations

import http.client
import json
import os
import threading

import numpy as np
import pytest

import llmi
import pyoracle as po

pytestmark = pytest.mark.gpu


def _oracle_run(path, prompt, n_ctx, n_gen, x86=0):
    """Oracle logits after the prompt (batched or_prefill for all but the last token)
    and for n_gen greedy steps after it (x86: the oracle's association flags)."""
    om = po.OracleModel(path, n_ctx=n_ctx, x86=x86)
    if len(prompt) > 1:
        om.prefill(prompt[:-1])
    lo = om.decode(prompt[-1], len(prompt) - 1)
    out = [lo]
    pos = len(prompt)
    for _ in range(n_gen):
        lo = om.decode(int(np.argmax(lo)), pos)
        out.append(lo)
        pos += 1
    om.close()
    return out


def _gpu_run(path, prompt, n_ctx, n_gen):
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


def _assert_same(got, want):
    for k, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, w), f"step {k}: max |d| {np.abs(g - w).max():.3g}"


# ---- C1: TinyLlama through the HTTP front end ---------------------------------------
@pytest.mark.parametrize("numerics", ["generic", "x86"])
def test_tinyllama_http_greedy16_vs_oracle(gpu, synth_dir, numerics):
    """TinyLlama-shaped Q8_0 GGUF (E 2048, 22 layers, V 32000), prompt
    BOS + 16 ids uniform in [3, V) (seed 2), greedy 16 tokens with temperature 0, top_k
    1, repeat_penalty 1.0, ignore_eos, sent as the gateway forwards it (lowercase
    headers, Bearer key, Connection: close); the ids equal the oracle's greedy ids, in
    both numerics (x86: `llama-server --numerics x86` against the oracle's x86 mode)."""
    from llmi.server import Engine, make_server

    path = str(synth_dir / "tinyllama-q8_0-full.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, "tinyllama-q8_0", seed=1)
    rng = np.random.default_rng(2)
    prompt = [1] + [int(t) for t in rng.integers(3, 32000, 16)]
    x86 = numerics == "x86"
    want_logits = _oracle_run(path, prompt, 64, 15, x86=po.X86_ALL if x86 else 0)
    want = [int(np.argmax(lo)) for lo in want_logits]

    eng = Engine(path, 64, 99, [0], numerics=llmi.NUMERICS_X86 if x86 else llmi.NUMERICS_GENERIC)
    eng.load()
    assert eng.ready, eng.error
    srv = make_server(eng, "127.0.0.1", 0, "k-test")
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        body = json.dumps({"prompt": prompt, "max_tokens": 16, "temperature": 0, "top_k": 1, "repeat_penalty": 1.0,
                           "ignore_eos": True})
        conn = http.client.HTTPConnection("127.0.0.1", srv.server_address[1], timeout=120)
        conn.request("POST", "/v1/completions", body=body,
                     headers={"content-type": "application/json", "Authorization": "Bearer k-test",
                              "Connection": "close"})
        r = conn.getresponse()
        d = json.loads(r.read())
        conn.close()
        assert r.status == 200
        assert d["llmi"]["tokens"] == want
        assert d["usage"] == {"prompt_tokens": 17, "completion_tokens": 16, "total_tokens": 33}
    finally:
        srv.shutdown()
        srv.server_close()


# ---- C4: 2048-token prompts at Mistral widths ----------------------------------------
@pytest.mark.parametrize("preset", ["mistral7b-q6k", "mistral7b-q5km"])
def test_mistral_2048_prefill_vs_oracle(gpu, synth_dir, preset):
    """SURVEY.md §8d C4 (2 layers, full V 32000): a 2048-token prompt through the batched
    prefill, then 3 decode steps; logits bit-identical to the oracle at every step."""
    path = str(synth_dir / f"{preset}-L2-full.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=2)
    rng = np.random.default_rng(11)
    prompt = [1] + [int(t) for t in rng.integers(3, 32000, 2047)]
    m, got = _gpu_run(path, prompt, 2304, 3)
    assert m.prefill_supported
    _assert_same(got, _oracle_run(path, prompt, 2304, 3))


# ---- >= 4096 positions on every attention path ----------------------------------------
_LONG = {}


def _long_oracle(path, prompt):
    key = (path, len(prompt))
    if key not in _LONG:
        _LONG[key] = _oracle_run(path, prompt, 4352, 4)
    return _LONG[key]


@pytest.mark.parametrize("preset,mode", [("tiny-mixed-d128", "0"), ("tiny-mixed-d128", "1"),
                                         ("tiny-mixed-d128", "3"), ("tiny-mixed-d128", "7"),
                                         ("tiny-mixed", "0"), ("tiny-mixed", "7")])
def test_decode_past_4096_positions(gpu, tiny_models, monkeypatch, preset, mode):
    """A 4100-token prompt (batched prefill) and 4 decode steps at positions 4100-4103
    with the attention path forced (LLMI_ATTN_MODE, read at context creation): 0 auto,
    1 fused one-workgroup-per-head, 3 two-kernel, 7 long-context four-launch."""
    path = tiny_models[preset]
    rng = np.random.default_rng(41)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 4099)]
    monkeypatch.setenv("LLMI_ATTN_MODE", mode)
    try:
        _, got = _gpu_run(path, prompt, 4352, 4)
    finally:
        monkeypatch.setenv("LLMI_ATTN_MODE", "0")
        llmi.Context(llmi.Model(path), n_ctx=32).close()  # reset the process-wide mode
    _assert_same(got, _long_oracle(path, prompt))


def test_prompt_past_prefill_kv_limit(gpu, tiny_models, monkeypatch):
    """A prompt reaching past the batched-prefill attention's KV limit (lowered to 200
    for the test) is prefilled up to the limit and continues as decode steps: logits
    bit-identical to the oracle and to all-decode-step processing."""
    path = tiny_models["tiny-mixed"]
    rng = np.random.default_rng(12)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 299)]
    old = llmi.test_option("pf_max_kv", 200)
    try:
        _, got = _gpu_run(path, prompt, 512, 2)
    finally:
        llmi.test_option("pf_max_kv", old)
    _assert_same(got, _oracle_run(path, prompt, 512, 2))
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    _, steps = _gpu_run(path, prompt, 512, 2)
    _assert_same(got, steps)


def _with_option(name, value, fn):
    old = llmi.test_option(name, value)
    try:
        return fn()
    finally:
        llmi.test_option(name, old)


def test_prefill_attention_past_16k_positions(gpu, tiny_models, monkeypatch):
    """A 16500-token prompt through every batched-prefill attention path: the tiled
    FP64-MFMA kernel (default), the G-heads-per-workgroup LDS kernel and the one-head LDS
    kernel (both then hold > 64 KiB of scores in LDS; both once failed with "invalid
    argument" from a refused LDS attribute call).  Prefilled logits and the decode steps
    after them (long-context decode attention) equal all-decode-step processing of the
    prompt bit for bit."""
    path = tiny_models["tiny-mixed-d128"]
    rng = np.random.default_rng(16)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 16499)]
    _, tiled = _gpu_run(path, prompt, 16640, 2)
    _, grouped = _with_option("pf_attn_fa", 0, lambda: _gpu_run(path, prompt, 16640, 2))  # G = 2: 130 KiB LDS
    _, pf = _with_option("pf_attn_simple", 1, lambda: _gpu_run(path, prompt, 16640, 2))
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    _, steps = _gpu_run(path, prompt, 16640, 2)
    _assert_same(tiled, steps)
    _assert_same(pf, steps)
    _assert_same(grouped, steps)


def test_prefill_past_the_lds_limit(gpu, tiny_models, monkeypatch):
    """A 33000-token prompt: past kPfAttnMaxKV (32768) positions the LDS attention kernels
    cannot run, so before the tiled kernel the run's tail went through decode steps; now
    the whole prompt prefills (prefill_max_kv = the context) and still equals
    all-decode-step processing bit for bit."""
    path = tiny_models["tiny-mixed"]
    rng = np.random.default_rng(33)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 32999)]
    _, pf = _gpu_run(path, prompt, 33280, 2)
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    _, steps = _gpu_run(path, prompt, 33280, 2)
    _assert_same(pf, steps)


def test_prefill_attention_head_subgroups(gpu, synth_dir, monkeypatch):
    """Llama-3-8B widths (2 layers, GQA 4), a 10500-token prompt: past ~10k positions the
    four heads' scores no longer fit in LDS and the batched-prefill attention runs
    sub-groups of 2 heads per workgroup (with the tiled kernel switched off).  Prefilled
    logits and the next decode steps equal the one-head-per-workgroup kernel's, the tiled
    kernel's and all-decode-step processing bit for bit."""
    path = str(synth_dir / "llama3-8b-q4km-L2-sub.gguf")
    llmi.write_synthetic_gguf(path, "llama3-8b-q4km", seed=21, n_layer=2)
    rng = np.random.default_rng(17)
    prompt = [1] + [int(t) for t in rng.integers(3, 120000, 10499)]
    _, sub = _with_option("pf_attn_fa", 0, lambda: _gpu_run(path, prompt, 10752, 2))
    _, simple = _with_option("pf_attn_simple", 1, lambda: _gpu_run(path, prompt, 10752, 2))
    _, tiled = _gpu_run(path, prompt, 10752, 2)
    _assert_same(sub, simple)
    _assert_same(tiled, simple)
    monkeypatch.setenv("LLMI_NO_PREFILL", "1")
    _, steps = _gpu_run(path, prompt, 10752, 2)
    _assert_same(sub, steps)


def test_bounded_wait_fault_is_reported(gpu, tiny_models, monkeypatch):
    """k_attn_x's hand-off waits are bounded; with the bound lowered to 0 polls and the
    consumers waiting for a tag no producer writes (test options, captured into the step
    graph of the next KV bucket), every wait gives up, and each decode call reports it (-6, llmi_last_error) instead of returning 0 with
    NaN logits.  With the options restored the context decodes normally again."""
    path = tiny_models["tiny-mixed-d128"]
    monkeypatch.setenv("LLMI_ATTN_MODE", "4")
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=512)
    rng = np.random.default_rng(13)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, 199)]
    assert c.decode(prompt) == 0
    old = llmi.test_option("xspin_limit", 0)
    llmi.test_option("xtag_skew", 1)
    codes, msgs = [], []
    try:
        t = c.greedy(-1)
        for k in range(4):  # positions 256+: a KV bucket whose step graph is captured now
            rc = c.decode([t], pos=[256 + k])
            codes.append(rc)
            if rc == -6:
                msgs.append(llmi.last_error())
            if rc == 0:
                lg = c.logits(-1)
                assert np.isfinite(lg).all(), "a call that returned 0 has non-finite logits"
    finally:
        llmi.test_option("xspin_limit", old)
        llmi.test_option("xtag_skew", 0)
        monkeypatch.setenv("LLMI_ATTN_MODE", "0")
    assert codes == [-6] * 4, codes
    assert all("bounded wait" in e for e in msgs), msgs
    c.kv_clear()
    assert c.decode(prompt) == 0 and np.isfinite(c.logits(-1)).all()
    c.close()
    llmi.Context(m, n_ctx=32).close()


# ---- north star: the configs' real trajectories against ggml's generic fp32 order ------
# (BASELINE.json north_star: "within 1e-3 of the NGL=0 path ... bit-exact token ids"; the
# oracle restates ggml's generic scalar order, SURVEY.md §8c, and the GPU computes in that
# order, so the bar asserted here is stricter: bit-identical logits at every step.)
@pytest.mark.parametrize("preset,n_vocab,n_prompt,n_gen", [
    ("llama3-8b-q4km", 0, 128, 512),      # C2: 128-token prompt -> 512-token decode (ctx 640)
    ("llama3-70b-q4km", 32000, 8, 128),   # C5 widths (8192 / 28672 / GQA 8), decode-only
    ("tinyllama-q8_0", 0, 16, 128),       # C1 widths
    ("mistral7b-q5km", 0, 64, 64),        # C4 widths, mixed Q5_K / Q6_K table
])
def test_generic_order_trajectory(gpu, synth_dir, preset, n_vocab, n_prompt, n_gen):
    """Prompt through the batched prefill, then n_gen greedy steps, in lockstep with the
    oracle: logits bit-identical at every step (so every step is within 1e-3) and the
    same greedy ids.  2 layers at the preset's exact widths; reported into
    $LLMI_REPORT_DIR/parity_generic.jsonl."""
    path = str(synth_dir / f"{preset}-L2-v{n_vocab}.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=2, n_vocab=n_vocab)
    rng = np.random.default_rng(21)
    prompt = [1] + [int(t) for t in rng.integers(3, 30000, n_prompt - 1)]
    n_ctx = (n_prompt + n_gen + 255) // 256 * 256
    om = po.OracleModel(path, n_ctx=n_ctx)
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=n_ctx)
    if len(prompt) > 1:
        om.prefill(prompt[:-1])
    lo = om.decode(prompt[-1], len(prompt) - 1)
    assert c.decode(prompt) == 0
    lg = c.logits(-1)
    diffs, pos = [], len(prompt)
    for step in range(n_gen + 1):
        d = float(np.abs(lg - lo).max())
        diffs.append(d)
        assert np.array_equal(lg, lo), f"{preset} step {step} (pos {pos - 1}): max |d| {d:.3g}"
        if step == n_gen:
            break
        t = int(np.argmax(lo))
        assert c.greedy(-1) == t
        lo = om.decode(t, pos)
        assert c.decode([t], pos=[pos]) == 0
        lg = c.logits(-1)
        pos += 1
    om.close()
    c.close()
    rep = {"preset": preset, "n_layer": 2, "n_vocab": n_vocab or "full", "prompt": n_prompt,
           "steps": len(diffs), "ctx_end": pos, "frac_within_1e-3": float(np.mean(np.array(diffs) <= 1e-3)),
           "worst_abs_diff": max(diffs), "bit_identical": True}
    print(json.dumps(rep))
    out_dir = os.environ.get("LLMI_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "parity_generic.jsonl"), "a") as f:
            f.write(json.dumps(rep) + "\n")
