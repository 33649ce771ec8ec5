"""GPU parity in the x86 association mode (model numerics LLMI_NUMERICS_X86): every
kernel bit-identical to the oracle's x86 mode (oracle/ggml_oracle.c or_set_x86_mode,
X86_ALL = upstream's AVX2 vec_dot lanes + round-half-even q8_0 + 4x8-lane f16 dots +
ggml_v_expf), the restatement of the reference's NGL=0 CPU build (Dockerfile.cpu:11,
:84-89).  VERDICT r4 item 1.

- activation quantization: q8_K (ref) and q8_0 (x86 AVX2 rounding) bit-exact;
- matvec per type and shape: bit-exact vs or_matvec under X86_DOTS | X86_Q80;
- decode attention: bit-exact vs a NumPy restatement of the x86 f16 dots / v_expf softmax;
- whole-model trajectories at the configs' widths: logits bit-identical at every step;
- the per-op taps at Llama-3-8B widths.
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np
import pytest

import llmi
import pyoracle as po
from helpers import Q4_K, Q5_K, Q6_K, Q8_0, QTYPES, TNAME, empty_dev, random_blocks, to_dev
from test_gpu_kernels import edge_inputs

pytestmark = pytest.mark.gpu

X86 = po.X86_ALL


class numerics:
    """llmi_test_option("numerics"): this thread's kernel-level hooks in x86 numerics."""

    def __enter__(self):
        self.old = llmi.test_option("numerics", 1)

    def __exit__(self, *exc):
        llmi.test_option("numerics", self.old)
        return False


def _p(t):
    return C.c_void_p(t.data_ptr())


def gpu_quant_x86(qtype, x, nw=None, eps=1e-5):
    import torch

    cols = x.size
    nbytes = cols // 256 * 292 if qtype != Q8_0 else cols // 32 * 34
    out = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    xd = to_dev(x.astype(np.float32))
    nd = to_dev(nw.astype(np.float32)) if nw is not None else None
    torch.cuda.synchronize()
    with numerics():
        rc = llmi.lib().llmi_quantize_act(qtype, cols, _p(xd), _p(nd) if nd is not None else None, eps, _p(out))
    assert rc == 0, llmi.last_error()
    return out.cpu().numpy()


def q80_half_even_inputs(cols, rng):
    """q8_0 blocks whose scaled values land exactly on .5 (where round-half-even and
    roundf differ): amax = 127 makes id = 1, so x = k + 0.5 maps onto itself."""
    h = rng.uniform(-100, 100, cols).astype(np.float32)
    for b in range(0, cols, 32):
        h[b] = 127.0
        h[b + 1: b + 17] = (np.arange(16, dtype=np.float32) - 8.0) + 0.5
    return h


@pytest.mark.parametrize("qtype", [Q4_K, Q8_0], ids=["q8_K", "q8_0"])
@pytest.mark.parametrize("cols", [256, 4096, 14336])
def test_x86_activation_quant_bitexact(gpu, qtype, cols):
    rng = np.random.default_rng(cols + 5)
    cases = edge_inputs(cols, rng) + [("half_even", q80_half_even_inputs(cols, rng))]
    for name, x in cases:
        ref = po.quantize_act(qtype, x, x86=X86)
        got = gpu_quant_x86(qtype, x)
        assert np.array_equal(ref, got), f"{name}: x86 quantized activation differs"
    if qtype == Q8_0:  # the two roundings really differ on these inputs
        h = q80_half_even_inputs(cols, rng)
        assert not np.array_equal(po.quantize_act(Q8_0, h), po.quantize_act(Q8_0, h, x86=X86))


def gpu_matvec_x86(qtype, raw, rows, cols, x, nw=None, eps=1e-5):
    import torch

    L = llmi.lib()
    with numerics():
        nbytes = L.llmi_device_layout_bytes(qtype, rows, cols)
        rd = to_dev(raw)
        wd = empty_dev(nbytes)
        torch.cuda.synchronize()
        assert L.llmi_repack(qtype, _p(rd), _p(wd), rows, cols) == 0
        xd = to_dev(x.astype(np.float32))
        nd = to_dev(nw.astype(np.float32)) if nw is not None else None
        yd = torch.zeros(rows, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rc = L.llmi_matvec(qtype, _p(wd), rows, cols, _p(xd), _p(nd) if nd is not None else None, eps, _p(yd), 0)
        assert rc == 0, llmi.last_error()
    return yd.cpu().numpy()


SHAPES = [(2, 256), (7, 512), (130, 1024), (1024, 4096), (333, 14336), (64, 8192), (130, 5632), (5, 28672),
          (2048, 14336)]


@pytest.mark.parametrize("qtype", QTYPES, ids=[TNAME[t] for t in QTYPES])
@pytest.mark.parametrize("rows,cols", SHAPES)
def test_x86_matvec_vs_oracle(gpu, qtype, rows, cols):
    rng = np.random.default_rng(rows * 17 + cols + qtype)
    raw = random_blocks(qtype, rows, cols, rng)
    x = rng.standard_normal(cols).astype(np.float32)
    got = gpu_matvec_x86(qtype, raw, rows, cols, x)
    ref = po.matvec(qtype, raw, rows, cols, x, x86=X86)
    gen = po.matvec(qtype, raw, rows, cols, x)
    err = float(np.abs(got - ref).max())
    assert np.array_equal(got, ref), f"not bit-exact vs the oracle's x86 mode (max |err| {err:.3g})"
    if rows * cols >= 1 << 16:  # the association really differs from the generic order
        assert not np.array_equal(ref, gen)


@pytest.mark.parametrize("qtype", QTYPES, ids=[TNAME[t] for t in QTYPES])
@pytest.mark.parametrize("rows,cols", [(96, 2048), (70, 8192)])
def test_x86_matvec_fused_rmsnorm(gpu, qtype, rows, cols):
    rng = np.random.default_rng(29 + qtype)
    raw = random_blocks(qtype, rows, cols, rng)
    x = (rng.standard_normal(cols) * 4).astype(np.float32)
    w = rng.uniform(0.8, 1.2, cols).astype(np.float32)
    ref = po.matvec(qtype, raw, rows, cols, po.rms_norm_mul(x, w, 1e-5), x86=X86)
    got = gpu_matvec_x86(qtype, raw, rows, cols, x, w, 1e-5)
    assert np.array_equal(got, ref)


# ---- attention ----------------------------------------------------------------------------
def _f16(a):
    return np.asarray(a, dtype=np.float32).astype(np.float16)


def _x86_dot(a, b):
    """ggml_vec_dot_f16 (x86 AVX2): rows of a . b over the last axis (a multiple of 32),
    element i into lane i % 32 by fp32 fma (the f16 x f16 products are exact in fp32, so
    fma == one fp32 add of the product), then the GGML_F16_VEC_REDUCE order."""
    n = a.shape[-1]
    acc = np.zeros(a.shape[:-1] + (32,), np.float32)
    for i in range(n):
        acc[..., i % 32] = (acc[..., i % 32] + (a[..., i] * b[..., i]).astype(np.float32)).astype(np.float32)
    c = (acc[..., 0:8] + acc[..., 16:24]) + (acc[..., 8:16] + acc[..., 24:32])
    t = c[..., 0:4] + c[..., 4:8]
    return ((t[..., 0] + t[..., 1]) + (t[..., 2] + t[..., 3])).astype(np.float32)


def _x86_expf(v):
    with po.x86_mode(po.X86_VEXP):
        return np.array([po.expf(float(x)) for x in v], dtype=np.float32)


def _ref_attention_x86(q, K, V, n_kv, G, scale):
    H, D = q.shape
    out = np.empty((H, D), np.float32)
    qf = _f16(q).astype(np.float32)
    np_ = (n_kv + 31) // 32 * 32
    for h in range(H):
        g = h // G
        k = K[g, :n_kv, :].astype(np.float32)
        w = (_x86_dot(k, np.broadcast_to(qf[h], k.shape)) * np.float32(scale)).astype(np.float32)
        mx = w.max()
        e = np.zeros(np_, np.float32)
        e[:n_kv] = _x86_expf((w - mx).astype(np.float32))
        e8 = e.reshape(-1, 8)
        t = e8[:, 0:4] + e8[:, 4:8]
        hs = ((t[:, 0] + t[:, 2]) + (t[:, 1] + t[:, 3])).astype(np.float32)
        s = np.cumsum(hs.astype(np.float64))[-1]
        inv = np.float32(1.0 / s)
        p = np.zeros(np_, np.float32)
        p[:n_kv] = _f16((e[:n_kv] * inv).astype(np.float32)).astype(np.float32)
        v = np.zeros((D, np_), np.float32)
        v[:, :n_kv] = V[g, :, :n_kv].astype(np.float32)
        out[h] = _x86_dot(v, np.broadcast_to(p, v.shape))
    return out


@pytest.mark.parametrize("H,HK,D,n_kv", [(32, 8, 128, 1), (32, 8, 128, 200), (32, 8, 128, 700),
                                         (64, 8, 128, 333), (32, 4, 64, 300), (32, 4, 64, 2100),
                                         (32, 8, 128, 2048), (8, 8, 64, 97), (16, 8, 128, 1500)])
@pytest.mark.parametrize("mode", [0, 3])  # 0: one launch (k_a86_d) up to 2048 positions, 3: three launches
def test_x86_attention_vs_numpy(gpu, H, HK, D, n_kv, mode):
    import torch

    rng = np.random.default_rng(77 + n_kv)
    n_ctx = (n_kv + 255) // 256 * 256
    G = H // HK
    K = np.zeros((HK, n_ctx, D), np.float16)
    V = np.zeros((HK, D, n_ctx), np.float16)
    K[:, :n_kv, :] = _f16(rng.standard_normal((HK, n_kv, D)) * 0.6)
    V[:, :, :n_kv] = _f16(rng.standard_normal((HK, D, n_kv)))
    q = (rng.standard_normal((H, D)) * 0.8).astype(np.float32)
    out = torch.empty(H * D, dtype=torch.float32, device="cuda")
    qd, kd, vd = to_dev(q.reshape(-1)), to_dev(K.view(np.uint16).reshape(-1)), to_dev(V.view(np.uint16).reshape(-1))
    with numerics():
        rc = llmi.lib().llmi_attention(H, HK, D, n_kv, n_ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(),
                                       out.data_ptr(), mode)
    assert rc == 0, llmi.last_error()
    got = out.cpu().numpy().reshape(H, D)
    want = _ref_attention_x86(q, K, V, n_kv, G, 1.0 / np.sqrt(np.float32(D)))
    bad = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} outputs differ, first {bad[:3].tolist()}"


# ---- whole model ----------------------------------------------------------------------------
@pytest.mark.parametrize("preset", ["tiny-mixed", "tiny-mixed-d128"])
def test_x86_tiny_decode_vs_oracle(gpu, tiny_models, preset):
    """Every quant type, both head dims: 40 decode steps bit-identical to the oracle's x86
    mode (and different from its generic order)."""
    path = tiny_models[preset]
    m = llmi.Model(path, numerics=llmi.NUMERICS_X86)
    assert m.numerics == llmi.NUMERICS_X86
    c = llmi.Context(m, n_ctx=256)
    om, og = po.OracleModel(path, n_ctx=256, x86=X86), po.OracleModel(path, n_ctx=256)
    differs = False
    t = 1
    for pos in range(40):
        assert c.decode([t], pos=[pos]) == 0
        lg, lo, ln = c.logits(-1), om.decode(t, pos), og.decode(t, pos)
        assert np.array_equal(lg, lo), f"pos {pos}: max |d| {np.abs(lg - lo).max():.3g}"
        differs |= not np.array_equal(lo, ln)
        assert c.greedy(-1) == int(np.argmax(lo))
        t = int(np.argmax(lo))
    assert differs, "x86 and generic orders gave identical logits (the mode is not exercised)"
    om.close(), og.close(), c.close(), m.close()


@pytest.mark.parametrize("preset,n_vocab,n_prompt,n_gen", [
    ("llama3-8b-q4km", 0, 128, 512),      # C2: 128-token prompt -> 512-token decode (ctx 640)
    ("llama3-70b-q4km", 32000, 8, 128),   # C5 widths (8192 / 28672 / GQA 8), decode-only
    ("tinyllama-q8_0", 0, 16, 128),       # C1 widths
    ("mistral7b-q5km", 0, 64, 64),        # C4 widths, mixed Q5_K / Q6_K table
    ("mistral7b-q6k", 0, 64, 64),         # C4 widths, all Q6_K
])
def test_x86_order_trajectory(gpu, synth_dir, preset, n_vocab, n_prompt, n_gen):
    """The configs' real trajectories (2 layers at the preset's exact widths) in x86
    numerics, in lockstep with the oracle's x86 mode: logits bit-identical at every step,
    the same greedy ids.  Reported into $LLMI_REPORT_DIR/parity_x86.jsonl."""
    path = str(synth_dir / f"{preset}-L2-v{n_vocab}.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=2, n_vocab=n_vocab)
    rng = np.random.default_rng(21)
    prompt = [1] + [int(t) for t in rng.integers(3, 30000, n_prompt - 1)]
    n_ctx = (n_prompt + n_gen + 255) // 256 * 256
    om = po.OracleModel(path, n_ctx=n_ctx, x86=X86)
    m = llmi.Model(path, numerics=llmi.NUMERICS_X86)
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
    rep = {"preset": preset, "numerics": "x86", "oracle_flags": X86, "n_layer": 2, "n_vocab": n_vocab or "full",
           "prompt": n_prompt, "steps": len(diffs), "ctx_end": pos,
           "frac_within_1e-3": float(np.mean(np.array(diffs) <= 1e-3)), "worst_abs_diff": max(diffs),
           "bit_identical": True, "ids_identical": True}
    print(json.dumps(rep))
    out_dir = os.environ.get("LLMI_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "parity_x86.jsonl"), "a") as f:
            f.write(json.dumps(rep) + "\n")


def test_x86_per_op_taps_8b_widths(gpu, synth_dir):
    """Each intermediate of the x86 decode step equals the oracle's x86 tap bit for bit
    (embedding row, RoPE'd q, K/V cache rows, attention output, SwiGLU, residual) at
    Llama-3-8B widths, positions 127 and 383."""
    from test_gpu_taps import _check_taps

    path = str(synth_dir / "llama3-8b-q4km-L2-v32000-taps86.gguf")
    llmi.write_synthetic_gguf(path, "llama3-8b-q4km", seed=3, n_layer=2, n_vocab=32000)
    n_ctx = 512
    rng = np.random.default_rng(43)
    prompt = [1] + [int(t) for t in rng.integers(3, 32000, 127)]
    om = po.OracleModel(path, n_ctx=n_ctx, x86=X86)
    m = llmi.Model(path, numerics=llmi.NUMERICS_X86)
    c = llmi.Context(m, n_ctx=n_ctx)
    try:
        om.prefill(prompt[:-1])
        om.decode(prompt[-1], 127, logits=False)
        assert c.decode(prompt) == 0
        _check_taps(c, om, 127, "x86 pos 127")
        for i, t in enumerate(int(t) for t in rng.integers(3, 32000, 383 - 127)):
            om.decode(t, 128 + i, logits=False)
            assert c.decode([t], pos=[128 + i]) == 0
        _check_taps(c, om, 383, "x86 pos 383")
    finally:
        om.close()
        c.close()
        m.close()


def test_x86_batch_api_sequential(gpu, tiny_models):
    """x86 numerics on a model with Q8_0 and K-quant tensors (tiny-mixed-d128: Q8_0
    attn_output / ffn_down): llmi_generate_greedy_batch (batched steps: k_mvn's x86 forms
    incl. Q8_0's 4-wave one) equals each sequence's own single-sequence generation."""
    path = tiny_models["tiny-mixed-d128"]
    m = llmi.Model(path, numerics=llmi.NUMERICS_X86)
    c = llmi.Context(m, n_ctx=128, n_seq=3)
    got = c.generate_greedy_batch([0, 1, 2], [5, 9, 11], [0, 0, 0], 12)
    c1 = llmi.Context(m, n_ctx=128)
    for k, first in enumerate([5, 9, 11]):
        c1.kv_clear()
        assert c1.generate_greedy(first, 0, 12) == got[k]
    c.close(), c1.close(), m.close()


# ---- prefill (batched MFMA GEMM + k_pf_a86) ---------------------------------------------------
@pytest.mark.parametrize("qtype", [Q4_K, Q5_K, Q6_K, Q8_0], ids=["q4_K", "q5_K", "q6_K", "q8_0"])
@pytest.mark.parametrize("rows,cols,n_tok", [(64, 256, 5), (128, 4096, 40), (1024, 4096, 130), (64, 14336, 64),
                                             (256, 5632, 33)])
def test_x86_pf_gemm_equals_matvecs(gpu, qtype, rows, cols, n_tok):
    """The x86 prefill GEMM (f16-MFMA integer sums, x86 fma lane chains, Q4_K's four min
    lanes from masked sumi MFMAs; Q8_0's eight lanes per block from masked-weight MFMAs)
    equals n_tok x86 matvecs and the oracle bit for bit."""
    import torch

    rng = np.random.default_rng(rows + cols + n_tok + qtype)
    raw = random_blocks(qtype, rows, cols, rng)
    X = rng.standard_normal((n_tok, cols)).astype(np.float32)
    L = llmi.lib()
    with numerics():
        nbytes = L.llmi_device_layout_bytes(qtype, rows, cols)
        rd, wd = to_dev(raw), empty_dev(nbytes)
        torch.cuda.synchronize()
        assert L.llmi_repack(qtype, _p(rd), _p(wd), rows, cols) == 0
        xd = to_dev(X.reshape(-1))
        yd = torch.zeros(n_tok * rows, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rc = L.llmi_pf_gemm(qtype, _p(wd), rows, cols, _p(xd), None, 1e-5, n_tok, _p(yd), None)
        assert rc == 0, llmi.last_error()
    got = yd.cpu().numpy().reshape(n_tok, rows)
    for t in range(n_tok):
        ref = po.matvec(qtype, raw, rows, cols, X[t], x86=X86)
        assert np.array_equal(got[t], ref), f"token {t}: max |d| {np.abs(got[t] - ref).max():.3g}"


@pytest.mark.parametrize("preset", ["mistral7b-q6k", "mistral7b-q5km"])
def test_x86_mistral_2048_prefill_vs_oracle(gpu, synth_dir, preset):
    """SURVEY.md §8d C4 in x86 numerics (2 layers, full V 32000): a 2048-token prompt through
    the batched prefill (x86 GEMM + k_pf_a86), then 3 decode steps; logits bit-identical
    to the oracle's x86 mode at every step."""
    from test_gpu_long import _assert_same

    path = str(synth_dir / f"{preset}-L2-full.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=2)
    rng = np.random.default_rng(11)
    prompt = [1] + [int(t) for t in rng.integers(3, 32000, 2047)]
    m = llmi.Model(path, numerics=llmi.NUMERICS_X86)
    assert m.prefill_supported
    c = llmi.Context(m, n_ctx=2304)
    assert c.decode(prompt) == 0
    got = [c.logits(-1)]
    pos = len(prompt)
    for _ in range(3):
        t = c.greedy(-1)
        assert c.decode([t], pos=[pos]) == 0
        got.append(c.logits(-1))
        pos += 1
    om = po.OracleModel(path, n_ctx=2304, x86=X86)
    om.prefill(prompt[:-1])
    want = [om.decode(prompt[-1], len(prompt) - 1)]
    pos = len(prompt)
    for _ in range(3):
        want.append(om.decode(int(np.argmax(want[-1])), pos))
        pos += 1
    om.close()
    _assert_same(got, want)



def test_x86_tinyllama_prefill_vs_oracle(gpu, synth_dir):
    """C1's model in x86 numerics (Q8_0 everywhere; 2 layers, full V 32000): a 300-token
    prompt through the batched prefill (the Q8_0 x86 GEMM + k_pf_a86),
    then 3 decode steps; logits bit-identical to the oracle's x86 mode at every step."""
    from test_gpu_long import _assert_same

    path = str(synth_dir / "tinyllama-q8_0-L2-full.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, "tinyllama-q8_0", seed=3, n_layer=2)
    rng = np.random.default_rng(12)
    prompt = [1] + [int(t) for t in rng.integers(3, 32000, 299)]
    m = llmi.Model(path, numerics=llmi.NUMERICS_X86)
    assert m.prefill_supported
    c = llmi.Context(m, n_ctx=512)
    assert c.decode(prompt) == 0
    got = [c.logits(-1)]
    pos = len(prompt)
    for _ in range(3):
        t = c.greedy(-1)
        assert c.decode([t], pos=[pos]) == 0
        got.append(c.logits(-1))
        pos += 1
    om = po.OracleModel(path, n_ctx=512, x86=X86)
    om.prefill(prompt[:-1])
    want = [om.decode(prompt[-1], len(prompt) - 1)]
    pos = len(prompt)
    for _ in range(3):
        want.append(om.decode(int(np.argmax(want[-1])), pos))
        pos += 1
    om.close()
    c.close(), m.close()
    _assert_same(got, want)


# ---- batched steps in x86 numerics (k_mvn's x86 form) -----------------------
@pytest.mark.parametrize("preset", ["llama3-8b-q4km", "tinyllama-q8_0"])
@pytest.mark.parametrize("numerics", [llmi.NUMERICS_X86, llmi.NUMERICS_X86 | llmi.NUMERICS_FA,
                                      llmi.NUMERICS_FA])
def test_x86_and_fa_batched_steps_vs_oracle(gpu, synth_dir, numerics, preset):
    """A K-quant model in x86 (and/or flash-attention) numerics advances 5 sequences per
    llama_decode call through the batched step (k_mvn x86 form / matrix cores, attention per
    slot), each sequence's logits bit-identical to the oracle's decode in the same mode;
    llmi_generate_greedy_batch (which fails rather than falling back) over 8 sequences
    equals each sequence's single decode."""
    path = str(synth_dir / f"{preset}-L2-v32000.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=2, n_vocab=32000)
    flags = (X86 if numerics & llmi.NUMERICS_X86 else 0) | (po.X86_FA if numerics & llmi.NUMERICS_FA else 0)
    rng = np.random.default_rng(41)
    prompts = [[1] + [int(t) for t in rng.integers(3, 30000, int(n))] for n in rng.integers(2, 40, 5)]
    oms = [po.OracleModel(path, n_ctx=256, x86=flags) for _ in prompts]
    m = llmi.Model(path, numerics=numerics)
    c = llmi.Context(m, n_ctx=256, n_seq=5)
    cur, pos = [], []
    for s, p in enumerate(prompts):
        for k, t in enumerate(p[:-1]):
            oms[s].decode(t, k, logits=False)
        assert c.decode(p[:-1], seq=[s] * (len(p) - 1)) == 0
        cur.append(p[-1])
        pos.append(len(p) - 1)
    for step in range(5):
        assert c.decode(cur, pos=pos, seq=[0, 1, 2, 3, 4], logits_all=True) == 0
        for s in range(5):
            want = oms[s].decode(cur[s], pos[s])
            got = c.logits(s)
            assert np.array_equal(got, want), f"step {step} seq {s}: max |d| {np.abs(got - want).max():.3g}"
            cur[s] = int(np.argmax(want))
            pos[s] += 1
    for om in oms:
        om.close()
    c.close()
    c8 = llmi.Context(m, n_ctx=128, n_seq=8)
    firsts = [int(t) for t in rng.integers(3, 30000, 8)]
    got = c8.generate_greedy_batch(list(range(8)), firsts, [0] * 8, 10)
    c1 = llmi.Context(m, n_ctx=128)
    for k in range(8):
        c1.kv_clear()
        assert c1.generate_greedy(firsts[k], 0, 10) == got[k], f"sequence {k}"
    c8.close(), c1.close(), m.close()
