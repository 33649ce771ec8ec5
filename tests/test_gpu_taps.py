"""Per-op GPU parity:
after the same decode step, each intermediate the GPU step produced (llmi_debug_tap)
equals the oracle's (or_tap) bit for bit, so a broken op fails its own assertion
instead of showing up only in the logits.  Llama-3-8B widths (E 4096, 32/8 heads of
128, FF 14336, Q4_K_M type table), 2 layers, at positions 127 (the prompt's last token,
after the batched prefill) and 639 (the end of the C2 trajectory).

Also the attention's double-absorption property: the GPU
reduces q.k and PV by lane butterflies in double where the oracle sums sequentially;
they agree because double absorbs the reordering.  test_attention_wide_dynamic_range
feeds K, V and q whose products span ~2^-40..2^20 and whose probabilities span the f16
range, on every attention path, and still requires bit equality with a NumPy restatement
of the oracle's sequential order.
"""
from __future__ import annotations

import numpy as np
import pytest

import llmi
import pyoracle as po

pytestmark = pytest.mark.gpu


def _gpu_kv_rows(raw: np.ndarray, hk: int, n_ctx: int, d: int, pos: int, transposed: bool) -> np.ndarray:
    """Position pos of the GPU cache (K [HK][n_ctx][D], V [HK][D][n_ctx]) as [HK*D]."""
    if transposed:
        return raw.reshape(hk, d, n_ctx)[:, :, pos].reshape(-1)
    return raw.reshape(hk, n_ctx, d)[:, pos, :].reshape(-1)


def _check_taps(c, om, pos, where):
    E, H, HK, D, F = om.n_embd, om.n_head, om.n_head_kv, om.head_dim, om.n_ff
    kvd = HK * D
    assert np.array_equal(c.tap(0, E), om.tap(0)), f"{where}: a10 get_rows (embedding row) differs"
    assert np.array_equal(c.tap(2, H * D), om.tap(2)), f"{where}: a12 RoPE'd q differs"
    gk = _gpu_kv_rows(c.tap(7, HK * c.n_ctx * D), HK, c.n_ctx, D, pos, False)
    gv = _gpu_kv_rows(c.tap(8, HK * c.n_ctx * D), HK, c.n_ctx, D, pos, True)
    ok = om.tap(7).reshape(om.n_ctx, kvd)[pos]
    ov = om.tap(8).reshape(om.n_ctx, kvd)[pos]
    assert np.array_equal(gk, ok), f"{where}: a12/a16 RoPE'd K row in the f16 cache differs"
    assert np.array_equal(gv, ov), f"{where}: a16 V row in the f16 cache differs"
    assert np.array_equal(c.tap(3, H * D), om.tap(3)), f"{where}: a13 attention output differs"
    assert np.array_equal(c.tap(4, F), om.tap(4)), f"{where}: a14 SwiGLU output differs"
    assert np.array_equal(c.tap(1, E), om.tap(1)), f"{where}: a14 residual stream after the last layer differs"


def test_per_op_taps_8b_widths(synth_dir):
    path = str(synth_dir / "llama3-8b-q4km-L2-v32000-taps.gguf")
    llmi.write_synthetic_gguf(path, "llama3-8b-q4km", seed=3, n_layer=2, n_vocab=32000)
    po.prefer_simd()
    n_ctx = 768
    rng = np.random.default_rng(41)
    prompt = [1] + [int(t) for t in rng.integers(3, 32000, 127)]
    om = po.OracleModel(path, n_ctx=n_ctx)
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=n_ctx)
    try:
        om.prefill(prompt[:-1])
        om.decode(prompt[-1], 127, logits=False)
        assert c.decode(prompt) == 0
        _check_taps(c, om, 127, "pos 127")
        toks = [int(t) for t in rng.integers(3, 32000, 639 - 127)]
        for i, t in enumerate(toks):  # teacher-forced, the same token on both sides
            p = 128 + i
            om.decode(t, p, logits=False)
            assert c.decode([t], pos=[p]) == 0
        _check_taps(c, om, 639, "pos 639")
    finally:
        om.close()
        c.close()
        m.close()


# ---- attention: wide dynamic range --------------------------------------------------------
def _f16(a):
    return np.asarray(a, dtype=np.float32).astype(np.float16)


def _ref_attention(q, K, V, n_kv, G, scale):
    """oracle/ggml_oracle.c attn_head per head: q rounded to f16; kq = sequential double
    sum of the exact f16 products; soft_max with llmi_expf and a sequential double sum;
    p rounded to f16; out = sequential double sum of v * p over the positions."""
    H, D = q.shape
    out = np.empty((H, D), np.float32)
    qf = _f16(q).astype(np.float32)
    for h in range(H):
        g = h // G
        k = K[g, :n_kv, :].astype(np.float32)                     # [n_kv, D]
        prod = (k * qf[h][None, :]).astype(np.float64)              # exact f16 x f16 products
        kq = np.cumsum(prod, axis=1)[:, -1].astype(np.float32)      # sequential double, then f32
        w = (kq * np.float32(scale)).astype(np.float32)
        mx = w.max()
        e = np.array([po.expf(float(x)) for x in (w - mx).astype(np.float32)], dtype=np.float32)
        s = np.cumsum(e.astype(np.float64))[-1]
        inv = np.float32(1.0 / s)
        p = _f16((e * inv).astype(np.float32)).astype(np.float32)
        v = V[g, :, :n_kv].astype(np.float32)                       # [D, n_kv]
        pv = (v * p[None, :]).astype(np.float64)
        out[h] = np.cumsum(pv, axis=1)[:, -1].astype(np.float32)
    return out


@pytest.mark.parametrize("H,HK,D,n_kv", [(32, 8, 128, 200), (32, 8, 128, 700), (32, 8, 128, 1500),
                                         (32, 4, 64, 300), (32, 4, 64, 2100)])
@pytest.mark.parametrize("mode", [0, 2, 6, 7])
def test_attention_wide_dynamic_range(H, HK, D, n_kv, mode):
    from helpers import to_dev
    import torch

    if mode == 6 and n_kv > 1024:
        pytest.skip("dim-split path is bounded at 1024 positions")
    rng = np.random.default_rng(1000 * mode + n_kv)
    n_ctx = (n_kv + 255) // 256 * 256
    G = H // HK
    # magnitudes over most of the f16 range, random signs: K rows and V values spanning
    # 2^-14 .. 2^14, q spanning 2^-6 .. 2^3; a few positions get large scores so the
    # probabilities spread from ~1 down to f16 subnormals
    def wide(shape, lo, hi):
        return (np.exp2(rng.uniform(lo, hi, shape)) * rng.choice([-1.0, 1.0], shape)).astype(np.float32)
    K = np.zeros((HK, n_ctx, D), np.float16)
    V = np.zeros((HK, D, n_ctx), np.float16)
    K[:, :n_kv, :] = _f16(wide((HK, n_kv, D), -14, 4) * 0.05)
    V[:, :, :n_kv] = _f16(wide((HK, D, n_kv), -14, 14))
    q = wide((H, D), -6, 3) * 0.5
    hot = rng.choice(n_kv, size=4, replace=False)
    for g in range(HK):
        for h in range(g * G, (g + 1) * G):
            for j, t in enumerate(hot):  # a few aligned keys: scores tens of units apart
                K[g, t, :] = _f16(np.sign(q[h]) * (0.5 + 0.25 * j) / max(1.0, np.abs(q[h]).mean()))
    out = torch.empty(H * D, dtype=torch.float32, device="cuda")
    qd, kd, vd = to_dev(q.reshape(-1)), to_dev(K.view(np.uint16).reshape(-1)), to_dev(V.view(np.uint16).reshape(-1))
    rc = llmi.lib().llmi_attention(H, HK, D, n_kv, n_ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), mode)
    assert rc == 0, llmi.last_error()
    got = out.cpu().numpy().reshape(H, D)
    want = _ref_attention(q, K, V, n_kv, G, 1.0 / np.sqrt(np.float32(D)))
    assert np.isfinite(want).all()
    bad = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} outputs differ, first {bad[:3].tolist()}: {got[tuple(bad[0])]} vs {want[tuple(bad[0])]}"
