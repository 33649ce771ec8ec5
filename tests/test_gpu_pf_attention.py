"""Batched-prefill attention at kernel level (llmi_pf_attention):
T query tokens at positions pos0.. attend causally to the f16 caches, and every path --
the tiled FP64-MFMA kernel k_pf_fa (mode 0), the grouped LDS kernel (1) and one head per
workgroup (2) -- equals a NumPy restatement of oracle/ggml_oracle.c attn_head bit for
bit: q rounded to f16; kq = sequential double sum of the exact f16 products; w = (float)kq
* scale; e = llmi_expf(w - max); S = double sum; p = f16(e * (float)(1/S)); out =
sequential double sum over the positions of the exact v * p products.

The data spans most of the f16 range (K and V values 2^-14 .. 2^14, q 2^-6 .. 2^3, a few
aligned keys per head so the probabilities run from ~1 down to f16 subnormals), the
shapes cover every GQA group k_pf_fa takes (1, 2, 4, 8) at head_dim 64 and 128, ragged
token counts (not a multiple of the 64 / G tokens of a tile), prompts starting mid-cache
(pos0 > 0, key tiles with partly live rows), and a scratch bound that forces one query
tile per launch.  Stale cache contents past the last live position are NaN here, so a
kernel that lets them meet a zero probability fails.
"""
from __future__ import annotations

import numpy as np
import pytest

import llmi
import pyoracle as po

pytestmark = pytest.mark.gpu

F32 = np.float32


def expf_np(x: np.ndarray) -> np.ndarray:
    """include/llmi_math.h llmi_expf, vectorized (float32 ops, one rounding each)."""
    x = np.asarray(x, F32)
    with np.errstate(over="ignore", invalid="ignore", under="ignore"):
        t = x * F32(1.44269502162933349609375)
        nf = (t + F32(12582912.0)) - F32(12582912.0)
        n = np.where(np.isfinite(nf), nf, 0).astype(np.int64)
        r = x - nf * F32(0.693359375)
        r = r - nf * F32(-2.12194440e-4)
        p = np.full_like(x, F32(1.98412698e-4))
        for c in (1.38888889e-3, 8.33333333e-3, 4.16666667e-2, 1.66666667e-1, 0.5, 1.0, 1.0):
            p = p * r + F32(c)
        big = n > 127
        p = np.where(big, p * F32(2.0), p)
        n = np.where(big, n - 1, n)
        small = n < -126
        nn = np.where(small, n + 126 + 127, n + 127).clip(0, 255).astype(np.uint32)
        sc = (nn << np.uint32(23)).view(F32)
        out = np.where(small, (p * sc) * F32(1.17549435e-38), p * sc)
        out = np.where(x < F32(-103.97208404541015625), F32(0.0), out)
        out = np.where(x > F32(88.72283935546875), F32(np.inf), out)
        out = np.where(np.isnan(x), x, out)
    return out.astype(F32)


def _f16(a):
    return np.asarray(a, dtype=F32).astype(np.float16)


def ref_pf_attention(q, K, V, pos0, G, scale):
    """q [T][H][D] f32; K [HK][n_ctx][D] f16; V [HK][D][n_ctx] f16 -> out [T][H][D]."""
    T, H, D = q.shape
    nkv = pos0 + T
    live = np.arange(nkv)[None, :] < (pos0 + np.arange(T) + 1)[:, None]  # [T][nkv]
    out = np.empty((T, H, D), F32)
    qf = _f16(q).astype(np.float64)
    for h in range(H):
        g = h // G
        k = K[g, :nkv, :].astype(np.float64)                               # [nkv][D]
        kq = np.cumsum(qf[:, h, None, :] * k[None, :, :], axis=2)[:, :, -1]  # [T][nkv], sequential over d
        w = kq.astype(F32) * F32(scale)
        mx = np.where(live, w, F32(-np.inf)).max(axis=1)
        e = np.where(live, expf_np(w - mx[:, None]), F32(0.0))
        s = np.cumsum(e.astype(np.float64), axis=1)[:, -1]
        inv = (1.0 / s).astype(F32)
        p = _f16(e * inv[:, None]).astype(np.float64)                      # [T][nkv]
        v = V[g, :, :nkv].astype(np.float64)                               # [D][nkv]
        out[:, h, :] = np.cumsum(p[:, None, :] * v[None, :, :], axis=2)[:, :, -1].astype(F32)
    return out


def _case(H, HK, D, T, pos0, seed):
    rng = np.random.default_rng(seed)
    nkv = pos0 + T
    n_ctx = (nkv + 64 + 255) // 256 * 256
    G = H // HK

    def wide(shape, lo, hi):
        return (np.exp2(rng.uniform(lo, hi, shape)) * rng.choice([-1.0, 1.0], shape)).astype(F32)

    K = np.full((HK, n_ctx, D), np.nan, np.float16)   # stale positions: NaN
    V = np.full((HK, D, n_ctx), np.nan, np.float16)
    K[:, :nkv, :] = _f16(wide((HK, nkv, D), -14, 4) * 0.05)
    V[:, :, :nkv] = _f16(wide((HK, D, nkv), -14, 14))
    q = wide((T, H, D), -6, 3) * F32(0.5)
    hot = rng.choice(nkv, size=min(6, nkv), replace=False)
    for g in range(HK):
        for j, t in enumerate(hot):  # aligned keys: scores tens of units apart
            h = g * G + j % G
            K[g, t, :] = _f16(np.sign(q[-1, h]) * (0.5 + 0.25 * j) / max(1.0, np.abs(q[-1, h]).mean()))
    return q, K, V, n_ctx, G


def _run(q, K, V, n_ctx, HK, pos0, mode, scratch=0):
    import torch
    from helpers import to_dev

    T, H, D = q.shape
    out = torch.full((T * H * D,), float("nan"), dtype=torch.float32, device="cuda")
    qd = to_dev(np.ascontiguousarray(q.reshape(-1)))
    kd = to_dev(K.view(np.uint16).reshape(-1))
    vd = to_dev(V.view(np.uint16).reshape(-1))
    us = llmi.lib().llmi_pf_attention(H, HK, D, T, pos0, n_ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(),
                                      out.data_ptr(), mode, scratch)
    assert us >= 0, llmi.last_error()
    return out.cpu().numpy().reshape(T, H, D)


def _assert_same(got, want, where):
    assert np.isfinite(want).all()
    bad = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, (f"{where}: {len(bad)} outputs differ, first {bad[:3].tolist()}: "
                           f"{got[tuple(bad[0])]} vs {want[tuple(bad[0])]}")


def test_expf_np_matches_the_oracle():
    xs = np.concatenate([np.linspace(-110.0, 0.0, 4001), np.linspace(0.0, 90.0, 601),
                         [-103.9, -87.5, -87.3, -0.0, 1e-30]]).astype(F32)
    want = np.array([po.expf(float(x)) for x in xs], dtype=F32)
    got = expf_np(xs)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("H,HK,D,T,pos0", [
    (32, 8, 128, 64, 0),      # Llama-3 / Mistral heads, the first ubatch
    (32, 8, 128, 37, 700),    # ragged, mid-cache
    (32, 4, 64, 40, 300),     # TinyLlama heads (G = 8)
    (64, 8, 128, 24, 500),    # 70B heads (G = 8)
    (16, 8, 128, 21, 260),    # G = 2
    (8, 8, 64, 70, 130),      # G = 1 (two query tiles, the second ragged)
])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_pf_attention_bit_identical(gpu, H, HK, D, T, pos0, mode):
    q, K, V, n_ctx, G = _case(H, HK, D, T, pos0, seed=97 * T + pos0 + mode)
    got = _run(q, K, V, n_ctx, HK, pos0, mode)
    want = ref_pf_attention(q, K, V, pos0, G, 1.0 / np.sqrt(F32(D)))
    _assert_same(got, want, f"mode {mode}")


def test_pf_attention_chunked_scratch(gpu):
    """A scratch of one query tile's rows: k_pf_fa runs one tile per launch, same bits."""
    H, HK, D, T, pos0 = 32, 8, 128, 48, 900
    q, K, V, n_ctx, G = _case(H, HK, D, T, pos0, seed=5)
    ldw = (pos0 + T + 63) // 64 * 64
    one_tile = HK * 64 * ldw * 4
    got = _run(q, K, V, n_ctx, HK, pos0, 0, scratch=one_tile)
    whole = _run(q, K, V, n_ctx, HK, pos0, 0)
    want = ref_pf_attention(q, K, V, pos0, G, 1.0 / np.sqrt(F32(D)))
    _assert_same(got, want, "one tile per launch")
    _assert_same(whole, want, "one launch")


def test_pf_attention_tiled_mode_never_falls_back(gpu):
    """Mode 0 asks for k_pf_fa alone: a scratch shorter than one query tile is an error,
    not a silent run of the LDS kernels."""
    import torch

    H, HK, D, T, pos0 = 32, 8, 128, 48, 900
    q, K, V, n_ctx, G = _case(H, HK, D, T, pos0, seed=6)
    ldw = (pos0 + T + 63) // 64 * 64
    out = torch.zeros(T * H * D, dtype=torch.float32, device="cuda")
    from helpers import to_dev
    qd = to_dev(np.ascontiguousarray(q.reshape(-1)))
    kd = to_dev(K.view(np.uint16).reshape(-1))
    vd = to_dev(V.view(np.uint16).reshape(-1))
    rc = llmi.lib().llmi_pf_attention(H, HK, D, T, pos0, n_ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(),
                                      out.data_ptr(), 0, HK * 64 * ldw * 4 // 2)
    assert rc < 0 and "not supported" in llmi.last_error().lower()


def test_pf_attention_rejects_bad_shapes(gpu):
    L = llmi.lib()
    assert L.llmi_pf_attention(32, 8, 96, 16, 0, 256, 1, 1, 1, 1, 0, 0) < 0   # head_dim
    assert L.llmi_pf_attention(32, 8, 128, 16, 250, 256, 1, 1, 1, 1, 0, 0) < 0  # past n_ctx
    assert L.llmi_pf_attention(24, 8, 128, 16, 0, 256, 1, 1, 1, 1, 0, 0) < 0   # G = 3: no tiled kernel


@pytest.mark.parametrize("cfg", [410, 420, 421, 441, 220, 221, 241])
@pytest.mark.parametrize("H,HK,D,T,pos0", [(32, 8, 128, 37, 700), (32, 4, 64, 40, 300), (8, 8, 64, 70, 130)])
def test_pf_attention_kernel_configurations(gpu, cfg, H, HK, D, T, pos0):
    """k_pf_fa's other configurations (row blocks per workgroup, waves per block, e kept
    from pass 2 or taken again; prefill.hip.inc pf_fa_launch): the same bits."""
    L = llmi.lib()
    old = L.llmi_test_option(b"pf_fa_cfg", cfg)
    try:
        q, K, V, n_ctx, G = _case(H, HK, D, T, pos0, seed=11 * T + pos0 + cfg)
        got = _run(q, K, V, n_ctx, HK, pos0, 0)
    finally:
        L.llmi_test_option(b"pf_fa_cfg", old)
    _assert_same(got, ref_pf_attention(q, K, V, pos0, G, 1.0 / np.sqrt(F32(D))), f"cfg {cfg}")
