"""GPU parity of the hot-path kernels against the CPU oracle.

- activation quantization (the matvec prologue, RMSNorm fused): BIT-EXACT vs
  quantize_row_q8_K_ref / quantize_row_q8_0_ref, incl. edge cases (all-zero block,
  +/- ties for the signed max, .5 rounding boundaries, tiny/huge magnitudes);
- quantized matvec per type: BIT-EXACT against the oracle, which restates ggml's
  generic scalar vec_dot (same integer block sums, the same fp32 operations in the same
  order: per-residue chains sums[l], the min chain, then sumf += sums[l]);
- the load-time repack is checked through the matvec and through get_rows elsewhere.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import pyoracle as po
from helpers import Q4_K, Q5_K, Q6_K, Q8_0, QTYPES, TNAME, empty_dev, random_blocks, to_dev

pytestmark = pytest.mark.gpu


def _lib():
    from llmi._lib import lib

    return lib()


def _p(t):
    return C.c_void_p(t.data_ptr())


def gpu_quant(qtype, x, nw=None, eps=1e-5):
    import torch

    cols = x.size
    nbytes = cols // 256 * 292 if qtype != Q8_0 else cols // 32 * 34
    out = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    xd = to_dev(x.astype(np.float32))
    nd = to_dev(nw.astype(np.float32)) if nw is not None else None
    torch.cuda.synchronize()
    rc = _lib().llmi_quantize_act(qtype, cols, _p(xd), _p(nd) if nd is not None else None, eps, _p(out))
    assert rc == 0
    return out.cpu().numpy()


def edge_inputs(cols, rng):
    xs = []
    x = rng.standard_normal(cols).astype(np.float32)
    xs.append(("normal", x))
    z = x.copy()
    z[:256] = 0.0  # all-zero Q8_K block (d = 0 path)
    xs.append(("zero_block", z))
    t = rng.standard_normal(cols).astype(np.float32) * 0.5
    t[3], t[200] = -2.0, 2.0  # equal |max| with opposite signs: first one (negative) wins
    if cols >= 512:
        t[256 + 7], t[256 + 9] = 3.0, -3.0
    xs.append(("ties", t))
    # values whose scaled image lands exactly on .5: -127/max * x = k + 0.5
    h = np.zeros(cols, dtype=np.float32)
    h[0] = -127.0
    h[1:64] = np.arange(1, 64, dtype=np.float32) + 0.5
    h[64:] = rng.uniform(-100, 100, cols - 64).astype(np.float32)
    xs.append(("half_boundaries", h))
    xs.append(("tiny", (rng.standard_normal(cols) * 1e-30).astype(np.float32)))
    xs.append(("huge", (rng.standard_normal(cols) * 1e30).astype(np.float32)))
    return xs


@pytest.mark.parametrize("qtype", [Q4_K, Q8_0], ids=["q8_K", "q8_0"])
@pytest.mark.parametrize("cols", [256, 4096, 14336])
def test_activation_quant_bitexact(gpu, qtype, cols):
    rng = np.random.default_rng(cols)
    for name, x in edge_inputs(cols, rng):
        ref = po.quantize_act(qtype, x)
        got = gpu_quant(qtype, x)
        assert np.array_equal(ref, got), f"{name}: quantized activation differs"


@pytest.mark.parametrize("qtype", [Q4_K, Q8_0], ids=["q8_K", "q8_0"])
@pytest.mark.parametrize("cols", [512, 4096])
def test_rmsnorm_quant_bitexact(gpu, qtype, cols):
    rng = np.random.default_rng(7 + cols)
    x = (rng.standard_normal(cols) * 3).astype(np.float32)
    w = rng.uniform(0.5, 1.5, cols).astype(np.float32)
    y = po.rms_norm_mul(x, w, 1e-5)
    ref = po.quantize_act(qtype, y)
    got = gpu_quant(qtype, x, w, 1e-5)
    assert np.array_equal(ref, got)


def gpu_matvec(qtype, raw, rows, cols, x, nw=None, eps=1e-5):
    import torch

    L = _lib()
    nbytes = L.llmi_device_layout_bytes(qtype, rows, cols)
    assert nbytes > 0
    rd = to_dev(raw)
    wd = empty_dev(nbytes)
    torch.cuda.synchronize()
    assert L.llmi_repack(qtype, _p(rd), _p(wd), rows, cols) == 0
    xd = to_dev(x.astype(np.float32))
    nd = to_dev(nw.astype(np.float32)) if nw is not None else None
    yd = torch.zeros(rows, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    assert L.llmi_matvec(qtype, _p(wd), rows, cols, _p(xd), _p(nd) if nd is not None else None, eps, _p(yd), 0) == 0
    return yd.cpu().numpy()


# cols > 4096 take the K-split kernel (KS=2 below 6 items per row, KS=1 from 6 items when
# its part buffer fits LDS; 28672 also exercises the prologue's tail loop beyond the
# register-held sub-blocks)
SHAPES = [(2, 256), (7, 512), (130, 1024), (1024, 4096), (333, 14336), (4096, 4096), (64, 8192), (130, 5632),
          (5, 28672), (2048, 14336)]


@pytest.mark.parametrize("qtype", QTYPES, ids=[TNAME[t] for t in QTYPES])
@pytest.mark.parametrize("rows,cols", SHAPES)
def test_matvec_vs_oracle(gpu, qtype, rows, cols):
    rng = np.random.default_rng(rows * 131 + cols + qtype)
    raw = random_blocks(qtype, rows, cols, rng)
    x = rng.standard_normal(cols).astype(np.float32)
    got = gpu_matvec(qtype, raw, rows, cols, x)
    ref = po.matvec(qtype, raw, rows, cols, x)
    err = float(np.abs(got - ref).max())
    assert np.array_equal(got, ref), f"not bit-exact vs the generic-order oracle (max |err| {err:.3g})"


@pytest.mark.parametrize("qtype", [12, 14], ids=["q4_K", "q6_K"])
def test_matvec_ks1_multi_round(gpu, qtype):
    """K-split width 1 past one round: 4224 pairs of 28672-column rows exceed the 16 pair
    slots x 256 resident workgroups, so slots take a second round and the double-buffered
    fold buffer is reused; bit-exact vs the generic-order oracle."""
    rows, cols = 8448, 28672
    rng = np.random.default_rng(91 + qtype)
    raw = random_blocks(qtype, rows, cols, rng)
    x = rng.standard_normal(cols).astype(np.float32)
    got = gpu_matvec(qtype, raw, rows, cols, x)
    exact = po.matvec(qtype, raw, rows, cols, x)
    assert np.array_equal(got, exact), "not bit-exact vs the generic-order oracle"


@pytest.mark.parametrize("qtype", QTYPES, ids=[TNAME[t] for t in QTYPES])
@pytest.mark.parametrize("rows,cols", [(96, 2048), (70, 8192)])
def test_matvec_fused_rmsnorm(gpu, qtype, rows, cols):
    rng = np.random.default_rng(11 + qtype)
    raw = random_blocks(qtype, rows, cols, rng)
    x = (rng.standard_normal(cols) * 4).astype(np.float32)
    w = rng.uniform(0.8, 1.2, cols).astype(np.float32)
    ref = po.matvec(qtype, raw, rows, cols, po.rms_norm_mul(x, w, 1e-5))
    got = gpu_matvec(qtype, raw, rows, cols, x, w, 1e-5)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("qtype", QTYPES, ids=[TNAME[t] for t in QTYPES])
def test_matvec_linearity_full_size(gpu, qtype):
    """Size-independent property at the Llama-3-8B ffn_gate shape (14336 x 4096): the
    matvec of an exactly-representable activation is linear in the weight scales —
    doubling every fp16 d (and dmin) doubles y exactly."""
    rows, cols = 14336, 4096
    rng = np.random.default_rng(5)
    raw = random_blocks(qtype, rows, cols, rng)
    x = rng.standard_normal(cols).astype(np.float32)
    y1 = gpu_matvec(qtype, raw, rows, cols, x)
    r2 = raw.reshape(-1, {Q4_K: 144, Q5_K: 176, Q6_K: 210, Q8_0: 34}[qtype]).copy()
    sl = {Q4_K: [slice(0, 2), slice(2, 4)], Q5_K: [slice(0, 2), slice(2, 4)], Q6_K: [slice(208, 210)],
          Q8_0: [slice(0, 2)]}[qtype]
    for s in sl:
        v = r2[:, s].copy().view(np.float16).astype(np.float32) * 2
        r2[:, s] = v.astype(np.float16).view(np.uint8).reshape(-1, 2)
    y2 = gpu_matvec(qtype, r2.reshape(-1), rows, cols, x)
    assert np.array_equal(y2, 2 * y1)
    # and a sampled subset against the oracle at full size
    idx = np.sort(rng.choice(rows, 64, replace=False))
    bpr = cols // {Q4_K: 256, Q5_K: 256, Q6_K: 256, Q8_0: 32}[qtype] * {Q4_K: 144, Q5_K: 176, Q6_K: 210, Q8_0: 34}[qtype]
    sub = raw.reshape(rows, bpr)[idx].reshape(-1)
    ref = po.matvec(qtype, sub, len(idx), cols, x)
    assert np.array_equal(y1[idx], ref)
