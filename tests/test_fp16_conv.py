"""fp32 -> fp16 rounding: the oracle's llmi_f2h (include/llmi_math.h, software RNE with
subnormals) equals IEEE round-to-nearest-even (numpy) over every fp32 exponent, the
f16 subnormal range and exact ties; on the GPU the hardware conversion (v_cvt_f16_f32,
used by the attention kernels for q and p) equals it too."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import pyoracle as po


def sample_floats(n=1 << 18, seed=0):
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    x = x[np.isfinite(x)]
    # exact ties and near-ties around f16 rounding points, normal and subnormal
    h = rng.integers(0, 0x7c00, 1 << 14, dtype=np.uint32).astype(np.uint16).view(np.float16).astype(np.float32)
    hn = np.nextafter(h.astype(np.float16), np.float16(np.inf)).astype(np.float32)
    mid = (h.astype(np.float64) + hn.astype(np.float64)) / 2
    ties = mid.astype(np.float32)
    sub = (rng.uniform(0, 6.2e-5, 1 << 14)).astype(np.float32)
    return np.concatenate([x, ties, np.nextafter(ties, np.float32(0)), np.nextafter(ties, np.float32(1)),
                           -ties, sub, -sub, np.float32([0.0, -0.0, 65504, 65519.99, 65520, 1e-8, 5.96e-8, 2.98e-8])])


def test_oracle_f2h_is_ieee_rne():
    x = sample_floats()
    f = po.lib().or_fp32_to_fp16
    got = np.array([f(C.c_float(v)) for v in x[:60000]], dtype=np.uint16)
    want = x[:60000].astype(np.float16).view(np.uint16)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_hw_conversion_is_ieee_rne(gpu):
    import torch

    x = sample_floats(1 << 22, seed=1)
    got = torch.from_numpy(x).cuda().half().cpu().numpy().view(np.uint16)
    want = x.astype(np.float16).view(np.uint16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, e.g. {x[bad[:5]]}"
