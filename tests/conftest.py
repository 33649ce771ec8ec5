"""Shared fixtures.  `-m gpu` tests need a real MI355X (run through gpurun); the rest
run on CPU.  GPU tests FAIL (not skip) when no device is visible, so a silent skip
can never masquerade as parity."""
from __future__ import annotations

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "llama-gguf-inference_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU; run via gpurun")
    config.addinivalue_line("markers", "slow: full-size (BASELINE.json config) checks")


@pytest.fixture(scope="session")
def synth_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("gguf")


@pytest.fixture(scope="session")
def tiny_models(synth_dir):
    """The two tiny mixed-type models (all four quant types, head_dim 64 and 128)."""
    import llmi

    out = {}
    for preset in ("tiny-mixed", "tiny-mixed-d128"):
        path = str(synth_dir / f"{preset}.gguf")
        llmi.write_synthetic_gguf(path, preset, seed=1)
        out[preset] = path
    return out


@pytest.fixture(scope="session")
def gpu():
    import torch

    assert torch.cuda.is_available(), "gpu-marked test needs a visible HIP device"
    import pyoracle

    pyoracle.prefer_simd()  # bit-identical to the -O2 build (tests/test_oracle_simd.py), faster
    torch.zeros(1, device="cuda")  # initialise torch's HIP state before any libllmi call
    import llmi

    assert llmi.device_count() > 0
    return torch.device("cuda:0")


def pytest_sessionstart(session):
    """LLMI_TEST_OPTIONS="name=value,...": set libllmi test options (A/B launch knobs,
    every value bit-identical) for the whole session, e.g. to run the parity tests under
    a non-default kernel configuration."""
    opts = os.environ.get("LLMI_TEST_OPTIONS")
    if not opts:
        return
    import llmi

    for kv in opts.split(","):
        name, value = kv.split("=")
        llmi.test_option(name.strip(), int(value))
