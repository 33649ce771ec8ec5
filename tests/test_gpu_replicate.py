"""llmi_replicate argument checks on the device (SURVEY.md §8e fan-out): a device listed
twice, the source model's own device, or an out-of-range index is refused before any
allocation or RCCL communicator (one rank per GPU)."""
from __future__ import annotations

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))


@pytest.mark.gpu
def test_replicate_rejects_duplicate_and_bad_devices():
    import llmi

    m = llmi.Model(os.path.join(ROOT, "tests", "golden", "tiny-mixed.gguf"))
    try:
        n = llmi.device_count()
        for devs, msg in (([m.device], "listed twice"), ([n], "out of range"), ([-1], "out of range")):
            with pytest.raises(llmi.LlmiError) as e:
                m.replicate(devs)
            assert msg in str(e.value), (devs, str(e.value))
        if n >= 3:
            with pytest.raises(llmi.LlmiError):
                m.replicate([1, 1])
    finally:
        m.close()
