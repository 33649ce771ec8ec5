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


@pytest.mark.gpu
def test_bmm_on_replica_device(synth_dir, monkeypatch):
    """k_bmm (8 sequences, matrix-core batched matvec) on a REPLICA's device: the occupancy
    cache and the dynamic-LDS attribute are per device (batch.hip bmm_cap), so a second
    device's first k_bmm launch is sized and attributed for that device.  Tokens equal the
    same sequences decoded one by one on device 0.  Needs two GPUs."""
    import numpy as np
    import llmi

    if llmi.device_count() < 2:
        pytest.skip("one GPU: no replica device")
    monkeypatch.setenv("LLMI_BMM_MIN", "1")
    path = str(synth_dir / "llama3-8b-q4km-batch-L2.gguf")
    llmi.write_synthetic_gguf(path, "llama3-8b-q4km", seed=11, n_layer=2)
    rng = np.random.default_rng(9)
    prompts = [[1] + [int(t) for t in rng.integers(3, 30000, int(rng.integers(2, 24)))] for _ in range(8)]
    m = llmi.Model(path)
    want = []
    for p in prompts:
        c = llmi.Context(m, n_ctx=256)
        assert c.decode(p) == 0
        f = c.greedy(-1)
        want.append([f] + c.generate_greedy(f, len(p), 8))
        c.close()
    (r,) = m.replicate([1])
    c = llmi.Context(r, n_ctx=256, n_seq=8)
    firsts = []
    for s, p in enumerate(prompts):
        assert c.decode(p, seq=[s] * len(p)) == 0
        firsts.append(c.greedy(-1))
    got = c.generate_greedy_batch(list(range(8)), firsts, [len(p) for p in prompts], 8)
    c.close()
    r.close()
    m.close()
    for s in range(8):
        assert [firsts[s]] + got[s] == want[s], f"seq {s}"
