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


@pytest.mark.gpu
def test_pipelined_loaders_single_device_equal_plain_load():
    """llmi_model_load_fanout at one rank and llmi_model_load_replicated with no replica
    take the same upload path (model_upload) as llama_model_load_from_file: a decode on
    each gives bit-identical logits and greedy tokens.  (The RCCL pieces themselves need
    two GPUs: unmeasured on this box.)"""
    import numpy as np
    import llmi

    path = os.path.join(ROOT, "tests", "golden", "tiny-mixed.gguf")
    prompt = [1, 50, 30, 7, 99, 100, 42]
    outs = []
    for load in (lambda: llmi.Model(path), lambda: llmi.Model.load_fanout(path, 0, b"\0" * 128, 1, 0),
                 lambda: llmi.Model.load_replicated(path, 0, [])[0]):
        m = load()
        c = llmi.Context(m, n_ctx=256)
        assert c.decode(prompt) == 0
        lg = c.logits(-1)
        first = c.greedy(-1)
        outs.append((lg, [first] + c.generate_greedy(first, len(prompt), 8)))
        c.close()
        m.close()
    for lg, toks in outs[1:]:
        assert np.array_equal(lg, outs[0][0]) and toks == outs[0][1]
