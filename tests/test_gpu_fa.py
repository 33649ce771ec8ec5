"""GPU parity in the flash-attention numerics (model numerics bit LLMI_NUMERICS_FA; VERDICT
r5 item 4): decode attention as upstream's CPU flash_attn_ext one_chunk
(online max / sum, f16 V accumulator rescaled on a new maximum, glibc expf), in both dot
associations, bit-identical to the oracle's OR_X86_FA mode (oracle/ggml_oracle.c
attn_head_fa).  The matvecs keep their association (generic or x86); prompts run as
decode steps (no batched prefill in this mode); batched steps run every slot's FA attention in one launch.

- every quant type and both head dims (tiny presets): 40 steps bit-identical, and
  different from the non-flash attention of the same association;
- the C2 trajectory at Llama-3-8B widths (2 layers, 128 -> 640) in both associations;
- a context past the one-launch kernels' sizes (1100 positions) at TinyLlama widths.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import llmi
import pyoracle as po

pytestmark = pytest.mark.gpu

ASSOC = {"generic": (llmi.NUMERICS_GENERIC, 0), "x86": (llmi.NUMERICS_X86, po.X86_ALL)}


@pytest.mark.parametrize("assoc", ["generic", "x86"])
@pytest.mark.parametrize("preset", ["tiny-mixed", "tiny-mixed-d128"])
def test_fa_tiny_decode_vs_oracle(gpu, tiny_models, preset, assoc):
    num, flags = ASSOC[assoc]
    path = tiny_models[preset]
    m = llmi.Model(path, numerics=num | llmi.NUMERICS_FA)
    assert m.numerics == num | llmi.NUMERICS_FA
    assert llmi.lib().llmi_prefill_supported(m._h) == 0
    c = llmi.Context(m, n_ctx=256)
    om = po.OracleModel(path, n_ctx=256, x86=flags | po.X86_FA)
    on = po.OracleModel(path, n_ctx=256, x86=flags)
    differs = False
    t = 1
    for pos in range(40):
        assert c.decode([t], pos=[pos]) == 0
        lg, lo, ln = c.logits(-1), om.decode(t, pos), on.decode(t, pos)
        assert np.array_equal(lg, lo), f"pos {pos}: max |d| {np.abs(lg - lo).max():.3g}"
        differs |= not np.array_equal(lo, ln)
        assert c.greedy(-1) == int(np.argmax(lo))
        t = int(np.argmax(lo))
    assert differs, "flash and non-flash attention gave identical logits (the mode is not exercised)"
    om.close(), on.close(), c.close(), m.close()


@pytest.mark.parametrize("assoc", ["generic", "x86"])
@pytest.mark.parametrize("preset,n_prompt,n_gen", [
    ("llama3-8b-q4km", 128, 512),   # C2: 128-token prompt -> 512-token decode (ctx 640)
    ("tinyllama-q8_0", 16, 1100),   # past the one-launch attention sizes
])
def test_fa_order_trajectory(gpu, synth_dir, preset, n_prompt, n_gen, assoc):
    """2 layers at the preset's widths in flash-attention numerics, in lockstep with the
    oracle: logits bit-identical at every step, the same greedy ids.  Reported into
    $LLMI_REPORT_DIR/parity_fa.jsonl."""
    num, flags = ASSOC[assoc]
    path = str(synth_dir / f"{preset}-L2-fa.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=2)
    rng = np.random.default_rng(21)
    prompt = [1] + [int(t) for t in rng.integers(3, 30000, n_prompt - 1)]
    n_ctx = (n_prompt + n_gen + 255) // 256 * 256
    om = po.OracleModel(path, n_ctx=n_ctx, x86=flags | po.X86_FA)
    m = llmi.Model(path, numerics=num | llmi.NUMERICS_FA)
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
        assert np.array_equal(lg, lo), f"{preset} {assoc} step {step} (pos {pos - 1}): max |d| {d:.3g}"
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
    rep = {"preset": preset, "numerics": f"{assoc}+fa", "oracle_flags": flags | po.X86_FA, "n_layer": 2,
           "prompt": n_prompt, "steps": len(diffs), "ctx_end": pos, "worst_abs_diff": max(diffs),
           "bit_identical": True, "ids_identical": True}
    print(json.dumps(rep))
    out_dir = os.environ.get("LLMI_REPORT_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "parity_fa.jsonl"), "a") as f:
            f.write(json.dumps(rep) + "\n")


def test_fa_batched_equals_single(gpu, tiny_models):
    """A flash-attention context with n_seq_max >= 2 advances its sequences through batched
    steps (matvecs batched, every slot's FA attention in one launch): each equals its own single-sequence
    decode (and that one equals the oracle: test_fa_tiny_decode_vs_oracle)."""
    path = tiny_models["tiny-mixed-d128"]
    m = llmi.Model(path, numerics=llmi.NUMERICS_FA)
    c = llmi.Context(m, n_ctx=128, n_seq=3)
    got = c.generate_greedy_batch([0, 1, 2], [5, 9, 11], [0, 0, 0], 12)
    c1 = llmi.Context(m, n_ctx=128)
    for k, first in enumerate((5, 9, 11)):
        c1.kv_clear()
        assert c1.generate_greedy(first, 0, 12) == got[k]
    c.close(), c1.close(), m.close()
