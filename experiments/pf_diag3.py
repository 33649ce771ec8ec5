"""Diagnostic: d128 prompts, prefill vs steps vs oracle (first divergent decode step)."""
import os, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi
import pyoracle as po

path = "/tmp/d128.gguf"
llmi.write_synthetic_gguf(path, "tiny-mixed-d128", seed=1)
for n in (37, 70):
    rng = np.random.default_rng(11 + n)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
    res = []
    for npf in ("0", "1"):
        os.environ["LLMI_NO_PREFILL"] = npf
        m = llmi.Model(path); c = llmi.Context(m, n_ctx=128)
        assert c.decode(prompt) == 0
        res.append(c.logits(-1)); c.close(); m.close()
    print(n, "prefill vs steps max|d|", float(np.abs(res[0] - res[1]).max()), flush=True)
    po.set_dot_order(po.DEVICE_ORDER)
    om = po.OracleModel(path, n_ctx=128)
    m = llmi.Model(path); c = llmi.Context(m, n_ctx=128)
    first = None
    for pos, t in enumerate(prompt):
        lo = om.decode(t, pos)
        assert c.decode([t], pos=[pos]) == 0
        d = float(np.abs(c.logits(-1) - lo).max())
        if d > 0 and first is None:
            first = (pos, t, d)
    print(n, "first decode-vs-oracle divergence", first, flush=True)
