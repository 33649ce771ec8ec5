"""Diagnostic: prefill vs decode steps vs oracle on one tiny preset, per attention mode."""
import os, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi
import pyoracle as po

path = "/tmp/d128.gguf"
preset = sys.argv[1] if len(sys.argv) > 1 else "tiny-mixed-d128"
llmi.write_synthetic_gguf(path, preset, seed=1)
for n in (3, 9, 17, 33, 37):
    rng = np.random.default_rng(11 + n)
    prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
    po.set_dot_order(po.DEVICE_ORDER)
    om = po.OracleModel(path, n_ctx=128)
    for pos, t in enumerate(prompt):
        lo = om.decode(t, pos)
    res = {}
    for mode in ("0", "1", "2"):
        for npf in ("0", "1"):
            os.environ["LLMI_ATTN_MODE"] = mode
            os.environ["LLMI_NO_PREFILL"] = npf
            m = llmi.Model(path)
            c = llmi.Context(m, n_ctx=128)
            assert c.decode(prompt) == 0
            lg = c.logits(-1)
            res[(mode, npf)] = float(np.abs(lg - lo).max())
            c.close(); m.close()
    print(n, res, flush=True)
