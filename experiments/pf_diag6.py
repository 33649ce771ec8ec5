"""Diagnostic: long prompt, GPU paths (prefill, decode steps per attention mode) vs the oracle."""
import os, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi
import pyoracle as po

preset = sys.argv[1] if len(sys.argv) > 1 else "tiny-mixed"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 500
path = f"/tmp/{preset}.gguf"
llmi.write_synthetic_gguf(path, preset, seed=1)
rng = np.random.default_rng(9)
prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
po.set_dot_order(po.DEVICE_ORDER)
om = po.OracleModel(path, n_ctx=768)
for pos, t in enumerate(prompt):
    lo = om.decode(t, pos)
res = {}
for key, npf, mode in (("prefill", "0", "0"), ("steps-fused", "1", "1"), ("steps-split", "1", "2"),
                       ("steps-2k", "1", "3"), ("steps-x", "1", "4")):
    os.environ["LLMI_NO_PREFILL"] = npf
    os.environ["LLMI_ATTN_MODE"] = mode
    m = llmi.Model(path); c = llmi.Context(m, n_ctx=768)
    assert c.decode(prompt) == 0
    res[key] = float(np.abs(c.logits(-1) - lo).max()); c.close(); m.close()
print(preset, n, "vs oracle:", res, flush=True)
