"""Diagnostic: first decode step where GPU logits leave the oracle's (device order)."""
import os, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi
import pyoracle as po

path = "/tmp/d128.gguf"
llmi.write_synthetic_gguf(path, "tiny-mixed-d128", seed=1)
n = 37
rng = np.random.default_rng(11 + n)
prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
po.set_dot_order(po.DEVICE_ORDER)
om = po.OracleModel(path, n_ctx=128)
m = llmi.Model(path)
c = llmi.Context(m, n_ctx=128)
for pos, t in enumerate(prompt):
    lo = om.decode(t, pos)
    assert c.decode([t], pos=[pos]) == 0
    lg = c.logits(-1)
    d = np.abs(lg - lo)
    if d.max() > 0:
        print("pos", pos, "tok", t, "max", d.max(), "n_diff", int((d > 0).sum()), flush=True)
        e_g = np.zeros(m.n_embd, np.float32)
print("prompt", prompt)
