"""Diagnostic: per-step taps (last layer q / attention out / SwiGLU out / residual) of the
GPU decode path vs the oracle (device order), to locate the first divergent quantity."""
import ctypes as C
import os
import sys

sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch

torch.zeros(1, device="cuda")
import llmi
from llmi._lib import lib
import pyoracle as po

preset = sys.argv[1] if len(sys.argv) > 1 else "tiny-mixed-d128"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 37
n_layer = int(sys.argv[3]) if len(sys.argv) > 3 else 0
path = f"/tmp/{preset}-L{n_layer}.gguf"
llmi.write_synthetic_gguf(path, preset, seed=1, n_layer=n_layer)
rng = np.random.default_rng(11 + n)
prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
po.set_dot_order(po.DEVICE_ORDER)
om = po.OracleModel(path, n_ctx=128)
m = llmi.Model(path)
c = llmi.Context(m, n_ctx=128)
E, F, QD = m.n_embd, None, None
names = {2: "q", 3: "att", 4: "swiglu", 1: "x_final"}
for pos, t in enumerate(prompt):
    lo = om.decode(t, pos)
    assert c.decode([t], pos=[pos]) == 0
    lg = c.logits(-1)
    diffs = {}
    for w in (2, 3, 4, 1):
        size = {1: E}.get(w)
        ob = np.zeros(1 << 16, np.float32)
        gb = np.zeros(1 << 16, np.float32)
        po.lib().or_tap(om._h, w, ob.ctypes.data_as(C.c_void_p))
        assert lib().llmi_debug_tap(c._h, w, gb.ctypes.data_as(C.c_void_p)) == 0
        d = np.abs(ob - gb)
        diffs[names[w]] = (float(d.max()), int((d > 0).sum()))
    dl = float(np.abs(lg - lo).max())
    if dl > 0 or any(v[0] > 0 for v in diffs.values()):
        print("pos", pos, "tok", t, "logits", dl, diffs, flush=True)
        break
print("done; prompt", prompt)
