"""Diagnostic: GPU fused RMSNorm+q8_K quantization vs the oracle (generic and device-order norm sums)."""
import ctypes as C, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
from llmi._lib import lib
import pyoracle as po
from helpers import to_dev

L = lib()
rng = np.random.default_rng(0)
bad = {"seq": 0, "dev": 0, "both": 0}
N = 3000
for it in range(N):
    cols = 512
    x = (rng.standard_normal(cols) * rng.choice([0.01, 1.0, 30.0, 1000.0])).astype(np.float32)
    if it % 3 == 0:
        x[rng.integers(0, cols, 4)] *= 50
    w = rng.uniform(0.2, 2.0, cols).astype(np.float32)
    xd, wd = to_dev(x), to_dev(w)
    out = torch.zeros(cols // 256 * 292, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert L.llmi_quantize_act(12, cols, C.c_void_p(xd.data_ptr()), C.c_void_p(wd.data_ptr()), 1e-5, C.c_void_p(out.data_ptr())) == 0
    g = out.cpu().numpy()
    res = []
    for mode in (po.GENERIC, po.DEVICE_ORDER):
        po.set_dot_order(mode)
        y = po.rms_norm_mul(x, w, 1e-5)
        res.append(np.array_equal(po.quantize_q8_K(y), g))
    po.set_dot_order(po.GENERIC)
    if not res[0]: bad["seq"] += 1
    if not res[1]: bad["dev"] += 1
    if not res[0] and not res[1]: bad["both"] += 1
print("mismatches over", N, bad)
