"""Matvec microbenchmark: rotating over >= 1 GB of distinct weight copies (defeats the
256 MB Infinity Cache); reports GB/s of algorithmic bytes per launch, next to a
perfectly coalesced streaming read of the same byte count."""
import ctypes as C, os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
from llmi._lib import lib
from helpers import random_blocks, Q4_K, Q5_K, Q6_K, Q8_0
L = lib()
P = lambda t: C.c_void_p(t.data_ptr())
res = {}
shapes = [(Q4_K, 28672, 4096), (Q4_K, 4096, 14336), (Q6_K, 4096, 14336), (Q6_K, 128256, 4096), (Q4_K, 6144, 4096),
          (Q5_K, 14336, 4096), (Q8_0, 5632, 2048)]
if os.environ.get("MV_SHAPES"):  # e.g. "12:28672x4096,14:128256x4096"
    shapes = []
    for tok in os.environ["MV_SHAPES"].split(","):
        t, rc = tok.split(":"); r, c = rc.split("x")
        shapes.append((int(t), int(r), int(c)))
REPS = int(os.environ.get("MV_REPS", "200"))
MODE = int(os.environ.get("MV_MODE", "0"))  # bit0 fused RMSNorm, bit1 logits epilogue
rng = np.random.default_rng(0)
for qt, rows, cols in shapes:
    lb = L.llmi_device_layout_bytes(qt, rows, cols)
    stride = (lb + 4095) // 4096 * 4096
    n = int(os.environ.get("MV_NCOPIES", "0")) or max(2, int(np.ceil(1.2e9 / stride)))
    raw = torch.from_numpy(random_blocks(qt, rows, cols, rng)).cuda()
    w = torch.empty(stride * n, dtype=torch.uint8, device="cuda")
    for k in range(n):
        assert L.llmi_repack(qt, P(raw), C.c_void_p(w.data_ptr() + stride * k), rows, cols) == 0
    x = torch.randn(cols, device="cuda"); y = torch.empty(rows, device="cuda")
    torch.cuda.synchronize()
    us = L.llmi_bench_matvec_ex(qt, P(w), n, rows, cols, P(x), P(y), REPS, MODE)
    alg = raw.numel()
    us_s = L.llmi_bench_stream(P(w), n, stride, alg, REPS, 2048)
    key = f"{qt}:{rows}x{cols}"
    res[key] = {"us": us, "GBps": alg / us / 1e3, "stream_us": us_s, "stream_GBps": alg / us_s / 1e3}
    print(key, json.dumps(res[key]), flush=True)
    del w, raw
print(json.dumps(res))
