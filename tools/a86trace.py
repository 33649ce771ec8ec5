"""Per-workgroup timeline of the x86 one-launch decode attention (attn86.hip k_a86_h; needs a
-DLLMI_EXP_TRACE build via LLMI_LIB).  Stamps (s_memrealtime, 10 ns) per workgroup: entry,
V and q issued, scores + max done, exp sum done, probabilities in LDS, exit.
Env ATT_KV, ATT_SHAPE (H,HK,D)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import llmi  # noqa: E402
from llmi._lib import lib  # noqa: E402

L = lib()
H, HK, D = (int(v) for v in os.environ.get("ATT_SHAPE", "32,8,128").split(","))
old = llmi.test_option("numerics", 1)
names = ["V, q issued", "scores + max", "exp sum", "p in LDS", "PV + store"]
for n in [int(v) for v in os.environ.get("ATT_KV", "160,384,640").split(",")]:
    tr = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    assert L.llmi_bench_attention(H, HK, D, n, 0, 1, C.c_void_p(tr.data_ptr())) == 0, llmi.last_error()
    t = tr.cpu().numpy().reshape(4096, 8)
    t = t[t[:, 0] != 0][:, :6]
    t0 = t[:, 0].min()

    def q(a):
        return " ".join(f"{np.percentile(a, x) * 10 / 1000:6.2f}" for x in (0, 50, 100))

    print(f"== x86 H{H} HK{HK} D{D} n_kv {n}: workgroups {len(t)}; us (min/median/max)")
    print("  start          ", q(t[:, 0] - t0))
    for i, nm in enumerate(names):
        print(f"  {nm:15s}", q(t[:, i + 1] - t[:, i]))
    print("  exit           ", q(t[:, 5] - t0), flush=True)
llmi.test_option("numerics", old)
