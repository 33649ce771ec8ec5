"""Per-workgroup phase timeline of the one-launch x86 decode attention k_a86_d (needs a
-DLLMI_EXP_TRACE build via LLMI_LIB).  Stamps (s_memrealtime, 10 ns) by thread 0: entry,
q staged, scores done, V in LDS (barrier), max, p, PV done.  Env ATT_KV, ATT_SHAPE."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from llmi._lib import lib  # noqa: E402

L = lib()
L.llmi_test_option(b"numerics", 1)
H, HK, D = (int(v) for v in os.environ.get("ATT_SHAPE", "32,8,128").split(","))
names = ["q staged", "scores", "V->LDS barrier", "max", "sum + p", "PV"]
for n in [int(v) for v in os.environ.get("ATT_KV", "128,640,2000").split(",")]:
    tr = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    assert L.llmi_bench_attention(H, HK, D, n, 0, 1, C.c_void_p(tr.data_ptr())) == 0
    t = tr.cpu().numpy().reshape(-1, 8)
    t = t[t[:, 0] != 0]
    t0 = t[:, 0].min()

    def q(x):
        return " ".join(f"{np.percentile(x, k) * 10 / 1000:6.2f}" for k in (0, 50, 100))

    print(f"== n_kv {n}: workgroups {len(t)}; us (min/median/max)")
    print("  start            ", q(t[:, 0] - t0))
    for i, nm in enumerate(names):
        print(f"  {nm:17s}", q(t[:, i + 1] - t[:, i]))
    print("  exit             ", q(t[:, 6] - t0))
