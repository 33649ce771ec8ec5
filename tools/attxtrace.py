"""Per-wave timeline of the one-launch exchange attention k_attn_x (needs a
-DLLMI_EXP_TRACE build via LLMI_LIB).  Stamps (s_memrealtime, 10 ns): entry, q staged,
scores published, granules swept, softmax done, PV done.  Env ATT_KV, ATT_SHAPE."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from llmi._lib import lib  # noqa: E402

L = lib()
H, HK, D = (int(v) for v in os.environ.get("ATT_SHAPE", "32,8,128").split(","))
for n in [int(v) for v in os.environ.get("ATT_KV", "128,640,1024").split(",")]:
    tr = torch.zeros(2 * 4096 * 64, dtype=torch.int64, device="cuda")
    assert L.llmi_bench_attention(H, HK, D, n, 4, 1, C.c_void_p(tr.data_ptr())) == 0
    t = tr.cpu().numpy().reshape(2, 4096 * 16, 4)
    a, b = t[0], t[1]
    keep = a[:, 0] != 0
    a, b = a[keep], b[keep]
    t0 = a[:, 0].min()

    def q(x):
        return " ".join(f"{np.percentile(x, k) * 10 / 1000:6.2f}" for k in (0, 50, 100))

    print(f"== n_kv {n}: waves {len(a)}; us (min/median/max)")
    print("  start             ", q(a[:, 0] - t0))
    print("  q staged          ", q(a[:, 1] - a[:, 0]))
    print("  scores published  ", q(a[:, 2] - a[:, 1]))
    print("  granules swept    ", q(a[:, 3] - a[:, 2]))
    print("  softmax           ", q(b[:, 0] - a[:, 3]))
    print("  PV                ", q(b[:, 1] - b[:, 0]))
    print("  exit              ", q(b[:, 1] - t0))
