"""Per-wave timeline of the split attention kernels (needs a -DLLMI_EXP_TRACE build via
LLMI_LIB).  Stamps (s_memrealtime, 10 ns): scores: entry, after loads+barrier, K data
used, exit; pv: entry, after score staging, after softmax, exit.  Env ATT_KV, ATT_SHAPE."""
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
for n in [int(v) for v in os.environ.get("ATT_KV", "128,640,4096").split(",")]:
    tr = torch.zeros(2 * 4096 * 64, dtype=torch.int64, device="cuda")
    assert L.llmi_bench_attention(H, HK, D, n, 2, 1, C.c_void_p(tr.data_ptr())) == 0
    t = tr.cpu().numpy().reshape(2, 4096 * 16, 4)
    s, p = t[0], t[1]
    s = s[s[:, 0] != 0]
    p = p[p[:, 0] != 0]
    t0 = min(s[:, 0].min(), p[:, 0].min())

    def q(a):
        return " ".join(f"{np.percentile(a, x) * 10 / 1000:6.2f}" for x in (0, 50, 100))

    print(f"== n_kv {n}: scores waves {len(s)}, pv waves {len(p)}; offsets in us (min/median/max)")
    print("  scores start      ", q(s[:, 0] - t0))
    print("  scores loads+bar  ", q(s[:, 1] - s[:, 0]))
    ok = s[:, 2] != 0
    if ok.any():
        print("  scores K arrived  ", q(s[ok, 2] - s[ok, 1]))
        print("  scores compute    ", q(s[ok, 3] - s[ok, 2]))
    print("  scores exit       ", q(s[:, 3][s[:, 3] != 0] - t0))
    print("  pv start          ", q(p[:, 0] - t0))
    print("  pv staging        ", q(p[:, 1] - p[:, 0]))
    print("  pv softmax        ", q(p[:, 2] - p[:, 1]))
    print("  pv PV             ", q(p[:, 3] - p[:, 2]))
    print("  pv exit           ", q(p[:, 3] - t0))
