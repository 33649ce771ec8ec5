"""Per-wave timeline of the one-workgroup-per-head attention kernels (k_attn_fused mode 1,
k_attn_r mode 5; needs a -DLLMI_EXP_TRACE build via LLMI_LIB).  Stamps (s_memrealtime,
10 ns): entry, scores done (K arrived), probabilities in LDS, exit.
Env ATT_KV, ATT_SHAPE, ATT_MODES."""
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
for mode in [int(v) for v in os.environ.get("ATT_MODES", "1,5").split(",")]:
    for n in [int(v) for v in os.environ.get("ATT_KV", "128,256,512").split(",")]:
        tr = torch.zeros(2 * 4096 * 64, dtype=torch.int64, device="cuda")
        assert L.llmi_bench_attention(H, HK, D, n, mode, 1, C.c_void_p(tr.data_ptr())) == 0
        t = tr.cpu().numpy().reshape(2, 4096 * 16, 4)[0]
        t = t[t[:, 0] != 0]
        t0 = t[:, 0].min()

        def q(a):
            return " ".join(f"{np.percentile(a, x) * 10 / 1000:6.2f}" for x in (0, 50, 100))

        print(f"== mode {mode} n_kv {n}: waves {len(t)}; us (min/median/max)")
        print("  start          ", q(t[:, 0] - t0))
        print("  scores (K in)  ", q(t[:, 1] - t[:, 0]))
        print("  softmax        ", q(t[:, 2] - t[:, 1]))
        print("  PV + store     ", q(t[:, 3] - t[:, 2]))
        print("  exit           ", q(t[:, 3] - t0), flush=True)
