#!/usr/bin/env python3
"""Batched-prefill attention alone (llmi_pf_attention): one ubatch of T query tokens at
position pos0 over random f16 caches, per path (0 tiled FP64-MFMA, 1 grouped LDS, 2 one
head per workgroup).  Device time per launch and FP64 TFLOP/s on the algorithmic flops
(2 * D per live (row, position) pair for q.k and again for p.v).  One JSON line.
usage: tools/pfattn_bench.py [H,HK,D] [T] [pos0 list] [modes]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.zeros(1, device="cuda")
import llmi  # noqa: E402

H, HK, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "32,8,128").split(","))
T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
P0 = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0,1536,7680,15872").split(",")]
MODES = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "0,1").split(",")]
L = llmi.lib()
res = {"heads": [H, HK, D], "T": T, "runs": []}
for pos0 in P0:
    n_ctx = (pos0 + T + 255) // 256 * 256
    g = torch.Generator(device="cuda").manual_seed(pos0)
    q = torch.randn(T * H * D, device="cuda", generator=g)
    kc = (torch.randn(HK * n_ctx * D, device="cuda", generator=g) * 0.3).half().view(torch.int16)
    vc = torch.randn(HK * D * n_ctx, device="cuda", generator=g).half().view(torch.int16)
    out = torch.empty(T * H * D, device="cuda")
    pairs = H * sum(pos0 + t + 1 for t in range(T))
    flops = 4.0 * D * pairs
    for mv in MODES + ([-410, -420, -421, -441, -221, -241] if 0 in MODES else []):
        mode = max(mv, 0)
        L.llmi_test_option(b"pf_fa_cfg", -mv if mv < 0 else 440)
        best = None
        for _ in range(3):
            us = L.llmi_pf_attention(H, HK, D, T, pos0, n_ctx, q.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                                     out.data_ptr(), mode, 0)
            if us < 0:
                break
            best = us if best is None else min(best, us)
        rec = {"pos0": pos0, "mode": mode, "us": None if best is None else round(best, 1)}
        if mode == 0:
            rec["fa_cfg"] = -mv if mv < 0 else 440
        if best is not None:
            rec["tflops"] = round(flops / best / 1e6, 2)
        else:
            rec["error"] = llmi.last_error()
        res["runs"].append(rec)
        print(f"[pfattn] pos0={pos0} mode={mode}: {rec}", file=sys.stderr, flush=True)
L.llmi_test_option(b"pf_fa_cfg", 440)
print(json.dumps(res))
