"""Attention microbenchmark over KV lengths and paths (llmi_bench_attention).
Env: ATT_SHAPE="32,8,128" (n_head, n_head_kv, head_dim), ATT_KV="128,640,2048,4096,8000",
ATT_MODES="1,2,3,4", ATT_REPS=20, ATT_NUMERICS=1 (the x86 numerics mode's kernels)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import torch  # noqa: F401,E402

from llmi._lib import lib  # noqa: E402

L = lib()
if os.environ.get("ATT_NUMERICS"):
    L.llmi_test_option(b"numerics", int(os.environ["ATT_NUMERICS"]))
H, HK, D = (int(v) for v in os.environ.get("ATT_SHAPE", "32,8,128").split(","))
kvs = [int(v) for v in os.environ.get("ATT_KV", "128,640,2048,4096,8000").split(",")]
modes = [int(v) for v in os.environ.get("ATT_MODES", "1,2,3,4").split(",")]
reps = int(os.environ.get("ATT_REPS", "20"))
res = {}
for n in kvs:
    row = {}
    for m in modes:
        us = L.llmi_bench_attention(H, HK, D, n, m, reps, None)
        row[m] = round(us, 2)
    kv_bytes = 2 * HK * n * D * 2
    res[n] = row
    print(f"n_kv {n:6d} KV {kv_bytes / 1e6:7.2f} MB  " + "  ".join(f"mode{m} {row[m]:7.2f} us" for m in modes), flush=True)
print(json.dumps(res))
