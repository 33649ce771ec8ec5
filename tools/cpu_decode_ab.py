#!/usr/bin/env python3
"""CPU-baseline A/B (bench.py's cpu_baseline leg in isolation): the oracle port's AVX2 decode
of a synthetic preset at the C2 window under the current OpenMP environment; prints tok/s,
GB/s and the host's streaming-read rate at the same thread count.  Env: PRESET, TH, N,
LOCAL (1: or_model_localize, the decode matrices in rows first-touched by their thread),
FAST (1 AVX2 dots, 2 AVX-512BW where the host has them)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import numpy as np  # noqa: E402

import pyoracle as po  # noqa: E402

preset = os.environ.get("PRESET", "llama3-8b-q4km")
th = int(os.environ.get("TH", "16"))
n = int(os.environ.get("N", "8"))
path = f"/tmp/llmi_bench/{preset}-s3.gguf"
if not os.path.exists(path):
    import llmi

    os.makedirs("/tmp/llmi_bench", exist_ok=True)
    llmi.write_synthetic_gguf(path + ".tmp", preset, seed=3)
    os.replace(path + ".tmp", path)
po.prefer_simd()
fast = po.set_fast_dots(int(os.environ.get("FAST", "1")))
om = po.OracleModel(path, n_ctx=512, threads=th)
local = os.environ.get("LOCAL", "0") == "1"
if local:
    om.localize()
rng = np.random.default_rng(1)
toks = [1] + [int(t) for t in rng.integers(3, 100000, 159)]
om.prefill(toks[:-1], 0)
tok = toks[-1]
best = 0.0
for rep in range(2):
    t0 = time.perf_counter()
    for k in range(n):
        out = om.decode(tok, len(toks) - 1 + rep * n + k)
        tok = int(np.argmax(out))
    best = max(best, n / (time.perf_counter() - t0))
bpt = om.bytes_per_token(len(toks) + n)
env = {k: v for k, v in os.environ.items() if k.startswith(("OMP_", "GOMP_"))}
print(f"{preset} threads {th} local {int(local)} dots {fast} {env}: {best:.2f} tok/s, {best * bpt / 1e9:.1f} GB/s; "
      f"stream {po.host_stream_gbps(1 << 30, 3, th):.1f} GB/s", flush=True)
