#!/usr/bin/env python3
"""Prefill (TTFT) benchmark — SURVEY.md §8f item 1 / BASELINE.json configs[3] (C4).

For each prompt length: a warm llama_decode of the whole prompt (batched MFMA prefill of
all but the last token + one decode step for its logits), timed on the host around the
synchronous call; the same with LLMI_NO_PREFILL=1 (every token a decode step) for the
shorter prompts.  Also the prefill GEMM alone (llmi_pf_gemm hook) per shape: device time
and int8 TOPS (2*T*rows*cols ops).  Prints one JSON line.
usage: tools/prefillbench.py [preset] [prompt lengths, comma-separated]
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.zeros(1, device="cuda")
import llmi  # noqa: E402
from llmi._lib import lib  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b-q4km"
lens = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "128,512,2048").split(",") if x.strip()]
GEMM_T = [int(x) for x in os.environ.get("PF_GEMM_T", "128,512").split(",")]
path = f"/tmp/llmi_bench/{preset}-s3.gguf"
if lens and not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    llmi.write_synthetic_gguf(path + ".tmp", preset, seed=3)
    os.replace(path + ".tmp", path)
out = {"preset": preset, "prompts": {}}
for env, opt in (("PF_GEMM_NG", b"pf_gemm_ng"), ("PF_XCD_MAP", b"pf_xcd_map"), ("PF_QKV_MERGE", b"pf_qkv_merge")):  # A/B knobs (test options)
    if os.environ.get(env):
        lib().llmi_test_option(opt, int(os.environ[env]))
        out[env.lower()] = int(os.environ[env])
if lens:  # an empty length list times the GEMM shapes alone (no model)
    m = llmi.Model(path)
    n_ctx = (max(lens + [1]) + 2 + 255) // 256 * 256
    c = llmi.Context(m, n_ctx=n_ctx)
    out["prefill_supported"] = m.prefill_supported
rng = np.random.default_rng(4)
for n in lens:
    prompt = [1] + [int(t) for t in rng.integers(3, min(30000, m.n_vocab), n - 1)]
    rec = {}
    for mode in ("mfma", "steps"):
        if mode == "steps" and n > 512:
            continue
        if mode == "steps":
            os.environ["LLMI_NO_PREFILL"] = "1"
        else:
            os.environ.pop("LLMI_NO_PREFILL", None)
        best = None
        for rep in range(2):
            c.kv_clear()
            torch.cuda.synchronize()
            t = time.perf_counter()
            assert c.decode(prompt) == 0
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        rec[mode] = {"ms": round(best * 1e3, 2), "tok_per_s": round(n / best, 1)}
        print(f"[prefillbench] {preset} n={n} {mode}: {best * 1e3:.1f} ms ({n / best:.0f} tok/s)", file=sys.stderr, flush=True)
    os.environ.pop("LLMI_NO_PREFILL", None)
    out["prompts"][n] = rec

# GEMM alone per shape (Q4_K weights of the 8B shapes), T tokens
from helpers import Q4_K, Q6_K, empty_dev, random_blocks, to_dev  # noqa: E402

L = lib()
g = {}
for (qt, rows, cols) in ((Q4_K, 14336, 4096), (Q4_K, 4096, 14336), (Q6_K, 4096, 14336), (Q4_K, 4096, 4096),
                         (Q6_K, 14336, 4096), (Q6_K, 4096, 4096)):
    r = np.random.default_rng(1)
    raw = random_blocks(qt, rows, cols, r)
    wd = empty_dev(L.llmi_device_layout_bytes(qt, rows, cols))
    rd = to_dev(raw)
    torch.cuda.synchronize()
    assert L.llmi_repack(qt, C.c_void_p(rd.data_ptr()), C.c_void_p(wd.data_ptr()), rows, cols) == 0
    del rd
    for T in GEMM_T:
        x = to_dev(r.standard_normal((T, cols)).astype(np.float32))
        y = torch.empty((T, rows), dtype=torch.float32, device="cuda")
        us = C.c_double()
        for _ in range(3):
            assert L.llmi_pf_gemm(qt, C.c_void_p(wd.data_ptr()), rows, cols, C.c_void_p(x.data_ptr()), None, 1e-5, T,
                                  C.c_void_p(y.data_ptr()), C.byref(us)) == 0
        tops = 2.0 * T * rows * cols / (us.value * 1e-6) / 1e12
        g[f"{'q4_K' if qt == Q4_K else 'q6_K'} {rows}x{cols} T={T}"] = {"us": round(us.value, 1), "TOPS": round(tops, 2)}
        print(f"[prefillbench] gemm {rows}x{cols} T={T}: {us.value:.1f} us {tops:.1f} TOPS", file=sys.stderr, flush=True)
out["gemm"] = g
print(json.dumps(out))
