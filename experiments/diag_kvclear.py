"""Diag: prompt -> kv_clear -> same prompt again at long contexts (8B synthetic)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llama-gguf-inference_amd"))
import numpy as np
import llmi
path = "/tmp/llmi_bench/llama3-8b-q4km-s3.gguf"
if not os.path.exists(path):
    os.makedirs("/tmp/llmi_bench", exist_ok=True)
    llmi.write_synthetic_gguf(path, "llama3-8b-q4km", seed=3)
m = llmi.Model(path)
for n in [int(v) for v in sys.argv[1:]]:
    c = llmi.Context(m, n_ctx=(n + 300) // 256 * 256 + 256)
    rng = np.random.default_rng(4)
    prompt = [1] + [int(t) for t in rng.integers(0, 128000, n - 1)]
    r1 = c.decode(prompt)
    e1 = llmi._lib.last_error() if r1 else ""
    c.kv_clear()
    r2 = c.decode(prompt)
    e2 = llmi._lib.last_error() if r2 else ""
    print(n, os.environ.get("LLMI_ATTN_MODE"), "first", r1, e1, "second", r2, e2, flush=True)
    c.close()
