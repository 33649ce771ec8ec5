"""Diagnose batched-vs-single divergence at real widths: determinism of each path and
the attention kernel choice (LLMI_ATTN_MODE for the single path)."""
import os, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi
from test_gpu_batch import _prompts, _single_reference, _batched

preset = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b-q4km"
path = f"/tmp/{preset}-L2.gguf"
llmi.write_synthetic_gguf(path, preset, seed=11, n_layer=2)
rng = np.random.default_rng(3)
prompts = _prompts(rng, 8, hi=30000, max_len=24)
def diff(a, b):
    return [(s, next((i for i in range(len(a[s])) if a[s][i] != b[s][i]), None)) for s in range(len(a)) if a[s] != b[s]]
A1, _ = _single_reference(path, prompts, 12, 256)
A2, _ = _single_reference(path, prompts, 12, 256)
print("single vs single:", diff(A1, A2), flush=True)
B1, _, c1 = _batched(path, prompts, 12, 256); c1.close()
B2, _, c2 = _batched(path, prompts, 12, 256); c2.close()
print("batched vs batched:", diff(B1, B2), flush=True)
print("single vs batched:", diff(A1, B1), flush=True)
for mode in ("2", "1"):
    os.environ["LLMI_ATTN_MODE"] = mode
    Am, _ = _single_reference(path, prompts, 12, 256)
    print(f"single(mode {mode}) vs single(auto):", diff(Am, A1), " vs batched:", diff(Am, B1), flush=True)
os.environ["LLMI_ATTN_MODE"] = "0"
os.environ["LLMI_NO_PREFILL"] = "1"
An, _ = _single_reference(path, prompts, 12, 256)
Bn, _, c3 = _batched(path, prompts, 12, 256); c3.close()
print("no-prefill single vs batched:", diff(An, Bn), " single vs single(prefill):", diff(An, A1), flush=True)
