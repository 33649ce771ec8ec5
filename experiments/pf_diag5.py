"""Diagnostic: long prompts, prompt logits per path: prefill, and decode steps per attention mode."""
import os, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi

for preset in ("tiny-mixed", "tiny-mixed-d128"):
    path = f"/tmp/{preset}.gguf"
    llmi.write_synthetic_gguf(path, preset, seed=1)
    for n in (500, 513):
        rng = np.random.default_rng(9)
        prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
        res = {}
        for key, npf, mode in (("prefill", "0", "0"), ("steps-auto", "1", "0"), ("steps-fused", "1", "1"),
                               ("steps-split", "1", "2"), ("steps-2k", "1", "3"), ("steps-x", "1", "4")):
            os.environ["LLMI_NO_PREFILL"] = npf
            os.environ["LLMI_ATTN_MODE"] = mode
            m = llmi.Model(path); c = llmi.Context(m, n_ctx=768)
            assert c.decode(prompt) == 0
            res[key] = c.logits(-1); c.close(); m.close()
        base = res["prefill"]
        print(preset, n, {k: float(np.abs(v - base).max()) for k, v in res.items()}, flush=True)
