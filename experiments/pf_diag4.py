"""Diagnostic: long prompts, prefill vs decode steps (max |d| of the prompt logits)."""
import os, sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi

for preset in ("tiny-mixed", "tiny-mixed-d128"):
    path = f"/tmp/{preset}.gguf"
    llmi.write_synthetic_gguf(path, preset, seed=1)
    for n in (100, 200, 300, 400, 500, 513, 520, 600):
        rng = np.random.default_rng(9)
        prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
        res = []
        for npf in ("0", "1"):
            os.environ["LLMI_NO_PREFILL"] = npf
            m = llmi.Model(path); c = llmi.Context(m, n_ctx=768)
            assert c.decode(prompt) == 0
            res.append(c.logits(-1)); c.close(); m.close()
        print(preset, n, "prefill vs steps max|d|", float(np.abs(res[0] - res[1]).max()), flush=True)
