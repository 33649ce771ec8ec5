"""Which stage of the batched step differs between two identical runs (1-layer model)."""
import sys
sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "tests")
import ctypes as C
import numpy as np
import torch
torch.zeros(1, device="cuda")
import llmi
from llmi._lib import lib
from test_gpu_batch import _prompts

preset = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b-q4km"
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 1
path = f"/tmp/{preset}-L{nl}.gguf"
llmi.write_synthetic_gguf(path, preset, seed=11, n_layer=nl)
rng = np.random.default_rng(3)
prompts = _prompts(rng, 8, hi=30000, max_len=24)
m = llmi.Model(path)
E, V, H = m.n_embd, m.n_vocab, m.n_head
sizes = {11: E, 12: H * 128, 13: H * 128, 14: 14336, 15: V}
runs = []
for rep in range(3):
    c = llmi.Context(m, n_ctx=256, n_seq=8)
    firsts = []
    for s, p in enumerate(prompts):
        assert c.decode(p, seq=[s] * len(p)) == 0
        firsts.append(c.greedy(-1))
    g = c.generate_greedy_batch(list(range(8)), firsts, [len(p) for p in prompts], 1)
    taps = {}
    for w, n in sizes.items():
        buf = np.zeros(n * 8, np.float32)
        assert lib().llmi_debug_tap(c._h, w, buf.ctypes.data_as(C.c_void_p)) == 0, llmi.last_error()
        taps[w] = buf.reshape(8, n)
    runs.append((g, taps))
    c.close()
for rep in (1, 2):
    g, taps = runs[rep]
    print(f"run {rep} vs 0: tokens equal {g == runs[0][0]}", flush=True)
    for w in sizes:
        a, b = runs[0][1][w], taps[w]
        bad = [s for s in range(8) if not np.array_equal(a[s], b[s])]
        nan = int(np.isnan(b).sum())
        print(f"  tap {w}: differing slots {bad} maxdiff {np.nanmax(np.abs(a - b)) if bad else 0:.3g} nan {nan}", flush=True)
