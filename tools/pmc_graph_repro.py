"""Profiler-crash isolation: hipGraph replay of plain PyTorch kernels, no
llmi code in the process, for `rocprofv3 --pmc FETCH_SIZE` (the pass that ends in a
SIGSEGV inside librocprofiler-sdk when bench.py replays llmi's decode graph)."""
import sys

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
x = torch.randn(1 << 22, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(3):
        y.copy_(x * 2 + 1)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(16):  # 16 dependent kernels per replay, like a decode layer's chain
        y.mul_(0.5).add_(x)
for i in range(n):
    g.replay()
    if i % 500 == 0:
        print("replay", i, flush=True)
torch.cuda.synchronize()
print("done", float(y[0]))
