"""Per-phase timeline of one persistent decode step (needs a -DLLMI_EXP_TRACE build via
LLMI_LIB): for every grid barrier, the spread of workgroup arrivals (phase work done)
and releases, in microseconds from the step's first release.  Usage:
  LLMI_LIB=.../libllmi_trace.so python tools/steptrace.py [preset] [ctx]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import llmi  # noqa: E402
from llmi._lib import lib  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b-q4km"
ctx_len = int(sys.argv[2]) if len(sys.argv) > 2 else 300
path = f"/tmp/llmi_bench/{preset}-s3.gguf"
if not os.path.exists(path):
    os.makedirs("/tmp/llmi_bench", exist_ok=True)
    llmi.write_synthetic_gguf(path, preset, seed=3)
m = llmi.Model(path)
c = llmi.Context(m, n_ctx=ctx_len + 64)
rng = np.random.default_rng(4)
prompt = [1] + [int(t) for t in rng.integers(0, 30000, ctx_len - 1)]
assert c.decode(prompt) == 0
t = c.greedy(-1)
seq = c.generate_greedy(t, len(prompt), 8)
n = 1024 * 512 * 2
buf = (C.c_uint64 * n)()
assert lib().llmi_step_trace_copy(c._h, buf, n) == 0
tr = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 512, 2).astype(np.int64)
nwg = int((tr[:, 0, 0] != 0).sum())
tr = tr[:nwg]
nb = int((tr[0, :, 0] != 0).sum())
t0 = tr[:, 0, 0].min()
names = []
L = m.n_layer
for l in range(L):
    names += [f"L{l} qkv", f"L{l} att-scores", f"L{l} att-pv", f"L{l} o", f"L{l} gate_up", f"L{l} down"]
print(f"{preset} ctx {ctx_len}: {nwg} workgroups, {nb} barriers; step span "
      f"{(tr[:, nb - 1, 1].max() - t0) * 10 / 1000:.1f} us until the last release")
prev_rel = np.full(nwg, t0)
tot = {}
for b in range(nb):
    arr, rel = tr[:, b, 0], tr[:, b, 1]
    work = (arr - prev_rel) * 10 / 1000  # us per workgroup from its previous release to arrival
    wait = (rel - arr) * 10 / 1000
    seam = (rel.max() - arr.max()) * 10 / 1000
    ph = names[b] if b < len(names) else f"b{b}"
    kind = ph.split(" ", 1)[1] if " " in ph else ph
    d = tot.setdefault(kind, [0, 0, 0, 0])
    d[0] += float(np.median(work)); d[1] += float(work.max()); d[2] += seam; d[3] += 1
    if b < 12 or b >= nb - 2:
        print(f"  {ph:16s} work med {np.median(work):6.2f} max {work.max():6.2f} us | last arrival->last release "
              f"{seam:5.2f} us | release spread {(rel.max() - rel.min()) * 10 / 1000:5.2f}")
    prev_rel = rel
print("per phase kind, summed over layers (us): work median / work max / seam")
for k, (a, b_, s_, nn) in tot.items():
    print(f"  {k:12s} {a:8.1f} {b_:8.1f} {s_:8.1f}  ({nn} barriers)")
