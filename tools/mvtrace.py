"""Per-wave timeline of one matvec launch (needs a -DLLMI_EXP_TRACE build via LLMI_LIB).
Prints the distribution of wave start offsets, prologue time, first-pair latency, loop
time and exit offsets (s_memrealtime, 100 MHz = 10 ns ticks).  Env: MV_SHAPES as mvbench."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import random_blocks  # noqa: E402
from llmi._lib import lib  # noqa: E402

L = lib()
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
shapes = []
for tok in os.environ.get("MV_SHAPES", "12:28672x4096,12:4096x14336").split(","):
    t, rc = tok.split(":")
    r, c = rc.split("x")
    shapes.append((int(t), int(r), int(c)))
rng = np.random.default_rng(0)


def pct(a):
    return " ".join(f"{q}%={np.percentile(a, q) * 10 / 1000:6.2f}" for q in (0, 10, 50, 90, 100))


for qt, rows, cols in shapes:
    lb = L.llmi_device_layout_bytes(qt, rows, cols)
    raw = torch.from_numpy(random_blocks(qt, rows, cols, rng)).cuda()
    # many copies so the traced launch reads cold weights
    n = max(2, int(np.ceil(1.2e9 / ((lb + 4095) // 4096 * 4096))))
    stride = (lb + 4095) // 4096 * 4096
    w = torch.empty(stride * n, dtype=torch.uint8, device="cuda")
    for k in range(n):
        assert L.llmi_repack(qt, P(raw), C.c_void_p(w.data_ptr() + stride * k), rows, cols) == 0
    x = torch.randn(cols, device="cuda")
    y = torch.empty(rows, device="cuda")
    hot = os.environ.get("MV_HOT") == "1"  # trace a copy just read by the previous launch
    for k in range(n - 1):  # warm code / TLB, leave copy n-1 cold
        L.llmi_trace_matvec(qt, C.c_void_p(w.data_ptr() + stride * k), rows, cols, P(x), P(y), int(os.environ.get("MV_MODE", "0")), None)
    tgt = (n - 2) if hot else (n - 1)
    tr = torch.zeros(2048 * 16 * 8, dtype=torch.int64, device="cuda")
    g = L.llmi_trace_matvec(qt, C.c_void_p(w.data_ptr() + stride * tgt), rows, cols, P(x), P(y), int(os.environ.get("MV_MODE", "0")), P(tr))
    t = tr.cpu().numpy().reshape(-1, 16)
    if os.environ.get("MV_DUMP"):
        np.save(os.path.join(os.environ["MV_DUMP"], f"trace_{qt}_{rows}x{cols}.npy"), t)
    t = t[t[:, 0] != 0].astype(np.int64)
    t0 = t[:, 0].min()
    start, pro, first, end = t[:, 0] - t0, t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t0
    items = (t[:, 5] & 0xffffffff)
    print(f"== type {qt} {rows}x{cols}: waves {len(t)} grid {g} span {end.max() * 10 / 1000:.2f} us "
          f"({lb / (end.max() * 10e-9) / 1e9:.0f} GB/s over the wave span)")
    print("  start offset us :", pct(start))
    print("  prologue us     :", pct(pro))
    print("  first sub us    :", pct(first[items > 0]))
    prev = t[:, 2]
    for k in range(2, 10):  # steady state: end of sub-item k - end of sub-item k-1
        m = (items >= k)
        if not m.any():
            break
        print(f"  sub {k} us       :", pct((t[m, 6 + k] - prev[m])))
        prev = np.where(items >= k, t[:, 6 + k], prev)
    print("  exit offset us  :", pct(end))
    print("  subs per wave   :", np.bincount(items).tolist())
    xcc = (t[:, 5] >> 32) & 0xff
    for xc in range(8):
        m = xcc == xc
        if m.any():
            print(f"  xcc {xc}: waves {m.sum():5d} start50 {np.percentile(start[m], 50) * 10 / 1000:6.2f} "
                  f"exit50 {np.percentile(end[m], 50) * 10 / 1000:6.2f} exit100 {end[m].max() * 10 / 1000:6.2f}")
    del w, raw
