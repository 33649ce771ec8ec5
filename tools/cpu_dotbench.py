#!/usr/bin/env python3
"""Per-core rate of the CPU baseline's AVX2 dots (oracle/, or_set_fast_dots) on an L2-resident
128 x 4096 matrix, one thread, best of 5 runs (tools/ helper for bench.py's cpu_baseline leg)."""
import sys, time, ctypes as C
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))), 'oracle'))
import numpy as np
import pyoracle as po
po.prefer_simd()
po.set_fast_dots(True)
L = po.lib()
rng = np.random.default_rng(0)
# type ids: or_* enums from ggml: Q4_K=12, Q5_K=13, Q6_K=14, Q8_0=8
sizes = {12: 144, 13: 176, 14: 210, 8: 34}
bs = {12: 256, 13: 256, 14: 256, 8: 32}
for t in (12, 14, 13, 8):
    rows, cols = 128, 4096
    nb = cols // bs[t]
    W = rng.integers(0, 256, rows * nb * sizes[t], dtype=np.uint8)
    Wv = W.reshape(rows * nb, sizes[t])
    # small finite f16 scales
    h = np.float16(0.01).view(np.uint16)
    if t in (12, 13):
        Wv[:, 0:2] = np.frombuffer(np.uint16(h).tobytes(), np.uint8); Wv[:, 2:4] = Wv[:, 0:2]
    elif t == 14:
        Wv[:, 208:210] = np.frombuffer(np.uint16(h).tobytes(), np.uint8)
    else:
        Wv[:, 0:2] = np.frombuffer(np.uint16(h).tobytes(), np.uint8)
    x = rng.standard_normal(cols).astype(np.float32)
    y = np.zeros(rows, np.float32)
    for _ in range(3):
        L.or_matvec(t, W.ctypes.data, rows, cols, x.ctypes.data, y.ctypes.data, 1)
    n = 200
    dt = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(n):
            L.or_matvec(t, W.ctypes.data, rows, cols, x.ctypes.data, y.ctypes.data, 1)
        dt = min(dt, time.perf_counter() - t0)
    print(f"type {t}: {W.nbytes * n / dt / 1e9:.2f} GB/s per core (L2-resident {W.nbytes/1024:.0f} KB), y0 {y[0]:.4f}")
