#!/usr/bin/env python3
"""The layer engine's weight stream in isolation (llmi_le_stream_bench): every CU streams
its contiguous share of a 2 GiB buffer in 1-KiB pieces; GB/s per mode (see llmi.h)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import torch  # noqa: E402

from llmi._lib import lib  # noqa: E402

buf = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
buf.random_(0, 255)
names = {0: "1 loader wave, asm DMA", 1: "1 loader wave, builtin DMA", 2: "2 loader waves", 3: "4 loader waves",
         4: "8 waves plain 16-B loads"}
for nt in (1, 0):
    for mode in (0, 1, 2, 3, 4):
        g = lib().llmi_le_stream_bench(C.c_void_p(buf.data_ptr()), buf.numel(), mode, 5, nt)
        print(f"nt={nt} mode {mode} ({names[mode]}): {g:8.1f} GB/s")
