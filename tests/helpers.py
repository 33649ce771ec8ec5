"""Test helpers: random quantized blocks with sane fp16 scales, device buffers."""
from __future__ import annotations

import numpy as np

F32, F16, Q8_0, Q4_K, Q5_K, Q6_K = 0, 1, 8, 12, 13, 14
BLOCK_ELEMS = {Q8_0: 32, Q4_K: 256, Q5_K: 256, Q6_K: 256}
BLOCK_BYTES = {Q8_0: 34, Q4_K: 144, Q5_K: 176, Q6_K: 210}
QTYPES = (Q4_K, Q5_K, Q6_K, Q8_0)
TNAME = {Q4_K: "q4_K", Q5_K: "q5_K", Q6_K: "q6_K", Q8_0: "q8_0"}


def f16_bytes(v: np.ndarray) -> np.ndarray:
    return np.asarray(v, dtype=np.float16).view(np.uint8).reshape(-1, 2)


def random_blocks(qtype: int, rows: int, cols: int, rng: np.random.Generator) -> np.ndarray:
    """Uniform random payload bytes with fp16 block scales of realistic magnitude."""
    nb = rows * (cols // BLOCK_ELEMS[qtype])
    bb = BLOCK_BYTES[qtype]
    raw = rng.integers(0, 256, size=(nb, bb), dtype=np.uint8)
    if qtype in (Q4_K, Q5_K):
        d = rng.uniform(2e-5, 1.2e-4, nb).astype(np.float32)
        raw[:, 0:2] = f16_bytes(d)
        raw[:, 2:4] = f16_bytes(d * 7.5)
    elif qtype == Q6_K:
        raw[:, 208:210] = f16_bytes(rng.uniform(1e-5, 5e-5, nb))
    else:
        raw[:, 0:2] = f16_bytes(rng.uniform(1e-4, 5e-4, nb))
    return raw.reshape(-1)


def to_dev(a: np.ndarray):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def empty_dev(nbytes: int):
    import torch

    return torch.empty(int(nbytes), dtype=torch.uint8, device="cuda")
