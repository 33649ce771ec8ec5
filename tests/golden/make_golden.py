#!/usr/bin/env python3
"""Generates the committed golden fixtures of tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).  Every vector comes from this repository's own
CPU oracle (oracle/ggml_oracle.c, a restatement of ggml's generic scalar path); the
reference repository holds no llama.cpp source, binary or fixture for this path, so
these pin the oracle against regressions and the GPU against the oracle — parity with
llama.cpp itself stays unpinned.

  tiny-mixed.gguf        the synthetic tiny-mixed preset (seed 1): E=256, 2 layers,
                         every quant type (Q4_K/Q5_K/Q6_K/Q8_0), 1.45 MB
  greedy16.npz           prompt, 16 greedy steps: per-step logits (f32, full vocab)
                         and ids
  blocks.npz             hand-built single blocks with closed-form dequant values
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import pyoracle as po  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
PROMPT = [1, 17, 300, 42, 999 % 1000, 5, 6, 123]
N_GEN = 16


def greedy(path):
    om = po.OracleModel(path, n_ctx=64, threads=1)
    logits, ids = [], []
    cur, pos = PROMPT[0], 0
    for step in range(len(PROMPT) + N_GEN - 1):
        lg = om.decode(cur, pos)
        logits.append(lg.copy())
        pos += 1
        if pos < len(PROMPT):
            cur = PROMPT[pos]
        else:
            cur = int(np.argmax(lg))
            ids.append(cur)
    om.close()
    return np.stack(logits).astype(np.float32), np.array(ids, dtype=np.int32)


def blocks():
    """Closed-form blocks: every quant type with scales chosen so y = q (or q - 32)."""
    out = {}
    # Q4_K: d = 1.0 (fp16 0x3c00), dmin = 0, all 6-bit scales 1, mins 0 -> y = nibble
    b = np.zeros(144, np.uint8)
    b[0:2] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)
    sc = np.zeros(12, np.uint8)
    sc[0:4] = 1          # scales 0..3 (low 6 bits)
    sc[8:12] = 0x01      # scales 4..7 low nibbles = 1, mins 4..7 high nibbles = 0
    b[4:16] = sc
    rng = np.random.default_rng(7)
    b[16:144] = rng.integers(0, 256, 128, dtype=np.uint8)
    qs = b[16:144]
    y = np.zeros(256, np.float32)
    for c in range(4):  # 64-weight chunk c: low nibbles of qs[32c..], then high nibbles
        y[64 * c: 64 * c + 32] = qs[32 * c: 32 * c + 32] & 0xF
        y[64 * c + 32: 64 * c + 64] = qs[32 * c: 32 * c + 32] >> 4
    out["q4_K_block"], out["q4_K_y"] = b, y
    # Q8_0: d = 0.5 -> y = 0.5 * q
    b = np.zeros(34, np.uint8)
    b[0:2] = np.frombuffer(np.float16(0.5).tobytes(), np.uint8)
    q = rng.integers(-127, 128, 32).astype(np.int8)
    b[2:34] = q.view(np.uint8)
    out["q8_0_block"], out["q8_0_y"] = b, (0.5 * q).astype(np.float32)
    # Q6_K: d = 1, all int8 scales 1 -> y = q6 - 32 with q6 = ql nibble | qh 2 bits << 4
    b = np.zeros(210, np.uint8)
    ql = rng.integers(0, 256, 128, dtype=np.uint8)
    qh = rng.integers(0, 256, 64, dtype=np.uint8)
    b[0:128], b[128:192] = ql, qh
    b[192:208] = 1
    b[208:210] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)
    y = np.zeros(256, np.float32)
    for n in range(2):
        for l in range(32):
            lq, hq = ql[64 * n:].astype(np.int32), qh[32 * n:].astype(np.int32)
            y[128 * n + l + 0] = ((lq[l] & 0xF) | (((hq[l] >> 0) & 3) << 4)) - 32
            y[128 * n + l + 32] = ((lq[l + 32] & 0xF) | (((hq[l] >> 2) & 3) << 4)) - 32
            y[128 * n + l + 64] = ((lq[l] >> 4) | (((hq[l] >> 4) & 3) << 4)) - 32
            y[128 * n + l + 96] = ((lq[l + 32] >> 4) | (((hq[l] >> 6) & 3) << 4)) - 32
    out["q6_K_block"], out["q6_K_y"] = b, y
    # Q5_K: like Q4_K plus the fifth bit from qh: weight 64c+l (+32) takes bit 2c (2c+1) of qh[l]
    b = np.zeros(176, np.uint8)
    b[0:2] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)
    b[4:16] = sc
    qh = rng.integers(0, 256, 32, dtype=np.uint8)
    qs = rng.integers(0, 256, 128, dtype=np.uint8)
    b[16:48], b[48:176] = qh, qs
    y = np.zeros(256, np.float32)
    for c in range(4):
        for l in range(32):
            y[64 * c + l] = (qs[32 * c + l] & 0xF) + 16 * ((qh[l] >> (2 * c)) & 1)
            y[64 * c + 32 + l] = (qs[32 * c + l] >> 4) + 16 * ((qh[l] >> (2 * c + 1)) & 1)
    out["q5_K_block"], out["q5_K_y"] = b, y
    return out


def main():
    import llmi

    path = os.path.join(HERE, "tiny-mixed.gguf")
    llmi.write_synthetic_gguf(path, "tiny-mixed", seed=1)
    lg, ids = greedy(path)
    np.savez_compressed(os.path.join(HERE, "greedy16.npz"), prompt=np.array(PROMPT, np.int32), logits=lg, ids=ids)
    np.savez_compressed(os.path.join(HERE, "blocks.npz"), **blocks())
    print("ids", ids.tolist())


if __name__ == "__main__":
    main()
