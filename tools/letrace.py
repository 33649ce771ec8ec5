#!/usr/bin/env python3
"""Timeline of one layer-engine launch (leng.hip) inside a real decode step.

Loads a synthetic preset (LE_PRESET, default llama3-8b-q4km; LE_LAYERS layers, 0 = all),
prefills a 128-token prompt, decodes up to LE_POS (default 384, the C2 window's mean
context), then llmi_engine_trace()s layer LE_LAYER (default the middle one) and prints,
in microseconds from the first workgroup's entry, the distribution over workgroups of:
  loader   (wave 0 of the LE_NL loader waves) op k issue start / end, loader done, ring-full waits
  consumers (per wave) op k edge seen, image built, first sub-item ready, op done,
           time spent waiting for ring data
Stamps: s_memrealtime (100 MHz).  LE_DUMP=<file.npy> saves the raw stamps.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import llmi  # noqa: E402

preset = os.environ.get("LE_PRESET", "llama3-8b-q4km")
nl = int(os.environ.get("LE_LAYERS", "0"))
pos = int(os.environ.get("LE_POS", "384"))
d = os.environ.get("LE_DIR", "/tmp/llmi_bench")
os.makedirs(d, exist_ok=True)
path = os.path.join(d, f"{preset}-s3.gguf" if nl == 0 else f"{preset}-L{nl}-s3.gguf")
if not os.path.exists(path):
    llmi.write_synthetic_gguf(path + ".tmp", preset, seed=3, n_layer=nl)
    os.replace(path + ".tmp", path)
m = llmi.Model(path)
c = llmi.Context(m, n_ctx=((pos + 64 + 255) // 256) * 256)
rng = np.random.default_rng(4)
prompt = [1] + [int(t) for t in rng.integers(0, min(128000, m.n_vocab), 127)]
assert c.decode(prompt) == 0
first = c.greedy(-1)
toks = c.generate_greedy(first, len(prompt), pos - len(prompt))
layer = int(os.environ.get("LE_LAYER", str(m.n_layer // 2)))
reps = int(os.environ.get("LE_REPS", "3"))
for rep in range(reps):
    t = c.engine_trace(toks[-1], pos, layer).astype(np.int64)
if os.environ.get("LE_DUMP"):
    np.save(os.environ["LE_DUMP"], t)
G = t.shape[0]
NL = int(os.environ.get("LE_NL", "2"))  # loader waves (leng.hip kLeNL), then 7 consumer waves
lds = t[:, :NL, :]
ld = t[:, 0, :]
cs = t[:, NL:NL + 7, :]
t0 = min(lds[:, :, 0].min(), cs[:, :, 0].min())
us = lambda a: (a - t0) * 0.01  # noqa: E731


def row(name, a):
    a = np.asarray(a, dtype=np.float64)
    q = np.percentile(a, [0, 10, 50, 90, 100])
    print(f"  {name:34s} " + " ".join(f"{v:8.2f}" for v in q))


print(f"== {preset} layer {layer} pos {pos}: {G} workgroups; us from first entry: min p10 p50 p90 max")
row("entry (all waves)", us(np.concatenate([lds[:, :, 0].ravel(), cs[:, :, 0].ravel()])))
ops = ["attn_output", "gate+up", "down", "qkv(next)"]
for k in range(4):
    if ld[:, 1 + 2 * k].max() == 0:
        continue
    row(f"loader {ops[k]} issue start", us(ld[:, 1 + 2 * k]))
    row(f"loader {ops[k]} issue end", us(ld[:, 2 + 2 * k]))
for k in range(4):
    if ld[:, 1 + 2 * k].max() == 0:
        continue
    vm = ld[:, 14 + 2 * k] - (ld[:, 12 + 2 * k] if k > 0 else 0)
    sp = ld[:, 15 + 2 * k] - (ld[:, 13 + 2 * k] if k > 0 else 0)
    row(f"loader {ops[k]} vmcnt-wait us", vm * 0.01)
    row(f"loader {ops[k]} ring-full us", sp * 0.01)
row("loader done (last loader)", us(lds[:, :, 9].max(axis=1)))
row("loader ring-full waits (count, sum)", lds[:, :, 10].sum(axis=1))
row("loader ring-full wait us (max)", lds[:, :, 11].max(axis=1) * 0.01)
for k in range(4):
    e = cs[:, :, 1 + 4 * k]
    if e.max() == 0:
        continue
    row(f"{ops[k]} edge seen (wave max)", us(e.max(axis=1)))
    row(f"{ops[k]} image built (wave max)", us(cs[:, :, 2 + 4 * k].max(axis=1)))
    fr = cs[:, :, 3 + 4 * k]
    row(f"{ops[k]} first ready (wave min)", us(np.where(fr > 0, fr, fr.max()).min(axis=1)))
    row(f"{ops[k]} done (wave max)", us(cs[:, :, 4 + 4 * k].max(axis=1)))
    row(f"{ops[k]} ring wait us (wave max)", cs[:, :, 20 + k].max(axis=1) * 0.01)
for k in range(3):
    if cs[:, :, 24 + k].max() == 0:
        continue
    row(f"{ops[k]} stores drained (wave max)", us(cs[:, :, 24 + k].max(axis=1)))
for k in range(1, 4):
    if cs[:, 0, 27 + k].max() == 0:
        continue
    row(f"{ops[k]} edge polls (poller)", cs[:, 0, 27 + k])
row("consumer exit (wave max)", us(cs[:, :, 17].max(axis=1)))
print(f"  launch span {us(max(cs[:, :, 17].max(), lds[:, :, 9].max())):.2f} us")
