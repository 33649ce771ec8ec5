#!/usr/bin/env python3
"""Distance of the GPU path from the reference's NGL=0 numerics.

The GPU is bit-identical to the oracle's generic order (tests/test_gpu_long.py
test_generic_order_trajectory), so the distance GPU <-> NGL=0 equals generic <-> x86:
this runs the oracle twice in lockstep on one synthetic model -- once in ggml's generic
order, once in upstream's x86 AVX2 association (oracle/ggml_oracle.c "x86 association
mode", recalled, not vendored) -- teacher-forced with the generic run's greedy ids, and
reports per trajectory:
  frac_within_1e-3      steps whose logits agree within 1e-3 (north_star's tolerance)
  worst_abs_diff        largest |logit difference| over all steps
  first_id_divergence   the first step whose greedy ids differ (= where a free-running
                        x86 decode leaves the GPU's trajectory), with both top-2 margins
CPU only.  Usage:
  tools/parity_x86.py [--preset llama3-8b-q4km] [--layers 2] [--vocab 0] [--prompt 128]
                      [--gen 512] [--flags 15] [--out profiles/r04/parity_x86.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))

import pyoracle as po  # noqa: E402


def top2(v: np.ndarray):
    i = int(np.argmax(v))
    w = v.copy()
    w[i] = -np.inf
    return i, float(v[i] - w.max())


def run(path: str, n_prompt: int, n_gen: int, flags: int, seed: int = 21, threads: int = 0,
        n_vocab_prompt: int = 30000, ref_flags: int = 0) -> dict:
    rng = np.random.default_rng(seed)
    prompt = [1] + [int(t) for t in rng.integers(3, n_vocab_prompt, n_prompt - 1)]
    n_ctx = (n_prompt + n_gen + 255) // 256 * 256
    g = po.OracleModel(path, n_ctx=n_ctx, threads=threads, x86=ref_flags)
    x = po.OracleModel(path, n_ctx=n_ctx, threads=threads, x86=flags)
    prompt = [t % g.n_vocab for t in prompt]
    t0 = time.time()
    if n_prompt > 1:
        g.prefill(prompt[:-1])
        x.prefill(prompt[:-1])
    lg = g.decode(prompt[-1], n_prompt - 1)
    lx = x.decode(prompt[-1], n_prompt - 1)
    diffs, first, mism = [], None, 0
    pos = n_prompt
    for step in range(n_gen + 1):
        d = float(np.abs(lg - lx).max())
        diffs.append(d)
        ig, mg = top2(lg)
        ix, mx = top2(lx)
        if ig != ix:
            mism += 1
            if first is None:
                first = {"step": step, "pos": pos - 1, "generic_id": ig, "x86_id": ix,
                         "generic_top2_margin": mg, "x86_top2_margin": mx, "abs_diff": d}
        if step == n_gen:
            break
        lg = g.decode(ig, pos)
        lx = x.decode(ig, pos)  # teacher-forced with the generic (= GPU) trajectory
        pos += 1
    g.close()
    x.close()
    a = np.array(diffs)
    return {"steps": len(diffs), "ctx_end": pos, "frac_within_1e-3": float(np.mean(a <= 1e-3)),
            "worst_abs_diff": float(a.max()), "median_abs_diff": float(np.median(a)),
            "p90_abs_diff": float(np.quantile(a, 0.9)), "first_id_divergence": first,
            "id_mismatch_steps": mism, "seconds": round(time.time() - t0, 1)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-8b-q4km")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--vocab", type=int, default=0, help="0 = the preset's full vocabulary")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--gen", type=int, default=512)
    ap.add_argument("--flags", type=int, default=po.X86_ALL)
    ap.add_argument("--ref-flags", type=int, default=0,
                    help="the reference run's oracle flags (0 = generic; e.g. 64 = generic + flash attention): "
                         "the trajectory is teacher-forced with ITS ids; the 'generic_*' fields then mean 'reference'")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--dir", default="/tmp/llmi_parity")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import llmi
    os.makedirs(args.dir, exist_ok=True)
    path = os.path.join(args.dir, f"{args.preset}-L{args.layers}-v{args.vocab}.gguf")
    if not os.path.exists(path):
        llmi.write_synthetic_gguf(path, args.preset, seed=3, n_layer=args.layers, n_vocab=args.vocab)
    po.prefer_simd()
    rep = {"preset": args.preset, "n_layer": args.layers, "n_vocab": args.vocab or "full",
           "prompt": args.prompt, "gen": args.gen, "x86_flags": args.flags, "ref_flags": args.ref_flags,
           "x86_parts": [n for n, b in (("dots", po.X86_DOTS), ("q8_0", po.X86_Q80), ("f16dot", po.X86_F16DOT),
                                        ("v_expf", po.X86_VEXP), ("libm_expf", po.X86_LIBM),
                                        ("no_fma", po.X86_NOFMA), ("flash_attn", po.X86_FA)) if args.flags & b],
           "ref_parts": [n for n, b in (("dots", po.X86_DOTS), ("q8_0", po.X86_Q80), ("f16dot", po.X86_F16DOT),
                                        ("v_expf", po.X86_VEXP), ("flash_attn", po.X86_FA)) if args.ref_flags & b] or ["generic"],
           "note": "generic (== GPU bit for bit) vs upstream x86 AVX2 association as restated in "
                   "oracle/ggml_oracle.c (recalled, not vendored); teacher-forced with the generic ids"}
    rep.update(run(path, args.prompt, args.gen, args.flags, threads=args.threads, ref_flags=args.ref_flags))
    line = json.dumps(rep)
    print(line, flush=True)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "a") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
