#!/bin/bash
# Matvec launch time without the per-weight integer VALU (LLMI_EXP_NOVALU build as
# libllmi_exp.so, Q4_K only) beside the product build: is the launch VALU-bound?
set -u
for lib in llama-gguf-inference_amd/lib/libllmi.so llama-gguf-inference_amd/lib/libllmi_exp.so; do
  for sh in "attn_out 64 12:4096x4096" "qkv 1 12:6144x4096" "down 64 12:4096x14336" "gate_up 32 12:28672x4096" "out 3 12:128256x4096"; do
    set -- $sh
    LLMI_LIB=$lib MV_MODE=$2 MV_SHAPES="$3" MV_REPS=64 timeout -k 10 120 python -u tools/mvbench.py 2>/dev/null | grep -v "^{" | sed "s|^|$(basename $lib) $1 |" || exit 1
  done
done
