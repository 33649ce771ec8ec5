#!/bin/bash
# Single-round matvec launches with their weights issued before the activation arrives
# (mode bit 8) vs after (default), cold weights
set -u
for sh in "attn_out 64 12:4096x4096" "qkv 1 12:6144x4096" "down 64 12:4096x14336" "down6 64 14:4096x14336"; do
  set -- $sh
  for m in $2 $((256 + $2)); do
    MV_MODE=$m MV_SHAPES="$3" MV_REPS=64 timeout -k 10 120 python -u tools/mvbench.py 2>/dev/null | grep -v "^{" | sed "s|^|$1 mode=$m |" | cut -c1-90 || exit 1
  done
done
