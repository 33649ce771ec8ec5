#!/bin/bash
# Grid sweep per matvec shape (LLMI_MV_BLOCKS = workgroups of 256 threads).
set -u
OUT=${1:-gpurun_out/blocks}
mkdir -p "$OUT"
sweep() {  # shape, block counts...
  local sh=$1; shift
  for b in "$@"; do
    LLMI_MV_BLOCKS=$b MV_SHAPES=$sh MV_REPS=400 timeout -k 10 60 python tools/mvbench.py > "$OUT/mv_${sh//[:x]/_}_$b.log" 2>&1 || { tail "$OUT/mv_${sh//[:x]/_}_$b.log"; exit 1; }
    echo "$sh blocks=$b $(grep GBps "$OUT/mv_${sh//[:x]/_}_$b.log" | grep -v '^{' | cut -c1-45)"
  done
}
sweep 12:6144x4096 256 384 512 640 768
sweep 12:28672x4096 512 640 768 896 1024
sweep 14:128256x4096 384 512 640 768 1024
sweep 12:4096x4096 256 384 512
