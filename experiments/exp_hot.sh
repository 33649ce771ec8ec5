#!/bin/bash
# Matvec launch time with its weights cache-hot (every launch of the graph reads copy 0,
# mode bit 7) vs cold (>= 1.2 GB of copies rotated): what the first sub-item's HBM latency
# costs a launch.  O (ADD), QKV (norm), down (ADD), gate+up (SwiGLU).
set -u
O=${1:-gpurun_out/hot}; mkdir -p "$O"
run() {  # name mode shape copies
  MV_NCOPIES=$4 MV_MODE=$2 MV_SHAPES="$3" MV_REPS=64 timeout -k 10 120 python -u tools/mvbench.py 2>/dev/null | grep -v "^{" | sed "s/^/$1 mode=$2 nc=$4 /"
}
for sh in "attn_out 64 12:4096x4096" "qkv 1 12:6144x4096" "down 64 12:4096x14336" "gate_up 32 12:28672x4096"; do
  set -- $sh
  run $1 $2 $3 0 || exit 1
  run $1 $((128 + $2)) $3 8 || exit 1
done
