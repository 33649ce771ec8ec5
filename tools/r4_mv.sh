#!/bin/bash
# Matvec shapes of the 8B decode step in isolation (tools/mvbench.py): burst off / on,
# rotating >= 1.2 GB of weight copies (HBM) and one copy (Infinity-Cache resident).
set -u
OUT=${1:-gpurun_out/mv}; mkdir -p "$OUT"
export TMPDIR=/tmp
SH="12:28672x4096,12:4096x14336,14:4096x14336,12:4096x4096,12:6144x4096"
run() {  # name env... -- mode
  local name=$1; shift
  timeout -k 10 240 env "$@" python tools/mvbench.py > "$OUT/$name.txt" 2> "$OUT/$name.err"
  local rc=$?; echo "$name rc=$rc"; grep -v '^{' "$OUT/$name.txt" | sed 's/^/  /'
  return $rc
}
run swiglu_b0 LLMI_MV_BURST=0 MV_MODE=33 MV_SHAPES=12:28672x4096 && \
run swiglu_b4 MV_MODE=33 MV_SHAPES=12:28672x4096 && \
run add_b0 LLMI_MV_BURST=0 MV_MODE=64 MV_SHAPES=12:4096x14336,14:4096x14336,12:4096x4096 && \
run add_b4 MV_MODE=64 MV_SHAPES=12:4096x14336,14:4096x14336,12:4096x4096 && \
run norm_b0 LLMI_MV_BURST=0 MV_MODE=1 MV_SHAPES=12:6144x4096 && \
run norm_b4 MV_MODE=1 MV_SHAPES=12:6144x4096 && \
run swiglu_b4_mall MV_NCOPIES=1 MV_MODE=33 MV_SHAPES=12:28672x4096 && \
run add_b4_mall MV_NCOPIES=1 MV_MODE=64 MV_SHAPES=12:4096x14336,14:4096x14336,12:4096x4096
