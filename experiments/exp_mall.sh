#!/bin/bash
# Experiment: matvec time with weights MALL-resident (one copy replayed) vs cold
# (rotating over >1 GB), plus the attention paths at short context.
set -u
OUT=${1:-gpurun_out/mall}
mkdir -p "$OUT"
export MV_SHAPES=12:4096x4096,12:6144x4096,12:28672x4096,12:4096x14336 MV_REPS=400
timeout -k 10 120 python tools/mvbench.py > "$OUT/cold.log" 2>&1 || exit $?
MV_NCOPIES=1 timeout -k 10 120 python tools/mvbench.py > "$OUT/hot.log" 2>&1 || exit $?
MV_NCOPIES=8 timeout -k 10 120 python tools/mvbench.py > "$OUT/hot8.log" 2>&1 || exit $?
ATT_KV=128,384,640,1024,2048 timeout -k 10 120 python tools/attnbench.py > "$OUT/attn.log" 2>&1 || exit $?
grep -h GBps "$OUT"/cold.log "$OUT"/hot.log "$OUT"/hot8.log | grep -v '^{'
cat "$OUT/attn.log"
