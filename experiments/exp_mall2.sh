#!/bin/bash
# MALL residency experiment: default-policy (LLMI_NT=0) weight loads, cold (rotating
# >1 GB) vs hot (8 copies, replayed: fits the 256 MB Infinity Cache for small shapes).
set -u
OUT=${1:-gpurun_out/mall2}
mkdir -p "$OUT"
export MV_SHAPES=12:4096x4096,12:6144x4096,12:28672x4096 MV_REPS=400
for lib in libllmi libllmi_nt0; do
  LLMI_LIB=llama-gguf-inference_amd/lib/$lib.so timeout -k 10 120 python tools/mvbench.py > "$OUT/cold_$lib.log" 2>&1 || exit $?
  LLMI_LIB=llama-gguf-inference_amd/lib/$lib.so MV_NCOPIES=8 timeout -k 10 120 python tools/mvbench.py > "$OUT/hot8_$lib.log" 2>&1 || exit $?
  LLMI_LIB=llama-gguf-inference_amd/lib/$lib.so MV_NCOPIES=24 timeout -k 10 120 python tools/mvbench.py > "$OUT/hot24_$lib.log" 2>&1 || exit $?
done
for f in "$OUT"/*.log; do echo "== $f"; grep GBps "$f" | grep -v '^{'; done
