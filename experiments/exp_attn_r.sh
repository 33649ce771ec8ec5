#!/bin/bash
# k_attn_r (mode 5) parity + microbench against fused (1) and exchange (4).
set -u
OUT=${1:-gpurun_out/a1}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_decode.py \
    -k "attention_paths or register_attention" > "$OUT/t.log" 2>&1 || exit $?
: > "$OUT/ab.log"
for shp in 32,8,128 32,4,128 64,8,128 32,4,64; do
  ATT_SHAPE=$shp ATT_MODES=1,4,5 ATT_KV=64,128,200,256,384,512 timeout -k 10 120 python tools/attnbench.py >> "$OUT/ab.log" 2>&1 || exit $?
done
