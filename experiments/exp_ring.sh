#!/bin/bash
# 3-deep matvec ring: parity (decode + kernels) then A/B (ring vs ring-off) mvbench + bench
set -u
OUT=${1:-gpurun_out/ring}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
    tests/test_gpu_decode.py > "$OUT/t.log" 2>&1 || exit $?
for lib in libllmi libllmi_ring0 libllmi; do
  MV_MODE=1 MV_SHAPES=12:28672x4096,12:6144x4096,12:4096x4096,14:4096x14336 LLMI_LIB=llama-gguf-inference_amd/lib/$lib.so \
    timeout -k 10 200 python tools/mvbench.py >> "$OUT/mv.log" 2>&1 || exit $?
  MV_MODE=3 MV_SHAPES=14:128256x4096 LLMI_LIB=llama-gguf-inference_amd/lib/$lib.so \
    timeout -k 10 200 python tools/mvbench.py >> "$OUT/mv.log" 2>&1 || exit $?
  LLMI_LIB=llama-gguf-inference_amd/lib/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --batch-seqs= \
    --steps 256 >> "$OUT/bench.json" 2>> "$OUT/bench.err" || exit $?
done
