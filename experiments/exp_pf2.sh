#!/bin/bash
set -u
OUT=${1:-gpurun_out/pf2}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_prefill.py \
    > "$OUT/t.log" 2>&1 || exit $?
timeout -k 10 300 python tools/prefillbench.py llama3-8b-q4km 128,512,2048 > "$OUT/pb.log" 2>&1 || exit $?
