#!/bin/bash
# new tests + the per-config bench lines (round 2)
set -u
OUT=${1:-gpurun_out/cfg2}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py \
    tests/test_gpu_kernels.py -k "past_attention or ks1_multi" > "$OUT/t.log" 2>&1 || exit $?
bash tools/bench_configs.sh "$OUT" > "$OUT/cfg.log" 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline --preset llama3-70b-q4km --steps 128 --warmup 8 --batch-seqs 8 \
    --batch-steps 16 > "$OUT/llama3-70b.json" 2> "$OUT/llama3-70b.err" || exit $?
