#!/bin/bash
# prefill GEMM: parity (pf_gemm == matvec, prefill logits) then speed (tools/prefillbench.py);
# batched decode + server tests; HTTP serving bench (benchmark.py shape) on TinyLlama shapes
set -u
OUT=${1:-gpurun_out/pf}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_prefill.py \
    tests/test_gpu_batch.py tests/test_gpu_server.py > "$OUT/t.log" 2>&1 || exit $?
timeout -k 10 300 python tools/prefillbench.py llama3-8b-q4km 128,512,2048 > "$OUT/pb.log" 2>&1 || exit $?
timeout -k 10 300 python tools/http_bench.py --serve llama3-8b-q4km --slots 8 --concurrency 1,4,8 --requests 16 \
    --max-tokens 128 > "$OUT/http.json" 2> "$OUT/http.err" || exit $?
