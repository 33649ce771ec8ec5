#!/bin/bash
# Round-4 prefill checks: the prefill attention parity tests, then the kernel-level
# attention bench and TTFT (tools/prefillbench.py) of the configs' prompts.
# usage: tools/r4_pf.sh [tests|bench|ttft|all] [out dir]
set -u
WHAT=${1:-all}; OUT=${2:-gpurun_out/r4pf}
mkdir -p "$OUT"
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_pf_attention.py tests/test_gpu_prefill.py tests/test_gpu_long.py > "$OUT/tests.txt" 2>&1 \
      || { tail -30 "$OUT/tests.txt"; exit 1; }
  tail -3 "$OUT/tests.txt"
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  timeout -k 10 300 python -u tools/pfattn_bench.py 32,8,128 512 0,1536,7680,15872 0,1 > "$OUT/pfattn_8b.json" 2> "$OUT/pfattn_8b.log" \
      || { tail -5 "$OUT/pfattn_8b.log"; exit 2; }
  cat "$OUT/pfattn_8b.log"
fi
if [ "$WHAT" = ttft ] || [ "$WHAT" = all ]; then
  PF_GEMM_T=512 timeout -k 10 600 python -u tools/prefillbench.py mistral7b-q6k 2048 > "$OUT/ttft_mistral.json" 2> "$OUT/ttft_mistral.log" \
      || { tail -5 "$OUT/ttft_mistral.log"; exit 3; }
  grep "n=" "$OUT/ttft_mistral.log"
  PF_GEMM_T=512 timeout -k 10 900 python -u tools/prefillbench.py llama3-8b-q4km 2048,16384 > "$OUT/ttft_8b.json" 2> "$OUT/ttft_8b.log" \
      || { tail -5 "$OUT/ttft_8b.log"; exit 4; }
  grep "n=" "$OUT/ttft_8b.log"
fi
