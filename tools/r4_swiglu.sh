#!/bin/bash
# Prefill gate+up fused (default) vs two launches (LLMI_PF_SWIGLU=0): prefill tests, TTFT.
set -u
OUT=${1:-gpurun_out/r4sw}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_prefill.py tests/test_gpu_long.py > "$OUT/tests.txt" 2>&1 \
    || { tail -20 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for v in 1 0; do
  LLMI_PF_SWIGLU=$v PF_GEMM_T=512 timeout -k 10 300 python -u tools/prefillbench.py mistral7b-q6k 2048 > "$OUT/m_$v.json" 2> "$OUT/m_$v.log" || exit 2
  LLMI_PF_SWIGLU=$v PF_GEMM_T=512 timeout -k 10 300 python -u tools/prefillbench.py llama3-8b-q4km 2048 > "$OUT/l_$v.json" 2> "$OUT/l_$v.log" || exit 3
  echo "== fused $v"; grep -h "n=" "$OUT/m_$v.log" "$OUT/l_$v.log"
done
