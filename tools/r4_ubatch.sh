#!/bin/bash
# Prefill ubatch size A/B (LLMI_PF_UBATCH): TTFT of Mistral Q6_K 2048 and 8B 2048 / 16384.
set -u
OUT=${1:-gpurun_out/r4ub}; mkdir -p "$OUT"
for u in 512 1024 2048; do
  LLMI_PF_UBATCH=$u PF_GEMM_T=512 timeout -k 10 300 python -u tools/prefillbench.py mistral7b-q6k 2048 > "$OUT/m_$u.json" 2> "$OUT/m_$u.log" || { tail -3 "$OUT/m_$u.log"; exit 1; }
  LLMI_PF_UBATCH=$u PF_GEMM_T=512 timeout -k 10 400 python -u tools/prefillbench.py llama3-8b-q4km 2048,16384 > "$OUT/l_$u.json" 2> "$OUT/l_$u.log" || { tail -3 "$OUT/l_$u.log"; exit 2; }
  echo "== ubatch $u"; grep -h "n=" "$OUT/m_$u.log" "$OUT/l_$u.log"
done
