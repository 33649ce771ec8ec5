#!/bin/bash
# k_pf_gemm 32- vs 64-token workgroups (test option pf_gemm_ng): Mistral-7B Q6_K and
# Llama-3-8B Q4_K_M 2048-token TTFT and the GEMM shapes alone at T = 512.
set -u
OUT=${1:-gpurun_out/r4ng}; mkdir -p "$OUT"
for p in mistral7b-q6k llama3-8b-q4km; do
  for ng in 1 2; do
    PF_GEMM_NG=$ng PF_GEMM_T=512 timeout -k 10 400 python -u tools/prefillbench.py $p 2048 > "$OUT/${p}_ng$ng.json" \
        2> "$OUT/${p}_ng$ng.log" || { tail -5 "$OUT/${p}_ng$ng.log"; exit 1; }
    echo "== $p ng=$ng"; grep "n=\|gemm" "$OUT/${p}_ng$ng.log"
  done
done
