#!/bin/bash
# Prefill GEMM with every lane reading its wave's first row (LLMI_PF_EXP=1: hot, coalesced
# weights; results garbage) vs the real access pattern: TTFT and the GEMM shapes
set -u
for e in 0 1; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_exp.so LLMI_PF_EXP=$e PF_GEMM_T=512 timeout -k 10 300 python -u tools/prefillbench.py mistral7b-q6k 2048 2>&1 | grep "prefillbench" | sed "s/^/exp=$e /" || exit 1
done
