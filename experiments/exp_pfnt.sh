#!/bin/bash
# Prefill weight loads: temporal (product build) vs nontemporal (LLMI_PF_NT=1 build as libllmi_exp.so)
set -u
for lib in libllmi.so libllmi_exp.so; do
  for p in mistral7b-q6k llama3-8b-q4km; do
    LLMI_LIB=llama-gguf-inference_amd/lib/$lib PF_GEMM_T=512 timeout -k 10 300 python -u tools/prefillbench.py $p 2048 2>&1 | grep "prefillbench" | sed "s/^/$lib /" || exit 1
  done
done
