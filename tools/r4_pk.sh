#!/bin/bash
# A/B of the prefill chains' packed f32 ops (lib/libllmi.so) against scalar ops
# (lib/libllmi_nopk.so: -fno-slp-vectorize -DLLMI_PK=0): GEMM shapes and Mistral TTFT.
set -u
OUT=${1:-gpurun_out/r4pk}; mkdir -p "$OUT"
for v in "" _nopk; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi$v.so PF_GEMM_T=512 timeout -k 10 300 python -u tools/prefillbench.py mistral7b-q6k 2048 \
      > "$OUT/pf$v.json" 2> "$OUT/pf$v.log" || { tail -5 "$OUT/pf$v.log"; exit 1; }
  echo "== lib$v"; grep "n=\|T=512" "$OUT/pf$v.log"
done
