#!/bin/bash
# Same-type q/k/v prefill GEMMs in one launch (pf_qkv_merge) on top of the XCD-aware tile
# order: prefill parity, then TTFT 2048 with the merge off / on (twice each).
set -u
OUT=${1:-gpurun_out/r4qkv2}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_prefill.py \
    tests/test_gpu_long.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -n 1 "$OUT/tests.txt"
for p in mistral7b-q6k llama3-8b-q4km; do
  for m in 0 1 0 1; do
    PF_QKV_MERGE=$m PF_GEMM_T=64 timeout -k 10 400 python -u tools/prefillbench.py $p 2048 >> "$OUT/${p}_m$m.json" \
        2>> "$OUT/${p}_m$m.log" || { tail -5 "$OUT/${p}_m$m.log"; exit 2; }
    echo "$p merge=$m: $(grep 'n=' "$OUT/${p}_m$m.log" | tail -n 1)"
  done
done
