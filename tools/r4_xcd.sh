#!/bin/bash
# k_pf_gemm XCD-aware tile order (pf_xcd_map): prefill parity, then TTFT 2048 and the GEMM
# shapes at T = 512 with the order off / on, then the FETCH_SIZE pass (order on).
set -u
OUT=${1:-gpurun_out/r4xcd}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_prefill.py \
    tests/test_gpu_long.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for m in 2 4; do
  LLMI_TEST_OPTIONS=pf_xcd_map=$m timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_prefill.py > "$OUT/tests_m$m.txt" 2>&1 || { tail -30 "$OUT/tests_m$m.txt"; exit 1; }
  echo "xcd_map=$m: $(tail -1 "$OUT/tests_m$m.txt")"
done
for p in mistral7b-q6k llama3-8b-q4km; do
  for m in 1 2 4; do
    PF_XCD_MAP=$m PF_GEMM_T=512 timeout -k 10 400 python -u tools/prefillbench.py $p 2048 > "$OUT/${p}_m$m.json" \
        2> "$OUT/${p}_m$m.log" || { tail -5 "$OUT/${p}_m$m.log"; exit 2; }
    echo "== $p xcd_map=$m"; grep "n=\|gemm" "$OUT/${p}_m$m.log"
  done
done

