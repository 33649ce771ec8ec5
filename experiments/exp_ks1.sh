#!/bin/bash
# K-split width 1 for rows of >= 6 items (70B ffn_down, 28672 columns): parity + A/B.
set -u
OUT=${1:-gpurun_out/ks1}
mkdir -p "$OUT"
export LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_ks1.so
LLMI_KS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q -k "real_widths" --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for k in 0 1 0 1; do
  LLMI_KS=$k timeout -k 10 400 python bench.py --no-cpu-baseline --preset llama3-70b-q4km --steps 128 --warmup 8 > "$OUT/b$k.json" 2> "$OUT/b$k.err" || { tail "$OUT/b$k.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$k.json'));print('ks$k', d['value'], d['kernels']['ffn_down']['us'])"
done
