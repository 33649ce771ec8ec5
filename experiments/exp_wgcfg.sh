#!/bin/bash
# LLMI_WG_PER_CU A/B on the headline and the small-model configs.
set -u
OUT=${1:-gpurun_out/wgcfg}
mkdir -p "$OUT"
for w in ${WGS:-4 2}; do
  for p in llama3-8b-q4km tinyllama-q8_0 mistral7b-q6k llama3-8b-q4km; do
    LLMI_WG_PER_CU=$w timeout -k 10 240 python bench.py --no-cpu-baseline --preset $p > "$OUT/$p.$w.json" 2> "$OUT/$p.$w.err" || { tail "$OUT/$p.$w.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$p.$w.json'));print('wg$w $p', d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
  done
done
