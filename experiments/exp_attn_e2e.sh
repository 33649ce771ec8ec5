#!/bin/bash
# Attention path A/B end to end on the headline bench (LLMI_ATTN_MODE: 0 auto, 1 fused,
# 2 split, 4 one-launch exchange).
set -u
OUT=${1:-gpurun_out/attn_e2e}
mkdir -p "$OUT"
for m in 0 4 2 1 0; do
  LLMI_ATTN_MODE=$m timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/m$m.json" 2> "$OUT/m$m.err" || { tail "$OUT/m$m.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/m$m.json'));print('mode$m', d['value'], d['kernels']['attention']['us'])"
done
