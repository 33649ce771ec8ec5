#!/bin/bash
# A/B of env settings on the e2e bench in one box: exp_ab.sh "VAR=a" "VAR=b" ...
set -u
OUT=gpurun_out/ab
mkdir -p "$OUT"
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 256 > "$OUT/b$i.json" 2> "$OUT/b$i.err" || { tail "$OUT/b$i.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$i.json'));print('$cfg', d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
done
