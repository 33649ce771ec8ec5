#!/bin/bash
# Launch-shape sweep: LLMI_WG_PER_CU values, matvec microbench per shape + headline bench.
set -u
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
for w in ${WGS:-1 2 3 4}; do
  LLMI_WG_PER_CU=$w MV_SHAPES=${MV_SHAPES:-12:4096x4096,12:6144x4096,12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096} MV_REPS=400 \
    timeout -k 10 120 python tools/mvbench.py > "$OUT/mv$w.log" 2>&1 || { tail "$OUT/mv$w.log"; exit 1; }
  grep GBps "$OUT/mv$w.log" | grep -v '^{' | cut -c1-40 | sed "s/^/wg$w /"
  LLMI_WG_PER_CU=$w timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/wg$w.json" 2> "$OUT/wg$w.err" || { tail "$OUT/wg$w.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/wg$w.json'));print('wg$w', d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
done
