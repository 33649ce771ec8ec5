#!/bin/bash
# Sweep of the resident workgroups per CU (LLMI_WG_PER_CU) on the matvec shapes and e2e.
set -u
OUT=${1:-gpurun_out/wg}
mkdir -p "$OUT"
for w in 1 2 3 4 8; do
  LLMI_WG_PER_CU=$w MV_SHAPES=12:4096x4096,12:6144x4096,12:28672x4096,14:128256x4096 MV_REPS=400 timeout -k 10 120 python tools/mvbench.py > "$OUT/mv_$w.log" 2>&1 || exit $?
  echo "== wg/cu $w"; grep GBps "$OUT/mv_$w.log" | grep -v '^{' | cut -c1-80
  LLMI_WG_PER_CU=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 256 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail "$OUT/bench_$w.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$w.json'));print(d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
done
