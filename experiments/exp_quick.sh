#!/bin/bash
# quick GPU check: full gpu test suite, matvec microbench, e2e bench (no CPU baseline)
set -u
OUT=${1:-gpurun_out/quick}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > "$OUT/tests.log" 2>&1; rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
MV_SHAPES=${MV_SHAPES:-12:4096x4096,12:6144x4096,12:28672x4096,12:4096x14336} MV_REPS=400 timeout -k 10 120 python tools/mvbench.py > "$OUT/mv.log" 2>&1 || { cat "$OUT/mv.log"; exit 1; }
grep GBps "$OUT/mv.log" | grep -v '^{' | cut -c1-60
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], {k:v['us'] for k,v in d['kernels'].items()})"
