#!/bin/bash
# ks kernel A/B: mvbench on the K-split shapes, then the GPU parity tests.
set -u
OUT=${1:-gpurun_out/ks}
mkdir -p "$OUT"
MV_SHAPES=12:4096x14336,14:4096x14336,12:8192x28672 MV_REPS=400 timeout -k 10 120 python tools/mvbench.py > "$OUT/mv.log" 2>&1 || exit $?
grep GBps "$OUT/mv.log" | grep -v '^{'
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > "$OUT/tests.log" 2>&1; rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], {k:v['us'] for k,v in d['kernels'].items()})"
