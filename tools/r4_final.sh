#!/bin/bash
# Round-end check of the tree: smoke(), the whole GPU test suite, the default bench line
# (with the CPU baseline leg).
set -u
OUT=${1:-gpurun_out/r4final}; mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.txt"
[ $rc -ne 0 ] && { grep -E "FAILED|ERROR" "$OUT/gpu_tests.txt" | head -20; exit 2; }
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 3; }
tail -1 "$OUT/bench_default.log" > "$OUT/bench_default.json"
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['roofline']['frac'], json.dumps(d.get('cpu_baseline'))[:300])"
