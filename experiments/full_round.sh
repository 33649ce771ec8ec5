#!/bin/bash
# full GPU gate: every -m gpu test, smoke(), the default bench line, rocprof stats + FETCH_SIZE
set -u
OUT=${1:-gpurun_out/full}; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
bash tools/bench_profile.sh "$OUT/prof" llama3-8b-q4km > "$OUT/prof.log" 2>&1 || exit $?
