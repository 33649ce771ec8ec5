#!/bin/bash
# One GPU session: gpu tests, default bench, rocprofv3 kernel-trace of a short bench.
# Stops at the first step that faults / aborts / times out (exit >= 2 except pytest's 1).
set -u
OUT=${1:-gpurun_out/r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "gpu tests exit=$rc" | tee -a "$OUT/gpu_tests.log"
tail -3 "$OUT/gpu_tests.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit=$rc"; cat "$OUT/bench.json"
if [ $rc -ne 0 ]; then tail -20 "$OUT/bench.err"; exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 64 --warmup 8 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
rc=$?; echo "rocprof exit=$rc"
exit $rc
