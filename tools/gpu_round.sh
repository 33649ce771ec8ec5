#!/bin/bash
# One GPU session producing the round's evidence (run on the box via gpurun):
#   1. pytest -m gpu (parity)                          -> $OUT/gpu_tests.log
#   2. python bench.py (default contract run)           -> $OUT/bench.json
#   3. rocprofv3 --kernel-trace --stats of the SAME command -> $OUT/prof/
#   4. rocprofv3 --pmc FETCH_SIZE (own pass) of a short bench -> $OUT/pmc_bench/
#   5. rocprofv3 --pmc FETCH_SIZE of the streaming-read calibration -> $OUT/pmc_cal/
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
OUT=${1:-gpurun_out/round}
STEPS=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@"
    local rc=$?
    echo "== $name exit=$rc" >&2
    return $rc
}
step tests 900 python -m pytest tests -m gpu -q -rf > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
step bench 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
[ "$STEPS" = "bench" ] && exit 0
step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -20 "$OUT/prof_bench.err"; exit 1; }
cat "$OUT/prof_bench.json"
step pmc_bench 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_bench" -o run --output-format csv -- \
    python3 bench.py --prompt 4 --steps 8 --warmup 2 --profile-steps 0 --no-cpu-baseline --eager \
    > "$OUT/pmc_bench.json" 2> "$OUT/pmc_bench.err" || { tail -20 "$OUT/pmc_bench.err"; exit 1; }
export MV_SHAPES=12:28672x4096 MV_REPS=5
step pmc_cal 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_cal" -o run \
    --output-format csv -- python3 tools/mvbench.py > "$OUT/pmc_cal.log" 2>&1 || { tail -20 "$OUT/pmc_cal.log"; exit 1; }
echo "all steps done"
