#!/bin/bash
# rocprof evidence for bench.py's roofline line: one
# --kernel-trace --stats pass and one --pmc FETCH_SIZE pass (separate runs, as the
# MI355X guide prescribes) over the same bench command, then
# tools/make_traffic.py -> traffic_<preset>.json (per-launch HBM bytes of the dominant
# kernel, x2 gfx950 FETCH_SIZE correction) + kernel_stats.csv.
set -u
OUT=${1:-gpurun_out/benchprof}; PRESET=${2:-llama3-8b-q4km}
ROOT=$(pwd)
mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS="--preset $PRESET --no-cpu-baseline --batch-seqs= --steps 100 --warmup 16 --profile-steps 0"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/stats.json" 2> "$ROOT/$OUT/stats.err" ) || exit $?
# counters on eager launches (graph replays under --pmc crashed the profiler's host side)
( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$ROOT/$OUT/pmc" -o run -- \
    python3 "$ROOT/bench.py" $ARGS --eager --steps 20 > "$ROOT/$OUT/pmc.json" 2> "$ROOT/$OUT/pmc.err" ) || exit $?
python3 tools/make_traffic.py "$OUT" "$PRESET"
