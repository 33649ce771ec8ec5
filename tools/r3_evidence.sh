#!/bin/bash
# Round-3 evidence on one GPU box (via gpurun).  Part A: smoke, default bench, rocprof
# stats + FETCH_SIZE of the headline preset, and one graph-replay --pmc pass (the round-2
# profiler SIGSEGV check).  Part B: the 70B preset's bench + rocprof, the other configs.
set -u
PART=${1:-A}; OUT=${2:-gpurun_out/r3ev}
mkdir -p "$OUT"; export TMPDIR=/tmp
R=$(pwd)
if [ "$PART" = A ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 2
  bash tools/bench_profile.sh "$OUT/prof8b" llama3-8b-q4km > "$OUT/prof8b.log" 2>&1 || exit 3
  # graph replay under --pmc (round 2 saw a host SIGSEGV here): outcome recorded, not fatal
  ( cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/pmc_graph" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline --batch-seqs= --steps 20 --warmup 16 --profile-steps 0 \
      > "$R/$OUT/pmc_graph.json" 2> "$R/$OUT/pmc_graph.err"; echo "pmc_graph rc=$?" > "$R/$OUT/pmc_graph.rc" )
else
  timeout -k 10 600 python -u bench.py --preset llama3-70b-q4km --prompt 8 --steps 128 --warmup 8 --no-cpu-baseline \
      > "$OUT/bench_70b.json" 2> "$OUT/bench_70b.err" || exit 4
  bash tools/bench_configs.sh "$OUT/cfg" > "$OUT/cfg.log" 2>&1 || exit 5
fi
