#!/bin/bash
# Round-4 evidence: per config a rocprofv3 --kernel-trace
# --stats pass and a --pmc FETCH_SIZE pass (tools/bench_profile.sh), then the config's
# bench line carrying that traffic and the rocprof duration; decode-matvec SQ counters
# of the headline preset.  Part A: 8B + TinyLlama + Mistral Q6_K / Q5_K_M (+ the 2048-token
# prefill line); part B: 70B.
set -u
PART=${1:-A}; OUT=${2:-gpurun_out/r4ev}
mkdir -p "$OUT"; export TMPDIR=/tmp
R=$(pwd)
prof_and_bench() {  # preset, extra bench args...
  local p=$1; shift
  bash tools/bench_profile.sh "$OUT/prof_$p" "$p" > "$OUT/prof_$p.log" 2>&1 || { echo "profile $p failed"; tail -5 "$OUT/prof_$p.log"; return 1; }
  find "$OUT/prof_$p" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +2M -delete
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --preset "$p" --profile-dir "$OUT/prof_$p" "$@" \
      > "$OUT/bench_$p.log" 2>&1 || { echo "bench $p failed"; tail -5 "$OUT/bench_$p.log"; return 1; }
  tail -1 "$OUT/bench_$p.log" > "$OUT/bench_$p.json"
  python3 -c "import json; d=json.load(open('$OUT/bench_$p.json')); r=d['roofline']; print('$p', d['value'], 'frac', r['frac'], 'rocprof_frac', r.get('rocprof_frac'), 'traffic', r.get('traffic'))"
}
if [ "$PART" = A ]; then
  prof_and_bench llama3-8b-q4km || exit 1
  prof_and_bench tinyllama-q8_0 || exit 1
  prof_and_bench mistral7b-q6k || exit 1
  prof_and_bench mistral7b-q5km || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --preset mistral7b-q6k --prompt 2048 --steps 256 \
      --profile-dir "$OUT/prof_mistral7b-q6k" > "$OUT/bench_mistral7b-q6k-p2048.log" 2>&1 || exit 2
  tail -1 "$OUT/bench_mistral7b-q6k-p2048.log" > "$OUT/bench_mistral7b-q6k-p2048.json"
  # decode-matvec SQ counters (eager launches; one --pmc pass per counter group)
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  ( cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/$OUT/sq" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline --batch-seqs= --eager --steps 8 --warmup 4 --profile-steps 0 \
      > "$R/$OUT/sq.json" 2> "$R/$OUT/sq.err" ) || exit 3
  python3 tools/sq_summary.py "$OUT/sq" k_matvec > "$OUT/sq_summary.json" 2>&1 || true
  find "$OUT/sq" -name "*counter_collection.csv" -size +2M -delete
fi
if [ "$PART" = B ]; then
  prof_and_bench llama3-70b-q4km --prompt 8 --steps 128 --warmup 8 || exit 4
fi
