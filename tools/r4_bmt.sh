#!/bin/bash
# Batched decode A/B: k_bmt (default) vs k_bmm (LLMI_BMT=0) -- batch tests, then the
# bench's continuous_batching leg at 8 sequences (8B), with a rocprof stats pass.
set -u
OUT=${1:-gpurun_out/r4bmt}; R=$(pwd); mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py > "$OUT/tests.txt" 2>&1 \
    || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for v in 1 0; do
  LLMI_BMT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 16 --warmup 4 --profile-steps 0 --no-c2-full \
      --batch-seqs 2,4,8 > "$OUT/bench_bmt$v.log" 2>&1 || { tail -5 "$OUT/bench_bmt$v.log"; exit 2; }
  tail -1 "$OUT/bench_bmt$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BMT=$v', json.dumps(d.get('continuous_batching')))"
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 8 --warmup 2 --profile-steps 0 --no-c2-full --batch-seqs 8 \
    > "$R/$OUT/prof.log" 2>&1 ) || { tail -5 "$OUT/prof.log"; exit 3; }
find "$OUT/prof" -name "*kernel_trace.csv" -size +2M -delete
python3 - "$OUT/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.1f} ms n={r["Calls"]:>6} avg={float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
PY
