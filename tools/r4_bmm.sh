#!/bin/bash
# k_bmm after a change: the batch tests, then the bench's continuous_batching leg (8B and
# 70B at 2 / 4 / 8 sequences).
set -u
OUT=${1:-gpurun_out/r4bmm}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py > "$OUT/tests.txt" 2>&1 \
    || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for p in llama3-8b-q4km llama3-70b-q4km; do
  a="--prompt 128"; [ $p = llama3-70b-q4km ] && a="--prompt 8"
  timeout -k 10 500 python -u bench.py --no-cpu-baseline --preset $p $a --steps 16 --warmup 4 --profile-steps 0 --no-c2-full \
      --batch-seqs 2,4,8 > "$OUT/bench_$p.log" 2>&1 || { tail -5 "$OUT/bench_$p.log"; exit 2; }
  tail -1 "$OUT/bench_$p.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', d['value'], json.dumps(d.get('continuous_batching',{}).get('sequences')))"
done
