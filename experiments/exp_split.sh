#!/bin/bash
# QKV type-group deal: by per-wave bytes (default) vs by pair count (LLMI_SPLIT_BY_PAIRS=1)
set -o pipefail
O=gpurun_out/split; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 0 1; do
    LLMI_SPLIT_BY_PAIRS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs '' > $O/b${v}_$r.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.load(open('$O/b${v}_$r.json')); print('by_pairs=$v run $r', d['value'], 'qkv', d['kernels']['qkv'])"
  done
done
