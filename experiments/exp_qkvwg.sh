#!/bin/bash
# QKV grid cap per CU (LLMI_QKV_WG_PER_CU 2 = default, 3: every QKV wave owns <= 1 pair, 4)
set -o pipefail
O=gpurun_out/qkvwg; mkdir -p $O
LLMI_QKV_WG_PER_CU=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_decode.py -k "parity or grid_cap" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 2 3 4; do
    LLMI_QKV_WG_PER_CU=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs '' > $O/b${v}_$r.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.load(open('$O/b${v}_$r.json')); print('qkv_wg=$v run $r', d['value'], 'qkv', d['kernels']['qkv'])"
  done
done
