#!/bin/bash
# k_matvec_ks: weights issued after the activation arrives (LLMI_KS_XFIRST=1) vs during the prologue
set -o pipefail
O=gpurun_out/ksxf; mkdir -p $O
LLMI_KS_XFIRST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_decode.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 0 1; do
    LLMI_KS_XFIRST=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs '' > $O/b${v}_$r.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.load(open('$O/b${v}_$r.json')); print('ks_xfirst=$v run $r', d['value'], 'down', d['kernels']['ffn_down'])"
  done
done
for v in 0 1; do
  LLMI_KS_XFIRST=$v timeout -k 10 500 python -u bench.py --no-cpu-baseline --batch-seqs '' --preset llama3-70b-q4km --prompt 8 --steps 64 --warmup 4 > $O/b70_$v.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('$O/b70_$v.json')); print('70B ks_xfirst=$v', d['value'], 'down', d['kernels']['ffn_down'], 'gu', d['kernels']['ffn_gate_up'])"
done
