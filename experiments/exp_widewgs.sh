#!/bin/bash
# ffn_down shapes with one or two 8-wave workgroups per CU (LLMI_MV_WIDE_WGS), isolated and in the step
set -u
for w in 1 2; do
  LLMI_MV_WIDE_WGS=$w MV_MODE=64 MV_SHAPES=12:4096x14336,14:4096x14336 MV_REPS=64 timeout -k 10 120 python -u tools/mvbench.py 2>/dev/null | grep -v "^{" | cut -c1-60 | sed "s/^/wgs=$w /" || exit 1
  LLMI_MV_WIDE_WGS=$w timeout -k 10 300 python -u bench.py --batch-seqs "" --no-cpu-baseline --no-other-numerics > /tmp/b$w.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('/tmp/b$w.json').read().strip().splitlines()[-1]); print('wgs=$w', d['value'], d['c2_full']['tok_s'], {k: v['us'] for k, v in d['kernels'].items()})"
done
