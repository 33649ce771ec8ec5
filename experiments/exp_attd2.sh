#!/bin/bash
# Round 2: full GPU suite with k_attn_d as the auto path, slice-count A/B, default bench.
set -o pipefail
O=gpurun_out/attd2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for sh in 32,8,128 64,8,128 32,4,64; do
  for S in 2 4 8; do
    LLMI_ATTN_S=$S ATT_SHAPE=$sh ATT_KV=128,256,512,768,1024 ATT_MODES=6 timeout -k 10 120 python -u tools/attnbench.py > $O/ab_${sh}_S$S.log 2>&1 || exit 1
    echo "== $sh S=$S"; grep n_kv $O/ab_${sh}_S$S.log
  done
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
