#!/bin/bash
# k_attn_d: K passes in the same order on every workgroup (default) vs rotated per workgroup (LLMI_ATTN_ROT=1)
set -o pipefail
O=gpurun_out/attrot2; mkdir -p $O
LLMI_ATTN_ROT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
  "tests/test_gpu_decode.py::test_attention_paths_bit_exact" "tests/test_gpu_decode.py::test_register_attention_all_buckets" \
  "tests/test_gpu_decode.py::test_dim_split_attention_long_buckets" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sh in 32,8,128 64,8,128 32,4,64; do
  for v in 0 1 2; do
    LLMI_ATTN_ROT=$v ATT_SHAPE=$sh ATT_KV=256,400,512,700,768,1000 ATT_MODES=6 timeout -k 10 120 python -u tools/attnbench.py > $O/${sh}_r$v.log 2>&1 || exit 1
  done
  echo "== $sh"; paste <(grep n_kv $O/${sh}_r0.log | awk "{print \$2, \$7}") <(grep n_kv $O/${sh}_r1.log | awk "{print \$7}") <(grep n_kv $O/${sh}_r2.log | awk "{print \$7}")
done
