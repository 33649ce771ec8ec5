#!/bin/bash
# k_attn_d: loads of the whole KV bucket (default) vs position-first bounded loads (LLMI_ATTN_PF=1)
set -o pipefail
O=gpurun_out/attpf; mkdir -p $O
LLMI_ATTN_PF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
  "tests/test_gpu_decode.py::test_attention_paths_bit_exact" "tests/test_gpu_decode.py::test_register_attention_all_buckets" \
  "tests/test_gpu_decode.py::test_dim_split_attention_long_buckets" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sh in 32,8,128 64,8,128 32,4,64; do
  for pf in 0 1; do
    LLMI_ATTN_PF=$pf ATT_SHAPE=$sh ATT_KV=200,256,300,400,512,520,600,700,768,800,1000 ATT_MODES=6 timeout -k 10 120 python -u tools/attnbench.py > $O/${sh}_pf$pf.log 2>&1 || exit 1
  done
  echo "== $sh"; paste <(grep n_kv $O/${sh}_pf0.log | awk '{print $2, $7}') <(grep n_kv $O/${sh}_pf1.log | awk '{print $7}')
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs '' > $O/b0.json 2>/dev/null && LLMI_ATTN_PF=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs '' > $O/b1.json 2>/dev/null || exit 1
python3 -c "
import json
for f in ('$O/b0.json','$O/b1.json'):
    d=json.load(open(f)); print(f, d['value'], d['kernels']['attention'])"
