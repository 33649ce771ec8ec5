#!/bin/bash
# k_attn_d (mode 6) vs the other attention paths: parity tests, then attnbench per shape.
set -o pipefail
mkdir -p gpurun_out/attd
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_decode.py::test_attention_paths_bit_exact" \
  "tests/test_gpu_decode.py::test_register_attention_all_buckets" \
  "tests/test_gpu_decode.py::test_dim_split_attention_long_buckets" \
  "tests/test_gpu_prefill.py::test_attention_variants_agree_long_context" > gpurun_out/attd/tests.log 2>&1 || { tail -30 gpurun_out/attd/tests.log; exit 1; }
tail -3 gpurun_out/attd/tests.log
for sh in 32,8,128 64,8,128 32,4,64; do
  ATT_SHAPE=$sh ATT_KV=128,256,384,512,640,768,1024 ATT_MODES=${ATT_MODES:-1,2,4,5,6} timeout -k 10 120 python -u tools/attnbench.py > gpurun_out/attd/bench_$sh.log 2>&1 || exit 1
  echo "== $sh"; grep n_kv gpurun_out/attd/bench_$sh.log
done
