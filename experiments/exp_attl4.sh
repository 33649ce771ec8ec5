#!/bin/bash
# Long-context attention: NP by size; per-kernel durations per context size.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/attl4; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_decode.py::test_attention_paths_bit_exact" \
  "tests/test_gpu_long.py::test_decode_past_4096_positions" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sh in 32,8,128 64,8,128 32,4,64; do
  ATT_SHAPE=$sh ATT_KV=1024,1536,2048,3072,4096,8192,16384 ATT_MODES=0,7 ATT_REPS=10 timeout -k 10 200 python -u tools/attnbench.py > $O/bench_$sh.log 2>&1 || { tail $O/bench_$sh.log; exit 1; }
  echo "== $sh"; grep n_kv $O/bench_$sh.log
done
ATT_SHAPE=32,8,128 ATT_KV=1024,2048,4096 ATT_MODES=7 ATT_REPS=10 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 tools/attnbench.py > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
