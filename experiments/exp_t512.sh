#!/bin/bash
# 512-thread matvec workgroups at 1 per CU vs 256-thread at 2 per CU (same waves per CU).
set -u
OUT=${1:-gpurun_out/t512}
mkdir -p "$OUT"
T=llama-gguf-inference_amd/lib/libllmi_t512.so
LLMI_WG_PER_CU=1 LLMI_LIB=$T timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in base t512 base t512; do
  if [ $v = t512 ]; then export LLMI_LIB=$T LLMI_WG_PER_CU=1; else unset LLMI_LIB LLMI_WG_PER_CU; fi
  MV_SHAPES=12:28672x4096,12:6144x4096,12:4096x4096,14:128256x4096 MV_REPS=400 timeout -k 10 60 python tools/mvbench.py > "$OUT/mv_$v.log" 2>&1 || { tail "$OUT/mv_$v.log"; exit 1; }
  grep GBps "$OUT/mv_$v.log" | grep -v '^{' | cut -c1-45 | sed "s/^/$v /"
  timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/b_$v.json" 2> "$OUT/b_$v.err" || { tail "$OUT/b_$v.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$v.json'));print('$v', d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
done
