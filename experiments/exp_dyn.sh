#!/bin/bash
# Dynamic-tail matvec (MVArgs::dyn_*): per-launch times by tail percent / heads per XCD
# (mvbench), parity of the kernel and decode suites with the tail on, end to end A/B.
set -u
OUT=${1:-gpurun_out/dyn}; mkdir -p "$OUT"
SH=12:28672x4096,12:6144x4096,12:4096x4096,14:128256x4096
for cfg in 0:4 25:4 40:4 60:4 40:8 40:2; do
  pct=${cfg%%:*}; hx=${cfg##*:}
  LLMI_MV_DYN=$pct LLMI_MV_DYN_HX=$hx MV_MODE=1 MV_SHAPES=$SH MV_REPS=300 \
    timeout -k 10 240 python3 tools/mvbench.py > "$OUT/mv_${pct}_${hx}.log" 2>&1 || exit $?
  echo "pct $pct hx $hx: $(grep -h '^1[24]:' $OUT/mv_${pct}_${hx}.log | awk '{print $1, $3}' | tr '\n' ' ')"
done
LLMI_MV_DYN=40 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_decode.py > "$OUT/tests_dyn40.log" 2>&1 || { tail -30 "$OUT/tests_dyn40.log"; exit 1; }
tail -3 "$OUT/tests_dyn40.log"
for r in 1 2; do
  for pct in 0 40; do
    LLMI_MV_DYN=$pct timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch-seqs "" --steps 256 \
      > "$OUT/bench_${pct}_$r.json" 2> "$OUT/bench_${pct}_$r.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['us_per_launch'], {k: v['us'] for k, v in d['kernels'].items()})" "$OUT/bench_${pct}_$r.json" "dyn=$pct"
  done
done
