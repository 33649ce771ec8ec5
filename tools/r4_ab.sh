#!/bin/bash
# A/B of a launch knob on the GPU: quick parity subset, then the default bench with the
# knob off and on.  Usage: tools/r4_ab.sh OUTDIR VAR OFFVAL [pytest files...]
set -u
OUT=${1:-gpurun_out/ab}; VAR=${2:-LLMI_MV_BURST}; OFF=${3:-0}; shift 3 || true
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=${*:-tests/test_gpu_kernels.py tests/test_gpu_decode.py}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for v in "$OFF" default; do
  if [ "$v" = default ]; then unset $VAR; else export $VAR=$v; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  rc=$?; echo "bench $VAR=$v rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/bench_$v.err"; exit $rc; fi
  python3 - "$OUT/bench_$v.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "c2_full", d.get("c2_full",{}).get("tok_s") if isinstance(d.get("c2_full"),dict) else d.get("c2_full"))
k=d.get("kernels",{})
for n,v in (k.items() if isinstance(k,dict) else []): print(" ", n, v)
PY
done
