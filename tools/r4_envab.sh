#!/bin/bash
# Default bench (no CPU baseline) under several environment settings, after a quick parity
# subset.  Usage: tools/r4_envab.sh OUTDIR "VAR=a VAR2=b" "VAR=c" ...   ("-" = defaults)
set -u
OUT=$1; shift; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_decode.py} > "$OUT/tests.log" 2>&1
  rc=$?; tail -2 "$OUT/tests.log"; if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
fi
i=0
for cfg in "$@"; do
  i=$((i+1)); envs=(); [ "$cfg" != "-" ] && envs=($cfg)
  timeout -k 10 300 env "${envs[@]}" python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
  rc=$?; echo "[$i] $cfg rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/bench_$i.err"; exit $rc; fi
  python3 - "$OUT/bench_$i.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
cb=d.get("continuous_batching",{}).get("sequences",{})
print("  value", d["value"], "ms", d["ms_per_step"], "c2_full", (d.get("c2_full") or {}).get("tok_s"), "batch", {k:v.get("tok_s") for k,v in cb.items()} if isinstance(cb,dict) else cb)
print("  " + " ".join(f"{n}={v['us']}" for n,v in d.get("kernels",{}).items()))
PY
done
