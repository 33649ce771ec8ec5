#!/bin/bash
# exchange attention (mode 4): parity tests, microbench vs the split path, e2e bench.
set -u
OUT=${1:-gpurun_out/attx}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 -k attention > "$OUT/tests.log" 2>&1; rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
ATT_MODES=2,4 ATT_KV=128,384,640,1024 timeout -k 10 120 python tools/attnbench.py > "$OUT/attn.log" 2>&1 || { cat "$OUT/attn.log"; exit 1; }
cat "$OUT/attn.log"
LLMI_ATTN_MODE=4 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 256 > "$OUT/bench4.json" 2> "$OUT/bench4.err" || { tail "$OUT/bench4.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench4.json'));print('mode4', d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 256 > "$OUT/bench0.json" 2> "$OUT/bench0.err" || { tail "$OUT/bench0.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench0.json'));print('mode0', d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
