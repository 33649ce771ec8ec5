#!/bin/bash
# SQ counters (one --pmc pass, 8 SQ_ counters) of the prefill GEMM shapes
# (tools/prefillbench.py with no prompt) and of the tiled prefill attention
# (tools/pfattn_bench.py, one ubatch at pos0 7680), summarized by tools/sq_summary.py.
set -u
OUT=${1:-gpurun_out/r4pf}; R=$(pwd); mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
( cd /tmp && PF_GEMM_T=512 timeout -s KILL 180 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/$OUT/sq_gemm" -o run -- \
    python3 "$R/tools/prefillbench.py" llama3-8b-q4km "" > "$R/$OUT/sq_gemm.json" 2> "$R/$OUT/sq_gemm.err" ) || { tail -5 "$OUT/sq_gemm.err"; exit 1; }
python3 tools/sq_summary.py "$OUT/sq_gemm" k_pf_gemm > "$OUT/sq_gemm_summary.json"
( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/$OUT/sq_fa" -o run -- \
    python3 "$R/tools/pfattn_bench.py" 32,8,128 512 7680 0 > "$R/$OUT/sq_fa.json" 2> "$R/$OUT/sq_fa.err" ) || { tail -5 "$OUT/sq_fa.err"; exit 2; }
python3 tools/sq_summary.py "$OUT/sq_fa" k_pf_fa > "$OUT/sq_fa_summary.json"
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +2M -delete
cat "$OUT/sq_gemm_summary.json" "$OUT/sq_fa_summary.json" | python3 -c "
import json,sys
txt=sys.stdin.read()
dec=json.JSONDecoder(); i=0
while i < len(txt):
    txt2=txt[i:].lstrip()
    if not txt2: break
    o,n=dec.raw_decode(txt2); i=len(txt)-len(txt2)+n
    for k,v in o.items(): print(k[:70], {c.replace('SQ_','').replace('_share',''):v[c] for c in v if c.endswith('_share')})
"
