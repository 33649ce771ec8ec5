#!/bin/bash
# TTFT of the configs' prompts (tools/prefillbench.py) under rocprofv3 --kernel-trace
# --stats: per-kernel time of the whole prefill.  usage: tools/r4_pfprof.sh <preset> <lens> [out]
set -u
P=$1; LENS=$2; OUT=${3:-gpurun_out/r4pf}; R=$(pwd); mkdir -p "$OUT"; export TMPDIR=/tmp
( cd /tmp && PF_GEMM_T=512 timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$P" -o run -- \
    python3 "$R/tools/prefillbench.py" "$P" "$LENS" > "$R/$OUT/ttft_$P.json" 2> "$R/$OUT/ttft_$P.log" ) || { tail -5 "$OUT/ttft_$P.log"; exit 1; }
grep "n=" "$OUT/ttft_$P.log"
find "$OUT/prof_$P" -name "*kernel_trace.csv" -size +2M -delete
python3 - "$OUT/prof_$P" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["Percentage"]):5.1f}% n={r["Calls"]:>6} avg={float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
print(f"total {tot/1e6:.1f} ms")
PY
