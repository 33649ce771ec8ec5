#!/bin/bash
# The continuous-batching step at 8 sequences (Llama-3-8B Q4_K_M) under rocprofv3
# --kernel-trace --stats: per-kernel time of k_bmm / k_pf_quant / attention.
set -u
OUT=${1:-gpurun_out/r4bprof}; R=$(pwd); mkdir -p "$OUT"; export TMPDIR=/tmp
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --preset llama3-8b-q4km --prompt 128 --steps 16 --warmup 4 --profile-steps 0 \
    --no-c2-full --batch-seqs 8 > "$R/$OUT/bench.log" 2>&1 ) || { tail -5 "$OUT/bench.log"; exit 1; }
find "$OUT/prof" -name "*kernel_trace.csv" -size +2M -delete
python3 - "$OUT/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["Percentage"]):5.1f}% n={r["Calls"]:>6} avg={float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:100]}')
PY
