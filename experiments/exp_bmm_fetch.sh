#!/bin/bash
# FETCH_SIZE (x2) per k_bmm launch in the 8-sequence batched step (eager)
set -u
O=${1:-gpurun_out/bmmfetch}; R=$(pwd); mkdir -p "$O"; export TMPDIR=/tmp
( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$O/pmc" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --preset llama3-8b-q4km --prompt 128 --steps 8 --warmup 2 --profile-steps 0 \
    --no-c2-full --no-other-numerics --eager --batch-seqs 8 --batch-steps 8 > "$R/$O/log.txt" 2>&1 ) || { tail -5 "$O/log.txt"; exit 1; }
python3 - "$O/pmc" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and ("k_bmm" in r["Kernel_Name"] or "k_pf_quant" in r["Kernel_Name"]):
            agg[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]) * 2048)
for k, v in sorted(agg.items()):
    print(f"{k:40s} n={len(v):5d} MB/launch {sum(v)/len(v)/1e6:9.2f}")
PY
find "$O" -name "*counter_collection.csv" -size +4M -delete
