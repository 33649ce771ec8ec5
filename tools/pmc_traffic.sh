#!/bin/bash
# FETCH_SIZE (HBM/MALL read bytes, x2 gfx950 correction) of one matvec shape, plain and
# with the fused RMSNorm prologue, next to the streaming-read reference.
set -u
OUT=${1:-gpurun_out/pmc_traffic}; SHAPE=${2:-12:28672x4096}
mkdir -p "$OUT"; export TMPDIR=/tmp MV_SHAPES=$SHAPE MV_REPS=20
for m in 0 1; do
  MV_MODE=$m timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/m$m" -o run --output-format csv -- \
      python3 tools/mvbench.py > "$OUT/m$m.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, sys, collections
out = sys.argv[1]
for m in (0, 1):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{out}/m{m}/run_counter_collection.csv")):
        if r["Counter_Name"] == "FETCH_SIZE":
            agg[r["Kernel_Name"][:70]].append(float(r["Counter_Value"]) * 2048)
    for k, v in agg.items():
        if "matvec" in k or "stream" in k:
            print(f"mode {m} {k:70s} n={len(v):4d} MB/launch {sum(v)/len(v)/1e6:8.2f}")
PY
