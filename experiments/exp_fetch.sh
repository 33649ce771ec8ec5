#!/bin/bash
# FETCH_SIZE (x2) per launch: gate+up (mode 32), down (64), QKV-shaped norm (1)

set -u
O=${1:-gpurun_out/fetch}; R=$(pwd); mkdir -p "$O"; export TMPDIR=/tmp
for m in 32 64 1; do
  ( cd /tmp && MV_SHAPES=$([ $m = 64 ] && echo 12:4096x14336 || echo 12:28672x4096) MV_REPS=20 MV_MODE=$m timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/$O/m$m" -o run \
      --output-format csv -- python3 "$R/tools/mvbench.py" > "$R/$O/m$m.log" 2>&1 ) || { tail -5 "$O/m$m.log"; exit 1; }
done
python3 - "$O" <<'PY'
import csv, collections, glob, sys
for m in (32, 64, 1):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/m{m}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE":
                agg[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]) * 2048)
    for k, v in agg.items():
        print(f"mode {m:3d} {k:60s} n={len(v):3d} MB/launch {sum(v)/len(v)/1e6:8.2f}")
PY
