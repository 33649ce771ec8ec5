#!/bin/bash
# Copy the round-4 evidence run (tools/r4_evidence.sh A / B output) into profiles/r04:
# per config the bench line, the rocprof kernel stats and the FETCH_SIZE traffic file
# bench.py reads (traffic_<preset>.json), plus the decode-matvec SQ counter summary.
set -u
SRC=${1:-gpurun_out/r4ev}; DST=profiles/r04
mkdir -p "$DST/configs"
for d in "$SRC"/prof_*/; do
  p=$(basename "$d"); p=${p#prof_}
  [ -f "$d/traffic_$p.json" ] && cp "$d/traffic_$p.json" "$DST/traffic_$p.json"
  [ -f "$d/kernel_stats.csv" ] && cp "$d/kernel_stats.csv" "$DST/configs/kernel_stats_$p.csv"
done
for f in "$SRC"/bench_*.json; do
  [ -f "$f" ] || continue
  b=$(basename "$f"); cp "$f" "$DST/configs/${b#bench_}"
done
[ -f "$SRC/sq_summary.json" ] && cp "$SRC/sq_summary.json" "$DST/sq_summary_matvec.json"
ls -la "$DST" "$DST/configs"
