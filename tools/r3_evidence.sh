#!/bin/bash
# Round-3 evidence on one GPU box (via gpurun).  Part A: smoke, default bench, rocprof
# stats + FETCH_SIZE of the headline preset, and one graph-replay --pmc pass (the round-2
# profiler SIGSEGV check).  Part B: the 70B preset's bench + rocprof, the other configs.
set -u
PART=${1:-A}; OUT=${2:-gpurun_out/r3ev}
mkdir -p "$OUT"; export TMPDIR=/tmp
R=$(pwd)
if [ "$PART" = A ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 2
  bash tools/bench_profile.sh "$OUT/prof8b" llama3-8b-q4km > "$OUT/prof8b.log" 2>&1 || exit 3
  # graph replay under --pmc (round 2 saw a host SIGSEGV here): outcome recorded, not fatal
  ( cd /tmp && LLMI_DUMP_MAPS="$R/$OUT/maps" timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/pmc_graph" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline --batch-seqs= --steps 20 --warmup 16 --profile-steps 0 \
      > "$R/$OUT/pmc_graph.json" 2> "$R/$OUT/pmc_graph.err"; echo "pmc_graph rc=$?" > "$R/$OUT/pmc_graph.rc" )
  python3 - "$OUT" <<'PY' || true
import csv, glob, json, sys
out = sys.argv[1]
f = glob.glob(f"{out}/pmc_graph/**/*counter_collection.csv", recursive=True)
res = {"files": f}
if f:
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f[0]))
         if r["Counter_Name"] == "FETCH_SIZE" and "k_matvec<0, true, 3," in r["Kernel_Name"]]
    res.update({"launches": len(v), "fetch_kib_mean": sum(v) / len(v) if v else None,
                "hbm_bytes_per_launch_x2": (2 * 1024 * sum(v) / len(v)) if v else None})
json.dump(res, open(f"{out}/pmc_graph_summary.json", "w"), indent=1)
PY
fi
# keep what comes back under gpurun's 64 MiB: the per-dispatch CSVs are summarised above
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*memory_copy*.csv" \) -size +2M -delete
if [ "$PART" = B ]; then
  timeout -k 10 600 python -u bench.py --preset llama3-70b-q4km --prompt 8 --steps 128 --warmup 8 --no-cpu-baseline \
      > "$OUT/bench_70b.json" 2> "$OUT/bench_70b.err" || exit 4
  bash tools/bench_profile.sh "$OUT/prof70b" llama3-70b-q4km > "$OUT/prof70b.log" 2>&1 || exit 6
  find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +2M -delete
  bash tools/bench_configs.sh "$OUT/cfg" > "$OUT/cfg.log" 2>&1 || exit 5
fi
