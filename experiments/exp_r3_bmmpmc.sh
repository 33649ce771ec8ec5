# SQ counters of the batched step's kernels (eager launches; one --pmc pass)
set -o pipefail
OUT=${1:-gpurun_out/r3bmmpmc}; mkdir -p $OUT; R=$(pwd); export TMPDIR=/tmp
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$R/$OUT/pmc" -o run -- \
  python3 "$R/bench.py" --eager --no-cpu-baseline --steps 8 --warmup 2 --prompt 16 --profile-steps 0 --no-c2-full --batch-seqs 8 --batch-steps 4 \
  > "$R/$OUT/bench.json" 2> "$R/$OUT/bench.err"; echo "rc=$?" > "$R/$OUT/rc"
cd "$R" && python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
f = glob.glob(f"{out}/pmc/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
if f:
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "bmm" in k or "pf_quant" in k or "k_matvec" in k:
            agg[k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}
json.dump(res, open(f"{out}/sq_summary.json", "w"), indent=1)
PY
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +2M -delete
