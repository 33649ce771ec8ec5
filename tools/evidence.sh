#!/bin/bash
# The round's GPU evidence, one parametrized script (run on the box through gpurun).
# Every GPU step has its own time limit and the script stops at the first failure.
#
#   evidence.sh final   OUT                      smoke(), the whole GPU suite, the default bench line
#   evidence.sh config  OUT PRESET [bench args]  rocprofv3 --stats pass + --pmc FETCH_SIZE pass over
#                                                the preset's bench (tools/make_traffic.py ->
#                                                traffic_<preset>.json), then the bench line carrying them
#   evidence.sh kernels OUT [PRESET]             per step-kernel class (qkv, attention, attn_output,
#                                                gate+up, down, output): FETCH_SIZE and two SQ passes
#                                                over eager decode steps (tools/kernel_classes.py)
#   evidence.sh calib   OUT [SHAPE]              FETCH_SIZE of one matvec shape beside the streaming
#                                                read of the same bytes (the x2 correction's check)
#   evidence.sh prefill OUT PRESET LENS          TTFT under --stats, k_pf_gemm FETCH_SIZE, SQ of
#                                                k_pf_gemm and k_pf_fa
#   evidence.sh batch   OUT [SEQS]               the continuous-batching step under --stats
#   evidence.sh envab   OUT "VAR=a" "VAR=b" ...  default bench under environment settings ("-" = none)
#   evidence.sh collect SRC ROUND                copy a run's summaries into profiles/<ROUND>/
set -u
CMD=${1:?usage: evidence.sh final|config|kernels|calib|prefill|batch|envab|collect OUT ...}
OUT=${2:?output directory}
shift 2
R=$(pwd)
export TMPDIR=/tmp
mkdir -p "$OUT"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
SQ2="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"

trim() { find "$1" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +4M -delete 2>/dev/null; true; }

stats_top() {  # dir with **/kernel_stats.csv, n
  python3 - "$1" "${2:-14}" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2])]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {float(r["Percentage"]):5.1f}% n={r["Calls"]:>6} '
          f'avg={float(r["AverageNs"])/1e3:8.2f}us {r["Name"][:96]}')
print(f"total {tot/1e6:.2f} ms")
PY
}

case "$CMD" in
final)
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
  timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > "$OUT/gpu_tests.txt" 2>&1
  rc=$?
  tail -3 "$OUT/gpu_tests.txt"
  [ $rc -ne 0 ] && { grep -E "FAILED|ERROR" "$OUT/gpu_tests.txt" | head -20; exit 2; }
  timeout -k 10 600 python -u bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 3; }
  tail -1 "$OUT/bench_default.log" > "$OUT/bench_default.json"
  python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['roofline']['frac'], (d.get('c2_full') or {}).get('tok_s'))"
  ;;
config)
  P=${1:?preset}; shift
  mkdir -p "$OUT/prof_$P"
  ARGS="--preset $P --no-cpu-baseline --batch-seqs= --no-other-numerics --steps 100 --warmup 16 --profile-steps 0"
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$P/stats" -o run -- \
      python3 "$R/bench.py" $ARGS "$@" > "$R/$OUT/prof_$P/stats.json" 2> "$R/$OUT/prof_$P/stats.err" ) || { tail -5 "$OUT/prof_$P/stats.err"; exit 1; }
  # counters on eager launches (graph replays under --pmc crashed the profiler's host side)
  ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/prof_$P/pmc" -o run -- \
      python3 "$R/bench.py" $ARGS "$@" --eager --steps 20 > "$R/$OUT/prof_$P/pmc.json" 2> "$R/$OUT/prof_$P/pmc.err" ) || { tail -5 "$OUT/prof_$P/pmc.err"; exit 2; }
  python3 tools/make_traffic.py "$OUT/prof_$P" "$P" > /dev/null || exit 3
  trim "$OUT/prof_$P"
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --preset "$P" --profile-dir "$OUT/prof_$P" "$@" \
      > "$OUT/bench_$P.log" 2>&1 || { tail -5 "$OUT/bench_$P.log"; exit 4; }
  tail -1 "$OUT/bench_$P.log" > "$OUT/bench_$P.json"
  python3 -c "import json; d=json.load(open('$OUT/bench_$P.json')); r=d['roofline']; print('$P', d['value'], 'frac', r['frac'], 'rocprof_frac', r.get('rocprof_frac'), 'traffic', r.get('traffic'), 'c2', (d.get('c2_full') or {}).get('tok_s'))"
  ;;
kernels)
  P=${1:-llama3-8b-q4km}
  mkdir -p "$OUT/kc_$P"
  ARGS="--preset $P --no-cpu-baseline --batch-seqs= --no-other-numerics --no-c2-full --eager --steps 12 --warmup 4 --profile-steps 0"
  i=0
  for set in "FETCH_SIZE" "$SQ1" "$SQ2"; do
    i=$((i+1))
    ( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/$OUT/kc_$P/p$i" -o run -- \
        python3 "$R/bench.py" $ARGS > "$R/$OUT/kc_$P/p$i.json" 2> "$R/$OUT/kc_$P/p$i.err" ) || { tail -5 "$OUT/kc_$P/p$i.err"; exit 1; }
  done
  python3 tools/kernel_classes.py "$OUT/kc_$P" "$P" > "$OUT/kernel_classes_$P.json" || exit 2
  trim "$OUT/kc_$P"
  cat "$OUT/kernel_classes_$P.json"
  ;;
calib)
  SHAPE=${1:-12:28672x4096}
  mkdir -p "$OUT/calib"
  for m in 0 1; do
    ( cd /tmp && MV_SHAPES=$SHAPE MV_REPS=20 MV_MODE=$m timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/$OUT/calib/m$m" -o run \
        --output-format csv -- python3 "$R/tools/mvbench.py" > "$R/$OUT/calib/m$m.log" 2>&1 ) || { tail -5 "$OUT/calib/m$m.log"; exit 1; }
  done
  python3 - "$OUT/calib" <<'PY'
import csv, collections, glob, json, sys
out = sys.argv[1]
res = {}
for m in (0, 1):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{out}/m{m}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE":
                agg[r["Kernel_Name"][:80]].append(float(r["Counter_Value"]) * 2048)
    for k, v in agg.items():
        if "matvec" in k or "stream" in k:
            res[f"mode{m} {k}"] = {"launches": len(v), "fetch_x2_MB_per_launch": round(sum(v) / len(v) / 1e6, 3)}
print(json.dumps(res, indent=1))
json.dump(res, open(out + "/calib.json", "w"), indent=1)
PY
  trim "$OUT/calib"
  ;;
prefill)
  P=${1:?preset}; LENS=${2:?lengths}
  ( cd /tmp && PF_GEMM_T=512 timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/pf_$P" -o run -- \
      python3 "$R/tools/prefillbench.py" "$P" "$LENS" > "$R/$OUT/ttft_$P.json" 2> "$R/$OUT/ttft_$P.log" ) || { tail -5 "$OUT/ttft_$P.log"; exit 1; }
  grep "n=" "$OUT/ttft_$P.log"
  trim "$OUT/pf_$P"
  stats_top "$OUT/pf_$P" 12 | tee "$OUT/pf_stats_$P.txt"
  ( cd /tmp && PF_GEMM_T=512 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/pf_pmc" -o run -- \
      python3 "$R/tools/prefillbench.py" llama3-8b-q4km "" > "$R/$OUT/pf_gemm.json" 2> "$R/$OUT/pf_gemm.err" ) || { tail -5 "$OUT/pf_gemm.err"; exit 2; }
  python3 tools/kernel_classes.py --pf-gemm "$OUT/pf_pmc" > "$OUT/pf_gemm_fetch.json" || exit 3
  ( cd /tmp && PF_GEMM_T=512 timeout -s KILL 180 rocprofv3 --pmc $SQ1 --kernel-trace --output-format csv -d "$R/$OUT/pf_sq" -o run -- \
      python3 "$R/tools/prefillbench.py" llama3-8b-q4km "" > "$R/$OUT/pf_sq.json" 2> "$R/$OUT/pf_sq.err" ) || { tail -5 "$OUT/pf_sq.err"; exit 4; }
  python3 tools/sq_summary.py "$OUT/pf_sq" k_pf_gemm > "$OUT/pf_sq_gemm.json"
  ( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $SQ1 --kernel-trace --output-format csv -d "$R/$OUT/pf_sqfa" -o run -- \
      python3 "$R/tools/pfattn_bench.py" 32,8,128 512 7680 0 > "$R/$OUT/pf_sqfa.json" 2> "$R/$OUT/pf_sqfa.err" ) || { tail -5 "$OUT/pf_sqfa.err"; exit 5; }
  python3 tools/sq_summary.py "$OUT/pf_sqfa" k_pf_fa > "$OUT/pf_sq_fa.json"
  trim "$OUT/pf_pmc"; trim "$OUT/pf_sq"; trim "$OUT/pf_sqfa"
  cat "$OUT/pf_gemm_fetch.json"
  ;;
batch)
  SEQS=${1:-8}
  ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/batch" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline --preset llama3-8b-q4km --prompt 128 --steps 16 --warmup 4 --profile-steps 0 \
      --no-c2-full --no-other-numerics --batch-seqs "$SEQS" > "$R/$OUT/batch.log" 2>&1 ) || { tail -5 "$OUT/batch.log"; exit 1; }
  trim "$OUT/batch"
  stats_top "$OUT/batch" 16 | tee "$OUT/batch_stats.txt"
  ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $SQ1 --kernel-trace --output-format csv -d "$R/$OUT/batch_sq" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline --preset llama3-8b-q4km --prompt 128 --steps 8 --warmup 2 --profile-steps 0 \
      --no-c2-full --no-other-numerics --eager --batch-seqs "$SEQS" --batch-steps 8 > "$R/$OUT/batch_sq.log" 2>&1 ) || { tail -5 "$OUT/batch_sq.log"; exit 2; }
  python3 tools/sq_summary.py "$OUT/batch_sq" k_bm > "$OUT/batch_sq_bmm.json"  # k_bmd / k_bmd2 (default) and k_bmm
  trim "$OUT/batch_sq"
  python3 -c "import json; d=json.load(open('$OUT/batch_sq_bmm.json')); [print(k[:70], {c: v[c] for c in v if c.endswith('_share')}) for k, v in d.items()]"
  ;;
envab)
  i=0
  for cfg in "$@"; do
    i=$((i+1)); envs=(); [ "$cfg" != "-" ] && envs=($cfg)
    timeout -k 10 300 env "${envs[@]}" python bench.py --no-cpu-baseline --no-other-numerics ${BENCH_ARGS:-} > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
    rc=$?; echo "[$i] $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_$i.err"; exit $rc; }
    python3 - "$OUT/bench_$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
cb = (d.get("continuous_batching") or {}).get("sequences") or {}
print("  value", d["value"], "ms", d["ms_per_step"], "c2_full", (d.get("c2_full") or {}).get("tok_s"),
      "batch", {k: v.get("tok_s") for k, v in cb.items()} if isinstance(cb, dict) else cb)
print("  " + " ".join(f"{n}={v['us']}" for n, v in d.get("kernels", {}).items()))
PY
  done
  ;;
collect)
  SRC=$OUT; DST=profiles/${1:?round, e.g. r05}
  mkdir -p "$DST/configs"
  for d in "$SRC"/prof_*/; do
    [ -d "$d" ] || continue
    p=$(basename "$d"); p=${p#prof_}
    [ -f "$d/traffic_$p.json" ] && cp "$d/traffic_$p.json" "$DST/traffic_$p.json"
    [ -f "$d/kernel_stats.csv" ] && cp "$d/kernel_stats.csv" "$DST/configs/kernel_stats_$p.csv"
  done
  for f in "$SRC"/bench_*.json "$SRC"/kernel_classes_*.json; do
    [ -f "$f" ] || continue
    b=$(basename "$f"); cp "$f" "$DST/configs/${b#bench_}"
  done
  [ -f "$SRC/calib/calib.json" ] && cp "$SRC/calib/calib.json" "$DST/fetch_calibration.json"
  ls -la "$DST" "$DST/configs"
  ;;
*)
  echo "unknown command $CMD"; exit 64 ;;
esac
