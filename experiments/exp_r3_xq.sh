# quantize-once (gate+up writes ffn_down's q8 image): GPU tests, bench A/B, and the
# graph-replay --pmc pass with address maps + faulthandler (profiler SIGSEGV forensics)
set -u
OUT=${1:-gpurun_out/r3xq}; mkdir -p $OUT; export TMPDIR=/tmp; R=$(pwd)
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_xq.json 2> $OUT/bench_xq.err || exit 2
LLMI_XQ=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs= --no-c2-full > $OUT/bench_noxq.json 2> $OUT/bench_noxq.err || exit 3
( cd /tmp && LLMI_DUMP_MAPS="$R/$OUT/maps" timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/pmc_graph" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --batch-seqs= --no-c2-full --steps 20 --warmup 16 --profile-steps 0 \
    > "$R/$OUT/pmc_graph.json" 2> "$R/$OUT/pmc_graph.err"; echo "pmc_graph rc=$?" > "$R/$OUT/pmc_graph.rc" )
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +2M -delete
