# profiler SIGSEGV isolation: graph replay without llmi under --pmc, with address maps
set -u
OUT=${1:-gpurun_out/r3repro}; mkdir -p $OUT; export TMPDIR=/tmp; R=$(pwd)
( cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/pmc_torch_graph" -o run -- \
    python3 "$R/tools/pmc_graph_repro.py" 4000 > "$R/$OUT/torch_graph.out" 2> "$R/$OUT/torch_graph.err"; echo "torch_graph rc=$?" > "$R/$OUT/torch_graph.rc" )
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +2M -delete
