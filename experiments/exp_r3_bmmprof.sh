# kernel times of the batched step (8 sequences) under rocprofv3 --kernel-trace --stats
set -o pipefail
OUT=${1:-gpurun_out/r3bmmprof}; mkdir -p $OUT; R=$(pwd); export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 0 --no-c2-full --batch-seqs 8 --batch-steps 16 \
  > "$R/$OUT/bench.json" 2> "$R/$OUT/bench.err" || exit 1
cd "$R" && find "$OUT" -name "*kernel_trace.csv" -size +2M -delete
