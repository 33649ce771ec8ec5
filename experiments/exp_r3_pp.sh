# ping-pong (2x unrolled, copy-free) matvec loop vs the copying loop
set -o pipefail
OUT=${1:-gpurun_out/r3pp}; mkdir -p $OUT
export MV_SHAPES="12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096,12:6144x4096,12:4096x4096"
MV_MODE=1 timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv_base.log 2>&1 || exit 1
LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_pp.so MV_MODE=1 timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv_pp.log 2>&1 || exit 1
LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_pp.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs= > $OUT/bench_pp.json 2> $OUT/bench_pp.err || exit 3
