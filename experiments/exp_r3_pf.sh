# prefill GEMM without the per-stage scratch copy: parity tests, GEMM times, TTFT
set -o pipefail
OUT=${1:-gpurun_out/r3pf2}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_prefill.py tests/test_gpu_long.py > $OUT/tests.log 2>&1 || exit 1
PF_GEMM_T=8,32,128,512 timeout -k 10 400 python -u tools/prefillbench.py llama3-8b-q4km 128,512,2048 > $OUT/pf.json 2> $OUT/pf.err || exit 2
