set -o pipefail
mkdir -p gpurun_out/r6_fa
LLMI_REPORT_DIR=gpurun_out/r6_fa timeout -k 10 900 python -u -m pytest tests/test_gpu_fa.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r6_fa/fa_tests.txt 2>&1 || { tail -40 gpurun_out/r6_fa/fa_tests.txt; exit 1; }
tail -12 gpurun_out/r6_fa/fa_tests.txt
cat gpurun_out/r6_fa/parity_fa.jsonl
