# batched step on the matrix cores (k_bmm): parity tests, then the bench's batched numbers
set -o pipefail
OUT=${1:-gpurun_out/r3bmm}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_server.py > $OUT/tests_server.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 2
