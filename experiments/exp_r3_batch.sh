# batched step with the per-token position/sequence loads hoisted out of the k_mvn loop
set -o pipefail
OUT=${1:-gpurun_out/r3batch}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_server.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 2
