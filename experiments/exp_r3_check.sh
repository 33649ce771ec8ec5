# GPU gate for a change: -m gpu tests (stop at first failure), matvec shapes, default bench
set -o pipefail
OUT=${1:-gpurun_out/r3chk}; mkdir -p $OUT
export MV_SHAPES="12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096,12:6144x4096,12:4096x4096"
timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
