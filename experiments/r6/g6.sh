set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6e/engine_tests.log 2>&1 || { tail -30 gpurun_out/r6e/engine_tests.log; exit 1; }
tail -1 gpurun_out/r6e/engine_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6e/mv_tests.log 2>&1 || { tail -30 gpurun_out/r6e/mv_tests.log; exit 1; }
tail -1 gpurun_out/r6e/mv_tests.log
bash tools/le_bench.sh 2>&1 | tee gpurun_out/r6e/le_bench.txt || exit 1
bash tools/le_ab.sh llama3-8b-q4km "LLMI_ENGINE=1" "LLMI_ENGINE=1 LLMI_LE_EXP=3" > gpurun_out/r6e/leab_8b.txt 2>&1 || exit 1
grep -E "===|drained|polls|edge seen|image built|first ready|done \(wave|launch span|ring-full us|ring wait" gpurun_out/r6e/leab_8b.txt
