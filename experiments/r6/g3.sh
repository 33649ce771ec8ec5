set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_batch.py tests/test_fanout_check.py tests/test_gpu_replicate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b/engine_tests.log 2>&1 || { tail -30 gpurun_out/r6b/engine_tests.log; exit 1; }
tail -2 gpurun_out/r6b/engine_tests.log
bash tools/le_bench.sh 2>&1 | tee gpurun_out/r6b/le_bench.txt || exit 1
for p in tinyllama-q8_0 llama3-8b-q4km; do
  LLMI_ENGINE=1 LE_PRESET=$p timeout -k 10 200 python -u tools/letrace.py > gpurun_out/r6b/letrace_$p.txt 2>&1 || exit 1
done
bash tools/le_ab.sh llama3-8b-q4km "LLMI_ENGINE=1 LLMI_LE_EXP=3" > gpurun_out/r6b/leab_8b.txt 2>&1 || exit 1
grep -E "===|loader done|launch span" gpurun_out/r6b/leab_8b.txt
