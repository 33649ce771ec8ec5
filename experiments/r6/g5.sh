set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "equals_separate" > gpurun_out/r6d/engine_tests.log 2>&1 || { tail -30 gpurun_out/r6d/engine_tests.log; exit 1; }
tail -1 gpurun_out/r6d/engine_tests.log
LLMI_LE_EXP=4 timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "equals_separate" > gpurun_out/r6d/engine_tests4.log 2>&1 || { tail -30 gpurun_out/r6d/engine_tests4.log; exit 1; }
tail -1 gpurun_out/r6d/engine_tests4.log
bash tools/le_ab.sh llama3-8b-q4km "LLMI_ENGINE=1" "LLMI_ENGINE=1 LLMI_LE_EXP=4" "LLMI_ENGINE=1 LLMI_LE_EXP=1" > gpurun_out/r6d/leab_8b.txt 2>&1 || exit 1
grep -E "===|drained|polls|edge seen|image built|done \(wave|launch span" gpurun_out/r6d/leab_8b.txt
