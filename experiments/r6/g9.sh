set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6h/engine_tests.log 2>&1 || { tail -30 gpurun_out/r6h/engine_tests.log; exit 1; }
tail -1 gpurun_out/r6h/engine_tests.log
bash tools/le_ab.sh llama3-8b-q4km "LLMI_ENGINE=1" "LLMI_ENGINE=1 LLMI_LE_EXP=8" "LLMI_ENGINE=1 LLMI_LE_EXP=3" "LLMI_ENGINE=1 LLMI_LE_EXP=11" > gpurun_out/r6h/leab_8b.txt 2>&1 || exit 1
grep -E "===|gate\+up (done|first)|launch span" gpurun_out/r6h/leab_8b.txt
