set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 120 python -u tools/lestream.py > gpurun_out/r6a/lestream.txt 2>&1 || exit 1
cat gpurun_out/r6a/lestream.txt
bash tools/le_ab.sh llama3-8b-q4km "LLMI_ENGINE=1 LLMI_LE_EXP=1" "LLMI_ENGINE=1 LLMI_LE_EXP=3" "LLMI_ENGINE=1 LLMI_LE_LAG=16" "LLMI_ENGINE=1 LLMI_LE_LAG=48" "LLMI_ENGINE=1 LLMI_LE_NT=0" > gpurun_out/r6a/leab_8b.txt 2>&1 || exit 1
grep -E "===|loader done|gate\+up (done|first)|launch span|ring-full wait us" gpurun_out/r6a/leab_8b.txt
