set -o pipefail
mkdir -p gpurun_out/r6_cpu
timeout -k 10 120 python -u tools/cpu_dotbench.py > gpurun_out/r6_cpu/dotbench.txt 2>&1 || exit 1
cat gpurun_out/r6_cpu/dotbench.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r6_cpu/bench_default.json 2> gpurun_out/r6_cpu/bench_default.log || { tail -20 gpurun_out/r6_cpu/bench_default.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6_cpu/bench_default.json'));c=d['cpu_baseline'];print(d['value'], c['value'], c['achieved_GBps'], c['stream_frac'], c['threads'], c['threads_8'])"
