set -o pipefail
mkdir -p gpurun_out/r6_x86b
true
tail -6 gpurun_out/r6_x86b/tests.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fa.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_x86b/batch_tests.txt 2>&1 || { tail -40 gpurun_out/r6_x86b/batch_tests.txt; exit 1; }
tail -2 gpurun_out/r6_x86b/batch_tests.txt
for num in generic x86; do
  timeout -k 10 300 python -u bench.py --numerics $num --no-cpu-baseline --no-c2-full --no-other-numerics --steps 32 --warmup 8 --batch-seqs 2,4,8 > gpurun_out/r6_x86b/bench_$num.json 2> gpurun_out/r6_x86b/bench_$num.log || { tail gpurun_out/r6_x86b/bench_$num.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6_x86b/bench_$num.json'));print('$num', d['value'], d.get('continuous_batching'))"
done
