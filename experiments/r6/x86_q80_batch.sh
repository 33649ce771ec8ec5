# x86 Q8_0 batched steps (k_mvn with 4 working waves): parity, then TinyLlama x86 batched bench
set -o pipefail
O=gpurun_out/${OUT:-r6_q80b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_x86.py tests/test_gpu_batch.py -x -q -k "batch" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for num in x86 generic; do
  timeout -k 10 300 python -u bench.py --preset tinyllama-q8_0 --numerics $num --no-cpu-baseline --no-c2-full --no-other-numerics --steps 64 --warmup 8 --batch-seqs 2,4,8 > $O/bench_$num.json 2> $O/bench_$num.log || { tail $O/bench_$num.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$num.json'));print('tinyllama $num', d['value'], {k:v['tok_s'] for k,v in d['continuous_batching']['sequences'].items()})"
done
