# x86 Q8_0 fold buffer without bank conflicts (padded chains, 16-B term stores) and the
# generic Q8_0 rows padded: parity (x86 + generic + batched) then TinyLlama / 8B benches
set -o pipefail
O=gpurun_out/r6_q80
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_x86.py tests/test_gpu_kernels.py tests/test_gpu_decode.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for p in tinyllama-q8_0 llama3-8b-q4km; do
  timeout -k 10 300 python -u bench.py --preset $p --no-cpu-baseline --no-c2-full --steps 256 --warmup 16 --batch-seqs '' > $O/bench_$p.json 2> $O/bench_$p.log || { tail $O/bench_$p.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$p.json'));o=d['other_numerics'];print('$p', d['value'], 'x86', o['tok_s'], {k:v['us'] for k,v in d['kernels'].items()}, {k:v['us'] for k,v in o['kernels'].items()})"
done
