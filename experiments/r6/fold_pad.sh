# generic K-quant fold chains padded (bank-conflict-free fold reads) + x86 attention
# (first K pass before q, one exp per thread): full GPU suite, then the configs' benches
set -o pipefail
O=gpurun_out/${OUT:-r6_foldpad}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for p in llama3-8b-q4km tinyllama-q8_0 mistral7b-q6k; do
  timeout -k 10 300 python -u bench.py --preset $p --no-cpu-baseline --no-c2-full --steps 256 --warmup 16 --batch-seqs '' > $O/bench_$p.json 2> $O/bench_$p.log || { tail $O/bench_$p.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$p.json'));o=d['other_numerics'];print('$p', d['value'], 'x86', o['tok_s'], {k:v['us'] for k,v in d['kernels'].items()}, {k:v['us'] for k,v in o['kernels'].items()})"
done
