# x86 Q8_0 prefill GEMM (masked-weight MFMAs, x86 lane chains): parity then TinyLlama x86 TTFT
set -o pipefail
O=gpurun_out/r6_q80pf
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_x86.py -x -q -k "pf_gemm or prefill" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for num in x86 generic; do
  timeout -k 10 300 python -u bench.py --preset tinyllama-q8_0 --numerics $num --no-cpu-baseline --no-c2-full --no-other-numerics --steps 256 --warmup 16 --batch-seqs '' > $O/bench_$num.json 2> $O/bench_$num.log || { tail $O/bench_$num.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$num.json'));print('$num', d['value'], d['prefill'])"
done
