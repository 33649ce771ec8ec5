# x86 attention (first K pass before q where registers allow, one exp per thread with DPP
# chunk sums): x86 + batch tests, then 8B / TinyLlama benches (batched 2/4/8 on the 8B)
set -o pipefail
O=gpurun_out/${OUT:-r6_x86attn}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_x86.py tests/test_gpu_batch.py tests/test_gpu_fa.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for num in x86 generic; do
  timeout -k 10 300 python -u bench.py --numerics $num --no-cpu-baseline --no-c2-full --steps 256 --warmup 16 --batch-seqs 2,4,8 > $O/bench_8b_$num.json 2> $O/bench_8b_$num.log || { tail $O/bench_8b_$num.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_8b_$num.json'));o=d['other_numerics'];print('8b $num', d['value'], {k:v['tok_s'] for k,v in d['continuous_batching']['sequences'].items()}, {k:v['us'] for k,v in d['kernels'].items()})"
done
timeout -k 10 300 python -u bench.py --preset tinyllama-q8_0 --numerics x86 --no-cpu-baseline --no-c2-full --steps 256 --warmup 16 --batch-seqs '' > $O/bench_tinyllama_x86.json 2> $O/bench_tinyllama_x86.log || { tail $O/bench_tinyllama_x86.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_tinyllama_x86.json'));print('tinyllama x86', d['value'], {k:v['us'] for k,v in d['kernels'].items()})"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bx86 -o run -- python3 -u bench.py --numerics x86 --no-cpu-baseline --no-c2-full --no-other-numerics --steps 16 --warmup 4 --batch-seqs 8 --batch-steps 32 > $O/prof_bx86.log 2>&1 || { tail -20 $O/prof_bx86.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof_bx86/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):7d} x {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:110]}')
PY
