# layer engine evidence (profiles/r06/engine): tests, engine vs launches, per-edge traces
set -o pipefail
O=gpurun_out/r6_engine
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/engine_tests.txt 2>&1 || { tail -30 $O/engine_tests.txt; exit 1; }
tail -1 $O/engine_tests.txt
for p in llama3-8b-q4km tinyllama-q8_0; do
  for e in 1 0; do
    LLMI_ENGINE=$e timeout -k 10 240 python -u bench.py --preset $p --steps 128 --warmup 16 --no-cpu-baseline --batch-seqs '' --no-other-numerics > $O/bench_${p}_engine$e.json 2> $O/bench_${p}_engine$e.log || exit 1
    python -c "import json;d=json.load(open('$O/bench_${p}_engine$e.json'));print('$p engine=$e', d['value'], {k:(v['us'],v['per_step']) for k,v in d['kernels'].items() if v['per_step']})"
  done
  LLMI_ENGINE=1 LE_PRESET=$p timeout -k 10 200 python -u tools/letrace.py > $O/letrace_$p.txt 2>&1 || exit 1
  LLMI_ENGINE=1 LLMI_LE_EXP=3 LE_PRESET=$p timeout -k 10 200 python -u tools/letrace.py > $O/letrace_${p}_stream_only.txt 2>&1 || exit 1
  LLMI_ENGINE=1 LLMI_LE_EXP=1 LE_PRESET=$p timeout -k 10 200 python -u tools/letrace.py > $O/letrace_${p}_no_math.txt 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/lestream.py > $O/lestream.txt 2>&1 || exit 1
grep -h "launch span" $O/letrace_*.txt
