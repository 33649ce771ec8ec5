set -o pipefail
mkdir -p gpurun_out/le2
for p in llama3-8b-q4km tinyllama-q8_0; do
  for e in 1 0; do
    LLMI_ENGINE=$e timeout -k 10 240 python -u bench.py --preset $p --steps 128 --warmup 16 --no-cpu-baseline --batch-seqs '' --no-other-numerics > gpurun_out/le2/b_${p}_e$e.json 2> gpurun_out/le2/b_${p}_e$e.log || exit 1
    python -c "import json;d=json.load(open('gpurun_out/le2/b_${p}_e$e.json'));print('$p e=$e', d['value'], d['c2_full'], {k:(v['us'],v['per_step']) for k,v in d['kernels'].items()})"
  done
done
