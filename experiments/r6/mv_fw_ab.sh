set -o pipefail
mkdir -p gpurun_out/r6_fw
for p in llama3-8b-q4km tinyllama-q8_0; do
  for fw in 0 1 0 1; do
    LLMI_MV_FW=$fw timeout -k 10 240 python -u bench.py --preset $p --steps 128 --warmup 16 --no-cpu-baseline --batch-seqs '' --no-other-numerics > gpurun_out/r6_fw/b_${p}_fw$fw.json 2> gpurun_out/r6_fw/b_${p}_fw$fw.log || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r6_fw/b_${p}_fw$fw.json'));print('$p fw=$fw', d['value'], d['c2_full']['tok_s'], {k:v['us'] for k,v in d['kernels'].items() if v['per_step']})"
  done
done
