#!/bin/bash
# Fold with batched LDS reads (libllmi.so) vs the per-4 loop (libllmi_base.so, the previous
# commit): decode bench per preset, both libraries on the same box
set -u
mkdir -p gpurun_out/fold
for P in tinyllama-q8_0 llama3-8b-q4km mistral7b-q6k; do
  for L in base new; do
    LIB=llama-gguf-inference_amd/lib/libllmi.so; [ $L = base ] && LIB=llama-gguf-inference_amd/lib/libllmi_base.so
    LLMI_LIB=$LIB timeout -k 10 300 python -u bench.py --preset $P --no-cpu-baseline --batch-seqs= --no-other-numerics \
      --steps 100 --warmup 16 --profile-steps 0 > gpurun_out/fold/${P}_$L.json 2> gpurun_out/fold/${P}_$L.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d.get('c2_full',{}).get('tok_s'), {k:v['us'] for k,v in d['kernels'].items()})" gpurun_out/fold/${P}_$L.json $P $L
  done
done
