#!/bin/bash
# Upper bound of a free once-per-edge activation image: bench lines of the experiment
# build with LLMI_EXP_XQ masks (1 QKV, 2 attn_output, 4 gate+up, 8 down, 16 output fed a
# zero q8 image; results garbage, timing only).
set -u
O=${1:-gpurun_out/xq}; mkdir -p "$O"
for m in 0 8 2 4 1 15 31; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_exp.so LLMI_EXP_XQ=$m timeout -k 10 300 python -u bench.py \
      --no-cpu-baseline --batch-seqs "" --no-other-numerics --experiment > "$O/xq$m.json" 2> "$O/xq$m.err" || { tail -5 "$O/xq$m.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/xq$m.json')); k=d['kernels']
print('xq=$m', d['value'], 'c2', d['c2_full']['tok_s'], ' '.join(f'{n}={v[\"us\"]}' for n,v in k.items()))"
done
