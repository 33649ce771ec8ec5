#!/bin/bash
# k_bmm at 8 sequences: product vs LLMI_BMM_EXP 1 (every lane reads row 0 of its tile:
# coalesced, L2 hits), 4 (no terms: the per-weight VALU removed), 5 (both); results garbage
set -u
for m in 0 1 4 5; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_exp.so LLMI_BMM_EXP=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other-numerics \
      --no-c2-full --steps 64 --warmup 8 --batch-seqs 8 --experiment > /tmp/bmm$m.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('/tmp/bmm$m.json').read().strip().splitlines()[-1]); print('bmm_exp=$m', d['continuous_batching']['sequences'])"
done
