#!/bin/bash
# crossover between k_mvn and k_bmd: batched step at 2/3/4 sequences with k_bmd from 2 (LLMI_BMM_MIN=2) vs default
set -u
for m in 2 5; do
  LLMI_BMM_MIN=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other-numerics --no-c2-full --steps 64 --warmup 8 \
      --batch-seqs 2,3,4,6,8 > /tmp/bmin$m.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('/tmp/bmin$m.json').read().strip().splitlines()[-1]); print('bmm_min=$m', {k: v['tok_s'] for k, v in d['continuous_batching']['sequences'].items()})"
done
for p in mistral7b-q6k llama3-70b-q4km; do
  for d in 1 0; do
    LLMI_BMM_DMA=$d timeout -k 10 400 python -u bench.py --preset $p --prompt 8 --no-cpu-baseline --no-other-numerics --no-c2-full --steps 32 --warmup 4 \
        --batch-seqs 8 > /tmp/bp$d.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/bp$d.json').read().strip().splitlines()[-1]); print('$p dma=$d', {k: v['tok_s'] for k, v in d['continuous_batching']['sequences'].items()})"
  done
done
