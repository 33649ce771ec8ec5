#!/bin/bash
# batched step at 2/4/8 sequences: k_bmd (LDS-DMA weights, default) vs k_bmm (LLMI_BMM_DMA=0)
set -u
for d in 1 0; do
  LLMI_BMM_DMA=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other-numerics --no-c2-full --steps 64 --warmup 8 \
      --batch-seqs 4,8 > /tmp/bmd$d.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('/tmp/bmd$d.json').read().strip().splitlines()[-1]); print('dma=$d', d['continuous_batching']['sequences'])"
done
