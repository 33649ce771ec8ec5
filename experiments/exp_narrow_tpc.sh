#!/bin/bash
# Narrow (one-wave workgroup) threshold: tasks per CU below which a launch goes narrow
# (4 = default: TinyLlama's QKV/O/gate+up; 5 adds the 8B's O (1024 tasks); 7 adds its QKV)
set -u
OUT=gpurun_out/ntpc; mkdir -p $OUT
for P in llama3-8b-q4km; do
  for F in 4 5 7 4; do
    LLMI_MV_NARROW_TPC=$F timeout -k 10 300 python -u bench.py --preset $P --no-cpu-baseline --batch-seqs= --no-other-numerics \
      --steps 100 --warmup 16 > $OUT/${P}_$F.json 2> $OUT/${P}_$F.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d.get('c2_full',{}).get('tok_s'), {k:v['us'] for k,v in d['kernels'].items()})" $OUT/${P}_$F.json $P $F
  done
done
