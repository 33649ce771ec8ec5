#!/bin/bash
# A/B of two builds on one box: libllmi_base.so (the previous commit) vs libllmi.so (the
# working tree), default-numerics decode bench per preset.
#   bash experiments/exp_ab.sh <out dir under gpurun_out> <preset>...
set -u
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for P in "$@"; do
  for L in base new; do
    LIB=llama-gguf-inference_amd/lib/libllmi.so; [ $L = base ] && LIB=llama-gguf-inference_amd/lib/libllmi_base.so
    LLMI_LIB=$LIB timeout -k 10 300 python -u bench.py --preset $P --no-cpu-baseline --batch-seqs= --no-other-numerics \
      --steps 100 --warmup 16 --profile-steps 0 > $OUT/${P}_$L.json 2> $OUT/${P}_$L.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d.get('c2_full',{}).get('tok_s'))" $OUT/${P}_$L.json $P $L
  done
done
