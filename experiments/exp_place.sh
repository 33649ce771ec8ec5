#!/bin/bash
# k_matvec task placement knobs (one build): launch order vs XCD-ordered deal
# (LLMI_MV_XCD_ORDER) and early exit of task-less workgroups (LLMI_MV_IDLE_EXIT)
set -u
OUT=gpurun_out/place; mkdir -p $OUT
run() {  # name preset env...
  local n=$1 p=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --preset $p --no-cpu-baseline --batch-seqs= --no-other-numerics \
    --steps 100 --warmup 16 --profile-steps 0 > $OUT/${p}_$n.json 2> $OUT/${p}_$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d.get('c2_full',{}).get('tok_s'))" $OUT/${p}_$n.json $p $n
}
for P in llama3-8b-q4km tinyllama-q8_0; do
  run base $P LLMI_MV_IDLE_EXIT=0
  run idle $P LLMI_MV_IDLE_EXIT=1
  run xcd $P LLMI_MV_XCD_ORDER=01237654
  run both $P LLMI_MV_IDLE_EXIT=1 LLMI_MV_XCD_ORDER=01237654
  run both2 $P LLMI_MV_IDLE_EXIT=1 LLMI_MV_XCD_ORDER=01234567
done
