#!/bin/bash
# SQ counters of the batched step's k_bmd launches (8 sequences): wave-cycle shares and
# instruction mix
set -u
R=$(pwd); OUT=gpurun_out/bmdsq; mkdir -p $OUT; export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
SQ2="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
i=0
for set in "$SQ1" "$SQ2"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/$OUT/p$i" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline --preset llama3-8b-q4km --prompt 128 --steps 8 --warmup 2 --profile-steps 0 \
      --no-c2-full --no-other-numerics --eager --batch-seqs 8 --batch-steps 8 > "$R/$OUT/p$i.log" 2>&1 ) || { tail -5 $OUT/p$i.log; exit 1; }
  python3 tools/sq_summary.py $OUT/p$i k_bmd > $OUT/sq$i.json || exit 2
done
find $OUT \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -size +4M -delete
cat $OUT/sq1.json $OUT/sq2.json
