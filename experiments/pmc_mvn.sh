#!/bin/bash
# PMC passes over the batched-step bench leg (eager launches): what bounds k_mvn at 8
# sequences (VALU issue, LDS, memory waits).  One counter group per pass.
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_mvn; mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
ARGS="--steps 4 --warmup 2 --no-cpu-baseline --batch-seqs 8 --batch-steps 8 --profile-steps 0 --eager --prompt 16"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $O/p$i.json 2> $O/p$i.err || echo "pass $i failed rc=$?"
done
ls $O
