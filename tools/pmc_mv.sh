#!/bin/bash
# PMC passes on one matvec shape + the streaming reference (tools/mvbench.py).
set -u
OUT=${1:-gpurun_out/pmc}; SHAPE=${2:-12:28672x4096}
mkdir -p "$OUT"; export TMPDIR=/tmp MV_SHAPES=$SHAPE MV_REPS=40
for wg in 4 8; do
  LLMI_WG_PER_CU=$wg timeout -k 10 120 python3 tools/mvbench.py > "$OUT/wg$wg.log" 2>&1 || exit $?
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- python3 tools/mvbench.py > "$OUT/p$i.log" 2>&1 || exit $?
done
