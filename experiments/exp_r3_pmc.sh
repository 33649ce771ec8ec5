# SQ cycle breakdown of the matvec (eager launches via tools/mvtrace.py, product library):
# WAVE_CYCLES = WAIT_ANY (waitcnt/barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY
set -u
OUT=${1:-gpurun_out/r3pmc}; mkdir -p "$OUT"; export TMPDIR=/tmp
R=$(pwd)
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  ( cd /tmp && MV_SHAPES=12:28672x4096,14:128256x4096,12:4096x14336 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$R/$OUT/p$i" -o run -- python3 "$R/tools/mvtrace.py" > "$R/$OUT/p$i.log" 2>&1 ) || exit $?
done
