# first-dispatch-round task share (LLMI_MV_OLD_SHARE) on long matvec launches
set -o pipefail
OUT=${1:-gpurun_out/r3share}; mkdir -p $OUT
export MV_SHAPES="14:128256x4096,12:28672x4096,12:4096x14336,14:4096x14336"
for sh in 0 1.25 1.4; do
  LLMI_MV_OLD_SHARE=$sh MV_MODE=1 timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv_sh$sh.log 2>&1 || exit 1
done
