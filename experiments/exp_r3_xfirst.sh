# x-first vs weights-first issue order in the matvec prologue (mvbench MV_MODE bit 2)
set -o pipefail
OUT=${1:-gpurun_out/r3x}; mkdir -p $OUT
export MV_SHAPES="12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096,12:6144x4096"
for m in 0 4 1 5; do
  MV_MODE=$m timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv_mode$m.log 2>&1 || exit 1
done
