# matvec workgroups per CU (LLMI_WG_PER_CU grid cap) with and without the pre-quantized image
set -o pipefail
OUT=${1:-gpurun_out/r3wg}; mkdir -p $OUT
export MV_SHAPES="12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096,12:6144x4096,12:4096x4096"
for w in 1 3 4; do
  for m in 1 8; do
    LLMI_WG_PER_CU=$w MV_MODE=$m timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv_w${w}_m$m.log 2>&1 || exit 1
  done
done
