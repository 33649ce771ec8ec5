# matvec isolated-shape sweep (tools/mvbench.py): lanes-per-row cap, and weights
# resident in the Infinity Cache (one copy) vs streamed from HBM (>= 1.2 GB of copies)
set -o pipefail
mkdir -p gpurun_out/r03g
export MV_SHAPES="12:4096x14336,14:4096x14336,12:28672x4096,14:128256x4096,12:6144x4096,12:4096x4096,13:4096x14336"
for lr in 64 32 16; do
  LLMI_MV_LR=$lr timeout -k 10 240 python -u tools/mvbench.py > gpurun_out/r03g/mv_lr$lr.log 2>&1 || exit 1
done
MV_NCOPIES=1 timeout -k 10 240 python -u tools/mvbench.py > gpurun_out/r03g/mv_mall.log 2>&1 || exit 1
