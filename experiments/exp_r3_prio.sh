# alternating s_setprio per sub-item between co-resident workgroups (experiment build)
set -o pipefail
OUT=${1:-gpurun_out/r3prio}; mkdir -p $OUT
export MV_SHAPES="12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096,12:6144x4096"
for m in 1 17; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_exp.so MV_MODE=$m timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv_mode$m.log 2>&1 || exit 1
done
