# pre-quantized activation image (MVArgs::xq) vs in-kernel norm + quantization: matvec
# shapes (mvbench MV_MODE 1 = fused RMSNorm, 0 = plain quantization, 8 = image) + timelines
set -o pipefail
OUT=${1:-gpurun_out/r3img}; mkdir -p $OUT
export MV_SHAPES="12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096,12:6144x4096,12:4096x4096"
for m in 1 0 8; do
  MV_MODE=$m timeout -k 10 240 python -u tools/mvbench.py > $OUT/mv_mode$m.log 2>&1 || exit 1
done
LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_tr.so MV_MODE=8 MV_SHAPES=12:28672x4096,12:4096x14336,12:4096x4096 timeout -k 10 240 python -u tools/mvtrace.py > $OUT/trace_img.log 2>&1 || exit 2
