set -o pipefail
mkdir -p gpurun_out/r3c
export MV_SHAPES="12:28672x4096,12:4096x14336,14:4096x14336,14:128256x4096,12:6144x4096,12:4096x4096"
LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_512.so LLMI_WG_PER_CU=1 timeout -k 10 240 python -u tools/mvbench.py > gpurun_out/r3c/mv512_w1.log 2>&1 || exit 1
LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_512.so LLMI_WG_PER_CU=2 timeout -k 10 240 python -u tools/mvbench.py > gpurun_out/r3c/mv512_w2.log 2>&1 || exit 1
LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_512tr.so LLMI_WG_PER_CU=1 MV_SHAPES=12:28672x4096,12:4096x14336,14:128256x4096 timeout -k 10 240 python -u tools/mvtrace.py > gpurun_out/r3c/trace512.log 2>&1 || exit 1
