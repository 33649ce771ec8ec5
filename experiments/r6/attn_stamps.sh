set -o pipefail
mkdir -p gpurun_out/r6_attn
LLMI_LIB=$PWD/llama-gguf-inference_amd/lib/libllmi_trace.so ATT_MODES=6 ATT_KV=160,384,640 timeout -k 10 120 python -u tools/attrtrace.py > gpurun_out/r6_attn/attn_d_stamps.txt 2>&1 || { cat gpurun_out/r6_attn/attn_d_stamps.txt; exit 1; }
cat gpurun_out/r6_attn/attn_d_stamps.txt
timeout -k 10 120 python -u tools/attnbench.py > gpurun_out/r6_attn/attnbench.txt 2>&1 || { tail gpurun_out/r6_attn/attnbench.txt; exit 1; }
tail -30 gpurun_out/r6_attn/attnbench.txt
