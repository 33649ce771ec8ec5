#!/bin/bash
# k_a86_h phase costs: the launch cut after the loads are issued (1), scores (2), sums (3),
# p (4), whole (0); at 16 and 32 dims per workgroup (LLMI_EXP_A86_DS)
set -u
O=${1:-gpurun_out/a86}; mkdir -p "$O"
for ds in 16; do
for st in 0; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_exp.so LLMI_EXP_A86_DS=$ds LLMI_EXP_A86_STOP=$st ATT_NUMERICS=1 ATT_KV=128,256,400,640,1000,2000 ATT_MODES=0 \
      timeout -k 10 120 python -u tools/attnbench.py 2>/dev/null | grep n_kv | sed "s/^/ds=$ds stop=$st /" || exit 1
done
done
