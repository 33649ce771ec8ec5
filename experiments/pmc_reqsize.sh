#!/bin/bash
# HBM read requests of the gate+up matvec by size (32/64/128 B) for nt and default-policy
# weight loads: does FETCH_SIZE x2 over-count the nt stream?
set -u
OUT=${1:-gpurun_out/pmcsz}; ROOT=$(pwd); mkdir -p "$OUT"; export TMPDIR=/tmp
for lib in libllmi libllmi_nt0; do
  ( cd /tmp && MV_MODE=1 MV_SHAPES=12:28672x4096 MV_REPS=40 LLMI_LIB=$ROOT/llama-gguf-inference_amd/lib/$lib.so \
    timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    --kernel-trace --output-format csv -d "$ROOT/$OUT/$lib" -o run -- python3 $ROOT/tools/mvbench.py > "$ROOT/$OUT/$lib.log" 2>&1 ) || exit $?
done
