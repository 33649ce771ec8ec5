#!/bin/bash
# k_pf_quant rows split over workgroups for few-token launches: batch + prefill parity
# tests, then the continuous-batching bench leg with the split (default lib, 2 blocks per
# workgroup), without it (libllmi_q0.so) and with 1 block (libllmi_q1.so).
set -u
OUT=${1:-gpurun_out/r4quant}; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py \
    tests/test_gpu_prefill.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for v in q0 def q1 q0 def; do
  lib=llama-gguf-inference_amd/lib/libllmi.so; [ $v != def ] && lib=llama-gguf-inference_amd/lib/libllmi_$v.so
  LLMI_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --preset llama3-8b-q4km --prompt 128 --steps 16 \
      --warmup 4 --profile-steps 0 --no-c2-full --batch-seqs 2,4,8 > "$OUT/bench_$v.log" 2>&1 || { tail -5 "$OUT/bench_$v.log"; exit 2; }
  tail -1 "$OUT/bench_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], json.dumps(d.get('continuous_batching',{}).get('sequences')))"
done
