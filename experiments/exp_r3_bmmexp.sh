# k_bmm time split: 1 = weight rows coalesced (row 0), 2 = no activation loads, 4 = no terms
set -o pipefail
OUT=${1:-gpurun_out/r3bmmexp}; mkdir -p $OUT
for e in 0 1 2 4 7; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_exp.so LLMI_BMM_EXP=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --prompt 16 --no-c2-full --batch-seqs 8 --batch-steps 16 --profile-steps 0 > $OUT/bench_$e.json 2> $OUT/bench_$e.err || exit 1
done
