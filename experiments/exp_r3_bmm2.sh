# v_and_or B build: batched + prefill parity, bench, then the k_bmm time split (experiment lib)
set -o pipefail
OUT=${1:-gpurun_out/r3bmm2}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_prefill.py tests/test_gpu_server.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 2
for e in 0 1 2 4; do
  LLMI_LIB=llama-gguf-inference_amd/lib/libllmi_exp.so LLMI_BMM_EXP=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 --prompt 16 --no-c2-full --batch-seqs 8 --batch-steps 16 --profile-steps 0 > $OUT/exp_$e.json 2> $OUT/exp_$e.err || exit 3
done
