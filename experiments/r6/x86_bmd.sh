# k_bmd's x86 fold (x86 batched steps on the matrix cores): parity, then 8B batched benches
set -o pipefail
export OUT=${OUT:-r6_x86bmd}
O=gpurun_out/${OUT:-r6_x86bmd}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fa.py tests/test_gpu_x86.py -x -q -k "batch" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for num in x86 generic; do
  timeout -k 10 300 python -u bench.py --numerics $num --no-cpu-baseline --no-c2-full --no-other-numerics --steps 32 --warmup 8 --batch-seqs 2,4,8 > $O/bench_$num.json 2> $O/bench_$num.log || { tail $O/bench_$num.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$num.json'));print('$num', d['value'], d.get('continuous_batching'))"
done
LLMI_LIB=$PWD/llama-gguf-inference_amd/lib/libllmi_trace.so ATT_SHAPE=32,4,64 timeout -k 10 120 python -u tools/a86trace.py > $O/a86_tinyllama.txt 2>&1 || { cat $O/a86_tinyllama.txt; exit 1; }
LLMI_LIB=$PWD/llama-gguf-inference_amd/lib/libllmi_trace.so ATT_SHAPE=32,8,128 timeout -k 10 120 python -u tools/a86trace.py > $O/a86_8b.txt 2>&1 || { cat $O/a86_8b.txt; exit 1; }
cat $O/a86_tinyllama.txt $O/a86_8b.txt
