set -o pipefail
mkdir -p gpurun_out/r6f
export LLMI_LIB=$PWD/llama-gguf-inference_amd/lib/libllmi_c10.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6f/engine_tests.log 2>&1 || { tail -30 gpurun_out/r6f/engine_tests.log; exit 1; }
tail -1 gpurun_out/r6f/engine_tests.log
for p in llama3-8b-q4km tinyllama-q8_0; do
  LLMI_ENGINE=1 timeout -k 10 240 python -u bench.py --preset $p --steps 128 --warmup 16 --no-cpu-baseline --batch-seqs '' --no-other-numerics > gpurun_out/r6f/b_$p.json 2> gpurun_out/r6f/b_$p.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6f/b_$p.json'));print('$p c10', d['value'], {k:(v['us'],v['per_step']) for k,v in d['kernels'].items() if v['per_step']})"
done
LE_NL=2 bash tools/le_ab.sh llama3-8b-q4km "LLMI_ENGINE=1" > gpurun_out/r6f/leab_8b.txt 2>&1 || exit 1
grep -E "===|drained|edge seen|image built|first ready|done \(wave|launch span|ring-full us|ring wait" gpurun_out/r6f/leab_8b.txt
