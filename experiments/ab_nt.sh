#!/bin/bash
# A/B of nt vs default-policy weight loads end to end (bench.py, ABAB) and per launch
# (mvbench, gate+up / down / lm_head shapes).  LLMI_LIB picks the build.
set -u
OUT=${1:-gpurun_out/abnt}; ROOT=$(pwd); L=$ROOT/llama-gguf-inference_amd/lib; mkdir -p "$OUT"
for lib in libllmi libllmi_nt0; do
  MV_MODE=1 MV_SHAPES=12:28672x4096,12:4096x14336,14:128256x4096 MV_REPS=300 LLMI_LIB=$L/$lib.so \
    timeout -k 10 180 python3 tools/mvbench.py > "$OUT/mv_$lib.log" 2>&1 || exit $?
done
for r in 1 2; do
  for lib in libllmi libllmi_nt0; do
    LLMI_LIB=$L/$lib.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch-seqs "" --steps 256 \
      > "$OUT/bench_${lib}_$r.json" 2> "$OUT/bench_${lib}_$r.err" || exit $?
  done
done
grep -h "^1[24]:" "$OUT"/mv_*.log; for f in "$OUT"/bench_*.json; do echo "$f"; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d.get('continuous_batching'))" "$f"; done
