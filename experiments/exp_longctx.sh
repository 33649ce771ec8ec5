#!/bin/bash
# End-to-end decode at long contexts (8B): 4000- and 16000-token prompts, then 128 steps.
set -o pipefail
O=gpurun_out/longctx; mkdir -p $O
for p in 4000 16000; do
  timeout -k 10 300 python -u bench.py --prompt $p --steps 128 --warmup 8 --no-cpu-baseline --batch-seqs '' --profile-steps 4 > $O/bench_p$p.json 2> $O/bench_p$p.err || { tail -20 $O/bench_p$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_p$p.json'));print($p, d['value'], d['ms_per_step'], d['kernels']['attention'], d.get('prefill'))"
done
