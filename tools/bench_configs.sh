#!/bin/bash
# Decode bench lines for the non-headline BASELINE.json configs (one GPU each):
# TinyLlama Q8_0, Mistral-7B Q6_K and Q5_K_M (128 -> 512), Mistral Q6_K after a
# 2048-token batched prefill (config C4).  Usage: tools/bench_configs.sh [outdir]
set -u
OUT=${1:-gpurun_out/cfg}
mkdir -p "$OUT"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > "$OUT/$name.log" 2>&1 || { echo "FAILED $name rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  tail -1 "$OUT/$name.log" > "$OUT/$name.json"
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['unit'], 'frac', d['roofline']['frac'], 'e2e', d['hbm_end_to_end'], 'prefill', d.get('prefill'))"
}
run tinyllama-q8_0 --preset tinyllama-q8_0
run mistral7b-q6k --preset mistral7b-q6k
run mistral7b-q5km --preset mistral7b-q5km
run mistral7b-q6k-p2048 --preset mistral7b-q6k --prompt 2048 --steps 256
