#!/bin/bash
# K-split width A/B (default 2 vs LLMI_KS=4): 70B (28672-column ffn_down) and Mistral.
set -u
OUT=${1:-gpurun_out/ks2}
mkdir -p "$OUT"
run() {  # tag, env value, bench args...
  local tag=$1 k=$2; shift 2
  LLMI_KS=$k timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail "$OUT/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['value'], d['kernels']['ffn_down']['us'], d['kernels']['qkv']['us'], d['kernels']['ffn_gate_up']['us'])"
}
run 70b-ks2 0 --preset llama3-70b-q4km --steps 128 --warmup 8
run 70b-ks4 4 --preset llama3-70b-q4km --steps 128 --warmup 8
run 70b-ks2b 0 --preset llama3-70b-q4km --steps 128 --warmup 8
run mistral-ks2 0 --preset mistral7b-q6k
run mistral-ks4 4 --preset mistral7b-q6k
