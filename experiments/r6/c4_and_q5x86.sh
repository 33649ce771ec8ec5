# the last tree: C4 (Mistral-7B Q6_K, 2048-token batched prefill then decode) TTFT in both
# numerics, and Mistral Q5_K_M decode in x86 numerics
set -o pipefail
O=gpurun_out/${OUT:-r6_c4}
mkdir -p $O
for num in generic x86; do
  timeout -k 10 400 python -u bench.py --preset mistral7b-q6k --prompt 2048 --numerics $num --no-cpu-baseline --no-c2-full --no-other-numerics --steps 64 --warmup 8 --batch-seqs '' > $O/c4_$num.json 2> $O/c4_$num.log || { tail $O/c4_$num.log; exit 1; }
  python -c "import json;d=json.load(open('$O/c4_$num.json'));print('C4 $num', d['value'], d['prefill'])"
done
timeout -k 10 300 python -u bench.py --preset mistral7b-q5km --numerics x86 --no-cpu-baseline --no-c2-full --no-other-numerics --steps 256 --warmup 16 --batch-seqs '' > $O/q5km_x86.json 2> $O/q5km_x86.log || { tail $O/q5km_x86.log; exit 1; }
python -c "import json;d=json.load(open('$O/q5km_x86.json'));print('Q5_K_M x86', d['value'])"
