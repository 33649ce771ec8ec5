# quantize-once without the noinline spill: matvec bench A/B + profiler crash isolation
set -u
OUT=${1:-gpurun_out/r3xq2}; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs= > $OUT/bench_xq.json 2> $OUT/bench_xq.err || exit 2
LLMI_XQ=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch-seqs= --no-c2-full > $OUT/bench_noxq.json 2> $OUT/bench_noxq.err || exit 3
bash experiments/exp_r3_pmcrepro.sh $OUT
