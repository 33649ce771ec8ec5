# CPU baseline: decode matrices left in the file's page cache vs copied into rows
# first-touched by their reading thread (or_model_localize), interleaved A/B at 16 threads
set -o pipefail
mkdir -p gpurun_out/r6_cpu
O=gpurun_out/r6_cpu/numa_ab.txt
: > $O
lscpu | grep -E "Model name|Socket|NUMA node" >> $O
for L in 0 1 0 1; do LOCAL=$L N=12 timeout -k 10 300 python -u tools/cpu_decode_ab.py >> $O 2>&1 || exit 1; done
cat $O
