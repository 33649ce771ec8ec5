# CPU baseline: AVX2 vs AVX-512BW fast dots (both with the NUMA-local weight copies), interleaved
set -o pipefail
mkdir -p gpurun_out/r6_cpu
O=gpurun_out/r6_cpu/avx512_ab.txt
: > $O
grep -o -m1 "avx512bw" /proc/cpuinfo >> $O
for F in 1 2 1 2; do LOCAL=1 FAST=$F N=12 timeout -k 10 300 python -u tools/cpu_decode_ab.py >> $O 2>&1 || exit 1; done
cat $O
