set -o pipefail
mkdir -p gpurun_out/r6_cpu
O=gpurun_out/r6_cpu/decode_ab.txt
: > $O
nproc >> $O; cat /sys/fs/cgroup/cpu.max >> $O 2>/dev/null; lscpu | grep -E "Model name|Socket|NUMA node|Core" >> $O
timeout -k 10 200 python -u tools/cpu_decode_ab.py >> $O 2>&1 || exit 1
OMP_PROC_BIND=close OMP_PLACES=cores timeout -k 10 200 python -u tools/cpu_decode_ab.py >> $O 2>&1 || exit 1
OMP_WAIT_POLICY=active timeout -k 10 200 python -u tools/cpu_decode_ab.py >> $O 2>&1 || exit 1
OMP_WAIT_POLICY=passive timeout -k 10 200 python -u tools/cpu_decode_ab.py >> $O 2>&1 || exit 1
TH=12 timeout -k 10 200 python -u tools/cpu_decode_ab.py >> $O 2>&1 || exit 1
cat $O
