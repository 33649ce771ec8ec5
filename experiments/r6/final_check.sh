# the last tree: smoke + whole GPU suite + default bench (cpu_baseline with the NUMA-local
# weights), reading the profiles/r06 traffic files of final_evidence.sh
set -o pipefail
O=gpurun_out/${OUT:-r6_final3}
mkdir -p $O
bash tools/evidence.sh final $O || exit 1
