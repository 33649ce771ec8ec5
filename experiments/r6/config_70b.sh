# C5 (Llama-3-70B Q4_K_M, one GPU, 8-token prompt): rocprof stats + FETCH_SIZE passes and
# the bench line on the last tree
set -o pipefail
O=gpurun_out/${OUT:-r6_70b}
mkdir -p $O
bash tools/evidence.sh config $O llama3-70b-q4km --prompt 8 || exit 1
