# Matvec time with weights that fit the 256 MB Infinity Cache (a few copies rotated) vs
# streamed from HBM (>= 1.2 GB of copies): is the per-launch time bound by HBM or not?
set -e
mkdir -p gpurun_out/mall
run() {  # name copies mode shapes
  MV_NCOPIES=$2 MV_MODE=$3 MV_SHAPES="$4" timeout -k 10 120 python -u tools/mvbench.py 2>/dev/null | grep -v "^{" | sed "s/^/$1 nc=$2 /"
}
for nc in 0 small; do
  run gate_up $([ $nc = small ] && echo 3 || echo 0) 33 "12:28672x4096"
  run down_q4k $([ $nc = small ] && echo 6 || echo 0) 64 "12:4096x14336"
  run down_q6k $([ $nc = small ] && echo 4 || echo 0) 64 "14:4096x14336"
  run attn_out $([ $nc = small ] && echo 20 || echo 0) 64 "12:4096x4096"
  run qkv $([ $nc = small ] && echo 14 || echo 0) 1 "12:6144x4096"
done
