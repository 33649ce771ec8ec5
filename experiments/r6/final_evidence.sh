# round-6 final evidence: per-config rocprof stats + FETCH_SIZE passes and bench lines
# (profiles/r06/configs), then smoke + the whole GPU suite + the default bench reading the
# 8B's fresh traffic file (profiles/r06/final)
set -o pipefail
O=gpurun_out/${OUT:-r6_final}
mkdir -p $O
bash tools/evidence.sh config $O llama3-8b-q4km || exit 1
cp $O/prof_llama3-8b-q4km/traffic_llama3-8b-q4km.json profiles/r06/ || exit 1
for p in tinyllama-q8_0 mistral7b-q6k mistral7b-q5km; do
  bash tools/evidence.sh config $O $p || exit 1
done
bash tools/evidence.sh final $O || exit 1
