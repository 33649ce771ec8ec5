# layer-engine A/B on one box: letrace timelines under LLMI_LE_* knobs (args: preset, then knob sets)
set -o pipefail
p=$1; shift
mkdir -p gpurun_out/leab
for kv in "$@"; do
  echo "=== $p $kv"
  env $kv LE_PRESET=$p timeout -k 10 200 python -u tools/letrace.py 2>&1 | grep -v amdgpu.ids || exit 1
done
