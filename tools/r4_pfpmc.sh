#!/bin/bash
# HBM traffic of the prefill GEMM (k_pf_gemm, T = 512, the six 8B/Mistral shapes of
# tools/prefillbench.py, 3 launches each): one rocprofv3 --pmc FETCH_SIZE pass of its
# own, per-dispatch counter next to the weight bytes of the shape.
set -u
OUT=${1:-gpurun_out/r4pfpmc}; R=$(pwd); mkdir -p "$OUT"; export TMPDIR=/tmp
( cd /tmp && PF_GEMM_T=512 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/pmc" -o run -- \
    python3 "$R/tools/prefillbench.py" llama3-8b-q4km "" > "$R/$OUT/gemm.json" 2> "$R/$OUT/gemm.err" ) || { tail -5 "$OUT/gemm.err"; exit 1; }
python3 - "$OUT/pmc" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_pf_gemm" in r["Kernel_Name"]]
shapes = [("q4_K", 14336, 4096, 144), ("q4_K", 4096, 14336, 144), ("q6_K", 4096, 14336, 210),
          ("q4_K", 4096, 4096, 144), ("q6_K", 14336, 4096, 210), ("q6_K", 4096, 4096, 210)]
by = {}
for r in rows:
    by.setdefault(int(r["Dispatch_Id"]), 0.0)
    by[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
ids = sorted(by)
out = []
for i, (t, rows_, cols, bpb) in enumerate(shapes):
    d = ids[3 * i:3 * i + 3]
    if not d:
        break
    fetch = sum(by[x] for x in d) / len(d)
    wbytes = rows_ * cols // 256 * bpb
    abytes = 512 * cols * 2 + 512 * (cols // 256) * (4 + 64)  # f16 fragments + d + sumi fragments
    rec = {"shape": f"{t} {rows_}x{cols} T=512", "fetch_size_raw_kb": round(fetch, 1),
           "hbm_MB_x2": round(fetch * 1024 * 2 / 1e6, 2),  # gfx950: FETCH_SIZE counts half the bytes
           "weight_MB": round(wbytes / 1e6, 2), "activation_MB": round(abytes / 1e6, 2)}
    out.append(rec)
    print(json.dumps(rec))
json.dump(out, open(sys.argv[1] + "/../pf_gemm_fetch.json", "w"), indent=1)
PY
