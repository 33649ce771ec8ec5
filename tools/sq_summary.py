#!/usr/bin/env python3
"""SQ counter summary of a rocprofv3 --pmc pass (counter_collection.csv): per kernel
name, mean of each counter over its dispatches and the wave-cycle shares
(SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stalls,
SQ_ACTIVE_INST_VALU = VALU issue; MI355X_MICROARCH.md §rocprofv3 PMC slots).
Usage: sq_summary.py <dir with **/counter_collection.csv> [name filter]"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
acc = defaultdict(lambda: defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = m.get("SQ_WAVE_CYCLES") or 0
    rec = {"dispatches": max(len(v) for v in cs.values()), **{c: round(v, 1) for c, v in m.items()}}
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if c in m:
                rec[c + "_share"] = round(m[c] / wc, 3)
    out[k[:120]] = rec
print(json.dumps(out, indent=1))
