#!/usr/bin/env python3
"""Per step-kernel class summary of rocprofv3 --pmc passes (tools/evidence.sh kernels).

Usage: kernel_classes.py <dir with p*/**/counter_collection.csv> [preset]
       kernel_classes.py --pf-gemm <dir>      (k_pf_gemm FETCH_SIZE per tools/prefillbench.py shape)

Dispatches of eager decode steps are classed by kernel name and, for the ADD-epilogue
matvecs, by their place in the step (attn_output follows attention, ffn_down follows
gate+up).  Per class: dispatches, mean duration (the pass's own timestamps, profiler
attached), FETCH_SIZE bytes per launch with the gfx950 x2 correction
(MI355X_MICROARCH.md §HBM), and the SQ counters as shares of SQ_WAVE_CYCLES."""
import collections
import csv
import glob
import json
import re
import sys

EPI = {0: "store", 1: "add", 2: "qkv", 3: "gate_up", 4: "output"}


def rows_of(d):
    out = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def klass(name, prev):
    m = re.search(r"k_matvec<(\d+), (true|false), (\d+),", name)
    if m:
        e = EPI.get(int(m.group(3)), "matvec")
        if e == "add":
            return "ffn_down" if prev == "gate_up" else "attn_output"
        return e
    if "k_attn" in name or "k_attl" in name or "k_a86" in name:
        return "attention"
    if "k_embed" in name:
        return "embed"
    return None


def step_classes(d, preset):
    by_disp = collections.OrderedDict()
    for r in rows_of(d):
        key = (r.get("Process_Id", ""), int(r["Dispatch_Id"]), r["Kernel_Name"])
        ent = by_disp.setdefault(key, {"name": r["Kernel_Name"], "counters": {},
                                       "ns": float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)})
        ent["counters"][r["Counter_Name"]] = ent["counters"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    prev = None
    for key in sorted(by_disp, key=lambda k: (k[0], k[1])):
        ent = by_disp[key]
        c = klass(ent["name"], prev)
        if c is None:
            continue
        if c != "attention":
            prev = c
        a = acc[c]
        a["_names"].append(ent["name"][:100])
        if ent["ns"] > 0:
            a["_ns"].append(ent["ns"])
        for k, v in ent["counters"].items():
            a[k].append(v)
    res = {"preset": preset, "source": "rocprofv3 --pmc (FETCH_SIZE pass, two SQ passes) over eager bench.py decode steps",
           "fetch_correction": "bytes = 2 * 1024 * FETCH_SIZE", "classes": {}}
    for c, a in acc.items():
        m = {k: sum(v) / len(v) for k, v in a.items() if not k.startswith("_") and v}
        rec = {"dispatches": len(a["_names"]), "kernels": sorted(set(a["_names"]))[:4]}
        if a["_ns"]:
            rec["us_profiled"] = round(sum(a["_ns"]) / len(a["_ns"]) / 1e3, 3)
        if "FETCH_SIZE" in m:
            rec["fetch_MB_per_launch"] = round(m["FETCH_SIZE"] * 2048 / 1e6, 3)
        wc = m.get("SQ_WAVE_CYCLES")
        for k, v in m.items():
            if k.startswith("SQ_"):
                rec[k] = round(v, 1)
                if wc and k not in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
                    rec[k + "_share"] = round(v / wc, 4)
        res["classes"][c] = rec
    return res


def pf_gemm(d):
    shapes = [("q4_K", 14336, 4096, 144), ("q4_K", 4096, 14336, 144), ("q6_K", 4096, 14336, 210),
              ("q4_K", 4096, 4096, 144), ("q6_K", 14336, 4096, 210), ("q6_K", 4096, 4096, 210)]
    by = collections.OrderedDict()
    for r in rows_of(d):
        if "k_pf_gemm" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            by[int(r["Dispatch_Id"])] = by.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    ids = sorted(by)
    out = []
    for i, (t, rows, cols, bpb) in enumerate(shapes):
        dd = ids[3 * i:3 * i + 3]
        if not dd:
            break
        fetch = sum(by[x] for x in dd) / len(dd)
        w = rows * cols // 256 * bpb
        act = 512 * cols * 2 + 512 * (cols // 256) * (4 + 64)
        out.append({"shape": f"{t} {rows}x{cols} T=512", "hbm_MB_x2": round(fetch * 2048 / 1e6, 2),
                    "weight_MB": round(w / 1e6, 2), "activation_MB": round(act / 1e6, 2)})
    return out


if __name__ == "__main__":
    if sys.argv[1] == "--pf-gemm":
        print(json.dumps(pf_gemm(sys.argv[2]), indent=1))
    else:
        print(json.dumps(step_classes(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "?"), indent=1))
