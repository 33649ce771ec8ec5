#!/usr/bin/env python3
"""Turn one tools/gpu_round.sh output directory into the committed evidence under
profiles/<round>/:
  kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `python3 bench.py`
  bench.json         the bench line printed by that same profiled command
  traffic.json       HBM bytes per launch of the dominant kernel from the separate
                     `--pmc FETCH_SIZE` pass, corrected per MI355X_MICROARCH.md §HBM
                     (FETCH_SIZE is KiB and reports half the bytes of a wide coalesced
                     read on gfx950: bytes = 2 * 1024 * FETCH_SIZE), calibrated on the
                     streaming-read kernel over a known byte count
  SUMMARY.md         the table the DESIGN.md roofline section quotes
Also writes profiles/traffic.json (read by bench.py for roofline.traffic).
Usage: summarize_round.py gpurun_out/round1 r01"""
import csv
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(ROOT, "profiles", tag)
os.makedirs(out, exist_ok=True)
DOM = "k_matvec<0, true, 3, 12"  # ffn_gate+ffn_up Q4_K + SwiGLU (any NP)

stats = list(csv.DictReader(open(os.path.join(src, "prof", "run_kernel_stats.csv"))))
shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), os.path.join(out, "kernel_stats.csv"))
def json_line(path):
    return json.loads([ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1])


bench = json_line(os.path.join(src, "prof_bench.json"))
json.dump(bench, open(os.path.join(out, "bench.json"), "w"), indent=1)
plain = json_line(os.path.join(src, "bench.json"))
json.dump(plain, open(os.path.join(out, "bench_plain.json"), "w"), indent=1)


def fetch(path, name_part):
    vals = []
    for r in csv.DictReader(open(path)):
        if name_part in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            vals.append(float(r["Counter_Value"]))
    return vals


# calibration: the streaming-read kernel over one 28672x4096 Q4_K copy (66,060,288 B)
cal_bytes = 28672 * 16 * 144
cal = fetch(os.path.join(src, "pmc_cal", "run_counter_collection.csv"), "k_stream_read")
cal_ratio = (2 * 1024 * sum(cal) / len(cal)) / cal_bytes if cal else None
dom = fetch(os.path.join(src, "pmc_bench", "run_counter_collection.csv"), DOM)
alg = bench["roofline"]["bytes_per_launch"]
hbm = 2 * 1024 * sum(dom) / len(dom) if dom else None
traffic = {"ffn_gate_up": {"kernel": bench["roofline"]["kernel"], "launches": len(dom),
                           "fetch_size_kib_mean": sum(dom) / len(dom) if dom else None,
                           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg,
                           "traffic_over_algorithmic": hbm / alg if hbm else None,
                           "correction": "bytes = 2 * 1024 * FETCH_SIZE (gfx950 half-count, KiB)",
                           "calibration_stream_read_ratio": cal_ratio}}
json.dump(traffic, open(os.path.join(out, "traffic.json"), "w"), indent=1)
json.dump(traffic, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)

rows = []
tot = sum(float(r["TotalDurationNs"]) for r in stats)
for r in stats:
    rows.append((r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
                 float(r["MaxNs"]) / 1e3, float(r["TotalDurationNs"]) / tot * 100))
dom_rows = [r for r in rows if DOM in r[0]]
with open(os.path.join(out, "SUMMARY.md"), "w") as f:
    f.write(f"# {tag}: rocprofv3 --kernel-trace --stats of `python3 bench.py`\n\n")
    f.write(f"bench line of the profiled run: {bench['value']} tok/s "
            f"(unprofiled run: {plain['value']} tok/s), ctx 128 -> {bench['config']['ctx_end']}\n\n")
    f.write("| kernel | calls | avg us | min us | max us | % time |\n|---|---|---|---|---|---|\n")
    for n, c, a, mi, ma, p in rows:
        f.write(f"| `{n[:90]}` | {c} | {a:.2f} | {mi:.2f} | {ma:.2f} | {p:.1f} |\n")
    if dom_rows:
        n, c, a, *_ = dom_rows[0]
        f.write(f"\nDominant kernel `{n}`: rocprof average {a:.2f} us (in-graph decode launches) -> "
                f"{alg / (a * 1e-6) / 1e9:.0f} GB/s algorithmic.  bench.py's live figure (start/stop events "
                f"on each launch, llmi_profile_kernels) in the unprofiled run: {plain['roofline']['us_per_launch']} us "
                f"({plain['roofline']['achieved']} GB/s, {100 * (plain['roofline']['us_per_launch'] / a - 1):+.1f} % vs "
                f"rocprof); under rocprofv3 the same event figure reads {bench['roofline']['us_per_launch']} us "
                f"(the profiler's per-launch interception inflates eager event timing).\n")
    if hbm:
        f.write(f"\nHBM traffic (separate `--pmc FETCH_SIZE` pass, {len(dom)} launches): "
                f"{hbm / 1e6:.2f} MB per launch vs {alg / 1e6:.2f} MB algorithmic "
                f"({hbm / alg:.3f}x); stream-read calibration ratio {cal_ratio:.3f}.\n")
print(open(os.path.join(out, "SUMMARY.md")).read())
