#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel summary (run_kernel_stats.csv): calls, avg/min/max us."""
import csv
import sys

for path in sys.argv[1:]:
    print(f"== {path}")
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        print(f"{r['Name'][:64]:64s} calls {int(r['Calls']):7d} avg_us {float(r['AverageNs']) / 1e3:8.2f} "
              f"min {float(r['MinNs']) / 1e3:8.2f} max {float(r['MaxNs']) / 1e3:8.2f} pct {float(r['Percentage']):6.2f}")
