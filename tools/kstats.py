#!/usr/bin/env python3
"""Per-kernel calls and mean duration (us) of one rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    name = r["Name"].split("(")[0].replace("void ", "").replace("art::", "")[:64]
    print(f"{name:64s} calls={int(r['Calls']):6d} avg_us={float(r['AverageNs']) / 1e3:9.1f}")
