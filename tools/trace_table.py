#!/usr/bin/env python3
"""Per-kernel mean durations (us) of tools/trace_variants.sh runs, one column per variant."""
import csv
import glob
import sys

cols = sys.argv[1:]
tab = {}
for v in cols:
    f = glob.glob(f"gpurun_out/tr/{v}/**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        name = r["Name"].split("(")[0].replace("void ", "").replace("art::", "")[:60]
        tab.setdefault(name, {})[v] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]))
rows = sorted(tab.items(), key=lambda kv: -max(x[0] * x[1] for x in kv[1].values()))
print(f"{'kernel':60s} " + " ".join(f"{c:>14s}" for c in cols))
for name, d in rows[:16]:
    print(f"{name:60s} " + " ".join(f"{d[c][0]:9.1f}x{d[c][1]:<4d}" if c in d else " " * 14 for c in cols))
