#!/usr/bin/env python3
"""Per-kernel mean of every counter in gpurun_out/pmc_<variant>/ (tools/pmc_sq.sh output)."""
import csv, glob, sys
from collections import defaultdict
d = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    acc = defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("art::", "")
        acc[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
    for (i, k, c), v in acc.items():
        d[k][c].append(v)
filt = sys.argv[2] if len(sys.argv) > 2 else "raytrace"
for k, cs in d.items():
    if filt not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:24s} {sum(v) / len(v):.4g}")
