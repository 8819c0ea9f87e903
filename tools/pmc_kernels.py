#!/usr/bin/env python3
"""Mean FETCH_SIZE / WRITE_SIZE (KB) per kernel from a gpu_round.sh output directory."""
import collections, csv, sys

d = sys.argv[1]
for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/pmc_{cnt}/run_counter_collection.csv")):
        agg[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("art::", "")].append(float(r["Counter_Value"]))
    print(cnt)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]) / len(kv[1]))[:10]:
        print("  %-40s n=%3d mean_KB=%10.1f" % (k[:40], len(v), sum(v) / len(v)))
