#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md) of the
tools/pmc_traffic_ab.sh passes:  python3 tools/pmc_traffic_print.py <variant>..."""
import collections
import csv
import glob
import sys

for v in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"gpurun_out/pmcab/{v}/{cnt}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("art::", "")
                if "<true" in k:
                    continue
                per[k][cnt].append(float(r["Counter_Value"]))
    print(f"== {v}")
    for k, c in sorted(per.items(), key=lambda kv: -sum(kv[1]["FETCH_SIZE"] or [0])):
        fe = sum(c["FETCH_SIZE"]) / max(1, len(c["FETCH_SIZE"]))
        wr = sum(c["WRITE_SIZE"]) / max(1, len(c["WRITE_SIZE"]))
        if fe + wr > 50:
            print(f"  {k[:44]:44s} fetch {fe / 1024:7.2f} MB (x2 {2 * fe / 1024:7.2f})  write {wr / 1024:6.2f} MB  "
                  f"bytes/launch {(2 * fe + wr) / 1024:7.2f} MB")
