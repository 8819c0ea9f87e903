#!/usr/bin/env python3
"""Per-bounce kernel durations of a multi-hit configuration from a rocprofv3 kernel trace.

  python3 tools/bounce_table.py <run_kernel_trace.csv> <H> [bench.json]

Every timed frame launches nearest_first_kernel, path_kernel and the echo vis_kernel once per
bounce, in bounce order, so the k-th launch of each throughput instantiation within a frame is
bounce k mod H (the counting instantiations, EX = true, are left out). Prints the mean duration
per bounce and kernel, and the bench line's live rays per bounce when a bench JSON is given.
"""
import csv
import json
import sys
from collections import defaultdict

path, H = sys.argv[1], int(sys.argv[2])
KINDS = ("nearest_first_kernel<false", "path_kernel<false", "vis_kernel<false")
seq = defaultdict(int)
dur = defaultdict(list)
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    name = r["Kernel_Name"]
    kind = next((k for k in KINDS if k in name), None)
    if kind is None:
        continue
    b = seq[kind] % H
    seq[kind] += 1
    dur[(kind, b)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

live = None
if len(sys.argv) > 3:
    line = open(sys.argv[3]).read().strip().splitlines()[-1]
    live = json.loads(line)["roofline"]["executed"].get("bounce_rays")
out = []
for b in range(H):
    row = {"bounce": b}
    if live:
        row["live_rays"] = live[b] if b < len(live) else None
    for k in KINDS:
        v = dur.get((k, b), [])
        row[k.split("<")[0] + "_us"] = round(sum(v) / len(v), 1) if v else None
        row[k.split("<")[0] + "_n"] = len(v)
    out.append(row)
for row in out:
    print(json.dumps(row))
