#!/usr/bin/env python3
"""Per-frame kernel durations and inter-kernel gaps of a rocprofv3 --kernel-trace of bench.py.

  python3 tools/trace_gaps.py <run_kernel_trace.csv> [first_kernel_substring] [frames]

Frames are delimited by the first kernel of the timed stage (default nearest_first_kernel<false); for
each frame: its period (start to next frame's start), the sum of its kernels' durations, and the
idle time between consecutive kernels (the dispatch gaps)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "nearest_first_kernel<false"
limit = int(sys.argv[3]) if len(sys.argv) > 3 else 40
frames, cur = [], None
for r in rows:
    n = r["Kernel_Name"]
    if "<true" in n or "raytrace_kernel" in n:  # counting launches
        continue
    if first in n:
        cur = []
        frames.append(cur)
    if cur is not None:
        cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0].replace("void ", "").replace("art::", "")[:28]))
for i, f in enumerate(frames[:limit]):
    nxt = frames[i + 1][0][0] if i + 1 < len(frames) else f[-1][1]
    busy = sum(e - s for s, e, _ in f)
    gaps = [f[j + 1][0] - f[j][1] for j in range(len(f) - 1)] + [nxt - f[-1][1]]
    print(f"frame {i:3d} period {(nxt - f[0][0]) / 1e3:7.1f} us  kernels {busy / 1e3:7.1f}  " +
          " ".join(f"{k}={(e - s) / 1e3:.1f}" for s, e, k in f) + "  gaps " + " ".join(f"{g / 1e3:.1f}" for g in gaps))
