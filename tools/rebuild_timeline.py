#!/usr/bin/env python3
"""One rebuild frame's GPU timeline (kernels and copies, per stream) from tools/rebuild_trace.sh.

    python3 tools/rebuild_timeline.py gpurun_out/rebuild/trace [frame_from_end] [first_kernel]"""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", ""),
                   r["Kernel_Name"].split("(")[0].replace("void ", "").replace("art::", "")[:44]))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", ""), "copy " + r.get("Direction", "")))
    ev.sort()
    first = sys.argv[3] if len(sys.argv) > 3 else "prep_kernel"  # (static frames: nearest_first_kernel)
    starts = [i for i, e in enumerate(ev) if e[3].startswith(first)]
    a, b = starts[-back], starts[-back + 1]
    while a > 0 and ev[a - 1][3].startswith("copy") and "HOST_TO_DEVICE" in ev[a - 1][3]:
        a -= 1
    t0 = ev[a][0]
    print(f"# one rebuild frame (frame {len(starts) - back} of {len(starts)}), us from its first event; s = stream id")
    for s, e, st, n in ev[a:b]:
        if n.startswith("copy") and "HOST_TO_DEVICE" in n and s > ev[b - 1][1]:
            break
        print(f"{(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f}  {(e - s) / 1e3:7.1f} us  s{st:>2s}  {n}")


if __name__ == "__main__":
    main()
