#!/usr/bin/env python3
"""Wave timelines of the last frame from a variants/libart_wt.so run (-DART_WAVE_TIMES).

    ART_LIB=variants/libart_wt.so ART_WAVE_TIMES_OUT=wt.bin python bench.py ...
    python3 tools/wave_times.py wt.bin [waves_per_frame]

Each record is one wave of nearest_first_kernel (kind 0) or echo_muffle_kernel (1 = echo
workgroup, 2 = muffle workgroup). The last `waves_per_frame` records of the ring are the last
frame; per kind the script prints the wave-duration quantiles, the span from the launch's first
wave start to its last wave end, when 50 / 90 / 99 % of its waves had finished, per-XCD end times and
the number of waves in flight over time (1-us bins)."""
import sys

import numpy as np


def main():
    path = sys.argv[1]
    per_frame = int(sys.argv[2]) if len(sys.argv) > 2 else 8192 + 16384
    raw = open(path, "rb").read()
    n, cap = np.frombuffer(raw[:8], dtype=np.uint32)
    t = np.frombuffer(raw[8:8 + cap * 16], dtype=np.uint64).reshape(cap, 2)
    ids = np.frombuffer(raw[8 + cap * 16:8 + cap * 16 + cap * 12], dtype=np.uint32).reshape(cap, 3)
    take = min(per_frame, n, cap)
    idx = (np.arange(n - take, n) % cap).astype(np.int64)
    t, ids = t[idx], ids[idx]
    kind = (t[:, 0] >> np.uint64(60)).astype(int)
    t0 = (t[:, 0] & np.uint64((1 << 60) - 1)).astype(np.int64)
    t1 = t[:, 1].astype(np.int64)
    base = t0.min()
    t0 = (t0 - base) / 100.0  # 100 MHz ticks -> us
    t1 = (t1 - base) / 100.0
    xcc = ids[:, 2] & 0xF
    names = {0: "nearest", 1: "echo", 2: "muffle"}
    print(f"records {n} (ring {cap}), last {take}")
    for k in sorted(set(kind.tolist())):
        m = kind == k
        dur = t1[m] - t0[m]
        s, e = t0[m].min(), t1[m].max()
        ends = np.sort(t1[m])
        q = lambda p: ends[min(len(ends) - 1, int(p * len(ends)))] - s
        print(f"{names.get(k, k)}: waves {m.sum()} span {e - s:.1f} us (start {s:.1f}); duration p10/50/90/99/max "
              f"{np.percentile(dur, 10):.1f}/{np.percentile(dur, 50):.1f}/{np.percentile(dur, 90):.1f}/"
              f"{np.percentile(dur, 99):.1f}/{dur.max():.1f} us; 50/90/99 % done at {q(.5):.1f}/{q(.9):.1f}/{q(.99):.1f} us")
        print("   start p50/max %.1f/%.1f us" % (np.percentile(t0[m] - s, 50), (t0[m] - s).max()))
        per_x = [f"{x}:{t1[m & (xcc == x)].max() - s:.1f}" for x in range(8) if (m & (xcc == x)).any()]
        print("   last end per XCD: " + " ".join(per_x))
    # waves in flight per 1-us bin over the whole frame
    hi = int(np.ceil(t1.max())) + 1
    for k in sorted(set(kind.tolist())):
        m = kind == k
        line = []
        for b in range(0, hi, 2):
            line.append(int(((t0[m] <= b + 1) & (t1[m] > b + 1)).sum()))
        print(f"in flight {names.get(k, k)} (2-us steps): " + " ".join(str(v) for v in line))


if __name__ == "__main__":
    main()
