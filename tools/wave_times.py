#!/usr/bin/env python3
"""Wave timelines of the last frame from a variants/libart_wt.so run (-DART_WAVE_TIMES).

    ART_LIB=variants/libart_wt.so ART_WAVE_TIMES_OUT=wt.bin python tools/wt_run.py 2
    python3 tools/wave_times.py wt.bin

Each record is one wave of nearest_first_kernel (kind 0) or echo_muffle_kernel (1 = echo
workgroup, 2 = muffle workgroup), one slot per wave, overwritten every frame: the last frame. Per
kind the script prints the wave-duration quantiles, the span from the launch's first wave start to
its last wave end, the wave-us over (8192 slots x span), when 50 / 90 / 99 % of its waves had finished, per-XCD end times and
the number of waves in flight over time (2-us bins)."""
import sys

import numpy as np


def main():
    path = sys.argv[1]
    raw = open(path, "rb").read()
    _, cap, khz = np.frombuffer(raw[:12], dtype=np.uint32)
    t = np.frombuffer(raw[12:12 + cap * 16], dtype=np.uint64).reshape(cap, 2)
    ids = np.frombuffer(raw[12 + cap * 16:12 + cap * 16 + cap * 12], dtype=np.uint32).reshape(cap, 3)
    tick_us = 1e3 / khz if khz else 0.01  # wall-clock ticks -> us (100 MHz when the rate is unknown)
    keep = t[:, 1] != 0  # written slots (one per wave of the last frame)
    t, ids = t[keep], ids[keep]
    take = int(keep.sum())
    kind = (t[:, 0] >> np.uint64(60)).astype(int)
    t0 = (t[:, 0] & np.uint64((1 << 60) - 1)).astype(np.int64)
    t1 = t[:, 1].astype(np.int64)
    base = t0.min()
    t0 = (t0 - base) * tick_us
    t1 = (t1 - base) * tick_us
    xcc = ids[:, 2] & 0xF
    names = {0: "nearest", 1: "echo", 2: "muffle"}
    print(f"waves {take} (ring {cap}), wall clock {khz} kHz")
    for k in sorted(set(kind.tolist())):
        m = kind == k
        dur = t1[m] - t0[m]
        s, e = t0[m].min(), t1[m].max()
        ends = np.sort(t1[m])
        q = lambda p: ends[min(len(ends) - 1, int(p * len(ends)))] - s
        print(f"{names.get(k, k)}: waves {m.sum()} span {e - s:.1f} us (start {s:.1f}); duration p10/50/90/99/max "
              f"{np.percentile(dur, 10):.1f}/{np.percentile(dur, 50):.1f}/{np.percentile(dur, 90):.1f}/"
              f"{np.percentile(dur, 99):.1f}/{dur.max():.1f} us; 50/90/99 % done at {q(.5):.1f}/{q(.9):.1f}/{q(.99):.1f} us")
        print("   wave-us %.0f = %.2f of 8192 slots x span" % (dur.sum(), dur.sum() / (8192 * (e - s))))
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
