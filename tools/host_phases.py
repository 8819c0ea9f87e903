#!/usr/bin/env python3
"""Host phases of the Unity-facing frame (art_schedule .. art_complete from host arrays, config k):
runs N frames with ART_HOST_TIMES=1 (steady_clock marks inside libart, means printed by
art_destroy) and prints them with the frames' p50 wall time. GPU box only.
  python3 tools/host_phases.py [config] [frames]"""
import os
import statistics
import sys
import time

os.environ["ART_HOST_TIMES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))
import art  # noqa: E402

ci = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cfg = art.CONFIGS[ci]
scene, org, params = art.synth(cfg)
frame = art.Frame(scene, params, org, art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None))
ctx = art.Context(1)
for _ in range(10):
    ctx.run(frame)
ctx.close()  # (warm-up phases discarded with this context)
ctx = art.Context(1)
ms = []
for i in range(n + 5):
    t0 = time.perf_counter()
    ctx.run(frame)
    if i >= 5:
        ms.append((time.perf_counter() - t0) * 1e3)
print(f"config {ci}: p50 frame {statistics.median(ms):.4f} ms over {n} frames (the phases below include the 5 warm-up frames)",
      flush=True)
ctx.close()
