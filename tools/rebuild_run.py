#!/usr/bin/env python3
"""Rebuild frames only (bench.py's p50_frame_ms_rebuild loop): every collider changes each frame
through the Unity-facing API (full H2D, decode, kd BVH and cell lists, kernels, D2H).

    python tools/rebuild_run.py [config] [frames] [static]   (under rocprofv3 --kernel-trace for the timeline)

static: the same scene every frame (bench.py's p50_frame_ms: no upload, no build; origins and slot
arrays H2D, kernels, result blocks D2H).

Prints the p50 / min frame time and the host-side split: art_schedule (upload + launches) and the
wait in art_complete."""
import os
import statistics
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))
import numpy as np  # noqa: E402

import art  # noqa: E402
from bench import jitter_records  # noqa: E402


def main():
    cfg = art.CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 2]
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    static = len(sys.argv) > 3 and sys.argv[3] == "static"
    rng = np.random.default_rng(7)
    scene, org, params = art.synth(cfg, S=cfg.S)
    org = np.ascontiguousarray(org)
    ctx = art.Context(1)
    fr = []
    for _ in range(2):
        sc = art.Scene(dirs=scene.dirs, targets=scene.targets,
                       spheres=jitter_records(rng, scene.spheres, 0.05) if scene.spheres.size else scene.spheres,
                       aabbs=jitter_records(rng, scene.aabbs, 0.05) if scene.aabbs.size else scene.aabbs,
                       obbs=jitter_records(rng, scene.obbs, 0.05) if scene.obbs.size else scene.obbs)
        fr.append(art.Frame(sc, params, org, art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)))
    ms, sched, wait = [], [], []
    for i in range(frames + 5):
        t0 = time.perf_counter()
        h = ctx.schedule(fr[0 if static else i % 2])
        t1 = time.perf_counter()
        h.complete()
        t2 = time.perf_counter()
        if i >= 5:
            ms.append((t2 - t0) * 1e3); sched.append((t1 - t0) * 1e3); wait.append((t2 - t1) * 1e3)
    ctx.close()
    print(f"{'static' if static else 'rebuild'} p50 {statistics.median(ms):.4f} ms (min {min(ms):.4f}); schedule p50 {statistics.median(sched):.4f}, "
          f"complete p50 {statistics.median(wait):.4f}")


if __name__ == "__main__":
    main()
