#!/usr/bin/env python3
"""Where the host-API frame time goes (config 2): schedule return time, wait, unpack; blocking
complete vs polling is_completed first. Diagnostic only (GPU box)."""
import os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))
import art  # noqa: E402

cfg = art.CONFIGS[2]
scene, org, params = art.synth(cfg)
S = org.shape[0]
frame = art.Frame(scene, params, org, art.FanOutputs(S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None))
ctx = art.Context(1)
res = {"run": [], "sched": [], "wait_poll": [], "complete_after_poll": [], "run_poll": []}
for i in range(60):
    t0 = time.perf_counter(); ctx.run(frame); t1 = time.perf_counter()
    h = ctx.schedule(frame); t2 = time.perf_counter()
    while not h.is_completed:
        pass
    t3 = time.perf_counter(); h.complete(); t4 = time.perf_counter()
    if i >= 10:
        res["run"].append((t1 - t0) * 1e3); res["sched"].append((t2 - t1) * 1e3)
        res["wait_poll"].append((t3 - t2) * 1e3); res["complete_after_poll"].append((t4 - t3) * 1e3)
        res["run_poll"].append((t4 - t1) * 1e3)
print({k: round(statistics.median(v), 4) for k, v in res.items()})
