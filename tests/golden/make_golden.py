#!/usr/bin/env python3
"""Generate tests/golden/*.npz: scene inputs + the oracle's outputs and test counts.

The reference (Unity/Burst C#) cannot run here and ships no fixtures, so
these vectors come from the CPU oracle (oracle/art_oracle.c), which tests/test_oracle_kats.py
pins against hand-derived answers. They freeze the oracle's behaviour (a regression in the
restatement shows up as a fixture mismatch) and give the GPU path a fixture-based check that
needs no oracle build. Re-run: python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "audio-raytracer_amd"))

import numpy as np  # noqa: E402

import art  # noqa: E402
import oracle  # noqa: E402

# name -> (config, S, R, collider scale, thread count, hits, stale seed)
CASES = {
    "config1": (1, 8, 64, None, 1, True, None),
    "config2_small": (2, 4, 64, 0.125, 1, False, None),
    "config3_small": (3, 4, 64, 0.0625, 1, False, None),
    "config4_small": (4, 4, 64, 1 / 32, 1, False, None),
    "config5_small": (5, 4, 64, 0.125, 1, True, None),
    "config1_tc3_stale": (1, 4, 50, None, 3, True, 9),
}


def build(name):
    ci, S, R, cs, tc, hits, stale = CASES[name]
    scene, org, params = art.synth(art.CONFIGS[ci], S=S, R=R, C_scale=cs)
    params.thread_count = tc
    out = art.FanOutputs(S, R, params.max_hits_per_ray, scene.T, tc, hits=hits, dsp=params.dsp is not None)
    if stale is not None:
        out.fill_random(stale)
    return scene, org, params, out


def params_json(p: art.FrameParams) -> str:
    d = {k: getattr(p, k) for k in ("max_ray_life", "max_hits_per_ray", "max_muffle_hit_distance",
                                    "muffle_effectiveness", "permeation_strength_per_ray",
                                    "permeation_effectiveness", "max_reverb_distance", "thread_count", "stages")}
    d["dsp"] = p.dsp is not None
    return json.dumps(d)


def main():
    for name in CASES:
        scene, org, params, out = build(name)
        stale = {k: getattr(out, k).copy() for k in ("echo", "muffle", "perm", "settings")}
        if out.hit_points is not None:
            stale["hit_points"] = out.hit_points.copy(); stale["hit_counts"] = out.hit_counts.copy()
            stale["hit_ids"] = out.hit_ids.copy()
        counts = oracle.run(scene, params, org, out, threads=8)[1]
        arrs = dict(dirs=scene.dirs, targets=scene.targets, spheres=scene.spheres, aabbs=scene.aabbs, obbs=scene.obbs,
                    origins=org, params=np.array(params_json(params)), counts=np.array(json.dumps(counts)),
                    out_echo=out.echo, out_muffle=out.muffle, out_perm=out.perm, out_settings=out.settings)
        for k, v in stale.items():
            arrs["in_" + k] = v
        if out.dsp is not None:
            arrs["out_dsp"] = out.dsp
        if out.hit_points is not None:
            arrs["out_hit_points"] = out.hit_points; arrs["out_hit_counts"] = out.hit_counts
            arrs["out_hit_ids"] = out.hit_ids
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
        print(name, {k: int(v) for k, v in counts.items() if v})


if __name__ == "__main__":
    main()
