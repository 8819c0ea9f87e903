"""Load tests/golden/*.npz fixtures back into Scene / FrameParams / FanOutputs."""
import glob
import json
import os

import numpy as np

import art

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    scene = art.Scene(dirs=z["dirs"], targets=z["targets"], spheres=z["spheres"], aabbs=z["aabbs"], obbs=z["obbs"])
    pj = json.loads(str(z["params"]))
    dsp = pj.pop("dsp")
    params = art.FrameParams(**pj, dsp=art.DspSettings.default() if dsp else None)
    S = z["origins"].shape[0]
    hits = "out_hit_points" in z
    fresh = art.FanOutputs(S, scene.R, params.max_hits_per_ray, scene.T, params.thread_count, hits=hits, dsp=dsp)
    for k in ("echo", "muffle", "perm", "settings", "hit_points", "hit_counts", "hit_ids"):
        if "in_" + k in z:
            getattr(fresh, k)[...] = z["in_" + k]
    expected = fresh.copy()
    for k in ("echo", "muffle", "perm", "settings", "dsp", "hit_points", "hit_counts", "hit_ids"):
        if "out_" + k in z:
            getattr(expected, k)[...] = z["out_" + k]
    return scene, np.ascontiguousarray(z["origins"]), params, fresh, expected, json.loads(str(z["counts"]))
