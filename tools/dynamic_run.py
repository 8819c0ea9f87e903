#!/usr/bin/env python3
"""bench.py's dynamic step alone (1 % of the colliders moved per step: art_collider_set_many +
art_colliders_sync + art_launch_device on torch's stream), for its kernel / copy timeline under
rocprofv3 --kernel-trace --memory-copy-trace, and its ms per step. GPU box only.
    python3 tools/dynamic_run.py [config] [steps]"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import art  # noqa: E402
from art import abi  # noqa: E402
from art.colliders import ColliderStore, resident_frame  # noqa: E402
from bench import jitter_records  # noqa: E402


def main():
    cfg = art.CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 2]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    scene, org, params = art.synth(cfg)
    S = org.shape[0]
    ctx = art.Context(1)
    store = ColliderStore(ctx)
    fields = {abi.ART_KIND_SPHERE: scene.spheres, abi.ART_KIND_AABB: scene.aabbs, abi.ART_KIND_OBB: scene.obbs}
    for k, arr in fields.items():
        for i in range(arr.size):
            store.add(k, arr[i])
    store.sync()
    ctx.set_flags(abi.ART_CTX_RESIDENT_COLLIDERS)
    out = art.FanOutputs(S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
    rframe = resident_frame(art.Frame(scene, params, org, out))
    lay = art.fan_layout(rframe)
    ctx.bind(rframe)
    d_org = torch.from_numpy(np.ascontiguousarray(org)).cuda()
    d_blk = torch.zeros(S * lay["stride"], dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(7)
    variants = []
    for _ in range(8):
        moves = {}
        for k, arr in fields.items():
            if arr.size:
                ids = rng.choice(arr.size, max(1, arr.size // 100), replace=False).astype(np.int32)
                moves[k] = (ids, jitter_records(rng, arr[ids], 0.05))
        variants.append(moves)

    def one(i):
        for k, (ids, recs) in variants[i % len(variants)].items():
            store.set_many(k, ids, recs)
        store.sync()
        ctx.launch_device(d_org.data_ptr(), S, d_blk.data_ptr(), 0, sp)

    for i in range(10):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one(i)
    torch.cuda.synchronize()
    print(f"config {cfg.index}: dynamic step {(time.perf_counter() - t0) / steps * 1e3:.4f} ms over {steps} steps", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
