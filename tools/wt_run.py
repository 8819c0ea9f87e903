#!/usr/bin/env python3
"""Device-resident frames back to back with the wave-timeline build, then the dump.

    ART_LIB=variants/libart_wt.so ART_WAVE_TIMES_OUT=gpurun_out/wt/c2.bin python tools/wt_run.py 2 [frames]

The context closes right after the frames, so the ring's last records are a steady-clock frame of
the same device loop bench.py times (tools/wave_times.py reads the file)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "audio-raytracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import art  # noqa: E402


def main():
    cfg = art.CONFIGS[int(sys.argv[1])]
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    dev = torch.device("cuda:0")
    scene, org, params = art.synth(cfg, S=cfg.S)
    org = np.ascontiguousarray(org)
    ctx = art.Context(1)
    out0 = art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
    frame = art.Frame(scene, params, org, out0)
    lay = art.fan_layout(frame)
    ctx.bind(frame)
    d_org = torch.from_numpy(org).to(dev)
    d_blk = torch.zeros(cfg.S * lay["stride"], dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(frames):
        ctx.launch_device(d_org.data_ptr(), cfg.S, d_blk.data_ptr(), 0, sp)
    torch.cuda.synchronize()
    ctx.close()
    print("frames", frames)


if __name__ == "__main__":
    main()
