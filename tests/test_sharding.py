"""The N>1 path on CPU: fan sharding + all-gather of packed fan blocks over gloo (world size 2
and 3). Each rank computes its shard through libart's C ABI on the CPU backend (art_create with
device_mask 0; tests/test_multigpu_gpu.py runs the same split on the HIP path), packs it in the
device block layout and all-gathers; the gathered bytes must equal the oracle's single-process
full frame bit for bit (the multi-GPU invariance of SURVEY.md §8 e)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import art


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, S, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "audio-raytracer_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import art as A
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = A.CONFIGS[5]
        scene, org, params = A.synth(cfg, S=S, R=64, C_scale=0.05)
        b, e = A.dist.shard_range(S, world, rank)
        out = A.FanOutputs(e - b, 64, cfg.H, cfg.T, 1, dsp=True)
        fr = A.Frame(scene, params, np.ascontiguousarray(org[b:e]), out)
        if e > b:
            with A.Context(0) as cpu:  # libart's CPU backend
                cpu.run(fr)
        lay = A.fan_layout(fr)
        local = torch.from_numpy(A.pack_block(out, lay))
        full = A.dist.all_gather_fan_blocks(local, S, lay["stride"], world)
        if rank == 0:
            q.put(full.numpy().tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,S", [(2, 8), (3, 7)])
def test_sharded_gather_equals_single_process(world, S):
    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = art.CONFIGS[5]
    scene, org, params = art.synth(cfg, S=S, R=64, C_scale=0.05)
    out = art.FanOutputs(S, 64, cfg.H, cfg.T, 1, dsp=True)
    fr = art.Frame(scene, params, org, out)
    oracle.run_frame(fr)
    ref = art.pack_block(out, art.fan_layout(fr))
    assert np.frombuffer(got, np.uint8).tobytes() == ref.tobytes()


def test_shard_ranges_cover_fans():
    for S in (1, 7, 256, 1024):
        for W in (1, 2, 3, 4, 8):
            r = [art.dist.shard_range(S, W, k) for k in range(W)]
            assert r[0][0] == 0 and r[-1][1] == S and all(r[i][1] == r[i + 1][0] for i in range(W - 1))


def test_pack_unpack_roundtrip():
    cfg = art.CONFIGS[5]
    scene, org, params = art.synth(cfg, S=3, R=64, C_scale=0.05)
    out = art.FanOutputs(3, 64, cfg.H, cfg.T, 1, dsp=True, hits=True).fill_random(2)
    out.settings.view(np.uint8)[...] = np.random.default_rng(1).integers(0, 255, out.settings.view(np.uint8).shape)
    fr = art.Frame(scene, params, org, out)
    lay = art.fan_layout(fr, art.abi.ART_OUT_HIT_RESULTS)
    back = art.unpack_block(art.pack_block(out, lay), lay, 3, 64, cfg.H, cfg.T, 1, hits=True, dsp=True)
    assert all(back.equal(out).values())
