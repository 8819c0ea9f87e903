"""The sharded paths on the HIP device (SURVEY.md §8 e): fans split over shards must give the same
bytes as one shard.

* In-process split (art_create_on): one context whose fans are sharded over several "devices" —
  here N entries naming device 0, i.e. N streams, N scene copies and N result blocks on one GPU —
  exactly the code path art_create(mask) takes on an 8-GPU node (per-device upload, enqueue,
  D2H into the shared pinned block, completion over every device's event).
* Multi-process split: world-2 gloo group whose ranks share device 0; each rank binds the scene and
  computes its contiguous fan shard through libart's device entry point (art_launch_device), the
  blocks are all-gathered (art.dist.all_gather_fan_blocks) and must equal the single-process
  frame byte for byte. Reference: one fan = one AudioRayTracer job graph
  (Audio/AudioRayTracer.cs:161-237); fans are independent.
"""
import os
import socket

import numpy as np
import pytest

import art
from art import abi
import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shards,ci,S", [(2, 5, 9), (3, 2, 16), (4, 1, 3)])
def test_in_process_shards_on_one_device(ctx, shards, ci, S):
    """art_create_on([0]*N): the multi-device split, one stream per shard, equals the single-device
    context and the oracle; more shards than fans leaves some shards empty (S=3, N=4)."""
    cfg = art.CONFIGS[ci]
    scene, org, params = art.synth(cfg, S=S, R=128 if ci != 1 else 64, C_scale=0.1 if ci != 1 else None)
    dsp = params.dsp is not None
    hits = True
    one = art.FanOutputs(S, scene.R, params.max_hits_per_ray, scene.T, 1, hits=hits, dsp=dsp).fill_random(4)
    many, ref = one.copy(), one.copy()
    ctx.set_flags(0)
    ctx.run(art.Frame(scene, params, org, one))
    with art.Context(devices=[0] * shards) as mctx:
        h = mctx.schedule(art.Frame(scene, params, org, many))
        h.complete()
        # a second frame through the same context (buffers and the cached device scenes reused)
        again = one.copy()
        mctx.run(art.Frame(scene, params, org, again))
        # counting frames accumulate the per-shard test counts
        cnt = one.copy()
        mctx.set_flags(abi.ART_CTX_COUNT_TESTS)
        mctx.run(art.Frame(scene, params, org, cnt))
        counts = mctx.last_test_counts()
    cref = oracle.run_frame(art.Frame(scene, params, org, ref), threads=16)
    assert all(many.equal(ref).values()), many.equal(ref)
    assert all(many.equal(one).values())
    assert all(again.equal(ref).values())
    assert all(cnt.equal(ref).values())
    assert counts == cref


def test_in_process_shards_thread_count_slots(ctx):
    """TC > 1 (stale slots travel with the frame) through a 2-shard context."""
    scene, org, params = art.synth(art.CONFIGS[1], S=5, R=64)
    params.thread_count = 3
    a = art.FanOutputs(5, 64, params.max_hits_per_ray, scene.T, 3, hits=True).fill_random(9)
    ref = a.copy()
    with art.Context(devices=[0, 0]) as mctx:
        mctx.run(art.Frame(scene, params, org, a))
    oracle.run_frame(art.Frame(scene, params, org, ref), threads=8)
    assert all(a.equal(ref).values())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ci, S, R, cs, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "audio-raytracer_amd"))
    import torch
    import torch.distributed as dist
    import art as A
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = A.CONFIGS[ci]
        scene, org, params = A.synth(cfg, S=S, R=R, C_scale=cs)
        b, e = A.dist.shard_range(S, world, rank)
        shard = np.ascontiguousarray(org[b:e])
        out = A.FanOutputs(max(e - b, 1), R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
        fr = A.Frame(scene, params, shard if e > b else org[:1], out)
        lay = A.fan_layout(fr)
        with A.Context(1) as c:
            c.bind(fr)
            d_org = torch.from_numpy(shard.copy() if e > b else np.zeros((1, 3), np.float32)).cuda()
            d_blk = torch.zeros(max(e - b, 1) * lay["stride"], dtype=torch.uint8, device="cuda")
            st = torch.cuda.current_stream()
            c.launch_device(d_org.data_ptr(), e - b, d_blk.data_ptr(), 0, st.cuda_stream)
            st.synchronize()
            local = d_blk[: (e - b) * lay["stride"]].cpu()
        full = A.dist.all_gather_fan_blocks(local, S, lay["stride"], world)
        if rank == 0:
            q.put(full.numpy().tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ci,S,R,cs", [(5, 9, 128, 0.1), (4, 6, 256, 1 / 16)])
def test_world2_ranks_compute_shards_through_libart(ctx, ci, S, R, cs):
    import torch.multiprocessing as mp
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    world = 2
    procs = [mpc.Process(target=_worker, args=(r, world, port, ci, S, R, cs, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    cfg = art.CONFIGS[ci]
    scene, org, params = art.synth(cfg, S=S, R=R, C_scale=cs)
    out = art.FanOutputs(S, R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
    fr = art.Frame(scene, params, org, out)
    ctx.set_flags(0)
    ctx.run(fr)
    ref = art.pack_block(out, art.fan_layout(fr))
    lay = art.fan_layout(fr)
    back = art.unpack_block(np.frombuffer(got, np.uint8), lay, S, R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
    assert all(back.equal(out).values()), back.equal(out)
    # and against the oracle
    o_ref = art.FanOutputs(S, R, cfg.H, cfg.T, 1, dsp=params.dsp is not None)
    oracle.run_frame(art.Frame(scene, params, org, o_ref), threads=16)
    assert all(out.equal(o_ref).values())
    assert ref.size == len(got)


@pytest.mark.parametrize("fail_shard", [1, 2])
def test_enqueue_failure_on_later_shard(ctx, monkeypatch, fail_shard):
    """An error while enqueueing shard k > 0 of art_create_on([0]*3) (injected after shard k's scene
    upload: shards < k already have copies and kernels in flight on their streams) returns the
    error from art_schedule after draining every stream; nothing stays in flight, and the next
    frame on the same context is complete and bit-exact."""
    cfg = art.CONFIGS[5]
    scene, org, params = art.synth(cfg, S=9, R=128, C_scale=0.1)
    with art.Context(devices=[0, 0, 0]) as mctx:
        bad = art.FanOutputs(9, 128, cfg.H, cfg.T, 1, hits=True, dsp=True)
        monkeypatch.setenv("ART_TEST_FAIL_SHARD", str(fail_shard))
        with pytest.raises(art.ArtError) as e:
            mctx.schedule(art.Frame(scene, params, org, bad))
        assert e.value.code == abi.ART_E_DEVICE and "injected" in str(e.value)
        monkeypatch.delenv("ART_TEST_FAIL_SHARD")
        good = art.FanOutputs(9, 128, cfg.H, cfg.T, 1, hits=True, dsp=True)
        ref = good.copy()
        mctx.run(art.Frame(scene, params, org, good))  # no frame in flight: schedule is accepted
    oracle.run_frame(art.Frame(scene, params, org, ref), threads=16)
    assert all(good.equal(ref).values()), good.equal(ref)


def test_bench_two_ranks_gloo_strong_shards():
    """bench.py's N > 1 path executes: config 4 (strong scaling, 1024 fans, reduced collider scale)
    as two ranks sharing device 0 over gloo (torch.distributed.run). The strong-scaled shards'
    reference test counts must add up to the single-rank count, and the line reports the
    all-gather time. The RCCL branch is the same code with --dist-backend nccl."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["--config", "4", "--collider-scale", "0.0625", "--steps", "3", "--warmup", "1", "--frames", "1",
              "--no-cpu-baseline", "--no-dynamic"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")

    def run(cmd):
        p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-4000:]
        return json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])

    one = run([sys.executable, "bench.py"] + common)
    two = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
               "--dist-backend", "gloo"] + common)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert two["config"]["fans_total"] == one["config"]["fans_total"] == 1024
    assert two["config"]["fans_rank0"] == 512
    assert two["config"]["reference_tests_per_frame_all"] == one["config"]["reference_tests_per_frame_rank0"]
    assert two["config"]["reference_tests_per_frame_rank0"] < one["config"]["reference_tests_per_frame_rank0"]
    assert two["allgather_ms"] is not None and two["allgather_ms"] > 0
    assert two["allgather_bytes"] > 0 and one["allgather_ms"] is None
    # the N > 1 self-check (outside the timed region): group size, device identities, and the gathered
    # blocks of first / middle / last fans of both shards byte-equal to rank 0's own launch of them
    v = two["allgather_verify"]
    assert two["allgather_verified"] is True and v["world_size"] == 2 and v["backend"] == "gloo"
    assert v["sampled_fans"] == [0, 256, 511, 512, 768, 1023] and v["bytes_compared"] > 0
    assert v["distinct_devices"] is False  # both gloo ranks share device 0 here; under nccl this must be True
    assert one["allgather_verified"] is None


def test_bench_rccl_branch_one_rank():
    """The RCCL branch of bench.py's N > 1 path on one GPU (--force-dist, one rank under
    torch.distributed.run, backend nccl): the process group, the overlap auto-tune (overlapped and
    serial all-gather timed before the timed region, the faster one kept), the all-gathers inside
    the timed steps and the self-check against rank 0's own launch all execute over RCCL (with one
    rank the serial gather measured faster: 0.099 against 0.113 ms per step)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--force-dist",
                        "--steps", "100", "--warmup", "2", "--frames", "1", "--no-cpu-baseline", "--no-dynamic"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    v = r["allgather_verify"]
    assert r["allgather_verified"] is True and v["backend"] == "nccl" and v["world_size"] == 1
    assert v["distinct_devices"] is True and v["bytes_compared"] > 0
    tune = v["overlap_tune"]
    assert tune["chosen"] in ("serial", "overlapped")
    assert tune["serial_ms_per_step"] > 0 and tune["overlapped_ms_per_step"] > 0
    assert r["allgather_ms"] is not None and r["allgather_ms"] > 0
