"""GPU parity: libart.so (HIP, through the C ABI) against the CPU oracle, bit-exact.

Every output array of the reference jobs is compared byte for byte: EchoRayDistances (half),
MuffleRayHits (u16), PermeationPowerRemains (f32 bits), AudioTargetSettings (f32 bits),
DSP parameters, RayHitResults / RayHitResultCounts. Floating-point outputs are required to be
bit-identical (tolerance 0 ULP), which is stricter than north_star's 1e-5 absolute bound.
Test counts (the tests/s metric's numerator) must equal the oracle's per-kind counts.
"""
import os

import numpy as np
import pytest

import art
from art import abi
import oracle

pytestmark = pytest.mark.gpu


def _diff_report(a: art.FanOutputs, b: art.FanOutputs) -> str:
    lines = []
    for name in ("echo", "muffle", "perm", "settings", "dsp", "hit_points", "hit_counts", "hit_ids"):
        x, y = getattr(a, name), getattr(b, name)
        if x is None or y is None:
            continue
        xv = x.view(np.uint8).reshape(x.shape[0], -1)
        yv = y.view(np.uint8).reshape(y.shape[0], -1)
        bad = np.argwhere(xv != yv)
        if bad.size:
            f = bad[0][0]
            lines.append(f"{name}: {len(np.unique(bad[:, 0]))} fans differ; first fan {f}: gpu={x[f].ravel()[:12]} "
                         f"ref={y[f].ravel()[:12]}")
    return "\n".join(lines)


def gpu_vs_oracle(ctx, scene, params, org, hits=False, stale=None, counts=True, prime=None):
    """Run the frame through both raytrace implementations — the throughput stage (BVH nearest
    hits, sorted-batch visibility; art_trace.hip) and the reference-order kernel (one ray per lane,
    every collider in reference order; its counting variant gives the metric's test counts) — and
    require each to equal the oracle bit for bit; the counting run's test counts must equal the
    oracle's."""
    S = org.shape[0]
    o_gpu = art.FanOutputs(S, scene.R, params.max_hits_per_ray, scene.T, params.thread_count, hits=hits,
                           dsp=params.dsp is not None)
    if stale is not None:
        o_gpu.fill_random(stale)
    if prime is not None:
        prime(o_gpu)
    o_ref = o_gpu.copy()
    o_cnt = o_gpu.copy()
    o_ro = o_gpu.copy()
    cref = oracle.run_frame(art.Frame(scene, params, org, o_ref), threads=16)
    ctx.set_flags(0)
    ctx.run(art.Frame(scene, params, org, o_gpu))
    eq = o_gpu.equal(o_ref)
    assert all(eq.values()), f"throughput stage: {eq}\n{_diff_report(o_gpu, o_ref)}"
    ctx.set_flags(abi.ART_CTX_FORCE_REFERENCE_ORDER)
    ctx.run(art.Frame(scene, params, org, o_ro))
    ctx.set_flags(0)
    eq = o_ro.equal(o_ref)
    assert all(eq.values()), f"reference-order kernel: {eq}\n{_diff_report(o_ro, o_ref)}"
    if counts:
        ctx.set_flags(abi.ART_CTX_COUNT_TESTS)
        ctx.run(art.Frame(scene, params, org, o_cnt))
        ctx.set_flags(0)
        eq = o_cnt.equal(o_ref)
        assert all(eq.values()), f"counting kernel: {eq}\n{_diff_report(o_cnt, o_ref)}"
        assert ctx.last_test_counts() == cref
    return o_gpu, cref


# Reduced sizes of BASELINE.json's five configs: (S, R, collider scale)
REDUCED = {1: (8, 64, None), 2: (16, 128, 0.25), 3: (8, 96, 0.125), 4: (8, 128, 1 / 16), 5: (8, 128, 0.25)}


@pytest.mark.parametrize("ci", [1, 2, 3, 4, 5])
def test_config_reduced(ctx, ci):
    S, R, cs = REDUCED[ci]
    scene, org, params = art.synth(art.CONFIGS[ci], S=S, R=R, C_scale=cs)
    out, counts = gpu_vs_oracle(ctx, scene, params, org, hits=True)
    # the case must exercise the path: some echoes returned, some muffle rays clear
    assert (out.echo != 0).any() and (out.muffle != 0).any()
    assert counts["rt_sphere"] + counts["rt_aabb"] + counts["rt_obb"] > 0


@pytest.mark.parametrize("tc,R", [(3, 64), (4, 9), (2, 31), (5, 64)])
def test_thread_count_batches(ctx, tc, R):
    """TC > 1: per-batch muffle slots, permeation slot collapse (Q7), mis-indexed echo reset (Q1),
    never-reset slots keep stale contents (Q18) — sequential-batch semantics."""
    scene, org, params = art.synth(art.CONFIGS[1], S=4, R=R)
    params.thread_count = tc
    gpu_vs_oracle(ctx, scene, params, org, hits=True, stale=7)


def test_stale_single_batch(ctx):
    """TC = 1: every output slot is reset, so stale contents must not leak."""
    scene, org, params = art.synth(art.CONFIGS[5], S=4, R=64, C_scale=0.1)
    gpu_vs_oracle(ctx, scene, params, org, hits=True, stale=3)


def test_stage_subsets(ctx):
    scene, org, params = art.synth(art.CONFIGS[5], S=4, R=64, C_scale=0.1)
    for stages in (abi.ART_STAGE_RAYTRACE, abi.ART_STAGE_PERMEATE, abi.ART_STAGE_REDUCE,
                   abi.ART_STAGE_PERMEATE | abi.ART_STAGE_REDUCE, abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_REDUCE):
        params.stages = stages
        params.dsp = None
        gpu_vs_oracle(ctx, scene, params, org, stale=11)


def test_no_colliders(ctx):
    """Every ray misses: no echoes, no muffle hits, permeation reset to 0 (reference :43-46)."""
    scene, org, params = art.synth(art.CONFIGS[1], S=2, R=64)
    scene.aabbs = scene.aabbs[:0]
    out, _ = gpu_vs_oracle(ctx, scene, params, org, hits=True, stale=5)
    assert not out.echo.any() and not out.muffle.any() and not out.perm.any()


def test_single_type_scenes(ctx):
    for ci, cs in ((2, 0.05), (3, 0.05)):
        scene, org, params = art.synth(art.CONFIGS[ci], S=4, R=64, C_scale=cs)
        params.max_hits_per_ray = 26  # maxBounces 25, the reference's slider maximum (AudioRayTracer.cs:14)
        params.stages = abi.ART_STAGE_ALL
        params.dsp = art.DspSettings.default()
        gpu_vs_oracle(ctx, scene, params, org, hits=True)


def test_one_target_many_targets(ctx):
    scene, org, params = art.synth(art.CONFIGS[5], S=4, R=64, C_scale=0.1)
    one = art.Scene(dirs=scene.dirs, targets=scene.targets[:1].copy(), spheres=scene.spheres, aabbs=scene.aabbs,
                    obbs=scene.obbs)
    gpu_vs_oracle(ctx, one, params, org)
    rng = np.random.default_rng(0)
    many = art.Scene(dirs=scene.dirs, targets=rng.uniform(-10, 10, (37, 3)).astype(np.float32), spheres=scene.spheres,
                     aabbs=scene.aabbs, obbs=scene.obbs)
    gpu_vs_oracle(ctx, many, params, org)


@pytest.mark.parametrize("T", [8, 12, 31, 64, 256])
def test_many_targets_fast_path(ctx, T):
    """The throughput path takes any target count (pair emission in rounds of 8 queries, coarser
    direction cells in the muffle sort key above 8 targets); AudioRaytracerJobBatched.cs:153 loops
    over every target. Multi-hit config-5 scene with permeation and DSP params; targets spread over
    the scene and owning colliders of every kind."""
    scene, org, params = art.synth(art.CONFIGS[5], S=4, R=128, C_scale=0.1)
    rng = np.random.default_rng(T)
    tg = rng.uniform(-20, 20, (T, 3)).astype(np.float32)
    sc = art.Scene(dirs=scene.dirs, targets=tg, spheres=scene.spheres.copy(), aabbs=scene.aabbs.copy(),
                   obbs=scene.obbs.copy())
    for arr in (sc.spheres, sc.aabbs, sc.obbs):
        arr["audio_target_id"] = rng.integers(-1, T, arr.size).astype(np.int16)
    out, _ = gpu_vs_oracle(ctx, sc, params, org, hits=True, counts=(T <= 64))
    assert (out.muffle != 0).any()


def test_full_size_config2_sampled(ctx):
    """Config 2 at full size (256 x 512 x 4096) through the host API with hit outputs: every fan
    checked against the oracle, plus size-independent properties (determinism, fan-permutation
    invariance)."""
    cfg = art.CONFIGS[2]
    scene, org, params = art.synth(cfg)
    out = art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1, hits=True)
    ctx.run(art.Frame(scene, params, org, out))
    sub = np.arange(cfg.S)
    ref = art.FanOutputs(len(sub), cfg.R, cfg.H, cfg.T, 1, hits=True)
    oracle.run(scene, params, org[sub], ref, threads=16)
    for name in ("echo", "muffle", "perm", "settings", "hit_points", "hit_counts", "hit_ids"):
        assert np.array_equal(getattr(out, name)[sub].view(np.uint8), getattr(ref, name).view(np.uint8)), name
    assert (out.hit_ids != abi.ART_HIT_NONE).any()
    # determinism
    out2 = art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1)
    ctx.run(art.Frame(scene, params, org, out2))
    assert all(out.equal(out2).values())
    # permutation invariance: fans are independent
    perm = np.random.default_rng(1).permutation(cfg.S)
    out3 = art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1)
    ctx.run(art.Frame(scene, params, np.ascontiguousarray(org[perm]), out3))
    assert np.array_equal(out3.echo, out.echo[perm]) and np.array_equal(out3.settings.view(np.uint8),
                                                                         out.settings[perm].view(np.uint8))


@pytest.mark.parametrize("ci,every", [(3, 4), (5, 4), (4, 64)])
def test_full_size_sampled(ctx, ci, every):
    """Full-size configs through the host API, every `every`-th fan byte-compared with the oracle.
    Config 4 (1024 fans x 1024 rays x 16384 mixed colliders: 16384 ray groups, 5.2 M visibility
    pairs) is the launch shape the sharded bench runs per rank at G = 1."""
    cfg = art.CONFIGS[ci]
    scene, org, params = art.synth(cfg)
    dsp = params.dsp is not None
    out = art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1, dsp=dsp, hits=True)
    ctx.set_flags(0)
    ctx.run(art.Frame(scene, params, org, out))
    sub = np.arange(0, cfg.S, every)
    ref = art.FanOutputs(len(sub), cfg.R, cfg.H, cfg.T, 1, dsp=dsp, hits=True)
    oracle.run(scene, params, np.ascontiguousarray(org[sub]), ref, threads=16)
    for name in ("echo", "muffle", "perm", "settings", "hit_points", "hit_counts", "hit_ids") + (("dsp",) if dsp else ()):
        assert np.array_equal(getattr(out, name)[sub].view(np.uint8), getattr(ref, name).view(np.uint8)), name


@pytest.mark.parametrize("ci,every,first", [(2, 1, 0), (3, 1, 0), (5, 1, 0), (4, 4, 0), (4, 4, 1), (4, 4, 2), (4, 4, 3)])
def test_full_size_bench_path(ctx, ci, every, first):
    """The launch bench.py times, at full size: art_scene_bind + art_launch_device on HBM buffers
    with no hit outputs (out_flags 0) and context flags 0. The one-hit configs (2, 3, 4) then run
    nearest_first_kernel -> echo_muffle_kernel -> reduce (no path kernel); config 5 (H = 5, one
    batch slot, no hit outputs) runs the folded plan: per bounce nearest_first_kernel<..., FOLD>
    (the path kernel's work in its epilogue) and that bounce's echo vis_kernel, then one
    muffle_kernel over every bounce's fixed slots. Every fan of configs 2, 3 and 5, and every fan
    of config 4 (the strong-scaled job's 1024 fans at G = 1, in four cases of 256 fans: fans
    first, first + 4, ...) are byte-compared with the oracle (AudioRaytracerJobBatched.cs:61-215, AudioPermeationJobBatched.cs:34-91,
    ProcessAudioDataJob.cs:32-76)."""
    torch = pytest.importorskip("torch")
    cfg = art.CONFIGS[ci]
    scene, org, params = art.synth(cfg)
    dsp = params.dsp is not None
    fr = art.Frame(scene, params, org, art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1, dsp=dsp))
    lay = art.fan_layout(fr)
    ctx.set_flags(0)
    ctx.bind(fr)
    d_org = torch.from_numpy(np.ascontiguousarray(org)).cuda()
    d_blk = torch.full((cfg.S * lay["stride"],), 0xA5, dtype=torch.uint8, device="cuda")  # no stale zeros
    st = torch.cuda.current_stream()
    for _ in range(2):  # the second launch reuses the first's accumulators and counters
        ctx.launch_device(d_org.data_ptr(), cfg.S, d_blk.data_ptr(), 0, st.cuda_stream)
    st.synchronize()
    got = art.unpack_block(d_blk.cpu().numpy(), lay, cfg.S, cfg.R, cfg.H, cfg.T, 1, dsp=dsp)
    sub = np.arange(first, cfg.S, every)
    # the oracle starts from the same stale bytes (slots a stage does not write keep them)
    ref = art.unpack_block(np.full(len(sub) * lay["stride"], 0xA5, np.uint8), lay, len(sub), cfg.R, cfg.H, cfg.T, 1,
                           dsp=dsp)
    oracle.run(scene, params, np.ascontiguousarray(org[sub]), ref, threads=16)
    for name in ("echo", "muffle", "perm", "settings") + (("dsp",) if dsp else ()):
        g, r = getattr(got, name)[sub].view(np.uint8), getattr(ref, name).view(np.uint8)
        bad = np.unique(np.argwhere(g.reshape(len(sub), -1) != r.reshape(len(sub), -1))[:, 0])
        assert bad.size == 0, f"{name}: {bad.size} of {len(sub)} fans differ (first: fan {sub[bad[0]]})"
    assert (got.echo != 0).any() and (got.muffle != 0).any()


def test_full_frame_test_counts_config2(ctx):
    """value's numerator: art_count_device over the whole config-2 frame (256 x 512 x 4096, the
    launch bench.py counts) equals the oracle's per-kind test counts over the same 256 fans
    (2,051,075,633 in total; SURVEY.md §8 d, ShootRayCast / CanRaySeePoint / CanRaySeeAudioTarget
    :225-449). The counting launch also writes every fan's outputs (the reference-order kernels):
    all 256 fans' echo, muffle and settings bytes must equal the oracle's."""
    torch = pytest.importorskip("torch")
    cfg = art.CONFIGS[2]
    scene, org, params = art.synth(cfg)
    fr = art.Frame(scene, params, org, art.FanOutputs(cfg.S, cfg.R, cfg.H, cfg.T, 1))
    lay = art.fan_layout(fr)
    ctx.set_flags(0)
    ctx.bind(fr)
    d_org = torch.from_numpy(np.ascontiguousarray(org)).cuda()
    d_blk = torch.full((cfg.S * lay["stride"],), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    counts = ctx.count_device(d_org.data_ptr(), cfg.S, d_blk.data_ptr(), 0, st.cuda_stream)
    st.synchronize()
    ref = art.unpack_block(np.full(cfg.S * lay["stride"], 0xA5, np.uint8), lay, cfg.S, cfg.R, cfg.H, cfg.T, 1)
    cref = oracle.run(scene, params, org, ref, threads=16)[1]
    assert counts == cref
    assert sum(counts.values()) == 2_051_075_633
    got = art.unpack_block(d_blk.cpu().numpy(), lay, cfg.S, cfg.R, cfg.H, cfg.T, 1)
    for name in ("echo", "muffle", "perm", "settings"):
        assert np.array_equal(getattr(got, name).view(np.uint8), getattr(ref, name).view(np.uint8)), name


def test_device_resident_path(ctx):
    """art_scene_bind + art_launch_device on torch-allocated HBM buffers gives the same bytes as
    art_schedule/art_complete."""
    torch = pytest.importorskip("torch")
    cfg = art.CONFIGS[5]
    scene, org, params = art.synth(cfg, S=16, R=128, C_scale=0.25)
    out = art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True, hits=True)
    fr = art.Frame(scene, params, org, out)
    ctx.run(fr)
    lay = art.fan_layout(fr, abi.ART_OUT_HIT_RESULTS)
    ctx.bind(fr)
    d_org = torch.from_numpy(org.copy()).cuda()
    d_blk = torch.zeros(16 * lay["stride"], dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    ctx.launch_device(d_org.data_ptr(), 16, d_blk.data_ptr(), abi.ART_OUT_HIT_RESULTS, st.cuda_stream)
    st.synchronize()
    got = art.unpack_block(d_blk.cpu().numpy(), lay, 16, 128, cfg.H, cfg.T, 1, hits=True, dsp=True)
    assert all(got.equal(out).values())
    counts = ctx.count_device(d_org.data_ptr(), 16, d_blk.data_ptr(), 0, st.cuda_stream)
    ref = art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True)
    assert counts == oracle.run(scene, params, org, ref, threads=16)[1]


def test_schedule_is_completed_complete(ctx):
    scene, org, params = art.synth(art.CONFIGS[1])
    out = art.FanOutputs(8, 64, 5, 4, 1)
    h = ctx.schedule(art.Frame(scene, params, org, out))
    with pytest.raises(art.ArtError):  # one frame in flight per context (AudioRayTracer.cs:95-97)
        ctx.schedule(art.Frame(scene, params, org, art.FanOutputs(8, 64, 5, 4, 1)))
    while not h.is_completed:
        pass
    h.complete()
    h.complete()  # idempotent, like JobHandle.Complete
    assert (out.echo != 0).any()


def test_invalid_arguments(ctx):
    scene, org, params = art.synth(art.CONFIGS[1], S=2)
    bad = art.Scene(dirs=scene.dirs, targets=scene.targets[:0], aabbs=scene.aabbs)
    with pytest.raises(art.ArtError) as e:
        ctx.run(art.Frame(bad, params, org, art.FanOutputs(2, 64, 5, 1, 1)))
    assert e.value.code == abi.ART_E_INVALID
    params.max_hits_per_ray = 40
    with pytest.raises(art.ArtError) as e:
        ctx.run(art.Frame(scene, params, org, art.FanOutputs(2, 64, 40, 4, 1)))
    assert e.value.code == abi.ART_E_UNSUPPORTED


# ---------------------------------------------------------------- known answers and fixtures
import golden_util as G  # noqa: E402
import kat_scenes as K  # noqa: E402


@pytest.mark.parametrize("name", sorted(K.KATS))
def test_kats_on_gpu(ctx, name):
    """Hand-derived answers hold on the HIP path, through both kernels."""
    sc, p, org, expect, *prime = K.KATS[name]()
    out, _ = gpu_vs_oracle(ctx, sc, p, org, hits=True, prime=prime[0] if prime else None)
    expect(out)


def test_k9_reduce_on_gpu(ctx):
    sc, p, org, expect, prime = K.k9_reduce()
    out = art.FanOutputs(1, sc.R, p.max_hits_per_ray, sc.T, 1)
    prime(out)
    ctx.run(art.Frame(sc, p, org, out))
    expect(out)


@pytest.mark.parametrize("name", G.names())
def test_golden_on_gpu(ctx, name):
    """The HIP path reproduces the committed fixtures (and their test counts) bit for bit."""
    scene, org, params, fresh, expected, counts = G.load(name)
    cnt_out = fresh.copy()
    ctx.set_flags(0)
    ctx.run(art.Frame(scene, params, org, fresh))
    assert all(fresh.equal(expected).values()), _diff_report(fresh, expected)
    ctx.set_flags(abi.ART_CTX_COUNT_TESTS)
    ctx.run(art.Frame(scene, params, org, cnt_out))
    ctx.set_flags(0)
    assert all(cnt_out.equal(expected).values())
    assert ctx.last_test_counts() == counts


@pytest.mark.gpu
def test_inputs_change_between_frames(ctx):
    """art_schedule reuses the device scene (records, sorted copies, BVH) when the packed inputs are
    byte-identical to the last frame's; any change — every sphere moved, one radius changed,
    the targets moved — must rebuild it. Each frame is checked against the oracle."""
    scene, org, params = art.synth(art.CONFIGS[2], S=8, R=128, C_scale=0.25)
    base_c = scene.spheres["center"].copy()
    base_r = scene.spheres["radius"].copy()
    base_t = scene.targets.copy()

    def check():
        o_gpu = art.FanOutputs(8, scene.R, params.max_hits_per_ray, scene.T, params.thread_count)
        o_ref = o_gpu.copy()
        oracle.run_frame(art.Frame(scene, params, org, o_ref), threads=16)
        ctx.set_flags(0)
        ctx.run(art.Frame(scene, params, org, o_gpu))
        eq = o_gpu.equal(o_ref)
        assert all(eq.values()), f"{eq}\n{_diff_report(o_gpu, o_ref)}"
        return o_gpu

    a = check()
    check()                                           # identical inputs: cached scene
    scene.spheres["center"][:] = base_c[::-1]         # every sphere moved
    b = check()
    scene.spheres["radius"][:] = base_r
    scene.spheres["center"][:] = base_c
    scene.spheres["radius"][3] = scene.spheres["radius"][3] ^ 0x0400  # one radius changed
    check()
    scene.spheres["radius"][:] = base_r
    scene.targets[:] = base_t[::-1]                   # only the targets moved
    check()
    scene.targets[:] = base_t
    c = check()                                       # back to the first frame's inputs
    assert all(c.equal(a).values()) and not all(b.equal(a).values())


def test_fan_chunks_equal_one_launch(ctx, monkeypatch):
    """Frames larger than the fast path's 32-bit pair / block offsets run as consecutive fan chunks
    (fast_fans_per_launch); forcing 3-fan chunks must not change a byte (muffle accumulators,
    pair counter reset per chunk, multi-hit ray state)."""
    for ci in (2, 5):
        scene, org, params = art.synth(art.CONFIGS[ci], S=11, R=128, C_scale=0.1)
        a = art.FanOutputs(11, 128, params.max_hits_per_ray, scene.T, 1, hits=True, dsp=params.dsp is not None)
        b = a.copy()
        ctx.set_flags(0)
        ctx.run(art.Frame(scene, params, org, a))
        monkeypatch.setenv("ART_FAST_CHUNK_FANS", "3")
        ctx.run(art.Frame(scene, params, org, b))
        monkeypatch.delenv("ART_FAST_CHUNK_FANS")
        assert all(a.equal(b).values()), a.equal(b)


def test_bind_and_launch_refused_while_in_flight(ctx):
    """art_scene_bind / art_launch_device between art_schedule and art_complete would overwrite the
    in-flight frame's layout and staging: they return ART_E_STATE; the frame still completes."""
    scene, org, params = art.synth(art.CONFIGS[1])
    out = art.FanOutputs(8, 64, 5, 4, 1)
    ref = out.copy()
    fr = art.Frame(scene, params, org, out)
    h = ctx.schedule(fr)
    with pytest.raises(art.ArtError) as e:
        ctx.bind(fr)
    assert e.value.code == abi.ART_E_STATE
    with pytest.raises(art.ArtError) as e:
        ctx.launch_device(1, 1, 1)
    assert e.value.code == abi.ART_E_STATE
    h.complete()
    oracle.run_frame(art.Frame(scene, params, org, ref), threads=8)
    assert all(out.equal(ref).values())


def test_deep_bvh_large_scene(ctx):
    """122,880 colliders: a 9-level BVH (87,381 nodes, past the old 16-bit traversal stacks) built
    level by level; nearest hits, echo traversal and the muffle sweep against the oracle."""
    scene, org, params = art.synth(art.CONFIGS[5], S=3, R=128, C_scale=30)
    params.max_hits_per_ray = 3
    assert scene.C > 4 * 4 ** 7
    out, _ = gpu_vs_oracle(ctx, scene, params, org, hits=True, counts=False)
    assert (out.echo != 0).any()


def test_launch_device_then_schedule_and_bind_without_sync(ctx):
    """art_launch_device returns without synchronizing; an art_schedule (or art_scene_bind) issued
    right after rewrites the device scene and reuses the context's buffers on the context stream,
    so it must wait for the launched frame. Scene A is bound and launched on torch's
    stream; frame B (other colliders) is scheduled at once through the host API, then A is bound
    again and launched, and scene C is bound with A's launch still queued: every result equals the
    oracle."""
    torch = pytest.importorskip("torch")
    cfg = art.CONFIGS[5]
    sa, org, params = art.synth(cfg, S=16, R=128, C_scale=0.25)
    sb, _, _ = art.synth(art.CONFIGS[2], S=16, R=128, C_scale=0.25)
    sb = art.Scene(dirs=sa.dirs, targets=sa.targets, spheres=sb.spheres, aabbs=sb.aabbs)
    fa = art.Frame(sa, params, org, art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True))
    lay = art.fan_layout(fa)
    ref_a = art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True)
    oracle.run_frame(art.Frame(sa, params, org, ref_a), threads=16)
    ref_b = art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True)
    oracle.run_frame(art.Frame(sb, params, org, ref_b), threads=16)
    d_org = torch.from_numpy(org.copy()).cuda()
    st = torch.cuda.current_stream()
    for rnd in range(3):
        ctx.set_flags(0)
        ctx.bind(fa)
        d_blk = torch.zeros(16 * lay["stride"], dtype=torch.uint8, device="cuda")
        ctx.launch_device(d_org.data_ptr(), 16, d_blk.data_ptr(), 0, st.cuda_stream)
        ob = art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True)
        if rnd == 2:  # bind another scene instead of scheduling
            ctx.bind(art.Frame(sb, params, org, ob))
        else:
            ctx.run(art.Frame(sb, params, org, ob))
            assert all(ob.equal(ref_b).values()), ob.equal(ref_b)
        st.synchronize()
        got = art.unpack_block(d_blk.cpu().numpy(), lay, 16, 128, cfg.H, cfg.T, 1, dsp=True)
        assert all(got.equal(ref_a).values()), (rnd, got.equal(ref_a))


def _hip_runtime():
    """The HIP runtime already loaded in this process (libart's and torch's), without loading another."""
    import ctypes
    for name in ("libamdhip64.so.7", "libamdhip64.so"):
        try:
            return ctypes.CDLL(name, mode=os.RTLD_NOLOAD)
        except OSError:
            continue
    pytest.skip("no loaded HIP runtime found")


def test_launch_streams_short_lived_and_busy():
    """The lazy completion event: art_launch_device records no event, the next call
    that reuses the scene records one on the launch stream. (1) A frame launched on a side stream
    that then gets more unrelated work, followed by a bind of a changed scene, a launch of it on
    another stream and art_destroy: both frames equal the oracle. (2) With ART_CTX_EVENT_EACH_LAUNCH
    the frame's event is recorded by the launch itself, so the caller may destroy its stream at once:
    a raw HIP stream is destroyed right after the launch, a changed scene is bound and launched, and
    the context destroyed, with every result equal to the oracle."""
    import ctypes
    torch = pytest.importorskip("torch")
    cfg = art.CONFIGS[5]
    sa, org, params = art.synth(cfg, S=16, R=128, C_scale=0.25)
    sb, _, _ = art.synth(art.CONFIGS[2], S=16, R=128, C_scale=0.25)
    sb = art.Scene(dirs=sa.dirs, targets=sa.targets, spheres=sb.spheres, aabbs=sb.aabbs)
    refs = {}
    for k, sc in (("a", sa), ("b", sb)):
        refs[k] = art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True)
        oracle.run_frame(art.Frame(sc, params, org, refs[k]), threads=16)
    fa = art.Frame(sa, params, org, art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True))
    fb = art.Frame(sb, params, org, art.FanOutputs(16, 128, cfg.H, cfg.T, 1, dsp=True))
    lay = art.fan_layout(fa)
    d_org = torch.from_numpy(org.copy()).cuda()
    hip = _hip_runtime()
    for mode in ("busy side stream", "destroyed stream"):
        c = art.Context(1)
        d_a = torch.zeros(16 * lay["stride"], dtype=torch.uint8, device="cuda")
        d_b = torch.zeros_like(d_a)
        c.set_flags(abi.ART_CTX_EVENT_EACH_LAUNCH if mode == "destroyed stream" else 0)
        c.bind(fa)
        if mode == "busy side stream":
            side = torch.cuda.Stream()
            c.launch_device(d_org.data_ptr(), 16, d_a.data_ptr(), 0, side.cuda_stream)
            with torch.cuda.stream(side):  # unrelated work queued behind the frame
                x = torch.randn(1 << 22, device="cuda")
                for _ in range(8):
                    x = torch.sin(x) * 1.0001
        else:
            raw = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
            c.launch_device(d_org.data_ptr(), 16, d_a.data_ptr(), 0, raw.value)
            assert hip.hipStreamDestroy(raw) == 0  # the caller drops its stream right after the launch
        c.bind(fb)
        st = torch.cuda.current_stream()
        c.launch_device(d_org.data_ptr(), 16, d_b.data_ptr(), 0, st.cuda_stream)
        c.close()
        torch.cuda.synchronize()
        for k, d in (("a", d_a), ("b", d_b)):
            got = art.unpack_block(d.cpu().numpy(), lay, 16, 128, cfg.H, cfg.T, 1, dsp=True)
            assert all(got.equal(refs[k]).values()), (mode, k, got.equal(refs[k]))


@pytest.mark.parametrize("ci", [2, 5])
def test_kernel_timing_launch_counts(ctx, ci):
    """ART_CTX_TIME_EACH_KERNEL (bench.py's per-kernel roofline times): the launches counted per
    kernel family follow the frame's plan — a one-hit frame (config 2) is one nearest_first_kernel and
    one echo_muffle_kernel launch; a folded multi-hit frame (config 5, H = 5) is H nearest launches,
    H echo vis_kernel launches and one muffle_kernel launch — no mark is dropped, and every family
    that ran has a positive time."""
    torch = pytest.importorskip("torch")
    cfg = art.CONFIGS[ci]
    scene, org, params = art.synth(cfg, S=32, R=cfg.R, C_scale=0.25)
    fr = art.Frame(scene, params, org, art.FanOutputs(32, cfg.R, cfg.H, cfg.T, 1, dsp=params.dsp is not None))
    lay = art.fan_layout(fr)
    ctx.set_flags(0)
    ctx.bind(fr)
    d_org = torch.from_numpy(np.ascontiguousarray(org)).cuda()
    d_blk = torch.zeros(32 * lay["stride"], dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    n = 6
    ctx.set_flags(abi.ART_CTX_TIME_KERNELS | abi.ART_CTX_TIME_EACH_KERNEL)
    ctx.kernel_timing()  # reset
    for _ in range(n):
        ctx.launch_device(d_org.data_ptr(), 32, d_blk.data_ptr(), 0, st.cuda_stream)
    t = ctx.kernel_timing()
    ctx.set_flags(0)
    want = ({"nearest_first_kernel": 1, "echo_muffle_kernel": 1, "vis_kernel": 0, "muffle_kernel": 0} if cfg.H == 1 else
            {"nearest_first_kernel": cfg.H, "echo_muffle_kernel": 0, "vis_kernel": cfg.H, "muffle_kernel": 1})
    assert t["launches"] == n and t["kernel_marks_dropped"] == 0
    assert {k: v // n for k, v in t["kernel_launches"].items()} == want
    assert all(t["kernel_launches"][k] == n * w for k, w in want.items())
    assert all((t["kernel_ms"][k] > 0) == (w > 0) for k, w in want.items())
