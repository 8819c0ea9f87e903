"""GPU parity of the broad phase on adversarial scenes.

The throughput kernel culls colliders per wave with a bounding box of the wave's segments widened
by a rounding margin (broad phase). A wrong margin can only show up where the
reference's float tests report hits that the true geometry does not have: grazing rays on tiny
or far spheres, rays in the plane of a box face, huge coordinates, degenerate and non-finite
colliders. Every scene here is compared bit for bit with the brute-force oracle, through the
throughput stage and the reference-order kernel (gpu_vs_oracle).
"""
import numpy as np
import pytest

import art
from art import abi
from art.synth import fibonacci_directions
from test_parity_gpu import gpu_vs_oracle

pytestmark = pytest.mark.gpu


def f16bits(x) -> np.ndarray:
    return np.asarray(x, np.float32).astype(np.float16).view(np.uint16)


def spheres(centers, radii, rng, tid=None):
    n = len(radii)
    s = np.zeros(n, abi.SPHERE)
    s["center"] = f16bits(centers).reshape(n, 3)
    s["radius"] = f16bits(radii)
    s["material"] = f16bits(rng.uniform(0.0, 1.0, (n, 3)))
    s["audio_target_id"] = -1 if tid is None else tid
    return s


def aabbs(centers, halves, rng, tid=None):
    n = len(centers)
    a = np.zeros(n, abi.AABB)
    a["center"] = f16bits(centers).reshape(n, 3)
    a["size"] = f16bits(halves).reshape(n, 3)
    a["material"] = f16bits(rng.uniform(0.0, 1.0, (n, 3)))
    a["audio_target_id"] = -1 if tid is None else tid
    return a


def obbs(centers, halves, rng):
    n = len(centers)
    b = np.zeros(n, abi.OBB)
    b["center"] = f16bits(centers).reshape(n, 3)
    b["size"] = f16bits(halves).reshape(n, 3)
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    q[q[:, 3] < 0] *= -1
    b["rot"] = f16bits(q[:, :3])
    b["material"] = f16bits(rng.uniform(0.0, 1.0, (n, 3)))
    b["audio_target_id"] = -1
    return b


def fib_dirs(R):
    return fibonacci_directions(R)


def run(ctx, scene, org, H=2, T_owned=False):
    # the permeation job too: its first-hit cast and loss rays run over the same BVH
    params = art.FrameParams(max_hits_per_ray=H, max_ray_life=1e4, max_muffle_hit_distance=1e5,
                             stages=abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_PERMEATE | abi.ART_STAGE_REDUCE)
    out, counts = gpu_vs_oracle(ctx, scene, params, org, hits=True, counts=False)
    return out


def test_grazing_tiny_far_spheres(ctx):
    """Spheres of radius 2^-10..2^-4 placed tangent to (or a hair off) the rays, far away: the
    discriminant cancels, so the float test reports hits the geometry does not have."""
    rng = np.random.default_rng(11)
    R = 128
    dirs_bits = fib_dirs(R)
    d = dirs_bits.view(np.float16).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    n = 1500
    k = rng.integers(0, R, n)
    dist = rng.uniform(50.0, 900.0, n).astype(np.float32)
    r = (2.0 ** rng.uniform(-10, -4, n)).astype(np.float32)
    perp = rng.normal(size=(n, 3)).astype(np.float32)
    perp -= (perp * d[k]).sum(1, keepdims=True) * d[k]
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    offset = r * rng.choice([0.999, 1.0, 1.001, 0.9, 1.1], n).astype(np.float32)
    centers = d[k] * dist[:, None] + perp * offset[:, None]
    targets = (rng.normal(size=(4, 3)) * 300).astype(np.float32)
    # a few big walls so that rays hit and spawn echo / muffle segments past the tiny spheres
    walls = aabbs(rng.uniform(-1000, 1000, (64, 3)), rng.uniform(20, 120, (64, 3)), rng)
    scene = art.Scene(dirs=dirs_bits, targets=targets, spheres=spheres(centers, r, rng), aabbs=walls)
    org = np.zeros((6, 3), np.float32)
    org[1:] = rng.uniform(-5, 5, (5, 3))
    out = run(ctx, scene, org)
    assert (out.echo != 0).any()


def test_huge_coordinates(ctx):
    """Coordinates near the half range (|x| up to 3e4) and long segments."""
    rng = np.random.default_rng(12)
    R = 96
    n = 800
    centers = rng.uniform(-30000, 30000, (n, 3)).astype(np.float32)
    scene = art.Scene(dirs=fib_dirs(R), targets=rng.uniform(-30000, 30000, (3, 3)).astype(np.float32),
                      spheres=spheres(centers[:400], rng.uniform(100, 4000, 400), rng),
                      aabbs=aabbs(centers[400:], rng.uniform(50, 3000, (400, 3)), rng))
    org = rng.uniform(-20000, 20000, (8, 3)).astype(np.float32)
    run(ctx, scene, org, H=3)


def test_axis_aligned_face_planes(ctx):
    """Rays along the axes (zero direction components, infinite 1/d) from origins lying exactly in
    box face planes, and boxes with zero or negative half-extents."""
    rng = np.random.default_rng(13)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1],
                     [1, 1, 0], [0, 1, -1], [1, 0, 1]], np.float32)
    dirs = f16bits(axes / np.linalg.norm(axes, axis=1, keepdims=True)).reshape(-1, 3)
    n = 600
    c = rng.integers(-20, 20, (n, 3)).astype(np.float32)
    hlf = rng.integers(0, 4, (n, 3)).astype(np.float32)
    hlf[rng.random((n, 3)) < 0.1] *= -1  # negative half-extents swap the slab bounds
    org = np.array([[0, 0, 0], [1, 1, 1], [2, 0, -3], [0.5, 0, 0]], np.float32)
    c[:8] = org[0] + np.array([1, 0, 0])  # faces exactly through the origin's planes
    hlf[:8] = 1
    scene = art.Scene(dirs=dirs, targets=np.array([[3, 3, 3], [-7, 2, 0]], np.float32),
                      aabbs=aabbs(c, hlf, rng), spheres=spheres(c[:50] + 0.5, np.full(50, 0.5), rng))
    run(ctx, scene, org, H=4)


def test_nonfinite_and_degenerate_colliders(ctx):
    """Colliders carrying NaN / inf half values, zero radius and zero size mixed into a normal scene."""
    rng = np.random.default_rng(14)
    cfg = art.CONFIGS[5]
    scene, org, params = art.synth(cfg, S=4, R=64, C_scale=0.1)
    sp, ab, ob = scene.spheres.copy(), scene.aabbs.copy(), scene.obbs.copy()
    nan, inf, ninf = np.uint16(0x7E00), np.uint16(0x7C00), np.uint16(0xFC00)
    sp["radius"][:3] = [nan, inf, 0]
    sp["center"][3] = [inf, 0, 0]
    ab["size"][:3] = [[nan, 1, 1], [inf, inf, inf], [0, 0, 0]]
    ab["center"][3] = [ninf, 0, 0]
    ob["rot"][:2] = [[nan, 0, 0], [0x3C00, 0x3C00, 0x3C00]]
    ob["size"][2] = [inf, 1, 1]
    scene = art.Scene(dirs=scene.dirs, targets=scene.targets, spheres=sp, aabbs=ab, obbs=ob)
    run(ctx, scene, org, H=3)


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_dense_random_scenes(ctx, seed):
    """Random mixed scenes with targets inside colliders and origins inside boxes."""
    rng = np.random.default_rng(seed)
    R = 128
    n = 1200
    c = rng.uniform(-40, 40, (n, 3)).astype(np.float32)
    scene = art.Scene(dirs=fib_dirs(R), targets=np.concatenate([c[:2], rng.uniform(-40, 40, (2, 3))]).astype(np.float32),
                      spheres=spheres(c[:500], rng.uniform(0.05, 3, 500), rng, tid=rng.integers(-1, 4, 500)),
                      aabbs=aabbs(c[500:1000], rng.uniform(0.05, 3, (500, 3)), rng, tid=rng.integers(-1, 4, 500)),
                      obbs=obbs(c[1000:], rng.uniform(0.05, 3, (200, 3)), rng))
    org = np.concatenate([c[500:503], rng.uniform(-40, 40, (5, 3))]).astype(np.float32)
    run(ctx, scene, org, H=3)


def test_razor_thin_segments_tiny_spheres(ctx):
    """The case the margin exists for. Every ray of a fan points along -x, so each wave's segments
    (echo back to the origin, muffle rays to targets on the x axis) form a box only ~1e-2 thick in
    y. Tiny spheres (r = 2^-7) sit just above that box: their exact bounds do not overlap it, but
    the reference's float discriminant (b^2 - 4ac cancels at |oc| ~ 100) still reports many of
    them as blocking (a float32 restatement finds blocks up to 0.03 off the sphere). A cull
    without the rounding margin misses those blocks; this scene then differs from the oracle."""
    rng = np.random.default_rng(31)
    R = 64
    dirs = np.tile(np.array([[0xBC00, 0, 0]], np.uint16), (R, 1))  # (-1, 0, 0) exactly
    deltas = np.array([1e-6, 1e-5, 1e-4, 1e-3, 4e-3, 1e-2, 2e-2, 3e-2], np.float32)
    org = np.stack([np.zeros(8), -deltas, np.zeros(8)], 1).astype(np.float32)
    targets = np.array([[100, -1e-5, 0], [100, -3e-3, 0], [100, -1.5e-2, 0], [60, -2.5e-2, 0]], np.float32)
    r = 2.0 ** -7
    cx = np.arange(-95, 96, 1.0, dtype=np.float32)
    centers = np.stack([cx, np.full_like(cx, r), np.zeros_like(cx)], 1)
    sp = spheres(centers, np.full(cx.size, r, np.float32), rng)
    wall = aabbs(np.array([[-101, 0, 0]], np.float32), np.array([[1, 50, 50]], np.float32), rng)
    scene = art.Scene(dirs=dirs, targets=targets, spheres=sp, aabbs=wall)
    params = art.FrameParams(max_hits_per_ray=1, max_ray_life=1e4, max_muffle_hit_distance=1e5,
                             stages=abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_REDUCE)
    out, _ = gpu_vs_oracle(ctx, scene, params, org, hits=True, counts=False)
    # the scene must contain both verdicts: some muffle rays blocked by a sphere, some clear
    assert (out.muffle != 0).any() and (out.muffle != R).any()


def test_bvh_exact_ties_across_leaves(ctx):
    """Exact distance ties spread over many BVH leaves: along each axis a sphere and an AABB both
    report distance 8 (K11), each duplicated 40 times at random list positions among 2000 clutter
    colliders, so the copies land in different leaves and subtrees. The nearest hit must still be
    the reference's first minimum (the lowest-index sphere), which needs every node whose entry
    equals the current best to be visited."""
    rng = np.random.default_rng(41)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    dirs = f16bits(axes).reshape(-1, 3)
    n_clutter, dup = 2000, 40
    sc_c = rng.uniform(-60, 60, (n_clutter, 3)).astype(np.float32)
    sc_c[np.abs(sc_c).min(1) < 12] += 30.0  # keep clutter off the axes near the origin
    s_centers = np.concatenate([sc_c[:1000], np.repeat(axes * 10.0, dup, 0)])
    s_radii = np.concatenate([rng.uniform(0.1, 2, 1000), np.full(6 * dup, 2.0)]).astype(np.float32)
    a_centers = np.concatenate([sc_c[1000:], np.repeat(axes * 9.0, dup, 0)])
    a_halves = np.concatenate([rng.uniform(0.1, 2, (1000, 3)), np.ones((6 * dup, 3))]).astype(np.float32)
    ps, pa = rng.permutation(len(s_radii)), rng.permutation(len(a_halves))
    scene = art.Scene(dirs=dirs, targets=np.array([[0, 0, 30], [25, 25, 0]], np.float32),
                      spheres=spheres(s_centers[ps], s_radii[ps], rng), aabbs=aabbs(a_centers[pa], a_halves[pa], rng))
    org = np.zeros((3, 3), np.float32)
    params = art.FrameParams(max_hits_per_ray=3, max_ray_life=1e4, max_muffle_hit_distance=1e5,
                             stages=abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_REDUCE)
    o_gpu, _ = gpu_vs_oracle(ctx, scene, params, org, hits=True, counts=False)
    assert (o_gpu.hit_counts != 0).all()
    # the first hit of axis ray k is the lowest-index copy of the sphere on that axis (hit ids)
    s_pos = s_centers[ps]
    for k in range(6):
        first = int(np.flatnonzero((s_pos == axes[k] * 10.0).all(1)).min())
        assert (o_gpu.hit_ids[:, k * 3] == abi.hit_id(abi.ART_COLLIDER_SPHERE, first)).all(), k


# ---------------------------------------------------------------- muffle cell-list limits
def _targets_scene(cfg_index, S, R, scale, T, seed):
    scene, org, params = art.synth(art.CONFIGS[cfg_index], S=S, R=R, C_scale=scale)
    rng = np.random.default_rng(seed)
    sc = art.Scene(dirs=scene.dirs, targets=rng.uniform(-20, 20, (T, 3)).astype(np.float32),
                   spheres=scene.spheres.copy(), aabbs=scene.aabbs.copy(), obbs=scene.obbs.copy())
    for arr in (sc.spheres, sc.aabbs, sc.obbs):
        arr["audio_target_id"] = rng.integers(-1, T, arr.size).astype(np.int16)
    return sc, org, params


def _muffle_fallback_rays(sc, params, org):
    with art.Context(1) as c:
        c.set_flags(abi.ART_CTX_COUNT_EXECUTED)
        c.executed_counts()
        c.run(art.Frame(sc, params, org, art.FanOutputs(org.shape[0], sc.R, params.max_hits_per_ray, sc.T,
                                                         params.thread_count, dsp=params.dsp is not None)))
        return c.executed_counts()["muffle_fallback"]


@pytest.mark.parametrize("hook,value", [("ART_CELLS_MAX_PAIRS", "100"), ("ART_CELLS_CAP", "3000")])
def test_cell_lists_disabled_or_overflowing(monkeypatch, hook, value):
    """Scenes past the list limits: above the (target, collider) pair threshold the lists
    are not built and every muffle ray tests every collider; past the entry capacity the targets that
    do not fit are dropped in order (the u32 scan of the kept counts cannot wrap) and only theirs fall
    back. Both lowered here by the test hooks; every output equals the oracle (CanRaySeeAudioTarget
    AudioRaytracerJobBatched.cs:405-449), and the fallback is seen in the executed counts."""
    sc, org, params = _targets_scene(5, 4, 128, 0.25, 6, 11)
    assert _muffle_fallback_rays(sc, params, org) == 0
    monkeypatch.setenv(hook, value)
    with art.Context(1) as c:  # a fresh context: the scene (and its lists) is rebuilt under the hook
        gpu_vs_oracle(c, sc, params, org, hits=True)
    assert _muffle_fallback_rays(sc, params, org) > 0


def test_cell_lists_threshold_real_size():
    """T * C just above the 2^23-pair threshold (256 targets x 32,784 colliders): the lists are skipped
    (no 512-MiB scratch, no launch past HIP's 2^32 work-item limit) and the frame still equals the
    oracle; just below it (255 targets) the lists are built and used."""
    for T, scale in ((256, 32784 / 4096), (255, 32784 / 4096)):
        sc, org, params = _targets_scene(2, 1, 32, scale, T, 5)
        assert T * sc.C > (1 << 23) if T == 256 else T * sc.C <= (1 << 23), sc.C
        with art.Context(1) as c:
            gpu_vs_oracle(c, sc, params, org, hits=False, counts=False)


def test_permeation_loss_rays_through_many_colliders(ctx):
    """Loss rays (AudioPermeationJobBatched.cs:61-85, :225-328) that cross far more colliders than
    the BVH loss pass keeps per ray (kLossCap = 48): rows of overlapping spheres (radius 0.6 at
    spacing 1) 128 long, boxes and OBBs among them, targets far out along the rows, owned
    colliders skipped; the sum over every collider in reference order must equal the oracle's, for
    the rays that fit and for the ones summed by the whole-wave overflow path."""
    rng = np.random.default_rng(23)
    xs = np.arange(-64, 64, dtype=np.float32)
    yz = np.array([-1.0, 0.0, 1.0], np.float32)
    c = np.array([(x, y, z) for x in xs for y in yz for z in yz], np.float32)
    T = 6
    tid = rng.integers(-1, T, len(c)).astype(np.int16)
    sph = spheres(c, np.full(len(c), 0.6, np.float32), rng, tid=tid)
    box = aabbs(c[::7] + np.float32(0.5), np.full((len(c[::7]), 3), 0.3, np.float32), rng)
    ob = obbs(c[3::11] + np.float32(0.25), np.full((len(c[3::11]), 3), 0.35, np.float32), rng)
    targets = np.array([[-1000, 0, 0], [1000, 0.2, 0.1], [-500, 3, 2], [300, -0.5, 0.4], [0, 0, 900], [-2000, 0.9, -0.9]],
                       np.float32)
    scene = art.Scene(dirs=fib_dirs(64), targets=targets, spheres=sph, aabbs=box, obbs=ob)
    org = np.array([[0.5, 0.0, 0.0], [-20.3, 0.4, -0.2], [40.0, 0.0, 0.7], [0.0, 5.0, 0.0]], np.float32)
    out = run(ctx, scene, org)
    assert (out.perm != 0).any()


def test_permeation_first_hit_far_from_batch_end():
    """The permeation slot value comes from the highest-index ray of the batch whose first hit exists
    (AudioPermeationJobBatched.cs:58, App. B Q7). One small box straight along ray 5 of 96: the BVH
    permeation pass casts the batch's rays from its end 16 at a time, so several rounds find no hit
    before the one holding ray 5's neighbours; TC = 1 and TC = 3 (three batch slots)."""
    rng = np.random.default_rng(31)
    dirs = fib_dirs(96)
    d5 = dirs[5].view(np.float16).astype(np.float32)
    d5 /= np.linalg.norm(d5)
    box = aabbs((d5 * 20.0)[None, :], np.full((1, 3), 1.5, np.float32), rng)
    scene = art.Scene(dirs=dirs, targets=np.array([[5, 5, 5], [-30, 2, 1]], np.float32), aabbs=box)
    org = np.zeros((3, 3), np.float32)
    org[1] = [0.1, -0.2, 0.05]
    for tc in (1, 3):
        params = art.FrameParams(max_hits_per_ray=1, max_ray_life=1e4, max_muffle_hit_distance=1e5,
                                 stages=abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_PERMEATE | abi.ART_STAGE_REDUCE)
        params.thread_count = tc
        with art.Context(1) as c:
            out, _ = gpu_vs_oracle(c, scene, params, org, hits=True, counts=False, stale=4)
        assert (out.perm != 0).any()


def _obb_world_points(ob, rng, m):
    """m world points on the surfaces of random OBBs of `ob` (corners, edge points, face points), as
    the tests map them: local = R (P - c) by the stored rotation R (halfQuaternion decode), so
    P = c + R^T local."""
    h2f = lambda a: np.asarray(a, np.uint16).view(np.float16).astype(np.float64)
    out = []
    for _ in range(m):
        k = rng.integers(len(ob))
        c = h2f(ob["center"][k]); h = np.abs(h2f(ob["size"][k]))
        x, y, z = h2f(ob["rot"][k])
        w2 = 1.0 - (x * x + y * y + z * z)
        q = np.array([x, y, z, np.sqrt(w2) if w2 > 0 else 0.0])
        q /= np.linalg.norm(q)
        x, y, z, w = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        kind = rng.integers(3)  # corner, edge point, face point
        s = rng.choice([-1.0, 1.0], 3)
        loc = s * h
        if kind >= 1:
            loc[0] = rng.uniform(-1, 1) * h[0]
        if kind == 2:
            loc[1] = rng.uniform(-1, 1) * h[1]
        out.append(c + R.T @ loc)
    return np.array(out)


def test_obb_rotated_bounds_grazing(ctx):
    """Rays aimed at the corners, edges and faces of rotated OBBs (round 4's OBB bounds are the
    world box of the rotated box, tight exactly there), flat and long boxes included, through the
    raytrace, echo, muffle and permeation casts (the permeation first hit rotates by the inverse)."""
    rng = np.random.default_rng(41)
    n = 400
    c = rng.uniform(-25, 25, (n, 3)).astype(np.float32)
    halves = rng.uniform(0.1, 3.0, (n, 3)).astype(np.float32)
    halves[::5, 0] *= 12.0   # long boxes
    halves[1::5, 1] = 0.02   # flat boxes
    ob = obbs(c, halves, rng)
    ob["rot"][::7] = f16bits(np.array([0.0, 0.0, 0.0]))          # identity
    ob["rot"][3::7] = f16bits(np.array([0.7071, 0.0, 0.0]))       # 90 degrees about x
    O = np.array([0.5, -0.25, 0.125], np.float32)
    P = _obb_world_points(ob, rng, 256)
    d = P - O.astype(np.float64)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    dirs = f16bits(d).reshape(-1, 3)
    org = np.concatenate([O[None], rng.uniform(-20, 20, (3, 3))]).astype(np.float32)
    targets = rng.uniform(-25, 25, (4, 3)).astype(np.float32)
    scene = art.Scene(dirs=dirs, targets=targets, obbs=ob,
                      spheres=spheres(c[:40] + 1.5, np.full(40, 0.4, np.float32), rng))
    run(ctx, scene, org, H=3)


@pytest.mark.parametrize("cfg_index,C_scale", [(2, 1.0), (4, 0.25), (4, 1.0), (3, 0.01)])
def test_kd_wave_pass_builds_the_same_tree(monkeypatch, cfg_index, C_scale):
    """The wave-level kd pass (segments of <= 64 positions, art_bvh.hip kd_wave_kernel) makes the
    same split decisions as the block passes it replaces (ART_KD_WAVE=0): the same leaf order
    (art_debug_leaf_order) and the same outputs, at the full config-2
    scene (4096 colliders: surface-area splits down to 64-position segments), 4096- and
    16384-collider config-4 scenes, and a scene below 64 colliders (the wave pass alone)."""
    cfg = art.CONFIGS[cfg_index]
    scene, org, params = art.synth(cfg, S=8, R=128, C_scale=C_scale)
    n = scene.spheres.size + scene.aabbs.size + scene.obbs.size
    orders, outs = {}, {}
    for wave, seg in (("0", "0"), ("1", "0")):
        monkeypatch.setenv("ART_KD_WAVE", wave)
        out = art.FanOutputs(8, scene.R, params.max_hits_per_ray, scene.T, params.thread_count, hits=True,
                             dsp=params.dsp is not None)
        with art.Context(1) as c:
            fr = art.Frame(scene, params, org, out)
            c.bind(fr)
            orders[wave + seg] = c.debug_leaf_order()
            c.run(fr)
        outs[wave + seg] = out
    assert orders["10"].size == n
    for key in ("00",):
        assert np.array_equal(orders[key], orders["10"]), (key, int((orders[key] != orders["10"]).sum()))
        assert all(outs[key].equal(outs["10"]).values()), key


@pytest.mark.parametrize("H,hits", [(1, False), (2, True)])
def test_cell_lists_long_and_mid(ctx, monkeypatch, capfd, H, hits):
    """Muffle direction-cell lists longer than the cells sort's register paths (art_cells.hip
    cells_sort_kernel: <= 64 entries one per lane, <= 256 several per lane, longer ones from memory):
    a cluster of 700 small spheres and one of 160 small boxes, each seen from the targets through a
    few cells, so those cells list hundreds of colliders; the muffle rays crossing them must still
    equal the brute-force oracle (CanRaySeeAudioTarget :405-449), through the bench's plan (H = 1, no
    hit outputs: echo_muffle_kernel) and the multi-hit plan with hit outputs."""
    monkeypatch.setenv("ART_DEBUG_CELLS", "1")
    rng = np.random.default_rng(2024)
    R = 256
    dirs = fib_dirs(R)
    sph = spheres(np.array([12.0, 0.0, 0.0]) + rng.uniform(-1.2, 1.2, (700, 3)), rng.uniform(0.05, 0.15, 700), rng)
    box = aabbs(np.array([0.0, 14.0, 0.0]) + rng.uniform(-1.0, 1.0, (160, 3)), rng.uniform(0.05, 0.2, (160, 3)), rng)
    walls = aabbs(np.array([[30.0, 0, 0], [-30.0, 0, 0], [0, 30.0, 0], [0, -30.0, 0], [0, 0, 30.0], [0, 0, -30.0]]),
                  np.array([[1.0, 40, 40], [1.0, 40, 40], [40, 1.0, 40], [40, 1.0, 40], [40, 40, 1.0], [40, 40, 1.0]]), rng)
    targets = np.array([[-2.0, 0.5, 0.3], [0.5, -3.0, 0.2], [1.0, 1.0, -2.0]], np.float32)
    org = np.array([[20.0, 2.0, 1.0], [3.0, 22.0, -1.0], [18.0, 10.0, 5.0], [-10.0, -10.0, 8.0]], np.float32)
    scene = art.Scene(dirs=dirs, targets=targets, spheres=sph, aabbs=np.concatenate([box, walls]))
    params = art.FrameParams(max_hits_per_ray=H, max_ray_life=1e4, max_muffle_hit_distance=1e5,
                             stages=abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_REDUCE)
    out, _ = gpu_vs_oracle(ctx, scene, params, org, hits=hits, counts=False)
    assert (out.muffle != 0).any()
    err = capfd.readouterr().err
    longest = max(int(l.split("longest ")[1].split(";")[0]) for l in err.splitlines() if "[cells]" in l)
    assert longest > 256, err[-2000:]
