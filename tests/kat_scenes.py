"""Hand-built scenes for the known-answer tests.

Each builder returns (scene, params, origins, expect) where `expect(out)` asserts the
hand-derived answer on a FanOutputs. The same scenes feed the oracle (CPU tests) and the HIP
path (GPU parity tests).
"""
import numpy as np

import art
from art import abi
import unity32 as U

def h(x: float) -> int:
    """Unity f32tof16 via the product's host helper (inputs only)."""
    from art.synth import f32tof16
    return f32tof16(float(np.float32(x)))


def hv(v):
    return [h(x) for x in v]


def half3_dirs(vs):
    return np.array([hv(v) for v in vs], dtype=np.uint16).reshape(-1, 3)


def aabb(center, half, absorption=0.0, density=1.0, echo=1.0, tid=-1):
    a = np.zeros(1, abi.AABB)
    a["center"] = hv(center); a["size"] = hv(half)
    a["material"] = hv((absorption, density, echo)); a["audio_target_id"] = tid
    return a


def sphere(center, radius, absorption=0.0, density=1.0, echo=1.0, tid=-1):
    s = np.zeros(1, abi.SPHERE)
    s["center"] = hv(center); s["radius"] = h(radius)
    s["material"] = hv((absorption, density, echo)); s["audio_target_id"] = tid
    return s


def obb(center, half, inv_q_xyz, absorption=0.0, density=1.0, echo=1.0, tid=-1):
    b = np.zeros(1, abi.OBB)
    b["center"] = hv(center); b["size"] = hv(half); b["rot"] = hv(inv_q_xyz)
    b["material"] = hv((absorption, density, echo)); b["audio_target_id"] = tid
    return b


def cat(dtype, *parts):
    parts = [p for p in parts if p is not None]
    return np.concatenate(parts).astype(dtype) if parts else np.zeros(0, dtype)


def params(H=1, stages=abi.ART_STAGE_RAYTRACE | abi.ART_STAGE_PERMEATE | abi.ART_STAGE_REDUCE, **kw):
    return art.FrameParams(max_hits_per_ray=H, stages=stages, **kw)


def f16(x):
    from art.synth import f16tof32
    return f16tof32(int(x))


# K6 — single wall: echo = f32tof16(dist * echo) for echo in {1, 3}
def k6_single_wall(echo_mult):
    # origin (0,0,0); ray +x; wall AABB x in [5, 7]; target far behind the origin (no occlusion)
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0)]), targets=np.array([[-3, 0, 0]], np.float32),
                   aabbs=cat(abi.AABB, aabb((6, 0, 0), (1, 4, 4), echo=echo_mult)))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        # hit at x = 5 exactly; echo ray back to the origin is clear; dist = 5
        assert out.echo[0, 0] == h(5.0 * echo_mult)
        assert out.muffle[0, 0] == 1  # the muffle ray back to the target is clear
    return sc, p, org, expect


# K7 — a collider owned by target t is skipped for t's muffle ray and blocks other rays
def k7_owner_skip():
    # origin (0,0,0), ray +x hits the wall x in [5, 7] at P = (5,0,0). Target 0 sits at (2,3,0)
    # inside its own sphere (r = 0.5); target 1 at (-1,6,0) is seen from P through that sphere.
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0)]), targets=np.array([[2, 3, 0], [-1, 6, 0]], np.float32),
                   spheres=cat(abi.SPHERE, sphere((2, 3, 0), 0.5, tid=0)),
                   aabbs=cat(abi.AABB, aabb((6, 0, 0), (1, 4, 4))))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        assert out.echo[0, 0] == h(5.0)     # echo ray back along the x axis is clear
        assert out.muffle[0, 0] == 1        # target 0: its own sphere is skipped
        assert out.muffle[0, 1] == 0        # target 1: blocked by target 0's sphere
    return sc, p, org, expect


# K8 — permeation: remains = R * Strength - loss, the LAST hitting ray's value wins (Q7)
def k8_slab():
    # ray 0 (+x) first-hits wall A (x in [5,6]); ray 1 (-x) first-hits wall B (x in [-6,-5]).
    # Target at (0,20,0). Ray 1's loss ray from (-5,0,0) crosses slab D (y in [7,9], density 1)
    # over a path of 2 / (20 / sqrt(425)) = sqrt(425) / 10; ray 0's loss ray crosses nothing.
    # Ray 1 is the last hitting ray, so remains = 2 - sqrt(425) / 10 (ray 0 alone would give 2).
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0), (-1, 0, 0)]), targets=np.array([[0, 20, 0]], np.float32),
                   aabbs=cat(abi.AABB, aabb((5.5, 0, 0), (0.5, 3, 3)), aabb((-5.5, 0, 0), (0.5, 3, 3)),
                             aabb((-3, 8, 0), (1, 1, 3), density=1.0)))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        # ray 1's value, evaluated step by step in float32 (unity32), compared bit for bit
        want = perm_value(sc, org[0], 1, 0)
        assert abs(float(want) - (2.0 - np.sqrt(425.0) / 10.0)) < 1e-3  # the closed form, for orientation
        assert out.perm[0, 0].view(np.uint32) == np.float32(want).view(np.uint32)
        assert perm_value(sc, org[0], 0, 0) == np.float32(2.0)  # ray 0 alone would leave 2

    return sc, p, org, expect


# K10 — absorption kill (life < 0 after the drain) and life == 0 before reflection
def k10_absorption(max_life):
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0)]), targets=np.array([[-3, 0, 0]], np.float32),
                   aabbs=cat(abi.AABB, aabb((6, 0, 0), (1, 4, 4), absorption=1.0),
                             aabb((-6, 0, 0), (1, 4, 4))))
    p = params(H=5, max_ray_life=max_life)
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        # first hit at distance 5; either life = max_life - 5 - max_life*1 < 0 (drained) or,
        # with max_life = 5, life == 0 before the reflection: the ray ends after one hit
        assert out.hit_counts[0, 0] == 1
    return sc, p, org, expect


# K11 — ties: sphere vs AABB at equal distance -> sphere wins; two AABBs -> lower index wins
def k11_ties():
    # ray 0 (+x): sphere centred (7,0,0) r=2 (front face x=5) and AABB x in [5, 9] -> tie at 5.
    # ray 1 (-x): two identical AABBs x in [-9, -5], different echo multipliers -> index 1 (first of
    # the pair in array order) wins.
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0), (-1, 0, 0)]), targets=np.array([[0, 0, 30]], np.float32),
                   spheres=cat(abi.SPHERE, sphere((7, 0, 0), 2.0, echo=1.0)),
                   aabbs=cat(abi.AABB, aabb((7, 0, 0), (2, 1, 1), echo=3.0), aabb((-7, 0, 0), (2, 1, 1), echo=2.0),
                             aabb((-7, 0, 0), (2, 1, 1), echo=3.0)))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        assert out.echo[0, 0] == h(5.0 * 1.0)   # the sphere (echo 1) won the tie
        assert out.echo[0, 1] == h(5.0 * 2.0)   # the lower-index AABB (echo 2) won
        assert out.hit_ids[0].tolist() == [abi.hit_id(abi.ART_COLLIDER_SPHERE, 0), abi.hit_id(abi.ART_COLLIDER_AABB, 1)]
    return sc, p, org, expect


# K12 — miss after k hits -> hit_counts = k
def k12_miss_after_hits():
    # ray +x hits a wall facing -x at x = 5, reflects to -x and escapes (nothing behind the origin)
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0)]), targets=np.array([[0, 0, 30]], np.float32),
                   aabbs=cat(abi.AABB, aabb((6, 0, 0), (1, 4, 4))))
    p = params(H=5)
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        assert out.hit_counts[0, 0] == 1
        assert out.echo[0, 1:].tolist() == [0, 0, 0, 0]
        assert out.hit_points[0, 0].tolist() == hv((5, 0, 0))
    return sc, p, org, expect


# K9 — ProcessAudioDataJob alone on hand-made arrays (stages = REDUCE)
def k9_reduce():
    R, H, T = 4, 2, 2
    dirs = half3_dirs([(1, 0, 0)] * R)
    sc = art.Scene(dirs=dirs, targets=np.array([[1, 2, 3], [4, 5, 6]], np.float32))
    p = params(H=H, stages=abi.ART_STAGE_REDUCE)
    org = np.zeros((1, 3), np.float32)
    echo = [0, h(7.0), 0x8000, h(3.5), 0, h(14.0), h(3.5), 0]   # -0 (0x8000) also counts as returned

    def prime(out):
        out.echo[0] = echo
        out.muffle[0] = [3, 5]
        out.perm[0] = [2.0, -1.0]

    def expect(out):
        total = np.float32(0)
        for e in echo:
            v = np.float32(f16(e))
            if v != 0:
                total = np.float32(total + v)
        n = np.float32(R * H)
        returned = np.float32(4)
        rs = np.float32(np.float32(total / n) / np.float32(35.0))
        rv = np.float32(returned / n)
        s = out.settings[0]
        assert s["reverb_strength"][0] == min(max(rs, 0), 1) and s["reverb_volume"][0] == rv
        m0 = np.float32(1) - np.float32(np.float32(3) / n) * np.float32(1)
        p0 = np.float32(np.float32(np.float32(2.0) / np.float32(R)) / np.float32(1)) * np.float32(0.5)
        assert s["muffle_strength"][0] == np.clip(np.float32(m0 - p0), 0, 1)
        assert tuple(s["perceived_position"][1]) == (4, 5, 6)
    return sc, p, org, expect, prime


# Q13 — MuffleRayHits is a ushort: the per-(hit, target) increment (:171) wraps above 65535
def q13_ushort_wrap():
    # 70000 Fibonacci rays from the centre of a radius-10 sphere owned by target 0: every ray hits
    # the sphere from inside (t1, :337-351), every muffle ray to the target at (1,0,0) skips its own
    # sphere (:413) and is clear, so the count is 70000 = 65536 + 4464.
    from art.synth import fibonacci_directions
    R = 70000
    sc = art.Scene(dirs=fibonacci_directions(R), targets=np.array([[1, 0, 0]], np.float32),
                   spheres=cat(abi.SPHERE, sphere((0, 0, 0), 10.0, tid=0)))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        assert out.muffle[0, 0] == 70000 - 65536
        assert out.echo[0, 0] == h(10.0)  # the echo ray starts inside the sphere: exit at ~20 > 10
    return sc, p, org, expect


# Q19 — degenerate Fibonacci rays i = 0 (+0, 1, +0) and i = R-1 (+-0, -1, +-0) through a frame
def q19_degenerate_dirs():
    # ray 0 runs in the face plane x = 0 of the box [0,2]x[4,6]x[-1,1]: (min.x - o.x) * inf is NaN,
    # Unity's min/max (App. A.2) then give tmin.x = tmax.x = inf, tNear = inf > tFar: a miss (Q19).
    # ray R-1 hits the box [-1,1]x[-6,-4]x[-1,1] at distance 4: x/z slabs (+-1) * (+-inf) = -+inf.
    from art.synth import fibonacci_directions
    R = 64
    sc = art.Scene(dirs=fibonacci_directions(R), targets=np.array([[0, 0, 3]], np.float32),
                   aabbs=cat(abi.AABB, aabb((1, 5, 0), (1, 1, 1)), aabb((0, -5, 0), (1, 1, 1))))
    assert tuple(sc.dirs[0]) == (0, h(1.0), 0) and sc.dirs[R - 1][1] == h(-1.0)
    assert sc.dirs[R - 1][0] & 0x7FFF == 0 and sc.dirs[R - 1][2] & 0x7FFF == 0
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        assert out.hit_counts[0, 0] == 0 and out.echo[0, 0] == 0
        assert out.hit_counts[0, R - 1] == 1
        assert out.echo[0, R - 1] == h(4.0)
        assert out.hit_points[0, R - 1][1] == h(-4.0)
    return sc, p, org, expect


KATS = {
    "q13_ushort_wrap": q13_ushort_wrap,
    "q19_degenerate_dirs": q19_degenerate_dirs,
    "k6_echo1": lambda: k6_single_wall(1.0),
    "k6_echo3": lambda: k6_single_wall(3.0),
    "k7_owner_skip": k7_owner_skip,
    "k8_slab": k8_slab,
    "k10_drained": lambda: k10_absorption(125.0),
    "k10_life_zero": lambda: k10_absorption(5.0),
    "k11_ties": k11_ties,
    "k12_miss": k12_miss_after_hits,
}


# ---------------------------------------------------------------- float32 step-by-step answers
def decoded(scene):
    """The scene's colliders decoded from their half bits: (spheres, aabbs, obbs) as lists of
    (center, size or radius, [q,] density, echo, absorption, tid), float32 (unity32)."""
    sph = [(U.hv3(*s["center"]), U.h2f(s["radius"]), U.h2f(s["material"][1]), s["audio_target_id"]) for s in scene.spheres]
    aab = [(U.hv3(*a["center"]), U.hv3(*a["size"]), U.h2f(a["material"][1]), a["audio_target_id"]) for a in scene.aabbs]
    obs = [(U.hv3(*b["center"]), U.hv3(*b["size"]), U.half_quaternion(*[int(x) for x in b["rot"]]), U.h2f(b["material"][1]),
            b["audio_target_id"]) for b in scene.obbs]
    return sph, aab, obs


def nearest(scene, o, d, perm=False):
    """ShootRayCast (AudioRaytracerJobBatched.cs:225-280; perm: AudioPermeationJobBatched.cs:101-141
    with the inverted stored rotation :174): (type, index, distance) of the first minimum in Sphere,
    AABB, OBB order, or None."""
    sph, aab, obs = decoded(scene)
    best, hit = (np.float32(np.inf) if perm else np.float32(3.40282347e+38)), None
    for i, (c, r, _, _) in enumerate(sph):
        t = U.ray_sphere(o, d, c, r)
        if t is not None and t < best:
            best, hit = t, (abi.ART_COLLIDER_SPHERE, i)
    for i, (c, hh, _, _) in enumerate(aab):
        t = U.ray_aabb(o, d, c, hh)
        if t is not None and t < best:
            best, hit = t, (abi.ART_COLLIDER_AABB, i)
    for i, (c, hh, q, _, _) in enumerate(obs):
        t = U.ray_obb(o, d, c, hh, U.qinverse(q) if perm else q)
        if t is not None and t < best:
            best, hit = t, (abi.ART_COLLIDER_OBB, i)
    return None if hit is None else (hit[0], hit[1], best)


def perm_loss(scene, o, d, t):
    """ShootPermeationRayCast's loss (:225-261): every non-owned collider, Sphere, AABB, OBB order."""
    sph, aab, obs = decoded(scene)
    total = np.float32(0)
    for c, r, dens, tid in sph:
        if tid != t:
            total = np.float32(total + U.perm_sphere(o, d, c, r, dens))
    for c, hh, dens, tid in aab:
        if tid != t:
            total = np.float32(total + U.perm_aabb(o, d, c, hh, dens))
    for c, hh, q, dens, tid in obs:
        if tid != t:
            total = np.float32(total + U.perm_aabb(U.qmul(q, U.sub(o, c)), U.qmul(q, d), U.v3(0, 0, 0), hh, dens))
    return total


def perm_value(scene, origin, ray, t, strength=1.0):
    """PermeationPowerRemains of `ray` for target t (:58-85, :260), or None when its first hit misses."""
    o = U.v3(*origin)
    d = U.hv3(*[int(x) for x in scene.dirs[ray]])
    hit = nearest(scene, o, d, perm=True)
    if hit is None:
        return None
    p = U.add(o, U.muls(d, hit[2]))
    off = U.sub(p, U.muls(d, U.EPS))
    dt = U.normalize(U.sub(U.v3(*scene.targets[t]), off))
    return np.float32(np.float32(np.float32(scene.R) * np.float32(strength)) - perm_loss(scene, off, dt, t))


def path(scene, origin, ray, H, max_life=125.0, reflect=None, offset=None):
    """The hit sequence of one ray (Execute :104-208) with the reference's ReflectRay: a list of
    (type, index, hit point). `reflect` / `offset` swap in a contrast convention."""
    sph, aab, obs = decoded(scene)
    o = U.v3(*origin)
    d = U.hv3(*[int(x) for x in scene.dirs[ray]])
    life = np.float32(max_life)
    out = []
    while True:
        hit = nearest(scene, o, d)
        if hit is None:
            break
        ty, idx, t = hit
        o = U.add(o, U.muls(d, t))
        life = np.float32(life - t)
        out.append((ty, idx, o))
        if len(out) >= H or life <= 0:
            break
        if reflect is not None:
            n = reflect(ty, idx, o)
        elif ty == abi.ART_COLLIDER_AABB:
            n = U.aabb_face_normal(o, aab[idx][0], aab[idx][1])
        elif ty == abi.ART_COLLIDER_OBB:
            n = U.obb_face_normal(o, obs[idx][0], obs[idx][1], obs[idx][2])
        else:
            n = U.normalize(U.sub(o, sph[idx][0]))
        dn = U.reflect(d, n)
        o = offset(o, d, dn) if offset is not None else U.add(o, U.muls(dn, U.EPS))  # :528 along the new dir
        d = dn
        absorption = {abi.ART_COLLIDER_SPHERE: scene.spheres, abi.ART_COLLIDER_AABB: scene.aabbs,
                      abi.ART_COLLIDER_OBB: scene.obbs}[ty][idx]["material"][0]
        life = np.float32(life - np.float32(np.float32(max_life) * U.h2f(absorption)))
        if life < 0:
            break
    return out


def concrete(**kw):
    return dict(absorption=0.25, density=1.0, echo=1.0, **kw)


# Q1 — the echo reset mis-index at TC > 1 (AudioRaytracerJobBatched.cs:72-80): each batch zeroes
# Echo[start + i] for i < count * H instead of start * H + i.
def q1_echo_reset_misindex():
    # R = 2, TC = 2 -> batch_size 1; H = 2. Batch 0 (ray 0) resets slots 0, 1; batch 1 (ray 1)
    # resets slots 1, 2 — after ray 0 wrote its second echo into slot 1 — and slot 3 (ray 1's
    # second slot) is never reset. Ray 0 bounces between walls at x = +-5 (two visible echoes);
    # ray 1 (+y) misses everything.
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0), (0, 1, 0)]), targets=np.array([[0, 0, 30]], np.float32),
                   aabbs=cat(abi.AABB, aabb((6, 0, 0), (1, 4, 4)), aabb((-6, 0, 0), (1, 4, 4))))
    p = params(H=2, thread_count=2)
    org = np.zeros((1, 3), np.float32)
    stale_echo, stale_pt, stale_id = 0x1234, [0x1111, 0x2222, 0x3333], 0x0BADF00D

    def prime(out):
        out.echo[0] = [0x4444, 0x4444, 0x4444, stale_echo]
        if out.hit_points is not None:
            out.hit_points[0] = [[0x5555] * 3] * 3 + [stale_pt]
            out.hit_counts[0] = [77, 77]
            out.hit_ids[0] = [7, 7, 7, stale_id]

    def expect(out):
        hits = path(sc, org[0], 0, 2)
        assert len(hits) == 2 and path(sc, org[0], 1, 2) == []
        O = U.v3(0, 0, 0)
        echo2 = U.f2h(np.float32(U.distance(O, hits[1][2]) * np.float32(1)))
        assert echo2 != 0  # ray 0's second echo was written ...
        assert out.echo[0].tolist() == [U.f2h(U.distance(O, hits[0][2])), 0, 0, stale_echo]  # ... then wiped (Q1)
        assert out.hit_counts[0].tolist() == [2, 0]
        assert out.hit_points[0].tolist() == [U.h3(hits[0][2]), [0, 0, 0], [0, 0, 0], stale_pt]  # Q17, same loop
        assert out.hit_ids[0].tolist() == [abi.hit_id(abi.ART_COLLIDER_AABB, 0), abi.ART_HIT_NONE, abi.ART_HIT_NONE,
                                           stale_id]
    return sc, p, org, expect, prime


# Q3 — the echo distance is measured from the UN-offset hit point (:130), the echo ray starts at
# the offset point (:124-127).
def q3_echo_unoffset_distance():
    # a wall ~0.05 in front of the origin: halves there are 3e-5 apart, so the 1e-4 offset would
    # change the stored echo
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0)]), targets=np.array([[0, 0, 30]], np.float32),
                   aabbs=cat(abi.AABB, aabb((0.55, 0, 0), (0.5, 0.5, 0.5), echo=3.0)))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        (ty, idx, hp), = path(sc, org[0], 0, 1)
        O = U.v3(0, 0, 0)
        em = U.h2f(sc.aabbs[0]["material"][2])
        want = U.f2h(np.float32(U.distance(O, hp) * em))
        off = U.sub(hp, U.muls(U.hv3(*[int(x) for x in sc.dirs[0]]), U.EPS))
        assert want != U.f2h(np.float32(U.distance(O, off) * em))  # the offset point would differ
        assert out.echo[0, 0] == want
        assert out.hit_ids[0, 0] == abi.hit_id(ty, idx)
    return sc, p, org, expect


# Q5 — OBB rotation conventions (App. B): ReflectRay goes to the local frame with inverse(stored)
# (:489) and back with stored (:510), i.e. the wrong rotation both ways.
def q5_obb_reflection():
    # cube (half 2) at (10, 0, 0) rotated 30 deg about y, stored as the inverse rotation
    # (AudioOBBCollider.cs:59); ray +x reflects off it to a surrounding sphere (r = 40). The
    # geometric normal would send the ray to z > 0, the reference's to z < 0.
    import math
    th = math.radians(30)
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0)]), targets=np.array([[0, 0, 30]], np.float32),
                   spheres=cat(abi.SPHERE, sphere((0, 0, 0), 40.0)),
                   obbs=cat(abi.OBB, obb((10, 0, 0), (2, 2, 2), (0.0, -math.sin(th / 2), 0.0))))
    p = params(H=2)
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        hits = path(sc, org[0], 0, 2)
        assert [(t, i) for t, i, _ in hits] == [(abi.ART_COLLIDER_OBB, 0), (abi.ART_COLLIDER_SPHERE, 0)]
        _, aab, obs = decoded(sc)
        geo = path(sc, org[0], 0, 2, reflect=lambda ty, i, o: U.obb_face_normal(o, obs[i][0], obs[i][1], obs[i][2], buggy=False))
        assert U.h3(geo[1][2]) != U.h3(hits[1][2]) and hits[1][2][2] < 0 < geo[1][2][2]
        assert out.hit_points[0].tolist() == [U.h3(hp) for _, _, hp in hits]
        assert out.hit_ids[0].tolist() == [abi.hit_id(t, i) for t, i, _ in hits]
    return sc, p, org, expect


def q5_permeation_first_hit():
    # AudioPermeationJobBatched.ShootRayCast intersects OBBs with inverse(stored) (:174): the
    # permeation job sees the mirror image of a rotated box. A long thin box (half (4, .25, .25))
    # rotated 45 deg about y: ray 0 (+x) hits both images, ray 1 only the raytracer's (real) box,
    # ray 2 only the permeation job's. The last ray whose PERMEATION first hit exists (ray 2) sets
    # PermeationPowerRemains (Q7); with the geometric rotation it would be ray 1.
    import math
    th = math.radians(45)
    d1, d2 = U.normalize(U.v3(10, 0, 3)), U.normalize(U.v3(10, 0, -3))
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0), d1, d2]), targets=np.array([[10, 0, 0]], np.float32),
                   obbs=cat(abi.OBB, obb((10, 0, 0), (4, 0.25, 0.25), (0.0, -math.sin(th / 2), 0.0), density=5.0)))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        assert out.hit_counts[0].tolist() == [1, 1, 0]
        assert out.hit_ids[0].tolist() == [abi.hit_id(abi.ART_COLLIDER_OBB, 0)] * 2 + [abi.ART_HIT_NONE]
        assert [perm_value(sc, org[0], r, 0) is None for r in range(3)] == [False, True, False]
        want = perm_value(sc, org[0], 2, 0)
        assert want != np.float32(3.0)  # the loss ray crosses the real box
        assert out.perm[0, 0].view(np.uint32) == np.float32(want).view(np.uint32)
    return sc, p, org, expect


# Q10 — two sphere formulas: the raytracer's general quadratic with a = dot(d, d) (:326-339), the
# permeation loss's unit-direction form b = dot(oc, d), disc = b^2 - c (AudioPermeationJobBatched.cs:307-319).
def q10_sphere_formulas():
    # ray 0 = (0, 0, 0.5), not unit: the general quadratic hits the sphere (0, 0, 10) r 2 at
    # t = 16, the point (0, 0, 8) (the unit form would miss: b^2 - c < 0). Ray 1 (+x) hits a wall
    # at x = 5; its loss ray to the target crosses the sphere (-2, 3, 1) r 1.5, where the unit form
    # and the general one round differently: the stored remains carry the unit form's bits.
    sc = art.Scene(dirs=np.array([hv((0, 0, 0.5)), hv((1, 0, 0))], np.uint16),
                   targets=np.array([[-10.2, 5.7, 4.1]], np.float32),
                   spheres=cat(abi.SPHERE, sphere((0, 0, 10), 2.0), sphere((-2, 3, 1), 1.5)),
                   aabbs=cat(abi.AABB, aabb((6, 0, 0), (1, 4, 4))))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        (t0, i0, p0), = path(sc, org[0], 0, 1)
        assert (t0, i0) == (abi.ART_COLLIDER_SPHERE, 0) and U.h3(p0) == hv((0, 0, 8))
        assert out.hit_points[0, 0].tolist() == hv((0, 0, 8)) and out.echo[0, 0] == h(8.0)
        want = perm_value(sc, org[0], 1, 0)
        # the contrast: the general quadratic on the same loss ray stores different bits
        d = U.hv3(*[int(x) for x in sc.dirs[1]])
        off = U.sub(U.add(U.v3(0, 0, 0), U.muls(d, nearest(sc, U.v3(0, 0, 0), d, perm=True)[2])), U.muls(d, U.EPS))
        dt = U.normalize(U.sub(U.v3(*sc.targets[0]), off))
        c1, r1, dens = U.hv3(*sc.spheres[1]["center"]), U.h2f(sc.spheres[1]["radius"]), U.h2f(sc.spheres[1]["material"][1])
        unit, gen = U.perm_sphere(off, dt, c1, r1, dens), U.perm_sphere_general(off, dt, c1, r1, dens)
        assert unit > 0 and unit != gen
        assert out.perm[0, 0].view(np.uint32) == np.float32(want).view(np.uint32)
    return sc, p, org, expect


# Q14 — after a reflection the origin moves 1e-4 along the NEW direction (:528); echo and muffle
# offsets go along the old -dir (:124, :158).
def q14_reflection_offset():
    # walls ~0.03 either side of the origin (halves ~6e-5 apart near 0.09): the ray (1, 1, 0)
    # zig-zags between them; an offset along the old direction would move the second hit point
    sc = art.Scene(dirs=half3_dirs([(1, 1, 0)]), targets=np.array([[0, 0, 30]], np.float32),
                   aabbs=cat(abi.AABB, aabb((0.05, 0, 0), (0.02, 1, 1)), aabb((-0.05, 0, 0), (0.02, 1, 1))))
    p = params(H=3)
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        hits = path(sc, org[0], 0, 3)
        old = path(sc, org[0], 0, 3, offset=lambda o, d, dn: U.sub(o, U.muls(d, U.EPS)))
        assert [(t, i) for t, i, _ in hits] == [(abi.ART_COLLIDER_AABB, k) for k in (0, 1, 0)]
        assert U.h3(old[1][2]) != U.h3(hits[1][2])
        assert out.hit_points[0].tolist() == [U.h3(hp) for _, _, hp in hits]
        assert out.hit_ids[0].tolist() == [abi.hit_id(t, i) for t, i, _ in hits]
        assert out.hit_counts[0, 0] == 3
    return sc, p, org, expect


# Q15 — face pick with strict '<' between the face deltas; ties go to z, and sign(0) = 0 gives a
# zero normal, so reflect() leaves the direction unchanged (:471-482, :497-508).
def q15_face_ties(kind):
    # the box [4, 6] x [-1, 1] x [-2, 2] is hit exactly on its edge x = 4, y = 1 (x and y deltas
    # both 0): ray 0 (4, 1, 0) at z = 0 gets the zero normal and passes on unchanged to the far wall;
    # ray 1 (4, 1, 0.5) at z = 0.5 gets the z normal although the z face is 1.5 away.
    box = dict(center=(5, 0, 0), half=(1, 1, 2))
    aabbs = [aabb((21, 0, 0), (1, 40, 40))]
    obbs = []
    if kind == "aabb":
        aabbs = [aabb(box["center"], box["half"])] + aabbs
    else:
        obbs = [obb(box["center"], box["half"], (0.0, 0.0, 0.0))]
    sc = art.Scene(dirs=half3_dirs([(4, 1, 0), (4, 1, 0.5)]), targets=np.array([[0, 0, 30]], np.float32),
                   aabbs=cat(abi.AABB, *aabbs), obbs=cat(abi.OBB, *obbs) if obbs else np.zeros(0, abi.OBB))
    p = params(H=2)
    org = np.zeros((1, 3), np.float32)
    box_id = abi.hit_id(abi.ART_COLLIDER_AABB, 0) if kind == "aabb" else abi.hit_id(abi.ART_COLLIDER_OBB, 0)
    wall_id = abi.hit_id(abi.ART_COLLIDER_AABB, 1 if kind == "aabb" else 0)

    def expect(out):
        _, aab, obs = decoded(sc)
        for r, want_n in ((0, (0, 0, 0)), (1, (0, 0, 1))):
            hits = path(sc, org[0], r, 2)
            assert U.h3(hits[0][2]) == hv((4, 1, 0.5 * r))
            bc, bh = (aab[0][0], aab[0][1]) if kind == "aabb" else (obs[0][0], obs[0][1])
            n = U.aabb_face_normal(hits[0][2], bc, bh) if kind == "aabb" else U.obb_face_normal(hits[0][2], bc, bh, obs[0][2])
            assert tuple(float(x) for x in n) == want_n  # x and y deltas tie at 0: z wins
            assert out.hit_ids[0, 2 * r:2 * r + 2].tolist() == [box_id, wall_id]
            assert out.hit_points[0, 2 * r:2 * r + 2].tolist() == [U.h3(hp) for _, _, hp in hits]
        # ray 0 passes straight on: the far hit is on the line of its direction (4, 1, 0)
        assert out.hit_points[0, 1].tolist() == hv((20, 5, 0))
        # ray 1 reflected by the z normal: its z shrinks again after the edge
        assert U.h2f(out.hit_points[0, 3][2]) < 0
    return sc, p, org, expect


# Q18 — muffle (and permeation) slots no batch maps to are never reset, yet ProcessAudioDataJob sums
# them (AudioRaytracerJobBatched.cs:82-85, ProcessAudioDataJob.cs:61-65).
def q18_stale_slots():
    # R = 2, TC = 3 -> batch_size 1, two batches: raytracer slots 0, 1 (batchId = start * TC / R)
    # and permeation slots 0, 1 (batchCount = 3 here); slot 2 keeps its stale 7 / -0.75 and the
    # settings include it.
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0), (-1, 0, 0)]), targets=np.array([[0, 0, 30]], np.float32),
                   aabbs=cat(abi.AABB, aabb((6, 0, 0), (1, 4, 4)), aabb((-6, 0, 0), (1, 4, 4))))
    p = params(thread_count=3, muffle_effectiveness=0.1, permeation_effectiveness=0.05)
    org = np.zeros((1, 3), np.float32)
    F = np.float32

    def prime(out):
        out.muffle[0] = [900, 900, 7]
        out.perm[0] = [5.5, 5.5, -0.75]

    def expect(out):
        assert out.muffle[0].tolist() == [1, 1, 7]
        pv = [perm_value(sc, org[0], r, 0) for r in (0, 1)]
        assert out.perm[0].view(np.uint32).tolist() == [F(v).view(np.uint32) for v in pv] + [F(-0.75).view(np.uint32)]
        O = U.v3(0, 0, 0)
        echo = [U.f2h(U.distance(O, path(sc, org[0], r, 1)[0][2])) for r in (0, 1)]
        assert out.echo[0].tolist() == echo
        # ProcessAudioDataJob.Execute :32-76, step by step
        n = F(2)
        total, returned = F(0), F(0)
        for e in echo:
            v = U.h2f(e)
            if v == 0:
                returned = F(returned + F(1))
            else:
                total = F(total + v)
        rs = F(F(total / n) / F(p.max_reverb_distance))
        rv = F(returned / n)
        hitsum = 1 + 1 + 7
        psum = F(F(F(F(0) + F(pv[0])) + F(pv[1])) + F(-0.75))
        muffle = F(F(1) - F(F(F(hitsum) / F(2 * 1)) * F(p.muffle_effectiveness)))
        perm = F(F(F(psum / F(2)) / F(p.permeation_strength_per_ray)) * F(p.permeation_effectiveness))
        sat = lambda x: U.umax(F(0), U.umin(F(1), x))
        want = sat(sat(F(muffle - perm)))
        s = out.settings[0]
        assert s["muffle_strength"][0].view(np.uint32) == want.view(np.uint32)
        assert s["reverb_strength"][0].view(np.uint32) == sat(rs).view(np.uint32)
        assert s["reverb_volume"][0].view(np.uint32) == sat(rv).view(np.uint32)
        assert 0 < want < 1  # not saturated: the stale slot moved it
    return sc, p, org, expect, prime


# Hit identities (north_star: bit-exact hit indices): equal-material colliders at the same
# distance, where only the index (or the type) tells the winner. ShootRayCast keeps the first
# minimum in Sphere, AABB, OBB order (:239-276).
def hit_id_ties():
    m = dict(absorption=0.25, density=1.0, echo=1.0)
    sc = art.Scene(dirs=half3_dirs([(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, 0, 1)]),
                   targets=np.array([[0, -30, 0]], np.float32),
                   spheres=cat(abi.SPHERE, sphere((0, 0, -20), 1.0, **m), sphere((10, 0, 0), 2.0, **m),
                               sphere((10, 0, 0), 2.0, **m), sphere((0, 0, 10), 2.0, **m)),
                   aabbs=cat(abi.AABB, aabb((0, -20, 0), (1, 1, 1), **m), aabb((-10, 0, 0), (2, 2, 2), **m),
                             aabb((-10, 0, 0), (2, 2, 2), **m), aabb((0, 10, 0), (2, 2, 2), **m),
                             aabb((0, 0, 10), (2, 2, 2), **m)),
                   obbs=cat(abi.OBB, obb((0, 10, 0), (2, 2, 2), (0.0, 0.0, 0.0), **m)))
    p = params()
    org = np.zeros((1, 3), np.float32)

    def expect(out):
        want = [abi.hit_id(abi.ART_COLLIDER_SPHERE, 1),   # two identical spheres: the first
                abi.hit_id(abi.ART_COLLIDER_AABB, 1),     # two identical boxes: the first
                abi.hit_id(abi.ART_COLLIDER_AABB, 3),     # AABB vs the identical identity OBB: AABB
                abi.hit_id(abi.ART_COLLIDER_SPHERE, 3)]   # sphere vs AABB at the same distance: sphere
        assert [abi.hit_id(*path(sc, org[0], r, 1)[0][:2]) for r in range(4)] == want
        assert out.hit_ids[0].tolist() == want
        assert out.echo[0].tolist() == [h(8.0)] * 4  # every candidate gives the same echo: only the id tells
    return sc, p, org, expect


KATS.update({
    "q1_echo_reset_misindex": q1_echo_reset_misindex,
    "q3_echo_unoffset_distance": q3_echo_unoffset_distance,
    "q5_obb_reflection": q5_obb_reflection,
    "q5_permeation_first_hit": q5_permeation_first_hit,
    "q10_sphere_formulas": q10_sphere_formulas,
    "q14_reflection_offset": q14_reflection_offset,
    "q15_face_ties_aabb": lambda: q15_face_ties("aabb"),
    "q15_face_ties_obb": lambda: q15_face_ties("obb"),
    "q18_stale_slots": q18_stale_slots,
    "hit_id_ties": hit_id_ties,
})
