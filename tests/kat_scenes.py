"""Hand-built scenes for the known-answer tests.

Each builder returns (scene, params, origins, expect) where `expect(out)` asserts the
hand-derived answer on a FanOutputs. The same scenes feed the oracle (CPU tests) and the HIP
path (GPU parity tests).
"""
import numpy as np

import art
from art import abi

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
        assert abs(out.perm[0, 0] - (2.0 - np.sqrt(425.0) / 10.0)) < 1e-3

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
