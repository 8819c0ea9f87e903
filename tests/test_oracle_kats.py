"""Known-answer tests that pin the CPU oracle.

The reference ships no tests or fixtures and cannot run here (Unity/Burst C#), so parity is
unpinned by the reference itself; these hand-derived answers pin the oracle instead.
"""
import ctypes as C
import math
import struct

import numpy as np
import pytest

import art
import kat_scenes as K
import oracle


def f32(bits: int) -> float:
    return struct.unpack("<f", struct.pack("<I", bits))[0]


# K1 — Unity f32tof16 (round half up after truncation, double rounding in the subnormal range)
@pytest.mark.parametrize("x,expected", [
    (1.0 + 2.0 ** -11, 0x3C01),       # tie: Unity rounds up, IEEE RNE would give 0x3C00
    (f32(0x3DCCCCCD), 0x2E66),        # 0.1f
    (65504.0, 0x7BFF),
    (65520.0, 0x7C00),
    (f32(0x358637BD), 0x0011),        # 1e-6f
    (f32(0x37BB4000), 0x0177),        # subnormal double-rounding case (RNE: 0x0176)
    (-2.5, 0xC100),
    (0.0, 0x0000),
    (-0.0, 0x8000),
    (math.inf, 0x7C00),
    (-math.inf, 0xFC00),
])
def test_k1_f32tof16(x, expected):
    assert oracle.f32tof16(x) == expected
    from art.synth import f32tof16 as prod
    assert prod(x) == expected  # the product host helper agrees


def test_k1_nan_and_roundtrip():
    assert oracle.f32tof16(f32(0x7FC00001)) == 0x7E00
    assert oracle.f32tof16(f32(0xFFC00000)) == 0xFE00
    lib = oracle.load()
    # f16tof32 is exact: every finite half round-trips
    for hbits in list(range(0, 0x7C00, 97)) + [0x0001, 0x03FF, 0x0400, 0x7BFF]:
        for s in (0, 0x8000):
            assert lib.or_f32tof16(lib.or_f16tof32(hbits | s)) == (hbits | s)


def test_k1_host_helpers_agree_on_random_bits():
    """Product host f32tof16 (unity_math.hpp) == oracle restatement on 2^12 random patterns (the
    exhaustive 2^32 check is tests/test_half_exhaustive.py)."""
    from art.synth import f32tof16 as prod
    rng = np.random.default_rng(5)
    for b in rng.integers(0, 2 ** 32, 2 ** 12, dtype=np.uint64):
        x = f32(int(b))
        assert prod(x) == oracle.f32tof16(x)


def _f3(v):
    return (C.c_float * 3)(*v)


def _hit(fn, *args):
    d = C.c_float()
    ok = fn(*args, C.byref(d))
    return bool(ok), d.value


def test_k2_aabb():
    lib = oracle.load()
    ok, d = _hit(lib.or_ray_intersects_aabb, _f3((0, 0, 0)), _f3((1, 0, 0)), _f3((5, 0, 0)), _f3((1, 1, 1)))
    assert ok and d == 4.0
    # origin inside the box: tNear < 0 -> distance = tFar
    ok, d = _hit(lib.or_ray_intersects_aabb, _f3((5, 0, 0)), _f3((1, 0, 0)), _f3((5, 0, 0)), _f3((1, 1, 1)))
    assert ok and d == 1.0
    # box behind the ray
    ok, _ = _hit(lib.or_ray_intersects_aabb, _f3((0, 0, 0)), _f3((-1, 0, 0)), _f3((5, 0, 0)), _f3((1, 1, 1)))
    assert not ok
    # zero direction components give 1/d = +-inf; the slab along that axis is [-inf, inf]
    ok, d = _hit(lib.or_ray_intersects_aabb, _f3((0, 0.5, 0)), _f3((0, 0, 1)), _f3((0, 0, 9)), _f3((1, 1, 1)))
    assert ok and d == 8.0


def test_k3_sphere():
    lib = oracle.load()
    ok, d = _hit(lib.or_ray_intersects_sphere, _f3((0, 0, 0)), _f3((0, 0, 1)), _f3((0, 0, 10)), C.c_float(2.0))
    assert ok and d == 8.0
    ok, d = _hit(lib.or_ray_intersects_sphere, _f3((0, 0, 10)), _f3((0, 0, 1)), _f3((0, 0, 10)), C.c_float(2.0))
    assert ok and d == 2.0  # inside: t0 < 0, t1 >= 0
    ok, _ = _hit(lib.or_ray_intersects_sphere, _f3((0, 3, 0)), _f3((0, 0, 1)), _f3((0, 0, 10)), C.c_float(2.0))
    assert not ok


def test_k4_obb_identity_equals_aabb():
    lib = oracle.load()
    rng = np.random.default_rng(4)
    q = (C.c_float * 4)(0, 0, 0, 1)
    for _ in range(500):
        o = rng.uniform(-10, 10, 3).astype(np.float32)
        dvec = rng.standard_normal(3).astype(np.float32)
        h = rng.uniform(0.25, 3, 3).astype(np.float32)
        a = _hit(lib.or_ray_intersects_aabb, _f3(o), _f3(dvec), _f3((0, 0, 0)), _f3(h))
        b = _hit(lib.or_ray_intersects_obb, _f3(o), _f3(dvec), _f3((0, 0, 0)), _f3(h), q)
        assert a == b


def test_k5_obb_rotated_90_about_y():
    """World rotation R_y(90deg) maps local x -> world -z and local z -> world x: a box with
    half-extents (1, 2, 3) spans 3 along world x. The stored quaternion is the inverse rotation
    (AudioOBBCollider.cs:59) and the raytracer applies it as-is (:316-317)."""
    lib = oracle.load()
    s = math.sqrt(0.5)
    inv = (0.0, -s, 0.0, s)  # inverse of (0, sin45, 0, cos45)
    q = (C.c_float * 4)()
    lib.or_half_quaternion_value(K.h(inv[0]), K.h(inv[1]), K.h(inv[2]), q)
    assert abs(q[1] + s) < 1e-3 and abs(q[3] - s) < 1e-3
    ok, d = _hit(lib.or_ray_intersects_obb, _f3((0, 0, 0)), _f3((1, 0, 0)), _f3((10, 0, 0)), _f3((1, 2, 3)), q)
    assert ok and abs(d - 7.0) < 1e-3
    ok, d = _hit(lib.or_ray_intersects_obb, _f3((10, 0, -10)), _f3((0, 0, 1)), _f3((10, 0, 0)), _f3((1, 2, 3)), q)
    assert ok and abs(d - 9.0) < 1e-3


def test_quaternion_inverse_formula():
    lib = oracle.load()
    qi = (C.c_float * 4)()
    lib.or_quat_inverse((C.c_float * 4)(0.5, 0.5, 0.5, 0.5), qi)
    assert list(qi) == [-0.5, -0.5, -0.5, 0.5]


@pytest.mark.parametrize("name", sorted(K.KATS))
def test_frame_kats_on_oracle(name):
    sc, p, org, expect, *prime = K.KATS[name]()
    out = art.FanOutputs(1, sc.R, p.max_hits_per_ray, sc.T, p.thread_count, hits=True)
    if prime:
        prime[0](out)
    oracle.run(sc, p, org, out)
    expect(out)


def test_k9_reduce_on_oracle():
    sc, p, org, expect, prime = K.k9_reduce()
    out = art.FanOutputs(1, sc.R, p.max_hits_per_ray, sc.T, 1)
    prime(out)
    oracle.run(sc, p, org, out)
    expect(out)


def test_unity32_f2h_matches_oracle():
    """The KATs' numpy f32tof16 (tests/unity32.py) is the same function as the oracle's."""
    import unity32 as U
    rng = np.random.default_rng(6)
    for b in rng.integers(0, 2 ** 32, 2 ** 12, dtype=np.uint64):
        x = f32(int(b))
        assert U.f2h(np.float32(x)) == oracle.f32tof16(x)
