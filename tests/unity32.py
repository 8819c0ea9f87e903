"""TEST INFRASTRUCTURE: Unity.Mathematics 1.3.2 primitives in numpy float32, scalar by scalar.

Known-answer tests derive their expected values with these step-by-step float32 evaluations
(SURVEY.md App. A), never through the oracle (oracle/art_oracle.c) or the product: each KAT's
answer is an independent third computation of the reference's arithmetic. Every operation below
is one IEEE binary32 operation (numpy scalar float32 arithmetic rounds each result), evaluated
in the reference's order; no contraction.
"""
from __future__ import annotations

import numpy as np

F = np.float32
EPS = F(0.0001)  # AudioRaytracerJobBatched.cs:57


def f(x) -> np.float32:
    return np.float32(x)


def h2f(bits: int) -> np.float32:
    """math.f16tof32: exact."""
    return np.array([bits], np.uint16).view(np.float16).astype(np.float32)[0]


def f2h(x) -> int:
    """math.f32tof16 (App. A.1): truncate bits 0-11, round half up on bit 12, double rounding in
    the subnormal range through an fp32 multiply."""
    ux = int(np.array([x], np.float32).view(np.uint32)[0])
    uux = ux & 0x7FFFF000
    with np.errstate(over="ignore", under="ignore"):
        m = np.array([uux], np.uint32).view(np.float32)[0] * F(1.92592994e-34)
    m = umin(m, F(260042752.0))
    h = (int(np.array([m], np.float32).view(np.uint32)[0]) + 0x1000) >> 13
    if uux >= 0x7F800000:
        h = 0x7E00 if uux > 0x7F800000 else 0x7C00
    return (h | (ux & 0x80000FFF) >> 16) & 0xFFFF


def umin(x, y):
    return x if (np.isnan(y) or x < y) else y


def umax(x, y):
    return x if (np.isnan(y) or x > y) else y


def sign(x) -> np.float32:
    return F((1.0 if x > 0 else 0.0) - (1.0 if x < 0 else 0.0))


def v3(x, y, z):
    return (F(x), F(y), F(z))


def hv3(hx, hy, hz):
    return (h2f(hx), h2f(hy), h2f(hz))


def add(a, b):
    return tuple(F(p + q) for p, q in zip(a, b))


def sub(a, b):
    return tuple(F(p - q) for p, q in zip(a, b))


def mulv(a, b):
    return tuple(F(p * q) for p, q in zip(a, b))


def muls(a, s):  # float3 * float
    return tuple(F(p * s) for p in a)


def smul(s, a):  # float * float3
    return tuple(F(s * p) for p in a)


def dot(a, b):
    return F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2]))


def dot4(a, b):
    return F(F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2])) + F(a[3] * b[3]))


def cross(a, b):
    c = (F(F(a[0] * b[1]) - F(a[1] * b[0])), F(F(a[1] * b[2]) - F(a[2] * b[1])), F(F(a[2] * b[0]) - F(a[0] * b[2])))
    return (c[1], c[2], c[0])


def rcp(a):
    with np.errstate(divide="ignore"):
        return tuple(F(F(1) / p) for p in a)


def normalize(v):
    return smul(F(F(1) / np.sqrt(dot(v, v))), v)


def length(v):
    return np.sqrt(dot(v, v))


def distance(a, b):
    return length(sub(b, a))


def reflect(i, n):
    return sub(i, muls(smul(F(2), n), dot(i, n)))


def qmul(q, v):
    qv = q[:3]
    t = smul(F(2), cross(qv, v))
    return add(add(v, smul(q[3], t)), cross(qv, t))


def qinverse(q):
    r = F(F(1) / dot4(q, q))
    return (F(F(r * q[0]) * F(-1)), F(F(r * q[1]) * F(-1)), F(F(r * q[2]) * F(-1)), F(F(r * q[3]) * F(1)))


def qnormalize(q):
    r = F(F(1) / np.sqrt(dot4(q, q)))
    return tuple(F(r * p) for p in q)


def half_quaternion(hx, hy, hz):
    """halfQuaternion.QuaternionValue (DataTypes/halfQuaternion.cs:34-46)."""
    x, y, z = h2f(hx), h2f(hy), h2f(hz)
    w_sq = F(F(1) - F(F(F(x * x) + F(y * y)) + F(z * z)))
    w = np.sqrt(w_sq) if w_sq > 0 else F(0)
    return qnormalize((x, y, z, F(w)))


# ---------------------------------------------------------------- intersection routines
def slab(o, d, mn, mx):
    """The slab core of RayIntersectsAABB (:284-308): (tNear, tFar)."""
    inv = rcp(d)
    with np.errstate(invalid="ignore"):
        t0 = mulv(sub(mn, o), inv)
        t1 = mulv(sub(mx, o), inv)
    tmin = tuple(umin(a, b) for a, b in zip(t0, t1))
    tmax = tuple(umax(a, b) for a, b in zip(t0, t1))
    return umax(umax(tmin[0], tmin[1]), tmin[2]), umin(umin(tmax[0], tmax[1]), tmax[2])


def ray_aabb(o, d, c, h):
    """RayIntersectsAABB (:284-308) -> distance or None."""
    t_near, t_far = slab(o, d, sub(c, h), add(c, h))
    if t_near > t_far or t_far < 0:
        return None
    return t_near if t_near > 0 else t_far


def ray_obb(o, d, c, h, q):
    """RayIntersectsOBB (:314-320): rotation q applied as given."""
    return ray_aabb(qmul(q, sub(o, c)), qmul(q, d), v3(0, 0, 0), h)


def ray_sphere(o, d, c, r):
    """RayIntersectsSphere (:323-355), the general quadratic (a = dot(d, d))."""
    oc = sub(o, c)
    a = dot(d, d)
    b = F(F(2) * dot(oc, d))
    cc = F(dot(oc, oc) - F(r * r))
    disc = F(F(b * b) - F(F(F(4) * a) * cc))
    if disc < 0:
        return None
    sq = np.sqrt(disc)
    t0 = F(F(F(-b) - sq) / F(F(2) * a))
    t1 = F(F(F(-b) + sq) / F(F(2) * a))
    if t0 >= 0:
        return t0
    if t1 >= 0:
        return t1
    return None


def perm_sphere(o, d, c, r, density):
    """RayIntersectsSpherePermeation (AudioPermeationJobBatched.cs:303-328): unit-direction form."""
    oc = sub(o, c)
    b = dot(oc, d)
    cc = F(dot(oc, oc) - F(r * r))
    disc = F(F(b * b) - cc)
    if disc < 0:
        return F(0)
    sq = np.sqrt(disc)
    t_enter, t_exit = F(F(-b) - sq), F(F(-b) + sq)
    if t_exit < 0:
        return F(0)
    return F(umax(F(0), F(t_exit - umax(t_enter, F(0)))) * density)


def perm_sphere_general(o, d, c, r, density):
    """What the permeation loss would be with the raytracer's general quadratic (Q10's contrast)."""
    oc = sub(o, c)
    a = dot(d, d)
    b = F(F(2) * dot(oc, d))
    cc = F(dot(oc, oc) - F(r * r))
    disc = F(F(b * b) - F(F(F(4) * a) * cc))
    if disc < 0:
        return F(0)
    sq = np.sqrt(disc)
    t_enter, t_exit = F(F(F(-b) - sq) / F(F(2) * a)), F(F(F(-b) + sq) / F(F(2) * a))
    if t_exit < 0:
        return F(0)
    return F(umax(F(0), F(t_exit - umax(t_enter, F(0)))) * density)


def perm_aabb(o, d, c, h, density):
    """RayIntersectsAABBPermeation (:265-288)."""
    t_enter, t_exit = slab(o, d, sub(c, h), add(c, h))
    if t_enter > t_exit or t_exit < 0:
        return F(0)
    return F(umax(F(0), F(t_exit - umax(t_enter, F(0)))) * density)


def aabb_face_normal(p, c, h):
    """ReflectRay's AABB normal (:463-485): strict '<' between face deltas, z on ties, sign(0) = 0."""
    lp = sub(p, c)
    ap = tuple(F(abs(x)) for x in lp)
    dx, dy, dz = F(h[0] - ap[0]), F(h[1] - ap[1]), F(h[2] - ap[2])
    n = [F(0), F(0), F(0)]
    if dx < dy and dx < dz:
        n[0] = sign(lp[0])
    elif dy < dx and dy < dz:
        n[1] = sign(lp[1])
    else:
        n[2] = sign(lp[2])
    return tuple(n)


def obb_face_normal(p, c, h, q_stored, buggy=True):
    """ReflectRay's OBB normal (:487-512). buggy=True is the reference: inverse(stored) into the
    local frame (:489) and the stored rotation back (:510) (App. B Q5); buggy=False the geometric
    normal (stored into local, inverse back) for contrast."""
    q_in, q_out = (qinverse(q_stored), q_stored) if buggy else (q_stored, qinverse(q_stored))
    lh = qmul(q_in, sub(p, c))
    ap = tuple(F(abs(x)) for x in lh)
    df = sub(h, ap)
    ln = [F(0), F(0), F(0)]
    if df[0] < df[1] and df[0] < df[2]:
        ln[0] = sign(lh[0])
    elif df[1] < df[0] and df[1] < df[2]:
        ln[1] = sign(lh[1])
    else:
        ln[2] = sign(lh[2])
    return qmul(q_out, tuple(ln))


def h3(v):
    """(half3)v as a list of half bits."""
    return [f2h(x) for x in v]
