// art_frame_math.hpp — per-collider decode, permeation loss terms and the baked-curve lookup,
// shared by the HIP kernels (art_kernels.hip) and the CPU backend (art_cpu.cpp) so both evaluate
// the reference's fp32 operation sequences from one source.
#pragma once

#include "art_device_fns.hpp"

#pragma clang fp contract(off)

namespace art {

// ------------------------------------------------------------------------------------------
// prep: decode colliders once per upload. Every value is computed exactly as the reference
// computes it per access (Center - Size, Radius * Radius, halfQuaternion decode, inverse), so
// hoisting is bit-identical.
// ------------------------------------------------------------------------------------------
// Broad-phase margins relative to the problem's scale (broad phase): the exact tests'
// rounding can report a blocking hit at most ~3 eps (boxes) or ~sqrt(20 eps) (sphere discriminant
// cancellation) times the scale away from the true shape; the factors below exceed those bounds
// by 10x or more.
#ifndef ART_CULL_MARGIN_SCALE
#define ART_CULL_MARGIN_SCALE 1.0f  // test hook: 0 disables the margins (tests/test_broadphase_gpu.py must fail)
#endif
constexpr float kCullBox = 1e-4f * ART_CULL_MARGIN_SCALE;
constexpr float kCullSphere = 4e-3f * ART_CULL_MARGIN_SCALE;
constexpr float kCullObb = 1e-3f * ART_CULL_MARGIN_SCALE;

ART_HD CullRec make_cull(float lx, float ly, float lz, float hx, float hy, float hz, float scale,
                                             float factor) {
  CullRec c;
  const bool fin = ufinite(lx) && ufinite(ly) && ufinite(lz) && ufinite(hx) && ufinite(hy) && ufinite(hz) &&
                   ufinite(scale);
  c.lox = fin ? lx : -INFINITY; c.loy = fin ? ly : -INFINITY; c.loz = fin ? lz : -INFINITY;
  c.hix = fin ? hx : INFINITY; c.hiy = fin ? hy : INFINITY; c.hiz = fin ? hz : INFINITY;
  c.fscale = fin ? factor * scale : 0.0f;
  c.factor = factor;
  return c;
}

// Per-collider decode (shared by the full prep and the resident store's scatter): the hot/cold
// records at in-kind index i and the broad-phase bounds at global index gi.
ART_HD void prep_sphere(const art_sphere& s, int i, int gi, SphereRec* __restrict__ osph,
                                            SphereCold* __restrict__ osphc, CullRec* __restrict__ cull) {
  SphereRec r;
  r.cx = f16tof32(s.center.x); r.cy = f16tof32(s.center.y); r.cz = f16tof32(s.center.z);
  float rad = f16tof32(s.radius);
  r.r2 = rad * rad;
  r.tid = s.audio_target_id;
  r.pad0 = r.pad1 = r.pad2 = 0;
  SphereCold c;
  c.density = f16tof32(s.material.density);
  c.absorption = f16tof32(s.material.absorption);
  c.echo = f16tof32(s.material.echo);
  c.pad = 0.0f;
  osph[i] = r;
  osphc[i] = c;
  const float ra = fabsf(rad);
  cull[gi] = make_cull(r.cx - ra, r.cy - ra, r.cz - ra, r.cx + ra, r.cy + ra, r.cz + ra,
                       fabsf(r.cx) + fabsf(r.cy) + fabsf(r.cz) + ra, kCullSphere);
}

ART_HD void prep_aabb(const art_aabb& a, int i, int gi, AabbRec* __restrict__ oaabb,
                                          AabbCold* __restrict__ oaabbc, CullRec* __restrict__ cull) {
  AabbCold c;
  c.cx = f16tof32(a.center.x); c.cy = f16tof32(a.center.y); c.cz = f16tof32(a.center.z);
  c.hx = f16tof32(a.size.x); c.hy = f16tof32(a.size.y); c.hz = f16tof32(a.size.z);
  c.density = f16tof32(a.material.density);
  c.absorption = f16tof32(a.material.absorption);
  c.echo = f16tof32(a.material.echo);
  c.pad0 = c.pad1 = c.pad2 = 0.0f;
  AabbRec r;
  r.mnx = c.cx - c.hx; r.mny = c.cy - c.hy; r.mnz = c.cz - c.hz;
  r.mxx = c.cx + c.hx; r.mxy = c.cy + c.hy; r.mxz = c.cz + c.hz;
  r.tid = a.audio_target_id;
  r.pad = 0.0f;
  oaabb[i] = r;
  oaabbc[i] = c;
  cull[gi] = make_cull(fminf(r.mnx, r.mxx), fminf(r.mny, r.mxy), fminf(r.mnz, r.mxz), fmaxf(r.mnx, r.mxx),
                       fmaxf(r.mny, r.mxy), fmaxf(r.mnz, r.mxz),
                       fabsf(c.cx) + fabsf(c.cy) + fabsf(c.cz) + fabsf(c.hx) + fabsf(c.hy) + fabsf(c.hz), kCullBox);
}

ART_HD void prep_obb(const art_obb& b, int i, int gi, ObbRec* __restrict__ oobb,
                                         ObbCold* __restrict__ oobbc, CullRec* __restrict__ cull) {
  ObbRec r;
  ObbCold c;
  r.cx = f16tof32(b.center.x); r.cy = f16tof32(b.center.y); r.cz = f16tof32(b.center.z);
  c.hx = f16tof32(b.size.x); c.hy = f16tof32(b.size.y); c.hz = f16tof32(b.size.z);
  r.lmnx = 0.0f - c.hx; r.lmny = 0.0f - c.hy; r.lmnz = 0.0f - c.hz;
  r.lmxx = 0.0f + c.hx; r.lmxy = 0.0f + c.hy; r.lmxz = 0.0f + c.hz;
  r.pad0 = r.pad1 = 0.0f;
  quat q = half_quaternion_value(b.rot_x, b.rot_y, b.rot_z);
  quat qi = qinverse(q);
  r.qx = q.x; r.qy = q.y; r.qz = q.z; r.qw = q.w;
  c.iqx = qi.x; c.iqy = qi.y; c.iqz = qi.z; c.iqw = qi.w;
  r.tid = b.audio_target_id;
  c.density = f16tof32(b.material.density);
  c.absorption = f16tof32(b.material.absorption);
  c.echo = f16tof32(b.material.echo);
  c.pad0 = c.pad1 = 0.0f;
  oobb[i] = r;
  oobbc[i] = c;
  // World bounds of the rotated box (round 4; round 3 used the cube of half-width |h|_1, up to 8x the
  // volume). The tests map P - c to the local frame by the stored rotation R (ShootRayCast
  // :314-320, permeation loss :294-300) or by its inverse R^T (permeation first hit :172-179), so a
  // point reported inside the local box [-h, h] lies within half_i = max(sum_j |R_ji| h_j,
  // sum_j |R_ij| h_j) of c on world axis i. Column i of R is qmul(q, e_i); the relative and absolute
  // slack covers the rounding of these entries (each within ~10 eps), the margins the rest
  // (the margin scale keeps |h|_1).
  const float h1 = fabsf(c.hx) + fabsf(c.hy) + fabsf(c.hz);
  const float rho = h1 * 1.001f;
  const bool qok = ufinite(q.x) && ufinite(q.y) && ufinite(q.z) && ufinite(q.w);
  const vec3 ax = qmul(q, mk3(1.0f, 0.0f, 0.0f)), ay = qmul(q, mk3(0.0f, 1.0f, 0.0f)), az = qmul(q, mk3(0.0f, 0.0f, 1.0f));
  const vec3 ha = abs3(mk3(c.hx, c.hy, c.hz));
  const vec3 cx = abs3(ax), cy = abs3(ay), cz = abs3(az);  // |columns| of R
  const float slack = 1e-5f * h1;
  const float wx = fmaxf(cx.x * ha.x + cx.y * ha.y + cx.z * ha.z, cx.x * ha.x + cy.x * ha.y + cz.x * ha.z);
  const float wy = fmaxf(cy.x * ha.x + cy.y * ha.y + cy.z * ha.z, cx.y * ha.x + cy.y * ha.y + cz.y * ha.z);
  const float wz = fmaxf(cz.x * ha.x + cz.y * ha.y + cz.z * ha.z, cx.z * ha.x + cy.z * ha.y + cz.z * ha.z);
  const float bx = fminf(wx * 1.0001f + slack, rho), by = fminf(wy * 1.0001f + slack, rho), bz = fminf(wz * 1.0001f + slack, rho);
  cull[gi] = make_cull(r.cx - bx, r.cy - by, r.cz - bz, r.cx + bx, r.cy + by, r.cz + bz,
                       qok ? fabsf(r.cx) + fabsf(r.cy) + fabsf(r.cz) + rho : INFINITY, kCullObb);
}


// ------------------------------------------------------------------------------------------
// Permeation loss terms (AudioPermeationJobBatched.cs:265-328)
// ------------------------------------------------------------------------------------------
ART_HD float perm_term_sphere(const Seg& s, const SphereRec& c, float density) {
  // RayIntersectsSpherePermeation :303-328
  vec3 oc = s.o - mk3(c.cx, c.cy, c.cz);
  float b = dot(oc, s.d);
  float cc = dot(oc, oc) - c.r2;
  float disc = b * b - cc;
  if (disc < 0.0f) return 0.0f;
  float sq = sqrtf(disc);
  float tEnter = -b - sq, tExit = -b + sq;
  if (tExit < 0.0f) return 0.0f;
  float enter = umax(tEnter, 0.0f);
  return umax(0.0f, tExit - enter) * density;
}
ART_HD float perm_term_slab(float ox, float oy, float oz, float ix, float iy, float iz, float mnx,
                                                float mny, float mnz, float mxx, float mxy, float mxz, float density) {
  // RayIntersectsAABBPermeation :265-288
  float tEnter, tExit;
  if (!slab<false>(ox, oy, oz, ix, iy, iz, mnx, mny, mnz, mxx, mxy, mxz, tEnter, tExit)) return 0.0f;
  float enter = umax(tEnter, 0.0f);
  return umax(0.0f, tExit - enter) * density;
}


// NativeSampledAnimationCurve.EvaluateWithBurst (DataTypes/NativeSampledAnimationCurve.cs:81-89)
ART_HD float curve_eval(const float* baked, int n, float length, float time) {
  float percent = time / length;
  float cp = umax(0.0f, umin((float)(n - 1), percent * (float)(n - 1)));
  int fi = (int)floorf(cp), ci = (int)ceilf(cp);
  return ulerp(baked[fi], baked[ci], cp - (float)fi);
}


}  // namespace art
