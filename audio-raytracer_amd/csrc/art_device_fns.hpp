// art_device_fns.hpp — device-side intersection primitives shared by the kernels.
//
// Restates Jobs/AudioRaytracerJobBatched.cs:225-449 and Jobs/AudioPermeationJobBatched.cs:101-141
// on the device records of art_internal.hpp (see unity_math.hpp for the exactness rules).
#pragma once

#include <float.h>
#include <hip/hip_runtime.h>

#include "art_internal.hpp"
#include "unity_math.hpp"

#pragma clang fp contract(off)

namespace art {

constexpr float kEps = 0.0001f;  // AudioRaytracerJobBatched.cs:57

// ------------------------------------------------------------------------------------------
// Ray segment with per-segment hoisted terms: 1/d (RayIntersectsAABB :289), dot(d,d) (:326).
// ------------------------------------------------------------------------------------------
struct Seg {
  vec3 o, d, inv;
  float a2;  // 2*a with a = dot(d, d); 4*a = 2 * a2 exactly (power-of-two scaling)
};

ART_HD Seg make_seg(vec3 o, vec3 d) {
  Seg s;
  s.o = o; s.d = d;
  s.inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float a = dot(d, d);
  s.a2 = 2.0f * a;
  return s;
}

// Slab test core — RayIntersectsAABB :289-307. EXACT selects Unity's min/max; otherwise IEEE
// minNum/maxNum (v_min3/v_max3), equal except for the sign of a zero distance.
template <bool EXACT>
ART_HD bool slab(float ox, float oy, float oz, float ix, float iy, float iz, float mnx,
                                     float mny, float mnz, float mxx, float mxy, float mxz, float& tNear,
                                     float& tFar) {
  float t0x = (mnx - ox) * ix, t0y = (mny - oy) * iy, t0z = (mnz - oz) * iz;
  float t1x = (mxx - ox) * ix, t1y = (mxy - oy) * iy, t1z = (mxz - oz) * iz;
  if (EXACT) {
    float tminx = umin(t0x, t1x), tminy = umin(t0y, t1y), tminz = umin(t0z, t1z);
    float tmaxx = umax(t0x, t1x), tmaxy = umax(t0y, t1y), tmaxz = umax(t0z, t1z);
    tNear = umax(umax(tminx, tminy), tminz);
    tFar = umin(umin(tmaxx, tmaxy), tmaxz);
  } else {
    float tminx = fmin_ieee(t0x, t1x), tminy = fmin_ieee(t0y, t1y), tminz = fmin_ieee(t0z, t1z);
    float tmaxx = fmax_ieee(t0x, t1x), tmaxy = fmax_ieee(t0y, t1y), tmaxz = fmax_ieee(t0z, t1z);
    tNear = fmax_ieee(fmax_ieee(tminx, tminy), tminz);
    tFar = fmin_ieee(fmin_ieee(tmaxx, tmaxy), tmaxz);
  }
  return !(tNear > tFar || tFar < 0.0f);
}

template <bool EXACT>
ART_HD bool aabb_test(const Seg& s, const AabbRec& b, float& dist) {
  float tNear, tFar;
  bool hit = slab<EXACT>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, b.mnx, b.mny, b.mnz, b.mxx, b.mxy, b.mxz,
                         tNear, tFar);
  dist = tNear > 0.0f ? tNear : tFar;
  return hit;
}

// RayIntersectsOBB :314-320 with rotation q (the stored one for the raytracer, its inverse for
// the permeation first hit :174).
template <bool EXACT>
ART_HD bool obb_test(const Seg& s, const ObbRec& b, quat q, float& dist) {
  vec3 lo = qmul(q, s.o - mk3(b.cx, b.cy, b.cz));
  vec3 ld = qmul(q, s.d);
  float ix = 1.0f / ld.x, iy = 1.0f / ld.y, iz = 1.0f / ld.z;
  float tNear, tFar;
  bool hit = slab<EXACT>(lo.x, lo.y, lo.z, ix, iy, iz, b.lmnx, b.lmny, b.lmnz, b.lmxx, b.lmxy, b.lmxz, tNear, tFar);
  dist = tNear > 0.0f ? tNear : tFar;
  return hit;
}

ART_HD quat stored_q(const ObbRec& b) { quat q; q.x = b.qx; q.y = b.qy; q.z = b.qz; q.w = b.qw; return q; }

// 1.0f / x bit for bit: where x's exponent field lies in [3, 251] the hardware reciprocal plus one
// Newton step (3 instructions) equals the IEEE division for every float (checked exhaustively on
// the GPU on this function itself through art_recip_exact_device, tests/test_recip_exhaustive.py);
// the other lanes (tiny, huge, zero, inf, NaN) divide. Device only.
#ifndef ART_FAST_RCP
#define ART_FAST_RCP 1
#endif
__device__ __forceinline__ float recip_exact(float x) {
  if (!ART_FAST_RCP) return 1.0f / x;
  float r;
  if (((__float_as_uint(x) >> 23) & 0xffu) - 3u <= 248u) {
    const float a = __builtin_amdgcn_rcpf(x);
    r = __builtin_fmaf(__builtin_fmaf(-x, a, 1.0f), a, a);
  } else {
    r = 1.0f / x;
  }
  return r;
}

// obb_test<false> with the stored rotation on the record at p, fetched in the order that keeps the
// fewest values live (the kernels' register budget): the rotation and the rotated direction's
// reciprocals, then the centre and the rotated origin, then the local bounds. Same operations.
__device__ __forceinline__ bool obb_test_staged(const Seg& s, const ObbRec* p, float& dist) {
  const float4* v = reinterpret_cast<const float4*>(p);
  const float4 qa = v[1];
  quat q;
  q.x = qa.x; q.y = qa.y; q.z = qa.z; q.w = qa.w;
  const vec3 ld = qmul(q, s.d);
  const float ix = recip_exact(ld.x), iy = recip_exact(ld.y), iz = recip_exact(ld.z);
  const float4 c = v[0];
  const vec3 lo = qmul(q, s.o - mk3(c.x, c.y, c.z));
  __builtin_amdgcn_sched_barrier(0);
  const float4 mn = v[2], mx = v[3];
  float tNear, tFar;
  const bool hit = slab<false>(lo.x, lo.y, lo.z, ix, iy, iz, mn.x, mn.y, mn.z, mx.x, mx.y, mx.z, tNear, tFar);
  dist = tNear > 0.0f ? tNear : tFar;
  return hit;
}
ART_HD quat inverse_q(const ObbCold& b) { quat q; q.x = b.iqx; q.y = b.iqy; q.z = b.iqz; q.w = b.iqw; return q; }

// RayIntersectsSphere :323-355 (general quadratic)
ART_HD bool sphere_test(const Seg& s, const SphereRec& c, float& dist) {
  vec3 oc = s.o - mk3(c.cx, c.cy, c.cz);
  float b = 2.0f * dot(oc, s.d);
  float cc = dot(oc, oc) - c.r2;
  float disc = b * b - (2.0f * s.a2) * cc;  // 4 * a * c (:329)
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc);
  float t0 = (-b - sq) / s.a2;
  float t1 = (-b + sq) / s.a2;
  if (t0 >= 0.0f) { dist = t0; return true; }
  if (t1 >= 0.0f) { dist = t1; return true; }
  return false;
}

struct LaneCounts {
  uint32_t s, a, o;
};

struct Hit {
  int type, idx;
  float dist;
};

// Scene records are read-only for the whole launch. Reading them through the constant address
// space (4) lets a wave-uniform index become a scalar (SMEM) load into SGPRs; through a generic
// pointer the compiler must assume the kernel's own stores may alias and emits vector loads.
template <typename T>
__device__ __forceinline__ T ldc(const T* p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) T* cptr;
  return ((cptr)(p))[i];
#else
  return p[i];
#endif
}

// Wave-uniform collider index: all lanes of a wave sweep the same collider, so the record is
// fetched with scalar loads (SMEM) into SGPRs even inside divergent control flow.
__device__ __forceinline__ int wave_uniform(int i) { return __builtin_amdgcn_readfirstlane(i); }

// ShootRayCast :225-280 (raytracer, float.MaxValue sentinel) and :101-141 (permeation, INFINITY
// sentinel, inverse rotation). Strict '<' keeps the first minimum in Sphere, AABB, OBB order.
template <bool PERM, bool COUNT>
__device__ __forceinline__ Hit nearest(const DevScene& sc, const Seg& s, LaneCounts& lc) {
  Hit h;
  h.type = kNone; h.idx = -1;
  h.dist = PERM ? __builtin_huge_valf() : FLT_MAX;
  for (int i = 0; i < sc.ns; ++i) {
    const SphereRec c = ldc(sc.sph, wave_uniform(i));
    float d;
    if (COUNT) lc.s++;
    if (sphere_test(s, c, d) && d < h.dist) { h.dist = d; h.type = kSphere; h.idx = i; }
  }
  for (int i = 0; i < sc.na; ++i) {
    const AabbRec b = ldc(sc.aabb, wave_uniform(i));
    float d;
    if (COUNT) lc.a++;
    if (aabb_test<false>(s, b, d) && d < h.dist) { h.dist = d; h.type = kAabb; h.idx = i; }
  }
  for (int i = 0; i < sc.no; ++i) {
    const ObbRec b = ldc(sc.obb, wave_uniform(i));
    float d;
    if (COUNT) lc.o++;
    const quat q = PERM ? inverse_q(ldc(sc.obbc, wave_uniform(i))) : stored_q(b);
    if (obb_test<false>(s, b, q, d) && d < h.dist) { h.dist = d; h.type = kObb; h.idx = i; }
  }
  // Re-evaluate the winner with Unity's exact min/max so a zero distance carries the reference sign.
  if (h.type == kAabb) { float d; aabb_test<true>(s, sc.aabb[h.idx], d); h.dist = d; }
  if (h.type == kObb) {
    const ObbRec b = sc.obb[h.idx];
    float d; obb_test<true>(s, b, PERM ? inverse_q(sc.obbc[h.idx]) : stored_q(b), d); h.dist = d;
  }
  if (PERM && h.dist == __builtin_huge_valf()) h.type = kNone;  // :140 closestDist != INFINITY
  return h;
}

// CanRaySeePoint :365-397 (SKIP=false) / CanRaySeeAudioTarget :405-449 (SKIP=true).
// A lane stops testing at its first blocker (its test count then matches the reference's early
// return); the wave leaves the sweep once every active lane is blocked.
template <bool SKIP, bool COUNT>
__device__ __forceinline__ bool visible(const DevScene& sc, const Seg& s, float maxd, int target, LaneCounts& lc) {
  bool blocked = false;
  for (int i = 0; i < sc.ns; ++i) {
    const SphereRec c = ldc(sc.sph, wave_uniform(i));
    if (SKIP && c.tid == target) continue;
    if (!blocked) {
      if (COUNT) lc.s++;
      float d;
      if (sphere_test(s, c, d) && d < maxd) blocked = true;
    }
    if (__all(blocked)) return false;
  }
  for (int i = 0; i < sc.na; ++i) {
    const AabbRec b = ldc(sc.aabb, wave_uniform(i));
    if (SKIP && b.tid == target) continue;
    if (!blocked) {
      if (COUNT) lc.a++;
      float d;
      if (aabb_test<false>(s, b, d) && d < maxd) blocked = true;
    }
    if (__all(blocked)) return false;
  }
  for (int i = 0; i < sc.no; ++i) {
    const ObbRec b = ldc(sc.obb, wave_uniform(i));
    if (SKIP && b.tid == target) continue;
    if (!blocked) {
      if (COUNT) lc.o++;
      float d;
      if (obb_test<false>(s, b, stored_q(b), d) && d < maxd) blocked = true;
    }
    if (__all(blocked)) return false;
  }
  return !blocked;
}

__device__ __forceinline__ vec3 load_dir(const uint16_t* dirs, int ray) {
  return mk3(f16tof32(dirs[3 * ray + 0]), f16tof32(dirs[3 * ray + 1]), f16tof32(dirs[3 * ray + 2]));
}
__device__ __forceinline__ vec3 load3(const float* p, int i) { return mk3(p[3 * i + 0], p[3 * i + 1], p[3 * i + 2]); }

__device__ __forceinline__ unsigned long long wave_sum_u32(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Final value of echo / hit-point slot j under sequential-batch semantics:
// batch b resets slots [b*bs, b*bs + cnt(b)*H) before writing its own rays' slots.
// Returns 0 = later reset (zero), 1 = keep written value if any (else zero if reset, else stale).
__device__ __forceinline__ int batch_slot_state(const FrameParams& fp, int j, int b, bool& any_reset) {
  auto covers = [&](int bb) {
    if (bb < 0 || bb >= fp.nb) return false;
    int start = bb * fp.bs;
    int cnt = min(fp.bs, fp.R - start);
    return j >= start && j < start + cnt * fp.H;
  };
  int hi = min(j / fp.bs, fp.nb - 1);
  bool later = false;
  for (int bb = hi; bb > b && bb >= hi - 1; --bb) later |= covers(bb);
  int lo = min(b, hi);
  any_reset = covers(lo) || covers(lo - 1);
  return later ? 0 : 1;
}

}  // namespace art
