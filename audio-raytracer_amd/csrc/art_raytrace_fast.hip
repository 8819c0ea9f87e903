// art_raytrace_fast.hip — the throughput raytrace kernel (AudioRaytracerJobBatched.Execute,
// Jobs/AudioRaytracerJobBatched.cs:61-215), K-way collider split.
//
// Work shape: one workgroup = one group of 64 rays of one fan, processed by K waves. Every wave
// holds the same 64 ray states (lane l <-> ray l of the group) and sweeps 1/K of each collider
// array, so the colliders stay wave-uniform (SGPR records via scalar loads) while the launch
// gets K times more waves than rays/64 — config 2 alone is only 2048 ray-waves (2 per SIMD).
//   * nearest hit: each wave finds the first minimum of its chunk; the K partials are merged
//     in LDS by (distance, global collider order), which reproduces the reference's strict-<
//     first-minimum in Sphere, AABB, OBB order (ShootRayCast :225-280);
//   * visibility (echo :124-145, muffle :150-173): any-hit is an OR over colliders, so each
//     wave sweeps its chunk (4-way unrolled, no per-lane masking, wave exit once every lane is
//     blocked) and ORs its verdict into an LDS bit per (ray, query).
// Ray slots are visited in a direction-coherent order (ray_order) so the 64 rays of a group
// point into a small solid angle and their visibility sweeps end together; every output is
// written at the ray's own index, so the order changes no result.
// This kernel does not count tests; the test-count metric comes from raytrace_kernel<COUNT>.
#include <algorithm>
#include <cstdlib>

#include "art_device_fns.hpp"

namespace art {

#ifdef ART_DIAG_CULL_STATS
__device__ unsigned g_diag[8];  // diagnostic build only: broad-phase statistics, printed per launch
#endif

constexpr int kNoHit = 0x7fffffff;

__device__ __forceinline__ void chunk_of(int n, int w, int K, int& b, int& e) {
  b = (int)(((long long)n * w) / K);
  e = (int)(((long long)n * (w + 1)) / K);
}

// Sphere test split so the common miss costs no branch: the square root and the two IEEE
// divisions run only for lanes whose discriminant is non-negative.
__device__ __forceinline__ bool sphere_hit_dist(const Seg& s, const SphereRec& c, float& dist) {
  vec3 oc = s.o - mk3(c.cx, c.cy, c.cz);
  float b = 2.0f * dot(oc, s.d);
  float cc = dot(oc, oc) - c.r2;
  float disc = b * b - s.a4 * cc;
  bool hit = false;
  dist = 0.0f;
  if (disc >= 0.0f) {
    float sq = sqrtf(disc);
    float t0 = (-b - sq) / s.a2;
    float t1 = (-b + sq) / s.a2;
    hit = (t0 >= 0.0f) || (t1 >= 0.0f);
    dist = (t0 >= 0.0f) ? t0 : t1;
  }
  return hit;
}

// First minimum of this wave's chunk (ShootRayCast :225-280 restricted to a sub-range).
// code = type rank (sphere 0, aabb 1, obb 2) << 28 | index: the global reference order.
template <int U>
__device__ __forceinline__ void nearest_chunk(const DevScene& sc, const Seg& s, int w, int K, float& best, int& code) {
  best = FLT_MAX;
  code = kNoHit;
  int b, e;
  chunk_of(sc.ns, w, K, b, e);
  int i = b;
  for (; i + U <= e; i += U) {
    SphereRec c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = ldc(sc.sph, wave_uniform(i + u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d;
      if (sphere_hit_dist(s, c[u], d) && d < best) { best = d; code = i + u; }
    }
  }
  for (; i < e; ++i) {
    const SphereRec c = ldc(sc.sph, wave_uniform(i));
    float d;
    if (sphere_hit_dist(s, c, d) && d < best) { best = d; code = i; }
  }
  chunk_of(sc.na, w, K, b, e);
  i = b;
  for (; i + U <= e; i += U) {
    AabbRec r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ldc(sc.aabb, wave_uniform(i + u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d;
      if (aabb_test<false>(s, r[u], d) && d < best) { best = d; code = (1 << 28) | (i + u); }
    }
  }
  for (; i < e; ++i) {
    const AabbRec r = ldc(sc.aabb, wave_uniform(i));
    float d;
    if (aabb_test<false>(s, r, d) && d < best) { best = d; code = (1 << 28) | i; }
  }
  chunk_of(sc.no, w, K, b, e);
  for (i = b; i < e; ++i) {
    const ObbRec r = ldc(sc.obb, wave_uniform(i));
    float d;
    if (obb_test<false>(s, r, stored_q(r), d) && d < best) { best = d; code = (2 << 28) | i; }
  }
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_mov(float v, float ident) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ident), __float_as_int(v), CTRL, ROW_MASK, 0xf, false));
}

// Wave-wide IEEE min / max (NaN lanes ignored), result wave-uniform. row_shr 1,2,4,8 within each
// row of 16, then row_bcast 15 / 31 fold the rows into lane 63.
__device__ __forceinline__ float wave_min(float v) {
  v = fminf(v, dpp_mov<0x111, 0xf>(v, INFINITY));
  v = fminf(v, dpp_mov<0x112, 0xf>(v, INFINITY));
  v = fminf(v, dpp_mov<0x114, 0xf>(v, INFINITY));
  v = fminf(v, dpp_mov<0x118, 0xf>(v, INFINITY));
  v = fminf(v, dpp_mov<0x142, 0xa>(v, INFINITY));
  v = fminf(v, dpp_mov<0x143, 0xc>(v, INFINITY));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0x111, 0xf>(v, -INFINITY));
  v = fmaxf(v, dpp_mov<0x112, 0xf>(v, -INFINITY));
  v = fmaxf(v, dpp_mov<0x114, 0xf>(v, -INFINITY));
  v = fmaxf(v, dpp_mov<0x118, 0xf>(v, -INFINITY));
  v = fmaxf(v, dpp_mov<0x142, 0xa>(v, -INFINITY));
  v = fmaxf(v, dpp_mov<0x143, 0xc>(v, -INFINITY));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Candidate colliders of a window of up to kCullW chunks of one type: bit i of m[j] = collider
// b + 64 j + i. Exact tests run U at a time while at least U candidates remain, then one by one.
#ifndef ART_CULL_U
#define ART_CULL_U 4
#endif
constexpr int kCullW = 1;  // chunks per candidate set (wider windows spill the masks)
constexpr int kCullU = ART_CULL_U;  // candidate tests per scalar-load group

// Executed-work accounting (ART_CTX_COUNT_EXECUTED): one atomic per call from lane 0, off when
// `ex` is null (a uniform branch).
__device__ __forceinline__ void exec_add(unsigned long long* ex, int slot, unsigned long long v) {
  if (ex && v && (threadIdx.x & 63) == 0) atomicAdd(ex + slot, v);
}

struct CandSet {
  unsigned long long m[kCullW];
  int left;
  __device__ __forceinline__ int pop() {  // next candidate offset from b (wave-uniform)
#pragma unroll
    for (int j = 0; j < kCullW; ++j)
      if (m[j]) {
        const int k = j * 64 + (int)__builtin_ctzll(m[j]);
        m[j] &= m[j] - 1;
        --left;
        return k;
      }
    return 0;
  }
};

// ------------------------------------------------------------------------------------------
// Broad-phase nearest hit for rays that share their origin O (the first segment of every ray of a
// fan). The wave's directions lie in a cone (axis a, half-angle theta); a collider can be hit by
// one of them only if its bounding sphere, widened by the rounding margin of the exact tests
// (CullRec), meets the cone. Candidates are tested in increasing index order with
// the same strict `<`, so the wave's first minimum over its range is unchanged.
// ------------------------------------------------------------------------------------------
struct WaveCone {
  float ox, oy, oz, om;   // shared origin, |O|_1
  float ax, ay, az;       // unit axis
  float cos_t, sin_t;     // half-angle (with slack); cos_t <= 0: no culling
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ WaveCone make_cone(vec3 O, vec3 d, bool alive) {
  WaveCone wc;
  wc.ox = O.x; wc.oy = O.y; wc.oz = O.z;
  wc.om = fabsf(O.x) + fabsf(O.y) + fabsf(O.z);
  const float n2 = d.x * d.x + d.y * d.y + d.z * d.z;
  const bool ok = alive && n2 > 0.0f && isfinite(n2);
  const float inv = ok ? 1.0f / sqrtf(n2) : 0.0f;
  const float dx = d.x * inv, dy = d.y * inv, dz = d.z * inv;
  float sx = wave_sum(dx), sy = wave_sum(dy), sz = wave_sum(dz);
  const float sn = sqrtf(sx * sx + sy * sy + sz * sz);
  // a wave with a degenerate (non-finite or zero) direction is not culled
  const bool bad = __any(alive && !ok);
  if (!(sn > 0.0f) || bad) {
    wc.ax = 1.0f; wc.ay = 0.0f; wc.az = 0.0f; wc.cos_t = -1.0f; wc.sin_t = 0.0f;
    return wc;
  }
  wc.ax = sx / sn; wc.ay = sy / sn; wc.az = sz / sn;
  float c = wave_min(ok ? dx * wc.ax + dy * wc.ay + dz * wc.az : INFINITY);
  c = fminf(c, 1.0f);
  // slack of 2e-3 rad for the rounding of the normalisations and dot products
  const float s0 = sqrtf(fmaxf(0.0f, 1.0f - c * c));
  constexpr float ce = 0.999998f, se = 0.002f;  // cos / sin of the slack angle
  wc.cos_t = c * ce - s0 * se;
  wc.sin_t = s0 * ce + c * se;
  return wc;
}

// Candidate test of collider bounds against the cone (lane = collider).
__device__ __forceinline__ bool cone_candidate(const WaveCone& wc, const CullRec& cr) {
  if (!(wc.cos_t > 0.0f)) return true;
  const float cx = 0.5f * (cr.lox + cr.hix), cy = 0.5f * (cr.loy + cr.hiy), cz = 0.5f * (cr.loz + cr.hiz);
  // bounding-sphere radius of the bounds box (|half diagonal|_1 >= |half diagonal|_2), widened
  const float rho = 0.5f * ((cr.hix - cr.lox) + (cr.hiy - cr.loy) + (cr.hiz - cr.loz)) * 1.001f +
                    cr.factor * (cr.scale + wc.om);
  const float vx = cx - wc.ox, vy = cy - wc.oy, vz = cz - wc.oz;
  const float L2 = vx * vx + vy * vy + vz * vz;
  if (!(L2 > rho * rho * 1.0001f)) return true;  // origin inside / near the bound (or non-finite)
  const float L = sqrtf(L2);
  const float sb = fminf(1.0f, rho / L * 1.0001f);
  const float cb = sqrtf(fmaxf(0.0f, 1.0f - sb * sb));
  const float cos_lim = wc.cos_t * cb - wc.sin_t * sb;  // cos(theta + beta), theta + beta < pi
  // slack (1e-4 L) only ever admits more colliders: cos_lim <= 1 and the threshold is lowered
  return vx * wc.ax + vy * wc.ay + vz * wc.az >= (cos_lim - 1e-4f) * L;
}

// Visibility cone of a wave of segments [o, o + maxd d] that (nearly) share their END point: the
// muffle rays of one target end at the target (:165), the echo rays of one fan at its origin
// (:130). Apex A = the first valid lane's computed end point; every lane's end point lies within
// `extra` of A (its computed distance, widened for the rounding of o + maxd d), so each segment
// lies in the hull of its start o and the ball (A, extra), and that hull lies in cone(A, axis,
// theta) (+) ball(extra) once o is inside the cone. Starts inside the ball need no cone. A wave
// with a non-finite segment, whose starts all lie in the ball, or whose cone is wider than a
// half-space, is not cone-culled (on = false). theta carries the 2e-3 rad slack of make_cone.
struct VisCone {
  float ax, ay, az;       // apex
  float nx, ny, nz;       // unit axis
  float cos2, sin_t;      // cos^2 and sin of the half-angle
  float extra;            // apex ball radius
  bool on;
};

__device__ __forceinline__ VisCone make_vis_cone(const Seg& s, float maxd, bool valid, float om) {
  VisCone vc;
  const vec3 e = s.o + s.d * maxd;
  const unsigned long long vm = __ballot(valid);
  const int first = vm ? (int)__builtin_ctzll(vm) : 0;
  vc.ax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e.x), first));
  vc.ay = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e.y), first));
  vc.az = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e.z), first));
  const float ex = e.x - vc.ax, ey = e.y - vc.ay, ez = e.z - vc.az;
  const float re = sqrtf(ex * ex + ey * ey + ez * ez);
  vc.extra = wave_max(valid ? re : 0.0f) * 1.001f + 1e-6f * om + 1e-6f;
  const float vx = s.o.x - vc.ax, vy = s.o.y - vc.ay, vz = s.o.z - vc.az;
  const float l2 = vx * vx + vy * vy + vz * vz;
  const float l = sqrtf(l2);
  const bool fin = isfinite(l2) && isfinite(re) && isfinite(maxd) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z);
  const bool use = valid && fin && l > vc.extra;
  const float inv = use ? 1.0f / l : 0.0f;
  const float ux = vx * inv, uy = vy * inv, uz = vz * inv;
  const float sx = wave_sum(ux), sy = wave_sum(uy), sz = wave_sum(uz);
  const float sn = sqrtf(sx * sx + sy * sy + sz * sz);
  vc.nx = 1.0f; vc.ny = 0.0f; vc.nz = 0.0f; vc.cos2 = 0.0f; vc.sin_t = 1.0f; vc.on = false;
  if (!(sn > 0.0f) || __any(valid && !fin) || !isfinite(vc.extra)) return vc;
  vc.nx = sx / sn; vc.ny = sy / sn; vc.nz = sz / sn;
  float c = wave_min(use ? ux * vc.nx + uy * vc.ny + uz * vc.nz : INFINITY);
  c = fminf(c, 1.0f);
  const float s0 = sqrtf(fmaxf(0.0f, 1.0f - c * c));
  constexpr float ce = 0.999998f, se = 0.002f;  // cos / sin of the slack angle
  const float cos_t = c * ce - s0 * se;
  vc.sin_t = s0 * ce + c * se;
  vc.cos2 = cos_t * cos_t;
  vc.on = cos_t > 0.0f;
  return vc;
}

// Does the collider's widened bounding sphere (centre c, radius rho) meet cone (+) ball(extra)?
// Distance from c to the cone's lateral surface is perp cos(theta) - proj sin(theta) (negative
// inside; for c behind the apex it is at most |c - A|, so the test only over-admits there):
// candidate iff perp cos <= rho' + proj sin =: rhs, evaluated squared (no sqrt or division) with
// an absolute slack of 1e-6 |c - A|^2 for the cancellation in perp^2 = |v|^2 - proj^2. Non-finite
// bounds give NaN/inf terms, which every comparison below admits.
__device__ __forceinline__ bool vis_cone_cand(const VisCone& vc, const CullRec& cr, float om) {
  const float cx = 0.5f * (cr.lox + cr.hix), cy = 0.5f * (cr.loy + cr.hiy), cz = 0.5f * (cr.loz + cr.hiz);
  const float rho = 0.5f * ((cr.hix - cr.lox) + (cr.hiy - cr.loy) + (cr.hiz - cr.loz)) * 1.001f +
                    cr.factor * (cr.scale + om) + vc.extra;
  const float vx = cx - vc.ax, vy = cy - vc.ay, vz = cz - vc.az;
  const float l2 = vx * vx + vy * vy + vz * vz;
  const float pj = vx * vc.nx + vy * vc.ny + vz * vc.nz;
  const float rhs = rho + pj * vc.sin_t;
  const float perp2 = l2 - pj * pj;
  return !(rhs < 0.0f) && !(perp2 * vc.cos2 > rhs * rhs + 1e-6f * l2);
}

// Front-to-back nearest hit over the spatially sorted chunks for rays sharing their origin O (the
// first segment). Wave w considers chunks c = w, w + K, ...; per pass of 64 of them, the chunks whose
// bounds meet the wave's cone are visited in increasing order of a conservative lower bound of any
// member's hit distance (distance from O to the chunk's widened bounds, shrunk for |d| != 1), and the
// sweep stops once that bound exceeds every lane's current best (shared by the block's waves through
// s_best, best only ever decreases, so a stale read only prunes less). Inside a chunk the members
// meeting the cone get the exact test; (distance, rank<<28 | original index) decides ties as the
// reference's first minimum over Sphere, AABB, OBB order does.
template <int K>
__device__ __forceinline__ void nearest_sorted(const DevScene& sc, const Seg& s, const WaveCone& wc, int w, int lane,
                                               bool alive, float (*s_best)[64], float& best, int& code,
                                               unsigned long long* ex) {
  best = FLT_MAX;
  code = kNoHit;
  const int cs_n = (sc.ns + 63) / 64, ca_n = (sc.na + 63) / 64;
  const int nch = sc.nchunks;
  const int nmine = (nch - w + K - 1) / K;  // chunks of this wave
  unsigned nt[3] = {0u, 0u, 0u}, nchk = 0u;
  s_best[w][lane] = FLT_MAX;
  for (int pb = 0; pb < nmine; pb += 64) {
    const int mine = pb + lane;
    float key = INFINITY;
    if (mine < nmine) {
      const CullRec cr = sc.chunks[w + mine * K];
      if (cone_candidate(wc, cr)) {
        const float m = cr.factor * (cr.scale + wc.om);
        const float dx = fmaxf(fmaxf(cr.lox - m - wc.ox, wc.ox - cr.hix - m), 0.0f);
        const float dy = fmaxf(fmaxf(cr.loy - m - wc.oy, wc.oy - cr.hiy - m), 0.0f);
        const float dz = fmaxf(fmaxf(cr.loz - m - wc.oz, wc.oz - cr.hiz - m), 0.0f);
        key = sqrtf(dx * dx + dy * dy + dz * dz) * 0.99f;  // |d| of a half3 direction is 1 +- 1e-3
        key = isfinite(key) ? key : 0.0f;
      }
    }
    for (;;) {
      const float kmin = wave_min(key);
      if (!(kmin < INFINITY)) break;
      // prune: no member of a chunk at distance >= kmin can beat a lane's best (all waves)
      float bl = best;
#pragma unroll
      for (int k = 0; k < K; ++k) bl = fminf(bl, s_best[k][lane]);
      const float bound = wave_max(alive ? bl : -INFINITY);
      if (kmin > bound) break;
      const int pick = (int)__builtin_ctzll(__ballot(key == kmin));
      if (lane == pick) key = INFINITY;
      const int c = w + (pb + pick) * K;
      int type, b, n;
      if (c < cs_n) { type = 0; b = c * 64; n = min(64, sc.ns - b); }
      else if (c < cs_n + ca_n) { type = 1; b = (c - cs_n) * 64; n = min(64, sc.na - b); }
      else { type = 2; b = (c - cs_n - ca_n) * 64; n = min(64, sc.no - b); }
      const int g = type == 0 ? b : (type == 1 ? sc.ns + b : sc.ns + sc.na + b);
      bool cand = false;
      if (lane < n) cand = cone_candidate(wc, sc.cull_s[g + lane]);
      CandSet cset;
      cset.m[0] = __ballot(cand);
      cset.left = __popcll(cset.m[0]);
      ++nchk;
      nt[type] += cset.left;
      if (type == 0) {
        while (cset.left > 0) {
          const SphereRec r = ldc(sc.sph_s, wave_uniform(b + cset.pop()));
          float d;
          const int cc = r.pad0;
          if (sphere_hit_dist(s, r, d) && (d < best || (d == best && cc < code))) { best = d; code = cc; }
        }
      } else if (type == 1) {
        while (cset.left > 0) {
          const AabbRec r = ldc(sc.aabb_s, wave_uniform(b + cset.pop()));
          float d;
          const int cc = (1 << 28) | __float_as_int(r.pad);
          if (aabb_test<false>(s, r, d) && (d < best || (d == best && cc < code))) { best = d; code = cc; }
        }
      } else {
        while (cset.left > 0) {
          const ObbRec r = ldc(sc.obb_s, wave_uniform(b + cset.pop()));
          float d;
          const int cc = (2 << 28) | __float_as_int(r.pad0);
          if (obb_test<false>(s, r, stored_q(r), d) && (d < best || (d == best && cc < code))) { best = d; code = cc; }
        }
      }
      s_best[w][lane] = best;
    }
  }
  exec_add(ex, kExecSphere, 64ull * nt[0]);
  exec_add(ex, kExecAabb, 64ull * nt[1]);
  exec_add(ex, kExecObb, 64ull * nt[2]);
  exec_add(ex, kExecCullCone, 64ull * (nchk + (unsigned)nmine));
}

// ------------------------------------------------------------------------------------------
// Per-lane nearest hit over the BVH (DevScene::bvh, art_bvh.hip), for any ray origin (first and
// later bounces). The lane descends into the nearest child whose widened box (margin
// factor * (scale + |o|_1), the bound of the exact tests' rounding) its ray enters
// no later than its current best distance; the farther such children wait on a per-lane LDS stack.
// A collider the ray can hit lies in every ancestor's widened box at least 3/4 of the margin
// inside, so its computed distance is strictly greater than each ancestor's computed entry and no
// ancestor is skipped while it could still win or tie. Leaves run the sweeps' exact tests, and
// (distance, type rank << 28 | index) decides, which is the reference's first minimum over
// Sphere, AABB, OBB order (ShootRayCast :225-280). Lanes with a non-finite or zero ray visit every
// node (the box tests then say nothing).
// ------------------------------------------------------------------------------------------
// Nodes of the BVH's top levels held in the workgroup's LDS (the rest is read from HBM / L2):
// levels 0..5, i.e. the whole tree up to 4096 colliders (44 KB).
constexpr int kBvhLdsNodes = 1365;
__host__ __device__ __forceinline__ int bvh_lds_nodes(const DevScene& sc) {
  return sc.bvh_levels ? min(4 * sc.bvh_leaf0 + 1, kBvhLdsNodes) : 0;
}

__device__ __forceinline__ void nearest_bvh(const DevScene& sc, const Seg& s, bool alive, const CullRec* s_nodes, int nl,
                                            uint16_t* stk, int lane, float& best, int& code, unsigned long long* ex) {
  best = FLT_MAX;
  code = kNoHit;
  unsigned nt0 = 0, nt1 = 0, nt2 = 0, nnode = 0, ndiag = 0;
  (void)ndiag;
  const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z);
  const bool force = !(isfinite(om) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
                     (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
  const int leaf0 = sc.bvh_leaf0;
  int g = alive ? 0 : -1, sp = 0;  // current node (heap order; -1: done), stack depth
  // while-while (Aila & Laine): descend inner nodes until every lane holds a leaf or is done, then
  // test the leaves together, so the two kinds of step do not interleave within the wave
  while (__any(g >= 0)) {
    while (g >= 0 && g < leaf0) {
#ifdef ART_DIAG_BVH_ITERS
      ++ndiag;
#endif
      const int c0 = 4 * g + 1;
      ++nnode;
      float e[4];
      int c[4] = {0, 1, 2, 3};
      CullRec rr[4];
      if (c0 + 3 < nl) {  // the 4 children: from LDS, or (deep levels of big scenes) from L2
#pragma unroll
        for (int k = 0; k < 4; ++k) rr[k] = s_nodes[c0 + k];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) rr[k] = sc.bvh[c0 + k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const CullRec& r = rr[k];
        const float m = r.factor * (r.scale + om);
        float tn, tf;
        const bool h = slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.lox - m, r.loy - m, r.loz - m,
                                   r.hix + m, r.hiy + m, r.hiz + m, tn, tf);
        const float en = fmaxf(tn, 0.0f);
        const bool live = r.lox <= r.hix;  // empty nodes (past the last collider) have lo > hi
        e[k] = INFINITY;
        if (live && (force || (h && en <= best))) e[k] = force ? 0.0f : en;
      }
      auto cswap = [&](int a, int b) {
        if (e[b] < e[a]) { const float te = e[a]; e[a] = e[b]; e[b] = te; const int tc = c[a]; c[a] = c[b]; c[b] = tc; }
      };
      cswap(0, 1); cswap(2, 3); cswap(0, 2); cswap(1, 3); cswap(1, 2);
      if (e[0] < INFINITY) {
#pragma unroll
        for (int k = 3; k >= 1; --k)
          if (e[k] < INFINITY) { stk[sp * 64 + lane] = (uint16_t)(c0 + c[k]); ++sp; }
        g = c0 + c[0];
      } else {
        g = sp ? (int)stk[(sp - 1) * 64 + lane] : -1;
        sp = sp ? sp - 1 : 0;
      }
    }
    if (g >= leaf0) {
#ifdef ART_DIAG_BVH_ITERS
      ++ndiag;
#endif
      // the leaf's kBvhLeaf 64-B slots: the first 32 B of each (everything but an OBB's local
      // bounds) loaded together, one memory latency per leaf
      const float4* sl = sc.bvh_leaf + (size_t)(g - leaf0) * (4 * kBvhLeaf);
      float4 qa[kBvhLeaf], qb[kBvhLeaf];
#pragma unroll
      for (int k = 0; k < kBvhLeaf; ++k) { qa[k] = sl[4 * k]; qb[k] = sl[4 * k + 1]; }
#pragma unroll
      for (int k = 0; k < kBvhLeaf; ++k) {
        const int cc = __float_as_int(qb[k].w);
        if (cc < 0) continue;  // empty slot past the last collider
        const int t = cc >> 28;
        float d = 0.0f;
        bool h;
        if (t == 0) {
          SphereRec r;
          r.cx = qa[k].x; r.cy = qa[k].y; r.cz = qa[k].z; r.r2 = qa[k].w;
          h = sphere_hit_dist(s, r, d); ++nt0;
        } else if (t == 1) {
          AabbRec r;
          r.mnx = qa[k].x; r.mny = qa[k].y; r.mnz = qa[k].z; r.mxx = qa[k].w; r.mxy = qb[k].x; r.mxz = qb[k].y;
          h = aabb_test<false>(s, r, d); ++nt1;
        } else {
          const float4 qc = sl[4 * k + 2], qd = sl[4 * k + 3];
          ObbRec r;
          r.cx = qa[k].x; r.cy = qa[k].y; r.cz = qa[k].z;
          r.qx = qa[k].w; r.qy = qb[k].x; r.qz = qb[k].y; r.qw = qb[k].z;
          r.lmnx = qc.x; r.lmny = qc.y; r.lmnz = qc.z; r.lmxx = qc.w; r.lmxy = qd.x; r.lmxz = qd.y;
          h = obb_test<false>(s, r, stored_q(r), d); ++nt2;
        }
        // a distance of exactly FLT_MAX never wins (the reference starts at float.MaxValue, strict <)
        if (h && d < FLT_MAX && (d < best || (d == best && cc < code))) { best = d; code = cc; }
      }
      g = sp ? (int)stk[(sp - 1) * 64 + lane] : -1;
      sp = sp ? sp - 1 : 0;
    }
  }
  if (ex) {
    exec_add(ex, kExecSphere, wave_sum_u32(nt0));
    exec_add(ex, kExecAabb, wave_sum_u32(nt1));
    exec_add(ex, kExecObb, wave_sum_u32(nt2));
    exec_add(ex, kExecCullBox, 4ull * wave_sum_u32(nnode));
#ifdef ART_DIAG_BVH_ITERS  // lane trips (sum) and wave trips (max) x 2^32
    {
      unsigned mx = ndiag;
      for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, off, 64));
      exec_add(ex, kExecCullCone, wave_sum_u32(ndiag) + ((unsigned long long)mx << 32));
    }
#endif
  }
}

// ------------------------------------------------------------------------------------------
// Quad-per-ray BVH traversal (nearest_bvh_quad): the K = 4 waves of a workgroup hold the same 64
// ray states (lane = ray, as the K-way split does); in the nearest-hit phase wave w traverses rays
// 16w .. 16w + 15 with 4 lanes per ray: lane q of a quad tests child q of an inner node or slot q
// of a leaf, the quad exchanges the four results through DPP quad permutes and every lane applies
// the same near-first ordering, so the ray's stack and current node stay identical in the quad.
// Four times the waves of one-lane-per-ray traversal (latency hiding at config 2's 2048 groups),
// and the inner-node / leaf steps are one test per lane instead of four.
// ------------------------------------------------------------------------------------------
#ifndef ART_QUAD_SPECULATIVE
#define ART_QUAD_SPECULATIVE 1
#endif
#ifndef ART_QUAD_SELECT_PUSH
#define ART_QUAD_SELECT_PUSH 0  // 1: stack pushes / pops as selects (measured 1-2 % slower)
#endif
#ifndef ART_QUAD_FULL_SORT
#define ART_QUAD_FULL_SORT 1  // 0: nearest child first, the rest in index order; 1: full near-first
#endif                        // order (own first-segment launch: config 3 / 5 -1 %, config 2 even);
                              // 2: full order for scenes with OBBs only
template <int SEL>
__device__ __forceinline__ int quad_bcast(int v) {
  return __builtin_amdgcn_mov_dpp(v, SEL | (SEL << 2) | (SEL << 4) | (SEL << 6), 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ int quad_perm(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false); }
constexpr int kQuadXor1 = 1 | (0 << 2) | (3 << 4) | (2 << 6), kQuadXor2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);

// Nearest hit of the quad's ray s (identical in the 4 lanes; `my` = the ray's kBvhStack u16
// stack): (distance, order) minimum in best / code of every lane of the quad.
template <bool EX>
__device__ __forceinline__ void quad_nearest_core(const DevScene& sc, const Seg& s, bool alive, int lane, uint16_t* my,
                                                  float& best, int& code, unsigned long long* ex) {
  const int qd = lane & 3;
  best = FLT_MAX;
  code = kNoHit;
  unsigned nt0 = 0, nt1 = 0, nt2 = 0, nnode = 0;
  const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z);
  const bool force = !(isfinite(om) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
                     (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
  const int leaf0 = sc.bvh_leaf0;
  const bool full_sort = ART_QUAD_FULL_SORT == 1 || (ART_QUAD_FULL_SORT == 2 && sc.no > 0);
  int g = alive ? 0 : -1, sp = 0;
  auto pop = [&]() { g = sp ? (int)my[sp - 1] : -1; sp = sp ? sp - 1 : 0; };
  auto inner_step = [&]() {
      const int c0 = 4 * g + 1;
    if (EX && qd == 0) ++nnode;
    const CullRec r = sc.bvh[c0 + qd];
    const float m = r.factor * (r.scale + om);
    float tn, tf;
    const bool h = slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.lox - m, r.loy - m, r.loz - m,
                               r.hix + m, r.hiy + m, r.hiz + m, tn, tf);
    const float en = fmaxf(tn, 0.0f);
    const bool live = r.lox <= r.hix;
    const float ek = (live && (force || (h && en <= best))) ? (force ? 0.0f : en) : INFINITY;
    if (full_sort) {  // far-to-near pushes (sorting network); pays for OBB scenes' long leaf tests
    const int eb = __float_as_int(ek);
    float e[4] = {__int_as_float(quad_bcast<0>(eb)), __int_as_float(quad_bcast<1>(eb)),
                  __int_as_float(quad_bcast<2>(eb)), __int_as_float(quad_bcast<3>(eb))};
    int c[4] = {0, 1, 2, 3};
    auto cswap = [&](int a, int b) {
      if (e[b] < e[a]) { const float te = e[a]; e[a] = e[b]; e[b] = te; const int tc = c[a]; c[a] = c[b]; c[b] = tc; }
    };
    cswap(0, 1); cswap(2, 3); cswap(0, 2); cswap(1, 3); cswap(1, 2);
#if ART_QUAD_SELECT_PUSH
    // branch-free: the entered children are the sorted prefix e[0 .. nv); lane q in 1 .. nv - 1
    // pushes child q (far first: c[nv - 1] lowest), the quad descends into c[0] or pops
    const int nv = (e[0] < INFINITY) + (e[1] < INFINITY) + (e[2] < INFINITY) + (e[3] < INFINITY);
    const int ck = qd == 1 ? c[1] : (qd == 2 ? c[2] : c[3]);
    const int top = (int)my[sp ? sp - 1 : 0];
    if (qd >= 1 && qd < nv) my[sp + nv - 1 - qd] = (uint16_t)(c0 + ck);
    g = nv > 0 ? c0 + c[0] : (sp ? top : -1);
    sp = nv > 0 ? sp + nv - 1 : (sp ? sp - 1 : 0);
#else
    if (e[0] < INFINITY) {
#pragma unroll
      for (int k = 3; k >= 1; --k)
        if (e[k] < INFINITY) {
          if (qd == 0) my[sp] = (uint16_t)(c0 + c[k]);
          ++sp;
        }
      g = c0 + c[0];
    } else {
      g = sp ? (int)my[sp - 1] : -1;
      sp = sp ? sp - 1 : 0;
    }
#endif
    } else {
    // descend into the nearest child ((entry, index) minimum over the quad, two DPP steps); the
    // other entered children go on the stack in index order, each lane writing its own
    float mn = ek;
    int mi = qd;
    {
      const float od = __int_as_float(quad_perm<kQuadXor1>(__float_as_int(mn)));
      const int oi = quad_perm<kQuadXor1>(mi);
      if (od < mn || (od == mn && oi < mi)) { mn = od; mi = oi; }
    }
    {
      const float od = __int_as_float(quad_perm<kQuadXor2>(__float_as_int(mn)));
      const int oi = quad_perm<kQuadXor2>(mi);
      if (od < mn || (od == mn && oi < mi)) { mn = od; mi = oi; }
    }
    const int qshift = lane & ~3;
    const bool push = ek < INFINITY && qd != mi;
    const uint32_t pb = (uint32_t)(__ballot(push) >> qshift) & 0xFu;
    if (mn < INFINITY) {
      if (push) my[sp + __popc(pb & ((1u << qd) - 1u))] = (uint16_t)(c0 + qd);
      sp += __popc(pb);
      g = c0 + mi;
    } else {
      g = sp ? (int)my[sp - 1] : -1;
      sp = sp ? sp - 1 : 0;
    }
    }
  };
  auto leaf_step = [&](int leaf) {
      const float4* sl = sc.bvh_leaf + (size_t)(leaf - leaf0) * (4 * kBvhLeaf) + 4 * qd;
    const float4 qa = sl[0], qb = sl[1];
    const int cc = __float_as_int(qb.w);
    float d = INFINITY;
    int dc = kNoHit;
    if (cc >= 0) {
      const int t = cc >> 28;
      float dd = 0.0f;
      bool h;
      if (t == 0) {
        SphereRec r;
        r.cx = qa.x; r.cy = qa.y; r.cz = qa.z; r.r2 = qa.w;
        h = sphere_hit_dist(s, r, dd); if (EX) ++nt0;
      } else if (t == 1) {
        AabbRec r;
        r.mnx = qa.x; r.mny = qa.y; r.mnz = qa.z; r.mxx = qa.w; r.mxy = qb.x; r.mxz = qb.y;
        h = aabb_test<false>(s, r, dd); if (EX) ++nt1;
      } else {
        const float4 qc = sl[2], qe = sl[3];
        ObbRec r;
        r.cx = qa.x; r.cy = qa.y; r.cz = qa.z;
        r.qx = qa.w; r.qy = qb.x; r.qz = qb.y; r.qw = qb.z;
        r.lmnx = qc.x; r.lmny = qc.y; r.lmnz = qc.z; r.lmxx = qc.w; r.lmxy = qe.x; r.lmxz = qe.y;
        h = obb_test<false>(s, r, stored_q(r), dd); if (EX) ++nt2;
      }
      // no hit, NaN and FLT_MAX-or-more never win (strict < against float.MaxValue)
      if (h && dd < FLT_MAX) { d = dd; dc = cc; }
    }
    // (distance, order) minimum over the quad's four slots
    {
      const float od = __int_as_float(quad_perm<kQuadXor1>(__float_as_int(d)));
      const int oc = quad_perm<kQuadXor1>(dc);
      if (od < d || (od == d && oc < dc)) { d = od; dc = oc; }
    }
    {
      const float od = __int_as_float(quad_perm<kQuadXor2>(__float_as_int(d)));
      const int oc = quad_perm<kQuadXor2>(dc);
      if (od < d || (od == d && oc < dc)) { d = od; dc = oc; }
    }
    if (d < best || (d == best && dc < code)) { best = d; code = dc; }
  };
#if ART_QUAD_SPECULATIVE
  // Speculative while-while (Aila & Laine): a quad that reaches a leaf parks it and keeps
  // descending; the wave tests leaves once every quad with work holds one, so both kinds of
  // step run with most quads busy. The order in which leaves are tested does not change the
  // (distance, order) minimum.
  int pend = -1;
  while (__any(g >= 0 || pend >= 0)) {
    for (;;) {
#if ART_QUAD_SELECT_PUSH
      {
        const bool park = g >= leaf0 && pend < 0;
        const int top = (int)my[sp ? sp - 1 : 0];
        pend = park ? g : pend;
        g = park ? (sp ? top : -1) : g;
        sp = park ? (sp ? sp - 1 : 0) : sp;
      }
#else
      if (g >= leaf0 && pend < 0) { pend = g; pop(); }
#endif
      const bool inner = g >= 0 && g < leaf0;
      if (!__any(inner) || !__any(pend < 0 && g >= 0)) break;
      if (inner) inner_step();
    }
    if (pend >= 0) { leaf_step(pend); pend = -1; }
  }
#else
  while (__any(g >= 0)) {
    while (g >= 0 && g < leaf0) inner_step();  // quad-uniform: the 4 lanes of a ray stay together
    if (g >= leaf0) { leaf_step(g); pop(); }
  }
#endif
  if (ex) {
    exec_add(ex, kExecSphere, wave_sum_u32(nt0));
    exec_add(ex, kExecAabb, wave_sum_u32(nt1));
    exec_add(ex, kExecObb, wave_sum_u32(nt2));
    exec_add(ex, kExecCullBox, 4ull * wave_sum_u32(nnode));
  }
}

// Ray r of the group (this wave's lanes 4 (r - 16 w) .. + 3) from lane r's state; writes
// s_best[r] / s_code[r] (the q = 0 lane). stk = [64 rays][kBvhStack] u16.
__device__ __forceinline__ void nearest_bvh_quad(const DevScene& sc, const Seg& own, bool own_alive, int w, int lane,
                                                 uint16_t* stk, float* s_best, int* s_code, unsigned long long* ex) {
  const int rr = 16 * w + (lane >> 2);
  Seg s;
  s.o = mk3(__shfl(own.o.x, rr, 64), __shfl(own.o.y, rr, 64), __shfl(own.o.z, rr, 64));
  s.d = mk3(__shfl(own.d.x, rr, 64), __shfl(own.d.y, rr, 64), __shfl(own.d.z, rr, 64));
  s.inv = mk3(__shfl(own.inv.x, rr, 64), __shfl(own.inv.y, rr, 64), __shfl(own.inv.z, rr, 64));
  s.a2 = __shfl(own.a2, rr, 64);
  s.a4 = __shfl(own.a4, rr, 64);
  const bool alive = __shfl((int)own_alive, rr, 64) != 0;
  float best;
  int code;
  quad_nearest_core<true>(sc, s, alive, lane, stk + rr * kBvhStack, best, code, ex);
  if ((lane & 3) == 0) { s_best[rr] = best; s_code[rr] = code; }
}

// First-segment nearest hits in a launch of their own (ART_FAST_PRE_NEAREST): one 64-ray group per
// workgroup, wave w traverses rays 16w .. 16w + 15 with 4 lanes each (quad_nearest_core). Without
// the path kernel's emission state live across the traversal, the registers allow more waves per
// SIMD. hits[g * 64 + r] = (distance bits, code) of the group's ray slot r.
#ifndef ART_FAST_COMPACT
#define ART_FAST_COMPACT 1  // multi-hit frames: later bounces traverse only the live rays
#endif
constexpr int kLiveCounters = 32;  // per-bounce list counters (H <= 32)
#ifndef ART_FAST_WPE_PRE
#define ART_FAST_WPE_PRE 8
#endif
template <bool EX>  // EX: count the executed tests (fp.exec)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ART_FAST_WPE_PRE))) void nearest_first_kernel(
    DevScene sc, FrameParams fp, const float* __restrict__ origins, const int* __restrict__ ray_order,
    int2* __restrict__ hits, float4* __restrict__ state, int step) {
  __shared__ uint16_t s_stk[kBvhStack * 64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nrb = (fp.R + 63) >> 6;
  const int g = blockIdx.x;
  const int fan = g / nrb;
  const int rr = 16 * w + (lane >> 2);
  const int slot = (g - fan * nrb) * 64 + rr;
  const bool valid = slot < fp.R;
  const int ray = valid ? ray_order[slot] : 0;
  Seg s;
  bool alive = valid;
  if (ART_FAST_COMPACT && state && step > 0) {  // the previous bounce's list of live ray slots
    const int ngroups = fp.S * nrb;
    const uint32_t* live = reinterpret_cast<const uint32_t*>(state + 2 * (size_t)ngroups * 64);
    const uint32_t cnt = live[(size_t)ngroups * 64 + step];
    if ((uint32_t)g * 64u >= cnt) return;  // the whole workgroup: past the list
    const uint32_t e = (uint32_t)g * 64u + (uint32_t)rr;
    const bool ok = e < cnt;
    const uint32_t i = ok ? live[e] : 0u;
    const float4 a = state[2 * (size_t)i], b = state[2 * (size_t)i + 1];
    s = make_seg(mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z));
    alive = ok && ((__float_as_int(b.w) >> 8) & 1) != 0;
    float best;
    int code;
    quad_nearest_core<EX>(sc, s, alive, lane, s_stk + rr * kBvhStack, best, code, EX ? fp.exec : nullptr);
    if ((lane & 3) == 0 && ok) hits[i] = make_int2(__float_as_int(best), code);
    return;
  }
  if (ART_FAST_COMPACT && state && step == 0 && blockIdx.x == 0 && threadIdx.x < kLiveCounters)
    (reinterpret_cast<uint32_t*>(state + 2 * (size_t)fp.S * nrb * 64) + (size_t)fp.S * nrb * 64)[threadIdx.x] = 0u;
  if (step == 0) {
    s = make_seg(load3(origins, fan), load_dir(sc.dirs, ray));
  } else {  // later bounce of a multi-hit frame: the path kernel's ray state
    const size_t i = (size_t)g * 64 + rr;
    const float4 a = state[2 * i], b = state[2 * i + 1];
    s = make_seg(mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z));
    alive = valid && ((__float_as_int(b.w) >> 8) & 1) != 0;
  }
  float best;
  int code;
  quad_nearest_core<EX>(sc, s, alive, lane, s_stk + rr * kBvhStack, best, code, EX ? fp.exec : nullptr);
  if ((lane & 3) == 0) hits[(size_t)g * 64 + rr] = make_int2(__float_as_int(best), code);
}

// brute-force nearest sweep of this wave's ranges (nearest_chunk): every collider of the range
__device__ __forceinline__ void exec_brute(const DevScene& sc, int w, int K, unsigned long long* ex) {
  if (!ex) return;
  int b, e;
  chunk_of(sc.ns, w, K, b, e); exec_add(ex, kExecSphere, 64ull * (e - b));
  chunk_of(sc.na, w, K, b, e); exec_add(ex, kExecAabb, 64ull * (e - b));
  chunk_of(sc.no, w, K, b, e); exec_add(ex, kExecObb, 64ull * (e - b));
}

#ifndef ART_CONE_MODE
#define ART_CONE_MODE 0
#endif
#ifndef ART_CONE_DYNAMIC
#define ART_CONE_DYNAMIC 1  // waves of a block take nearest-hit chunks dynamically (balance)
#endif
// Nearest-hit tests of a chunk's candidates in increasing index order with a strict `<`.
template <int U, typename Rec, typename Test>
__device__ __forceinline__ void nearest_group(const Rec* recs, int b, CandSet& cs, int rank, float& best, int& code,
                                              Test test) {
  while (cs.left >= U) {
    int idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) idx[u] = b + cs.pop();
    Rec r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ldc(recs, wave_uniform(idx[u]));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d;
      if (test(r[u], d) && d < best) { best = d; code = rank | idx[u]; }
    }
  }
  while (cs.left > 0) {
    const int i = b + cs.pop();
    const Rec r = ldc(recs, wave_uniform(i));
    float d;
    if (test(r, d) && d < best) { best = d; code = rank | i; }
  }
}
template <typename Rec, typename Test>
__device__ __forceinline__ void nearest_pipe(const Rec* recs, int b, CandSet& cs, int rank, float& best, int& code,
                                             Test test) {
  if (cs.left <= 0) return;
  int i = b + cs.pop();
  Rec cur = ldc(recs, wave_uniform(i));
  for (;;) {
    const bool more = cs.left > 0;
    const int inx = more ? b + cs.pop() : i;
    const Rec nxt = ldc(recs, wave_uniform(inx));
    float d;
    if (test(cur, d) && d < best) { best = d; code = rank | i; }
    if (!more) break;
    cur = nxt;
    i = inx;
  }
}

template <int U>
__device__ __forceinline__ void nearest_cone(const DevScene& sc, const Seg& s, const WaveCone& wc, int w, int K,
                                             int lane, float& best, int& code, unsigned long long* ex, int* s_chead) {
  best = FLT_MAX;
  code = kNoHit;
  unsigned nt[3] = {0u, 0u, 0u}, nchk = 0u;
#if ART_CONE_DYNAMIC
  // Waves take 64-collider chunks (global order: spheres, AABBs, OBBs) from the block's counter;
  // each wave's chunks come in increasing order, so its partial is the first minimum over them.
  (void)K;
  const int cs_n = (sc.ns + 63) / 64, ca_n = (sc.na + 63) / 64, co_n = (sc.no + 63) / 64;
  const int nch = cs_n + ca_n + co_n;
  for (;;) {
    int gc = 0;
    if (lane == 0) gc = atomicAdd(s_chead, 1);
    gc = __builtin_amdgcn_readfirstlane(__shfl(gc, 0, 64));
    if (gc >= nch) break;
    int type, cb, e, gofs;
    if (gc < cs_n) { type = 0; cb = gc * 64; e = min(cb + 64, sc.ns); gofs = 0; }
    else if (gc < cs_n + ca_n) { type = 1; cb = (gc - cs_n) * 64; e = min(cb + 64, sc.na); gofs = sc.ns; }
    else { type = 2; cb = (gc - cs_n - ca_n) * 64; e = min(cb + 64, sc.no); gofs = sc.ns + sc.na; }
    {
#else
  (void)s_chead;
  for (int type = 0; type < 3; ++type) {
    const int n = type == 0 ? sc.ns : (type == 1 ? sc.na : sc.no);
    const int gofs = type == 0 ? 0 : (type == 1 ? sc.ns : sc.ns + sc.na);
    int b, e;
    chunk_of(n, w, K, b, e);
    for (int cb = b; cb < e; cb += 64) {
#endif
      const int k = cb + lane;
      bool cand = false;
      if (k < e) cand = cone_candidate(wc, sc.cull[gofs + k]);
      CandSet cs;
      cs.m[0] = __ballot(cand);
      cs.left = __popcll(cs.m[0]);
      ++nchk;
      nt[type] += cs.left;
#ifdef ART_DIAG_CULL_STATS
      if (lane == 0) { atomicAdd(&g_diag[4], (unsigned)min(64, e - cb)); atomicAdd(&g_diag[5], (unsigned)cs.left); }
#endif
#if ART_CONE_MODE == 1
      // groups of kCullU records per scalar-load wait, then singles
      if (type == 0) {
        nearest_group<kCullU>(sc.sph, cb, cs, 0, best, code, [&](const SphereRec& r, float& d) { return sphere_hit_dist(s, r, d); });
      } else if (type == 1) {
        nearest_group<kCullU>(sc.aabb, cb, cs, 1 << 28, best, code, [&](const AabbRec& r, float& d) { return aabb_test<false>(s, r, d); });
      } else {
        nearest_group<1>(sc.obb, cb, cs, 2 << 28, best, code, [&](const ObbRec& r, float& d) { return obb_test<false>(s, r, stored_q(r), d); });
      }
#elif ART_CONE_MODE == 2
      // one-deep pipeline: the next candidate's record load is issued before this one's test
      if (type == 0) {
        nearest_pipe(sc.sph, cb, cs, 0, best, code, [&](const SphereRec& r, float& d) { return sphere_hit_dist(s, r, d); });
      } else if (type == 1) {
        nearest_pipe(sc.aabb, cb, cs, 1 << 28, best, code, [&](const AabbRec& r, float& d) { return aabb_test<false>(s, r, d); });
      } else {
        nearest_pipe(sc.obb, cb, cs, 2 << 28, best, code, [&](const ObbRec& r, float& d) { return obb_test<false>(s, r, stored_q(r), d); });
      }
#else
      if (type == 0) {
        while (cs.left > 0) {
          const int i = cb + cs.pop();
          const SphereRec c = ldc(sc.sph, wave_uniform(i));
          float d;
          if (sphere_hit_dist(s, c, d) && d < best) { best = d; code = i; }
        }
      } else if (type == 1) {
        while (cs.left > 0) {
          const int i = cb + cs.pop();
          const AabbRec r = ldc(sc.aabb, wave_uniform(i));
          float d;
          if (aabb_test<false>(s, r, d) && d < best) { best = d; code = (1 << 28) | i; }
        }
      } else {
        while (cs.left > 0) {
          const int i = cb + cs.pop();
          const ObbRec r = ldc(sc.obb, wave_uniform(i));
          float d;
          if (obb_test<false>(s, r, stored_q(r), d) && d < best) { best = d; code = (2 << 28) | i; }
        }
      }
#endif
    }
  }
  exec_add(ex, kExecSphere, 64ull * nt[0]);
  exec_add(ex, kExecAabb, 64ull * nt[1]);
  exec_add(ex, kExecObb, 64ull * nt[2]);
  exec_add(ex, kExecCullCone, 64ull * nchk);
}

// ------------------------------------------------------------------------------------------
// Compacted any-hit visibility (CanRaySeePoint :365-397, CanRaySeeAudioTarget :405-449).
// Every (ray, query) pair of the block — the echo ray and the T muffle rays of each ray that hit
// something — goes into an LDS queue. Each wave rotates through the collider chunks in lockstep
// (the collider index stays wave-uniform, so records stay in SGPRs); a lane holds one pair, tests
// it against the current chunk, and leaves as soon as the pair is blocked or has seen every
// chunk; free lanes are refilled from the queue at chunk boundaries. Any-hit is an OR over the
// colliders, so the cyclic chunk order gives the reference's verdict, and a wave only keeps
// sweeping for lanes that are still unblocked.
// ------------------------------------------------------------------------------------------
#ifndef ART_FAST_TWO_LEVEL
// 1: visibility walks the spatially sorted chunks' union bounds first when the scene has more than
// 64 chunks (config 4: +1 %; the larger kernel cost configs 2/5 1-4 %, so off by default)
#define ART_FAST_TWO_LEVEL 0
#endif
#ifndef ART_FAST_SORTED_NEAREST
#define ART_FAST_SORTED_NEAREST 0  // 1: first-segment nearest hit front to back over sorted chunks
// (measured no faster on config 2: pruning needs every lane of a wide cone to have a hit; and the
// cross-wave best sharing would need a barrier-protected reset before it is exact)
#endif
#ifndef ART_FAST_SPLIT
#define ART_FAST_SPLIT 1  // visibility in its own kernel (vis_kernel) fed by a global pair array
#endif
#ifndef ART_FAST_CULL
#define ART_FAST_CULL 1  // broad-phase visibility (exact; see visibility_culled)
#endif
#ifndef ART_FAST_STAGED
#define ART_FAST_STAGED 0  // 1: visibility records staged through LDS (measured slower: lower occupancy, barrier waits)
#endif
#ifndef ART_FAST_CHUNK
#define ART_FAST_CHUNK 64
#endif
constexpr int kChunk = ART_FAST_CHUNK;  // colliders per chunk
constexpr int kMaxQueries = 8; // echo + up to 7 targets per ray (larger T uses raytrace_kernel)
constexpr int kNoOwner = 0x7fffffff;  // echo rays skip no collider (AudioTargetId is 16-bit)

// One (ray, query) visibility segment, 48 B (3 x ds_read_b128). a4 = 4a is not stored: it equals
// 2 * a2 exactly (a power-of-two scaling of the same value).
struct alignas(16) PairSeg {
  float ox, oy, oz, dx;
  float dy, dz, ix, iy;
  float iz, a2, maxd;
  int owner;
};

struct ChunkMap {
  int cs, ca, co;  // chunk counts per type (spheres, AABBs, OBBs)
  __device__ __forceinline__ int total() const { return cs + ca + co; }
};

// Test one chunk for this lane's pair. `done` lanes (free or blocked) do not change.
template <int U, typename Rec, typename Test>
__device__ __forceinline__ bool sweep_records(const Rec* recs, int b, int e, bool blocked, bool done, Test test) {
  int i = b;
#ifdef ART_FAST_PIPELINE
  // software-pipelined: the scalar loads of the next pair are in flight while this pair is tested
  if (i + 2 <= e) {
    Rec c0 = ldc(recs, i), c1 = ldc(recs, i + 1);
    for (; i + 4 <= e; i += 2) {
      const Rec n0 = ldc(recs, i + 2), n1 = ldc(recs, i + 3);
      blocked |= test(c0);
      blocked |= test(c1);
      c0 = n0; c1 = n1;
      if (((i - b) & 2) && __all(blocked || done)) return blocked;
    }
    blocked |= test(c0);
    blocked |= test(c1);
    i += 2;
  }
  for (; i < e; ++i) blocked |= test(ldc(recs, i));
  return blocked;
#endif
  for (; i + U <= e; i += U) {
    Rec r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ldc(recs, wave_uniform(i + u));
#pragma unroll
    for (int u = 0; u < U; ++u) blocked |= test(r[u]);
    if (__all(blocked || done)) return blocked;
  }
  for (; i < e; ++i) blocked |= test(ldc(recs, wave_uniform(i)));
  return blocked;
}

template <int U>
__device__ __forceinline__ bool sweep_chunk(const DevScene& sc, const ChunkMap& cm, int c, const Seg& s, float maxd,
                                            int owner, bool blocked, bool done) {
  if (c < cm.cs) {
    const int b = c * kChunk, e = min(b + kChunk, sc.ns);
    return sweep_records<U>(sc.sph, b, e, blocked, done, [&](const SphereRec& r) {
      float d;
      return sphere_hit_dist(s, r, d) && d < maxd && r.tid != owner;
    });
  }
  c -= cm.cs;
  if (c < cm.ca) {
    const int b = c * kChunk, e = min(b + kChunk, sc.na);
    return sweep_records<U>(sc.aabb, b, e, blocked, done, [&](const AabbRec& r) {
      float d;
      return aabb_test<false>(s, r, d) && d < maxd && r.tid != owner;
    });
  }
  c -= cm.ca;
  const int b = c * kChunk, e = min(b + kChunk, sc.no);
  for (int i = b; i < e; ++i) {
    const ObbRec r = ldc(sc.obb, wave_uniform(i));
    float d;
    blocked |= obb_test<false>(s, r, stored_q(r), d) && d < maxd && r.tid != owner;
    if ((i & 3) == 3 && __all(blocked || done)) return blocked;
  }
  return blocked;
}

// Drain the block's pair queue. Results: s_res[p] = 1 if pair p is blocked.
template <int U>
__device__ __forceinline__ void visibility_queue(const DevScene& sc, const PairSeg* s_seg, uint8_t* s_res, int* s_head,
                                                 int np, int w, int K, int lane) {
  const ChunkMap cm = {(sc.ns + kChunk - 1) / kChunk, (sc.na + kChunk - 1) / kChunk, (sc.no + kChunk - 1) / kChunk};
  const int nchunks = cm.total();
  if (nchunks == 0 || np == 0) {  // no collider: nothing blocks
    for (int p = w * 64 + lane; p < np; p += K * 64) s_res[p] = 0;
    return;
  }
  // Every wave starts at chunk 0: the waves on a CU then stream the same records and share the
  // scalar cache (a per-wave stagger measured 5 % slower on config 2).
  int c = 0;
  int my = -1, left = 0;
  bool blocked = false;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwner;
  const unsigned long long lt = (1ull << lane) - 1ull;
  while (true) {
    const bool need = my < 0;
    const unsigned long long m = __ballot(need);
    if (m) {
      int base = 0;
      if (lane == 0) base = atomicAdd(s_head, __popcll(m));
      base = __shfl(base, 0, 64);
      if (need) {
        const int p = base + __popcll(m & lt);
        if (p < np) {
          const PairSeg g = s_seg[p];
          s.o = mk3(g.ox, g.oy, g.oz); s.d = mk3(g.dx, g.dy, g.dz); s.inv = mk3(g.ix, g.iy, g.iz);
          s.a2 = g.a2; s.a4 = 2.0f * g.a2;
          maxd = g.maxd; owner = g.owner;
          my = p; left = nchunks; blocked = false;
        }
      }
    }
    const bool active = my >= 0;
    if (__all(!active)) break;
    blocked = sweep_chunk<U>(sc, cm, c, s, maxd, owner, blocked, !active);
    if (active) {
      left -= 1;
      if (blocked || left == 0) { s_res[my] = blocked ? 1 : 0; my = -1; }
    }
    c = (c + 1 == nchunks) ? 0 : c + 1;
  }
}

// ------------------------------------------------------------------------------------------
// LDS-staged variant of the visibility queue. The block's waves sweep the rotating chunk order
// together: chunk c+1 is copied global -> LDS (global_load_lds, no VGPR staging) while chunk c is
// tested, and every wave reads the records of the current chunk from LDS (broadcast ds_read_b128:
// one LDS cycle per lane group). This takes the collider stream off the scalar path, where about
// half of all record loads waited for an L2 round trip (SQC_DCACHE_MISSES + _DUPLICATE, r01
// profile). The per-lane logic (refill at chunk boundaries, leave when blocked or after a full
// cycle) is that of visibility_queue.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;

// Bytes of one staging buffer: a chunk of the largest record type present in the scene.
__host__ __device__ __forceinline__ int stage_stride(const DevScene& sc) {
  return kChunk * (sc.no > 0 ? (int)sizeof(ObbRec) : (int)sizeof(SphereRec) > (int)sizeof(AabbRec) ? (int)sizeof(SphereRec) : (int)sizeof(AabbRec));
}

// Copy `bytes` (a multiple of 1 KiB) starting at g into LDS at dst; wave w of K copies KiB w, w+K,
// ... (one global_load_lds_dwordx4 = 64 lanes x 16 B per KiB).
__device__ __forceinline__ void stage_chunk(const uint8_t* g, uint8_t* dst, int bytes, int w, int K, int lane) {
  for (int off = w * 1024; off < bytes; off += K * 1024)
    __builtin_amdgcn_global_load_lds((const void*)(g + off + lane * 16), (lds_void_t*)(dst + off), 16, 0, 0);
}

__device__ __forceinline__ void chunk_src(const DevScene& sc, const ChunkMap& cm, int c, const uint8_t*& src, int& n,
                                          int& bytes) {
  if (c < cm.cs) {
    const int b = c * kChunk;
    n = min(kChunk, sc.ns - b);
    src = reinterpret_cast<const uint8_t*>(sc.sph + b);
    bytes = kChunk * (int)sizeof(SphereRec);
    return;
  }
  c -= cm.cs;
  if (c < cm.ca) {
    const int b = c * kChunk;
    n = min(kChunk, sc.na - b);
    src = reinterpret_cast<const uint8_t*>(sc.aabb + b);
    bytes = kChunk * (int)sizeof(AabbRec);
    return;
  }
  c -= cm.ca;
  const int b = c * kChunk;
  n = min(kChunk, sc.no - b);
  src = reinterpret_cast<const uint8_t*>(sc.obb + b);
  bytes = kChunk * (int)sizeof(ObbRec);
}

template <int U, typename Test>
__device__ __forceinline__ bool sweep_lds(int n, bool blocked, bool done, Test test) {
  int i = 0;
  for (; i + U <= n; i += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) blocked |= test(i + u);
    if (__all(blocked || done)) return blocked;
  }
  for (; i < n; ++i) blocked |= test(i);
  return blocked;
}

template <int U>
__device__ __forceinline__ bool sweep_chunk_lds(const ChunkMap& cm, int c, int n, const uint8_t* buf, const Seg& s,
                                                float maxd, int owner, bool blocked, bool done) {
  if (c < cm.cs) {
    const float4* r4 = reinterpret_cast<const float4*>(buf);
    return sweep_lds<U>(n, blocked, done, [&](int i) {
      const float4 a = r4[2 * i];  // cx, cy, cz, r2
      SphereRec r;
      r.cx = a.x; r.cy = a.y; r.cz = a.z; r.r2 = a.w;
      float d;
      bool hit = sphere_hit_dist(s, r, d) && d < maxd;
      if (hit) hit = reinterpret_cast<const int*>(buf)[8 * i + 4] != owner;  // tid, read only on a hit
      return hit;
    });
  }
  if (c - cm.cs < cm.ca) {
    const AabbRec* rr = reinterpret_cast<const AabbRec*>(buf);
    return sweep_lds<U>(n, blocked, done, [&](int i) {
      const AabbRec r = rr[i];
      float d;
      return aabb_test<false>(s, r, d) && d < maxd && r.tid != owner;
    });
  }
  const ObbRec* rr = reinterpret_cast<const ObbRec*>(buf);
  for (int i = 0; i < n; ++i) {
    const ObbRec r = rr[i];
    float d;
    blocked |= obb_test<false>(s, r, stored_q(r), d) && d < maxd && r.tid != owner;
    if ((i & 3) == 3 && __all(blocked || done)) return blocked;
  }
  return blocked;
}

// stage: 2 buffers of kChunk * 64 B (the largest record) after the pair segments.
template <int U>
__device__ __forceinline__ void visibility_staged(const DevScene& sc, const PairSeg* s_seg, uint8_t* s_res, int* s_head,
                                                  int* s_go, uint8_t* stage, int np, int w, int K, int lane) {
  const ChunkMap cm = {(sc.ns + kChunk - 1) / kChunk, (sc.na + kChunk - 1) / kChunk, (sc.no + kChunk - 1) / kChunk};
  const int nchunks = cm.total();
  if (nchunks == 0 || np == 0) {  // no collider: nothing blocks
    for (int p = w * 64 + lane; p < np; p += K * 64) s_res[p] = 0;
    return;
  }
  const int kBuf = stage_stride(sc);
  int c = 0;
  {
    const uint8_t* src; int n, bytes;
    chunk_src(sc, cm, 0, src, n, bytes);
    stage_chunk(src, stage, bytes, w, K, lane);
  }
  int my = -1, left = 0;
  bool blocked = false;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwner;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int it = 0;; ++it) {
    // refill free lanes from the block's pair queue
    const bool need = my < 0;
    const unsigned long long m = __ballot(need);
    if (m) {
      int base = 0;
      if (lane == 0) base = atomicAdd(s_head, __popcll(m));
      base = __shfl(base, 0, 64);
      if (need) {
        const int p = base + __popcll(m & lt);
        if (p < np) {
          const PairSeg g = s_seg[p];
          s.o = mk3(g.ox, g.oy, g.oz); s.d = mk3(g.dx, g.dy, g.dz); s.inv = mk3(g.ix, g.iy, g.iz);
          s.a2 = g.a2; s.a4 = 2.0f * g.a2;
          maxd = g.maxd; owner = g.owner;
          my = p; left = nchunks; blocked = false;
        }
      }
    }
    const bool active = my >= 0;
    const bool wave_active = __any(active);
    // block vote (triple-buffered flag: slot it%3 is read after this barrier, reset two rounds later)
    if (threadIdx.x == 0) s_go[(it + 1) % 3] = 0;
    if (lane == 0 && wave_active) s_go[it % 3] = 1;
    __syncthreads();  // also retires the staging copy of chunk c (vmcnt drained before the barrier)
    if (!s_go[it % 3]) break;
    const int cn = (c + 1 == nchunks) ? 0 : c + 1;
    const uint8_t* cur = stage + (it & 1) * kBuf;
    {
      const uint8_t* src; int n, bytes;
      chunk_src(sc, cm, cn, src, n, bytes);
      stage_chunk(src, stage + ((it + 1) & 1) * kBuf, bytes, w, K, lane);
    }
    if (wave_active) {
      const uint8_t* src; int n, bytes;
      chunk_src(sc, cm, c, src, n, bytes);
      blocked = sweep_chunk_lds<U>(cm, c, n, cur, s, maxd, owner, blocked, !active);
      if (active) {
        left -= 1;
        if (blocked || left == 0) { s_res[my] = blocked ? 1 : 0; my = -1; }
      }
    }
    c = cn;
  }
}

// ------------------------------------------------------------------------------------------
// Broad-phase visibility (SURVEY.md §8 f rank 4): results identical to the brute-force sweep.
// A wave takes a batch of 64 consecutive pairs of the block's queue (same query, direction-
// coherent rays), reduces the bounding box of their segments [o, o + maxd d] once, and sweeps the
// collider chunks in order: per chunk the lanes load the 64 colliders' broad-phase bounds
// (coalesced vector loads) and ballot the candidates whose bounds, widened by the rounding margin
// of the exact tests, overlap the box; only candidates get the exact wave-uniform test. A
// collider that is not a candidate cannot block any lane's segment (broad phase),
// so every pair's verdict equals the brute-force OR. Test counts reported by the metric stay the
// reference algorithm's (brute-force-equivalent, SURVEY.md §8 d).
// ------------------------------------------------------------------------------------------
struct WaveBox {
  float lx, ly, lz, hx, hy, hz, om;
};

template <int U, typename Rec, typename Test>
__device__ __forceinline__ bool test_candidates(const Rec* recs, int b, CandSet& cs, bool blocked, bool done, Test test,
                                                unsigned& nt) {
  while (cs.left >= U) {
    nt += U;
    int idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) idx[u] = b + cs.pop();
    Rec r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ldc(recs, wave_uniform(idx[u]));
#pragma unroll
    for (int u = 0; u < U; ++u) blocked |= test(r[u]);
    if (__all(blocked || done)) return blocked;
  }
  while (cs.left > 0) {
    const Rec r = ldc(recs, wave_uniform(b + cs.pop()));
    blocked |= test(r);
    ++nt;
  }
  return blocked;
}

// Broad-phase any-hit sweep of one lane's segment (s, maxd, owner) for a wave of up to 64
// segments (`valid` lanes): the wave's segment box (and, for vis_kernel, the visibility cone of
// make_vis_cone), then per chunk the bound ballot and the exact tests of the candidates. Flat:
// every chunk of [c_lo, c_hi) in reference order. Two-level (`two`, needs the spatially sorted
// scene of art_bvh.hip): chunks [c_lo, c_hi) of the sorted order are tested as a whole first
// (lane = chunk, union bounds), then the members of the candidate chunks. Any-hit is an OR over
// the colliders, so the order is free. Returns the lane's verdict (true = blocked).
// The box of a wave's segments [o, o + maxd d] (valid lanes) and the margin term max |o|_1 + maxd.
__device__ __forceinline__ WaveBox make_wave_box(const Seg& s, float maxd, bool valid) {
  WaveBox wb;
  const vec3 e = s.o + s.d * maxd;
  const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
  wb.lx = wave_min(valid ? fminf(s.o.x, e.x) : INFINITY);
  wb.ly = wave_min(valid ? fminf(s.o.y, e.y) : INFINITY);
  wb.lz = wave_min(valid ? fminf(s.o.z, e.z) : INFINITY);
  wb.hx = wave_max(valid ? fmaxf(s.o.x, e.x) : -INFINITY);
  wb.hy = wave_max(valid ? fmaxf(s.o.y, e.y) : -INFINITY);
  wb.hz = wave_max(valid ? fmaxf(s.o.z, e.z) : -INFINITY);
  wb.om = wave_max(valid ? om : 0.0f);
  return wb;
}

#ifndef ART_VIS_ALL_PRE
#define ART_VIS_ALL_PRE 0
#endif
#ifndef ART_VIS_OBB_PRE
#define ART_VIS_OBB_PRE 1
#endif
// wbp: a precomputed box of (a superset of) the wave's segments, else computed here.
__device__ __forceinline__ bool cull_sweep(const DevScene& sc, const Seg& s, float maxd, int owner, bool valid, int lane,
                                           unsigned long long* ex, bool done_in = false, int c_lo = 0, int c_hi = 1 << 30,
                                           const VisCone* vc = nullptr, bool two = false, const WaveBox* wbp = nullptr) {
  const ChunkMap cm = {(sc.ns + kChunk - 1) / kChunk, (sc.na + kChunk - 1) / kChunk, (sc.no + kChunk - 1) / kChunk};
  const int nchunks = min(cm.total(), c_hi);
  if (c_lo >= nchunks) return false;
  const WaveBox wb = wbp ? *wbp : make_wave_box(s, maxd, valid);
  bool blocked = false;
  const bool done = !valid || done_in;
  if (__all(done)) return false;
  unsigned nt[3] = {0u, 0u, 0u}, nchk = 0u;
  // broad-phase candidate: widened bounds meet the wave box (and the cone)
  auto candidate = [&](const CullRec& cr) {
    const float m = cr.factor * (cr.scale + wb.om);
    bool c = (cr.lox - m <= wb.hx) & (cr.hix + m >= wb.lx) & (cr.loy - m <= wb.hy) & (cr.hiy + m >= wb.ly) &
             (cr.loz - m <= wb.hz) & (cr.hiz + m >= wb.lz);
    if (vc && vc->on && __any(c)) c = c && vis_cone_cand(*vc, cr, wb.om);
    return c;
  };
  // chunk c: type, first (sorted) index within the type, member count; returns the global index
  auto chunk_at = [&](int c, int& type, int& b, int& n) {
    if (c < cm.cs) { type = 0; b = c * kChunk; n = min(kChunk, sc.ns - b); return b; }
    if (c - cm.cs < cm.ca) { type = 1; b = (c - cm.cs) * kChunk; n = min(kChunk, sc.na - b); return sc.ns + b; }
    type = 2; b = (c - cm.cs - cm.ca) * kChunk; n = min(kChunk, sc.no - b);
    return sc.ns + sc.na + b;
  };
  // exact tests of one chunk's candidates (records `sph`/`aabb`/`obb`: reference or sorted order)
  auto test_chunk = [&](int type, int b, CandSet& cs, const SphereRec* sph, const AabbRec* aabb, const ObbRec* obb) {
    if (ART_VIS_ALL_PRE && type < 2) {  // the same prefilter for spheres and boxes
      const CullRec* cb = (sph == sc.sph_s ? sc.cull_s : sc.cull) + (type == 0 ? 0 : sc.ns);
      const float oml = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
      const bool force = !(isfinite(oml) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
                         (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
      while (cs.left > 0) {
        const int i = wave_uniform(b + cs.pop());
        const CullRec c = ldc(cb, i);
        const float m = c.factor * (c.scale + oml);
        float tn, tf;
        const bool h = slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, c.lox - m, c.loy - m, c.loz - m,
                                   c.hix + m, c.hiy + m, c.hiz + m, tn, tf);
        const bool near = force || (h && tn <= maxd);
        if (!__any(near && !blocked && !done)) continue;
        ++nt[type];
        if (type == 0) {
          const SphereRec r = ldc(sph, i);
          if (near && !blocked) { float d; blocked = sphere_hit_dist(s, r, d) && d < maxd && r.tid != owner; }
        } else {
          const AabbRec r = ldc(aabb, i);
          if (near && !blocked) { float d; blocked = aabb_test<false>(s, r, d) && d < maxd && r.tid != owner; }
        }
        if (__all(blocked || done)) break;
      }
    } else if (type == 0) {
      blocked = test_candidates<kCullU>(sph, b, cs, blocked, done, [&](const SphereRec& r) {
        float d;
        return sphere_hit_dist(s, r, d) && d < maxd && r.tid != owner;
      }, nt[0]);
    } else if (type == 1) {
      blocked = test_candidates<kCullU>(aabb, b, cs, blocked, done, [&](const AabbRec& r) {
        float d;
        return aabb_test<false>(s, r, d) && d < maxd && r.tid != owner;
      }, nt[1]);
    } else if (!ART_VIS_OBB_PRE) {
      blocked = test_candidates<1>(obb, b, cs, blocked, done, [&](const ObbRec& r) {
        float d;
        return obb_test<false>(s, r, stored_q(r), d) && d < maxd && r.tid != owner;
      }, nt[2]);
    } else {
      // OBB candidates (118-op exact test): first each lane's slab test against the collider's own
      // widened bounds (the per-lane BVH node test of anyhit_bvh: a blocker's segment enters them
      // before maxd); the exact test runs only where a live lane passes
      const CullRec* cb = (obb == sc.obb_s ? sc.cull_s : sc.cull) + sc.ns + sc.na;
      const float oml = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
      const bool force = !(isfinite(oml) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
                         (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
      while (cs.left > 0) {
        const int i = wave_uniform(b + cs.pop());
        const CullRec c = ldc(cb, i);
        const float m = c.factor * (c.scale + oml);
        float tn, tf;
        const bool h = slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, c.lox - m, c.loy - m, c.loz - m,
                                   c.hix + m, c.hiy + m, c.hiz + m, tn, tf);
        const bool near = force || (h && tn <= maxd);
        if (!__any(near && !blocked && !done)) continue;
        const ObbRec r = ldc(obb, i);
        ++nt[2];
        if (near && !blocked) {
          float d;
          blocked = obb_test<false>(s, r, stored_q(r), d) && d < maxd && r.tid != owner;
        }
        if (__all(blocked || done)) break;
      }
    }
  };
  if (!two) {
    // Flat: every chunk's members (the bounds of chunk c + 1 are loaded while chunk c's candidates
    // are tested).
    CullRec nxt;
    {
      int t0, b0, n0;
      const int g0 = chunk_at(c_lo, t0, b0, n0);
      nxt = sc.cull[g0 + min(lane, n0 - 1)];
    }
    for (int c = c_lo; c < nchunks; ++c) {
      int type, b, n;
      chunk_at(c, type, b, n);
      const CullRec cr = nxt;
      if (c + 1 < nchunks) {
        int t1, b1, n1;
        const int g1 = chunk_at(c + 1, t1, b1, n1);
        nxt = sc.cull[g1 + min(lane, n1 - 1)];
      }
      CandSet cs;
      cs.m[0] = __ballot((lane < n) && candidate(cr));
      cs.left = __popcll(cs.m[0]);
      ++nchk;
#ifdef ART_DIAG_CULL_STATS
      if (lane == 0) { atomicAdd(&g_diag[1], 1u); atomicAdd(&g_diag[2], (unsigned)cs.left); }
#endif
      if (cs.left == 0) continue;
      test_chunk(type, b, cs, sc.sph, sc.aabb, sc.obb);
      if (__all(blocked || done)) break;
    }
  } else {
    for (int pb = c_lo; pb < nchunks; pb += 64) {
      const int pc = pb + lane;
      bool ccand = false;
      if (pc < nchunks) ccand = candidate(sc.chunks[pc]);
      unsigned long long cm_mask = __ballot(ccand);
      ++nchk;
      while (cm_mask) {
        const int c = pb + (int)__builtin_ctzll(cm_mask);
        cm_mask &= cm_mask - 1;
        int type, b, n;
        const int g = chunk_at(c, type, b, n);
        bool cand = false;
        if (lane < n) cand = candidate(sc.cull_s[g + lane]);
        CandSet cs;
        cs.m[0] = __ballot(cand);
        cs.left = __popcll(cs.m[0]);
        ++nchk;
#ifdef ART_DIAG_CULL_STATS
        if (lane == 0) { atomicAdd(&g_diag[1], 1u); atomicAdd(&g_diag[2], (unsigned)cs.left); }
#endif
        if (cs.left == 0) continue;
        test_chunk(type, b, cs, sc.sph_s, sc.aabb_s, sc.obb_s);
        if (__all(blocked || done)) break;
      }
      if (__all(blocked || done)) break;
    }
  }
  exec_add(ex, kExecSphere, 64ull * nt[0]);
  exec_add(ex, kExecAabb, 64ull * nt[1]);
  exec_add(ex, kExecObb, 64ull * nt[2]);
  exec_add(ex, kExecCullBox, 64ull * nchk);
  return blocked;
}

template <int U>
__device__ __forceinline__ void visibility_culled(const DevScene& sc, const PairSeg* s_seg, uint8_t* s_res, int* s_head,
                                                  int np, int lane, unsigned long long* ex) {
  for (;;) {
    int base = 0;
    if (lane == 0) base = atomicAdd(s_head, 64);
    base = __builtin_amdgcn_readfirstlane(__shfl(base, 0, 64));
    if (base >= np) break;
    const int p = base + lane;
    const bool valid = p < np;
    const PairSeg g = s_seg[valid ? p : base];
    Seg s;
    s.o = mk3(g.ox, g.oy, g.oz); s.d = mk3(g.dx, g.dy, g.dz); s.inv = mk3(g.ix, g.iy, g.iz);
    s.a2 = g.a2; s.a4 = 2.0f * g.a2;
#ifdef ART_DIAG_CULL_STATS
    {
      const unsigned nv = (unsigned)__popcll(__ballot(valid));
      if (lane == 0) { atomicAdd(&g_diag[0], 1u); atomicAdd(&g_diag[3], nv); }
    }
#endif
    const bool blocked = cull_sweep(sc, s, g.maxd, g.owner, valid, lane, ex);
    if (valid) s_res[p] = blocked ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Split visibility (ART_FAST_SPLIT): the path kernel emits every (hit, query) pair with its output
// destination into a global array; vis_kernel sweeps them in batches of 64 with the broad phase
// and writes the visible echoes and muffle counts. Visibility never feeds back into ray paths
// (echo :124-145 and muffle :150-173 only write outputs), so the two kernels give the same
// results as the fused sweep, and each runs with its own, much smaller, register state.
// ------------------------------------------------------------------------------------------
// Pair arrays (struct of arrays, pair index = emission order):
//   seg[2 i], seg[2 i + 1]  (o.xyz, maxd), (d.xyz, owner)   32 B, read by the visibility sweep;
//                           1/d and dot(d, d) are recomputed there by make_seg (same operations)
//   out[i]                  (dest, val)                      8 B, read by vis_finalize
//   flag[i]                 0 = no blocker found yet, 1 = blocked
// Echo pairs fill [0, echo_cap) in emission order (the 64 rays of a wave share the fan origin, one
// batch each); muffle pairs fill [echo_cap, echo_cap + S R H T). counts[0] / counts[1] = echo /
// muffle pairs emitted.
struct VisPairs {
  float4* seg;
  uint2* out;      // dest: echo u16 index into the fan blocks / muffle_acc index; val: echo half | kPairMuffle
  uint32_t* flag;
  uint32_t echo_cap;  // multiple of 64
};
constexpr uint32_t kPairMuffle = 1u << 16;

// The segment of pair i as the sweeps see it.
__device__ __forceinline__ void load_pair_seg(const VisPairs& vp, uint32_t i, Seg& s, float& maxd, int& owner) {
  const float4 q0 = vp.seg[2 * (size_t)i], q1 = vp.seg[2 * (size_t)i + 1];
  s = make_seg(mk3(q0.x, q0.y, q0.z), mk3(q1.x, q1.y, q1.z));
  maxd = q0.w;
  owner = __float_as_int(q1.w);
}

#ifndef ART_VIS_WPE  // 8 waves per SIMD once the test counters compile out (vis_kernel<false>): config 2
#define ART_VIS_WPE 8  // vis 228 -> 215 us, config 5 -2 %, config 3 even (a few spills, measured faster)
#endif
#ifndef ART_VIS_PLAIN_FLAG
#define ART_VIS_PLAIN_FLAG 0
#endif
// Chunk ranges per 64-pair batch (work items of the muffle sweep), by scene kind: each range
// repeats the batch's setup, while OBB tests are long and balance better over more items.
// Measured (raytrace stage): no OBBs 2 ranges (config 2: 218 vs 231 us at 4, 274 at 1); OBB
// majority 8 (config 3: 0.98 vs 1.01 ms at 4); some OBBs 4 (config 4: 5.73 vs 5.84 ms at 8,
// config 5: 2.69 vs 2.81).
#ifndef ART_VIS_RANGES_OBB
#define ART_VIS_RANGES_OBB 8
#endif
#ifndef ART_VIS_RANGES_MIXED
#define ART_VIS_RANGES_MIXED 4
#endif
#ifndef ART_VIS_RANGES
#define ART_VIS_RANGES 2
#endif
__host__ __device__ __forceinline__ int vis_ranges(const DevScene& sc) {
  return 2 * sc.no > sc.ns + sc.na + sc.no ? ART_VIS_RANGES_OBB : (sc.no > 0 ? ART_VIS_RANGES_MIXED : ART_VIS_RANGES);
}
#ifndef ART_VIS_SORT
#define ART_VIS_SORT 1  // visibility batches in (target, direction from the target) order (vis_sort_key)
#endif
#ifndef ART_VIS_ECHO_QUAD
#define ART_VIS_ECHO_QUAD 1  // echo pairs by quad-per-segment BVH traversal (vis_echo_quad_kernel)
#endif
#ifndef ART_VIS_ALL_QUAD
#define ART_VIS_ALL_QUAD 0  // 1: the muffle batches by quad traversal too
#endif
#ifndef ART_VIS_DESC
#define ART_VIS_DESC 0  // 1: batch box + cone computed once per batch (vis_batch_kernel): config 2 -3 us in vis_kernel, +12 us kernel
#endif
#ifndef ART_VIS_TWO_LEVEL
#define ART_VIS_TWO_LEVEL 1  // vis_kernel walks the sorted scene's chunk bounds first (art_bvh.hip)
#endif
#ifndef ART_VIS_CONE
#define ART_VIS_CONE 1  // cone broad phase around the batch's shared end point (make_vis_cone)
#endif

// Sort key of a muffle pair: target t and the octahedral Morton cell (32 x 32) of the ray's
// direction seen from the target, so 64 consecutive sorted pairs form a thin cone with apex t
// (1024 cells per target: 1.8 % broad-phase candidates in simulation, 4096: 1.6 %).
#ifndef ART_SORT_DIR_BITS
#define ART_SORT_DIR_BITS 10
#endif
constexpr int kSortDirBits = ART_SORT_DIR_BITS, kSortBins = kMaxQueries << kSortDirBits;
__device__ __forceinline__ uint16_t vis_sort_key(int t, vec3 u) {
  const float n = fabsf(u.x) + fabsf(u.y) + fabsf(u.z);
  float a = 0.0f, c = 0.0f;
  if (n > 0.0f && isfinite(n)) {
    const float x = u.x / n, y = u.y / n, z = u.z / n;
    a = z < 0.0f ? (1.0f - fabsf(y)) * (x >= 0.0f ? 1.0f : -1.0f) : x;
    c = z < 0.0f ? (1.0f - fabsf(x)) * (y >= 0.0f ? 1.0f : -1.0f) : y;
  }
  constexpr float kCells = (float)(1 << (kSortDirBits / 2));  // cells per octahedral axis
  auto q5 = [](float v) { return (uint32_t)fminf(fmaxf((v + 1.0f) * (0.5f * kCells), 0.0f), kCells - 1.0f); };
  auto sp = [](uint32_t v) {  // 5 bits -> even bit positions
    v = (v | (v << 4)) & 0x0F0Fu; v = (v | (v << 2)) & 0x3333u; v = (v | (v << 1)) & 0x5555u;
    return v;
  };
  return (uint16_t)(((uint32_t)t << kSortDirBits) | sp(q5(a)) | (sp(q5(c)) << 1));
}

// Pair of lane `lane` in batch b: echo batches cover [0, echo_cap) in emission order, muffle batches
// the sorted muffle pairs (order = sorted position -> muffle pair, or identity). Returns false for
// a batch past the emitted pairs; n_in = the batch's valid lanes (the others get the batch's first
// pair, so every lane holds a real segment).
__device__ __forceinline__ bool batch_pair(const VisPairs& vp, const uint32_t* count, const uint32_t* order, uint32_t b,
                                           int lane, uint32_t& pi, uint32_t& n_in) {
  const uint32_t base = b * 64u;
  uint32_t rel, n, off;
  if (base < vp.echo_cap) { rel = base; n = ldc(count, 0); off = 0u; }
  else { rel = base - vp.echo_cap; n = ldc(count, 1); off = vp.echo_cap; }
  if (rel >= n) return false;
  n_in = min(64u, n - rel);
  const uint32_t q = rel + ((uint32_t)lane < n_in ? (uint32_t)lane : 0u);
  pi = off + ((order && off) ? order[q] : q);
  return true;
}

// Broad-phase descriptor of one 64-pair batch, computed once (vis_batch_kernel) for all its chunk
// ranges: the segments' box and margin term, and the apex cone (cos2 <= 0: no cone).
struct alignas(16) BatchDesc {
  float lx, ly, lz, om;
  float hx, hy, hz, extra;
  float ax, ay, az, cos2;
  float nx, ny, nz, sin_t;
};

__global__ __launch_bounds__(256) void vis_batch_kernel(VisPairs vp, const uint32_t* __restrict__ count, uint32_t nb_max,
                                                        const uint32_t* __restrict__ order, BatchDesc* __restrict__ desc) {
  const int lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * 4u + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t pi, n_in;
  if (b >= nb_max || !batch_pair(vp, count, order, b, lane, pi, n_in)) return;
  const bool valid = (uint32_t)lane < n_in;
  Seg s;
  float maxd;
  int owner;
  load_pair_seg(vp, pi, s, maxd, owner);
  const WaveBox wb = make_wave_box(s, maxd, valid);
  const VisCone vc = make_vis_cone(s, maxd, valid, wb.om);
  if (lane == 0) {
    BatchDesc d;
    d.lx = wb.lx; d.ly = wb.ly; d.lz = wb.lz; d.om = wb.om;
    d.hx = wb.hx; d.hy = wb.hy; d.hz = wb.hz; d.extra = vc.extra;
    d.ax = vc.ax; d.ay = vc.ay; d.az = vc.az; d.cos2 = vc.on ? vc.cos2 : -1.0f;
    d.nx = vc.nx; d.ny = vc.ny; d.nz = vc.nz; d.sin_t = vc.sin_t;
    desc[b] = d;
  }
}

// Work item i of vis_kernel = (chunk range r, batch b), range-major: r = i / nb_max, b = i % nb_max.
// A batch's later ranges usually start after its earlier ones finished and skip the pairs those
// already blocked (a stale read only costs work). Verdicts meet in VisPairs::flag through relaxed
// device-scope atomicOr (no fences: an agent-scope release writes back the XCD's L2);
// vis_finalize writes the outputs after the kernel boundary.
__device__ __forceinline__ void vis_sweep_body(const DevScene& sc, const VisPairs& vp, const uint32_t* count,
                                               uint32_t nb_max, const uint32_t* order, const BatchDesc* desc,
                                               unsigned long long* ex, uint32_t b_first, uint32_t blk,
                                               bool force_two = false) {
  const int lane = threadIdx.x & 63;
  // items cover batches [b_first, nb_max) (b_first > 0: the echo batches run in vis_echo_quad_kernel)
  const uint32_t nbv = nb_max - b_first;
  const uint32_t item = blk * 4u + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t r = item / nbv, b = b_first + (item - r * nbv);
  const int nranges = vis_ranges(sc);
  uint32_t pi, n_in;
  if (r >= (uint32_t)nranges || !batch_pair(vp, count, order, b, lane, pi, n_in)) return;
#ifdef ART_DIAG_VIS_ONLY_ECHO  // diagnostic builds only: time one region of the pairs
  if (b * 64u >= vp.echo_cap) return;
#endif
#ifdef ART_DIAG_VIS_ONLY_MUFFLE
  if (b * 64u < vp.echo_cap) return;
#endif
  uint32_t* flag = vp.flag + pi;
  // pairs an earlier range already blocked are skipped (not loaded, and out of the wave's box)
#if ART_VIS_PLAIN_FLAG
  // plain load: a stale 0 (another XCD's verdict not yet visible) only repeats work
  const bool valid = (uint32_t)lane < n_in && *flag == 0u;
#else
  const bool valid = (uint32_t)lane < n_in && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
#endif
  if (!__any(valid)) return;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwner;
  s.o = s.d = s.inv = mk3(0.0f, 0.0f, 0.0f);
  s.a2 = s.a4 = 0.0f;
  if (valid) load_pair_seg(vp, pi, s, maxd, owner);
  const int nch = (sc.ns + kChunk - 1) / kChunk + (sc.na + kChunk - 1) / kChunk + (sc.no + kChunk - 1) / kChunk;
  // force_two (compile-time true in vis_kernel<., true>): the scene has the sorted chunks
  const bool two = force_two || (sc.chunks != nullptr && (ART_VIS_TWO_LEVEL || (ART_FAST_TWO_LEVEL && sc.nchunks > 64)));
  const int c_lo = (int)(((long long)nch * r) / nranges), c_hi = (int)(((long long)nch * (r + 1)) / nranges);
#if ART_VIS_CONE
  bool blocked;
  if (desc) {  // the batch's box and cone, computed once for its ranges (scalar loads)
    const BatchDesc d = ldc(desc, (int)b);
    WaveBox wb;
    wb.lx = d.lx; wb.ly = d.ly; wb.lz = d.lz; wb.om = d.om; wb.hx = d.hx; wb.hy = d.hy; wb.hz = d.hz;
    VisCone vc;
    vc.ax = d.ax; vc.ay = d.ay; vc.az = d.az; vc.nx = d.nx; vc.ny = d.ny; vc.nz = d.nz;
    vc.cos2 = d.cos2; vc.sin_t = d.sin_t; vc.extra = d.extra; vc.on = d.cos2 > 0.0f;
    blocked = cull_sweep(sc, s, maxd, owner, valid, lane, ex, false, c_lo, c_hi, &vc, two, &wb);
  } else {
    const float om = wave_max(valid ? fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd : 0.0f);
    const VisCone vc = make_vis_cone(s, maxd, valid, om);
    blocked = cull_sweep(sc, s, maxd, owner, valid, lane, ex, false, c_lo, c_hi, &vc, two);
  }
#else
  const bool blocked = cull_sweep(sc, s, maxd, owner, valid, lane, ex, false, c_lo, c_hi, nullptr, two);
#endif
  if (valid && blocked) __hip_atomic_fetch_or(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------
// Any-hit visibility by per-lane BVH traversal (CanRaySeePoint :365-397 / CanRaySeeAudioTarget
// :405-449): the lane's segment [o, o + maxd d] visits the nodes whose widened box (margin
// factor * (scale + |o|_1 + maxd), the box broad phase's bound) it enters before maxd, and stops at
// its first blocker. A blocker's computed distance d < maxd lies strictly after the entry of every
// ancestor (nearest_bvh), so no ancestor of a blocker is skipped; the verdict is the OR over all
// colliders, the reference's verdict (order-free).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool anyhit_bvh(const DevScene& sc, const Seg& s, float maxd, int owner, bool valid,
                                           const CullRec* s_nodes, int nl, uint16_t* stk, int lane, unsigned* nt) {
  const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
  const bool force = !(isfinite(om) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
                     (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
  const int leaf0 = sc.bvh_leaf0;
  bool blocked = false;
  int g = valid ? 0 : -1, sp = 0;
  while (__any(g >= 0)) {
    while (g >= 0 && g < leaf0) {
      const int c0 = 4 * g + 1;
      ++nt[3];
      CullRec rr[4];
      if (c0 + 3 < nl) {
#pragma unroll
        for (int k = 0; k < 4; ++k) rr[k] = s_nodes[c0 + k];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) rr[k] = sc.bvh[c0 + k];
      }
      int nxt = -1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const CullRec& r = rr[k];
        const float m = r.factor * (r.scale + om);
        float tn, tf;
        const bool h = slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.lox - m, r.loy - m, r.loz - m,
                                   r.hix + m, r.hiy + m, r.hiz + m, tn, tf);
        const bool live = r.lox <= r.hix;
        if (live && (force || (h && tn <= maxd))) {
          if (nxt < 0) nxt = c0 + k;
          else { stk[sp * 64 + lane] = (uint16_t)(c0 + k); ++sp; }
        }
      }
      if (nxt >= 0) g = nxt;
      else { g = sp ? (int)stk[(sp - 1) * 64 + lane] : -1; sp = sp ? sp - 1 : 0; }
    }
    if (g >= leaf0) {
      const float4* sl = sc.bvh_leaf + (size_t)(g - leaf0) * (4 * kBvhLeaf);
      float4 qa[kBvhLeaf], qb[kBvhLeaf];
#pragma unroll
      for (int k = 0; k < kBvhLeaf; ++k) { qa[k] = sl[4 * k]; qb[k] = sl[4 * k + 1]; }
#pragma unroll
      for (int k = 0; k < kBvhLeaf; ++k) {
        const int cc = __float_as_int(qb[k].w);
        if (cc < 0 || blocked) continue;
        const int t = cc >> 28;
        float d = 0.0f;
        bool h;
        int tid;
        if (t == 0) {
          SphereRec r;
          r.cx = qa[k].x; r.cy = qa[k].y; r.cz = qa[k].z; r.r2 = qa[k].w;
          h = sphere_hit_dist(s, r, d); tid = __float_as_int(qb[k].z); ++nt[0];
        } else if (t == 1) {
          AabbRec r;
          r.mnx = qa[k].x; r.mny = qa[k].y; r.mnz = qa[k].z; r.mxx = qa[k].w; r.mxy = qb[k].x; r.mxz = qb[k].y;
          h = aabb_test<false>(s, r, d); tid = __float_as_int(qb[k].z); ++nt[1];
        } else {
          const float4 qc = sl[4 * k + 2], qd = sl[4 * k + 3];
          ObbRec r;
          r.cx = qa[k].x; r.cy = qa[k].y; r.cz = qa[k].z;
          r.qx = qa[k].w; r.qy = qb[k].x; r.qz = qb[k].y; r.qw = qb[k].z;
          r.lmnx = qc.x; r.lmny = qc.y; r.lmnz = qc.z; r.lmxx = qc.w; r.lmxy = qd.x; r.lmxz = qd.y;
          h = obb_test<false>(s, r, stored_q(r), d); tid = __float_as_int(qd.z); ++nt[2];
        }
        blocked = h && d < maxd && tid != owner;  // :373-394, :411-447
      }
      if (blocked) { g = -1; sp = 0; }
      else { g = sp ? (int)stk[(sp - 1) * 64 + lane] : -1; sp = sp ? sp - 1 : 0; }
    }
  }
  return blocked;
}

constexpr int kVisBvhWaves = 8;

// One wave per batch of 64 sorted pairs, the block's waves sharing the LDS copy of the top BVH
// nodes; the verdict goes to VisPairs::flag (vis_finalize writes the outputs).
__global__ __launch_bounds__(64 * kVisBvhWaves) void vis_bvh_kernel(DevScene sc, VisPairs vp,
                                                                    const uint32_t* __restrict__ count, uint32_t nb_max,
                                                                    const uint32_t* __restrict__ order,
                                                                    unsigned long long* ex) {
  extern __shared__ CullRec s_vnodes[];
  __shared__ uint16_t s_vstk[kVisBvhWaves * kBvhStack * 64];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nl = bvh_lds_nodes(sc);
  for (int i = threadIdx.x; i < nl; i += blockDim.x) s_vnodes[i] = sc.bvh[i];
  __syncthreads();
  const uint32_t b = blockIdx.x * (uint32_t)kVisBvhWaves + (uint32_t)w;
  uint32_t pi, n_in;
  if (b >= nb_max || !batch_pair(vp, count, order, b, lane, pi, n_in)) return;
  const bool valid = (uint32_t)lane < n_in;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwner;
  s.o = s.d = s.inv = mk3(0.0f, 0.0f, 0.0f);
  s.a2 = s.a4 = 0.0f;
  if (valid) load_pair_seg(vp, pi, s, maxd, owner);
  unsigned nt[4] = {0u, 0u, 0u, 0u};
  const bool blocked = anyhit_bvh(sc, s, maxd, owner, valid, s_vnodes, nl, s_vstk + w * (kBvhStack * 64), lane, nt);
  if (valid && blocked) vp.flag[pi] = 1u;
  if (ex) {
    exec_add(ex, kExecSphere, wave_sum_u32(nt[0]));
    exec_add(ex, kExecAabb, wave_sum_u32(nt[1]));
    exec_add(ex, kExecObb, wave_sum_u32(nt[2]));
    exec_add(ex, kExecCullBox, 4ull * wave_sum_u32(nt[3]));
  }
}

// ------------------------------------------------------------------------------------------
// Echo visibility by quad-per-segment BVH traversal (ART_VIS_ECHO_QUAD). An echo batch is one
// wave's rays of one fan traced back to the fan origin: 64 segments fanning over an eighth of the
// sphere, whose box and cone admit ~10 % of the colliders, so the chunk sweep spends most of its
// time there. Per segment the BVH visits only the nodes along it. 4 lanes per segment (lane q:
// child q / leaf slot q; the quad agrees through ballots), first blocker ends the segment. Same
// exactness argument as anyhit_bvh.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void vis_quad_body(const DevScene& sc, const VisPairs& vp, const uint32_t* count,
                                              const uint32_t* order, unsigned long long* ex, uint32_t blk, uint16_t* s_stk) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), qd = lane & 3;
  const int slot = w * 16 + (lane >> 2);                       // segment of the block's 64-pair batch
  uint32_t p, n_in;
  if (!batch_pair(vp, count, order, blk, slot, p, n_in)) return;
  if ((uint32_t)(w * 16) >= n_in) return;                      // this wave's 16 segments are past the batch's end
  const bool valid = (uint32_t)slot < n_in;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwner;
  s.o = s.d = s.inv = mk3(0.0f, 0.0f, 0.0f);
  s.a2 = s.a4 = 0.0f;
  if (valid) load_pair_seg(vp, p, s, maxd, owner);
  const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
  const bool force = !(isfinite(om) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
                     (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
  const int leaf0 = sc.bvh_leaf0, qshift = lane & ~3;
  uint16_t* my = s_stk + slot * kBvhStack;
  unsigned nt0 = 0, nt1 = 0, nt2 = 0, nnode = 0;
  bool blocked = false;
  int g = valid ? 0 : -1, sp = 0;
  while (__any(g >= 0)) {
    while (g >= 0 && g < leaf0) {  // quad-uniform
      const int c0 = 4 * g + 1;
      if (qd == 0) ++nnode;
      const CullRec r = sc.bvh[c0 + qd];
      const float m = r.factor * (r.scale + om);
      float tn, tf;
      const bool h = slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.lox - m, r.loy - m, r.loz - m,
                                 r.hix + m, r.hiy + m, r.hiz + m, tn, tf);
      const bool enter = r.lox <= r.hix && (force || (h && tn <= maxd));
      const uint32_t eb = (uint32_t)(__ballot(enter) >> qshift) & 0xFu;
      if (eb) {
        const int first = __builtin_ctz(eb);
        const uint32_t rest = eb & (eb - 1u);
        if (enter && qd != first) my[sp + __popc(rest & ((1u << qd) - 1u))] = (uint16_t)(c0 + qd);
        sp += __popc(rest);
        g = c0 + first;
      } else {
        g = sp ? (int)my[sp - 1] : -1;
        sp = sp ? sp - 1 : 0;
      }
    }
    if (g >= leaf0) {
      const float4* sl = sc.bvh_leaf + (size_t)(g - leaf0) * (4 * kBvhLeaf) + 4 * qd;
      const float4 qa = sl[0], qb = sl[1];
      const int cc = __float_as_int(qb.w);
      bool blk = false;
      if (cc >= 0) {
        const int t = cc >> 28;
        float d = 0.0f;
        bool hh;
        int tid;
        if (t == 0) {
          SphereRec rr;
          rr.cx = qa.x; rr.cy = qa.y; rr.cz = qa.z; rr.r2 = qa.w;
          hh = sphere_hit_dist(s, rr, d); tid = __float_as_int(qb.z); ++nt0;
        } else if (t == 1) {
          AabbRec rr;
          rr.mnx = qa.x; rr.mny = qa.y; rr.mnz = qa.z; rr.mxx = qa.w; rr.mxy = qb.x; rr.mxz = qb.y;
          hh = aabb_test<false>(s, rr, d); tid = __float_as_int(qb.z); ++nt1;
        } else {
          const float4 qc = sl[2], qe = sl[3];
          ObbRec rr;
          rr.cx = qa.x; rr.cy = qa.y; rr.cz = qa.z;
          rr.qx = qa.w; rr.qy = qb.x; rr.qz = qb.y; rr.qw = qb.z;
          rr.lmnx = qc.x; rr.lmny = qc.y; rr.lmnz = qc.z; rr.lmxx = qc.w; rr.lmxy = qe.x; rr.lmxz = qe.y;
          hh = obb_test<false>(s, rr, stored_q(rr), d); tid = __float_as_int(qe.z); ++nt2;
        }
        blk = hh && d < maxd && tid != owner;  // :373-394
      }
      if ((uint32_t)(__ballot(blk) >> qshift) & 0xFu) {
        blocked = true;
        g = -1;
      } else {
        g = sp ? (int)my[sp - 1] : -1;
        sp = sp ? sp - 1 : 0;
      }
    }
  }
  if (valid && blocked && qd == 0) vp.flag[p] = 1u;
  if (ex) {
    exec_add(ex, kExecSphere, wave_sum_u32(nt0));
    exec_add(ex, kExecAabb, wave_sum_u32(nt1));
    exec_add(ex, kExecObb, wave_sum_u32(nt2));
    exec_add(ex, kExecCullBox, 4ull * wave_sum_u32(nnode));
  }
}

// One launch for both visibility halves, so they overlap on the chip: blocks [0, n_echo) trace
// the echo batches by quad BVH traversal (longer jobs first), the others run the sweep's items.
// EX: count the executed tests (fp.exec); without it the counters compile out.
template <bool EX, bool TWO>  // TWO: two-level sweep known on the host (the flat sweep compiles out)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ART_VIS_WPE)))
void vis_kernel(DevScene sc, VisPairs vp, const uint32_t* __restrict__ count, uint32_t nb_max,
                const uint32_t* __restrict__ order, const BatchDesc* __restrict__ desc, unsigned long long* ex,
                uint32_t n_echo) {
  __shared__ uint16_t s_stk[64 * kBvhStack];
  unsigned long long* e = EX ? ex : nullptr;
  const BatchDesc* dsc = ART_VIS_DESC ? desc : nullptr;  // off: the descriptor branch compiles out
  if (blockIdx.x < n_echo) vis_quad_body(sc, vp, count, order, e, blockIdx.x, s_stk);
  else vis_sweep_body(sc, vp, count, nb_max, order, dsc, e, n_echo, blockIdx.x - n_echo, TWO);
}

// Outputs of the visibility pairs once every range has run (the kernel boundary makes the verdicts
// visible): visible echoes are stored, visible muffle rays counted.
__global__ __launch_bounds__(256) void vis_finalize(VisPairs vp, const uint32_t* __restrict__ count,
                                                    uint8_t* __restrict__ block, uint32_t* __restrict__ muffle_acc) {
  const int lane = threadIdx.x & 63;
  const uint32_t p = blockIdx.x * 256u + threadIdx.x, wbase = __builtin_amdgcn_readfirstlane(p - lane);
  const bool echo_region = wbase < vp.echo_cap;  // echo_cap is a multiple of 64: one region per wave
  const uint32_t n = echo_region ? ldc(count, 0) : ldc(count, 1), rel = echo_region ? p : p - vp.echo_cap;
  if (__builtin_amdgcn_readfirstlane(rel - lane) >= n) return;
  const bool valid = rel < n;
  uint32_t flag = 1u, dest = 0u, val = 0u;
  if (valid) { flag = vp.flag[p]; const uint2 o = vp.out[p]; dest = o.x; val = o.y; }
  const bool vis = valid && flag == 0u;
  const bool muf = (val & kPairMuffle) != 0;
  if (vis && !muf) reinterpret_cast<uint16_t*>(block)[dest] = (uint16_t)(val & 0xffffu);  // :142-144
  // muffle counts (:171): one atomic per distinct counter of the wave (its pairs come from one or
  // two (fan, target) groups of the emission order)
  unsigned long long mv = __ballot(vis && muf);
  while (mv) {
    const uint32_t d0 = __builtin_amdgcn_readlane(dest, __builtin_ctzll(mv));
    const unsigned long long eq = __ballot(vis && muf && dest == d0);
    if (lane == 0) atomicAdd(&muffle_acc[d0], (uint32_t)__popcll(eq));
    mv &= ~eq;
  }
}

__device__ __forceinline__ float echo_of(const DevScene& sc, int type, int idx) {
  return type == kSphere ? sc.sphc[idx].echo : (type == kAabb ? sc.aabbc[idx].echo : sc.obbc[idx].echo);
}

// Occupancy target (amdgpu_waves_per_eu) and sweep unroll per scene kind, chosen by measurement on
// MI355X: scenes without OBBs (config 2) run best at 6 waves/SIMD with 8 records per scalar-load
// group (more loads in flight per s_waitcnt); OBB scenes (configs 3-5) at 7 waves/SIMD, unroll 4.
#ifndef ART_FAST_BVH
#define ART_FAST_BVH 1  // nearest hits by per-lane BVH traversal (nearest_bvh) when the scene has a BVH
#endif
#ifndef ART_FAST_WPE_BVH
#define ART_FAST_WPE_BVH 4  // 122 VGPRs, no scratch (8: 82 VGPR spills)
#endif
#ifndef ART_FAST_WPE_NO_OBB
#define ART_FAST_WPE_NO_OBB 6
#endif
#ifndef ART_FAST_U_NO_OBB
#define ART_FAST_U_NO_OBB 8
#endif
#ifndef ART_FAST_WPE_OBB
#define ART_FAST_WPE_OBB 7
#endif
#ifndef ART_FAST_U_OBB
#define ART_FAST_U_OBB 4
#endif

// MULTI = false: frames with one hit per ray (H == 1, configs 2-4) compile without the later-bounce
// nearest sweep and the reflection, which removes their registers from the kernel.
#ifndef ART_FAST_AGG_RESERVE
#define ART_FAST_AGG_RESERVE 1
#endif
template <int K, bool HITS, int U, int WPE, bool MULTI, bool BVH, bool QUAD, bool PRE, bool STEP>
__global__ __launch_bounds__(64 * K) __attribute__((amdgpu_waves_per_eu(WPE))) void raytrace_fast_kernel(DevScene sc, FrameParams fp, FanLayout L,
                                                               const float* __restrict__ origins,
                                                               uint8_t* __restrict__ block,
                                                               uint32_t* __restrict__ muffle_acc,
                                                               const int* __restrict__ ray_order,
                                                               uint32_t* __restrict__ work,
                                                               VisPairs vp,
                                                               uint32_t* __restrict__ pair_count,
                                                               uint16_t* __restrict__ pkeys,
                                                               const int2* __restrict__ pre_hits,
                                                               float4* __restrict__ state, int step) {
  // STEP (multi-hit frames, PRE): one bounce per launch; the ray state (o, life | d, hits, alive)
  // carries over in `state` between the launches of the frame.
  // PRE (independent waves): the first segment's nearest hits come from nearest_first_kernel.
  // BVH: the K waves of a workgroup are independent (each pulls its own 64-ray groups and owns
  // their writes); they share the workgroup's LDS copy of the top BVH nodes.
  // QUAD: the K = 4 waves hold the same 64 rays and split the nearest-hit traversal 16 rays each
  // (nearest_bvh_quad); results meet in LDS as the K-way split's partials do.
  constexpr bool IND = BVH && !QUAD;
  // AGG: the K waves of a workgroup reserve their pair positions with one atomic per counter for
  // the whole workgroup (one wave per group: 4096 same-line atomics serialize to ~46 us at config
  // 2); the waves step through their groups together (block-uniform loop and bounce count).
  constexpr bool AGG = IND && (!MULTI || STEP) && ART_FAST_AGG_RESERVE;
  constexpr bool ONCE = AGG || STEP;  // one bounce per group (block-uniform)
  __shared__ uint32_t s_agg[AGG ? 2 : 1][AGG ? K : 1][2];
  __shared__ uint32_t s_aggb[2][2];
  __shared__ uint32_t s_live[AGG && STEP ? 2 : 1][AGG && STEP ? K : 1], s_liveb[2];
  (void)s_live; (void)s_liveb;
  (void)s_agg; (void)s_aggb;
  int it = 0;  // block-uniform group iteration (AGG buffers alternate by its parity)
  __shared__ float s_dist[K][64];
  __shared__ float s_best[K][64];  // running per-lane best of each wave (front-to-back pruning)
  (void)s_best;
  __shared__ int s_chead;  // next nearest-hit chunk of the block (dynamic cone sweep)
  __shared__ int s_code[K][64];
  __shared__ short s_pairof[kMaxQueries][64];
  __shared__ uint8_t s_res[kMaxQueries * 64];
  __shared__ int s_head, s_np;
  __shared__ uint32_t s_muf[kMaxTargets];
  __shared__ int s_ticket[IND ? K : 1];
  __shared__ int s_go[3];  // staged visibility only
  __shared__ uint16_t s_stk[QUAD ? kBvhStack * 64 : (BVH ? kBvhStack * 64 * K : 1)];  // BVH traversal stacks
  (void)s_stk;
  (void)s_go; (void)s_pairof; (void)s_res; (void)s_head; (void)s_np;
#ifdef ART_TEST_NO_OBB
  sc.no = 0;
#endif
  extern __shared__ PairSeg s_seg[];  // [64 * (T + 1)], then (staged visibility) 2 chunk buffers
  uint8_t* s_stage = reinterpret_cast<uint8_t*>(s_seg + 64 * (fp.T + 1));
  (void)s_stage;
  // wave index as an SGPR value: chunk bounds and loop counters of the sweeps stay scalar
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const bool lead = IND || w == 0;  // the wave that owns the group's global writes
  const int nrb = (fp.R + 63) >> 6;  // 64-ray groups per fan
  const int ngroups = fp.S * nrb;
  // BVH: the top bvh_lds_nodes(...) nodes in LDS (dynamic shared memory, BVH mode only)
  const CullRec* s_nodes = reinterpret_cast<const CullRec*>(s_seg);
  constexpr bool NODES = IND && (!PRE || (MULTI && !STEP));  // later bounces traverse per lane
  (void)state; (void)step;
  const int nl = NODES ? bvh_lds_nodes(sc) : 0;
  (void)s_nodes; (void)nl; (void)pre_hits;
  if (NODES) {
    CullRec* dst = reinterpret_cast<CullRec*>(s_seg);
    for (int i = threadIdx.x; i < nl; i += blockDim.x) dst[i] = sc.bvh[i];
    __syncthreads();
  }
  // Persistent grid: the launch holds as many workgroups as are co-resident, and each pulls
  // 64-ray groups from a global ticket counter until the frame is drained (no partial last
  // round of workgroups, and uneven visibility work balances itself).
  // BVH (independent waves): a static grid-stride assignment of groups to waves (a ticket per wave
  // would serialize on one counter: about 88 dequeues per microsecond).
  int gnext = IND ? (int)blockIdx.x * K + w : (int)blockIdx.x;
  for (;;) {
  int g;
  if (IND) {
    g = gnext;
    gnext += (int)gridDim.x * K;
    ++it;
  } else if (QUAD) {  // static assignment, one group per workgroup
    __syncthreads();  // the previous group's LDS reads are done
    g = gnext;
    gnext += (int)gridDim.x;
  } else {
    __syncthreads();  // the previous group's LDS reads are done
    if (threadIdx.x == 0) s_ticket[0] = (int)atomicAdd(&work[0], 1u);
    __syncthreads();
    g = __builtin_amdgcn_readfirstlane(s_ticket[0]);
  }
  if (AGG ? g - w >= ngroups : g >= ngroups) break;
  const bool gvalid = !AGG || g < ngroups;  // AGG: a wave past the end takes part with no rays
  const int fan = gvalid ? g / nrb : 0;
  const int slot = gvalid ? (g - fan * nrb) * 64 + lane : fp.R;
  const bool valid = slot < fp.R;
  const int ray = valid ? ray_order[slot] : 0;
  const int T = fp.T, H = MULTI ? fp.H : 1;
  if (!IND)
    for (int t = threadIdx.x; t < T; t += blockDim.x) s_muf[t] = 0;

  uint8_t* fb = block + (size_t)fan * L.stride;
  uint16_t* echo = reinterpret_cast<uint16_t*>(fb + L.echo_off);
  art_half3* hpo = reinterpret_cast<art_half3*>(fb + L.hit_points_off);
  const bool single_slot = fp.TC == 1;
  const int my_slot = (int)(((long long)((ray / fp.bs) * fp.bs) * fp.TC) / fp.R);  // batchId (:63-64)

  // Reset (:72-80) with sequential-batch semantics; wave 0 owns every global write.
  uint32_t frozen = 0;
  if (valid) {
    const int my_batch = ray / fp.bs;
    const art_half3 z = {0, 0, 0};
    for (int k = 0; k < H; ++k) {
      const int j = ray * H + k;
      bool any_reset;
      const int keep = batch_slot_state(fp, j, my_batch, any_reset);
      if (!keep) frozen |= 1u << k;
      if (lead && !single_slot && (!keep || any_reset) && (!STEP || step == 0)) {  // TC == 1: every slot is written once below
        echo[j] = 0;
        if (HITS) hpo[j] = z;
      }
    }
  }
  if (!IND) {
    if (threadIdx.x == 0) s_chead = 0;
    __syncthreads();
  }

  const vec3 O = load3(origins, fan);
  vec3 o = O;
  vec3 d = load_dir(sc.dirs, valid ? ray : 0);
  float life = fp.max_life;
  int hits = 0;
  bool alive = valid;
  const size_t sidx = (size_t)g * 64 + lane;  // ray slot of the state / pre-hit arrays
  if (STEP && step > 0 && valid) {
    const float4 a = state[2 * sidx], b = state[2 * sidx + 1];
    o = mk3(a.x, a.y, a.z);
    life = a.w;
    d = mk3(b.x, b.y, b.z);
    hits = __float_as_int(b.w) & 0xff;
    alive = ((__float_as_int(b.w) >> 8) & 1) != 0;
  }
  const bool alive0 = alive;
  (void)alive0;

  const int b0 = STEP ? step : 0;
  int bounce = b0;  // wave-uniform (lanes that stopped keep their own `hits`)
  while (ONCE ? bounce == b0 : __any(alive)) {  // identical in every wave of the block -> uniform barriers
    const Seg s = make_seg(o, d);
    float best;
    int code;
#if ART_FAST_CULL
    if (BVH && QUAD) {
#ifdef ART_DIAG_NO_NEAREST  // diagnostic build only: every live ray hits sphere 0 at distance 1
      if (w == 0) { s_dist[0][lane] = alive ? 1.0f : FLT_MAX; s_code[0][lane] = alive ? 0 : kNoHit; }
#else
      nearest_bvh_quad(sc, s, alive, w, lane, s_stk, &s_dist[0][0], &s_code[0][0], fp.exec);
#endif
      best = FLT_MAX;
      code = kNoHit;
    } else if (BVH) {
#ifdef ART_DIAG_NO_NEAREST  // diagnostic build only: every live ray hits sphere 0 at distance 1
      best = alive ? 1.0f : FLT_MAX; code = alive ? 0 : kNoHit;
#else
      if (PRE && (STEP || bounce == 0)) {
        const int2 h = gvalid ? pre_hits[sidx] : make_int2(__float_as_int(FLT_MAX), kNoHit);
        best = __int_as_float(h.x);
        code = h.y;
      } else if (!PRE || MULTI) {
        nearest_bvh(sc, s, alive, s_nodes, nl, s_stk + w * (kBvhStack * 64), lane, best, code, fp.exec);
      } else {  // not reached: PRE one-hit frames have one segment
        best = FLT_MAX;
        code = kNoHit;
      }
#endif
    } else if (!MULTI || bounce == 0) {  // first segment: every ray of the fan starts at O
      const WaveCone wc = make_cone(O, d, alive);
#if ART_FAST_SORTED_NEAREST
      nearest_sorted<K>(sc, s, wc, w, lane, alive, s_best, best, code, fp.exec);
#else
      nearest_cone<U>(sc, s, wc, w, K, lane, best, code, fp.exec, &s_chead);
#endif
    } else if (MULTI) {
      nearest_chunk<U>(sc, s, w, K, best, code);
      exec_brute(sc, w, K, fp.exec);
    }
#else
    nearest_chunk<U>(sc, s, w, K, best, code);
    exec_brute(sc, w, K, fp.exec);
#endif
    float bd = best;
    int bc = code;
    if (QUAD) {
      __syncthreads();
      // one bounce: waves 1-3 were only needed for the traversal; wave 0 owns the rest
      if (!MULTI && w != 0) break;
      bd = s_dist[0][lane];
      bc = s_code[0][lane];
    } else if (!IND) {
      s_dist[w][lane] = best;
      s_code[w][lane] = code;
      __syncthreads();
      bd = s_dist[0][lane];
      bc = s_code[0][lane];
#pragma unroll
      for (int k = 1; k < K; ++k) {
        const float dk = s_dist[k][lane];
        const int ck = s_code[k][lane];
        if (dk < bd || (dk == bd && ck < bc)) { bd = dk; bc = ck; }
      }
    }
    const bool hit = alive && bc != kNoHit;
    alive = hit;  // a miss ends the ray (:200-207)
    int type = kNone, idx = 0;
    float dist = bd;
    if (hit) {
      const int rank = bc >> 28;
      idx = bc & 0x0fffffff;
      type = rank == 0 ? kSphere : (rank == 1 ? kAabb : kObb);
      // exact (Unity min/max) re-evaluation: a zero distance keeps the reference's sign
      if (type == kAabb) aabb_test<true>(s, sc.aabb[idx], dist);
      if (type == kObb) { const ObbRec r = sc.obb[idx]; obb_test<true>(s, r, stored_q(r), dist); }
      o = o + d * dist;  // :111
      life -= dist;      // :112
      hits += 1;         // :113
    }
    const int k = hits - 1;
    const bool live_slot = hit && !((frozen >> k) & 1u);
    if (HITS && lead && live_slot) {  // :118, :197
      art_half3 p;
      p.x = f32tof16(o.x); p.y = f32tof16(o.y); p.z = f32tof16(o.z);
      hpo[ray * H + k] = p;
    }

    // visibility pairs: q = 0 echo ray to the origin (:124-145), q = 1..T muffle rays (:150-173)
    const vec3 off = o - d * kEps;                 // :124, :158
    const float dist0 = distance(O, o);            // :130 (un-offset hit point)
#if ART_FAST_SPLIT
    // Emit the pairs with their output destinations for vis_kernel (wave 0 owns the group's rays).
    if (lead) {
      const unsigned long long lt = (1ull << lane) - 1ull;
      unsigned long long mq[kMaxQueries];
      uint32_t actbits = 0;
      uint32_t np = 0;
#pragma unroll
      for (int q = 0; q < kMaxQueries; ++q) {
        bool act = false;
        if (q <= T) {
          if (q == 0) act = live_slot;  // the echo is written only into a live slot (:118)
          else act = hit && distance(off, load3(sc.targets, q - 1)) < fp.max_muffle;  // :165-168
        }
        mq[q] = __ballot(act);
        actbits |= act ? (1u << q) : 0u;
        np += (uint32_t)__popcll(mq[q]);
      }
#ifdef ART_DIAG_NO_EMIT  // diagnostic build only: time the path without the pair emission
      np = 0;
#endif
      // echo pairs to the echo region, muffle pairs to the muffle region (one reservation each)
      const uint32_t ne = (uint32_t)__popcll(mq[0]), nm = np - ne;
      uint32_t eb = 0, mb = 0;
      if (AGG) {  // every wave of the workgroup is here (block-uniform loop, one bounce)
        const int par = it & 1;
        if (lane == 0) { s_agg[par][w][0] = ne; s_agg[par][w][1] = nm; }
        __syncthreads();
        if (threadIdx.x < 2) {
          uint32_t t = 0;
#pragma unroll
          for (int k = 0; k < K; ++k) t += s_agg[par][k][threadIdx.x];
          s_aggb[par][threadIdx.x] = t ? atomicAdd(&pair_count[threadIdx.x], t) : 0u;
        }
        __syncthreads();
        eb = s_aggb[par][0];
        mb = s_aggb[par][1];
        for (int k = 0; k < w; ++k) { eb += s_agg[par][k][0]; mb += s_agg[par][k][1]; }
      }
      if (np) {
#ifdef ART_DIAG_NO_PAIR_ATOMICS  // diagnostic build only (H = 1 timing): fixed per-group positions
        eb = (uint32_t)g * 64u; mb = (uint32_t)g * 64u * (uint32_t)T;
#else
        if (!AGG && lane == 0) {
          if (ne) eb = atomicAdd(&pair_count[0], ne);
          if (nm) mb = atomicAdd(&pair_count[1], nm);
        }
#endif
        eb = __builtin_amdgcn_readfirstlane(__shfl(eb, 0, 64));
        mb = __builtin_amdgcn_readfirstlane(__shfl(mb, 0, 64));
        uint32_t pos = mb;  // muffle position (region-relative)
#pragma unroll
        for (int q = 0; q < kMaxQueries; ++q) {
          if (q <= T && ((actbits >> q) & 1u)) {
            vec3 qdir;
            float maxd;
            int owner;
            uint2 ov;
            if (q == 0) {
              qdir = normalize(O - off); maxd = dist0; owner = kNoOwner;
              ov.x = (uint32_t)(((size_t)fan * L.stride + L.echo_off) / 2) + (uint32_t)(ray * H + k);
              ov.y = f32tof16(dist0 * echo_of(sc, type, idx));  // :142-144
            } else {
              const vec3 tp = load3(sc.targets, q - 1);
              maxd = distance(off, tp);
              qdir = normalize(tp - off);
              owner = q - 1;                                      // :413, :426, :439
              ov.x = (uint32_t)(((size_t)fan * fp.TC + my_slot) * T + (q - 1));
              ov.y = kPairMuffle;
            }
            const uint32_t rank = (uint32_t)__popcll(mq[q] & lt);
            const uint32_t at = q == 0 ? eb + rank : vp.echo_cap + pos + rank;
            vp.seg[2 * (size_t)at] = make_float4(off.x, off.y, off.z, maxd);
            vp.seg[2 * (size_t)at + 1] = make_float4(qdir.x, qdir.y, qdir.z, __int_as_float(owner));
            vp.out[at] = ov;
            vp.flag[at] = 0u;
            if (q > 0 && pkeys) pkeys[pos + rank] = vis_sort_key(q - 1, mk3(-qdir.x, -qdir.y, -qdir.z));
          }
          if (q > 0 && q <= T) pos += (uint32_t)__popcll(mq[q]);
        }
      }
      // a blocked echo leaves the reset value (:76); vis_kernel overwrites the visible ones
      if (live_slot && single_slot) echo[ray * H + k] = 0;
    }
#else
    if (w == 0) {
      const unsigned long long lt = (1ull << lane) - 1ull;
      int np = 0;
      for (int q = 0; q <= T; ++q) {
        vec3 qdir;
        float maxd;
        bool act;
        int owner;
        if (q == 0) {
          qdir = normalize(O - off); maxd = dist0; act = hit; owner = kNoOwner;
        } else {
          const vec3 tp = load3(sc.targets, q - 1);
          maxd = distance(off, tp);                 // :165
          act = hit && maxd < fp.max_muffle;        // :168
          qdir = normalize(tp - off);
          owner = q - 1;                            // :413, :426, :439
        }
        const unsigned long long m = __ballot(act);
        const int pos = np + __popcll(m & lt);
        if (act) {
          const Seg g = make_seg(off, qdir);
          PairSeg r;
          r.ox = g.o.x; r.oy = g.o.y; r.oz = g.o.z; r.dx = g.d.x; r.dy = g.d.y; r.dz = g.d.z;
          r.ix = g.inv.x; r.iy = g.inv.y; r.iz = g.inv.z; r.a2 = g.a2; r.maxd = maxd;
          r.owner = owner;
          s_seg[pos] = r;
        }
        s_pairof[q][lane] = act ? (short)pos : (short)-1;
        np += __popcll(m);
      }
      if (lane == 0) { s_np = np; s_head = 0; }
    }
    __syncthreads();
#ifdef ART_DIAG_NO_VISIBILITY  // diagnostic build only: time the nearest-hit phase alone
    for (int p = w * 64 + lane; p < s_np; p += K * 64) s_res[p] = 0;
#elif ART_FAST_CULL
    visibility_culled<U>(sc, s_seg, s_res, &s_head, s_np, lane, fp.exec);
#elif ART_FAST_STAGED
    visibility_staged<U>(sc, s_seg, s_res, &s_head, s_go, s_stage, s_np, w, K, lane);
#else
    visibility_queue<U>(sc, s_seg, s_res, &s_head, s_np, w, K, lane);
#endif
    __syncthreads();
    if (w == 0) {
      const int pe = s_pairof[0][lane];
      if (hit && live_slot) {
        if (pe >= 0 && !s_res[pe]) echo[ray * H + k] = f32tof16(dist0 * echo_of(sc, type, idx));  // :142-144
        else if (single_slot) echo[ray * H + k] = 0;  // reset value (:76), written once
      }
      for (int t = 0; t < T; ++t) {
        const int p = s_pairof[t + 1][lane];
        if (p >= 0 && !s_res[p]) {  // :171
          if (single_slot) atomicAdd(&s_muf[t], 1u);
          else atomicAdd(&muffle_acc[((size_t)fan * fp.TC + my_slot) * T + t], 1u);
        }
      }
    }

#endif

    // termination / reflection — :179-193, ReflectRay :456-532 (every wave, identical state)
    if (!MULTI) {
      alive = false;  // hits >= H == 1 after the first hit; a miss has already ended the ray
    } else if (hit) {
      if (hits >= H || life <= 0.0f) {
        alive = false;
      } else {
        vec3 n = mk3(0.0f, 0.0f, 0.0f);
        float absorption = 0.0f;
        if (type == kAabb) {
          const AabbCold b = sc.aabbc[idx];
          vec3 lp = o - mk3(b.cx, b.cy, b.cz);
          vec3 ap = abs3(lp);
          float dx = b.hx - ap.x, dy = b.hy - ap.y, dz = b.hz - ap.z;
          if (dx < dy && dx < dz) n.x = usign(lp.x);
          else if (dy < dx && dy < dz) n.y = usign(lp.y);
          else n.z = usign(lp.z);
          absorption = b.absorption;
        } else if (type == kObb) {
          const ObbRec b = sc.obb[idx];
          const ObbCold bc = sc.obbc[idx];
          vec3 lh = qmul(inverse_q(bc), o - mk3(b.cx, b.cy, b.cz));
          vec3 ap = abs3(lh);
          vec3 df = mk3(bc.hx, bc.hy, bc.hz) - ap;
          vec3 ln = mk3(0.0f, 0.0f, 0.0f);
          if (df.x < df.y && df.x < df.z) ln.x = usign(lh.x);
          else if (df.y < df.x && df.y < df.z) ln.y = usign(lh.y);
          else ln.z = usign(lh.z);
          n = qmul(stored_q(b), ln);
          absorption = bc.absorption;
        } else {
          const SphereRec c = sc.sph[idx];
          n = normalize(o - mk3(c.cx, c.cy, c.cz));
          absorption = sc.sphc[idx].absorption;
        }
        d = reflect(d, n);
        o = o + d * kEps;
        life -= fp.max_life * absorption;
        if (life < 0.0f) alive = false;
      }
    }
    ++bounce;
  }
  if (STEP && valid) {  // the next launch's ray state (a ray that stopped records alive = 0)
    state[2 * sidx] = make_float4(o.x, o.y, o.z, life);
    state[2 * sidx + 1] = make_float4(d.x, d.y, d.z, __int_as_float(hits | (alive ? 256 : 0)));
  }
  if (STEP && ART_FAST_COMPACT) {  // the rays still alive: the next bounce's traversal list
    uint32_t* live = reinterpret_cast<uint32_t*>(state + 2 * (size_t)ngroups * 64);
    uint32_t* live_n = live + (size_t)ngroups * 64;
    const bool app = valid && alive && step + 1 < fp.H;
    const unsigned long long m = __ballot(app);
    uint32_t base = 0;
    if (AGG) {  // every wave of the workgroup is here (one bounce per launch)
      const int par = it & 1;
      if (lane == 0) s_live[par][w] = (uint32_t)__popcll(m);
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) t += s_live[par][k];
        s_liveb[par] = t ? atomicAdd(&live_n[step + 1], t) : 0u;
      }
      __syncthreads();
      base = s_liveb[par];
      for (int k = 0; k < w; ++k) base += s_live[par][k];
    } else {
      if (lane == 0 && m) base = atomicAdd(&live_n[step + 1], (uint32_t)__popcll(m));
      base = __builtin_amdgcn_readfirstlane(__shfl(base, 0, 64));
    }
    if (app) live[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)sidx;
  }
  if (valid && lead && (!STEP || (alive0 && !alive))) {  // STEP: in the launch where the ray stops
    if (single_slot) {  // slots past the last hit keep the reset value 0 (:72-80)
      const art_half3 z = {0, 0, 0};
      for (int k = hits; k < H; ++k) {
        echo[ray * H + k] = 0;
        if (HITS) hpo[ray * H + k] = z;
      }
    }
    if (HITS) fb[L.hit_counts_off + ray] = (uint8_t)hits;  // :204, :212
  }
  if (!IND) {  // muffle counts of the fused visibility (the split path counts in vis_finalize)
    __syncthreads();
    if (single_slot)
      for (int t = threadIdx.x; t < T; t += blockDim.x)
        if (s_muf[t]) atomicAdd(&muffle_acc[(size_t)fan * T + t], s_muf[t]);
  }
  }
  // Every workgroup has drawn its final (out-of-range) ticket before it arrives here, so the last
  // arrival can rearm the counter for the next launch on this stream.
  if (!BVH && threadIdx.x == 0 && atomicAdd(&work[1], 1u) == gridDim.x - 1) {
    atomicExch(&work[0], 0u);
    atomicExch(&work[1], 0u);
#ifdef ART_DIAG_CULL_STATS
    printf("[cull] batches %u pairs %u chunks %u candidates %u | nearest colliders %u candidates %u\n",
           atomicExch(&g_diag[0], 0u), atomicExch(&g_diag[3], 0u), atomicExch(&g_diag[1], 0u), atomicExch(&g_diag[2], 0u),
           atomicExch(&g_diag[4], 0u), atomicExch(&g_diag[5], 0u));
#endif
  }
}

int fast_max_targets() { return kMaxQueries - 1; }

// Waves per 64-ray group. K = 8 measured best on every config once the visibility moved to its own
// kernel (config 2: 0.79 ms vs 0.83 at K = 4 and 0.90 at K = 16; config 4: 16.4 ms vs 20.3 at
// the K = 1 the old occupancy rule picked).
int fast_split(int S, int R) {
  (void)S; (void)R;
#ifdef ART_FAST_FORCE_K
  return ART_FAST_FORCE_K;
#endif
  return 8;
}

static size_t fast_lds_bytes(const DevScene& sc, int T) {
  if (ART_FAST_SPLIT) return 0;
  return sizeof(PairSeg) * 64 * (size_t)(T + 1) + (ART_FAST_STAGED ? 2 * (size_t)stage_stride(sc) : 0);
}

// Co-resident workgroups of one kernel instance on the current device, cached per (device,
// kernel, dynamic LDS bytes).
template <typename Kern>
static int resident_blocks(Kern kern, int threads, size_t lds) {
  struct Entry { int dev; const void* fn; size_t lds; int blocks; };
  static thread_local std::vector<Entry> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const void* fn = reinterpret_cast<const void*>(kern);
  for (const Entry& e : cache)
    if (e.dev == dev && e.fn == fn && e.lds == lds) return e.blocks;
  int cus = 0, per_cu = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess) per_cu = 0;
  const int blocks = std::max(1, per_cu) * std::max(1, cus);
  cache.push_back({dev, fn, lds, blocks});
  return blocks;
}

template <int K, bool HITS, int U, int WPE, bool MULTI, bool BVH, bool QUAD = false, bool PRE = false, bool STEP = false>
static void launch_fast_kh(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                           uint8_t* block, uint32_t* muffle_acc, const int* ray_order, uint32_t* work, const VisPairs& pairs,
                           uint32_t* pair_count, uint16_t* pkeys, hipStream_t st, const int2* pre = nullptr,
                           float4* state = nullptr, int step = 0) {
  const size_t lds = QUAD || (PRE && (!MULTI || STEP)) ? 0
                     : (BVH ? (size_t)bvh_lds_nodes(sc) * sizeof(CullRec) : fast_lds_bytes(sc, fp.T));
  const long long groups = (long long)fp.S * ((fp.R + 63) / 64);
  // BVH: K independent waves per workgroup, one group each (grid-stride past 2^31 / K groups);
  // quad BVH: one group per workgroup; otherwise a persistent grid of co-resident workgroups
  // pulling groups from a ticket counter
  const int nblk = QUAD ? (int)std::min<long long>(groups, 1ll << 30)
                 : BVH  ? (int)std::min<long long>((groups + K - 1) / K, 1ll << 30)
                        : (int)std::min<long long>(groups, resident_blocks(raytrace_fast_kernel<K, HITS, U, WPE, MULTI, BVH, QUAD, PRE, STEP>,
                                                                            64 * K, lds));
  hipLaunchKernelGGL((raytrace_fast_kernel<K, HITS, U, WPE, MULTI, BVH, QUAD, PRE, STEP>), dim3(nblk), dim3(64 * K), lds, st, sc, fp,
                     L, origins, block, muffle_acc, ray_order, work, pairs, pair_count, pkeys, pre, state, step);
}

template <int K>
static void launch_fast_k(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                          uint8_t* block, uint32_t* muffle_acc, const int* ray_order, uint32_t* work, const VisPairs& pairs,
                          uint32_t* pair_count, uint16_t* pkeys, hipStream_t st) {
  // instantiation by scene kind (OBBs or not), hit outputs, and one or several hits per ray
#define ART_LAUNCH(H_, U_, W_, M_) \
  launch_fast_kh<K, H_, U_, W_, M_, false>(sc, fp, L, origins, block, muffle_acc, ray_order, work, pairs, pair_count, \
                                           pkeys, st)
  const bool multi = fp.H > 1;
  if (sc.no > 0) {
    if (L.has_hits) { if (multi) ART_LAUNCH(true, ART_FAST_U_OBB, ART_FAST_WPE_OBB, true); else ART_LAUNCH(true, ART_FAST_U_OBB, ART_FAST_WPE_OBB, false); }
    else { if (multi) ART_LAUNCH(false, ART_FAST_U_OBB, ART_FAST_WPE_OBB, true); else ART_LAUNCH(false, ART_FAST_U_OBB, ART_FAST_WPE_OBB, false); }
  } else {
    if (L.has_hits) { if (multi) ART_LAUNCH(true, ART_FAST_U_NO_OBB, ART_FAST_WPE_NO_OBB, true); else ART_LAUNCH(true, ART_FAST_U_NO_OBB, ART_FAST_WPE_NO_OBB, false); }
    else { if (multi) ART_LAUNCH(false, ART_FAST_U_NO_OBB, ART_FAST_WPE_NO_OBB, true); else ART_LAUNCH(false, ART_FAST_U_NO_OBB, ART_FAST_WPE_NO_OBB, false); }
  }
#undef ART_LAUNCH
}

static_assert(!ART_FAST_BVH || ART_FAST_SPLIT, "the BVH path kernel emits visibility pairs (split visibility)");
#ifndef ART_FAST_BVH_WAVES
#define ART_FAST_BVH_WAVES 8  // independent waves per workgroup sharing the LDS node cache
#endif

#ifndef ART_FAST_WPE_QUAD
#define ART_FAST_WPE_QUAD 4
#endif
#ifndef ART_FAST_QUAD_GROUPS
#define ART_FAST_QUAD_GROUPS 8192  // quad traversal up to this many 64-ray groups per launch (config 2/3/5:
                                   // 2048 groups, quad 16 / 10 / 1 % faster; config 4: 16384, lanes 3 % faster)
#endif
static bool bvh_quad(const FrameParams& fp) {
  return (long long)fp.S * ((fp.R + 63) / 64) <= (long long)ART_FAST_QUAD_GROUPS;
}
#ifndef ART_FAST_PRE_NEAREST
#define ART_FAST_PRE_NEAREST 1  // 1: one-hit frames take the first segment from nearest_first_kernel
#endif                          // (any size: config 4 5.58 -> 4.74 ms); 2: multi-hit quad frames too
#ifndef ART_FAST_STEP_MULTI
#define ART_FAST_STEP_MULTI 1  // multi-hit frames: one first-segment + path launch pair per bounce
#endif
static bool bvh_step(const FrameParams& fp) {
  return ART_FAST_PRE_NEAREST && ART_FAST_STEP_MULTI && fp.H > 1 && fp.H <= kLiveCounters;
}
static bool bvh_pre(const FrameParams& fp) {
  const long long groups = (long long)fp.S * ((fp.R + 63) / 64);
  return ART_FAST_PRE_NEAREST && groups < (1ll << 30) &&
         (fp.H == 1 || bvh_step(fp) || (ART_FAST_PRE_NEAREST > 1 && bvh_quad(fp)));
}

// BVH path kernel: one wave per 64-ray group (no collider split), per-lane traversal; or (quad)
// 4 waves per group, 4 lanes per ray; or (pre) the quad first-segment launch, then the path
// kernel's independent waves from its hits.
static void launch_fast_bvh(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                            uint8_t* block, uint32_t* muffle_acc, const int* ray_order, uint32_t* work, const VisPairs& pairs,
                            uint32_t* pair_count, uint16_t* pkeys, int2* pre, float4* state, hipStream_t st) {
#define ART_LAUNCH_P(H_, M_) \
  launch_fast_kh<ART_FAST_BVH_WAVES, H_, 1, ART_FAST_WPE_BVH, M_, true, false, true>(sc, fp, L, origins, block, muffle_acc, \
                                                                                     ray_order, work, pairs, pair_count, pkeys, \
                                                                                     st, pre)
  const bool multi_ = fp.H > 1;
  if (pre && bvh_pre(fp)) {
    const long long groups = (long long)fp.S * ((fp.R + 63) / 64);  // < 2^30
    auto first = [&](int step) {
      if (fp.exec)
        hipLaunchKernelGGL(nearest_first_kernel<true>, dim3((unsigned)groups), dim3(256), 0, st, sc, fp, origins, ray_order, pre,
                           state, step);
      else
        hipLaunchKernelGGL(nearest_first_kernel<false>, dim3((unsigned)groups), dim3(256), 0, st, sc, fp, origins, ray_order, pre,
                           state, step);
    };
    if (state && bvh_step(fp)) {  // one launch pair per bounce; all rays stop by bounce H - 1
      for (int k = 0; k < fp.H; ++k) {
        first(k);
        if (L.has_hits)
          launch_fast_kh<ART_FAST_BVH_WAVES, true, 1, ART_FAST_WPE_BVH, true, true, false, true, true>(
              sc, fp, L, origins, block, muffle_acc, ray_order, work, pairs, pair_count, pkeys, st, pre, state, k);
        else
          launch_fast_kh<ART_FAST_BVH_WAVES, false, 1, ART_FAST_WPE_BVH, true, true, false, true, true>(
              sc, fp, L, origins, block, muffle_acc, ray_order, work, pairs, pair_count, pkeys, st, pre, state, k);
      }
      return;
    }
    first(0);
    if (L.has_hits) { if (multi_) ART_LAUNCH_P(true, true); else ART_LAUNCH_P(true, false); }
    else { if (multi_) ART_LAUNCH_P(false, true); else ART_LAUNCH_P(false, false); }
    return;
  }
#undef ART_LAUNCH_P
#define ART_LAUNCH(H_, M_) \
  launch_fast_kh<ART_FAST_BVH_WAVES, H_, 1, ART_FAST_WPE_BVH, M_, true>(sc, fp, L, origins, block, muffle_acc, ray_order, \
                                                                        work, pairs, pair_count, pkeys, st)
#define ART_LAUNCH_Q(H_, M_) \
  launch_fast_kh<4, H_, 1, ART_FAST_WPE_QUAD, M_, true, true>(sc, fp, L, origins, block, muffle_acc, ray_order, work, pairs, \
                                                              pair_count, pkeys, st)
  const bool multi = fp.H > 1;
  if (bvh_quad(fp)) {
    if (L.has_hits) { if (multi) ART_LAUNCH_Q(true, true); else ART_LAUNCH_Q(true, false); }
    else { if (multi) ART_LAUNCH_Q(false, true); else ART_LAUNCH_Q(false, false); }
  } else {
    if (L.has_hits) { if (multi) ART_LAUNCH(true, true); else ART_LAUNCH(true, false); }
    else { if (multi) ART_LAUNCH(false, true); else ART_LAUNCH(false, false); }
  }
#undef ART_LAUNCH_Q
#undef ART_LAUNCH
}

bool fast_uses_bvh() { return ART_FAST_BVH != 0; }

bool fast_uses_sorted_scene() {
  return ART_FAST_TWO_LEVEL || ART_FAST_SORTED_NEAREST || (ART_FAST_SPLIT && ART_VIS_TWO_LEVEL) || ART_FAST_BVH;
}

// Counting sort of the muffle pairs by key (T << kSortDirBits buckets; the order inside a bucket
// is free: the any-hit verdicts do not depend on it). Block j of kSortBlock pairs: LDS histogram
// -> row j of hist[block][bucket]; a column prefix per bucket and the buckets' totals; each
// scatter block scans the totals and hands out positions with LDS atomics.
constexpr int kSortThreads = 256, kSortBlock = 16 * kSortThreads;

// The 16 keys of one thread with two 16-B loads (one memory latency). i0 is a multiple of 16 below
// the key count and the key array is 256-B aligned and padded, so a read past the last key stays
// in the buffer; those keys are ignored.
__device__ __forceinline__ void load_keys16(const uint16_t* keys, uint32_t i0, uint16_t* kk) {
  const uint4* p = reinterpret_cast<const uint4*>(keys + i0);
  const uint4 a = p[0], b = p[1];
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) { kk[2 * j] = (uint16_t)(w[j] & 0xffffu); kk[2 * j + 1] = (uint16_t)(w[j] >> 16); }
}

__global__ __launch_bounds__(kSortThreads) void pair_hist_kernel(const uint16_t* __restrict__ keys,
                                                                 const uint32_t* __restrict__ count,
                                                                 uint32_t* __restrict__ hist, int nblk, int nbins) {
  __shared__ uint32_t h[kSortBins];
  for (int i = threadIdx.x; i < nbins; i += kSortThreads) h[i] = 0u;
  __syncthreads();
  // each thread counts 16 consecutive keys, one LDS atomic per run of equal keys (the keys of a
  // wave's rays are coherent, so per-key atomics would serialize on a few bins)
  const uint32_t n = ldc(count, 1), i0 = blockIdx.x * (uint32_t)kSortBlock + threadIdx.x * 16u;
  const uint32_t e = min(n, i0 + 16u);
  uint16_t kk[16];
  if (i0 < n) load_keys16(keys, i0, kk);
  uint32_t run = 0, rk = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16u; ++j) {
    if (i0 + j >= e) break;
    const uint32_t k = kk[j];
    if (run && k != rk) { atomicAdd(&h[rk], run); run = 0; }
    rk = k;
    ++run;
  }
  if (run) atomicAdd(&h[rk], run);
  __syncthreads();
  for (int i = threadIdx.x; i < nbins; i += kSortThreads) hist[(size_t)blockIdx.x * nbins + i] = h[i];  // row = block
}

// Column prefix: thread = bucket; hist[block][bucket] becomes the count of the bucket's keys in
// earlier blocks, and tot[bucket] the bucket's total (rows are read and written coalesced).
__global__ __launch_bounds__(64) void pair_colscan_kernel(const uint32_t* __restrict__ hist, uint32_t* __restrict__ prefix,
                                                          uint32_t* __restrict__ tot, int nblk, int nbins) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= nbins) return;
  uint32_t run = 0;
  int b = 0;
  for (; b + 8 <= nblk; b += 8) {  // 8 independent loads in flight per step
    uint32_t c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = hist[(size_t)(b + j) * nbins + k];
#pragma unroll
    for (int j = 0; j < 8; ++j) { prefix[(size_t)(b + j) * nbins + k] = run; run += c[j]; }
  }
  for (; b < nblk; ++b) {
    const uint32_t c = hist[(size_t)b * nbins + k];
    prefix[(size_t)b * nbins + k] = run;
    run += c;
  }
  tot[k] = run;
}

// Each block scans the bucket totals itself (nbins <= kSortBins, 32 per thread) and adds its row
// of column prefixes: cur[bucket] = first position of this block's keys of that bucket.
__global__ __launch_bounds__(kSortThreads) void pair_scatter_kernel(const uint16_t* __restrict__ keys,
                                                                    const uint32_t* __restrict__ count,
                                                                    const uint32_t* __restrict__ prefix,
                                                                    const uint32_t* __restrict__ tot,
                                                                    uint32_t* __restrict__ order, int nblk, int nbins) {
  __shared__ uint32_t cur[kSortBins];
  __shared__ uint32_t s_part[kSortThreads];
  constexpr int kPer = kSortBins / kSortThreads;
  const int t = threadIdx.x;
  uint32_t v[kPer], sum = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = t * kPer + j;
    v[j] = k < nbins ? tot[k] : 0u;
    sum += v[j];
  }
  s_part[t] = sum;
  __syncthreads();
  for (int off = 1; off < kSortThreads; off <<= 1) {  // inclusive scan of the per-thread sums
    const uint32_t x = t >= off ? s_part[t - off] : 0u;
    __syncthreads();
    s_part[t] += x;
    __syncthreads();
  }
  uint32_t run = s_part[t] - sum;  // exclusive
  const uint32_t* row = prefix + (size_t)blockIdx.x * nbins;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = t * kPer + j;
    if (k < nbins) cur[k] = run + row[k];
    run += v[j];
  }
  __syncthreads();
  const uint32_t n = ldc(count, 1), i0 = blockIdx.x * (uint32_t)kSortBlock + threadIdx.x * 16u;
  const uint32_t e = min(n, i0 + 16u);
  uint16_t kk[16];
  if (i0 < n) load_keys16(keys, i0, kk);
#pragma unroll
  for (uint32_t j = 0; j < 16u; ++j) {
    if (i0 + j >= e) break;
    order[atomicAdd(&cur[kk[j]], 1u)] = i0 + j;
  }
}

// Pair buffer: VisPairs (seg | out | flag) | muffle keys u16 | sorted order u32 | hist, scanned
// hist u32[bins x blocks] | scan temp.
struct PairBufs {
  VisPairs vp;
  uint16_t* keys;
  uint32_t *order, *hist, *prefix, *tot;
  BatchDesc* desc;  // [batches], when the batch descriptors are precomputed
  int2* pre;        // [groups * 64] first-segment nearest hits (ART_FAST_PRE_NEAREST)
  float4* state;    // [groups * 64][2] ray state between the bounce launches (multi-hit frames)
  size_t total;
  int nblk, nbins;
};

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

static size_t echo_cap_of(const FrameParams& fp) { return ((size_t)fp.S * fp.R * fp.H + 63) & ~(size_t)63; }
static size_t muffle_cap_of(const FrameParams& fp) { return (size_t)fp.S * fp.R * fp.H * fp.T; }

static PairBufs pair_bufs(void* base, const FrameParams& fp) {
  PairBufs b{};
  const size_t ecap = echo_cap_of(fp), mcap = muffle_cap_of(fp), max_pairs = ecap + mcap;
  uint8_t* p = static_cast<uint8_t*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) { uint8_t* q = p ? p + off : nullptr; off += align256(bytes); return q; };
  b.vp.seg = reinterpret_cast<float4*>(take(max_pairs * 32));
  b.vp.out = reinterpret_cast<uint2*>(take(max_pairs * 8));
  b.vp.flag = reinterpret_cast<uint32_t*>(take(max_pairs * 4));
  b.vp.echo_cap = (uint32_t)ecap;
  b.desc = ART_VIS_DESC ? reinterpret_cast<BatchDesc*>(take((ecap / 64 + (mcap + 63) / 64) * sizeof(BatchDesc))) : nullptr;
  if (bvh_pre(fp))
    b.pre = reinterpret_cast<int2*>(take((size_t)fp.S * ((fp.R + 63) / 64) * 64 * sizeof(int2)));
  if (bvh_pre(fp) && bvh_step(fp))
    b.state = reinterpret_cast<float4*>(take((size_t)fp.S * ((fp.R + 63) / 64) * 64 * (2 * sizeof(float4) + 4) +
                                             kLiveCounters * 4));  // + live list and counters
  if (ART_VIS_SORT && mcap) {
    b.nblk = (int)((mcap + kSortBlock - 1) / kSortBlock);
    b.nbins = fp.T << kSortDirBits;  // keys (target << kSortDirBits | cell) < T << kSortDirBits
    const size_t cells = (size_t)b.nbins * b.nblk;
    b.keys = reinterpret_cast<uint16_t*>(take(mcap * 2 + 64));  // + padding for load_keys16 past the end
    b.order = reinterpret_cast<uint32_t*>(take(mcap * 4));
    b.hist = reinterpret_cast<uint32_t*>(take(cells * 4));
    b.prefix = reinterpret_cast<uint32_t*>(take(cells * 4));
    b.tot = reinterpret_cast<uint32_t*>(take((size_t)b.nbins * 4));
  }
  b.total = off;
  return b;
}

size_t fast_pair_bytes(const FrameParams& fp) { return ART_FAST_SPLIT ? pair_bufs(nullptr, fp).total : 0; }

// Fans per launch_raytrace_fast call: pair slots (echo + muffle, R*H*(T+1) per fan) stay below
// 2^31 (the sorted-visibility bound, u32 slots) and a fan's echo halves stay addressable with a
// 32-bit half offset into the block (fan * stride / 2 < 2^32).
int fast_fans_per_launch(int R, int H, int T, uint32_t stride) {
  const unsigned long long per_fan = (unsigned long long)R * H * (T + 1) + 64;
  const unsigned long long by_pairs = ((1ull << 31) - 64) / per_fan;
  const unsigned long long by_block = ((1ull << 33) - 1) / (stride ? stride : 1) - 1;
  unsigned long long n = std::min(std::min(by_pairs, by_block), (unsigned long long)(1 << 30));
  if (const char* e = getenv("ART_FAST_CHUNK_FANS")) {  // test hook: force small chunks
    const long long v = atoll(e);
    if (v > 0) n = std::min(n, (unsigned long long)v);
  }
  return (int)std::max(1ull, n);
}

void launch_raytrace_fast(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                          uint8_t* block, uint32_t* muffle_acc, const int* ray_order, uint32_t* work, void* pair_buf,
                          uint32_t* pair_count, hipStream_t st) {
  if (fp.S == 0) return;
  const PairBufs pb = pair_bufs(ART_FAST_SPLIT ? pair_buf : nullptr, fp);
  const size_t mcap = muffle_cap_of(fp), max_pairs = (size_t)pb.vp.echo_cap + mcap;
  const bool sorted = ART_FAST_SPLIT && ART_VIS_SORT && mcap && pb.nbins <= kSortBins && max_pairs < (1u << 31);
  uint16_t* pkeys = sorted ? pb.keys : nullptr;
  if (ART_FAST_BVH && sc.bvh_levels > 0) {
    launch_fast_bvh(sc, fp, L, origins, block, muffle_acc, ray_order, work, pb.vp, pair_count, pkeys, pb.pre, pb.state, st);
  } else switch (fast_split(fp.S, fp.R)) {
    case 4: launch_fast_k<4>(sc, fp, L, origins, block, muffle_acc, ray_order, work, pb.vp, pair_count, pkeys, st); break;
    default: launch_fast_k<8>(sc, fp, L, origins, block, muffle_acc, ray_order, work, pb.vp, pair_count, pkeys, st); break;
  }
#if ART_FAST_SPLIT
  const uint32_t nb_max = (uint32_t)(pb.vp.echo_cap / 64 + (mcap + 63) / 64);
  const size_t items = (size_t)nb_max * vis_ranges(sc);
  if (items) {
    if (sorted) {
      hipLaunchKernelGGL(pair_hist_kernel, dim3(pb.nblk), dim3(kSortThreads), 0, st, pb.keys, pair_count, pb.hist, pb.nblk,
                         pb.nbins);
      hipLaunchKernelGGL(pair_colscan_kernel, dim3((pb.nbins + 63) / 64), dim3(64), 0, st, pb.hist, pb.prefix, pb.tot, pb.nblk,
                         pb.nbins);
      hipLaunchKernelGGL(pair_scatter_kernel, dim3(pb.nblk), dim3(kSortThreads), 0, st, pb.keys, pair_count, pb.prefix, pb.tot,
                         pb.order, pb.nblk, pb.nbins);
    }
    const uint32_t* order = sorted ? (const uint32_t*)pb.order : nullptr;
    const bool use_desc = pb.desc && ART_VIS_CONE && vis_ranges(sc) > 1 && !(fp.vis_bvh && sc.bvh_levels > 0);
    if (use_desc)
      hipLaunchKernelGGL(vis_batch_kernel, dim3((nb_max + 3) / 4), dim3(256), 0, st, pb.vp, pair_count, nb_max, order, pb.desc);
    if (fp.vis_bvh && sc.bvh_levels > 0)  // ART_CTX_VIS_BVH (measured 1.7x slower than vis_kernel on config 2)
      hipLaunchKernelGGL(vis_bvh_kernel, dim3((unsigned)((nb_max + kVisBvhWaves - 1) / kVisBvhWaves)), dim3(64 * kVisBvhWaves),
                         (size_t)bvh_lds_nodes(sc) * sizeof(CullRec), st, sc, pb.vp, pair_count, nb_max, order, fp.exec);
    else {
      // echo batches by quad BVH traversal (when the scene has a BVH), the rest by the sweep
      const uint32_t eb = (ART_VIS_ECHO_QUAD && sc.bvh_levels > 0) ? (ART_VIS_ALL_QUAD ? nb_max : pb.vp.echo_cap / 64) : 0u;
      const size_t vitems = (size_t)(nb_max - eb) * vis_ranges(sc);
      const size_t blocks = eb + (vitems + 3) / 4;
      const BatchDesc* dsc = use_desc ? (const BatchDesc*)pb.desc : nullptr;
      if (blocks) {
        const bool two = sc.chunks != nullptr && ART_VIS_TWO_LEVEL;
        if (fp.exec)
          hipLaunchKernelGGL((vis_kernel<true, false>), dim3((unsigned)blocks), dim3(256), 0, st, sc, pb.vp, pair_count, nb_max,
                             order, dsc, fp.exec, eb);
        else if (two)
          hipLaunchKernelGGL((vis_kernel<false, true>), dim3((unsigned)blocks), dim3(256), 0, st, sc, pb.vp, pair_count, nb_max,
                             order, dsc, nullptr, eb);
        else
          hipLaunchKernelGGL((vis_kernel<false, false>), dim3((unsigned)blocks), dim3(256), 0, st, sc, pb.vp, pair_count, nb_max,
                             order, dsc, nullptr, eb);
      }
    }
    hipLaunchKernelGGL(vis_finalize, dim3((unsigned)((max_pairs + 255) / 256)), dim3(256), 0, st, pb.vp, pair_count, block,
                       muffle_acc);
  }
#endif
}

}  // namespace art
