// art_cells.hip — muffle candidate lists: per audio target, a cube map of direction cells around
// the target, each listing the colliders that can block a muffle ray arriving through it.
//
// A muffle ray (CanRaySeeAudioTarget, Jobs/AudioRaytracerJobBatched.cs:405-449, cast at :150-173)
// runs from an offset hit point `off` to target t and is blocked by a collider not owned by t
// (:413, :426, :439) whose test reports a hit closer than distance(off, target) (:165). Every such
// segment ends at the target, so the colliders that can block it are exactly those met by the
// target's ray through `off`. Cell lists make that a lookup: muffle_kernel (art_trace.hip) tests
// only the entries of the segment's cell, instead of sorting per-(hit, target) pair records and
// sweeping collider chunks.
//
// Exactness. A collider whose float test blocks the segment contains, in its
// widened bounding sphere (margin factor * (far_t + |h| + 1), the broad-phase factors of §5 item 8
// applied to the rounding scale |off - c| <= maxd + |h| <= far_t + |h|), the exact point at the
// reported parameter of the float ray (off, normalize(t - off)). That ray deviates from the exact
// segment [off, target] by at most eta = 2e-6 far_t, so the
// collider's widened bounding sphere (+ 2 eta) meets the exact ray from the target towards `off`:
// either it contains the target (entered in every cell) or the direction from the target to
// `off` lies within the angular radius asin(rho / D) of the sphere, and that direction lies in
// the segment's cell (up to the rounding of the cell lookup, covered by the cones' 1e-4 rad
// slack). Entries also carry D - rho, a lower bound of the target distance of any blocking point;
// muffle_kernel skips entries beyond maxd. A segment longer than far_t (the bound the lists were
// built for), a degenerate segment, or a target whose lists overflowed tests every collider.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "art_device_fns.hpp"

namespace art {

constexpr float kCellEta = 2e-6f;  // relative deviation of a float muffle ray from its exact segment

// test hooks (read per call): ART_CELLS_MAX_PAIRS lowers the list threshold, ART_CELLS_CAP the
// entry capacity, so the no-list and dropped-target paths run at small sizes
static long long env_ll(const char* name, long long dflt) {
  const char* e = getenv(name);
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? v : dflt;
}


// far_t: the largest distance from target t to the scene's bounds (every muffle segment of t
// starts on a collider, so maxd <= far_t; muffle_kernel tests a longer segment against every
// collider).
__device__ __forceinline__ float cells_far_of(const CullRec& root, vec3 tg) {
  const float dx = fmaxf(fabsf(root.lox - tg.x), fabsf(root.hix - tg.x));
  const float dy = fmaxf(fabsf(root.loy - tg.y), fabsf(root.hiy - tg.y));
  const float dz = fmaxf(fabsf(root.loz - tg.z), fabsf(root.hiz - tg.z));
  return sqrtf(dx * dx + dy * dy + dz * dz) * 1.001f + 1e-3f;
}

// far_t of target t from the colliders' bounds box (cells_box_kernel: the box the BVH root holds),
// or INFINITY (no colliders or non-finite ones: every muffle ray of t tests every collider)
__device__ __forceinline__ float cells_far_t(const DevScene& sc, const CellBufs& cb, int t) {
  const CullRec& b = cb.box[0];
  return (b.lox == INFINITY && b.hix == INFINITY) ? INFINITY : cells_far_of(b, load3(sc.targets, t));
}

// The union of every collider's cull bounds (fminf / fmaxf, as the BVH's nodes; no colliders: the
// empty box at +infinity, as cull_stored), so the lists need no BVH and build beside it. One
// workgroup.
__global__ __launch_bounds__(1024) void cells_box_kernel(const CullRec* __restrict__ cull, int n, CullRec* __restrict__ box) {
  __shared__ float s[6][16];
  float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const CullRec c = cull[i];
    v[0] = fminf(v[0], c.lox); v[1] = fminf(v[1], c.loy); v[2] = fminf(v[2], c.loz);
    v[3] = fmaxf(v[3], c.hix); v[4] = fmaxf(v[4], c.hiy); v[5] = fmaxf(v[5], c.hiz);
  }
  for (int q = 0; q < 6; ++q)
    for (int m = 32; m >= 1; m >>= 1) {
      const float o = __shfl_xor(v[q], m, 64);
      v[q] = q < 3 ? fminf(v[q], o) : fmaxf(v[q], o);
    }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int q = 0; q < 6; ++q) s[q][w] = v[q];
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (int)(blockDim.x >> 6);
    for (int q = 0; q < 6; ++q) {
      v[q] = s[q][0];
      for (int k = 1; k < nw; ++k) v[q] = q < 3 ? fminf(v[q], s[q][k]) : fmaxf(v[q], s[q][k]);
    }
    CullRec r;
    r.fscale = 0.0f; r.factor = 0.0f;
    if (!(v[0] > v[3])) {
      r.lox = v[0]; r.loy = v[1]; r.loz = v[2]; r.hix = v[3]; r.hiy = v[4]; r.hiz = v[5];
    } else {
      r.lox = r.loy = r.loz = r.hix = r.hiy = r.hiz = INFINITY;
    }
    box[0] = r;
  }
}

// Global collider g (spheres, AABBs, OBBs): its order code and AudioTargetId.
__device__ __forceinline__ void collider_code(const DevScene& sc, int g, uint32_t& code, int& tid) {
  if (g < sc.ns) { code = (uint32_t)g; tid = sc.sph[g].tid; return; }
  g -= sc.ns;
  if (g < sc.na) { code = (1u << 28) | (uint32_t)g; tid = sc.aabb[g].tid; return; }
  g -= sc.na;
  code = (2u << 28) | (uint32_t)g;
  tid = sc.obb[g].tid;
}

// Cell range [i0, i1] of one face axis: the gnomonic coordinate u = (p . e_u) / (p . n) over the
// cone of half-angle gamma around a (components a_u, a_n; s = sin^2 gamma) is bounded by the roots
// of (a_n^2 - s) u^2 - 2 a_u a_n u + (a_u^2 - s) = 0 (the tangents of the cone's conic section).
__device__ __forceinline__ void face_range(float a_u, float a_n, float s, int& i0, int& i1) {
  const float den = a_n * a_n - s;
  const float disc = s * (a_u * a_u + a_n * a_n - s);
  if (!(den > 1e-3f) || !(disc >= 0.0f)) { i0 = 0; i1 = kCellG - 1; return; }
  const float sq = sqrtf(disc);
  const float r0 = (a_u * a_n - sq) / den, r1 = (a_u * a_n + sq) / den;
  const float lo = fminf(r0, r1), hi = fmaxf(r0, r1);
  i0 = (int)floorf((fmaxf(lo, -1.0f) + 1.0f) * (0.5f * kCellG)) - 1;
  i1 = (int)floorf((fminf(hi, 1.0f) + 1.0f) * (0.5f * kCellG)) + 1;
  i0 = max(i0, 0);
  i1 = min(i1, kCellG - 1);
  if (!(lo <= 1.0f && hi >= -1.0f)) { i0 = 1; i1 = 0; }  // outside the face
}

// Geometry of one (target, collider) pair for the enumeration: the unit direction to the widened
// bounding sphere, sin / cos of its angular radius, the entry (code, near) and per face the cell
// rectangle its cone can touch (i0, i1, j0, j1; empty when i0 > i1).
struct alignas(16) CellGeo {
  float ux, uy, uz, sb;
  float cb, near;
  uint32_t code, all;      // all: the sphere holds the target (every cell)
  uint8_t rect[6][4];
  uint32_t pad[2];
};

// Each pair's face rectangles also as one packed word per (target, face, collider), after the T * n
// CellGeo records: the row passes read 4 coalesced bytes per item and fetch the 64-B record only
// for the rows the rectangle covers.
__device__ __forceinline__ uint32_t* cell_rects(CellGeo* geo, int T, int n) {
  return reinterpret_cast<uint32_t*>(geo + (size_t)T * n);
}
__device__ __forceinline__ void cell_rects_write(CellGeo* geo, int T, int n, int t, int g, const CellGeo& G) {
  uint32_t* r = cell_rects(geo, T, n);
  for (int f = 0; f < 6; ++f)
    r[((size_t)t * 6 + f) * n + g] = (uint32_t)G.rect[f][0] | ((uint32_t)G.rect[f][1] << 8) | ((uint32_t)G.rect[f][2] << 16) |
                                     ((uint32_t)G.rect[f][3] << 24);
}

// One work-item per (target, collider), and per (target, cell, type) counter (zeroed, with the
// sentinel); the first T also set each target's segment bound, list flag and entry total.
// (grid-stride: one launch stays far below HIP's 2^32 work-item limit)
__device__ void cells_geo_one(const DevScene& sc, const CellBufs& cb, int n, int T, long long k, CellGeo* __restrict__ geo);
__global__ __launch_bounds__(256) void cells_geo_kernel(DevScene sc, CellBufs cb, int T, CellGeo* __restrict__ geo,
                                                        uint32_t counters) {
  const int n = sc.ns + sc.na + sc.no;
  const long long items = std::max((long long)n * T, (long long)counters);
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < items; k += (long long)gridDim.x * blockDim.x) {
    if (k < counters) cb.count[k] = 0u;
    if (k < T) {
      const float v = cells_far_t(sc, cb, (int)k);
      cb.far[k] = v;
      cb.ok[k] = isfinite(v) ? 1u : 0u;
      cb.tcount[k] = 0ull;
    }
    if (k < (long long)n * T) cells_geo_one(sc, cb, n, T, k, geo);
  }
}
__device__ void cells_geo_one(const DevScene& sc, const CellBufs& cb, int n, int T, long long k, CellGeo* __restrict__ geo) {
  const int t = (int)(k / n), g = (int)(k - (long long)t * n);
  CellGeo G;
  for (int f = 0; f < 6; ++f) { G.rect[f][0] = 1; G.rect[f][1] = 0; G.rect[f][2] = 1; G.rect[f][3] = 0; }
  G.pad[0] = G.pad[1] = 0u;
  uint32_t code;
  int tid;
  collider_code(sc, g, code, tid);
  G.code = code;
  G.all = 0u;
  G.ux = G.uy = G.uz = G.sb = G.cb = G.near = 0.0f;
  // owned by the target (its muffle rays skip it, :413, :426, :439) or no lists: no cells
  const float far = cells_far_t(sc, cb, t);  // (cb.far[t], written by another work-item of this launch)
  if (!isfinite(far) || tid == t) { geo[k] = G; cell_rects_write(geo, T, n, t, g, G); return; }
  // The collider's bounding sphere and its error margin. Every test's rounding is relative to the
  // segment-start-to-collider vector (the operands o and the record are exact floats): a reported
  // blocking point lies within factor * (|o - c| + |h|_1) of the shape,
  // and |o - c| <= maxd + rho <= far_t + rho for a collider the segment meets.
  const vec3 tg = load3(sc.targets, t);
  const CullRec cr = sc.cull[g];
  vec3 cc0;
  float r, h1, widen;
  const uint32_t ty = code >> 28, ix = code & 0x0fffffffu;
  if (ty == 0) {
    const SphereRec q = sc.sph[ix];
    cc0 = mk3(q.cx, q.cy, q.cz);
    r = sqrtf(q.r2) * 1.000001f;
    h1 = 3.0f * r;
    widen = 1.0f;
  } else {
    vec3 hh;
    if (ty == 1) {
      const AabbRec q = sc.aabb[ix];
      cc0 = mk3(0.5f * (q.mnx + q.mxx), 0.5f * (q.mny + q.mxy), 0.5f * (q.mnz + q.mxz));
      hh = mk3(0.5f * fabsf(q.mxx - q.mnx), 0.5f * fabsf(q.mxy - q.mny), 0.5f * fabsf(q.mxz - q.mnz));
    } else {
      const ObbRec q = sc.obb[ix];
      cc0 = mk3(q.cx, q.cy, q.cz);
      hh = mk3(0.5f * fabsf(q.lmxx - q.lmnx), 0.5f * fabsf(q.lmxy - q.lmny), 0.5f * fabsf(q.lmxz - q.lmnz));
    }
    r = sqrtf(hh.x * hh.x + hh.y * hh.y + hh.z * hh.z) * 1.00001f;
    h1 = hh.x + hh.y + hh.z;
    widen = 1.7321f;  // a box widened by m per axis: its half-diagonal grows by sqrt(3) m
  }
  const float m = cr.factor * (far + r + h1 + 1.0f);
  const float rho = r + widen * m + 2.0f * (kCellEta * far + 1e-6f) + 1e-6f * (fabsf(cc0.x) + fabsf(cc0.y) + fabsf(cc0.z)) +
                    cell_slack(r);
  const vec3 w = mk3(cc0.x - tg.x, cc0.y - tg.y, cc0.z - tg.z);
  const float D = sqrtf(w.x * w.x + w.y * w.y + w.z * w.z);
  const bool all = !(D > rho * 1.0001f) || !isfinite(D) || !isfinite(rho);  // the sphere holds the target
  const float sb = all ? 1.0f : rho / D;
  const float cb_ = sqrtf(fmaxf(0.0f, 1.0f - sb * sb));
  const float near = all ? 0.0f : fmaxf(0.0f, (D - rho) * 0.99999f - 1e-5f);
  const vec3 u = all ? mk3(1.0f, 0.0f, 0.0f) : mk3(w.x / D, w.y / D, w.z / D);
  const float gamma = cb.alpha_max + asinf(fminf(sb, 1.0f)) + 1e-3f;
  const bool wide = all || gamma >= 1.5f;
  const float sg = sinf(fminf(gamma, 1.5707963f)), s2 = sg * sg;
  const float uc[3] = {u.x, u.y, u.z};
  G.ux = u.x; G.uy = u.y; G.uz = u.z; G.sb = sb; G.cb = cb_; G.near = near; G.all = all ? 1u : 0u;
  for (int f = 0; f < 6; ++f) {
    const int ax = f >> 1;
    const float sgn = (f & 1) ? -1.0f : 1.0f;
    const float a_n = sgn * uc[ax], a_u = uc[(ax + 1) % 3], a_v = uc[(ax + 2) % 3];
    int i0 = 0, i1 = kCellG - 1, j0 = 0, j1 = kCellG - 1;
    if (!wide) {
      if (a_n <= -sg) continue;  // the cone stays in the opposite half-space
      face_range(a_u, a_n, s2, i0, i1);
      face_range(a_v, a_n, s2, j0, j1);
    }
    G.rect[f][0] = (uint8_t)i0; G.rect[f][1] = (uint8_t)i1; G.rect[f][2] = (uint8_t)j0; G.rect[f][3] = (uint8_t)j1;
  }
  geo[k] = G;
  cell_rects_write(geo, T, n, t, g, G);
}

// One workgroup per (target, face, cell row) and 256 colliders (grid-stride over these units): each
// work-item tests the row's cells of its collider's face rectangle against the pair's cone (the
// row's 32 cones staged in LDS), and the workgroup aggregates its hits per (cell, collider type) in
// LDS, so the global counters see one atomic per touched (cell, type) and workgroup instead of one
// per entry (round 4: the per-entry atomics and the 64-B record per item set the passes' 96 + 107
// us at config 2). FILL = false counts per cell; FILL = true reserves each (cell, type)'s range
// once, counting the cell's counter down from its count (ranges start + [new, old) are disjoint and
// fill the cell exactly), and writes the entries of the targets whose lists fit
// (cells_block_scan_kernel). (Round 4 also measured one workgroup per (target, face): 128 + 256 us with
// per-item load balancing over each wave — 32x fewer waves left every step's latency exposed.)
template <bool FILL>
__global__ __launch_bounds__(256) void cells_row_kernel(CellGeo* __restrict__ geo, int T, CellBufs cb, int n) {
  __shared__ uint32_t s_cnt[kCellG * 3];
  __shared__ float4 s_cone[kCellG];  // axis, cos_a
  __shared__ float s_sin[kCellG];
  const int tid = threadIdx.x;
  const int chunks = (n + 255) >> 8;
  const long long units = (long long)T * 6 * kCellG * chunks;
  const uint32_t* rects = cell_rects(geo, T, n);
  for (long long u = blockIdx.x; u < units; u += gridDim.x) {  // (workgroup-uniform)
    const long long row = u / chunks;
    const int gc = (int)(u - row * chunks);
    const int t = (int)(row / (6 * kCellG)), fr = (int)(row - (long long)t * 6 * kCellG), f = fr / kCellG, j = fr - f * kCellG;
    if (FILL && !cb.ok[t]) continue;  // (workgroup-uniform: a dropped target's lists stay empty)
    const int g = gc * 256 + tid;
    if (tid < kCellG * 3) s_cnt[tid] = 0u;
    if (tid < kCellG) {
      const CellCone cc = cb.cones[(f * kCellG + j) * kCellG + tid];
      s_cone[tid] = make_float4(cc.ax, cc.ay, cc.az, cc.cos_a);
      s_sin[tid] = cc.sin_a;
    }
    const uint32_t rc = g < n ? rects[((size_t)t * 6 + f) * n + g] : 0x00000001u;  // (i0 1 > i1 0: empty)
    const int i0 = (int)(rc & 0xffu), i1 = (int)((rc >> 8) & 0xffu), j0 = (int)((rc >> 16) & 0xffu), j1 = (int)(rc >> 24);
    const bool rows = !(j < j0 || j > j1 || i0 > i1);
    CellGeo G;
    uint32_t ty = 0u;
    if (rows) {
      G = geo[(size_t)t * n + g];
      ty = G.code >> 28;  // one list per collider type
    }
    __syncthreads();
    uint32_t hm = 0u;  // the row's cells this collider's cone touches (kCellG = 32 bits)
    for (int i = i0; rows && i <= i1; ++i) {
      // angle(u, axis) <= alpha_c + beta  <=>  u . axis >= cos(alpha_c + beta)
      const float4 cc = s_cone[i];
      if (G.all || (G.ux * cc.x + G.uy * cc.y + G.uz * cc.z >= (cc.w * G.cb - s_sin[i] * G.sb) - 1e-5f)) {
        hm |= 1u << i;
        atomicAdd(&s_cnt[i * 3 + ty], 1u);
      }
    }
    __syncthreads();
    const size_t rbase = ((size_t)t * kCells + (size_t)(f * kCellG + j) * kCellG) * 3;  // the row's counters
    if (!FILL) {
      if (tid < kCellG * 3 && s_cnt[tid]) atomicAdd(cb.count + rbase + tid, s_cnt[tid]);
    } else {
      if (tid < kCellG * 3) {
        const uint32_t c = s_cnt[tid];
        if (c) s_cnt[tid] = cb.start[rbase + tid] + atomicSub(cb.count + rbase + tid, c) - c;
      }
      __syncthreads();
      if (hm) {
        const uint32_t key = near_key(__float_as_uint(G.near));
        for (uint32_t m = hm; m; m &= m - 1u) {
          const int i = __builtin_ctz(m);
          const uint32_t pos = atomicAdd(&s_cnt[i * 3 + ty], 1u);
          if (pos < cb.cap) {  // the entry and its sort key (the segmented sort orders each cell by near bound)
            if (cb.compact) reinterpret_cast<uint32_t*>(cb.ent)[pos] = (G.code & 0xffffu) | (key << 16);
            else cb.ent[pos] = make_uint2(G.code, __float_as_uint(G.near));
            cb.keys[pos] = key;
          } else {
            cb.ok[t] = 0u;  // (cannot happen after the capacity check; kept as a guard)
          }
        }
      }
    }
    __syncthreads();  // (the LDS arrays are reused by the next unit)
  }
}

// Each (target, cell, type) list by ascending near key (muffle_kernel stops at the first entry past
// its segment), one wave per list, every entry ranked among its list's (the keys below it, equal
// keys by fill position) and scattered into the sorted array: a list of at most 64 entries holds one
// entry per lane and broadcasts the keys by readlane; up to kCellSortReg entries, each lane holds
// several; a longer list reads the keys from memory (O(n^2 / 64) per wave; no list of configs 2-5
// comes near: the longest lists have 29 / 64 / 48 / 26 entries at configs 2 / 3 / 4 / 5,
// ART_DEBUG_CELLS histograms in profiles/r05_cell_lists.txt). (Round 4 sorted every list with a segmented radix sort: 51 us of a
// config-2 rebuild frame.)
constexpr int kCellSortReg = 256;
template <bool COMPACT>
__device__ __forceinline__ void cells_scatter(const CellBufs& cb, uint32_t from, uint32_t to) {
  if (COMPACT) reinterpret_cast<uint32_t*>(cb.ent_s)[to] = reinterpret_cast<const uint32_t*>(cb.ent)[from];
  else cb.ent_s[to] = cb.ent[from];
}
template <bool COMPACT>
__global__ __launch_bounds__(256) void cells_sort_kernel(CellBufs cb, int cells) {
  constexpr int kR = kCellSortReg / 64;
  const int lane = threadIdx.x & 63;
  const int i = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (i >= cells) return;  // (wave-uniform)
  const uint32_t b = cb.start[i], e = cb.start[i + 1], n = e - b;
  if (n <= 1u) {
    if (n == 1u && lane == 0) cells_scatter<COMPACT>(cb, b, b);
    return;
  }
  if (n <= 64u) {  // one entry per lane
    const bool in = (uint32_t)lane < n;
    const uint32_t key = in ? cb.keys[b + lane] : 0xffffffffu;
    uint32_t rank = 0u;
    for (uint32_t j = 0; j < n; ++j) {
      const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)j);
      rank += (kj < key || (kj == key && j < (uint32_t)lane)) ? 1u : 0u;
    }
    if (in) cells_scatter<COMPACT>(cb, b + lane, b + rank);
    return;
  }
  if (n <= (uint32_t)kCellSortReg) {  // kR entries per lane (lane l: l, l + 64, ...)
    const uint32_t nr = (n + 63u) >> 6;
    uint32_t key[kR], rank[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t p = (uint32_t)(r * 64 + lane);
      key[r] = p < n ? cb.keys[b + p] : 0xffffffffu;
      rank[r] = 0u;
    }
#pragma unroll
    for (int r2 = 0; r2 < kR; ++r2) {
      if ((uint32_t)r2 >= nr) break;
      const uint32_t m = min(64u, n - (uint32_t)r2 * 64u);
      for (uint32_t j = 0; j < m; ++j) {
        const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key[r2], (int)j), pj = (uint32_t)r2 * 64u + j;
#pragma unroll
        for (int r = 0; r < kR; ++r) rank[r] += (kj < key[r] || (kj == key[r] && pj < (uint32_t)(r * 64 + lane))) ? 1u : 0u;
      }
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t p = (uint32_t)(r * 64 + lane);
      if (p < n) cells_scatter<COMPACT>(cb, b + p, b + rank[r]);
    }
    return;
  }
  for (uint32_t p = (uint32_t)lane; p < n; p += 64u) {  // long list: the other keys from memory
    const uint32_t key = cb.keys[b + p];
    uint32_t rank = 0u;
    for (uint32_t j = 0; j < n; ++j) {
      const uint32_t kj = cb.keys[b + j];
      rank += (kj < key || (kj == key && j < p)) ? 1u : 0u;
    }
    cells_scatter<COMPACT>(cb, b + p, b + rank);
  }
}

// The list starts (round 4: a per-target total kernel, a drop kernel and hipCUB's two-launch scan;
// a one-workgroup version of all three measured 72 us, its waves walking their groups serially):
//   cells_block_sum_kernel   one workgroup per 256 counters (a block lies in one target: kCells * 3
//                            is a multiple of 256): the block's sum, and one 64-bit atomic into its
//                            target's entry total;
//   cells_block_scan_kernel  one workgroup: the capacity check in target order (a target keeps its
//                            lists while the running total fits the capacity, else ok = 0 and its
//                            muffle rays test every collider), then the exclusive scan of the block
//                            sums with a dropped target's blocks taken as 0 (its lists stay empty; the
//                            fill pass skips it);
//   cells_start_kernel       one workgroup per block: its starts, the block's offset plus the
//                            exclusive scan of its counts.
// The block sums and offsets sit in the cursor array, the targets' totals in `tot` (T x u64).
__global__ __launch_bounds__(256) void cells_block_sum_kernel(CellBufs cb, unsigned long long* __restrict__ tot) {
  static_assert((kCells * 3) % 256 == 0, "a block lies in one target");
  __shared__ uint32_t s[4];
  uint32_t v = cb.count[(size_t)blockIdx.x * 256 + threadIdx.x];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t sum = s[0] + s[1] + s[2] + s[3];
    cb.cursor[blockIdx.x] = sum;
    if (sum) atomicAdd(tot + blockIdx.x / ((kCells * 3) / 256), (unsigned long long)sum);
  }
}
__global__ __launch_bounds__(1024) void cells_block_scan_kernel(CellBufs cb, int T, uint32_t blocks,
                                                                unsigned long long* __restrict__ tot) {
  __shared__ uint32_t s_keep[kMaxTargets];
  __shared__ uint32_t s_w[16];
  constexpr uint32_t kPerT = (kCells * 3) / 256;  // blocks per target
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) {
    unsigned long long run = 0ull;
    for (int t = 0; t < T; ++t) {
      const unsigned long long c = tot[t];
      const bool keep = cb.ok[t] && run + c <= (unsigned long long)cb.cap;
      if (keep) run += c;
      else cb.ok[t] = 0u;
      s_keep[t] = keep ? 1u : 0u;
    }
  }
  __syncthreads();
  // thread i scans blocks [i * per, (i + 1) * per) (the kept total is at most cap < 2^32)
  const uint32_t per = (blocks + 1023u) / 1024u, b0 = min(blocks, (uint32_t)tid * per), b1 = min(blocks, b0 + per);
  uint32_t sum = 0u;
  for (uint32_t b = b0; b < b1; ++b) sum += s_keep[b / kPerT] ? cb.cursor[b] : 0u;
  uint32_t inc = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (int k = 0; k < w; ++k) run += s_w[k];
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t v = s_keep[b / kPerT] ? cb.cursor[b] : 0u;
    cb.cursor[b] = run;  // the block's offset
    run += v;
  }
  if (b1 == blocks && b0 < b1) cb.start[(size_t)blocks * 256] = run;  // the sentinel: every kept entry
  if (blocks == 0 && tid == 0) cb.start[0] = 0u;
}
__global__ __launch_bounds__(256) void cells_start_kernel(CellBufs cb) {
  __shared__ uint32_t s[4];
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t v = cb.ok[blockIdx.x / ((kCells * 3) / 256)] ? cb.count[i] : 0u;
  uint32_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s[w] = inc;
  __syncthreads();
  uint32_t base = cb.cursor[blockIdx.x];
  for (int k = 0; k < w; ++k) base += s[k];
  cb.start[i] = base + inc - v;
}

size_t cells_scan_temp_bytes(int T, uint32_t cap) {  // (no library scratch since round 5: cells_block_scan_kernel)
  (void)T;
  (void)cap;
  return 0;
}

// Entry capacity: 128 cells per (target, collider) on average (a collider near its target spans
// hundreds, a far one a few); a target whose lists do not fit falls back to testing every collider.
size_t cells_entry_cap(int T, int C) {
  if (!cells_enabled(T, C)) return 0;
  const size_t want = (size_t)128 * (size_t)T * (size_t)(C > 0 ? C : 1);
  return std::min<size_t>(std::min<size_t>(std::max<size_t>(want, (size_t)1 << 16), (size_t)1 << 26),
                          (size_t)env_ll("ART_CELLS_CAP", 1ll << 26));
}

// Lists are built when the per-(target, collider) geometry stays within kCellsMaxPairs records
// (512 MiB of scratch); larger scenes run without lists (every muffle ray tests every collider).
constexpr long long kCellsMaxPairs = 1ll << 23;
bool cells_enabled(int T, int C) {
  return (long long)T * (long long)C <= env_ll("ART_CELLS_MAX_PAIRS", kCellsMaxPairs);
}

// grid of a grid-stride launch over `items` work-items (at most 2^16 workgroups of 256)
static unsigned stride_grid(long long items) { return (unsigned)std::max(1ll, std::min((items + 255) / 256, 1ll << 16)); }

// workgroups of a row pass: one per (target, face, row, 256 colliders), at most 2^16 (grid-stride)
static unsigned row_grid(int T, int n) {
  return (unsigned)std::max(1ll, std::min((long long)T * 6 * kCellG * ((n + 255) >> 8), 1ll << 16));
}

int launch_build_cells(DevScene& sc, const CellBufs& cb, hipStream_t st) {
  const int T = sc.T, n = sc.ns + sc.na + sc.no;
  const int cells = T * kCells * 3;  // lists: (target, cell, collider type)
  sc.cell_start = cb.start;
  sc.cell_ent = cb.ent_s;
  sc.cell_ent32 = reinterpret_cast<const uint32_t*>(cb.ent_s);
  sc.cell_compact = cb.compact;
  sc.cell_far = cb.far;
  sc.cell_ok = cb.ok;
  sc.cell_cap = cb.cap;
  if (cb.cap == 0) {  // no lists for this scene size (cells_enabled): every target tests every collider
    if (T > 0 && hipMemsetAsync(cb.ok, 0, (size_t)T * sizeof(uint32_t), st) != hipSuccess) return -1;
    return 0;
  }
  const long long pairs = (long long)n * T;
  CellGeo* geo = reinterpret_cast<CellGeo*>(cb.geo);
  hipLaunchKernelGGL(cells_box_kernel, dim3(1), dim3(1024), 0, st, sc.cull, n, cb.box);
  hipLaunchKernelGGL(cells_geo_kernel, dim3(stride_grid(std::max(pairs, (long long)cells + 1))), dim3(256), 0, st, sc, cb, T,
                     geo, (uint32_t)cells + 1);
  if (pairs > 0) {
    hipLaunchKernelGGL(cells_row_kernel<false>, dim3(row_grid(T, n)), dim3(256), 0, st, geo, T, cb, n);
  }
  // per-target totals, the capacity check and the list starts (three launches)
  {
    const uint32_t blocks = (uint32_t)cells / 256u;
    unsigned long long* tot = cb.tcount;  // (zeroed by cells_geo_kernel)
    if (blocks) hipLaunchKernelGGL(cells_block_sum_kernel, dim3(blocks), dim3(256), 0, st, cb, tot);
    hipLaunchKernelGGL(cells_block_scan_kernel, dim3(1), dim3(1024), 0, st, cb, T, blocks, tot);
    if (blocks) hipLaunchKernelGGL(cells_start_kernel, dim3(blocks), dim3(256), 0, st, cb);
  }
  if (pairs > 0)
    hipLaunchKernelGGL(cells_row_kernel<true>, dim3(row_grid(T, n)), dim3(256), 0, st, geo, T, cb, n);
  // each cell's entries by ascending near bound: muffle_kernel stops at the first one past its
  // segment (every start is <= cap after the drop pass)
  if (cb.compact)
    hipLaunchKernelGGL(cells_sort_kernel<true>, dim3((unsigned)((cells + 3) / 4)), dim3(256), 0, st, cb, cells);
  else
    hipLaunchKernelGGL(cells_sort_kernel<false>, dim3((unsigned)((cells + 3) / 4)), dim3(256), 0, st, cb, cells);
  if (env_ll("ART_DEBUG_CELLS", 0)) {  // diagnostics: the built lists' size and length histogram (synchronizes)
    std::vector<uint32_t> hs((size_t)cells + 1);
    if (hipMemcpyAsync(hs.data(), cb.start, hs.size() * 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
        hipStreamSynchronize(st) == hipSuccess) {
      unsigned long long hist[18] = {};  // lists of length 0, 1, 2-3, 4-7, ... (log2 buckets)
      uint32_t longest = 0;
      for (int i = 0; i < cells; ++i) {
        const uint32_t len = hs[(size_t)i + 1] - hs[i];
        longest = std::max(longest, len);
        hist[len == 0 ? 0 : std::min(17, 32 - __builtin_clz(len))]++;
      }
      fprintf(stderr, "[cells] T %d colliders %d: %u entries (capacity %u, %.1f per pair), %d lists, longest %u; lengths", T,
              n, hs[(size_t)cells], cb.cap, (double)hs[(size_t)cells] / std::max(1ll, pairs), cells, longest);
      for (int b = 0; b < 18; ++b)
        if (hist[b]) fprintf(stderr, " [%u..%u]:%llu", b == 0 ? 0u : 1u << (b - 1), b == 0 ? 0u : (1u << b) - 1u, hist[b]);
      fprintf(stderr, "\n");
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t cells_geo_bytes(int T, int C) {  // the CellGeo records, then the packed face rectangles (cell_rects)
  return cells_enabled(T, C) ? (size_t)T * (size_t)(C > 0 ? C : 1) * (sizeof(CellGeo) + 6 * sizeof(uint32_t)) : 0;
}

}  // namespace art
