// art_trace.hip — the throughput raytrace stage (AudioRaytracerJobBatched.Execute,
// Jobs/AudioRaytracerJobBatched.cs:61-215) on gfx950.
//
// One frame of S fans x R rays is, per bounce k = 0 .. H-1:
//   nearest_first_kernel  nearest hit of every live ray segment (ShootRayCast :225-280) by a
//                         quad-per-ray traversal of the collider BVH (art_bvh.hip);
//   path_kernel           the exact re-evaluation of the winner, the hit point, the echo pair
//                         (:121-145) and the hit record of the muffle rays (:150-173) and, for
//                         multi-hit frames, the reflection / termination (:179-193, ReflectRay
//                         :456-532) and the ray state of the next bounce;
//   vis_kernel            (side stream) the bounce's echo rays (CanRaySeePoint :365-397) by quad
//                         BVH any-hit traversal; a visible echo is stored at once;
// then, once for the frame:
//   muffle_kernel         every hit's muffle rays (CanRaySeeAudioTarget :405-449) against the
//                         target's direction-cell candidate lists (art_cells.hip), visible rays
//                         counted into the muffle accumulators.
// Every output equals the reference's bit for bit: the broad phases are exact, the
// nearest hit is the (distance, reference order) minimum, any-hit verdicts are ORs.
#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <cstdlib>

#include "art_device_fns.hpp"
#include "art_frame_math.hpp"

namespace art {

constexpr int kNoHit = 0x7fffffff;
#ifndef ART_MEASURE_PARTS
#define ART_MEASURE_PARTS 0  // (measurement builds only, wrong outputs: 1 = no muffle rays in echo_muffle_kernel, 2 = no echo rays)
#endif
constexpr int kNoOwner = 0x7fffffff;  // echo rays skip no collider (AudioTargetId is 16-bit)

// Sphere test split so the common miss costs no branch: the square root and the two IEEE
// divisions run only for lanes whose discriminant is non-negative (RayIntersectsSphere :323-355).
// (A one-division form, selecting the quotient by the numerators' signs, measured 1-3 % slower in
// both traversals: DESIGN.md §4.)
__device__ __forceinline__ bool sphere_hit_dist(const Seg& s, const SphereRec& c, float& dist) {
  vec3 oc = s.o - mk3(c.cx, c.cy, c.cz);
  float b = 2.0f * dot(oc, s.d);
  float cc = dot(oc, oc) - c.r2;
  float disc = b * b - (2.0f * s.a2) * cc;  // 4 * a * c (:329)
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

// Executed-work accounting (ART_CTX_COUNT_EXECUTED): one atomic per call from lane 0, off when
// `ex` is null (a uniform branch).
__device__ __forceinline__ void exec_add(unsigned long long* ex, int slot, unsigned long long v) {
  if (ex && v && (threadIdx.x & 63) == 0) atomicAdd(ex + slot, v);
}

#ifdef ART_DIAG
// Diagnostic build only (tools/build_variant.sh diag -DART_DIAG): log2 histograms of per-wave
// cycles (0 nearest, 1 echo) and per-ray traversal steps (2 nearest, 3 echo), printed by
// art_destroy.
__device__ unsigned long long g_diag[4][64];
__device__ __forceinline__ void diag_add(int k, unsigned long long v) {
  atomicAdd(&g_diag[k][v ? 64 - __builtin_clzll(v) : 0], 1ull);
}
#define ART_DIAG_STEP(x) (++(x))
#else
#define ART_DIAG_STEP(x) ((void)0)
#endif

#ifdef ART_WAVE_TIMES
// Diagnostic build only (tools/build_variant.sh wt -DART_WAVE_TIMES): every wave of the nearest and
// echo+muffle launches writes (start | kind << 60, end) in wall-clock ticks and its (block, HW_ID,
// XCC_ID) to its own slot (nearest waves in the first half, echo+muffle waves in the second; no
// atomics, each frame overwrites the previous one's), which art_destroy writes to
// $ART_WAVE_TIMES_OUT (tools/wave_times.py reads it): the launches' wave timelines of the last frame.
constexpr unsigned kWtCap = 1u << 18;
__device__ unsigned long long g_wt[kWtCap][2];
__device__ uint32_t g_wt_id[kWtCap][3];
struct WaveTimer {
  unsigned long long t0;
  unsigned kind;
  __device__ explicit WaveTimer(unsigned k) : t0(wall_clock64()), kind(k) {}
  __device__ ~WaveTimer() {
    const unsigned long long t1 = wall_clock64();
    if ((threadIdx.x & 63) == 0) {
      const unsigned i = (kind ? kWtCap / 2 : 0u) + (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % (kWtCap / 2);
      g_wt[i][0] = t0 | ((unsigned long long)kind << 60);
      g_wt[i][1] = t1;
      g_wt_id[i][0] = blockIdx.x | (threadIdx.x >> 6) << 24;
      g_wt_id[i][1] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID
      g_wt_id[i][2] = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // XCC_ID
    }
  }
};
#define ART_WAVE_TIMER(k) WaveTimer art_wave_timer_(k)
#else
#define ART_WAVE_TIMER(k) ((void)0)
#endif

// A ray whose direction or origin is non-finite, or whose direction is zero, makes every box test
// inconclusive: its traversals visit every node (the exact tests alone decide).
__device__ __forceinline__ bool force_all(const Seg& s, float om) {
  return !(isfinite(om) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
         (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
}

// The widened box of a BVH node / collider (margin factor * (scale + om)):
// entry distance of the segment, or false when it misses the box.
__device__ __forceinline__ bool node_entry(const Seg& s, const CullRec& r, float om, float& tn) {
  const float m = __builtin_fmaf(r.factor, om, r.fscale);  // factor * (scale + om), fscale = factor * scale
  float tf;
  return slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.lox - m, r.loy - m, r.loz - m, r.hix + m, r.hiy + m,
                     r.hiz + m, tn, tf);
}

// ------------------------------------------------------------------------------------------
// Quad-per-ray BVH traversal. The BVH (DevScene::bvh) is a complete 4-ary tree over the Morton
// order of the colliders' bounds, kBvhLeaf colliders per leaf. 4 lanes hold one ray: lane q of the
// quad tests child q of an inner node or slot q of a leaf, the quad exchanges the four results
// through DPP quad permutes, and every lane applies the same near-first ordering, so the ray's
// stack and current node stay identical in the quad (one test per lane per step, 4x the waves of
// one lane per ray).
// Exactness: a collider the ray can hit lies in every ancestor's widened box
// at least 3/4 of the margin inside, so its computed distance is strictly greater than each
// ancestor's computed entry; pruning at entry <= best never drops the winner or a tie, and ties are
// broken by the global order code (type rank << 28 | index), the reference's first minimum over
// Sphere, AABB, OBB order (ShootRayCast :225-280).
// ------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ int quad_perm(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false); }
constexpr int kQuadXor1 = 1 | (0 << 2) | (3 << 4) | (2 << 6), kQuadXor2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);
constexpr int kQuadRot1 = 1 | (2 << 2) | (3 << 4) | (0 << 6), kQuadRot3 = 3 | (0 << 2) | (1 << 4) | (2 << 6);


// (distance, order) keys (nearest_key) minimum over the quad: one 64-bit compare per DPP round.
__device__ __forceinline__ unsigned long long quad_min_u64(unsigned long long v) {
  {
    const unsigned long long o = ((unsigned long long)(uint32_t)quad_perm<kQuadXor1>((int)(v >> 32)) << 32) |
                                 (uint32_t)quad_perm<kQuadXor1>((int)v);
    v = o < v ? o : v;
  }
  const unsigned long long o = ((unsigned long long)(uint32_t)quad_perm<kQuadXor2>((int)(v >> 32)) << 32) |
                               (uint32_t)quad_perm<kQuadXor2>((int)v);
  return o < v ? o : v;
}

// Quad reductions without ballots (the result lands in every lane of the quad).
__device__ __forceinline__ uint32_t quad_min_u32(uint32_t v) {
  v = min(v, (uint32_t)quad_perm<kQuadXor1>((int)v));
  return min(v, (uint32_t)quad_perm<kQuadXor2>((int)v));
}

// The BVH node and leaf arrays as buffer resources (wave-uniform bases, 32-bit lane offsets).
struct BvhRes {
  __amdgpu_buffer_rsrc_t nodes, leaves;
};
__device__ __forceinline__ BvhRes bvh_res(const DevScene& sc) {
  BvhRes b;
  const int leaf0 = sc.bvh_leaf0, nleaf = 3 * leaf0 + 1, total = leaf0 + nleaf;
  b.nodes = __builtin_amdgcn_make_buffer_rsrc(const_cast<CullRec*>(sc.bvh), 0, total * (int)sizeof(CullRec), 0x00020000);
  b.leaves = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(sc.bvh_leaf), 0, nleaf * kBvhLeaf * 64, 0x00020000);
  return b;
}
__device__ __forceinline__ CullRec load_node(const BvhRes& b, int i) {
  const float4 a = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(b.nodes, i * 32, 0, 0));
  const float4 c = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(b.nodes, i * 32 + 16, 0, 0));
  CullRec r;
  r.lox = a.x; r.loy = a.y; r.loz = a.z; r.fscale = a.w;
  r.hix = c.x; r.hiy = c.y; r.hiz = c.z; r.factor = c.w;
  return r;
}

// Shared-origin node table (TAB kernels): every ray of a workgroup starts at the fan origin O, so a
// node's widened box relative to O, (lo - m) - O and (hi + m) - O with m = factor * (scale + |O|_1),
// is the same for all of them. Built once per workgroup in LDS (node_table_build), the node test is
// then the slab's multiplies and min / max on the very operands node_entry computes (bit-identical:
// the same operations in the same order, DESIGN.md §5 item 8 unchanged). Up to kTabNodes nodes
// (the BVH of <= 4096 colliders: 1365 nodes, 32 KB).
constexpr int kTabNodes = 1365;
#ifndef ART_TAB_USE
#define ART_TAB_USE 1  // (measurement builds: 0 = the table is built but the node tests load the nodes; -1 = not built either)
#endif
struct NodeTab {
  float4 a[kTabNodes];  // (lo.x, lo.y, lo.z, hi.x) relative to O, widened
  float2 b[kTabNodes];  // (hi.y, hi.z)
};
__device__ __forceinline__ void node_table_build(const DevScene& sc, vec3 O, NodeTab* tab) {
  const BvhRes br = bvh_res(sc);
  const int nn = sc.bvh_leaf0 + 3 * sc.bvh_leaf0 + 1;
  const float om = fabsf(O.x) + fabsf(O.y) + fabsf(O.z);  // quad_nearest_core's om of every ray at O
  for (int i = (int)threadIdx.x; i < nn; i += (int)blockDim.x) {
    const CullRec r = load_node(br, i);
    const float m = __builtin_fmaf(r.factor, om, r.fscale);  // node_entry's margin
    tab->a[i] = make_float4((r.lox - m) - O.x, (r.loy - m) - O.y, (r.loz - m) - O.z, (r.hix + m) - O.x);
    tab->b[i] = make_float2((r.hiy + m) - O.y, (r.hiz + m) - O.z);
  }
}
__device__ __forceinline__ bool node_entry_tab(const Seg& s, const NodeTab* tab, int i, float& tn) {
  const float4 a = tab->a[i];
  const float2 b = tab->b[i];
  const float t0x = a.x * s.inv.x, t0y = a.y * s.inv.y, t0z = a.z * s.inv.z;  // slab<false>'s (mn - o) * inv
  const float t1x = a.w * s.inv.x, t1y = b.x * s.inv.y, t1z = b.y * s.inv.z;
  tn = fmax_ieee(fmax_ieee(fmin_ieee(t0x, t1x), fmin_ieee(t0y, t1y)), fmin_ieee(t0z, t1z));
  const float tf = fmin_ieee(fmin_ieee(fmax_ieee(t0x, t1x), fmax_ieee(t0y, t1y)), fmax_ieee(t0z, t1z));
  return !(tn > tf || tf < 0.0f);
}

// One inner step of a quad traversal (lane qd holds child c0 + qd; `enter` / entry `en` its
// verdict): descend into the nearest entered child and push the other entered children far first
// onto the ray's stack, or pop when none is entered. Near-first order by rank: each lane's key is
// its child's entry bits with the child index in the two low bits (unique in the quad; non-entered
// children 0xffffffff), its rank the number of smaller keys among the quad's other three (three DPP
// rotations); the quad minimum of the keys names the nearest child, 1 + the largest rank of an
// entered lane counts them. No ballots: every value is a quad DPP reduction (measured 3 % faster in
// the nearest traversal; the echo any-hit keeps its ballot form, index order, which measured 6 %
// faster there than this near-first form).
#ifndef ART_NEAREST_ONE_ANY
#define ART_NEAREST_ONE_ANY 1
#endif
__device__ __forceinline__ void quad_descend(bool enter, float en, bool force, int qd, int c0, uint32_t* my, int& g,
                                             int& sp, int* bp = nullptr) {
  const uint32_t key = enter ? (((uint32_t)__float_as_int(en) & (force ? 0u : ~3u)) | (uint32_t)qd) : 0xffffffffu;
  const uint32_t k1 = (uint32_t)quad_perm<kQuadRot1>((int)key), k2 = (uint32_t)quad_perm<kQuadXor2>((int)key),
                 k3 = (uint32_t)quad_perm<kQuadRot3>((int)key);
  const int rank = (int)(k1 < key) + (int)(k2 < key) + (int)(k3 < key);
  const uint32_t kmin = min(min(key, k1), min(k2, k3));
  // entered children (one ballot of the key itself: an entered key is at most 0x7f800003, en >= 0)
  const int nent = __popc((uint32_t)(__builtin_amdgcn_ballot_w64(key != 0xffffffffu) >> (__lane_id() & ~3)) & 0xFu);
  const int spn = sp + nent - 1;  // the stack pointer after the push (one add shared by both uses)
  if (enter && rank > 0) my[spn - rank] = (uint32_t)(c0 + qd);
  if (nent) {
    g = c0 + (int)(kmin & 3u);
    sp = spn;
  } else {  // branch-free pop: the stack slot is read unconditionally (clamped), -1 when empty
    const int t = (int)my[sp > 0 ? sp - 1 : 0];
    g = sp > 0 ? t : -1;
    sp = sp > 0 ? sp - 1 : 0;
    if (ART_NEAREST_ONE_ANY && bp != nullptr && sp == *bp) sp = *bp = 0;  // the entries below bp were taken
  }
}

// Exact test of leaf slot `sl` (64 B: the hot record's test fields and the order code, art_bvh.hip
// bvh_leaf_kernel) against segment s; tid = the collider's AudioTargetId. OBB = false: the scene has
// no OBBs (no rank-2 slots), their test compiles out. PERM: the permeation job's first-hit cast,
// whose OBB test rotates by the inverse of the stored rotation (AudioPermeationJobBatched.cs
// :172-179, App. B Q5), read from the cold record (obbc).
template <bool OBB, bool PERM = false>
__device__ __forceinline__ bool leaf_slot_test(const Seg& s, const BvhRes& br, int slot, int& cc, float& dist, int& tid,
                                               unsigned* nt, const ObbCold* obbc = nullptr) {
  // (slots are 64 B with OBBs in the scene, 32 B without: art_bvh.hip bvh_leaf_kernel)
  auto ld = [&](int k) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(br.leaves, slot * (OBB ? 64 : 32) + 16 * k, 0, 0));
  };
  const float4 qa = ld(0), qb = ld(1);
  cc = __float_as_int(qb.w);
  dist = 0.0f;
  tid = kNoOwner;
  if (cc < 0) return false;  // empty slot past the last collider
  const int t = cc >> 28;
  if (t == 0) {
    SphereRec r;
    r.cx = qa.x; r.cy = qa.y; r.cz = qa.z; r.r2 = qa.w;
    tid = __float_as_int(qb.z);
    ++nt[0];
    return sphere_hit_dist(s, r, dist);
  }
  if (t == 1 || !OBB) {
    AabbRec r;
    r.mnx = qa.x; r.mny = qa.y; r.mnz = qa.z; r.mxx = qa.w; r.mxy = qb.x; r.mxz = qb.y;
    tid = __float_as_int(qb.z);
    ++nt[1];
    return aabb_test<false>(s, r, dist);
  }
  // RayIntersectsOBB (:314-320) in the order that keeps the fewest values live: the rotated
  // direction's reciprocals first (the direction dies), then the rotated origin, and the local
  // bounds fetched only then (same operations as obb_test)
  quat q;
  if (PERM) {
    q = inverse_q(obbc[cc & 0x0fffffff]);
  } else {
    q.x = qa.w; q.y = qb.x; q.z = qb.y; q.w = qb.z;
  }
  const vec3 ld3 = qmul(q, s.d);
  const float ix = recip_exact(ld3.x), iy = recip_exact(ld3.y), iz = recip_exact(ld3.z);
  const vec3 lo = qmul(q, s.o - mk3(qa.x, qa.y, qa.z));
  __builtin_amdgcn_sched_barrier(0);
  const float4 qc = ld(2), qe = ld(3);
  tid = __float_as_int(qe.z);
  ++nt[2];
  float tNear, tFar;
  const bool hit = slab<false>(lo.x, lo.y, lo.z, ix, iy, iz, qc.x, qc.y, qc.z, qc.w, qe.x, qe.y, tNear, tFar);
  dist = tNear > 0.0f ? tNear : tFar;
  return hit;
}

// Population count of a 64-bit lane mask as two 32-bit counts: an int result that compares with
// 32-bit scalar / vector compares (a 64-bit count compares with VALU 64-bit compares).
__device__ __forceinline__ int pop64(unsigned long long x) {
  return __builtin_popcount((uint32_t)x) + __builtin_popcount((uint32_t)(x >> 32));
}

// Work sharing inside a wave (nearest and echo traversals): a wave lasts as long as its longest
// traversal, so a quad whose traversal has ended takes over the bottom entry of a busy quad's
// stack (the largest pending subtree) together with that quad's ray, and traverses it for the
// ray's home quad. (ART_*_STEAL=0 builds the plain traversals, for A/B runs.)
#ifndef ART_VIS_STEAL
#define ART_VIS_STEAL 1
#endif
#ifndef ART_ECHO_PARK
#define ART_ECHO_PARK 1  // (0: echo_muffle_kernel's echo traversal tests a leaf as soon as its quad reaches it, for A/B runs)
#endif
#ifndef ART_NEAREST_STEAL
#define ART_NEAREST_STEAL 1
#endif
// Idle quads a wave waits for before it shares work (round 4: waiting for 3 in the nearest and 2 in
// the echo traversal runs the steal sequence, 13 lane shuffles and a select, less often; config 2
// nearest 55.4 -> 52.7 us, config 3 74.1 -> 70.5 us, config 5 91.4 -> 89.0 us per bounce).
#ifndef ART_STEAL_MIN_IDLE
#define ART_STEAL_MIN_IDLE 3
#endif
#ifndef ART_VIS_STEAL_MIN_IDLE
#define ART_VIS_STEAL_MIN_IDLE 2
#endif
constexpr unsigned long long kQuad0 = 0x1111111111111111ull;  // lane 0 of every quad

// Waves per SIMD of the traversal kernels: 8 (64 VGPRs). Register spills inside the divergent
// traversal loops hung a fused kernel once, so the counting instantiations and
// the echo traversal's OBB one run at the occupancy that holds them without spills. Every
// instantiation in this file compiles without scratch, the OBB nearest one at 8 waves included
// (its round-3 spills went with the round-4 leaf layout; profiles/r06_spill_check.txt).
#ifndef ART_NEAREST_OBB_WAVES
#define ART_NEAREST_OBB_WAVES 8
#endif
template <bool EX, bool OBB>
constexpr int kNearestWaves = EX ? 6 : (OBB ? ART_NEAREST_OBB_WAVES : 8);
template <bool EX, bool OBB>
constexpr int kEchoWaves = EX ? 6 : (OBB ? 7 : 8);
// echo_muffle_kernel<false, true>: 7 waves per SIMD (72 VGPRs: the muffle rays' prefetching list
// walks, muffle_blocked) without spills (round 6; 8 waves before them)
#ifndef ART_ECHO_MUFFLE_OBB_WAVES
#define ART_ECHO_MUFFLE_OBB_WAVES 7
#endif
// Work sharing's pairing: the quad base lane (l4) of the donor whose rank among the donors equals
// this thief's rank ir. Two cross-lane moves instead of a select-bit search: lane 0 of each robbed
// donor (rank dr) forwards its l4 to lane 4 dr + 1 (ds_permute; every other lane writes into a
// 4k + 2 lane nobody reads), then each lane reads lane 4 ir + 1 (ds_bpermute). Both run in every
// lane of the wave; the caller uses the result in its thieves only.
__device__ __forceinline__ int rank_match(int l4, int qd, bool robbed, int dr, int ir) {
  const int dst = (robbed && qd == 0) ? 4 * dr + 1 : l4 + 2;
  const int tab = __builtin_amdgcn_ds_permute(dst << 2, l4);
  return __builtin_amdgcn_ds_bpermute(((4 * ir + 1) & 63) << 2, tab);
}

// (distance, order) as one ordered 64-bit key; distances are >= 0 or -0, the two zeros equal
__device__ __forceinline__ unsigned long long nearest_key(float d, int code) {
  return ((unsigned long long)(d == 0.0f ? 0u : __float_as_uint(d)) << 32) | (uint32_t)code;
}

// Nearest hit of the quad's ray s (identical in the 4 lanes; `my` = the ray's kBvhStack-entry
// stack inside the wave's 16 stacks; s_bound / s_key = the wave's 16 shared pruning bounds and
// result keys): (distance, order) minimum in best / code of every lane of the quad.
// With work sharing, the quads that traverse parts of one ray's tree prune against the smallest
// distance any of them found (s_bound, published once the wave has shared work), and the ray's
// result is the (distance, order) minimum of their results (a 64-bit LDS minimum of (distance
// bits, order); the two zeros compare equal, as in the reference's `<`, and the path kernel
// re-evaluates a zero distance).
// PERM: the permeation job's first-hit cast (ShootRayCast :101-141: INFINITY sentinel, inverse OBB
// rotation); otherwise the raytracer's (:225-280: float.MaxValue sentinel).
// TAB: every ray of the workgroup starts at one origin (a fan's bounce-0 casts), and `tab` holds
// each BVH node's widened box relative to it (node_table): a node test is 6 multiplies and the
// min / max, with the same operands as node_entry's.
template <bool EX, bool OBB, bool PERM = false, bool TAB = false>
__device__ __forceinline__ void quad_nearest_core(const DevScene& sc, Seg s, bool alive, int lane, uint32_t* my,
                                                  int* s_bound, unsigned long long* s_key, float& best, int& code,
                                                  unsigned long long* ex, const NodeTab* tab = nullptr) {
  const int qd = lane & 3, wq = lane >> 2;
  uint32_t* const s_wave = my - wq * kBvhStack;
  best = FLT_MAX;
  code = kNoHit;
  if (sc.bvh_levels == 0) return;  // no colliders: every ray misses
  if (ART_NEAREST_STEAL && qd == 0) s_key[wq] = ~0ull;  // the ray's shared result key, opened before the loop
  unsigned nt[3] = {0u, 0u, 0u}, nnode = 0;
  float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z);
  bool force = force_all(s, om);
  // the forced lanes as a lane mask (wave-uniform, kept in SGPRs): a node test ORs it in with scalar
  // instructions (__builtin_amdgcn_inverse_ballot_w64) instead of a per-lane 0/1 value
  unsigned long long fmk = __builtin_amdgcn_ballot_w64(force);
  const int leaf0 = sc.bvh_leaf0;
  const BvhRes br = bvh_res(sc);
  int g = alive ? 0 : -1, sp = 0, bp = 0, home = wq;
  float lim = FLT_MAX;   // pruning bound: best, and (shared work) the other quads' results for the ray
  bool shared = false;   // wave-uniform: work was shared in this wave
  // this quad's own (distance, order) minimum over the leaves it tested, as a nearest_key (~0: none)
  unsigned long long mykey = ~0ull;
  unsigned nsteps = 0;
  (void)nsteps;
  // branch-free pop of entries [bp, sp): the slot is read unconditionally (clamped), -1 when empty
  auto pop = [&]() {
    const bool has = sp > bp;
    const int t = (int)my[has ? sp - 1 : 0];
    g = has ? t : -1;
    sp = has ? sp - 1 : sp;
    if (sp == bp) sp = bp = 0;
  };
  // A child is entered when its widened box is entered at or before the bound (a winner or tie
  // lies strictly after every ancestor's entry); quad_descend orders the entered ones.
  auto inner_step = [&]() {
    const int c0 = 4 * g + 1;
    if (EX && qd == 0) ++nnode;
    ART_DIAG_STEP(nsteps);
    float tn;
    bool h;
    if (TAB && ART_TAB_USE > 0) {
      h = node_entry_tab(s, tab, c0 + qd, tn);
    } else {
      const CullRec r = load_node(br, c0 + qd);
      h = node_entry(s, r, om, tn);
    }
    const float en = fmaxf(tn, 0.0f);
    const bool enter = __builtin_amdgcn_inverse_ballot_w64(fmk) | (h & (en <= lim));  // (empty nodes: art_bvh.hip cull_stored)
    quad_descend(enter, en, force, qd, c0, my, g, sp, ART_NEAREST_ONE_ANY ? &bp : nullptr);
    if (!ART_NEAREST_ONE_ANY && sp == bp) sp = bp = 0;  // (else quad_descend's pop keeps sp == bp => 0)
  };
  auto leaf_step = [&](int leaf) {
    ART_DIAG_STEP(nsteps);
    int cc, tid;
    float dd;
    const bool h = leaf_slot_test<OBB, PERM>(s, br, (leaf - leaf0) * kBvhLeaf + qd, cc, dd, tid, nt, sc.obbc);
    // no hit, NaN and FLT_MAX-or-more never win (strict < against float.MaxValue; the permeation
    // cast: against INFINITY, so a hit at FLT_MAX counts). A hit distance is >= 0 or -0, so the key
    // (distance bits, order code) orders as the reference's sequential strict-< first minimum.
    const unsigned long long k = quad_min_u64(h && (PERM ? dd < INFINITY : dd < FLT_MAX) ? nearest_key(dd, cc) : ~0ull);
    if (k < mykey) {
      mykey = k;
      const float d = __uint_as_float((uint32_t)(k >> 32));
      lim = fminf(lim, d);
      if (ART_NEAREST_STEAL && shared && qd == 0) atomicMin(s_bound + home, __float_as_int(d));
    }
  };
  // Speculative while-while (Aila & Laine): a quad that reaches a leaf parks it and keeps
  // descending; the wave tests leaves once every quad with work holds one, so both kinds of step
  // run with most quads busy. The order in which leaves are tested does not change the minimum.
  int pend = -1;
  for (;;) {
    const unsigned long long act = __builtin_amdgcn_ballot_w64((g & pend) >= 0) & kQuad0;  // g >= 0 || pend >= 0
    if (!act) break;
    {  // Wave priority by unfinished rays: the waves with the most rays left (the ones that set the
       // kernel's length) issue first, the nearly finished ones fill the gaps (s_setprio, 0..3)
      const int na = pop64(act);
      if (na > 12) __builtin_amdgcn_s_setprio(3);
      else if (na > 8) __builtin_amdgcn_s_setprio(2);
      else if (na > 4) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    if (ART_NEAREST_STEAL) {
      const unsigned long long donors = __builtin_amdgcn_ballot_w64(sp > bp) & kQuad0, idle = ~act & kQuad0;
      if (donors && pop64(idle) >= ART_STEAL_MIN_IDLE) {  // wave-uniform: the k-th idle quad takes the k-th donor's stack bottom
        if (!shared) {       // publish every ray's bound once
          shared = true;
          if (qd == 0) s_bound[wq] = __float_as_int(lim);
        }
        // (the quad's lane masks are recomputed here, not hoisted out of the loop: four live VGPRs)
        int l4 = lane & ~3;
        asm volatile("" : "+v"(l4));
        const unsigned long long below = (1ull << l4) - 1ull;
        const int ir = pop64(idle & below), dr = pop64(donors & below);
        const bool thief = (act >> l4 & 1ull) == 0ull && ir < pop64(donors);
        const bool robbed = sp > bp && dr < pop64(idle);
        const int match = rank_match(l4, qd, robbed, dr, ir);  // (every lane takes part)
        const int src = (thief ? match : l4) + qd;
        const int dbp = __shfl(bp, src), dhome = __shfl(home, src);
        const float ox = __shfl(s.o.x, src), oy = __shfl(s.o.y, src), oz = __shfl(s.o.z, src);
        const float dx = __shfl(s.d.x, src), dy = __shfl(s.d.y, src), dz = __shfl(s.d.z, src);
        const float dlim = __shfl(lim, src);
        // the ray's derived values too (1/d, 2a, |o|_1, force: the home's own values, so no divisions)
        const float ix = __shfl(s.inv.x, src), iy = __shfl(s.inv.y, src), iz = __shfl(s.inv.z, src);
        const float da2 = __shfl(s.a2, src), dom = __shfl(om, src);
        const int dforce = __shfl((int)force, src);
        if (thief && mykey != ~0ull && qd == 0) atomicMin(s_key + home, mykey);
        if (thief) {
          g = (int)s_wave[(src >> 2) * kBvhStack + dbp];
          sp = bp = 0;
          home = dhome;
          s.o = mk3(ox, oy, oz); s.d = mk3(dx, dy, dz); s.inv = mk3(ix, iy, iz); s.a2 = da2;
          om = dom;
          force = dforce != 0;
          lim = dlim;
          mykey = ~0ull;  // (the finished ray's result went to its key above)
        }
        fmk = __builtin_amdgcn_ballot_w64(force);
        if (robbed && ++bp == sp) sp = bp = 0;
      }
      if (shared) lim = fminf(lim, __int_as_float(s_bound[home]));
    }
    for (;;) {
      if (g >= leaf0 && pend < 0) { pend = g; pop(); }
      const bool inner = g >= 0 && g < leaf0;
#if ART_NEAREST_ONE_ANY
      // (after the park above, a quad with no parked leaf and a node holds an inner node, so "some
      // quad has no parked leaf and work" implies "some quad is inner": one ballot decides)
      if (__builtin_amdgcn_ballot_w64((pend & ~g) < 0) == 0ull) break;  // pend < 0 && g >= 0, one compare
#else
      if (!__any(inner) || !__any(pend < 0 && g >= 0)) break;
#endif
      if (inner) inner_step();
    }
    if (pend >= 0) { leaf_step(pend); pend = -1; }
  }
#ifdef ART_DIAG
  if (qd == 0 && alive) diag_add(2, nsteps);
#endif
  unsigned long long k = mykey;
  if (ART_NEAREST_STEAL && shared) {  // the ray's result: the minimum over the quads that traversed it
    if (mykey != ~0ull && qd == 0) atomicMin(s_key + home, mykey);
    k = s_key[wq];
  }
  best = k == ~0ull ? FLT_MAX : __uint_as_float((uint32_t)(k >> 32));
  code = k == ~0ull ? kNoHit : (int)(uint32_t)k;
  if (ex) {
    exec_add(ex + kExecNearest, kExecSphere, wave_sum_u32(nt[0]));
    exec_add(ex + kExecNearest, kExecAabb, wave_sum_u32(nt[1]));
    exec_add(ex + kExecNearest, kExecObb, wave_sum_u32(nt[2]));
    exec_add(ex + kExecNearest, kExecCullBox, 4ull * wave_sum_u32(nnode));
  }
}

// ------------------------------------------------------------------------------------------
// Nearest hits of one bounce: one 64-ray group per workgroup, wave w traverses rays 16w .. 16w+15
// with 4 lanes each (quad_nearest_core), 8 waves per SIMD. hits[g * 64 + r] = (distance bits,
// code) of the group's ray slot r. Bounce 0 starts every ray at its fan's origin; later bounces
// read the path kernel's ray state and traverse only the rays its live list holds (the workgroups
// past the list return at once).
// ------------------------------------------------------------------------------------------
constexpr int kLiveCounters = 32;  // per-bounce live-list counters (H <= 32)

// Ray state between bounce launches: [groups * 64][2] float4 (o, life | d, hits | alive << 8),
// then the live list u32[groups * 64], its per-bounce counters u32[kLiveCounters] and the echo
// pairs each bounce emitted u32[kLiveCounters] (bounce k's echo pairs follow bounce k-1's).
__device__ __forceinline__ uint32_t* live_list(float4* state, int ngroups) {
  return reinterpret_cast<uint32_t*>(state + 2 * (size_t)ngroups * 64);
}
__device__ __forceinline__ uint32_t* echo_counts(float4* state, int ngroups) {
  return live_list(state, ngroups) + (size_t)ngroups * 64 + kLiveCounters;
}

// Visibility work (struct of arrays, below): echo segments and outputs, hit records. `fixed`
// (multi-hit frames with one batch slot and no hit outputs, nearest_first_kernel<..., FOLD>): the
// records sit at fixed positions bounce * fixed + ray slot and are compact (round 6): no echo
// segment, out = (echo distance bits, echo half) with out.y = kNoRecord marking a slot with no hit
// that bounce (then nothing else is written for it), hrec = (off.xyz, muffle destination); the
// echo traversal rebuilds the segment from off and the fan origin, and the echo's index from the
// slot (fold_path).
constexpr uint32_t kNoRecord = 0xffffffffu;
struct VisPairs {
  float4* seg;
  uint2* out;
  float4* hrec;
  uint32_t echo_cap;  // multiple of 64
  uint32_t fixed;     // 0: records compacted in emission order; else ray slots per bounce
};

__device__ __forceinline__ float echo_of(const DevScene& sc, int type, int idx) {
  return type == kSphere ? sc.sphc[idx].echo : (type == kAabb ? sc.aabbc[idx].echo : sc.obbc[idx].echo);
}

// ReflectRay (:456-532) at hit point o of collider (type, idx), then the offset (:528) and the
// absorption (:531); false when the ray's life runs out (:189).
__device__ __forceinline__ bool reflect_at_hit(const DevScene& sc, const FrameParams& fp, int type, int idx, vec3& o, vec3& d,
                                               float& life) {
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
    const ObbCold bc2 = sc.obbc[idx];
    vec3 lh = qmul(inverse_q(bc2), o - mk3(b.cx, b.cy, b.cz));  // :489 (Q5: inverse of the stored inverse)
    vec3 ap = abs3(lh);
    vec3 df = mk3(bc2.hx, bc2.hy, bc2.hz) - ap;
    vec3 ln = mk3(0.0f, 0.0f, 0.0f);
    if (df.x < df.y && df.x < df.z) ln.x = usign(lh.x);
    else if (df.y < df.x && df.y < df.z) ln.y = usign(lh.y);
    else ln.z = usign(lh.z);
    n = qmul(stored_q(b), ln);                                 // :510
    absorption = bc2.absorption;
  } else {
    const SphereRec c = sc.sph[idx];
    n = normalize(o - mk3(c.cx, c.cy, c.cz));                  // :516
    absorption = sc.sphc[idx].absorption;
  }
  d = reflect(d, n);                    // :525
  o = o + d * kEps;                     // :528
  life -= fp.max_life * absorption;     // :531
  return !(life < 0.0f);
}

// The winner's collider from its order code, and the exact (Unity min / max) re-evaluation of a zero
// distance (IEEE and Unity min / max differ only in the sign of an equal-magnitude zero pair).
__device__ __forceinline__ void winner_of(const DevScene& sc, const Seg& s, int code, int& type, int& idx, float& dist) {
  const int rank = code >> 28;
  idx = code & 0x0fffffff;
  type = rank == 0 ? kSphere : (rank == 1 ? kAabb : kObb);
  if (dist == 0.0f) {
    if (type == kSphere) sphere_hit_dist(s, sc.sph[idx], dist);  // (a -0 the result key made +0)
    if (type == kAabb) aabb_test<true>(s, sc.aabb[idx], dist);
    if (type == kObb) { const ObbRec r = sc.obb[idx]; obb_test<true>(s, r, stored_q(r), dist); }
  }
}
// FOLD (multi-hit frames with one batch slot and no hit outputs): the path kernel's work for each
// ray runs in this kernel's epilogue (fold_path), every ray keeps its slot for all bounces (no live
// list: a finished ray's quad only helps the others through work sharing), and the echo segments and
// hit records go to fixed per-bounce slots (VisPairs::fixed): no path launch and no reservation
// atomics per bounce.
__device__ __forceinline__ void fold_path(const DevScene& sc, const FrameParams& fp, const FanLayout& L, uint8_t* block,
                                          const float* origins, const VisPairs& vp, float4* state, int step, uint32_t sidx,
                                          int fan, int ray,
                                          bool slot_ok, vec3 o, vec3 d, float life, int hits, bool alive, float dist, int code,
                                          bool lead) {
  const int H = fp.H;
  const vec3 O = load3(origins, fan);
  const bool hit = alive && code != kNoHit;
  int type = kNone, idx = 0;
  if (hit) {
    winner_of(sc, make_seg(o, d), code, type, idx, dist);
    o = o + d * dist;  // :111
    life -= dist;      // :112
    hits += 1;         // :113
  }
  uint16_t* echo = reinterpret_cast<uint16_t*>(block + (size_t)fan * L.stride + L.echo_off);
  const size_t rec = (size_t)step * vp.fixed + sidx;
  if (lead) {  // this bounce's echo ray (:124-145) and the muffle rays' hit record (:150-173), or none
    if (hit) {   // (the echo's index is ray * H + hits - 1 = ray * H + step: every earlier bounce hit)
      const vec3 off = o - d * kEps;                 // :124, :158
      const float dist0 = distance(O, o);            // :130 (un-offset hit point)
      vp.out[rec] = make_uint2(__float_as_uint(dist0), f32tof16(dist0 * echo_of(sc, type, idx)));  // :142-144
      vp.hrec[rec] = make_float4(off.x, off.y, off.z, __uint_as_float((uint32_t)fan * (uint32_t)fp.T));  // batch slot 0
      echo[ray * H + hits - 1] = 0;  // a blocked echo keeps the reset value (:76); the echo traversal stores the rest
    } else {
      vp.out[rec] = make_uint2(0u, kNoRecord);
    }
  }
  // termination / reflection (:179-193, ReflectRay :456-532)
  bool next = hit;  // a miss ends the ray (:200-207)
  if (hit) next = (hits >= H || life <= 0.0f) ? false : reflect_at_hit(sc, fp, type, idx, o, d, life);
  if (lead && slot_ok && alive) {  // (an ended ray's state already says so: later bounces leave it)
    state[2 * (size_t)sidx] = make_float4(o.x, o.y, o.z, life);
    state[2 * (size_t)sidx + 1] = make_float4(d.x, d.y, d.z, __int_as_float(hits | (next ? 256 : 0)));
    if (alive && !next)  // the ray stops here: slots past its last hit keep the reset value 0 (:72-80)
      for (int k = hits; k < H; ++k) echo[ray * H + k] = 0;
  }
}

// EX: count the executed tests (fp.exec); OBB: the scene has OBBs; FOLD: fold_path above.
// TAB (bounce 0 only, 64-ray groups per fan a multiple of 4, <= kTabNodes BVH nodes): workgroups of
// 1024 lanes, the 4 consecutive 64-ray groups of one fan, all rays at the fan origin, traverse with
// the shared-origin node table in LDS (node_table_build; 2 workgroups and 8 waves per SIMD per CU,
// 70 KB of LDS each).
template <bool EX, bool OBB, bool FOLD, bool TAB = false>
__global__ __launch_bounds__(TAB ? 1024 : 256) __attribute__((amdgpu_waves_per_eu(kNearestWaves<EX, OBB>))) void nearest_first_kernel(
    DevScene sc, FrameParams fp, const float* __restrict__ origins, const int* __restrict__ ray_order,
    int2* __restrict__ hits, float4* __restrict__ state, int step, uint32_t* __restrict__ zero, uint32_t nzero,
    uint32_t* __restrict__ counters, FanLayout L, uint8_t* __restrict__ block, VisPairs vp) {
  constexpr int kGroupsPerWg = TAB ? 4 : 1;
  __shared__ uint32_t s_stk[kBvhStack * 64 * kGroupsPerWg];
  __shared__ int s_bound[64 * kGroupsPerWg];
  __shared__ unsigned long long s_key[64 * kGroupsPerWg];
  __shared__ std::conditional_t<TAB, NodeTab, int> s_tab;
  ART_WAVE_TIMER(0);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nrb = (fp.R + 63) >> 6;
  const int ngroups = fp.S * nrb;
  const int g = (int)blockIdx.x * kGroupsPerWg + (w >> 2);  // TAB: 4 groups of one fan per workgroup
  const int rr = 16 * (w & 3) + (lane >> 2);
  uint32_t* my = s_stk + (16 * w + (lane >> 2)) * kBvhStack;
  if constexpr (TAB) {  // the fan origin's node table (every ray of the workgroup starts there)
    if (ART_TAB_USE >= 0) {
      node_table_build(sc, load3(origins, g / nrb), &s_tab);
      __syncthreads();
    }
  }
  unsigned long long* ex = EX ? fp.exec : nullptr;
  float best;
  int code;
  vec3 o, d;
  bool alive, write;
  uint32_t out;  // ray slot (< 2^31: fast_fans_per_launch)
  float life = fp.max_life;
  int nhits = 0, fan = 0, ray = 0;
  bool slot_ok = true;
  if (FOLD) {  // every ray in its slot for every bounce
    if (step == 0) {
      for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nzero; i += gridDim.x * blockDim.x) zero[i] = 0u;
      if (counters && blockIdx.x == 0 && threadIdx.x < 4) counters[threadIdx.x] = 0u;
    }
    fan = g / nrb;
    const int sl = (g - fan * nrb) * 64 + rr;
    slot_ok = sl < fp.R;
    ray = slot_ok ? ray_order[sl] : 0;
    out = (uint32_t)g * 64u + (uint32_t)rr;
    if (step == 0) {
      o = load3(origins, fan);
      d = load_dir(sc.dirs, ray);
      alive = slot_ok;
    } else {
      const float4 a = state[2 * (size_t)out], b = state[2 * (size_t)out + 1];
      o = mk3(a.x, a.y, a.z);
      life = a.w;
      d = mk3(b.x, b.y, b.z);
      nhits = __float_as_int(b.w) & 0xff;
      alive = slot_ok && ((__float_as_int(b.w) >> 8) & 1) != 0;
    }
    write = false;
  } else if (step > 0) {  // the previous bounce's list of live ray slots
    const uint32_t* live = live_list(state, ngroups);
    const uint32_t cnt = live[(size_t)ngroups * 64 + step];
    if ((uint32_t)g * 64u >= cnt) return;  // the whole workgroup: past the list
    const uint32_t e = (uint32_t)g * 64u + (uint32_t)rr;
    const bool ok = e < cnt;
    const uint32_t i = ok ? live[e] : 0u;
    const float4 a = state[2 * (size_t)i], b = state[2 * (size_t)i + 1];
    o = mk3(a.x, a.y, a.z);
    d = mk3(b.x, b.y, b.z);
    alive = ok && ((__float_as_int(b.w) >> 8) & 1) != 0;
    write = ok;
    out = i;
    asm volatile("" : "+v"(out));  // (a 32-bit copy, apart from the 64-bit state offset above)
  } else {
    if (state && blockIdx.x == 0 && threadIdx.x < 2 * kLiveCounters)  // multi-hit frame: clear the counters
      live_list(state, ngroups)[(size_t)ngroups * 64 + threadIdx.x] = 0u;
    // the frame's muffle accumulators and pair counters, consumed only by later launches (no
    // memset dispatch between frames)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nzero; i += gridDim.x * blockDim.x) zero[i] = 0u;
    if (counters && blockIdx.x == 0 && threadIdx.x < 4) counters[threadIdx.x] = 0u;
    const int fan = g / nrb;
    const int slot = (g - fan * nrb) * 64 + rr;
    alive = slot < fp.R;
    const int ray = alive ? ray_order[slot] : 0;
    o = load3(origins, fan);
    d = load_dir(sc.dirs, ray);
    write = true;
    out = (uint32_t)g * 64u + (uint32_t)rr;
  }
  if (EX && step < kExecBounces)  // live rays traced this bounce (one per quad)
    exec_add(ex, kExecBounce0 + step, (unsigned long long)__popcll(__builtin_amdgcn_ballot_w64(alive) & kQuad0));
#ifdef ART_DIAG
  const unsigned long long t0 = clock64();
#endif
  quad_nearest_core<EX, OBB, false, TAB>(sc, make_seg(o, d), alive, lane, my, s_bound + 16 * w, s_key + 16 * w, best, code,
                                         ex, TAB ? reinterpret_cast<const NodeTab*>(&s_tab) : nullptr);
  if (FOLD) {
    // The ray's state is fetched again rather than kept live across the traversal (a memory
    // clobber: the compiler may not reuse the values loaded before it): 64 VGPRs, no spills.
    asm volatile("" ::: "memory");
    {
      const int rr2 = 16 * (w & 3) + (lane >> 2);
      fan = g / nrb;
      const int sl = (g - fan * nrb) * 64 + rr2;
      slot_ok = sl < fp.R;
      ray = slot_ok ? ray_order[sl] : 0;
      out = (uint32_t)g * 64u + (uint32_t)rr2;
      if (step == 0) {
        o = load3(origins, fan);
        d = load_dir(sc.dirs, ray);
        life = fp.max_life;
        nhits = 0;
        alive = slot_ok;
      } else {
        const float4 a = state[2 * (size_t)out], b = state[2 * (size_t)out + 1];
        o = mk3(a.x, a.y, a.z);
        life = a.w;
        d = mk3(b.x, b.y, b.z);
        nhits = __float_as_int(b.w) & 0xff;
        alive = slot_ok && ((__float_as_int(b.w) >> 8) & 1) != 0;
      }
    }
    if (EX) exec_add(fp.exec, kExecEchoPairs, (unsigned long long)__popcll(__builtin_amdgcn_ballot_w64(alive && code != kNoHit) & kQuad0));
    fold_path(sc, fp, L, block, origins, vp, state, step, out, fan, ray, slot_ok, o, d, life, nhits, alive, best, code,
              (lane & 3) == 0);
    return;
  }
  // (the ray slot stays a 32-bit value across the traversal: an opaque copy keeps the compiler from
  // widening it to a 64-bit offset before the loop, two more live VGPRs)
  asm volatile("" : "+v"(out));
  if ((lane & 3) == 0 && write) hits[out] = make_int2(__float_as_int(best), code);
#ifdef ART_DIAG
  if (lane == 0) diag_add(0, clock64() - t0);
#endif
}

// ------------------------------------------------------------------------------------------
// Visibility work. The path kernel emits every echo ray and one hit record per hit; visibility
// never feeds back into ray paths (echo :124-145 and muffle :150-173 only write outputs), so the
// verdicts can be computed beside the next bounces. Struct of arrays:
//   seg[2 i], seg[2 i + 1]  echo pair i, emission order: (o.xyz, maxd), (d.xyz, kNoOwner) 32 B, read by
//                           the echo traversal (1/d and dot(d, d) recomputed by make_seg)
//   out[i]                  (u16 index of the echo in the fan blocks, echo half) 8 B: the traversal
//                           stores the half when no collider blocks the ray
//   hrec[j]                 hit record j: (off.xyz, dest) 16 B — the muffle rays' common start
//                           (:158) and the muffle accumulator index (fan * TC + batch slot) * T of
//                           target 0; muffle_kernel casts its T rays
// counts[0] / counts[1] = echo pairs / hit records emitted.
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ void load_pair_seg(const VisPairs& vp, uint32_t i, Seg& s, float& maxd, int& owner) {
  const float4 q0 = vp.seg[2 * (size_t)i], q1 = vp.seg[2 * (size_t)i + 1];
  s = make_seg(mk3(q0.x, q0.y, q0.z), mk3(q1.x, q1.y, q1.z));
  maxd = q0.w;
  owner = __float_as_int(q1.w);
}



// ------------------------------------------------------------------------------------------
// Path kernel: everything of one bounce of AudioRaytracerJobBatched.Execute (:61-215) except the
// nearest-hit search (nearest_first_kernel's hits). 8 independent waves per workgroup, one 64-ray
// group each (grid-stride); the waves reserve their pair positions with one atomic per region for
// the whole workgroup (one per wave: same-line atomics serialize). MULTI (H > 1): one launch per
// bounce; the ray state (o, life | d, hits, alive) carries over in `state`, and the rays still
// alive are appended to the next bounce's live list.
// ------------------------------------------------------------------------------------------
constexpr int kPathWaves = 8;

template <bool HITS, bool MULTI>
__global__ __launch_bounds__(64 * kPathWaves) __attribute__((amdgpu_waves_per_eu(4))) void path_kernel(
    DevScene sc, FrameParams fp, FanLayout L, const float* __restrict__ origins, uint8_t* __restrict__ block,
    const int* __restrict__ ray_order, VisPairs vp, uint32_t* __restrict__ pair_count,
    const int2* __restrict__ pre_hits, float4* __restrict__ state, int step, int emit_echo) {
  constexpr int K = kPathWaves;
  __shared__ uint32_t s_agg[2][K][2];
  __shared__ uint32_t s_aggb[2][2];
  __shared__ uint32_t s_live[2][K], s_liveb[2];
  int agg_round = 0;  // block-uniform reservation round (the LDS buffers alternate by its parity)
  __builtin_amdgcn_s_setprio(3);  // on the critical path; in multi-hit frames the echo traversal runs beside it
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nrb = (fp.R + 63) >> 6;  // 64-ray groups per fan
  const int ngroups = fp.S * nrb;
  const int T = fp.T, H = MULTI ? fp.H : 1;
  const unsigned long long lt = (1ull << lane) - 1ull;
  // one reservation for the workgroup: returns this wave's base in each of the two regions
  auto reserve = [&](uint32_t n0, uint32_t n1, uint32_t* counter, uint32_t& b0, uint32_t& b1) {
    const int par = agg_round++ & 1;
    if (lane == 0) { s_agg[par][w][0] = n0; s_agg[par][w][1] = n1; }
    __syncthreads();
    if (threadIdx.x < 2) {
      uint32_t t = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) t += s_agg[par][k][threadIdx.x];
      s_aggb[par][threadIdx.x] = t ? atomicAdd(&counter[threadIdx.x], t) : 0u;
      if (MULTI && threadIdx.x == 0 && t) atomicAdd(echo_counts(state, ngroups) + step, t);  // bounce step's echoes
    }
    __syncthreads();
    b0 = s_aggb[par][0];
    b1 = s_aggb[par][1];
    for (int k = 0; k < w; ++k) { b0 += s_agg[par][k][0]; b1 += s_agg[par][k][1]; }
  };
  for (int g = (int)blockIdx.x * K + w;; g += (int)gridDim.x * K) {
    if (g - w >= ngroups) break;  // block-uniform: a wave past the end takes part with no rays
    const bool gvalid = g < ngroups;
    const int fan = gvalid ? g / nrb : 0;
    const int slot = gvalid ? (g - fan * nrb) * 64 + lane : fp.R;
    const bool valid = slot < fp.R;
    const int ray = valid ? ray_order[slot] : 0;
    uint8_t* fb = block + (size_t)fan * L.stride;
    uint16_t* echo = reinterpret_cast<uint16_t*>(fb + L.echo_off);
    art_half3* hpo = reinterpret_cast<art_half3*>(fb + L.hit_points_off);
    uint32_t* hid = reinterpret_cast<uint32_t*>(fb + L.hit_ids_off);
    const bool single_slot = fp.TC == 1;
    const int my_slot = (int)(((long long)((ray / fp.bs) * fp.bs) * fp.TC) / fp.R);  // batchId (:63-64)

    // Reset (:72-80) with sequential-batch semantics (TC > 1 only; at TC == 1 every slot is written
    // once below): frozen bit k = a later batch resets this ray's slot k.
    uint32_t frozen = 0;
    if (valid) {
      const int my_batch = ray / fp.bs;
      const art_half3 z = {0, 0, 0};
      for (int k = 0; k < H; ++k) {
        const int j = ray * H + k;
        bool any_reset;
        const int keep = batch_slot_state(fp, j, my_batch, any_reset);
        if (!keep) frozen |= 1u << k;
        if (!single_slot && (!keep || any_reset) && step == 0) {
          echo[j] = 0;
          if (HITS) { hpo[j] = z; hid[j] = ART_HIT_NONE; }
        }
      }
    }

    const vec3 O = load3(origins, fan);
    vec3 o = O;
    vec3 d = load_dir(sc.dirs, valid ? ray : 0);
    float life = fp.max_life;
    int hits = 0;
    bool alive = valid;
    const size_t sidx = (size_t)g * 64 + lane;  // ray slot of the state / hit arrays
    if (MULTI && step > 0 && valid) {
      const float4 a = state[2 * sidx], b = state[2 * sidx + 1];
      o = mk3(a.x, a.y, a.z);
      life = a.w;
      d = mk3(b.x, b.y, b.z);
      hits = __float_as_int(b.w) & 0xff;
      alive = ((__float_as_int(b.w) >> 8) & 1) != 0;
    }
    const bool alive0 = alive;

    // this bounce's nearest hit (nearest_first_kernel)
    const Seg s = make_seg(o, d);
    const int2 ph = gvalid ? pre_hits[sidx] : make_int2(__float_as_int(FLT_MAX), kNoHit);
    const int bc = ph.y;
    const bool hit = alive && bc != kNoHit;
    alive = hit;  // a miss ends the ray (:200-207)
    int type = kNone, idx = 0;
    float dist = __int_as_float(ph.x);
    if (hit) {
      winner_of(sc, s, bc, type, idx, dist);
      o = o + d * dist;  // :111
      life -= dist;      // :112
      hits += 1;         // :113
    }
    const int k = hits - 1;
    const bool live_slot = hit && !((frozen >> k) & 1u);
    if (HITS && live_slot) {  // :118, :197
      art_half3 p;
      p.x = f32tof16(o.x); p.y = f32tof16(o.y); p.z = f32tof16(o.z);
      hpo[ray * H + k] = p;
      hid[ray * H + k] = ART_HIT_ID(type, idx);  // ShootRayCast's (hitColliderType, collider) :225-280
    }

    // the echo ray to the fan origin (:124-145), emitted into a live slot only (:118), and the hit
    // record the T muffle rays start from (:150-173); one reservation for the workgroup
    const vec3 off = o - d * kEps;                 // :124, :158
    const float dist0 = distance(O, o);            // :130 (un-offset hit point)
    {
      const unsigned long long me = __builtin_amdgcn_ballot_w64(live_slot), mr = __builtin_amdgcn_ballot_w64(hit);
      exec_add(fp.exec, kExecEchoPairs, (unsigned long long)__popcll(me));
      uint32_t eb, rb;
      reserve(emit_echo ? (uint32_t)__popcll(me) : 0u, (uint32_t)__popcll(mr), pair_count, eb, rb);
      if (emit_echo && live_slot) {
        const uint32_t at = eb + (uint32_t)__popcll(me & lt);
        const vec3 qdir = normalize(O - off);
        vp.seg[2 * (size_t)at] = make_float4(off.x, off.y, off.z, dist0);
        vp.seg[2 * (size_t)at + 1] = make_float4(qdir.x, qdir.y, qdir.z, __int_as_float(kNoOwner));
        vp.out[at] = make_uint2((uint32_t)(((size_t)fan * L.stride + L.echo_off) / 2) + (uint32_t)(ray * H + k),
                                f32tof16(dist0 * echo_of(sc, type, idx)));  // :142-144
      }
      if (hit) {
        const uint32_t at = rb + (uint32_t)__popcll(mr & lt);
        vp.hrec[at] = make_float4(off.x, off.y, off.z, __uint_as_float((uint32_t)(((size_t)fan * fp.TC + my_slot) * T)));
      }
    }
    // a blocked echo leaves the reset value (:76); the echo traversal overwrites the visible ones
    // (or, tracing from the hits (!emit_echo), writes both itself)
    if (emit_echo && live_slot && single_slot) echo[ray * H + k] = 0;

    // termination / reflection — :179-193, ReflectRay :456-532
    if (!MULTI) {
      alive = false;  // hits >= H == 1 after the first hit; a miss has already ended the ray
    } else if (hit) {
      if (hits >= H || life <= 0.0f) {
        alive = false;
      } else {
        alive = reflect_at_hit(sc, fp, type, idx, o, d, life);
      }
    }
    if (MULTI) {
      if (valid) {  // the next launch's ray state (a ray that stopped records alive = 0)
        state[2 * sidx] = make_float4(o.x, o.y, o.z, life);
        state[2 * sidx + 1] = make_float4(d.x, d.y, d.z, __int_as_float(hits | (alive ? 256 : 0)));
      }
      // the rays still alive: the next bounce's traversal list (one reservation per workgroup)
      uint32_t* live = live_list(state, ngroups);
      uint32_t* live_n = live + (size_t)ngroups * 64;
      const bool app = valid && alive && step + 1 < fp.H;
      const unsigned long long m = __builtin_amdgcn_ballot_w64(app);
      const int par = agg_round++ & 1;
      if (lane == 0) s_live[par][w] = (uint32_t)__popcll(m);
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int kk = 0; kk < K; ++kk) t += s_live[par][kk];
        s_liveb[par] = t ? atomicAdd(&live_n[step + 1], t) : 0u;
      }
      __syncthreads();
      uint32_t base = s_liveb[par];
      for (int kk = 0; kk < w; ++kk) base += s_live[par][kk];
      if (app) live[base + (uint32_t)__popcll(m & lt)] = (uint32_t)sidx;
    }
    if (valid && (!MULTI || (alive0 && !alive))) {  // in the launch where the ray stops
      if (single_slot) {  // slots past the last hit keep the reset value 0 (:72-80)
        const art_half3 z = {0, 0, 0};
        for (int kk = hits; kk < H; ++kk) {
          echo[ray * H + kk] = 0;
          if (HITS) { hpo[ray * H + kk] = z; hid[ray * H + kk] = ART_HIT_NONE; }
        }
      }
      if (HITS) fb[L.hit_counts_off + ray] = (uint8_t)hits;  // :204, :212
    }
  }
}

// ------------------------------------------------------------------------------------------
// Echo visibility by quad-per-segment BVH traversal. An echo batch is one wave's rays of one fan
// traced back to the fan origin: 64 segments fanning over an eighth of the sphere, whose box and
// cone admit ~10 % of the colliders, so a sweep would spend most of its time there. Per segment
// the BVH visits only the nodes along it: a segment enters a node when its widened box is entered
// before maxd (a blocker's computed distance d < maxd lies strictly after every ancestor's
// entry), 4 lanes per segment (lane q: child q / leaf slot q; the quad agrees through ballots),
// the first blocker ends the segment; a segment no collider blocks stores its echo.
// Work sharing inside the wave: a wave lasts as long as its longest traversal, so a quad whose
// traversal has ended takes over the bottom entry of a busy quad's stack (the largest pending
// subtree) together with that quad's segment, and traverses it for the segment's home quad. The
// subtrees of a segment are then split between quads; any of them finding a blocker marks the home
// blocked (wave-uniform mask), which ends every traversal of that segment. Any-hit is an OR over
// the subtrees, so the split does not change a verdict.
// ------------------------------------------------------------------------------------------
// One-hit frames with one batch slot (H == 1, TC == 1) trace the echo rays straight from the
// nearest hits (HM: `blk` = a 64-ray group), so the traversal does not wait for the path kernel:
// the segment, its output index and value are the path kernel's own expressions (:111, :124-145,
// the zero-distance re-evaluation included), and the traversal stores the echo half or, when a
// collider blocks it, the reset value 0 (the path kernel, running beside it, then leaves those
// slots alone). With H == 1 no later batch resets a ray's slot, so every hit slot is live.
struct EchoFromHits {
  FrameParams fp;
  FanLayout L;
  const float* origins;
  const int* ray_order;
  const int2* pre;
  int no_path;  // the frame runs no path kernel: the echo traversal writes the misses' reset 0 and counts the echo rays
};
// The hit of ray slot r of 64-ray group g from its nearest-hit record, as path_kernel computes it
// (:111, :124, the zero-distance re-evaluation included): false for a slot past the fan's rays
// (slot_ok false) or a miss.
__device__ __forceinline__ bool hit_from_pre(const DevScene& sc, const EchoFromHits& eh, uint32_t g, int r, bool& slot_ok,
                                             int& fan, int& ray, vec3& O, vec3& o, vec3& off, int& type, int& idx) {
  const FrameParams& fp = eh.fp;
  const int nrb = (fp.R + 63) >> 6;
  fan = (int)(g / (uint32_t)nrb);
  const int slot = (int)(g - (uint32_t)fan * nrb) * 64 + r;
  slot_ok = fan < fp.S && slot < fp.R;
  if (!slot_ok) return false;
  ray = eh.ray_order[slot];
  const int2 ph = eh.pre[(size_t)g * 64 + r];
  if (ph.y == kNoHit) return false;  // a miss: no echo ray, no muffle rays
  O = load3(eh.origins, fan);
  const vec3 d = load_dir(sc.dirs, ray);
  const Seg s0 = make_seg(O, d);
  const int rank = ph.y >> 28;
  idx = ph.y & 0x0fffffff;
  type = rank == 0 ? kSphere : (rank == 1 ? kAabb : kObb);
  float dist = __int_as_float(ph.x);
  if (dist == 0.0f) {  // as path_kernel
    if (type == kSphere) sphere_hit_dist(s0, sc.sph[idx], dist);
    if (type == kAabb) aabb_test<true>(s0, sc.aabb[idx], dist);
    if (type == kObb) { const ObbRec rr = sc.obb[idx]; obb_test<true>(s0, rr, stored_q(rr), dist); }
  }
  o = O + d * dist;      // :111
  off = o - d * kEps;    // :124, :158
  return true;
}
__device__ __forceinline__ bool echo_seg_from_hit(const DevScene& sc, const EchoFromHits& eh, uint32_t g, int r, Seg& s,
                                                  float& maxd, uint32_t& out_at, uint16_t& out_val, bool& slot_ok) {
  int fan = 0, ray = 0, type = kNone, idx = 0;
  vec3 O, o, off;
  const bool hit = hit_from_pre(sc, eh, g, r, slot_ok, fan, ray, O, o, off, type, idx);
  out_at = slot_ok ? (uint32_t)(((size_t)fan * eh.L.stride + eh.L.echo_off) / 2) + (uint32_t)ray : 0u;  // ray * H + 0
  if (!hit) return false;
  const float dist0 = distance(O, o);            // :130
  s = make_seg(off, normalize(O - off));
  maxd = dist0;
  out_val = (uint16_t)f32tof16(dist0 * echo_of(sc, type, idx));   // :142-144
  return true;
}

// Any-hit traversal of the wave's 16 segments, one per quad (lane & 3 = the quad's child / slot;
// s_wave = the wave's 16 stacks of kBvhStack entries): true in every lane of a quad whose segment
// no collider blocks (hit and d < maxd, tid != owner: CanRaySeePoint :365-397 / :411-447 with
// owner = the target). `valid` must be quad-uniform; an invalid segment is reported visible.
// Work sharing as in the nearest traversal (a blocker of a shared segment ends every traversal of
// it); nt / nnode accumulate the exact tests and node visits (EX counters).
template <bool OBB, bool PARK = false>
__device__ __forceinline__ bool quad_echo_core(const DevScene& sc, Seg s, float maxd, int owner, bool valid, int lane,
                                               uint32_t* s_wave, unsigned* nt, unsigned& nnode) {
  const int qd = lane & 3, wq = lane >> 2;
  if (sc.bvh_levels == 0) return true;                         // no colliders: nothing blocks
  float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
  bool force = force_all(s, om);
  unsigned long long fmk = __builtin_amdgcn_ballot_w64(force);  // (the forced lanes as a lane mask, as in the nearest core)
  const int leaf0 = sc.bvh_leaf0, qshift = lane & ~3;
  const BvhRes br = bvh_res(sc);
  uint32_t* const my = s_wave + wq * kBvhStack;                // entries [bp, sp) pending
  uint32_t wblocked = 0u;                                      // wave-uniform: home quads found blocked
  int home = wq;
  int g = valid ? 0 : -1, sp = 0, bp = 0;
  unsigned nsteps = 0;
  (void)nsteps;
#ifdef ART_DIAG
  const unsigned long long t0 = clock64();
#endif
  auto pop = [&]() {
    const bool has = sp > bp;
    const int t = (int)my[has ? sp - 1 : 0];
    g = has ? t : -1;
    sp = has ? sp - 1 : sp;
    if (sp == bp) sp = bp = 0;
  };
  // PARK: the speculative while-while of the nearest traversal (a quad that reaches a leaf parks it
  // and keeps descending; the wave tests leaves once every quad with work holds one), so a quad
  // that found its leaf early does not idle while the others descend. Any-hit needs every entered
  // leaf tested anyway, so the order changes nothing but the lanes' occupancy. Measured (round 6):
  // the echo half of echo_muffle_kernel config 2 53.0 -> 50.9 us, config 4 495 -> 490 us; the
  // folded frames' vis_kernel (config 5) 440 -> 444 us, so vis_kernel keeps the plain loop.
  int pend = -1;
  for (;;) {
    const unsigned long long act = __builtin_amdgcn_ballot_w64((g & (PARK ? pend : -1)) >= 0) & kQuad0;  // g >= 0 || (PARK && pend >= 0)
    if (!act) break;
    const unsigned long long donors = __builtin_amdgcn_ballot_w64(g >= 0 && sp > bp) & kQuad0, idle = ~act & kQuad0;
    if (ART_VIS_STEAL && donors && pop64(idle) >= ART_VIS_STEAL_MIN_IDLE) {  // wave-uniform: the k-th idle quad takes the k-th donor's stack bottom
      int l4 = lane & ~3;
      asm volatile("" : "+v"(l4));  // (recomputed here, not hoisted out of the loop)
      const unsigned long long below = (1ull << l4) - 1ull;
      const int ir = pop64(idle & below), dr = pop64(donors & below);
      const bool thief = (act >> l4 & 1ull) == 0ull && ir < pop64(donors);
      const bool robbed = g >= 0 && sp > bp && dr < pop64(idle);
      const int match = rank_match(l4, qd, robbed, dr, ir);  // (every lane takes part)
      const int src = (thief ? match : l4) + qd;
      const int dbp = __shfl(bp, src), dhome = __shfl(home, src), downer = __shfl(owner, src);
      const float ox = __shfl(s.o.x, src), oy = __shfl(s.o.y, src), oz = __shfl(s.o.z, src);
      const float dx = __shfl(s.d.x, src), dy = __shfl(s.d.y, src), dz = __shfl(s.d.z, src);
      const float dmaxd = __shfl(maxd, src);
      // the segment's derived values too (1/d, 2a, |o|_1 + maxd, force: the home's own, no divisions)
      const float ix = __shfl(s.inv.x, src), iy = __shfl(s.inv.y, src), iz = __shfl(s.inv.z, src), dom = __shfl(om, src);
      const float da2 = __shfl(s.a2, src);
      const int dforce = __shfl((int)force, src);
      if (thief) {
        g = (int)s_wave[(src >> 2) * kBvhStack + dbp];
        sp = bp = 0;
        home = dhome; owner = downer; maxd = dmaxd;
        s.o = mk3(ox, oy, oz); s.d = mk3(dx, dy, dz); s.inv = mk3(ix, iy, iz); s.a2 = da2;
        om = dom;
        force = dforce != 0;
      }
      fmk = __builtin_amdgcn_ballot_w64(force);
      if (robbed && ++bp == sp) sp = bp = 0;
    }
    for (;;) {  // quad-uniform steps
      if (PARK) {
        if (g >= leaf0 && pend < 0) { pend = g; pop(); }
        // (after the park, a quad with no parked leaf and a node holds an inner node)
        if (__builtin_amdgcn_ballot_w64((pend & ~g) < 0) == 0ull) break;  // pend < 0 && g >= 0, one compare
        if (!(g >= 0 && g < leaf0)) continue;
      } else if (!(g >= 0 && g < leaf0)) {
        break;
      }
      const int c0 = 4 * g + 1;
      if (qd == 0) ++nnode;
      ART_DIAG_STEP(nsteps);
      const CullRec r = load_node(br, c0 + qd);
      float tn;
      const bool h = node_entry(s, r, om, tn);
#ifdef ART_ECHO_CAP_MEAS  // (measurement builds only, wrong outputs: segments traversed only up to this distance)
      const bool enter = force | (h & (tn <= fminf(maxd, ART_ECHO_CAP_MEAS)));
      const unsigned long long em = __builtin_amdgcn_ballot_w64(enter);
#else
      // the entered lanes as a mask of scalar ANDs / ORs of single-compare ballots (a ballot of the
      // combined flag would round-trip it through a 0/1 VGPR); empty nodes: art_bvh.hip cull_stored
      const unsigned long long em = fmk | (__builtin_amdgcn_ballot_w64(h) & __builtin_amdgcn_ballot_w64(tn <= maxd));
      const bool enter = __builtin_amdgcn_inverse_ballot_w64(em);
#endif
      const uint32_t eb = (uint32_t)(em >> qshift) & 0xFu;
      if (eb) {
        const int first = __builtin_ctz(eb);
        const uint32_t rest = eb & (eb - 1u);
        if (enter && qd != first) my[sp + __popc(rest & ((1u << qd) - 1u))] = (uint32_t)(c0 + qd);
        sp += __popc(rest);
        g = c0 + first;
      } else {
        pop();
      }
    }
    bool hit_quad = false;
    const int leaf = PARK ? pend : g;
    if (leaf >= leaf0) {
      ART_DIAG_STEP(nsteps);
      int cc, tid;
      float d;
      const bool hh = leaf_slot_test<OBB>(s, br, (leaf - leaf0) * kBvhLeaf + qd, cc, d, tid, nt);
      const bool blk_here = hh && d < maxd && tid != owner;  // :373-394, :411-447
      hit_quad = ((uint32_t)(__builtin_amdgcn_ballot_w64(blk_here) >> qshift) & 0xFu) != 0u;
      if (!PARK && !hit_quad) pop();
    }
    pend = -1;
    for (unsigned long long bq = __builtin_amdgcn_ballot_w64(hit_quad) & kQuad0; bq; bq &= bq - 1ull)
      wblocked |= 1u << __builtin_amdgcn_readlane(home, __builtin_ctzll(bq));
    if ((wblocked >> home) & 1u) { g = -1; sp = bp = 0; }  // the segment is decided: every quad on it stops
  }
#ifdef ART_DIAG
  if (qd == 0 && valid) diag_add(3, nsteps);
  if (lane == 0) diag_add(1, clock64() - t0);
#endif
  return !((wblocked >> wq) & 1u);
}

template <bool OBB, bool HM>
__device__ __forceinline__ void vis_quad_body(const DevScene& sc, const VisPairs& vp, const uint32_t* count,
                                              unsigned long long* ex, uint32_t blk, int w, uint32_t* s_wave,
                                              const uint32_t* ecnt, int bounce, uint8_t* block, const EchoFromHits& eh) {
  const int lane = threadIdx.x & 63, qd = lane & 3;
  const int wq = lane >> 2, slot = w * 16 + wq;                // segment of the block's 64-pair batch
  if (sc.bvh_levels == 0 && !HM) return;                       // no colliders: nothing blocks
  bool valid;
  uint32_t p = 0u, out_at = 0u;
  uint16_t out_val = 0;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwner;
  s.o = s.d = s.inv = mk3(0.0f, 0.0f, 0.0f);
  s.a2 = 0.0f;
  if (HM) {
    bool slot_ok;
    valid = echo_seg_from_hit(sc, eh, blk, slot, s, maxd, out_at, out_val, slot_ok);
    if (eh.no_path) {  // the path kernel's duties for this frame: a miss keeps the reset 0 (:76, :200-207)
      if (slot_ok && !valid && qd == 0) reinterpret_cast<uint16_t*>(block)[out_at] = 0;
      if (ex) exec_add(ex, kExecEchoPairs, (unsigned long long)__popcll(__builtin_amdgcn_ballot_w64(valid) & kQuad0));
    }
    if (!__any(valid)) return;
  } else {
    if (vp.fixed) {  // bounce `bounce`'s compact records at fixed slots: 64-slot group blk (fold_path)
      p = (uint32_t)bounce * vp.fixed + blk * 64u + (uint32_t)slot;
      const uint2 ov = vp.out[p];
      valid = ov.y != kNoRecord;
      if (!__any(valid)) return;
      if (valid) {  // the segment as fold_path's reference expressions give it: off -> fan origin (:124-130)
        const FrameParams& fp = eh.fp;
        const int nrb = (fp.R + 63) >> 6;
        const int fan = (int)(blk / (uint32_t)nrb);
        const int ray = eh.ray_order[(int)(blk - (uint32_t)fan * nrb) * 64 + slot];
        const float4 hr = vp.hrec[p];
        const vec3 off = mk3(hr.x, hr.y, hr.z), O = load3(eh.origins, fan);
        s = make_seg(off, normalize(O - off));
        maxd = __uint_as_float(ov.x);
        owner = kNoOwner;
        out_at = (uint32_t)(((size_t)fan * eh.L.stride + eh.L.echo_off) / 2) + (uint32_t)(ray * fp.H + bounce);
        out_val = (uint16_t)(ov.y & 0xffffu);
      }
    } else {
      // all echo pairs, or (bounce >= 0) those bounce `bounce` emitted: they follow the earlier bounces'
      uint32_t start = 0u, n;
      if (bounce < 0) {
        n = ldc(count, 0);
      } else {
        for (int j = 0; j < bounce; ++j) start += ldc(ecnt, j);
        n = start + ldc(ecnt, bounce);
      }
      const uint32_t base = start + blk * 64u;
      if (base + (uint32_t)(w * 16) >= n) return;                // this wave's 16 segments are past the emitted pairs
      valid = base + (uint32_t)slot < n;
      p = valid ? base + (uint32_t)slot : base;
      if (valid) load_pair_seg(vp, p, s, maxd, owner);
    }
  }
  unsigned nt[3] = {0u, 0u, 0u}, nnode = 0;
  const bool visible = quad_echo_core<OBB, HM && ART_ECHO_PARK>(sc, s, maxd, owner, valid, lane, s_wave, nt, nnode);
  if (HM) {
    if (valid && qd == 0) reinterpret_cast<uint16_t*>(block)[out_at] = visible ? out_val : (uint16_t)0;  // :76, :142-144
  } else if (vp.fixed) {
    if (valid && visible && qd == 0) reinterpret_cast<uint16_t*>(block)[out_at] = out_val;  // :142-144
  } else if (valid && visible && qd == 0) {  // visible: the echo is stored (:142-144)
    const uint2 o = vp.out[p];
    reinterpret_cast<uint16_t*>(block)[o.x] = (uint16_t)(o.y & 0xffffu);
  }
  if (ex) {
    exec_add(ex + kExecEcho, kExecSphere, wave_sum_u32(nt[0]));
    exec_add(ex + kExecEcho, kExecAabb, wave_sum_u32(nt[1]));
    exec_add(ex + kExecEcho, kExecObb, wave_sum_u32(nt[2]));
    exec_add(ex + kExecEcho, kExecCullBox, 4ull * wave_sum_u32(nnode));
  }
}

// The echo traversal: one 64-pair batch per workgroup. EX: count the executed tests (fp.exec);
// without it the counters compile out. 8 waves per SIMD.
template <bool EX, bool OBB, bool HM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kEchoWaves<EX, OBB>)))
void vis_kernel(DevScene sc, VisPairs vp, const uint32_t* __restrict__ count, unsigned long long* ex,
                const uint32_t* __restrict__ ecnt, int bounce, uint8_t* __restrict__ block, EchoFromHits eh) {
  __shared__ uint32_t s_stk[64 * kBvhStack];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  vis_quad_body<OBB, HM>(sc, vp, count, EX ? ex : nullptr, blockIdx.x, w, s_stk + w * 16 * kBvhStack, ecnt, bounce, block, eh);
}

// ------------------------------------------------------------------------------------------
// Muffle rays (:150-173, CanRaySeeAudioTarget :405-449). One lane per hit record and target (grid
// y = target; more waves in flight for the latency-bound list walks): the lane's ray from `off` to
// the target (distance < MaxMuffleHitDistance,
// :165-168) is tested against the colliders of its direction cell around the target
// (art_cells.hip: not owned by t, widened bounding sphere on the ray) and stops at its first
// blocker; the wave counts its visible rays into the muffle accumulators with one atomic per
// distinct counter (its records come from one or two 64-ray groups). Any-hit is an OR over the
// colliders, so the cell lists' order is free.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int cube_cell(vec3 v) {
  const float ax = fabsf(v.x), ay = fabsf(v.y), az = fabsf(v.z);
  const int m = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
  const float c[3] = {v.x, v.y, v.z};
  const float n = fabsf(c[m]);
  const float u = c[(m + 1) % 3] / n, w = c[(m + 2) % 3] / n;
  const int i = min(max((int)floorf((u + 1.0f) * (0.5f * kCellG)), 0), kCellG - 1);
  const int j = min(max((int)floorf((w + 1.0f) * (0.5f * kCellG)), 0), kCellG - 1);
  const int f = 2 * m + (c[m] < 0.0f ? 1 : 0);
  return (f * kCellG + j) * kCellG + i;
}

// Exact test of collider `code` (rank << 28 | index, reference records) against segment s.
template <bool OBB>
__device__ __forceinline__ bool muffle_test(const DevScene& sc, const Seg& s, uint32_t code, float maxd, unsigned* nt) {
  const uint32_t type = code >> 28, idx = code & 0x0fffffffu;
  float d;
  bool h;
  if (type == 0) {
    const float4 a = *reinterpret_cast<const float4*>(sc.sph + idx);
    SphereRec r;
    r.cx = a.x; r.cy = a.y; r.cz = a.z; r.r2 = a.w;
    ++nt[0];
    h = sphere_hit_dist(s, r, d);
  } else if (type == 1 || !OBB) {
    const AabbRec r = sc.aabb[idx];
    ++nt[1];
    h = aabb_test<false>(s, r, d);
  } else {
    ++nt[2];
    h = obb_test_staged(s, sc.obb + idx, d);
  }
  return h && d < maxd;
}

// Every collider not owned by target t, in reference order (lists unavailable or not applicable).
template <bool OBB>
__device__ bool muffle_brute(const DevScene& sc, const Seg& s, float maxd, int t, unsigned* nt) {
  for (int i = 0; i < sc.ns; ++i)
    if (sc.sph[i].tid != t && muffle_test<OBB>(sc, s, (uint32_t)i, maxd, nt)) return true;
  for (int i = 0; i < sc.na; ++i)
    if (sc.aabb[i].tid != t && muffle_test<OBB>(sc, s, (1u << 28) | (uint32_t)i, maxd, nt)) return true;
  for (int i = 0; i < sc.no; ++i)
    if (sc.obb[i].tid != t && muffle_test<true>(sc, s, (2u << 28) | (uint32_t)i, maxd, nt)) return true;
  return false;
}

// The muffle ray of target t from `off` (the hit point stepped back along the ray, :158), tp the
// target's position and maxd = distance(off, tp) (:165, the caller checks maxd < MaxMuffleHitDistance
// :168): true when a collider not owned by t blocks it (CanRaySeeAudioTarget :405-449). The ray
// walks the three type lists of its direction cell around the target, each by ascending near
// bound, stopping at the first entry past the segment; a segment longer than the lists' cell_far,
// a degenerate one or a dropped target tests every collider in reference order. nt / ne / nfb
// count exact tests, list entries and fallback rays (EX).
#ifndef ART_MUFFLE_PREFETCH
#define ART_MUFFLE_PREFETCH 2  // (0: the round-6 walks, each list's entries fetched step by step; 1: OBB scenes prefetch the sphere list only; for A/B runs)
#endif
template <bool EX, bool OBB>
__device__ __forceinline__ bool muffle_blocked(const DevScene& sc, vec3 off, vec3 tp, float maxd, int t, unsigned* nt,
                                               unsigned& ne, unsigned& nfb) {
  bool blocked = false;
  const Seg s = make_seg(off, normalize(tp - off));               // :158-160
  const vec3 v = off - tp;                                        // the ray seen from the target
  const bool lists = sc.cell_ok[t] != 0u && maxd <= sc.cell_far[t] && (v.x != 0.0f || v.y != 0.0f || v.z != 0.0f) &&
                     isfinite(v.x) && isfinite(v.y) && isfinite(v.z);
  if (lists) {
    // the cell's Sphere, AABB and OBB lists in turn (a type-uniform test per loop), each by
    // ascending near bound: a walk stops at the first entry past the segment
    const uint32_t* st = sc.cell_start + ((size_t)t * kCells + cube_cell(v)) * 3;
    const float lim = maxd * 1.00001f + 1e-6f;
    const uint32_t klim = near_key(__float_as_uint(lim));
    const uint4 se = make_uint4(st[0], st[1], st[2], st[3]);
    // two entries per step: both records are fetched before either is tested (two dependent
    // fetch chains in flight per lane instead of one); OBB records (64 B) one at a time, which
    // keeps the kernel within 64 VGPRs
    // entry k: in-type index, near key and near bound (4-B entries carry the key, whose float
    // is a lower bound of the near bound: the per-entry bound check then admits a little more)
    auto entry = [&](uint32_t k, uint32_t& idx, uint32_t& key, float& nearf) {
      if (sc.cell_compact) {  // (wave-uniform)
        const uint32_t v = sc.cell_ent32[k];
        idx = v & 0xffffu; key = v >> 16; nearf = __uint_as_float(key << 16);
      } else {
        const uint2 v = sc.cell_ent[k];
        idx = v.x & 0x0fffffffu; key = near_key(v.y); nearf = __uint_as_float(v.y);
      }
    };
#if ART_MUFFLE_PREFETCH
    if (sc.cell_compact) {  // (wave-uniform; 8-B entries take the step-by-step walks below)
    // Software-pipelined walks over the 4-B entries: the first entries of all three lists are
    // fetched together as soon as the cell's starts arrive, and each step fetches the next step's
    // entries beside its records, so a walk costs one dependent fetch per step instead of two and
    // the AABB and OBB walks start without an entry fetch of their own. An entry past its list's
    // end reads as 0xffffffff (key 0xffff, beyond every segment) without a fetch.
    auto fetch = [&](uint32_t k, uint32_t e) { return k < e ? sc.cell_ent32[k] : 0xffffffffu; };
    auto nearf_of = [](uint32_t v) { return __uint_as_float(v & 0xffff0000u); };
    // (ART_MUFFLE_PREFETCH 1: with OBBs in the scene the AABB list's first entries are fetched when
    // its walk starts and the OBB walk fetches entry by entry, which needs fewer live registers.
    // Measured: keeping the cell's bounds and first entries in one 48-B head per cell, fetched at
    // once, gained nothing further: the entries are already fetched beside one another)
    constexpr bool kAll = ART_MUFFLE_PREFETCH >= 2 || !OBB;
    const uint32_t s0 = fetch(se.x, se.y), s1 = fetch(se.x + 1, se.y);
    uint32_t a0 = 0u, a1 = 0u, o0 = 0xffffffffu;
    if (kAll) { a0 = fetch(se.y, se.z); a1 = fetch(se.y + 1, se.z); }
    if (kAll && OBB) o0 = fetch(se.z, se.w);
    auto walk2 = [&](uint32_t b, uint32_t e, uint32_t c0, uint32_t c1, auto load, auto test) {
      for (uint32_t k = b; k < e; k += 2) {  // c0, c1 = entries k, k + 1
        if ((c0 >> 16) > klim) break;        // this and every later entry lie beyond the segment
        const bool use1 = (c1 >> 16) <= klim;
        const auto r0 = load(c0 & 0xffffu);
        const auto r1 = load((use1 ? c1 : c0) & 0xffffu);
        const uint32_t n0 = fetch(k + 2, e), n1 = fetch(k + 3, e);  // (beside the records)
        if (EX) ne += use1 ? 2u : 1u;
        if (!(nearf_of(c0) > lim) && test(r0)) { blocked = true; break; }
        if (!use1) break;
        if (!(nearf_of(c1) > lim) && test(r1)) { blocked = true; break; }
        c0 = n0; c1 = n1;
      }
    };
    walk2(se.x, se.y, s0, s1,
          [&](uint32_t idx) {
            const float4 a = *reinterpret_cast<const float4*>(sc.sph + idx);
            SphereRec r;
            r.cx = a.x; r.cy = a.y; r.cz = a.z; r.r2 = a.w;
            return r;
          },
          [&](const SphereRec& r) {
            ++nt[0];
            float d;
            return sphere_hit_dist(s, r, d) && d < maxd;
          });
    if (!kAll && !blocked) { a0 = fetch(se.y, se.z); a1 = fetch(se.y + 1, se.z); }
    if (!blocked)
      walk2(se.y, se.z, a0, a1, [&](uint32_t idx) { return sc.aabb[idx]; },
            [&](const AabbRec& r) {
              ++nt[1];
              float d;
              return aabb_test<false>(s, r, d) && d < maxd;
            });
    if (OBB && !blocked) {  // OBB records (64 B) one at a time (kAll: the next entry fetched beside each test)
      uint32_t c = o0;
      for (uint32_t k = se.z; k < se.w; ++k) {
        if (!kAll) c = sc.cell_ent32[k];
        if ((c >> 16) > klim) break;
        if (EX) ++ne;
        const uint32_t n = kAll ? fetch(k + 1, se.w) : 0u;
        if (!(nearf_of(c) > lim)) {
          ++nt[2];
          float d;
          if (obb_test_staged(s, sc.obb + (c & 0xffffu), d) && d < maxd) { blocked = true; break; }
        }
        c = n;
      }
    }
    } else {
#endif
    auto walk = [&](uint32_t b, uint32_t e, auto load, auto test, auto pair) {
      uint32_t i0, k0, i1, k1;
      float n0, n1;
      if (!decltype(pair)::value) {
        for (uint32_t k = b; k < e; ++k) {
          entry(k, i0, k0, n0);
          if (k0 > klim) break;  // this and every later entry lie beyond the segment
          if (EX) ++ne;
          if (!(n0 > lim) && test(load(i0))) { blocked = true; break; }
        }
        return;
      }
      for (uint32_t k = b; k < e && !blocked; k += 2) {
        const bool has1 = k + 1 < e;
        entry(k, i0, k0, n0);
        entry(has1 ? k + 1 : k, i1, k1, n1);
        if (k0 > klim) break;             // this and every later entry lie beyond the segment
        const bool use1 = has1 && k1 <= klim;
        const auto r0 = load(i0);
        const auto r1 = load(use1 ? i1 : i0);
        if (EX) ne += use1 ? 2u : 1u;
        if (!(n0 > lim) && test(r0)) { blocked = true; break; }
        if (!use1) break;
        if (!(n1 > lim) && test(r1)) { blocked = true; break; }
      }
    };
    walk(se.x, se.y,
         [&](uint32_t idx) {
           const float4 a = *reinterpret_cast<const float4*>(sc.sph + idx);
           SphereRec r;
           r.cx = a.x; r.cy = a.y; r.cz = a.z; r.r2 = a.w;
           return r;
         },
         [&](const SphereRec& r) {
           ++nt[0];
           float d;
           return sphere_hit_dist(s, r, d) && d < maxd;
         },
         std::true_type{});
    walk(se.y, se.z, [&](uint32_t idx) { return sc.aabb[idx]; },
         [&](const AabbRec& r) {
           ++nt[1];
           float d;
           return aabb_test<false>(s, r, d) && d < maxd;
         },
         std::true_type{});
    if (OBB)
      walk(se.z, se.w, [&](uint32_t idx) { return sc.obb + idx; },
           [&](const ObbRec* r) {
             ++nt[2];
             float d;
             return obb_test_staged(s, r, d) && d < maxd;
           },
           std::false_type{});
#if ART_MUFFLE_PREFETCH
    }
#endif
  } else {
    if (EX) ++nfb;
    blocked = muffle_brute<OBB>(sc, s, maxd, t, nt);
  }
  return blocked;
}

// HM: one-hit frames with one batch slot whose path kernel does not run: lane i is ray slot i
// (64-ray group i / 64) and its muffle rays start from the nearest hit as the path kernel computes
// it (hit_from_pre); the accumulator base is fan * T (TC == 1: batch slot 0).
// i = this lane's hit record / ray slot (i - lane wave-uniform); targets by, by + gy, ...
template <bool EX, bool OBB, bool HM>
__device__ __forceinline__ void muffle_body(const DevScene& sc, const FrameParams& fp, const VisPairs& vp,
                                            const uint32_t* __restrict__ count, uint32_t* __restrict__ acc,
                                            const EchoFromHits& eh, uint32_t i, int by, int gy) {
  const int lane = threadIdx.x & 63;
  // (fixed slots: every bounce's records, kNoRecord marking the slots with no hit)
  const uint32_t n = HM ? (uint32_t)fp.S * (uint32_t)((fp.R + 63) >> 6) * 64u : (vp.fixed ? vp.fixed * (uint32_t)fp.H : ldc(count, 1));
  if (__builtin_amdgcn_readfirstlane(i - (uint32_t)lane) >= n) return;
  bool valid = i < n;
  vec3 off = mk3(0.0f, 0.0f, 0.0f);
  uint32_t dbase = 0u;
  if (HM) {
    bool slot_ok;
    int fan = 0, ray = 0, type = kNone, idx = 0;
    vec3 O, o;
    valid = valid && hit_from_pre(sc, eh, i >> 6, (int)(i & 63u), slot_ok, fan, ray, O, o, off, type, idx);
    dbase = (uint32_t)fan * (uint32_t)fp.T;
  } else {
    // (compact records: fold_path; the hit record is fetched beside the marker, not after it: a
    // slot without a record holds a stale one, never used)
    const float4 r = vp.hrec[i < n ? i : 0u];
    if (vp.fixed) valid = valid && vp.out[i].y != kNoRecord;
    off = mk3(r.x, r.y, r.z);
    dbase = __float_as_uint(r.w);
    valid = valid && dbase != kNoRecord;
  }
  unsigned nt[3] = {0u, 0u, 0u}, ne = 0u, nfb = 0u;  // tests, list entries scanned, fallback rays
  for (int t = by; t < fp.T; t += gy) {  // workgroup-uniform
    const vec3 tp = load3(sc.targets, t);
    const float maxd = distance(off, tp);                             // :165
    const bool act = valid && maxd < fp.max_muffle;                   // :168
    bool blocked = false;
    if (act) {
      blocked = muffle_blocked<EX, OBB>(sc, off, tp, maxd, t, nt, ne, nfb);
    }
    const bool vis = act && !blocked;                                 // :171
    unsigned long long mv = __builtin_amdgcn_ballot_w64(vis);
    const uint32_t dest = dbase + (uint32_t)t;
    while (mv) {
      const uint32_t d0 = __builtin_amdgcn_readlane(dest, __builtin_ctzll(mv));
      const unsigned long long eq = __builtin_amdgcn_ballot_w64(vis && dest == d0);
      if (lane == 0) atomicAdd(&acc[d0], (uint32_t)__popcll(eq));
      mv &= ~eq;
    }
  }
  if (EX) {  // lane-tests executed (each lane's own tests; the loop is per lane)
    exec_add(fp.exec + kExecMuffle, kExecSphere, wave_sum_u32(nt[0]));
    exec_add(fp.exec + kExecMuffle, kExecAabb, wave_sum_u32(nt[1]));
    exec_add(fp.exec + kExecMuffle, kExecObb, wave_sum_u32(nt[2]));
    exec_add(fp.exec + kExecMuffle, kExecCellEntries, wave_sum_u32(ne));
    exec_add(fp.exec + kExecMuffle, kExecMuffleFallback, wave_sum_u32(nfb));
  }
}

// Muffle block b of M ray blocks x mt targets in echo_muffle_kernel (its 4 one-wave workgroups on the
// XCD of block b, as below). Consecutive blocks are
// dispatched to the chip's 8 XCDs in turn (each with its own L2), so when mt divides 8 the XCD of
// block b serves one target, b % 8 % mt: each L2 then holds that target's direction-cell lists
// only, not all targets' (config 2: echo_muffle traffic 12.9 -> 10.8 MB per frame with the 4-B
// entries). The muffle blocks there fill the echo traversal's tails; in the standalone muffle_kernel
// the uneven work per target left XCDs idle (config 5: 171 -> 193 us), so it keeps the plain order.
// Any other shape keeps the plain (b % M, b / M) order. Round 6 (ART_MUFFLE_XCD 2, the default
// when the group count is a multiple of 8): each muffle wave runs on the XCD that traced its 64-ray
// group's echoes (echo_muffle_kernel), so a group's nearest hits are read from that XCD's L2 and
// each L2 holds every target's lists: echo+muffle config 4 594.5 -> 585.7 us, config 3 88.5 ->
// 87.4, config 2 54.2 -> 53.6 (HBM bytes per launch at config 4 73.3 -> 75.1 MB: the time is not
// set by the traffic).
#ifndef ART_MUFFLE_XCD
#define ART_MUFFLE_XCD 2
#endif
__device__ __forceinline__ void muffle_block(uint32_t b, uint32_t M, int mt, uint32_t& rb, int& t) {
  if (ART_MUFFLE_XCD >= 1 && 8 % mt == 0 && ((unsigned long long)M * mt) % 8 == 0) {
    const uint32_t x = b & 7u;
    t = (int)(x % (uint32_t)mt);
    rb = (b >> 3) * (8u / (uint32_t)mt) + x / (uint32_t)mt;
  } else {
    rb = b % M;
    t = (int)(b / M);
  }
}

// 8 waves per SIMD; the counting OBB instantiations at 7, where they need no spills
template <bool EX, bool OBB, bool HM>
#ifndef ART_MUFFLE_OBB_WAVES
#define ART_MUFFLE_OBB_WAVES 7  // (the prefetching walks need 72 VGPRs with OBB tests)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(EX && OBB ? 5 : (OBB ? ART_MUFFLE_OBB_WAVES : (EX ? 7 : 8))))) void muffle_kernel(DevScene sc, FrameParams fp, VisPairs vp,
                                                     const uint32_t* __restrict__ count, uint32_t* __restrict__ acc,
                                                     EchoFromHits eh) {
  muffle_body<EX, OBB, HM>(sc, fp, vp, count, acc, eh, blockIdx.x * 256u + threadIdx.x, (int)blockIdx.y, (int)gridDim.y);
}

// One-hit frames with one batch slot and no path kernel (HM2): the echo traversal and the muffle
// rays, both from the nearest hits, as one launch on the launch stream: workgroups [0, 4 groups) are
// the echo batches (one wave each) (dispatched first, one round of waves), the rest the muffle blocks (mblocks x
// mt, filling the echo traversal's tails). No side stream, so no fork / join on the frame's path.
// With OBB tests the joint kernel runs at 6 waves per SIMD (5 counting), where it needs no spills.
// One-wave workgroups (4 per 64-ray echo group / 256-ray muffle block), so a muffle wave can start in
// any single wave slot an echo wave frees (with 4-wave workgroups a CU waited for 4 free slots:
// config 3 0.1686 -> 0.1660 ms/step, config 4 1.164 -> 1.149, config 2 even); the 4 waves of a
// group or block stay on one XCD (workgroup b runs on XCD b % 8).
template <bool EX, bool OBB>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OBB ? (EX ? 5 : ART_ECHO_MUFFLE_OBB_WAVES) : kEchoWaves<EX, OBB>)))
void echo_muffle_kernel(DevScene sc, FrameParams fp, VisPairs vp, const uint32_t* __restrict__ count,
                        unsigned long long* ex, uint8_t* __restrict__ block, EchoFromHits eh, uint32_t* __restrict__ acc,
                        uint32_t groups, uint32_t mblocks, int mt) {
  __shared__ uint32_t s_stk[16 * kBvhStack];
  const uint32_t b = blockIdx.x;
  const uint32_t ne = 4u * groups;  // echo workgroups
  ART_WAVE_TIMER(b < ne ? 1u : 2u);
  // (group or muffle block, wave): a group's 4 waves on one XCD when the counts are multiples of 8,
  // else consecutive
  auto split = [](uint32_t x, uint32_t n, uint32_t& u, int& wv) {
    if (n % 8u == 0u) {
      const uint32_t j = x >> 3;
      u = (j >> 2) * 8u + (x & 7u);
      wv = (int)(j & 3u);
    } else {
      u = x >> 2;
      wv = (int)(x & 3u);
    }
  };
  if (b < ne) {
    if (ART_MEASURE_PARTS == 2) return;
    uint32_t g;
    int w;
    split(b, groups, g, w);
    vis_quad_body<OBB, true>(sc, vp, count, EX ? ex : nullptr, g, w, s_stk, nullptr, -1, block, eh);
    return;
  }
  if (ART_MUFFLE_XCD == 2 && groups % 8u == 0u) {
    // group-local muffle waves (muffle_block's note): the wave of (64-ray group G, target t) runs on the XCD
    // that traced G's echo rays (workgroup index % 8 == G % 8), so each XCD fetches only its own
    // groups' nearest hits (from its L2) and every target's cell lists
    const uint32_t m = b - ne, x = m & 7u, j = m >> 3;
    const int t = (int)(j % (uint32_t)mt);
    const uint32_t G = (j / (uint32_t)mt) * 8u + x;
    muffle_body<EX, OBB, true>(sc, fp, vp, count, acc, eh, G * 64u + threadIdx.x, t, mt);
    return;
  }
  uint32_t mb, rb;
  int sub, t;
  split(b - ne, mblocks * (uint32_t)mt, mb, sub);
  muffle_block(mb, mblocks, mt, rb, t);  // (groups is a multiple of 8 in the bench shapes)
  muffle_body<EX, OBB, true>(sc, fp, vp, count, acc, eh, rb * 256u + (uint32_t)sub * 64u + threadIdx.x, t, mt);
}


// ------------------------------------------------------------------------------------------
// Permeation job (AudioPermeationJobBatched.Execute :34-91) over the BVH. One wave per (batch slot,
// fan), 16 quads:
//   1. the slot's value is written by the highest-index ray of its last batch whose permeation
//      first hit exists (each hitting ray overwrites it, :85; App. B Q7): quads cast the batch's
//      rays from its end, 16 at a time (quad_nearest_core<PERM>: INFINITY sentinel, inverse OBB
//      rotation, :101-141 / :172-179), and the highest-index hitting ray wins;
//   2. its T loss rays (:61-85), one per quad: every collider whose widened box the ray enters at
//      t >= 0 is visited (no pruning: the loss sums penetrations along the whole ray), its loss
//      term evaluated (:225-328), the non-zero terms kept as (order code, term) in LDS, ranked by
//      order code and summed serially in reference order (Sphere, AABB, OBB, ascending index).
// Exactness: a collider the ray misses contributes exactly +0, and an entered-but-missed node's
// colliders are missed (DESIGN.md §5 item 8 for the slab tests; the sphere loss test's b^2 - c
// discriminant carries at most ~32 eps |oc|^2 of rounding, inside the sphere margin); +-0 terms never
// change the running sum (it starts at +0 and is never -0), so only non-zero terms are summed. A loss
// ray meeting more than kLossCap colliders is summed by the whole wave over every collider instead.
// ------------------------------------------------------------------------------------------
constexpr int kLossCap = 48;  // kept (code, term) entries per loss ray
#ifndef ART_PERM_LAST1
#define ART_PERM_LAST1 1  // (0: the first-hit search casts 16 rays from the first iteration on, for A/B runs)
#endif
#ifndef ART_PERM_SPLIT
#define ART_PERM_SPLIT 1  // (0: one quad per loss ray, for A/B runs)
#endif

// Loss term of global collider g (Sphere, AABB, OBB ranges) for segment s and target t (0 when t
// owns it), the reference expressions (:225-328).
__device__ __forceinline__ float loss_term_global(const DevScene& sc, const Seg& s, int g, int t) {
  if (g < sc.ns) {
    const SphereRec r = sc.sph[g];
    return r.tid != t ? perm_term_sphere(s, r, sc.sphc[g].density) : 0.0f;
  }
  g -= sc.ns;
  if (g < sc.na) {
    const AabbRec r = sc.aabb[g];
    return r.tid != t ? perm_term_slab(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.mnx, r.mny, r.mnz, r.mxx, r.mxy,
                                       r.mxz, sc.aabbc[g].density)
                      : 0.0f;
  }
  g -= sc.na;
  if (g >= sc.no) return 0.0f;
  const ObbRec r = sc.obb[g];
  if (r.tid == t) return 0.0f;
  const quat q = stored_q(r);  // RayIntersectsOBBPermeation :294-300 rotates by the stored rotation
  const vec3 lo = qmul(q, s.o - mk3(r.cx, r.cy, r.cz));
  const vec3 ld = qmul(q, s.d);
  return perm_term_slab(lo.x, lo.y, lo.z, 1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z, r.lmnx, r.lmny, r.lmnz, r.lmxx, r.lmxy, r.lmxz,
                        sc.obbc[g].density);
}

// The whole wave over every collider in reference order (lanes over colliders, non-zero terms
// added serially): the overflow path. Wave-uniform result.
__device__ float loss_sum_wave(const DevScene& sc, const Seg& s, int t) {
  const int lane = threadIdx.x & 63, ctot = sc.ns + sc.na + sc.no;
  float sum = 0.0f;
  for (int base = 0; base < ctot; base += 64) {
    const float term = base + lane < ctot ? loss_term_global(sc, s, base + lane, t) : 0.0f;
    for (unsigned long long m = __builtin_amdgcn_ballot_w64(term != 0.0f); m; m &= m - 1ull)
      sum += __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, term), __builtin_ctzll(m)));
  }
  return sum;
}

// Loss term of leaf slot `slot` (its order code in cc; 0 for an empty slot or a collider t owns).
template <bool OBB>
__device__ __forceinline__ float leaf_loss_term(const DevScene& sc, const Seg& s, const BvhRes& br, int slot, int t, int& cc) {
  auto ld = [&](int k) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(br.leaves, slot * (OBB ? 64 : 32) + 16 * k, 0, 0));
  };
  const float4 qa = ld(0), qb = ld(1);
  cc = __float_as_int(qb.w);
  if (cc < 0) return 0.0f;
  const int type = cc >> 28, idx = cc & 0x0fffffff;
  if (type == 0) {
    if (__float_as_int(qb.z) == t) return 0.0f;
    SphereRec r;
    r.cx = qa.x; r.cy = qa.y; r.cz = qa.z; r.r2 = qa.w;
    return perm_term_sphere(s, r, sc.sphc[idx].density);
  }
  if (type == 1 || !OBB) {
    if (__float_as_int(qb.z) == t) return 0.0f;
    return perm_term_slab(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, qa.x, qa.y, qa.z, qa.w, qb.x, qb.y,
                          sc.aabbc[idx].density);
  }
  quat q;
  q.x = qa.w; q.y = qb.x; q.z = qb.y; q.w = qb.z;
  const vec3 ld3 = qmul(q, s.d);
  const float ix = recip_exact(ld3.x), iy = recip_exact(ld3.y), iz = recip_exact(ld3.z);
  const vec3 lo = qmul(q, s.o - mk3(qa.x, qa.y, qa.z));
  const float4 qc = ld(2), qe = ld(3);
  if (__float_as_int(qe.z) == t) return 0.0f;
  return perm_term_slab(lo.x, lo.y, lo.z, ix, iy, iz, qc.x, qc.y, qc.z, qc.w, qe.x, qe.y, sc.obbc[idx].density);
}

template <bool OBB>
__global__ __launch_bounds__(64) void permeate_bvh_kernel(DevScene sc, FrameParams fp, FanLayout L, const float* __restrict__ origins,
                                                         uint8_t* __restrict__ block, const int2* __restrict__ slot_batch) {
  __shared__ uint32_t s_stk[16 * kBvhStack];
  __shared__ int s_bound[16];
  __shared__ unsigned long long s_key[16];
  __shared__ uint32_t s_code[16][kLossCap];
  __shared__ float s_term[16][kLossCap], s_sorted[16][kLossCap];
  const int fan = blockIdx.y, slot = blockIdx.x, lane = threadIdx.x, qd = lane & 3, wq = lane >> 2;
  const int2 br = slot_batch[slot];
  if (br.y <= br.x) return;  // no batch maps to this slot: the value stays (stale / uninitialized, Q7)
  const vec3 O = load3(origins, fan);
  uint32_t* const my = s_stk + wq * kBvhStack;
  float* const ppr = reinterpret_cast<float*>(block + (size_t)fan * L.stride + L.perm_off);
  const int T = fp.T;

  // 1. the highest-index ray of [br.x, br.y) with a permeation first hit (ShootRayCast :58)
  int found = -1, code = kNoHit;
  float dist = 0.0f;
  int rtop = br.y - 1;  // the highest ray not yet cast
  if (ART_PERM_LAST1) {  // the batch's last ray alone first (it usually hits): quad 0 casts it and the
                         // wave's 15 idle quads share its traversal (the work sharing of quad_nearest_core)
    float best;
    int c;
    quad_nearest_core<false, OBB, true>(sc, make_seg(O, load_dir(sc.dirs, rtop)), wq == 0, lane, my, s_bound, s_key, best,
                                        c, nullptr);
    const int c0 = __builtin_amdgcn_readlane(c, 0);
    if (c0 != kNoHit) {
      found = rtop;
      code = c0;
      dist = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, best), 0));
    }
    --rtop;
  }
  for (int r0 = rtop; r0 >= br.x && found < 0; r0 -= 16) {  // (wave-uniform)
    const int ray = r0 - wq;
    const bool alive = ray >= br.x;
    float best;
    int c;
    quad_nearest_core<false, OBB, true>(sc, make_seg(O, load_dir(sc.dirs, alive ? ray : br.x)), alive, lane, my, s_bound,
                                        s_key, best, c, nullptr);
    const unsigned long long hq = __builtin_amdgcn_ballot_w64(qd == 0 && alive && c != kNoHit);
    if (hq) {  // the lowest such quad holds the highest ray index
      const int src = __builtin_ctzll(hq);
      found = r0 - (src >> 2);
      code = __builtin_amdgcn_readlane(c, src);
      dist = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, best), src));
    }
  }
  if (found < 0) {  // reset (:43-46) and no ray hit
    for (int t = lane; t < T; t += 64) ppr[slot * T + t] = 0.0f;
    return;
  }
  const vec3 d = load_dir(sc.dirs, found);
  {  // the exact (Unity min / max) distance of a zero first hit: only its sign can differ
    const Seg s0 = make_seg(O, d);
    const int type = code >> 28, idx = code & 0x0fffffff;
    if (dist == 0.0f) {
      if (type == 0) sphere_hit_dist(s0, sc.sph[idx], dist);
      else if (type == 1) aabb_test<true>(s0, sc.aabb[idx], dist);
      else obb_test<true>(s0, sc.obb[idx], inverse_q(sc.obbc[idx]), dist);
    }
  }
  const vec3 o = O + d * dist;  // :61
  const vec3 off = o - d * kEps;

  // 2. the T loss rays (:67-85). P quads per ray (ART_PERM_SPLIT; P = 16 / rays in the chunk, at
  // most 4, with an inner root): quad j of a ray traverses the root's children c with c % P == j, so
  // the ray's subtrees run side by side instead of leaving 16 - T quads idle (config 4: the job's
  // waves hold wave slots beside the nearest traversal for their whole length). The subtrees are
  // disjoint, so the ray's kept terms are its quads' lists together, ranked by order code across
  // them and summed serially in reference order as before.
  const BvhRes bres = bvh_res(sc);
  const int leaf0 = sc.bvh_leaf0, qshift = lane & ~3;
  for (int t0 = 0; t0 < T;) {  // (wave-uniform)
    const int P = (ART_PERM_SPLIT && leaf0 > 0) ? min(4, 16 / min(16, T - t0)) : 1;  // quads per ray
    const int nr = min(T - t0, 16 / P);                                              // rays in this chunk
    const int rq = wq / P, j = wq - rq * P, wq0 = rq * P;                            // ray, part, its first quad
    const int t = t0 + rq;
    const bool valid = rq < nr;
    const Seg s = make_seg(off, normalize(load3(sc.targets, valid ? t : 0) - off));
    const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z);
    const bool force = force_all(s, om);
    int g = valid && sc.bvh_levels > 0 ? 0 : -1, sp = 0, n = 0;
    while (__any(g >= 0)) {
      while (g >= 0 && g < leaf0) {  // (quad-uniform) descend in index order, every entered child
        const int c0 = 4 * g + 1;
        const CullRec r = load_node(bres, c0 + qd);
        float tn;
        const bool h = node_entry(s, r, om, tn);
        // (an empty node's entry is +inf: cull_stored); at the root, this quad's share of the children
        const bool enter = (force | (h & (tn < INFINITY))) & (g != 0 || qd % P == j);
        const uint32_t eb = (uint32_t)(__builtin_amdgcn_ballot_w64(enter) >> qshift) & 0xFu;
        if (eb) {
          const int first = __builtin_ctz(eb);
          const uint32_t rest = eb & (eb - 1u);
          if (enter && qd != first) my[sp + __popc(rest & ((1u << qd) - 1u))] = (uint32_t)(c0 + qd);
          sp += __popc(rest);
          g = c0 + first;
        } else {
          g = sp > 0 ? (int)my[--sp] : -1;
        }
      }
      if (g >= leaf0) {
        int cc;
        const float term = leaf_loss_term<OBB>(sc, s, bres, (g - leaf0) * kBvhLeaf + qd, t, cc);
        const uint32_t nz = (uint32_t)(__builtin_amdgcn_ballot_w64(term != 0.0f) >> qshift) & 0xFu;
        const int at = n + __popc(nz & ((1u << qd) - 1u));
        if (term != 0.0f && at < kLossCap) { s_code[wq][at] = (uint32_t)cc; s_term[wq][at] = term; }
        n += __popc(nz);
        g = sp > 0 ? (int)my[--sp] : -1;
      }
    }
    // the ray's lists: the P quads' counts (every lane takes part in the shuffles)
    int nk[4], ntot = 0;
    bool fits = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      nk[k] = __shfl(n, 4 * min(wq0 + k, 15));
      if (k < P) { ntot += nk[k]; fits = fits && nk[k] <= kLossCap; }
    }
    // rank the kept terms by order code across the ray's lists (the lanes of its quads share the
    // entries), then sum them serially in that order in the ray's first lane
    // (lanes read each other's LDS entries: order the leaf loop's writes before the ranking and the
    // ranks' scatter before the sum, as kd_wave_kernel does)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    float* const srt = &s_sorted[0][0] + wq0 * kLossCap;  // the ray's P x kLossCap sorted entries
    if (valid && fits) {
      for (int i = qd; i < n; i += 4) {
        const uint32_t ci = s_code[wq][i];
        int rank = 0;
        for (int k = 0; k < P; ++k)
          for (int jj = 0; jj < nk[k]; ++jj) rank += s_code[wq0 + k][jj] < ci ? 1 : 0;
        srt[rank] = s_term[wq][i];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (valid && fits && j == 0) {
      float sum = 0.0f;
      for (int i = 0; i < ntot; ++i) sum += srt[i];
      if (qd == 0) ppr[slot * T + t] = (float)fp.R * fp.perm_strength - sum;  // :260
    }
    for (unsigned long long ov = __builtin_amdgcn_ballot_w64(qd == 0 && j == 0 && valid && !fits); ov; ov &= ov - 1ull) {  // (wave-uniform)
      const int src = __builtin_ctzll(ov), tt = t0 + (src >> 2) / P;
      const Seg so = make_seg(off, normalize(load3(sc.targets, tt) - off));
      const float sum = loss_sum_wave(sc, so, tt);
      if (lane == 0) ppr[slot * T + tt] = (float)fp.R * fp.perm_strength - sum;
    }
    t0 += nr;
  }
}

void launch_permeate(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins, uint8_t* block,
                     const int2* slot_batch, hipStream_t st) {
  if (fp.S == 0) return;
  if (sc.no > 0)
    hipLaunchKernelGGL((permeate_bvh_kernel<true>), dim3(fp.TC, fp.S), dim3(64), 0, st, sc, fp, L, origins, block, slot_batch);
  else
    hipLaunchKernelGGL((permeate_bvh_kernel<false>), dim3(fp.TC, fp.S), dim3(64), 0, st, sc, fp, L, origins, block, slot_batch);
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
// Pair buffer: echo segments | echo outputs | hit records | first-segment hits | ray state + live
// list (multi-hit).
struct PairBufs {
  VisPairs vp;
  int2* pre;        // [groups * 64] nearest hits of the current bounce
  float4* state;    // [groups * 64][2] ray state between the bounce launches (multi-hit frames)
  size_t total;
};

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
static size_t echo_cap_of(const FrameParams& fp) { return ((size_t)fp.S * fp.R * fp.H + 63) & ~(size_t)63; }

static PairBufs pair_bufs(void* base, const FrameParams& fp) {
  PairBufs b{};
  const size_t slots = (size_t)fp.S * ((fp.R + 63) / 64) * 64;
  // (multi-hit frames: room for the fixed per-bounce slots of the folded path, H * slots records)
  const size_t ecap = std::max(echo_cap_of(fp), fp.H > 1 ? slots * fp.H : 0),
               hcap = std::max((size_t)fp.S * fp.R * fp.H, fp.H > 1 ? slots * fp.H : 0);
  uint8_t* p = static_cast<uint8_t*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) { uint8_t* q = p ? p + off : nullptr; off += align256(bytes); return q; };
  b.vp.seg = reinterpret_cast<float4*>(take(ecap * 32));
  b.vp.out = reinterpret_cast<uint2*>(take(ecap * 8));
  b.vp.hrec = reinterpret_cast<float4*>(take(hcap * 16));
  b.vp.echo_cap = (uint32_t)ecap;
  b.pre = reinterpret_cast<int2*>(take(slots * sizeof(int2)));
  if (fp.H > 1) b.state = reinterpret_cast<float4*>(take(slots * (2 * sizeof(float4) + 4) + 2 * kLiveCounters * 4));
  b.total = off;
  return b;
}

size_t fast_pair_bytes(const FrameParams& fp) { return pair_bufs(nullptr, fp).total; }

// Fans per launch_raytrace_fast call: echo pairs and hit records (R*H per fan each) stay below
// 2^31 (u32 indices), the muffle accumulator index (fan * TC + slot) * T + t fits 32 bits, and a
// fan's echo halves stay addressable with a 32-bit half offset into the block
// (fan * stride / 2 < 2^32).
int fast_fans_per_launch(int R, int H, int T, int TC, uint32_t stride) {
  const unsigned long long per_fan = (unsigned long long)R * H + 64;
  const unsigned long long by_pairs = ((1ull << 31) - 64) / per_fan;
  const unsigned long long by_dest = ((1ull << 32) - 1) / ((unsigned long long)(TC > 0 ? TC : 1) * (T > 0 ? T : 1));
  const unsigned long long by_block = ((1ull << 33) - 1) / (stride ? stride : 1) - 1;
  unsigned long long n = std::min(std::min(std::min(by_pairs, by_dest), by_block), (unsigned long long)(1 << 24));
  if (const char* e = getenv("ART_FAST_CHUNK_FANS")) {  // test hook: force small chunks
    const long long v = atoll(e);
    if (v > 0) n = std::min(n, (unsigned long long)v);
  }
  return (int)std::max(1ull, n);
}

// An event pair around one launch (marks may be null); a launch past the pairs is counted as dropped.
template <class F>
static void marked(KernelMarks* marks, int kind, hipStream_t s, F&& launch) {
  const bool m = marks && marks->used < marks->cap;
  if (marks && !m) marks->dropped++;
  if (m) { marks->kind[marks->used] = kind; (void)hipEventRecord(marks->ev[2 * marks->used], s); }
  launch();
  if (m) { (void)hipEventRecord(marks->ev[2 * marks->used + 1], s); marks->used++; }
}

void launch_raytrace_fast(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                          uint8_t* block, uint32_t* muffle_acc, const int* ray_order, void* pair_buf, uint32_t* pair_count,
                          hipStream_t st, const SideStream& echo, KernelMarks* marks) {
  if (fp.S == 0) return;
  const unsigned groups = (unsigned)((size_t)fp.S * ((fp.R + 63) / 64));
  const bool obb = sc.no > 0;  // OBB-free scenes run instantiations without the OBB tests
  PairBufs pb = pair_bufs(pair_buf, fp);
  const unsigned path_blocks = (groups + kPathWaves - 1) / kPathWaves;
  const bool multi = fp.H > 1;
  const uint32_t nacc = (uint32_t)((size_t)fp.S * fp.TC * fp.T);  // this chunk's muffle accumulators
  const uint32_t eb = pb.vp.echo_cap / 64;                         // echo batches (one workgroup each)
  const size_t hcap = (size_t)fp.S * fp.R * fp.H;
  uint32_t* ecnt = pb.state ? reinterpret_cast<uint32_t*>(pb.state + 2 * (size_t)groups * 64) + (size_t)groups * 64 + kLiveCounters
                            : nullptr;  // per-bounce echo counts (echo_counts)
  // One-hit frames with one batch slot trace the echo rays straight from the nearest hits (HM)
  // when the frame's echo traversal fits the chip in one round of waves (4 per 64-ray group, 8 per
  // SIMD): a larger one would hold every wave slot and starve the path kernel beside it (config 4:
  // path 30 -> 977 us).
  const bool split = echo.st != nullptr;
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  const bool hm = split && !multi && fp.TC == 1 && groups <= (unsigned)cus * 8u;
  // Multi-hit frames with one batch slot and no hit outputs fold the path kernel into the nearest
  // kernel (nearest_first_kernel<..., FOLD>): records at fixed per-bounce slots, no live list
  const bool fold = split && multi && fp.TC == 1 && !L.has_hits;
  pb.vp.fixed = fold ? groups * 64u : 0u;
  EchoFromHits eh;
  eh.fp = fp; eh.L = L; eh.origins = origins; eh.ray_order = ray_order; eh.pre = pb.pre;
#define ART_VIS(S_, BLOCKS_, B_, EX_, OBB_, HM_)                                                                   \
  hipLaunchKernelGGL((vis_kernel<EX_, OBB_, HM_>), dim3((unsigned)(BLOCKS_)), dim3(256), 0, S_, sc, pb.vp, pair_count, \
                     EX_ ? fp.exec : nullptr, ecnt, B_, block, eh)
#define ART_VIS_ANY(S_, BLOCKS_, B_, HM_)                                                                              \
  do {                                                                                                                \
    if (fp.exec) { if (obb) ART_VIS(S_, BLOCKS_, B_, true, true, HM_); else ART_VIS(S_, BLOCKS_, B_, true, false, HM_); } \
    else { if (obb) ART_VIS(S_, BLOCKS_, B_, false, true, HM_); else ART_VIS(S_, BLOCKS_, B_, false, false, HM_); }       \
  } while (0)
  // One-hit frames with one batch slot, no hit outputs (HM2): no path kernel at all; the echo
  // traversal writes the misses' reset and the muffle kernel starts from the nearest hits too, at
  // any frame size (no path kernel is left to starve; config 4 1.684 -> 1.660 ms/step)
  const bool hm2 = split && !multi && fp.TC == 1 && !L.has_hits;
  // ... and the two as one launch on st (echo_muffle_kernel)
  const bool fused = hm2;
  eh.no_path = hm2 ? 1 : 0;
  const unsigned mblocks = (ART_MEASURE_PARTS == 1 && hm2) ? 0u : hm2 ? (groups + 3) / 4
                               : (unsigned)(((fold ? (size_t)groups * 64 * fp.H : hcap) + 255) / 256);  // ray slots / hit records
  const unsigned mt = (unsigned)std::min(fp.T, 64);           // targets over the grid (the rest looped)
#define ART_MUFFLE(S_, EX_, OBB_, HM_)                                                                                  \
  hipLaunchKernelGGL((muffle_kernel<EX_, OBB_, HM_>), dim3(mblocks, mt), dim3(256), 0, S_, sc, fp, pb.vp, pair_count, \
                     muffle_acc, eh)
#define ART_MUFFLE_ANY(S_)                                                                                             \
  do {                                                                                                                 \
    if (hm2) {                                                                                                         \
      if (fp.exec) { if (obb) ART_MUFFLE(S_, true, true, true); else ART_MUFFLE(S_, true, false, true); }             \
      else { if (obb) ART_MUFFLE(S_, false, true, true); else ART_MUFFLE(S_, false, false, true); }                   \
    } else {                                                                                                           \
      if (fp.exec) { if (obb) ART_MUFFLE(S_, true, true, false); else ART_MUFFLE(S_, true, false, false); }           \
      else { if (obb) ART_MUFFLE(S_, false, true, false); else ART_MUFFLE(S_, false, false, false); }                 \
    }                                                                                                                  \
  } while (0)
  // Stream plan. Multi-hit frames: per bounce nearest → path on st, that bounce's echo traversal
  // on the side stream right after its path kernel (beside the next bounces' nearest traversals,
  // whose tails leave CUs idle), the muffle kernel after the last bounce on st. One-hit frames
  // with one batch slot (HM): nearest → echo traversal from the hits on st, path → muffle on the
  // side stream (the path kernel leaves the critical path). Other one-hit frames: nearest → path →
  // echo traversal on st, the muffle kernel on the side stream (the longer kernel stays on st: a
  // fork costs ~10 us before the side stream starts). Without a side stream everything runs on st.
  const bool per_bounce = split && multi && ecnt;
  // bounce 0 with the shared-origin node table (nearest_first_kernel<..., TAB>) when a fan's 64-ray
  // groups come in fours, the BVH fits the table and the scene has OBBs. Measured (round 6, A/B of
  // per-kernel HIP-event times): config 3 (4096 OBBs) nearest 68.4 -> 63.3 us, config 5 even; in
  // OBB-free scenes the 1024-lane workgroups and the table build cost more than the table saves
  // (config 2 nearest 50.8 -> 53.6 us), so they keep the 256-lane kernel.
#ifndef ART_NEAREST_TAB
#define ART_NEAREST_TAB 1  // (2: every scene, for A/B runs)
#endif
  const bool tab = ART_NEAREST_TAB && (ART_NEAREST_TAB == 2 || sc.no > 0) && ((fp.R + 63) / 64) % 4 == 0 &&
                   sc.bvh_levels > 0 && (long long)sc.bvh_leaf0 * 4 + 1 <= kTabNodes;
  for (int k = 0; k < (multi ? fp.H : 1); ++k) {
#define ART_NEAREST(EX_, OBB_, F_)                                                                                  \
  do {                                                                                                              \
    if (tab && k == 0)                                                                                              \
      hipLaunchKernelGGL((nearest_first_kernel<EX_, OBB_, F_, true>), dim3(groups / 4), dim3(1024), 0, st, sc, fp, origins, \
                         ray_order, pb.pre, pb.state, k, muffle_acc, nacc, pair_count, L, block, pb.vp);           \
    else                                                                                                            \
      hipLaunchKernelGGL((nearest_first_kernel<EX_, OBB_, F_>), dim3(groups), dim3(256), 0, st, sc, fp, origins, ray_order,  \
                         pb.pre, pb.state, k, muffle_acc, k == 0 ? nacc : 0u, k == 0 ? pair_count : nullptr, L, block, pb.vp); \
  } while (0)
    marked(marks, kMarkNearest, st, [&] {
      if (fold) {
        if (fp.exec) { if (obb) ART_NEAREST(true, true, true); else ART_NEAREST(true, false, true); }
        else { if (obb) ART_NEAREST(false, true, true); else ART_NEAREST(false, false, true); }
      } else {
        if (fp.exec) { if (obb) ART_NEAREST(true, true, false); else ART_NEAREST(true, false, false); }
        else { if (obb) ART_NEAREST(false, true, false); else ART_NEAREST(false, false, false); }
      }
    });
#undef ART_NEAREST
    hipStream_t pst = st;
    if (hm && !hm2) {  // (HM2 forks the muffle rays below)
      (void)hipEventRecord(echo.fork, st);
      (void)hipStreamWaitEvent(echo.st, echo.fork, 0);
      pst = echo.st;
    }
#define ART_PATH(H_, M_)                                                                                              \
  hipLaunchKernelGGL((path_kernel<H_, M_>), dim3(path_blocks), dim3(64 * kPathWaves), 0, pst, sc, fp, L, origins, block, \
                     ray_order, pb.vp, pair_count, pb.pre, pb.state, k, (int)!hm)
    if (hm2 || fold) {}
    else if (L.has_hits) { if (multi) ART_PATH(true, true); else ART_PATH(true, false); }
    else { if (multi) ART_PATH(false, true); else ART_PATH(false, false); }
#undef ART_PATH
    if (per_bounce) {  // this bounce's echoes (at most one per ray slot: `groups` batches)
      (void)hipEventRecord(echo.fork, st);
      (void)hipStreamWaitEvent(echo.st, echo.fork, 0);
      marked(marks, kMarkEcho, echo.st, [&] { ART_VIS_ANY(echo.st, groups, k, false); });
    }
  }
  if (per_bounce) {
    marked(marks, kMarkMuffle, st, [&] { ART_MUFFLE_ANY(st); });  // the bounces' echoes are already on the side stream
  } else if (fused) {
#define ART_ECHO_MUFFLE(EX_, OBB_)                                                                                    \
  hipLaunchKernelGGL((echo_muffle_kernel<EX_, OBB_>), dim3(4 * (groups + mblocks * mt)), dim3(64), 0, \
                     st, sc, fp, pb.vp,   \
                     pair_count, EX_ ? fp.exec : nullptr, block, eh, muffle_acc, groups, mblocks, (int)mt)
    marked(marks, kMarkEchoMuffle, st, [&] {
      if (fp.exec) { if (obb) ART_ECHO_MUFFLE(true, true); else ART_ECHO_MUFFLE(true, false); }
      else { if (obb) ART_ECHO_MUFFLE(false, true); else ART_ECHO_MUFFLE(false, false); }
    });
#undef ART_ECHO_MUFFLE
  } else if (hm) {
    if (hm2) {  // no path kernel: fork the muffle rays here
      (void)hipEventRecord(echo.fork, st);
      (void)hipStreamWaitEvent(echo.st, echo.fork, 0);
    }
    marked(marks, kMarkMuffle, echo.st, [&] { ART_MUFFLE_ANY(echo.st); });  // after the path kernel there
    marked(marks, kMarkEcho, st, [&] { ART_VIS_ANY(st, groups, -1, true); });  // one 64-ray group per workgroup
  } else if (split) {
    (void)hipEventRecord(echo.fork, st);
    (void)hipStreamWaitEvent(echo.st, echo.fork, 0);
    marked(marks, kMarkMuffle, echo.st, [&] { ART_MUFFLE_ANY(echo.st); });
    marked(marks, kMarkEcho, st, [&] { ART_VIS_ANY(st, eb, -1, false); });
  } else {
    marked(marks, kMarkEcho, st, [&] { ART_VIS_ANY(st, eb, -1, false); });
    marked(marks, kMarkMuffle, st, [&] { ART_MUFFLE_ANY(st); });
  }
#undef ART_MUFFLE_ANY
#undef ART_MUFFLE
#undef ART_VIS_ANY
#undef ART_VIS
  if (split && !fused) {
    (void)hipEventRecord(echo.join, echo.st);
    (void)hipStreamWaitEvent(st, echo.join, 0);
  }
}

#ifdef ART_DIAG
extern "C" void art_diag_dump_impl() {
  unsigned long long h[4][64];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_diag), sizeof h) != hipSuccess) return;
  const char* names[4] = {"nearest wave cycles", "echo wave cycles", "nearest ray steps", "echo ray steps"};
  for (int k = 0; k < 4; ++k) {
    fprintf(stderr, "[diag] %s (log2 bucket: count)", names[k]);
    for (int b = 0; b < 64; ++b)
      if (h[k][b]) fprintf(stderr, " %d:%llu", b, h[k][b]);
    fprintf(stderr, "\n");
  }
}
#endif
#ifdef ART_WAVE_TIMES
extern "C" void art_wave_times_dump_impl() {
  const char* path = getenv("ART_WAVE_TIMES_OUT");
  if (!path || hipDeviceSynchronize() != hipSuccess) return;
  static unsigned long long t[kWtCap][2];
  static uint32_t id[kWtCap][3];
  const unsigned n = 0;  // (header word kept for the reader)
  if (hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wt), sizeof t) != hipSuccess ||
      hipMemcpyFromSymbol(id, HIP_SYMBOL(g_wt_id), sizeof id) != hipSuccess)
    return;
  FILE* f = fopen(path, "wb");
  if (!f) return;
  const unsigned cap = kWtCap;
  int dev = 0, khz = 0;  // wall-clock rate
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) khz = 0;
  fwrite(&n, sizeof n, 1, f);
  fwrite(&cap, sizeof cap, 1, f);
  fwrite(&khz, sizeof khz, 1, f);
  fwrite(t, sizeof t, 1, f);
  fwrite(id, sizeof id, 1, f);
  fclose(f);
}
#endif
}  // namespace art
