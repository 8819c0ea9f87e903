// art_trace.hip — the throughput raytrace stage (AudioRaytracerJobBatched.Execute,
// Jobs/AudioRaytracerJobBatched.cs:61-215) on gfx950.
//
// One frame of S fans x R rays is, per bounce k = 0 .. H-1:
//   nearest_first_kernel  nearest hit of every live ray segment (ShootRayCast :225-280) by a
//                         quad-per-ray traversal of the collider BVH (art_bvh.hip);
//   path_kernel           the exact re-evaluation of the winner, the hit point, the echo and
//                         muffle visibility pairs (:121-173) and, for multi-hit frames, the
//                         reflection / termination (:179-193, ReflectRay :456-532) and the ray
//                         state of the next bounce;
// then, once for the frame:
//   pair sort (3 kernels) muffle pairs counting-sorted by (target, direction seen from it);
//   vis_kernel            every pair's any-hit verdict (CanRaySeePoint :365-397,
//                         CanRaySeeAudioTarget :405-449): echo batches by quad BVH traversal,
//                         muffle batches by a box + apex-cone sweep over sorted collider chunks;
//   vis_finalize          visible echoes stored, visible muffle rays counted.
// Every output equals the reference's bit for bit: the broad phases are exact, the
// nearest hit is the (distance, reference order) minimum, any-hit verdicts are ORs.
#include <algorithm>
#include <cstdlib>

#include "art_device_fns.hpp"

namespace art {

constexpr int kNoHit = 0x7fffffff;
constexpr int kNoOwner = 0x7fffffff;  // echo rays skip no collider (AudioTargetId is 16-bit)
constexpr int kMaxQueries = 8;        // pair-emission round: echo + 7 targets, then 8 targets per round
constexpr int kChunk = 64;            // colliders per sorted chunk (art_bvh.hip chunk_bounds_kernel)

// Sphere test split so the common miss costs no branch: the square root and the two IEEE
// divisions run only for lanes whose discriminant is non-negative (RayIntersectsSphere :323-355).
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
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// Executed-work accounting (ART_CTX_COUNT_EXECUTED): one atomic per call from lane 0, off when
// `ex` is null (a uniform branch).
__device__ __forceinline__ void exec_add(unsigned long long* ex, int slot, unsigned long long v) {
  if (ex && v && (threadIdx.x & 63) == 0) atomicAdd(ex + slot, v);
}

// Candidate colliders of one 64-collider chunk: bit i = member i (wave-uniform mask).
struct CandSet {
  unsigned long long m;
  int left;
  __device__ __forceinline__ int pop() {  // next candidate offset (wave-uniform)
    const int k = (int)__builtin_ctzll(m);
    m &= m - 1;
    --left;
    return k;
  }
};

// A ray whose direction or origin is non-finite, or whose direction is zero, makes every box test
// inconclusive: its traversals visit every node (the exact tests alone decide).
__device__ __forceinline__ bool force_all(const Seg& s, float om) {
  return !(isfinite(om) && isfinite(s.d.x) && isfinite(s.d.y) && isfinite(s.d.z)) ||
         (s.d.x == 0.0f && s.d.y == 0.0f && s.d.z == 0.0f);
}

// The widened box of a BVH node / collider (margin factor * (scale + om)):
// entry distance of the segment, or false when it misses the box.
__device__ __forceinline__ bool node_entry(const Seg& s, const CullRec& r, float om, float& tn) {
  const float m = r.factor * (r.scale + om);
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

// (distance, order) minimum over the quad's four lanes.
__device__ __forceinline__ void quad_min(float& d, int& dc) {
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
}

// Quad reductions without ballots (the result lands in every lane of the quad).
__device__ __forceinline__ uint32_t quad_min_u32(uint32_t v) {
  v = min(v, (uint32_t)quad_perm<kQuadXor1>((int)v));
  return min(v, (uint32_t)quad_perm<kQuadXor2>((int)v));
}
__device__ __forceinline__ int quad_max_i32(int v) {
  v = max(v, quad_perm<kQuadXor1>(v));
  return max(v, quad_perm<kQuadXor2>(v));
}

// The BVH node and leaf arrays as buffer resources (wave-uniform bases, 32-bit lane offsets).
struct BvhRes {
  __amdgpu_buffer_rsrc_t nodes, leaves;
};
__device__ __forceinline__ BvhRes bvh_res(const DevScene& sc) {
  BvhRes b;
  const int leaf0 = sc.bvh_leaf0, nleaf = 3 * leaf0 + 1;
  b.nodes = __builtin_amdgcn_make_buffer_rsrc(const_cast<CullRec*>(sc.bvh), 0, (leaf0 + nleaf) * (int)sizeof(CullRec),
                                              0x00020000);
  b.leaves = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(sc.bvh_leaf), 0, nleaf * kBvhLeaf * 64, 0x00020000);
  return b;
}
__device__ __forceinline__ CullRec load_node(const BvhRes& b, int i) {
  const float4 a = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(b.nodes, i * 32, 0, 0));
  const float4 c = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(b.nodes, i * 32 + 16, 0, 0));
  CullRec r;
  r.lox = a.x; r.loy = a.y; r.loz = a.z; r.scale = a.w;
  r.hix = c.x; r.hiy = c.y; r.hiz = c.z; r.factor = c.w;
  return r;
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
__device__ __forceinline__ void quad_descend(bool enter, float en, bool force, int qd, int c0, uint32_t* my, int& g,
                                             int& sp) {
  const uint32_t key = enter ? (((force ? 0u : (uint32_t)__float_as_int(en)) & ~3u) | (uint32_t)qd) : 0xffffffffu;
  const uint32_t k1 = (uint32_t)quad_perm<kQuadRot1>((int)key), k2 = (uint32_t)quad_perm<kQuadXor2>((int)key),
                 k3 = (uint32_t)quad_perm<kQuadRot3>((int)key);
  const int rank = (int)(k1 < key) + (int)(k2 < key) + (int)(k3 < key);
  const uint32_t kmin = min(min(key, k1), min(k2, k3));
  const int nent = quad_max_i32(enter ? rank + 1 : 0);
  if (enter && rank > 0) my[sp + nent - 1 - rank] = (uint32_t)(c0 + qd);
  if (nent) {
    g = c0 + (int)(kmin & 3u);
    sp += nent - 1;
  } else {  // branch-free pop: the stack slot is read unconditionally (clamped), -1 when empty
    const int t = (int)my[sp > 0 ? sp - 1 : 0];
    g = sp > 0 ? t : -1;
    sp = sp > 0 ? sp - 1 : 0;
  }
}

// Exact test of leaf slot `sl` (64 B: the hot record's test fields and the order code, art_bvh.hip
// bvh_leaf_kernel) against segment s; tid = the collider's AudioTargetId. OBB = false: the scene has
// no OBBs (no rank-2 slots), their test compiles out.
template <bool OBB>
__device__ __forceinline__ bool leaf_slot_test(const Seg& s, const BvhRes& br, int slot, int& cc, float& dist, int& tid,
                                               unsigned* nt) {
  auto ld = [&](int k) { return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(br.leaves, slot * 64 + 16 * k, 0, 0)); };
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
  const float4 qc = ld(2), qe = ld(3);
  ObbRec r;
  r.cx = qa.x; r.cy = qa.y; r.cz = qa.z;
  r.qx = qa.w; r.qy = qb.x; r.qz = qb.y; r.qw = qb.z;
  r.lmnx = qc.x; r.lmny = qc.y; r.lmnz = qc.z; r.lmxx = qc.w; r.lmxy = qe.x; r.lmxz = qe.y;
  tid = __float_as_int(qe.z);
  ++nt[2];
  return obb_test<false>(s, r, stored_q(r), dist);
}

// Nearest hit of the quad's ray s (identical in the 4 lanes; `my` = the ray's kBvhStack-entry
// stack): (distance, order) minimum in best / code of every lane of the quad.
template <bool EX, bool OBB>
__device__ __forceinline__ void quad_nearest_core(const DevScene& sc, const Seg& s, bool alive, int lane, uint32_t* my,
                                                  float& best, int& code, unsigned long long* ex) {
  const int qd = lane & 3;
  best = FLT_MAX;
  code = kNoHit;
  if (sc.bvh_levels == 0) return;  // no colliders: every ray misses
  unsigned nt[3] = {0u, 0u, 0u}, nnode = 0;
  const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z);
  const bool force = force_all(s, om);
  const int leaf0 = sc.bvh_leaf0;
  const BvhRes br = bvh_res(sc);
  int g = alive ? 0 : -1, sp = 0;
  // branch-free pop: the stack slot is read unconditionally (clamped), the select picks -1 when empty
  auto pop = [&]() {
    const int t = (int)my[sp > 0 ? sp - 1 : 0];
    g = sp > 0 ? t : -1;
    sp = sp > 0 ? sp - 1 : 0;
  };
  // A child is entered when its widened box is entered at or before the best distance (a winner or
  // tie lies strictly after every ancestor's entry); quad_descend orders the entered ones.
  auto inner_step = [&]() {
    const int c0 = 4 * g + 1;
    if (EX && qd == 0) ++nnode;
    const CullRec r = load_node(br, c0 + qd);
    float tn;
    const bool h = node_entry(s, r, om, tn);
    const float en = fmaxf(tn, 0.0f);
    const bool enter = (r.lox <= r.hix) & (force | (h & (en <= best)));  // bitwise: no branch
    quad_descend(enter, en, force, qd, c0, my, g, sp);
  };
  auto leaf_step = [&](int leaf) {
    int cc, tid;
    float dd;
    const bool h = leaf_slot_test<OBB>(s, br, (leaf - leaf0) * kBvhLeaf + qd, cc, dd, tid, nt);
    // no hit, NaN and FLT_MAX-or-more never win (strict < against float.MaxValue)
    float d = INFINITY;
    int dc = kNoHit;
    if (h && dd < FLT_MAX) { d = dd; dc = cc; }
    quad_min(d, dc);
    if (d < best || (d == best && dc < code)) { best = d; code = dc; }
  };
  // Speculative while-while (Aila & Laine): a quad that reaches a leaf parks it and keeps
  // descending; the wave tests leaves once every quad with work holds one, so both kinds of step
  // run with most quads busy. The order in which leaves are tested does not change the minimum.
  int pend = -1;
  while (__any(g >= 0 || pend >= 0)) {
    {  // Wave priority by unfinished rays: the waves with the most rays left (the ones that set the
       // kernel's length) issue first, the nearly finished ones fill the gaps (s_setprio, 0..3)
      const int act = __popcll(__ballot((g >= 0 || pend >= 0) && qd == 0));
      if (act > 12) __builtin_amdgcn_s_setprio(3);
      else if (act > 8) __builtin_amdgcn_s_setprio(2);
      else if (act > 4) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    for (;;) {
      if (g >= leaf0 && pend < 0) { pend = g; pop(); }
      const bool inner = g >= 0 && g < leaf0;
      if (!__any(inner) || !__any(pend < 0 && g >= 0)) break;
      if (inner) inner_step();
    }
    if (pend >= 0) { leaf_step(pend); pend = -1; }
  }
  if (ex) {
    exec_add(ex, kExecSphere, wave_sum_u32(nt[0]));
    exec_add(ex, kExecAabb, wave_sum_u32(nt[1]));
    exec_add(ex, kExecObb, wave_sum_u32(nt[2]));
    exec_add(ex, kExecCullBox, 4ull * wave_sum_u32(nnode));
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

// EX: count the executed tests (fp.exec); OBB: the scene has OBBs.
template <bool EX, bool OBB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void nearest_first_kernel(
    DevScene sc, FrameParams fp, const float* __restrict__ origins, const int* __restrict__ ray_order,
    int2* __restrict__ hits, float4* __restrict__ state, int step, uint32_t* __restrict__ zero, uint32_t nzero,
    uint32_t* __restrict__ counters) {
  __shared__ uint32_t s_stk[kBvhStack * 64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nrb = (fp.R + 63) >> 6;
  const int ngroups = fp.S * nrb;
  const int g = blockIdx.x;
  const int rr = 16 * w + (lane >> 2);
  uint32_t* my = s_stk + rr * kBvhStack;
  unsigned long long* ex = EX ? fp.exec : nullptr;
  float best;
  int code;
  vec3 o, d;
  bool alive, write;
  uint32_t out;  // ray slot (< 2^31: fast_fans_per_launch)
  if (step > 0) {  // the previous bounce's list of live ray slots
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
  } else {
    if (state && blockIdx.x == 0 && threadIdx.x < 2 * kLiveCounters)  // multi-hit frame: clear the counters
      live_list(state, ngroups)[(size_t)ngroups * 64 + threadIdx.x] = 0u;
    // the frame's muffle accumulators and pair counters, consumed only by later launches (no
    // memset dispatch between frames)
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nzero; i += gridDim.x * 256u) zero[i] = 0u;
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
  quad_nearest_core<EX, OBB>(sc, make_seg(o, d), alive, lane, my, best, code, ex);
  if ((lane & 3) == 0 && write) hits[out] = make_int2(__float_as_int(best), code);
}

// ------------------------------------------------------------------------------------------
// Visibility pairs. The path kernel emits every (hit, query) pair with its output destination;
// visibility never feeds back into ray paths (echo :124-145 and muffle :150-173 only write
// outputs), so the verdicts can be computed after all bounces.
// Pair arrays (struct of arrays). Echo pairs i in [0, echo_cap), emission order (the 64 rays of a
// wave share the fan origin, one batch each):
//   seg[2 i], seg[2 i + 1]  (o.xyz, maxd), (d.xyz, kNoOwner)  32 B, read by the echo traversal;
//                           1/d and dot(d, d) are recomputed there by make_seg (same operations)
//   out[i]                  (u16 index of the echo in the fan blocks, echo half)  8 B, vis_finalize
// Muffle pairs e in [0, S R H T), emission order:
//   mrec[e]                 (off.xyz, e << tbits | t)  16 B: the segment's start and its target
//                           (bit 31 of w: blocked, set in the sorted copy by the sweep);
//                           maxd and the direction to the target are recomputed by the sweep with
//                           the path kernel's operations
//   mdest[e]                muffle_acc index  4 B, read by vis_finalize
//   msorted[]               mrec counting-sorted by key (pair_scatter_kernel): the sweep reads its
//                           batches of 64 coalesced, 16 B per pair
// flag[i] / flag[echo_cap + e]: 0 = no blocker found yet, 1 = blocked. counts[0] / counts[1] = echo /
// muffle pairs emitted.
// ------------------------------------------------------------------------------------------
struct VisPairs {
  float4* seg;
  uint2* out;
  uint32_t* flag;
  float4* mrec;
  float4* msorted;
  uint32_t* mdest;
  uint32_t echo_cap;  // multiple of 64
  int tbits;          // target bits of a muffle record's w
};

// Bits of a target index (T targets): the muffle records pack (e << bits | t) into 32 bits.
__host__ __device__ inline int target_bits(int T) {
  int b = 0;
  while ((1 << b) < T) ++b;
  return b;
}

__device__ __forceinline__ void load_pair_seg(const VisPairs& vp, uint32_t i, Seg& s, float& maxd, int& owner) {
  const float4 q0 = vp.seg[2 * (size_t)i], q1 = vp.seg[2 * (size_t)i + 1];
  s = make_seg(mk3(q0.x, q0.y, q0.z), mk3(q1.x, q1.y, q1.z));
  maxd = q0.w;
  owner = __float_as_int(q1.w);
}

// Sort key of a muffle pair: target t and the octahedral Morton cell (32 x 32) of the ray's
// direction seen from the target, so 64 consecutive sorted pairs form a thin cone with apex t
// (1024 cells per target: 1.8 % broad-phase candidates in simulation, 4096: 1.6 %). Above 8
// targets the low Morton bits are dropped so that T << bits stays within the LDS histogram.
constexpr int kSortDirBits = 10, kSortBins = 8 << kSortDirBits;
__host__ __device__ inline int sort_dir_bits(int T) {
  int b = kSortDirBits;
  while (b > 1 && (T << b) > kSortBins) --b;
  return b;
}
__device__ __forceinline__ uint16_t vis_sort_key(int t, int T, vec3 u) {
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
  const int bits = sort_dir_bits(T);
  const uint32_t cell = (sp(q5(a)) | (sp(q5(c)) << 1)) >> (kSortDirBits - bits);
  return (uint16_t)(((uint32_t)t << bits) | cell);
}

__device__ __forceinline__ float echo_of(const DevScene& sc, int type, int idx) {
  return type == kSphere ? sc.sphc[idx].echo : (type == kAabb ? sc.aabbc[idx].echo : sc.obbc[idx].echo);
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
    const int* __restrict__ ray_order, VisPairs vp, uint32_t* __restrict__ pair_count, uint16_t* __restrict__ pkeys,
    const int2* __restrict__ pre_hits, float4* __restrict__ state, int step) {
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
      const int rank = bc >> 28;
      idx = bc & 0x0fffffff;
      type = rank == 0 ? kSphere : (rank == 1 ? kAabb : kObb);
      // exact (Unity min/max) re-evaluation of a zero distance: IEEE and Unity min/max differ only
      // in the sign of an equal-magnitude zero pair, so only a zero result can differ (its sign)
      if (dist == 0.0f) {
        if (type == kAabb) aabb_test<true>(s, sc.aabb[idx], dist);
        if (type == kObb) { const ObbRec r = sc.obb[idx]; obb_test<true>(s, r, stored_q(r), dist); }
      }
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

    // visibility pairs: q = 0 echo ray to the origin (:124-145), q = 1..T muffle rays (:150-173),
    // in rounds of kMaxQueries queries (the ballot masks stay in registers), one reservation each
    const vec3 off = o - d * kEps;                 // :124, :158
    const float dist0 = distance(O, o);            // :130 (un-offset hit point)
    for (int q0 = 0; q0 <= T; q0 += kMaxQueries) {  // block-uniform
      unsigned long long mq[kMaxQueries];
      uint32_t actbits = 0, np = 0;
#pragma unroll
      for (int qq = 0; qq < kMaxQueries; ++qq) {
        const int q = q0 + qq;
        bool act = false;
        if (q <= T) {
          if (q == 0) act = live_slot;  // the echo is written only into a live slot (:118)
          else act = hit && distance(off, load3(sc.targets, q - 1)) < fp.max_muffle;  // :165-168
        }
        mq[qq] = __ballot(act);
        actbits |= act ? (1u << qq) : 0u;
        np += (uint32_t)__popcll(mq[qq]);
      }
      const uint32_t ne = q0 == 0 ? (uint32_t)__popcll(mq[0]) : 0u, nm = np - ne;
      uint32_t eb, mb;
      reserve(ne, nm, pair_count, eb, mb);
      if (np) {
        uint32_t pos = mb;  // muffle position (region-relative)
#pragma unroll
        for (int qq = 0; qq < kMaxQueries; ++qq) {
          const int q = q0 + qq;
          if (q <= T && ((actbits >> qq) & 1u)) {
            const uint32_t rank = (uint32_t)__popcll(mq[qq] & lt);
            if (q == 0) {  // the echo ray to the fan origin (:124-145): its segment in full
              const uint32_t at = eb + rank;
              const vec3 qdir = normalize(O - off);
              vp.seg[2 * (size_t)at] = make_float4(off.x, off.y, off.z, dist0);
              vp.seg[2 * (size_t)at + 1] = make_float4(qdir.x, qdir.y, qdir.z, __int_as_float(kNoOwner));
              vp.out[at] = make_uint2((uint32_t)(((size_t)fan * L.stride + L.echo_off) / 2) + (uint32_t)(ray * H + k),
                                      f32tof16(dist0 * echo_of(sc, type, idx)));  // :142-144
              vp.flag[at] = 0u;
            } else {  // a muffle ray to target q - 1 (:150-173): its start, target and counter
              const uint32_t e = pos + rank;
              const vec3 qdir = normalize(load3(sc.targets, q - 1) - off);  // :158-160
              vp.mrec[e] = make_float4(off.x, off.y, off.z, __uint_as_float((e << vp.tbits) | (uint32_t)(q - 1)));
              vp.mdest[e] = (uint32_t)(((size_t)fan * fp.TC + my_slot) * T + (q - 1));
              vp.flag[vp.echo_cap + e] = 0u;
              pkeys[e] = vis_sort_key(q - 1, T, mk3(-qdir.x, -qdir.y, -qdir.z));
            }
          }
          if (q > 0 && q <= T) pos += (uint32_t)__popcll(mq[qq]);
        }
      }
    }
    // a blocked echo leaves the reset value (:76); vis_finalize overwrites the visible ones
    if (live_slot && single_slot) echo[ray * H + k] = 0;

    // termination / reflection — :179-193, ReflectRay :456-532
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
        if (life < 0.0f) alive = false;
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
      const unsigned long long m = __ballot(app);
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
// Counting sort of the muffle pairs by key (T << bits buckets; the order inside a bucket is free:
// the any-hit verdicts do not depend on it). Block j of kSortBlock pairs: LDS histogram -> row j
// of hist[block][bucket]; a column prefix per bucket and the buckets' totals; each scatter block
// scans the totals and hands out positions with LDS atomics.
// ------------------------------------------------------------------------------------------
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
                                                                    const float4* __restrict__ mrec,
                                                                    float4* __restrict__ msorted, int nblk, int nbins) {
  __shared__ uint32_t cur[kSortBins];
  __shared__ uint32_t s_part[kSortThreads];
  __builtin_amdgcn_s_setprio(3);  // on the critical path; issues ahead of the echo traversal beside it
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
    msorted[atomicAdd(&cur[kk[j]], 1u)] = mrec[i0 + j];
  }
}

// ------------------------------------------------------------------------------------------
// Broad phase of the muffle sweep. A batch of 64 sorted pairs (one target, nearby directions seen
// from it) is reduced to the box of its segments [o, o + maxd d] and an apex cone: all its
// segments end at (nearly) the same point, the target (:165); echo segments of one wave end at the
// fan origin (:130). A collider whose widened bounds miss the box or the cone cannot block any
// lane's segment, so every verdict equals the brute-force OR.
// ------------------------------------------------------------------------------------------
struct WaveBox {
  float lx, ly, lz, hx, hy, hz, om;
};

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

// Apex cone of a wave of segments that (nearly) share their END point. Apex A = the first valid
// lane's computed end point; every lane's end point lies within `extra` of A (its computed
// distance, widened for the rounding of o + maxd d), so each segment lies in the hull of its
// start o and the ball (A, extra), and that hull lies in cone(A, axis, theta) (+) ball(extra) once
// o is inside the cone. Starts inside the ball need no cone. A wave with a non-finite segment,
// whose starts all lie in the ball, or whose cone is wider than a half-space, is not cone-culled
// (on = false). theta carries a 2e-3 rad slack for the rounding of the normalisations.
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

constexpr int kCullU = 4;  // candidate tests per scalar-load group

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

// Any-hit sweep of one lane's segment (s, maxd, owner) over the sorted chunks [c_lo, c_hi) for a
// wave of up to 64 segments (`valid` lanes): the chunks' union bounds first (lane = chunk), then
// the members of the candidate chunks (lane = collider), then exact wave-uniform tests of the
// candidates. Any-hit is an OR over the colliders, so the order is free. Returns the lane's
// verdict (true = blocked).
template <bool OBB>
__device__ __forceinline__ bool cull_sweep(const DevScene& sc, const Seg& s, float maxd, int owner, bool valid, int lane,
                                           unsigned long long* ex, int c_lo, int c_hi, const VisCone& vc) {
  const int cs_n = (sc.ns + kChunk - 1) / kChunk, ca_n = (sc.na + kChunk - 1) / kChunk;
  const int nchunks = min(sc.nchunks, c_hi);
  if (c_lo >= nchunks) return false;
  const WaveBox wb = make_wave_box(s, maxd, valid);
  bool blocked = false;
  const bool done = !valid;
  if (__all(done)) return false;
  unsigned nt[3] = {0u, 0u, 0u}, nchk = 0u;
  // broad-phase candidate: widened bounds meet the wave box and the cone
  auto candidate = [&](const CullRec& cr) {
    const float m = cr.factor * (cr.scale + wb.om);
    bool c = (cr.lox - m <= wb.hx) & (cr.hix + m >= wb.lx) & (cr.loy - m <= wb.hy) & (cr.hiy + m >= wb.ly) &
             (cr.loz - m <= wb.hz) & (cr.hiz + m >= wb.lz);
    if (vc.on && __any(c)) c = c && vis_cone_cand(vc, cr, wb.om);
    return c;
  };
  const float oml = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
  const bool force = force_all(s, oml);
  for (int pb = c_lo; pb < nchunks; pb += 64) {
    const int pc = pb + lane;
    bool ccand = false;
    if (pc < nchunks) ccand = candidate(sc.chunks[pc]);
    unsigned long long cm_mask = __ballot(ccand);
    ++nchk;
    while (cm_mask) {
      const int c = pb + (int)__builtin_ctzll(cm_mask);
      cm_mask &= cm_mask - 1;
      int type, b, n, g;
      if (c < cs_n) { type = 0; b = c * kChunk; n = min(kChunk, sc.ns - b); g = b; }
      else if (c < cs_n + ca_n) { type = 1; b = (c - cs_n) * kChunk; n = min(kChunk, sc.na - b); g = sc.ns + b; }
      else { type = 2; b = (c - cs_n - ca_n) * kChunk; n = min(kChunk, sc.no - b); g = sc.ns + sc.na + b; }
      bool cand = false;
      if (lane < n) cand = candidate(sc.cull_s[g + lane]);
      CandSet cs;
      cs.m = __ballot(cand);
      cs.left = __popcll(cs.m);
      ++nchk;
      if (cs.left == 0) continue;
      if (type == 0) {
        blocked = test_candidates<kCullU>(sc.sph_s, b, cs, blocked, done, [&](const SphereRec& r) {
          float d;
          return sphere_hit_dist(s, r, d) && d < maxd && r.tid != owner;
        }, nt[0]);
      } else if (type == 1) {
        blocked = test_candidates<kCullU>(sc.aabb_s, b, cs, blocked, done, [&](const AabbRec& r) {
          float d;
          return aabb_test<false>(s, r, d) && d < maxd && r.tid != owner;
        }, nt[1]);
      } else if (OBB) {
        // OBB candidates (118-op exact test): first each lane's slab test against the collider's own
        // widened bounds (a blocker's segment enters them before maxd); the
        // exact test runs only where a live lane passes
        const CullRec* cb = sc.cull_s + sc.ns + sc.na;
        while (cs.left > 0) {
          const int i = wave_uniform(b + cs.pop());
          const CullRec cr = ldc(cb, i);
          float tn;
          const bool h = node_entry(s, cr, oml, tn);
          const bool near = force || (h && tn <= maxd);
          if (!__any(near && !blocked && !done)) continue;
          const ObbRec r = ldc(sc.obb_s, i);
          ++nt[2];
          if (near && !blocked) {
            float d;
            blocked = obb_test<false>(s, r, stored_q(r), d) && d < maxd && r.tid != owner;
          }
          if (__all(blocked || done)) break;
        }
      }
      if (__all(blocked || done)) break;
    }
    if (__all(blocked || done)) break;
  }
  exec_add(ex, kExecSphere, 64ull * nt[0]);
  exec_add(ex, kExecAabb, 64ull * nt[1]);
  exec_add(ex, kExecObb, 64ull * nt[2]);
  exec_add(ex, kExecCullBox, 64ull * nchk);
  return blocked;
}

// Chunk ranges per 64-pair batch (work items of the muffle sweep), by scene kind: each range
// repeats the batch's setup, while OBB tests are long and balance better over more items.
// Measured (raytrace stage): no OBBs 2 ranges (config 2: 218 vs 231 us at 4, 274 at 1); OBB
// majority 8 (config 3: 0.98 vs 1.01 ms at 4); some OBBs 4 (config 4: 5.73 vs 5.84 ms at 8,
// config 5: 2.69 vs 2.81).
__host__ __device__ __forceinline__ int vis_ranges(const DevScene& sc) {
  return 2 * sc.no > sc.ns + sc.na + sc.no ? 8 : (sc.no > 0 ? 4 : 2);
}

// Work item i of the muffle sweep = (chunk range r, sorted batch b), range-major: r = i / nbm,
// b = i % nbm. Lane = sorted position 64 b + lane: its record gives the segment's start, its target
// t and its emission index e; maxd and the direction to the target are recomputed with the path
// kernel's operations (:158-168), so the segment is the one the reference tests. A batch's later
// ranges usually start after its earlier ones finished and skip the pairs those already blocked:
// a blocker sets bit 31 of the sorted record (coalesced, read with the record; a stale read only
// costs work) and the pair's flag[echo_cap + e] for vis_finalize, both by relaxed device-scope
// atomicOr (no fences: an agent-scope release writes back the XCD's L2); vis_finalize writes the
// outputs after the kernel boundary.
template <bool OBB>
__device__ __forceinline__ void vis_sweep_body(const DevScene& sc, const VisPairs& vp, const uint32_t* count,
                                               uint32_t nbm, unsigned long long* ex, uint32_t blk) {
  const int lane = threadIdx.x & 63;
  __builtin_amdgcn_s_setprio(1);  // the sweep ends the frame's critical path; the echo waves beside it have slack
  const uint32_t item = blk * 4u + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t r = item / nbm, b = item - r * nbm;
  const int nranges = vis_ranges(sc);
  const uint32_t base = b * 64u, n = ldc(count, 1);
  if (r >= (uint32_t)nranges || base >= n) return;
  const uint32_t n_in = min(64u, n - base);
  const uint32_t p = base + ((uint32_t)lane < n_in ? (uint32_t)lane : 0u);
  const float4 rec = vp.msorted[p];
  const uint32_t wv = __float_as_uint(rec.w), e = (wv & 0x7fffffffu) >> vp.tbits;
  const int t = (int)(wv & ((1u << vp.tbits) - 1u));
  // pairs an earlier range already blocked (bit 31 of the sorted record) are skipped (out of the
  // wave's box)
  const bool valid = (uint32_t)lane < n_in && (wv >> 31) == 0u;
  if (!__any(valid)) return;
  Seg s;
  float maxd = 0.0f;
  s.o = s.d = s.inv = mk3(0.0f, 0.0f, 0.0f);
  s.a2 = 0.0f;
  if (valid) {
    const vec3 off = mk3(rec.x, rec.y, rec.z), tp = load3(sc.targets, t);
    maxd = distance(off, tp);                // :165
    s = make_seg(off, normalize(tp - off));  // :158-160
  }
  const int nch = sc.nchunks;
  const int c_lo = (int)(((long long)nch * r) / nranges), c_hi = (int)(((long long)nch * (r + 1)) / nranges);
  const float om = wave_max(valid ? fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd : 0.0f);
  const VisCone vc = make_vis_cone(s, maxd, valid, om);
  const bool blocked = cull_sweep<OBB>(sc, s, maxd, t, valid, lane, ex, c_lo, c_hi, vc);  // owner = t (:413, :426, :439)
  if (valid && blocked) {
    __hip_atomic_fetch_or(reinterpret_cast<uint32_t*>(vp.msorted + p) + 3, 0x80000000u, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_or(vp.flag + vp.echo_cap + e, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------------------------------
// Echo visibility by quad-per-segment BVH traversal. An echo batch is one wave's rays of one fan
// traced back to the fan origin: 64 segments fanning over an eighth of the sphere, whose box and
// cone admit ~10 % of the colliders, so a sweep would spend most of its time there. Per segment
// the BVH visits only the nodes along it: a segment enters a node when its widened box is entered
// before maxd (a blocker's computed distance d < maxd lies strictly after every ancestor's
// entry), 4 lanes per segment (lane q: child q / leaf slot q; the quad agrees through ballots),
// the first blocker ends the segment.
// ------------------------------------------------------------------------------------------
template <bool OBB>
__device__ __forceinline__ void vis_quad_body(const DevScene& sc, const VisPairs& vp, const uint32_t* count,
                                              unsigned long long* ex, uint32_t blk, uint32_t* s_stk,
                                              const uint32_t* ecnt, int bounce) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), qd = lane & 3;
  const int slot = w * 16 + (lane >> 2);                       // segment of the block's 64-pair batch
  // all echo pairs, or (bounce >= 0) those bounce `bounce` emitted: they follow the earlier bounces'
  uint32_t start = 0u, n;
  if (bounce < 0) {
    n = ldc(count, 0);
  } else {
    for (int j = 0; j < bounce; ++j) start += ldc(ecnt, j);
    n = start + ldc(ecnt, bounce);
  }
  const uint32_t base = start + blk * 64u;
  if (sc.bvh_levels == 0) return;                              // no colliders: nothing blocks
  if (base + (uint32_t)(w * 16) >= n) return;                  // this wave's 16 segments are past the emitted pairs
  const bool valid = base + (uint32_t)slot < n;
  const uint32_t p = valid ? base + (uint32_t)slot : base;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwner;
  s.o = s.d = s.inv = mk3(0.0f, 0.0f, 0.0f);
  s.a2 = 0.0f;
  if (valid) load_pair_seg(vp, p, s, maxd, owner);
  const float om = fabsf(s.o.x) + fabsf(s.o.y) + fabsf(s.o.z) + maxd;
  const bool force = force_all(s, om);
  const int leaf0 = sc.bvh_leaf0, qshift = lane & ~3;
  const BvhRes br = bvh_res(sc);
  uint32_t* my = s_stk + slot * kBvhStack;
  unsigned nt[3] = {0u, 0u, 0u}, nnode = 0;
  bool blocked = false;
  int g = valid ? 0 : -1, sp = 0;
  while (__any(g >= 0)) {
    while (g >= 0 && g < leaf0) {  // quad-uniform
      const int c0 = 4 * g + 1;
      if (qd == 0) ++nnode;
      const CullRec r = load_node(br, c0 + qd);
      float tn;
      const bool h = node_entry(s, r, om, tn);
      const bool enter = (r.lox <= r.hix) & (force | (h & (tn <= maxd)));  // bitwise: no branch
      const uint32_t eb = (uint32_t)(__ballot(enter) >> qshift) & 0xFu;
      if (eb) {
        const int first = __builtin_ctz(eb);
        const uint32_t rest = eb & (eb - 1u);
        if (enter && qd != first) my[sp + __popc(rest & ((1u << qd) - 1u))] = (uint32_t)(c0 + qd);
        sp += __popc(rest);
        g = c0 + first;
      } else {
        g = sp ? (int)my[sp - 1] : -1;
        sp = sp ? sp - 1 : 0;
      }
    }
    if (g >= leaf0) {
      int cc, tid;
      float d;
      const bool hh = leaf_slot_test<OBB>(s, br, (g - leaf0) * kBvhLeaf + qd, cc, d, tid, nt);
      const bool blk_here = hh && d < maxd && tid != owner;  // :373-394, :411-447
      if ((uint32_t)(__ballot(blk_here) >> qshift) & 0xFu) {
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
    exec_add(ex, kExecSphere, wave_sum_u32(nt[0]));
    exec_add(ex, kExecAabb, wave_sum_u32(nt[1]));
    exec_add(ex, kExecObb, wave_sum_u32(nt[2]));
    exec_add(ex, kExecCullBox, 4ull * wave_sum_u32(nnode));
  }
}

// One launch for both visibility halves, so they overlap on the chip: blocks [0, n_echo) trace
// the echo batches by quad BVH traversal (longer jobs first), the others run the sweep's items.
// EX: count the executed tests (fp.exec); without it the counters compile out. 8 waves per SIMD
// (a few VGPRs spill; measured faster than 6 or 7).
template <bool EX, bool OBB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8)))
void vis_kernel(DevScene sc, VisPairs vp, const uint32_t* __restrict__ count, uint32_t nbm, unsigned long long* ex,
                uint32_t n_echo, const uint32_t* __restrict__ ecnt, int bounce) {
  __shared__ uint32_t s_stk[64 * kBvhStack];
  unsigned long long* e = EX ? ex : nullptr;
  if (blockIdx.x < n_echo) vis_quad_body<OBB>(sc, vp, count, e, blockIdx.x, s_stk, ecnt, bounce);
  else vis_sweep_body<OBB>(sc, vp, count, nbm, e, blockIdx.x - n_echo);
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
  const bool muf = !echo_region;
  if (valid) {
    flag = vp.flag[p];
    if (muf) { dest = vp.mdest[rel]; } else { const uint2 o = vp.out[p]; dest = o.x; val = o.y; }
  }
  const bool vis = valid && flag == 0u;
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

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
// Pair buffer: VisPairs (echo seg | echo out | flag | muffle records | sorted records | muffle dest)
// | first-segment hits | ray state + live list (multi-hit) | muffle keys u16 | hist, scanned hist
// u32[bins x blocks] | bucket totals.
struct PairBufs {
  VisPairs vp;
  uint16_t* keys;
  uint32_t *hist, *prefix, *tot;
  int2* pre;        // [groups * 64] nearest hits of the current bounce
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
  const size_t slots = (size_t)fp.S * ((fp.R + 63) / 64) * 64;
  uint8_t* p = static_cast<uint8_t*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) { uint8_t* q = p ? p + off : nullptr; off += align256(bytes); return q; };
  b.vp.seg = reinterpret_cast<float4*>(take(ecap * 32));
  b.vp.out = reinterpret_cast<uint2*>(take(ecap * 8));
  b.vp.flag = reinterpret_cast<uint32_t*>(take(max_pairs * 4));
  b.vp.mrec = reinterpret_cast<float4*>(take(mcap * 16));
  b.vp.msorted = reinterpret_cast<float4*>(take(mcap * 16));
  b.vp.mdest = reinterpret_cast<uint32_t*>(take(mcap * 4));
  b.vp.echo_cap = (uint32_t)ecap;
  b.vp.tbits = target_bits(fp.T);
  b.pre = reinterpret_cast<int2*>(take(slots * sizeof(int2)));
  if (fp.H > 1) b.state = reinterpret_cast<float4*>(take(slots * (2 * sizeof(float4) + 4) + 2 * kLiveCounters * 4));
  if (mcap) {
    b.nblk = (int)((mcap + kSortBlock - 1) / kSortBlock);
    b.nbins = fp.T << sort_dir_bits(fp.T);  // keys (target << bits | cell) < T << bits <= kSortBins
    const size_t cells = (size_t)b.nbins * b.nblk;
    b.keys = reinterpret_cast<uint16_t*>(take(mcap * 2 + 64));  // + padding for load_keys16 past the end
    b.hist = reinterpret_cast<uint32_t*>(take(cells * 4));
    b.prefix = reinterpret_cast<uint32_t*>(take(cells * 4));
    b.tot = reinterpret_cast<uint32_t*>(take((size_t)b.nbins * 4));
  }
  b.total = off;
  return b;
}

size_t fast_pair_bytes(const FrameParams& fp) { return pair_bufs(nullptr, fp).total; }

// Fans per launch_raytrace_fast call: pair slots (echo + muffle, R*H*(T+1) per fan) stay below
// 2^31 (u32 slots and sorted positions), muffle emission indices fit the records' 31 - tbits bits,
// and a fan's echo halves stay addressable with a 32-bit half offset into the block
// (fan * stride / 2 < 2^32).
int fast_fans_per_launch(int R, int H, int T, uint32_t stride) {
  const unsigned long long per_fan = (unsigned long long)R * H * (T + 1) + 64;
  const unsigned long long by_pairs = ((1ull << 31) - 64) / per_fan;
  const unsigned long long mper_fan = (unsigned long long)R * H * (T > 0 ? T : 1);
  const unsigned long long by_rec = ((1ull << (31 - target_bits(T))) - 1) / mper_fan;
  const unsigned long long by_block = ((1ull << 33) - 1) / (stride ? stride : 1) - 1;
  unsigned long long n = std::min(std::min(std::min(by_pairs, by_rec), by_block), (unsigned long long)(1 << 24));
  if (const char* e = getenv("ART_FAST_CHUNK_FANS")) {  // test hook: force small chunks
    const long long v = atoll(e);
    if (v > 0) n = std::min(n, (unsigned long long)v);
  }
  return (int)std::max(1ull, n);
}

void launch_raytrace_fast(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                          uint8_t* block, uint32_t* muffle_acc, const int* ray_order, void* pair_buf, uint32_t* pair_count,
                          hipStream_t st, const SideStream& echo) {
  if (fp.S == 0) return;
  const PairBufs pb = pair_bufs(pair_buf, fp);
  const size_t mcap = muffle_cap_of(fp), max_pairs = (size_t)pb.vp.echo_cap + mcap;
  const unsigned groups = (unsigned)((size_t)fp.S * ((fp.R + 63) / 64));
  const unsigned path_blocks = (groups + kPathWaves - 1) / kPathWaves;
  const bool multi = fp.H > 1;
  const bool obb = sc.no > 0;  // OBB-free scenes run instantiations without the OBB tests
  const uint32_t nacc = (uint32_t)((size_t)fp.S * fp.TC * fp.T);  // this chunk's muffle accumulators
  const uint32_t nb_max = (uint32_t)(pb.vp.echo_cap / 64 + (mcap + 63) / 64);
  const uint32_t eb = pb.vp.echo_cap / 64;  // echo batches (one workgroup each)
  const uint32_t nbm = nb_max - eb;         // muffle batches (vis_ranges items each, 4 per workgroup)
  const size_t mblocks = ((size_t)nbm * vis_ranges(sc) + 3) / 4;
  uint32_t* ecnt = pb.state ? reinterpret_cast<uint32_t*>(pb.state + 2 * (size_t)groups * 64) + (size_t)groups * 64 + kLiveCounters
                            : nullptr;  // per-bounce echo counts (echo_counts)
#define ART_VIS(S_, BLOCKS_, NECHO_, B_, EX_, OBB_)                                                                \
  hipLaunchKernelGGL((vis_kernel<EX_, OBB_>), dim3((unsigned)(BLOCKS_)), dim3(256), 0, S_, sc, pb.vp, pair_count, nbm, \
                     EX_ ? fp.exec : nullptr, NECHO_, ecnt, B_)
#define ART_VIS_ANY(S_, BLOCKS_, NECHO_, B_)                                                                      \
  do {                                                                                                           \
    if (fp.exec) { if (obb) ART_VIS(S_, BLOCKS_, NECHO_, B_, true, true); else ART_VIS(S_, BLOCKS_, NECHO_, B_, true, false); } \
    else { if (obb) ART_VIS(S_, BLOCKS_, NECHO_, B_, false, true); else ART_VIS(S_, BLOCKS_, NECHO_, B_, false, false); }    \
  } while (0)
  // The echo traversal (latency-bound) needs only the path kernel's pairs, so it runs on the side
  // stream: in multi-hit frames each bounce's echoes right after that bounce's path kernel, beside
  // the next bounces' nearest traversals (their tails leave CUs idle) and then the pair sort; in
  // one-hit frames beside the pair sort and the VALU-bound muffle sweep. Without a side stream both
  // halves share one vis_kernel launch (echo workgroups first).
  const bool split = echo.st && eb && mcap;
  const bool per_bounce = split && multi && ecnt;
  for (int k = 0; k < (multi ? fp.H : 1); ++k) {
#define ART_NEAREST(EX_, OBB_)                                                                                      \
  hipLaunchKernelGGL((nearest_first_kernel<EX_, OBB_>), dim3(groups), dim3(256), 0, st, sc, fp, origins, ray_order, pb.pre, \
                     pb.state, k, muffle_acc, k == 0 ? nacc : 0u, k == 0 ? pair_count : nullptr)
    if (fp.exec) { if (obb) ART_NEAREST(true, true); else ART_NEAREST(true, false); }
    else { if (obb) ART_NEAREST(false, true); else ART_NEAREST(false, false); }
#undef ART_NEAREST
#define ART_PATH(H_, M_)                                                                                              \
  hipLaunchKernelGGL((path_kernel<H_, M_>), dim3(path_blocks), dim3(64 * kPathWaves), 0, st, sc, fp, L, origins, block, \
                     ray_order, pb.vp, pair_count, pb.keys, pb.pre, pb.state, k)
    if (L.has_hits) { if (multi) ART_PATH(true, true); else ART_PATH(true, false); }
    else { if (multi) ART_PATH(false, true); else ART_PATH(false, false); }
#undef ART_PATH
    if (per_bounce) {  // this bounce's echoes (at most one per ray slot: `groups` batches)
      (void)hipEventRecord(echo.fork, st);
      (void)hipStreamWaitEvent(echo.st, echo.fork, 0);
      ART_VIS_ANY(echo.st, groups, groups, k);
    }
  }
  if (!nb_max) return;
  if (split && !per_bounce) {
    (void)hipEventRecord(echo.fork, st);
    (void)hipStreamWaitEvent(echo.st, echo.fork, 0);
    ART_VIS_ANY(echo.st, eb, eb, -1);
  }
  if (split) (void)hipEventRecord(echo.join, echo.st);
  if (mcap) {
    hipLaunchKernelGGL(pair_hist_kernel, dim3(pb.nblk), dim3(kSortThreads), 0, st, pb.keys, pair_count, pb.hist, pb.nblk,
                       pb.nbins);
    hipLaunchKernelGGL(pair_colscan_kernel, dim3((pb.nbins + 63) / 64), dim3(64), 0, st, pb.hist, pb.prefix, pb.tot, pb.nblk,
                       pb.nbins);
    hipLaunchKernelGGL(pair_scatter_kernel, dim3(pb.nblk), dim3(kSortThreads), 0, st, pb.keys, pair_count, pb.prefix, pb.tot,
                       pb.vp.mrec, pb.vp.msorted, pb.nblk, pb.nbins);
  }
  if (split) {
    ART_VIS_ANY(st, mblocks, 0u, -1);
    (void)hipStreamWaitEvent(st, echo.join, 0);
  } else if (eb + mblocks) {
    ART_VIS_ANY(st, eb + mblocks, eb, -1);
  }
#undef ART_VIS_ANY
#undef ART_VIS
  hipLaunchKernelGGL(vis_finalize, dim3((unsigned)((max_pairs + 255) / 256)), dim3(256), 0, st, pb.vp, pair_count, block,
                     muffle_acc);
}

}  // namespace art
