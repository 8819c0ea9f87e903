// art_bvh.hip — the collider BVH of the quad traversals (art_trace.hip).
//
// The reference sweeps colliders in their list order (Sphere, AABB, OBB; AudioRaytracerJobBatched.cs
// :225-280), and the exact tests keep that order's tie-break (the global order code). The broad
// phase is a complete 4-ary tree over all colliders in a spatial leaf order (the kd order below;
// Morton above kKdMaxColliders), built once per scene upload on the device and refit in place when
// a resident sync only moved colliders.
#include <cstdlib>
#include <hipcub/hipcub.hpp>

#include "art_device_fns.hpp"
#include "art_frame_math.hpp"

namespace art {

// Centre of a collider's bounds, or false for non-finite bounds (those sort anywhere).
__device__ __forceinline__ bool bound_centre(const CullRec& c, float& x, float& y, float& z) {
  x = 0.5f * (c.lox + c.hix); y = 0.5f * (c.loy + c.hiy); z = 0.5f * (c.loz + c.hiz);
  return isfinite(x) && isfinite(y) && isfinite(z);
}

// Scene box of the finite centres (one workgroup; the scene has at most a few 10^5 colliders).
__global__ __launch_bounds__(1024) void scene_box_kernel(const CullRec* __restrict__ cull, int n, float* __restrict__ box) {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float c[3];
    if (!bound_centre(cull[i], c[0], c[1], c[2])) continue;
    for (int a = 0; a < 3; ++a) { lo[a] = fminf(lo[a], c[a]); hi[a] = fmaxf(hi[a], c[a]); }
  }
  __shared__ float s[6][1024];
  for (int a = 0; a < 3; ++a) { s[a][threadIdx.x] = lo[a]; s[3 + a][threadIdx.x] = hi[a]; }
  __syncthreads();
  for (int st = blockDim.x / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st)
      for (int a = 0; a < 3; ++a) {
        s[a][threadIdx.x] = fminf(s[a][threadIdx.x], s[a][threadIdx.x + st]);
        s[3 + a][threadIdx.x] = fmaxf(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + st]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 6) box[threadIdx.x] = s[threadIdx.x][0];
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

size_t sort_scene_temp_bytes(int n) {
  size_t bytes = 0, scan = 0;
  if (n <= 0) return 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const int*)nullptr, (int*)nullptr, n, 0, 32) != hipSuccess)
    return 0;
  // (the multi-workgroup kd order scans 3 n side flags per binary level)
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const int*)nullptr, (int*)nullptr, 3 * n) != hipSuccess) return 0;
  // (the kd order's three axis sorts as one segmented sort of 3 n keys)
  size_t seg = 0;
  if (hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, seg, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                  (const int*)nullptr, (int*)nullptr, 3 * n, 3, (const int*)nullptr,
                                                  (const int*)nullptr, 0, 32) != hipSuccess)
    return 0;
  return std::max(std::max(bytes, scan), seg);
}

int launch_build_bvh(DevScene& sc, const SortBufs& sb, hipStream_t st);

// The scene's broad-phase structure: the BVH (nothing else is sorted).
int launch_sort_scene(DevScene& sc, const SortBufs& sb, hipStream_t st) { return launch_build_bvh(sc, sb, st); }

// ------------------------------------------------------------------------------------------
// BVH of the quad traversals (art_trace.hip): all colliders (types mixed) in one spatial order of
// their bounds' centres (the kd order below; Morton above kKdMaxColliders), kBvhLeaf per leaf, an
// implicit complete 4-ary tree above. Node bounds are unions of CullRecs with the largest margin scale and factor,
// so a node's widened box contains every widened member box (broad phase).
// ------------------------------------------------------------------------------------------
// Levels of the heap-ordered tree over n colliders: the smallest L with 4^(L-1) leaves holding n.
static int bvh_layout(int n, int& leaf0, int& total) {
  if (n <= 0) return 0;
  const int nleaf = (n + kBvhLeaf - 1) / kBvhLeaf;
  int L = 1, w = 1;
  while (w < nleaf) { w *= 4; ++L; if (L > kBvhMaxLevels) return 0; }
  leaf0 = (w - 1) / 3;           // nodes above the leaf level: (4^(L-1) - 1) / 3
  total = leaf0 + w;
  return L;
}

size_t bvh_node_count(int n) {
  int leaf0 = 0, total = 0;
  return bvh_layout(n, leaf0, total) ? (size_t)total : 0;
}

size_t bvh_slot_count(int n) {
  int leaf0 = 0, total = 0;
  return bvh_layout(n, leaf0, total) ? (size_t)(total - leaf0) * kBvhLeaf : 0;
}

__global__ void morton_all_kernel(const CullRec* __restrict__ cull, int n, const float* __restrict__ box,
                                  uint32_t* __restrict__ keys, int* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float c[3];
  uint32_t code = 0;
  if (bound_centre(cull[i], c[0], c[1], c[2])) {
    uint32_t q[3];
    for (int a = 0; a < 3; ++a) {
      const float ext = box[3 + a] - box[a];
      const float t = ext > 0.0f ? (c[a] - box[a]) / ext : 0.0f;
      q[a] = (uint32_t)fminf(fmaxf(t * 1023.0f, 0.0f), 1023.0f);
    }
    code = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
  }
  keys[i] = code;
  vals[i] = i;
}

__device__ __forceinline__ void cull_union(CullRec& a, const CullRec& b) {
  a.lox = fminf(a.lox, b.lox); a.loy = fminf(a.loy, b.loy); a.loz = fminf(a.loz, b.loz);
  a.hix = fmaxf(a.hix, b.hix); a.hiy = fmaxf(a.hiy, b.hiy); a.hiz = fmaxf(a.hiz, b.hiz);
  a.fscale = fmaxf(a.fscale, b.fscale); a.factor = fmaxf(a.factor, b.factor);
}

__device__ __forceinline__ CullRec cull_empty() {
  CullRec r;
  r.lox = r.loy = r.loz = INFINITY; r.hix = r.hiy = r.hiz = -INFINITY; r.fscale = 0.0f; r.factor = 0.0f;
  return r;
}

// An empty node is stored as the box at +infinity (lo = hi = +inf, no margin): no finite ray enters
// it (each axis' slab bounds are the same +-inf, so either the exit is -inf or the entry is +inf,
// past every pruning bound and segment length), so the traversals need no emptiness test; a ray
// that visits every node (non-finite or zero direction) enters it harmlessly (its slots are empty).
__device__ __forceinline__ CullRec cull_stored(const CullRec& u) {
  if (!(u.lox > u.hix)) return u;
  CullRec r;
  r.lox = r.loy = r.loz = r.hix = r.hiy = r.hiz = INFINITY;
  r.fscale = 0.0f; r.factor = 0.0f;
  return r;
}
// union with a stored node (an empty one adds nothing)
__device__ __forceinline__ void cull_union_stored(CullRec& a, const CullRec& b) {
  if (!(b.lox == INFINITY && b.hix == INFINITY)) cull_union(a, b);
}

// Leaf j = sorted colliders [kBvhLeaf j, kBvhLeaf (j + 1)) (empty past the last); writes the
// leaf references.
// REFIT: the leaf order is kept (ref holds it) and only bounds and slots are recomputed.
// Leaf slot k holding collider g (global order; g < 0: an empty slot past the last collider).
__device__ __forceinline__ void bvh_write_slot(int k, int g, int ns, int na, int n, const SphereRec* __restrict__ sph,
                                               const AabbRec* __restrict__ aabb, const ObbRec* __restrict__ obb,
                                               float4* __restrict__ slots) {
  const int per = n - ns - na > 0 ? 4 : 2;  // float4s per slot (bvh_slot_bytes)
  float4* sl = slots + per * (size_t)k;
  float4 a = make_float4(0, 0, 0, 0), b = a, c = a, d = a;
  int code = -1;
  if (g >= 0) {
    if (g < ns) {
      const SphereRec r = sph[g];
      a = make_float4(r.cx, r.cy, r.cz, r.r2);
      b.z = __int_as_float(r.tid);
      code = g;
    } else if (g < ns + na) {
      const AabbRec r = aabb[g - ns];
      a = make_float4(r.mnx, r.mny, r.mnz, r.mxx);
      b = make_float4(r.mxy, r.mxz, __int_as_float(r.tid), 0.0f);
      code = (1 << 28) | (g - ns);
    } else {
      const ObbRec r = obb[g - ns - na];
      a = make_float4(r.cx, r.cy, r.cz, r.qx);
      b = make_float4(r.qy, r.qz, r.qw, 0.0f);
      c = make_float4(r.lmnx, r.lmny, r.lmnz, r.lmxx);
      d = make_float4(r.lmxy, r.lmxz, __int_as_float(r.tid), 0.0f);
      code = (2 << 28) | (g - ns - na);
    }
  }
  b.w = __int_as_float(code);
  sl[0] = a; sl[1] = b;
  if (per == 4) { sl[2] = c; sl[3] = d; }
}
// the global index of the collider in leaf position k (bvh_ref: type << 30 | in-type index)
__device__ __forceinline__ int bvh_ref_global(uint32_t r, int ns, int na) {
  const uint32_t t = r >> 30, i = r & 0x3fffffffu;
  return (int)i + (t == 0 ? 0 : (t == 1 ? ns : ns + na));
}

template <bool REFIT>
__device__ __forceinline__ void bvh_leaf_one(int j, const CullRec* __restrict__ cull, const int* __restrict__ perm, int ns,
                                             int na, int n, const SphereRec* __restrict__ sph, const AabbRec* __restrict__ aabb,
                                             const ObbRec* __restrict__ obb, CullRec* __restrict__ leaves,
                                             uint32_t* __restrict__ ref, float4* __restrict__ slots,
                                             uint32_t* __restrict__ pos = nullptr) {
  CullRec u = cull_empty();
  // slot (64 B; 32 B in scenes without OBBs, so a leaf is one 128-B line): a = first 16 B,
  // b = next 16 B (b.w = code), c, d = an OBB's local bounds
  //   sphere: a = (cx, cy, cz, r2), b.z = AudioTargetId
  //   AABB:   a = (mn.xyz, mx.x), b.xy = mx.yz, b.z = AudioTargetId
  //   OBB:    a = (c.xyz, q.x), b.xyz = q.yzw, c = (lmn.xyz, lmx.x), d.xy = lmx.yz, d.z = AudioTargetId
  for (int k = j * kBvhLeaf; k < (j + 1) * kBvhLeaf; ++k) {
    int g = -1;
    if (k < n) {
      g = REFIT ? bvh_ref_global(ref[k], ns, na) : perm[k];
      cull_union(u, cull[g]);
      if (!REFIT) {
        ref[k] = g < ns ? (uint32_t)g : (g < ns + na ? (1u << 30) | (uint32_t)(g - ns) : (2u << 30) | (uint32_t)(g - ns - na));
        if (pos) pos[g] = (uint32_t)k;
      }
    }
    bvh_write_slot(k, g, ns, na, n, sph, aabb, obb, slots);
  }
  leaves[j] = cull_stored(u);
}
template <bool REFIT>
__global__ void bvh_leaf_kernel(const CullRec* __restrict__ cull, const int* __restrict__ perm, int ns, int na, int n,
                                const SphereRec* __restrict__ sph, const AabbRec* __restrict__ aabb,
                                const ObbRec* __restrict__ obb, CullRec* __restrict__ leaves, int nleaf,
                                uint32_t* __restrict__ ref, float4* __restrict__ slots, uint32_t* __restrict__ pos) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nleaf) bvh_leaf_one<REFIT>(j, cull, perm, ns, na, n, sph, aabb, obb, leaves, ref, slots, pos);
}

// One inner level l (large trees: levels with more nodes than one workgroup handles quickly).
__global__ __launch_bounds__(256) void bvh_level_kernel(CullRec* __restrict__ nodes, int l) {
  const int first = ((1 << (2 * l)) - 1) / 3, cnt = 1 << (2 * l);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cnt) return;
  const int g = first + i;
  CullRec u = cull_empty();
  for (int k = 1; k <= 4; ++k) cull_union_stored(u, nodes[4 * g + k]);
  nodes[g] = cull_stored(u);
}

// Inner levels top_level .. 0, bottom-up, in one workgroup (they hold a third of the leaf count).
__global__ __launch_bounds__(1024) void bvh_upper_kernel(CullRec* __restrict__ nodes, int top_level) {
  for (int l = top_level; l >= 0; --l) {
    const int first = ((1 << (2 * l)) - 1) / 3, cnt = 1 << (2 * l);
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
      const int g = first + i;
      CullRec u = cull_empty();
      for (int k = 1; k <= 4; ++k) cull_union_stored(u, nodes[4 * g + k]);
      nodes[g] = cull_stored(u);
    }
    __syncthreads();
  }
}

// Inner levels L-2 .. 0: levels of more than 4096 nodes one launch each, the rest in one workgroup.
static void launch_bvh_upper(CullRec* nodes, int L, hipStream_t st) {
  int l = L - 2;
  for (; l >= 0 && (1 << (2 * l)) > 4096; --l)
    hipLaunchKernelGGL(bvh_level_kernel, dim3(((1 << (2 * l)) + 255) / 256), dim3(256), 0, st, nodes, l);
  if (l >= 0) hipLaunchKernelGGL(bvh_upper_kernel, dim3(1), dim3(1024), 0, st, nodes, l);
}

// ------------------------------------------------------------------------------------------
// kd leaf order (scenes of up to kKdMaxColliders colliders). The tree's layout is fixed: node
// blocks are aligned power-of-4 ranges of leaf positions, left-packed with the colliders. A
// complete tree over the Morton order lets a node straddle a jump of the Z curve, and its box then
// spans two distant cells; this order instead splits every node's block in two halves twice
// (binary level by binary level), with the first half (capacity seg / 2) taking the colliders of
// smallest centre on the split axis: every node is a compact, equal-count kd cell. The axis: on the
// upper levels (at most kKdSahSegs segments) the one of least surface-area cost of the two halves,
// below them the one on which the segment's centres extend furthest. Measured on config 2's scene (host
// simulation of the near-first traversal): 11.5 inner steps and 3.8 leaves per ray vs 28 and 9.3
// over the Morton order. Any order gives an exact BVH (node bounds are unions).
//
// Method: three index arrays, each sorted by one axis of the centres (hipCUB radix sort), stay
// sorted inside every segment through stable partitions: per binary level, each segment's axis is
// read off its own sorted array (last - first centre), the side of each collider is its rank on
// that axis, and every array is stably partitioned by side. One workgroup holds the three arrays
// in LDS (u16 ids, 96 KB at the 2^14-collider limit); each thread keeps its chunk's ids in
// registers (two u16 per VGPR) across the block scan, so the partition scatters in place. 5 barriers
// per level.
// ------------------------------------------------------------------------------------------
constexpr int kKdMaxColliders = 1 << 14;

struct KdBufs {
  float4* cen;          // [n] centre (non-finite components -> FLT_MAX)
  int* p;               // [3][n] index arrays sorted by x, y, z
  const CullRec* cull;  // [n] the colliders' bounds (surface-area split costs)
  // scenes above kKdMaxColliders (kd_big_*): the partitioned copies, side flags and their scan
  int* p2;              // [3][n]
  int* flag;            // [3][n] 1: left half of its segment
  int* scan;            // [3][n] exclusive scan of flag
  uint8_t* side;        // [n] by collider id
  uint32_t* keys;       // [3][n] radix keys of the centres per axis (kd_keys_kernel)
  uint32_t* keys_s;     // [3][n] their sorted copies
  int* vals;            // [3][n] collider ids (the sorts' values)
};
static size_t kd_al(size_t v) { return (v + 255) & ~(size_t)255; }
static KdBufs kd_bufs(void* base, int n) {
  char* b = static_cast<char*>(base);
  KdBufs k{};
  size_t o = 0;
  k.cen = reinterpret_cast<float4*>(b + o); o += kd_al(16 * (size_t)n);
  k.p = reinterpret_cast<int*>(b + o); o += kd_al(12 * (size_t)n);
  k.keys = reinterpret_cast<uint32_t*>(b + o); o += kd_al(12 * (size_t)n);
  k.keys_s = reinterpret_cast<uint32_t*>(b + o); o += kd_al(12 * (size_t)n);
  k.vals = reinterpret_cast<int*>(b + o); o += kd_al(12 * (size_t)n);
  if (n > kKdMaxColliders) {
    k.p2 = reinterpret_cast<int*>(b + o); o += kd_al(12 * (size_t)n);
    k.flag = reinterpret_cast<int*>(b + o); o += kd_al(12 * (size_t)n);
    k.scan = reinterpret_cast<int*>(b + o); o += kd_al(12 * (size_t)n);
    k.side = reinterpret_cast<uint8_t*>(b + o);
  }
  k.cull = nullptr;
  return k;
}
size_t kd_scratch_bytes(int n) {
  if (n <= 0) return 0;
  const size_t base = kd_al(16 * (size_t)n) + 4 * kd_al(12 * (size_t)n);
  return n <= kKdMaxColliders ? base : base + 3 * kd_al(12 * (size_t)n) + kd_al((size_t)n);
}

// Centres (non-finite components -> FLT_MAX, sorting last) and their radix-sortable keys on the
// three axes, with the identity values of the sorts (one launch; round 4: one centre launch and one
// key launch per axis)
__global__ void kd_keys_kernel(const CullRec* __restrict__ cull, int n, KdBufs k, int* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const CullRec c = cull[i];
  float v[3] = {0.5f * (c.lox + c.hix), 0.5f * (c.loy + c.hiy), 0.5f * (c.loz + c.hiz)};
  for (int a = 0; a < 3; ++a) {
    v[a] = isfinite(v[a]) ? v[a] : FLT_MAX;
    const uint32_t u = __float_as_uint(v[a]);
    k.keys[(size_t)a * n + i] = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  }
  k.cen[i] = make_float4(v[0], v[1], v[2], 0.0f);
  vals[i] = i;
  for (int a = 0; a < 3; ++a) k.vals[(size_t)a * n + i] = i;
}

// The three axis orders of the kd build for up to 1024 * ITEMS colliders: one workgroup per axis
// sorts its (key, id) pairs in LDS (rocprim block radix sort, stable: ties keep id order, as the
// device-wide radix sorts it replaces for these sizes). One launch instead of three device-wide
// sorts with their helper launches (round 4: about 54 us of a config-2 rebuild frame).
// The centre of collider i on axis a (non-finite -> FLT_MAX, sorting last) and its radix-sortable key.
__device__ __forceinline__ float kd_centre(const CullRec& c, int a) {
  const float v = a == 0 ? 0.5f * (c.lox + c.hix) : (a == 1 ? 0.5f * (c.loy + c.hiy) : 0.5f * (c.loz + c.hiz));
  return isfinite(v) ? v : FLT_MAX;
}
__device__ __forceinline__ uint32_t kd_key(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// (the centres and keys are computed here from the bounds, workgroup 0 storing the centres: no
// separate kd_keys_kernel launch for these sizes)
template <int ITEMS>
__global__ __launch_bounds__(1024) void kd_axis_sort_kernel(KdBufs k, int n) {
  using Sort = hipcub::BlockRadixSort<uint32_t, 1024, ITEMS, int>;
  __shared__ typename Sort::TempStorage tmp;
  const int a = blockIdx.x;
  uint32_t key[ITEMS];
  int val[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {  // blocked arrangement in id order (padding sorts last: keys of
    const int i = (int)threadIdx.x * ITEMS + j;  // finite centres stay below 0xff800000)
    key[j] = 0xffffffffu;
    if (i < n) {
      const CullRec c = k.cull[i];
      key[j] = kd_key(kd_centre(c, a));
      if (a == 0) k.cen[i] = make_float4(kd_centre(c, 0), kd_centre(c, 1), kd_centre(c, 2), 0.0f);
    }
    val[j] = i;
  }
  Sort(tmp).SortBlockedToStriped(key, val);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int i = j * 1024 + (int)threadIdx.x;
    if (i < n) k.p[(size_t)a * n + i] = val[j];
  }
}

__device__ __forceinline__ float kd_comp(const float4& c, int a) { return a == 0 ? c.x : (a == 1 ? c.y : c.z); }

// Block-wide exclusive scan of three counters per thread (NT threads, NT / 64 waves).
template <int NT>
__device__ __forceinline__ void kd_block_scan3(int v[3], int (*s_wave)[16]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc[3];
  for (int x = 0; x < 3; ++x) {
    int t = v[x];
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(t, d);
      if (lane >= d) t += o;
    }
    inc[x] = t;
    if (lane == 63) s_wave[x][w] = t;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int run = 0;
    for (int k = 0; k < NT / 64; ++k) { const int t = s_wave[threadIdx.x][k]; s_wave[threadIdx.x][k] = run; run += t; }
  }
  __syncthreads();
  for (int x = 0; x < 3; ++x) v[x] = s_wave[x][w] + inc[x] - v[x];
  __syncthreads();
}

// Surface-area split costs on the upper binary levels (at most kKdSahSegs segments): for each
// segment and axis, the bounds of the two halves the split on that axis would make, accumulated in
// LDS as order-preserving integers (atomic min / max).
#ifndef ART_KD_SAH_SEGS
#define ART_KD_SAH_SEGS 64
#endif
constexpr int kKdSahSegs = ART_KD_SAH_SEGS;
__device__ __forceinline__ int kd_ord(float f) {  // monotone float -> int (for atomicMin / atomicMax)
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float kd_unord(int v) { return __int_as_float(v >= 0 ? v : v ^ 0x7fffffff); }
// Min / max over aligned groups of gsz lanes (a power of two <= 64), the result in every lane of the
// group: DPP within rows of 16 lanes (xor 1, xor 2, half-row mirror, row mirror), shuffles across
// rows. (Round 4: shuffles at every step left the surface-area pass at ~12 us per level.)
template <int CTRL>
__device__ __forceinline__ float kd_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <bool MIN>
__device__ __forceinline__ float kd_grp(float v, int gsz) {
  auto op = [](float a, float b) { return MIN ? fminf(a, b) : fmaxf(a, b); };
  if (gsz >= 2) v = op(v, kd_dpp<0xB1>(v));   // quad_perm [1, 0, 3, 2]
  if (gsz >= 4) v = op(v, kd_dpp<0x4E>(v));   // quad_perm [2, 3, 0, 1]
  if (gsz >= 8) v = op(v, kd_dpp<0x141>(v));  // row_half_mirror
  if (gsz >= 16) v = op(v, kd_dpp<0x140>(v)); // row_mirror
  if (gsz >= 32) v = op(v, __shfl_xor(v, 16, 64));
  if (gsz >= 64) v = op(v, __shfl_xor(v, 32, 64));
  return v;
}
__device__ __forceinline__ float kd_area(float ex, float ey, float ez) {
  ex = fmaxf(ex, 0.0f); ey = fmaxf(ey, 0.0f); ez = fmaxf(ez, 0.0f);
  return ex * ey + ey * ez + ez * ex;
}

// CAP: the largest scene of the instantiation. Up to kKdLdsBounds colliders the bounds live in LDS
// too (6 floats each), so the surface-area pass and the axis choice read no global memory.
// One workgroup of NT threads splits the window of 2^lg_top positions starting at blockIdx.x << lg_top
// through the binary levels lg_top .. lg_stop + 1 (round 4: the whole order in one 1024-thread
// workgroup spent ~13 us per level on its barriers and block scans; the levels below 512 positions
// now run as one 256-thread workgroup per 512-position window, side by side). `last`: the window's
// first array is the leaf order (perm), otherwise the three arrays go back to k.p for the next pass.
constexpr int kKdLdsBounds = 4096;
constexpr int kKdWindowLg = 9;  // windows of the second pass: 512 positions
// BM: where the surface-area pass and the axis choice read the bounds — 0 global memory, 1 LDS by
// collider id (the whole scene, up to kKdLdsBounds colliders), 2 LDS by window position (the
// window's colliders, through an id -> position map).
template <int CAP, int NT, int MAXCHUNK, int BM>
__global__ __launch_bounds__(NT) void kd_split_kernel(KdBufs k, int n, int lg_top, int lg_stop, int last,
                                                      int* __restrict__ perm) {
  constexpr bool LB = BM != 0;
  __shared__ uint16_t s_p[3][NT * MAXCHUNK];  // the window's three index arrays (relative positions)
  __shared__ uint8_t s_side[CAP];             // 1: left half of its segment (by collider id)
  __shared__ int8_t s_axis[NT * MAXCHUNK / 8];   // per segment of the window: split axis, -1 = fits its left half
  __shared__ uint16_t s_segpre[3][NT * MAXCHUNK / 8];  // left-flag prefix at each segment's start
  __shared__ int s_wave[3][16];
  __shared__ int s_box[2][3][kKdSahSegs][6];  // [half][axis][segment]: lo.xyz, hi.xyz (kd_ord)
  constexpr int kBb = BM == 1 ? CAP : (BM == 2 ? NT * MAXCHUNK : 1);
  __shared__ float s_bb[LB ? 6 : 1][kBb];               // lo.xyz, hi.xyz by collider id (BM 1) or window position (BM 2)
  __shared__ uint16_t s_slot[BM == 2 ? CAP : 1];        // BM 2: a collider's position in the window (array 0)
  const int tid = threadIdx.x;
  constexpr int kChunk = MAXCHUNK;  // positions per thread, at most
  const int base = (int)blockIdx.x << lg_top;  // (the window's segments are aligned: base is a multiple of 2^lg)
  const int nw = min(1 << lg_top, n - base);
  if (nw <= 0) return;
  const int chunk = (nw + NT - 1) / NT;
  const int i0 = base + min(nw, tid * chunk), i1 = base + min(nw, tid * chunk + chunk);
  // the window's arrays (and bounds) into LDS: every load of a work-item issued before its first
  // store, so the prologue waits for one round of memory latency per dependent step, not per
  // element (round 4: the per-element loop serialized ~16 global round trips in the top pass)
  {
    int pv[3][kChunk];
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int r = tid + j * NT;
        pv[x][j] = r < nw ? k.p[(size_t)x * n + base + r] : 0;
      }
    if (BM == 2) {  // bounds by window position (array 0's order)
      CullRec cv[kChunk];
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int r = tid + j * NT;
        if (r < nw) cv[j] = k.cull[pv[0][j]];
      }
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int r = tid + j * NT;
        if (r < nw) {
          s_slot[pv[0][j]] = (uint16_t)r;
          s_bb[0][r] = cv[j].lox; s_bb[1][r] = cv[j].loy; s_bb[2][r] = cv[j].loz;
          s_bb[3][r] = cv[j].hix; s_bb[4][r] = cv[j].hiy; s_bb[5][r] = cv[j].hiz;
        }
      }
    }
    if (BM == 1) {  // bounds by collider id (the whole scene: n <= CAP = NT * kChunk)
      CullRec cv[kChunk];
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int i = tid + j * NT;
        if (i < n) cv[j] = k.cull[i];
      }
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int i = tid + j * NT;
        if (i < n) {
          s_bb[0][i] = cv[j].lox; s_bb[1][i] = cv[j].loy; s_bb[2][i] = cv[j].loz;
          s_bb[3][i] = cv[j].hix; s_bb[4][i] = cv[j].hiy; s_bb[5][i] = cv[j].hiz;
        }
      }
    }
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int r = tid + j * NT;
        if (r < nw) s_p[x][r] = (uint16_t)pv[x][j];
      }
  }
#ifdef ART_KD_PROF  // diagnostics: per-phase wall clock of workgroup 0 (printf at the end)
  unsigned long long kp_t[64];
  int kp_n = 0;
  auto kp = [&]() { if (kp_n < 64) kp_t[kp_n++] = wall_clock64(); };
  kp();
#define KP() kp()
#else
#define KP() (void)0
#endif
  auto bb = [&](int q, int v) -> float { return s_bb[q][BM == 2 ? (int)s_slot[v] : v]; };
  // centre component a of collider v (kd_keys_kernel's value: non-finite -> FLT_MAX)
  auto cen = [&](int v, int a) -> float {
    if (!LB) return kd_comp(k.cen[v], a);
    const float c = 0.5f * (bb(a, v) + bb(3 + a, v));
    return isfinite(c) ? c : FLT_MAX;
  };
  __syncthreads();
  KP();
  for (int lg = lg_top; lg > lg_stop; --lg) {  // segments of seg = 2^lg positions
    const int seg = 1 << lg, half = seg >> 1, nseg = (nw + seg - 1) >> lg;  // (this window's segments)
    const bool sah = ((n + seg - 1) >> lg) <= kKdSahSegs;  // (the policy counts the whole order's segments)
    if (sah) {  // bounds of both halves of every segment for a split on each axis
      for (int e = tid; e < 2 * 3 * kKdSahSegs * 6; e += NT)
        (&s_box[0][0][0][0])[e] = (e % 6) < 3 ? kd_ord(INFINITY) : kd_ord(-INFINITY);
      __syncthreads();
      // lanes whose positions lie in one half-segment reduce their bounds across the group first
      // (xor shuffles), so one lane per group does the LDS atomics: whole waves on the upper levels,
      // aligned groups of half / chunk lanes below (round 4: the per-lane atomics on a few LDS words
      // serialized the lower surface-area levels); chunks that are not a power of two keep per-lane
      // atomics
      const int per = (chunk & (chunk - 1)) == 0 ? half / chunk : 0;
      const int gsz = per >= 64 ? 64 : (per >= 2 ? per : 1);  // lanes per half-segment group
      for (int x = 0; x < 3; ++x) {
        float b[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
        int key = -1;  // (segment << 1 | half) of the run accumulated in b
        auto flush = [&]() {
          if (key < 0) return;
          int* o = s_box[key & 1][x][key >> 1];
          for (int q = 0; q < 3; ++q) { atomicMin(o + q, kd_ord(b[q])); atomicMax(o + 3 + q, kd_ord(b[3 + q])); }
          for (int q = 0; q < 3; ++q) { b[q] = INFINITY; b[3 + q] = -INFINITY; }
        };
        for (int i = i0; i < i1; ++i) {
          const int kk = (((i - base) >> lg) << 1) | ((i & (seg - 1)) >= half ? 1 : 0);
          if (kk != key && gsz == 1) { flush(); }
          key = kk;
          const int v = s_p[x][i - base];
          if (LB) {
            for (int q = 0; q < 3; ++q) { b[q] = fminf(b[q], bb(q, v)); b[3 + q] = fmaxf(b[3 + q], bb(3 + q, v)); }
          } else {
            const CullRec c = k.cull[v];
            b[0] = fminf(b[0], c.lox); b[1] = fminf(b[1], c.loy); b[2] = fminf(b[2], c.loz);
            b[3] = fmaxf(b[3], c.hix); b[4] = fmaxf(b[4], c.hiy); b[5] = fmaxf(b[5], c.hiz);
          }
        }
        if (gsz > 1) {  // (block-uniform) min / max over each group, then its first lane publishes
          for (int q = 0; q < 6; ++q) b[q] = q < 3 ? kd_grp<true>(b[q], gsz) : kd_grp<false>(b[q], gsz);
          // the group's key is its first lane's (-1 when that chunk is empty: then every later one is)
          key = __shfl(key, (tid & 63) & ~(gsz - 1), 64);
          if ((tid & (gsz - 1)) == 0) flush();
        } else {
          flush();
        }
      }
      __syncthreads();
    }
    KP();
    for (int s = tid; s < nseg; s += NT) {  // each segment's axis: the cheapest split (SAH) or the widest spread of centres
      const int a0 = s << lg, cnt = min(seg, nw - a0);  // (window-relative)
      int ax = -1;
      if (cnt > half && sah) {
        float best = INFINITY;
        for (int x = 0; x < 3; ++x) {
          const int* l = s_box[0][x][s];
          const int* r = s_box[1][x][s];
          const float cost =
              kd_area(kd_unord(l[3]) - kd_unord(l[0]), kd_unord(l[4]) - kd_unord(l[1]), kd_unord(l[5]) - kd_unord(l[2])) * (float)half +
              kd_area(kd_unord(r[3]) - kd_unord(r[0]), kd_unord(r[4]) - kd_unord(r[1]), kd_unord(r[5]) - kd_unord(r[2])) *
                  (float)(cnt - half);
          if (cost < best) { best = cost; ax = x; }  // (a non-finite cost never wins)
        }
      }
      if (cnt > half && ax < 0) {
        float best = -1.0f;
        for (int x = 0; x < 3; ++x) {
          const float e = cen(s_p[x][a0 + cnt - 1], x) - cen(s_p[x][a0], x);
          if (ax < 0 || e > best) { best = e; ax = x; }
        }
      }
      s_axis[s] = (int8_t)ax;
    }
    __syncthreads();
    KP();
    for (int r = tid; r < nw; r += NT) {  // side of each collider: its rank on its segment's axis
      const int ax = s_axis[r >> lg];
      if (ax >= 0) s_side[s_p[ax][r]] = (r & (seg - 1)) < half ? 1 : 0;
    }
    __syncthreads();
    uint32_t pk[3][kChunk / 2];  // the chunk's ids, two u16 per register
    for (int x = 0; x < 3; ++x)
      for (int j = 0; j < kChunk / 2; ++j) pk[x][j] = 0u;
    uint32_t fl[3] = {0u, 0u, 0u};
    int c[3] = {0, 0, 0};
#pragma unroll
    for (int j = 0; j < kChunk; ++j) {
      const int i = i0 + j;
      if (i < i1) {
        const int ax = s_axis[(i - base) >> lg];
        for (int x = 0; x < 3; ++x) {
          const uint32_t v = s_p[x][i - base];
          pk[x][j >> 1] |= v << (16 * (j & 1));
          const uint32_t f = ax < 0 ? 1u : s_side[v];
          fl[x] |= f << j;
          c[x] += (int)f;
        }
      }
    }
    KP();
    kd_block_scan3<NT>(c, s_wave);  // (its barriers also order every read of s_p above before the scatter)
    {
      int run[3] = {c[0], c[1], c[2]};
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int i = i0 + j;
        if (i < i1) {
          const bool start = (i & (seg - 1)) == 0;
          for (int x = 0; x < 3; ++x) {
            if (start) s_segpre[x][(i - base) >> lg] = (uint16_t)run[x];
            run[x] += (int)((fl[x] >> j) & 1u);
          }
        }
      }
    }
    __syncthreads();
    {  // stable partition of every array: left half first
      int run[3] = {c[0], c[1], c[2]};
#pragma unroll
      for (int j = 0; j < kChunk; ++j) {
        const int i = i0 + j;
        if (i < i1) {
          const int r = i - base, s = r >> lg, a0 = s << lg;  // (window-relative)
          for (int x = 0; x < 3; ++x) {
            const bool left = ((fl[x] >> j) & 1u) != 0u;
            const int lr = run[x] - (int)s_segpre[x][s];
            s_p[x][left ? a0 + lr : a0 + half + (r - a0 - lr)] = (uint16_t)(pk[x][j >> 1] >> (16 * (j & 1)));
            run[x] += left ? 1 : 0;
          }
        }
      }
    }
    __syncthreads();
    KP();
  }
#ifdef ART_KD_PROF
  if (blockIdx.x == 0 && tid == 0) {
    printf("[kd] NT %d BM %d nw %d lg %d..%d load %llu\n", NT, BM, nw, lg_top, lg_stop, (kp_t[1] - kp_t[0]) * 10ull);
    for (int q = 1; q + 4 <= kp_n - 1; q += 4)
      printf("[kd]   level: sah %llu axis %llu side %llu scan+part %llu ns\n", (kp_t[q + 1] - kp_t[q]) * 10ull,
             (kp_t[q + 2] - kp_t[q + 1]) * 10ull, (kp_t[q + 3] - kp_t[q + 2]) * 10ull, (kp_t[q + 4] - kp_t[q + 3]) * 10ull);
  }
#endif
#undef KP
  if (last) {
    for (int r = tid; r < nw; r += NT) perm[base + r] = s_p[0][r];
  } else {
    for (int x = 0; x < 3; ++x)
      for (int r = tid; r < nw; r += NT) k.p[(size_t)x * n + base + r] = s_p[x][r];
  }
}

// The binary levels of segments of at most 64 positions (lg_top <= 6), one wave per aligned block of
// 64 positions and no workgroup barriers (round 4: below 512 positions the window pass spent its
// time in block scans and barriers). The block's 64 colliders stay the same through these levels,
// so the three arrays hold block-local slots (the collider's position in array 0 on entry) and the
// bounds sit in LDS by slot. Per level: the split axis (the same surface-area cost or spread of
// centres as kd_split_kernel, from half-segment reductions over xor shuffles), the side of each
// slot by its rank on that axis, and a stable partition of every array from ballot ranks, moved
// through a per-wave LDS row. Writes the leaf order (perm).
constexpr int kKdWaveLg = 6;
static bool kd_wave_enabled() {  // ART_KD_WAVE=0 (read per build): the block passes run every level (A/B, tests)
  const char* e = getenv("ART_KD_WAVE");
  return !(e && e[0] == '0');
}
template <int CAP>
__global__ __launch_bounds__(256) void kd_wave_kernel(KdBufs k, int n, int lg_top, int* __restrict__ perm) {
  __shared__ uint16_t s_slot[CAP];         // collider id -> slot (the block's array-0 position)
  __shared__ int s_id[4][64];              // slot -> collider id
  __shared__ float s_bb[4][6][64];         // slot -> lo.xyz, hi.xyz
  __shared__ uint8_t s_side[4][64];        // slot -> 1: left half of its segment
  __shared__ uint8_t s_row[4][3][64];      // the partition's destination rows
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int base = (int)blockIdx.x * 256 + wv * 64;
  const int cnt = min(64, n - base);
  if (cnt <= 0) return;  // (no workgroup barriers below: a wave may leave)
  const bool live = lane < cnt;
  int id[3] = {0, 0, 0};
  for (int x = 0; x < 3; ++x) id[x] = live ? k.p[(size_t)x * n + base + lane] : 0;
  CullRec c;
  if (live) c = k.cull[id[0]];
  if (live) {
    s_slot[id[0]] = (uint16_t)lane;
    s_id[wv][lane] = id[0];
    s_bb[wv][0][lane] = c.lox; s_bb[wv][1][lane] = c.loy; s_bb[wv][2][lane] = c.loz;
    s_bb[wv][3][lane] = c.hix; s_bb[wv][4][lane] = c.hiy; s_bb[wv][5][lane] = c.hiz;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
  int v[3];  // this lane's slot in each array
  v[0] = lane;
  v[1] = live ? (int)s_slot[id[1]] : 0;
  v[2] = live ? (int)s_slot[id[2]] : 0;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int lg = lg_top; lg > 2; --lg) {
    const int seg = 1 << lg, half = seg >> 1;
    const int s_lo = lane & ~(seg - 1), cnt_s = min(seg, max(0, cnt - s_lo));
    const bool sah = ((n + seg - 1) >> lg) <= kKdSahSegs;  // (the policy counts the whole order's segments)
    const bool left_half = (lane - s_lo) < half;
    int ax = -1;
    if (sah) {  // (wave-uniform) bounds of both halves of the segment for a split on each axis
      float best = INFINITY;
      for (int x = 0; x < 3; ++x) {
        float b[6];
        for (int q = 0; q < 3; ++q) {
          b[q] = live ? s_bb[wv][q][v[x]] : INFINITY;
          b[3 + q] = live ? s_bb[wv][3 + q][v[x]] : -INFINITY;
        }
        for (int q = 0; q < 6; ++q) b[q] = q < 3 ? kd_grp<true>(b[q], half) : kd_grp<false>(b[q], half);  // this half's bounds
        float ob[6];  // the other half's
        for (int q = 0; q < 6; ++q) ob[q] = __shfl_xor(b[q], half, 64);
        const float* l = left_half ? b : ob;
        const float* r = left_half ? ob : b;
        const float cost = kd_area(l[3] - l[0], l[4] - l[1], l[5] - l[2]) * (float)half +
                           kd_area(r[3] - r[0], r[4] - r[1], r[5] - r[2]) * (float)(cnt_s - half);
        if (cnt_s > half && cost < best) { best = cost; ax = x; }  // (a non-finite cost never wins)
      }
    }
    if (cnt_s > half && ax < 0) {  // the widest spread of centres (kd_keys_kernel's values)
      float best = -1.0f;
      for (int x = 0; x < 3; ++x) {
        const int vf = __shfl(v[x], s_lo, 64), vl = __shfl(v[x], s_lo + max(cnt_s, 1) - 1, 64);
        const float cf = 0.5f * (s_bb[wv][x][vf] + s_bb[wv][3 + x][vf]), cl = 0.5f * (s_bb[wv][x][vl] + s_bb[wv][3 + x][vl]);
        const float e = (isfinite(cl) ? cl : FLT_MAX) - (isfinite(cf) ? cf : FLT_MAX);
        if (ax < 0 || e > best) { best = e; ax = x; }
      }
    }  // (segment-uniform branch: the lanes read are live lanes of the same segment)
    if (ax >= 0 && live) {
      const int va = ax == 0 ? v[0] : (ax == 1 ? v[1] : v[2]);
      s_side[wv][va] = left_half ? 1 : 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    const uint64_t segmask = (seg == 64 ? ~0ull : (((1ull << seg) - 1ull) << s_lo));
    for (int x = 0; x < 3; ++x) {
      const bool left = ax < 0 ? true : s_side[wv][v[x]] != 0;
      const uint64_t m = __ballot(live && left);
      const int lr = __popcll(m & segmask & lt);
      const int dst = left ? s_lo + lr : s_lo + half + (lane - s_lo - lr);
      if (live) s_row[wv][x][dst] = (uint8_t)v[x];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    for (int x = 0; x < 3; ++x) v[x] = live ? (int)s_row[wv][x][lane] : 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
  if (live) perm[base + lane] = s_id[wv][v[0]];
}

// ------------------------------------------------------------------------------------------
// kd leaf order of larger scenes (above kKdMaxColliders, up to 2^24 colliders): the same binary
// splits over global arrays, one launch sequence per binary level: side flags by collider id,
// per-array flags, one exclusive scan of the 3 n flags, a stable scatter into the other copy. Every
// segment splits on the axis its centres extend furthest on (no surface-area costs).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int kd_big_axis(const KdBufs& k, int n, int s, int lg) {
  const int seg = 1 << lg, half = seg >> 1, a0 = s << lg, cnt = min(seg, n - a0);
  if (cnt <= half) return -1;  // fits its left half: stays
  int ax = -1;
  float best = -1.0f;
  for (int x = 0; x < 3; ++x) {
    const int* px = k.p + (size_t)x * n;
    const float e = kd_comp(k.cen[px[a0 + cnt - 1]], x) - kd_comp(k.cen[px[a0]], x);
    if (ax < 0 || e > best) { best = e; ax = x; }
  }
  return ax;
}
__global__ void kd_big_side_kernel(KdBufs k, int n, int lg) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int ax = kd_big_axis(k, n, i >> lg, lg);
  if (ax >= 0) k.side[k.p[(size_t)ax * n + i]] = (i & ((1 << lg) - 1)) < (1 << (lg - 1)) ? 1 : 0;
}
__global__ void kd_big_flag_kernel(KdBufs k, int n, int lg) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 3ll * n) return;
  const int i = (int)(e % n);
  const int ax = kd_big_axis(k, n, i >> lg, lg);
  k.flag[e] = ax < 0 ? 1 : (int)k.side[k.p[e]];
}
__global__ void kd_big_scatter_kernel(KdBufs k, int n, int lg) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 3ll * n) return;
  const int x = (int)(e / n), i = (int)(e - (long long)x * n);
  const int a0 = (i >> lg) << lg, half = 1 << (lg - 1);
  const size_t row = (size_t)x * n;
  const int lr = k.scan[e] - k.scan[row + a0];  // left-flagged entries before i in its segment
  const int dst = k.flag[e] ? a0 + lr : a0 + half + (i - a0 - lr);
  k.p2[row + dst] = k.p[e];
}
static int launch_kd_big(KdBufs k, int n, int cap, const SortBufs& sb, hipStream_t st) {
  const unsigned b1 = (unsigned)((n + 255) / 256), b3 = (unsigned)((3ll * n + 255) / 256);
  for (int lg = 31 - __builtin_clz(cap); lg > 2; --lg) {
    hipLaunchKernelGGL(kd_big_side_kernel, dim3(b1), dim3(256), 0, st, k, n, lg);
    hipLaunchKernelGGL(kd_big_flag_kernel, dim3(b3), dim3(256), 0, st, k, n, lg);
    size_t bytes = sb.temp_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(sb.temp, bytes, k.flag, k.scan, 3 * n, st) != hipSuccess) return -1;
    hipLaunchKernelGGL(kd_big_scatter_kernel, dim3(b3), dim3(256), 0, st, k, n, lg);
    std::swap(k.p, k.p2);
  }
  return hipMemcpyAsync(sb.perm, k.p, (size_t)n * sizeof(int), hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : -1;
}

int launch_build_bvh(DevScene& sc, const SortBufs& sb, hipStream_t st) {
  const int n = sc.ns + sc.na + sc.no;
  int leaf0 = 0, total = 0;
  const int L = bvh_layout(n, leaf0, total);
  sc.bvh = nullptr; sc.bvh_ref = nullptr; sc.bvh_leaf = nullptr; sc.bvh_levels = 0; sc.bvh_leaf0 = 0;
  if (L == 0 || !sb.bvh || !sb.bvh_ref || !sb.bvh_leaf) return 0;
  const int nleaf = total - leaf0;
  if (sb.kd) {  // kd leaf order
    KdBufs k = kd_bufs(sb.kd, n);
    k.cull = sc.cull;
    if (n > kKdMaxColliders) hipLaunchKernelGGL(kd_keys_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc.cull, n, k, sb.vals);
    if (n <= 4096) {  // the three axis orders (stable: ties keep id order), one workgroup per axis
      hipLaunchKernelGGL(kd_axis_sort_kernel<4>, dim3(3), dim3(1024), 0, st, k, n);
    } else if (n <= kKdMaxColliders) {
      hipLaunchKernelGGL(kd_axis_sort_kernel<kKdMaxColliders / 1024>, dim3(3), dim3(1024), 0, st, k, n);
    } else {
      for (int a = 0; a < 3; ++a) {
        size_t bytes = sb.temp_bytes;
        if (hipcub::DeviceRadixSort::SortPairs(sb.temp, bytes, k.keys + (size_t)a * n, sb.keys_s, sb.vals, k.p + (size_t)a * n,
                                               n, 0, 32, st) != hipSuccess)
          return -1;
      }
    }
    if (n <= kKdMaxColliders && kd_wave_enabled()) {
      // one 1024-thread workgroup down to 512-position segments, then one 256-thread workgroup per
      // 512-position window down to 64-position segments, then one wave per 64-position block
      const int lg_top = 31 - __builtin_clz((unsigned)(nleaf * kBvhLeaf));  // (a power of 4)
      const int lg_wave = lg_top < kKdWaveLg ? lg_top : kKdWaveLg;
      const int lg_mid = lg_top > kKdWindowLg ? kKdWindowLg : lg_wave;
      if (lg_top > lg_mid) {
        if (n <= kKdLdsBounds)
          hipLaunchKernelGGL((kd_split_kernel<kKdLdsBounds, 1024, kKdLdsBounds / 1024, 1>), dim3(1), dim3(1024), 0, st, k, n,
                             lg_top, lg_mid, 0, sb.perm);
        else
          hipLaunchKernelGGL((kd_split_kernel<kKdMaxColliders, 1024, kKdMaxColliders / 1024, 0>), dim3(1), dim3(1024), 0, st,
                             k, n, lg_top, lg_mid, 0, sb.perm);
      }
      if (lg_mid > lg_wave) {
        const unsigned windows = (unsigned)((n + (1 << kKdWindowLg) - 1) >> kKdWindowLg);
        if (n <= kKdLdsBounds)
          hipLaunchKernelGGL((kd_split_kernel<kKdLdsBounds, 256, (1 << kKdWindowLg) / 256, 2>), dim3(windows), dim3(256), 0,
                             st, k, n, kKdWindowLg, lg_wave, 0, sb.perm);
        else
          hipLaunchKernelGGL((kd_split_kernel<kKdMaxColliders, 256, (1 << kKdWindowLg) / 256, 2>), dim3(windows), dim3(256),
                             0, st, k, n, kKdWindowLg, lg_wave, 0, sb.perm);
      }
      hipLaunchKernelGGL((kd_wave_kernel<kKdMaxColliders>), dim3((n + 255) / 256), dim3(256), 0, st, k, n, lg_wave, sb.perm);
    } else if (n <= kKdMaxColliders) {  // (ART_KD_WAVE=0: the block passes down to 4-position segments)
      const int lg_top = 31 - __builtin_clz((unsigned)(nleaf * kBvhLeaf));  // (a power of 4)
      const int lg_mid = lg_top > kKdWindowLg ? kKdWindowLg : 2;
      if (n <= kKdLdsBounds)
        hipLaunchKernelGGL((kd_split_kernel<kKdLdsBounds, 1024, kKdLdsBounds / 1024, 1>), dim3(1), dim3(1024), 0, st, k, n,
                           lg_top, lg_mid, lg_mid == 2 ? 1 : 0, sb.perm);
      else
        hipLaunchKernelGGL((kd_split_kernel<kKdMaxColliders, 1024, kKdMaxColliders / 1024, 0>), dim3(1), dim3(1024), 0, st,
                           k, n, lg_top, lg_mid, lg_mid == 2 ? 1 : 0, sb.perm);
      if (lg_mid > 2) {
        const unsigned windows = (unsigned)((n + (1 << kKdWindowLg) - 1) >> kKdWindowLg);
        if (n <= kKdLdsBounds)
          hipLaunchKernelGGL((kd_split_kernel<kKdLdsBounds, 256, (1 << kKdWindowLg) / 256, 2>), dim3(windows), dim3(256), 0,
                             st, k, n, kKdWindowLg, 2, 1, sb.perm);
        else
          hipLaunchKernelGGL((kd_split_kernel<kKdMaxColliders, 256, (1 << kKdWindowLg) / 256, 2>), dim3(windows), dim3(256),
                             0, st, k, n, kKdWindowLg, 2, 1, sb.perm);
      }
    }
    else if (launch_kd_big(k, n, nleaf * kBvhLeaf, sb, st) != 0) return -1;
  } else {  // Morton order of the centres (larger scenes)
    hipLaunchKernelGGL(scene_box_kernel, dim3(1), dim3(1024), 0, st, sc.cull, n, sb.box);
    hipLaunchKernelGGL(morton_all_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc.cull, n, sb.box, sb.keys, sb.vals);
    size_t bytes = sb.temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(sb.temp, bytes, sb.keys, sb.keys_s, sb.vals, sb.perm, n, 0, 30, st) != hipSuccess)
      return -1;
  }
  hipLaunchKernelGGL(bvh_leaf_kernel<false>, dim3((nleaf + 255) / 256), dim3(256), 0, st, sc.cull, sb.perm, sc.ns, sc.na, n,
                     sc.sph, sc.aabb, sc.obb, sb.bvh + leaf0, nleaf, sb.bvh_ref, sb.bvh_leaf, sb.bvh_pos);
  launch_bvh_upper(sb.bvh, L, st);
  sc.bvh = sb.bvh; sc.bvh_ref = sb.bvh_ref; sc.bvh_leaf = sb.bvh_leaf; sc.bvh_levels = L; sc.bvh_leaf0 = leaf0;
  return 0;
}

// A resident-store sync of a scene of up to kSyncRefitMax colliders (art_colliders_sync, round 6)
// in one workgroup and one launch, touching only what moved: the dirty records written and decoded
// (scatter_prep_kernel's work, read straight from the pinned host image: no copy), their leaf
// slots rewritten at their leaf positions (bvh_pos), the boxes of their leaves recomputed, then
// every ancestor of a changed node, level by level up to the root (a bitmap of changed nodes in
// LDS). The result equals a full refit (bvh_leaf_kernel<true> + the inner levels): untouched nodes
// are unions of unchanged children. Config 2's dynamic step: one ~6-us launch in place of a copy,
// three kernels and their gaps.
constexpr int kSyncRefitNodes = (int)(kSyncRefitMax / kBvhLeaf) * 4 / 3 + 1;  // nodes of the largest such tree
__global__ __launch_bounds__(1024) void sync_refit_kernel(ScatterArgs a, DevScene sc, CullRec* __restrict__ nodes,
                                                          const uint32_t* __restrict__ ref, const uint32_t* __restrict__ pos,
                                                          float4* __restrict__ slots) {
  __shared__ uint32_t s_dirty[(kSyncRefitNodes + 31) / 32];
  const int tid = threadIdx.x;
  const int n = sc.ns + sc.na + sc.no, leaf0 = sc.bvh_leaf0, nleaf = 3 * leaf0 + 1;
  const int nd = a.ds + a.da + a.dob;
  for (int w = tid; w < (leaf0 + nleaf + 31) / 32; w += blockDim.x) s_dirty[w] = 0u;
  __syncthreads();
  for (int j = tid; j < nd; j += blockDim.x) {  // 1. the dirty records
    int k = j, g;
    if (k < a.ds) {
      const int i = a.idx_s[k];
      const art_sphere r = a.rec_s[k];
      a.sph[i] = r;
      prep_sphere(r, i, i, a.osph, a.osphc, a.cull);
      g = i;
    } else if ((k -= a.ds) < a.da) {
      const int i = a.idx_a[k];
      const art_aabb r = a.rec_a[k];
      a.aabb[i] = r;
      prep_aabb(r, i, a.ns + i, a.oaabb, a.oaabbc, a.cull);
      g = a.ns + i;
    } else {
      k -= a.da;
      const int i = a.idx_o[k];
      const art_obb r = a.rec_o[k];
      a.obb[i] = r;
      prep_obb(r, i, a.ns + a.na + i, a.oobb, a.oobbc, a.cull);
      g = a.ns + a.na + i;
    }
    const int leaf = leaf0 + (int)(pos[g] / kBvhLeaf);
    atomicOr(&s_dirty[leaf >> 5], 1u << (leaf & 31));
  }
  __syncthreads();
  for (int j = tid; j < nd; j += blockDim.x) {  // 2. their leaf slots, from the records written above
    int k = j, g;
    if (k < a.ds) g = a.idx_s[k];
    else if ((k -= a.ds) < a.da) g = a.ns + a.idx_a[k];
    else g = a.ns + a.na + a.idx_o[k - a.da];
    bvh_write_slot((int)pos[g], g, sc.ns, sc.na, n, sc.sph, sc.aabb, sc.obb, slots);
  }
  for (int i = tid; i < nleaf; i += blockDim.x) {  // ... and the boxes of their leaves
    const int node = leaf0 + i;
    if (!((s_dirty[node >> 5] >> (node & 31)) & 1u)) continue;
    CullRec u = cull_empty();
    for (int k = i * kBvhLeaf; k < (i + 1) * kBvhLeaf && k < n; ++k) cull_union(u, sc.cull[bvh_ref_global(ref[k], sc.ns, sc.na)]);
    nodes[node] = cull_stored(u);
  }
  __syncthreads();
  for (int l = sc.bvh_levels - 2; l >= 0; --l) {  // 3. the changed nodes' ancestors
    const int first = ((1 << (2 * l)) - 1) / 3, cnt = 1 << (2 * l);
    for (int i = tid; i < cnt; i += blockDim.x) {
      const int g = first + i;
      bool any = false;
      for (int k = 1; k <= 4; ++k) any |= ((s_dirty[(4 * g + k) >> 5] >> ((4 * g + k) & 31)) & 1u) != 0u;
      if (!any) continue;
      CullRec u = cull_empty();
      for (int k = 1; k <= 4; ++k) cull_union_stored(u, nodes[4 * g + k]);
      nodes[g] = cull_stored(u);
      atomicOr(&s_dirty[g >> 5], 1u << (g & 31));
    }
    __syncthreads();
  }
}

bool launch_sync_refit(const ScatterArgs& a, DevScene& sc, const SortBufs& sb, hipStream_t st) {
  const long long n = (long long)sc.ns + sc.na + sc.no;
  if (n == 0 || n > kSyncRefitMax || sc.bvh_levels == 0 || !sb.bvh || !sb.bvh_pos) return false;
  hipLaunchKernelGGL(sync_refit_kernel, dim3(1), dim3(1024), 0, st, a, sc, sb.bvh, sb.bvh_ref, sb.bvh_pos, sb.bvh_leaf);
  return true;
}

// Colliders moved but their counts did not: keep the leaf order and recompute the leaf slots and
// node bounds in place (no sort). Bounds stay exact unions, so the culls stay exact; only their
// tightness drifts until the next rebuild (a count change, or art_scene_bind).
int launch_refit_scene(DevScene& sc, const SortBufs& sb, hipStream_t st) {
  const int n = sc.ns + sc.na + sc.no;
  if (n == 0 || sc.bvh_levels == 0) return launch_sort_scene(sc, sb, st);
  const int leaf0 = sc.bvh_leaf0, nleaf = 3 * leaf0 + 1;  // 4^(L-1) leaves
  hipLaunchKernelGGL(bvh_leaf_kernel<true>, dim3((nleaf + 255) / 256), dim3(256), 0, st, sc.cull, (const int*)nullptr,
                     sc.ns, sc.na, n, sc.sph, sc.aabb, sc.obb, sb.bvh + leaf0, nleaf, sb.bvh_ref, sb.bvh_leaf,
                     (uint32_t*)nullptr);
  launch_bvh_upper(sb.bvh, sc.bvh_levels, st);
  return 0;
}

}  // namespace art
