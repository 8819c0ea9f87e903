// art_bvh.hip — spatially sorted collider copies and per-chunk bounds for the broad phase.
//
// The reference sweeps colliders in their list order (Sphere, AABB, OBB; AudioRaytracerJobBatched.cs
// :225-280), and the exact kernels keep that order. The throughput kernel's broad phase works on a
// second, spatially sorted copy of the hot records: each collider type is sorted by the Morton code
// of its bounds' centre (30 bits over the scene box), so a chunk of 64 consecutive sorted colliders
// is spatially compact and its bounds (the union of its members' CullRec, with the largest margin
// scale and factor of its members) reject whole chunks. Every sorted record carries its original
// index, which is what the nearest-hit tie-break and the outputs use.
//
// Built once per scene upload on the device: scene box -> Morton keys -> hipcub radix sort ->
// gather -> chunk bounds.
#include <hipcub/hipcub.hpp>

#include "art_device_fns.hpp"

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

__global__ void morton_kernel(const CullRec* __restrict__ cull, int ns, int na, int no, const float* __restrict__ box,
                              uint32_t* __restrict__ keys, int* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = ns + na + no;
  if (i >= n) return;
  const uint32_t type = i < ns ? 0u : (i < ns + na ? 1u : 2u);
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
  keys[i] = (type << 30) | code;
  vals[i] = i;
}

// sorted position j <- original global index perm[j]; records keep their original in-type index
__global__ void gather_kernel(const int* __restrict__ perm, int ns, int na, int no, const SphereRec* __restrict__ sph,
                              const AabbRec* __restrict__ aabb, const ObbRec* __restrict__ obb,
                              const CullRec* __restrict__ cull, SphereRec* __restrict__ sph_s,
                              AabbRec* __restrict__ aabb_s, ObbRec* __restrict__ obb_s, CullRec* __restrict__ cull_s) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ns + na + no) return;
  const int g = perm[j];
  cull_s[j] = cull[g];
  if (j < ns) {
    SphereRec r = sph[g];
    r.pad0 = g;
    sph_s[j] = r;
  } else if (j < ns + na) {
    AabbRec r = aabb[g - ns];
    r.pad = __int_as_float(g - ns);
    aabb_s[j - ns] = r;
  } else {
    ObbRec r = obb[g - ns - na];
    r.pad0 = __int_as_float(g - ns - na);
    obb_s[j - ns - na] = r;
  }
}

// Refit of the sorted copies after colliders moved (same counts): every sorted record keeps its
// position and is re-read from its original index (held in the record's pad field).
__global__ void refit_gather_kernel(int ns, int na, int no, const SphereRec* __restrict__ sph,
                                    const AabbRec* __restrict__ aabb, const ObbRec* __restrict__ obb,
                                    const CullRec* __restrict__ cull, SphereRec* __restrict__ sph_s,
                                    AabbRec* __restrict__ aabb_s, ObbRec* __restrict__ obb_s, CullRec* __restrict__ cull_s) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ns + na + no) return;
  if (j < ns) {
    const int g = sph_s[j].pad0;
    SphereRec r = sph[g];
    r.pad0 = g;
    sph_s[j] = r;
    cull_s[j] = cull[g];
  } else if (j < ns + na) {
    const int i = __float_as_int(aabb_s[j - ns].pad);
    AabbRec r = aabb[i];
    r.pad = __int_as_float(i);
    aabb_s[j - ns] = r;
    cull_s[j] = cull[ns + i];
  } else {
    const int i = __float_as_int(obb_s[j - ns - na].pad0);
    ObbRec r = obb[i];
    r.pad0 = __int_as_float(i);
    obb_s[j - ns - na] = r;
    cull_s[j] = cull[ns + na + i];
  }
}

// One wave per chunk of 64 sorted colliders of one type: union of the members' bounds, largest
// margin scale and factor.
__global__ __launch_bounds__(64) void chunk_bounds_kernel(const CullRec* __restrict__ cull_s, int ns, int na, int no,
                                                          CullRec* __restrict__ chunks) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const int cs = (ns + 63) / 64, ca = (na + 63) / 64;
  int b, n;
  if (c < cs) { b = c * 64; n = min(64, ns - b); }
  else if (c < cs + ca) { b = ns + (c - cs) * 64; n = min(64, ns + na - b); }
  else { b = ns + na + (c - cs - ca) * 64; n = min(64, ns + na + no - b); }
  CullRec r;
  if (lane < n) {
    r = cull_s[b + lane];
  } else {
    r.lox = r.loy = r.loz = INFINITY; r.hix = r.hiy = r.hiz = -INFINITY; r.scale = 0.0f; r.factor = 0.0f;
  }
  // block reductions through LDS (one wave): NaN-free by construction (non-finite -> +-inf)
  __shared__ float s[8][64];
  s[0][lane] = r.lox; s[1][lane] = r.loy; s[2][lane] = r.loz; s[3][lane] = r.scale;
  s[4][lane] = r.hix; s[5][lane] = r.hiy; s[6][lane] = r.hiz; s[7][lane] = r.factor;
  __syncthreads();
  for (int st = 32; st > 0; st >>= 1) {
    if (lane < st) {
      for (int a = 0; a < 3; ++a) s[a][lane] = fminf(s[a][lane], s[a][lane + st]);
      for (int a = 3; a < 8; ++a) s[a][lane] = fmaxf(s[a][lane], s[a][lane + st]);
    }
    __syncthreads();
  }
  if (lane == 0) {
    CullRec o;
    o.lox = s[0][0]; o.loy = s[1][0]; o.loz = s[2][0]; o.scale = s[3][0];
    o.hix = s[4][0]; o.hiy = s[5][0]; o.hiz = s[6][0]; o.factor = s[7][0];
    chunks[c] = o;
  }
}

size_t sort_scene_temp_bytes(int n) {
  size_t bytes = 0;
  if (n <= 0) return 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const int*)nullptr, (int*)nullptr, n, 0, 32) != hipSuccess)
    return 0;
  return bytes;
}

int launch_build_bvh(DevScene& sc, const SortBufs& sb, hipStream_t st);

int launch_sort_scene(DevScene& sc, const SortBufs& sb, hipStream_t st) {
  const int n = sc.ns + sc.na + sc.no;
  sc.nchunks = 0;
  sc.bvh = nullptr; sc.bvh_ref = nullptr; sc.bvh_leaf = nullptr; sc.bvh_levels = 0;
  if (n == 0) return 0;
  hipLaunchKernelGGL(scene_box_kernel, dim3(1), dim3(1024), 0, st, sc.cull, n, sb.box);
  hipLaunchKernelGGL(morton_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc.cull, sc.ns, sc.na, sc.no, sb.box, sb.keys,
                     sb.vals);
  size_t bytes = sb.temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(sb.temp, bytes, sb.keys, sb.keys_s, sb.vals, sb.perm, n, 0, 32, st) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(gather_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sb.perm, sc.ns, sc.na, sc.no, sc.sph, sc.aabb,
                     sc.obb, sc.cull, sb.sph_s, sb.aabb_s, sb.obb_s, sb.cull_s);
  const int nch = (sc.ns + 63) / 64 + (sc.na + 63) / 64 + (sc.no + 63) / 64;
  hipLaunchKernelGGL(chunk_bounds_kernel, dim3(nch), dim3(64), 0, st, sb.cull_s, sc.ns, sc.na, sc.no, sb.chunks);
  sc.sph_s = sb.sph_s; sc.aabb_s = sb.aabb_s; sc.obb_s = sb.obb_s; sc.cull_s = sb.cull_s; sc.chunks = sb.chunks;
  sc.nchunks = nch;
  // the BVH reuses the key / value / temp buffers: stream order puts it after the gather above
  return launch_build_bvh(sc, sb, st);
}

// ------------------------------------------------------------------------------------------
// BVH of the quad traversals (art_trace.hip) and the permeation loss rays (art_kernels.hip): all colliders in
// one Morton order of their bounds' centres (types mixed), kBvhLeaf per leaf, an implicit complete
// 4-ary tree above. Node bounds are unions of CullRecs with the largest margin scale and factor,
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
  a.scale = fmaxf(a.scale, b.scale); a.factor = fmaxf(a.factor, b.factor);
}

__device__ __forceinline__ CullRec cull_empty() {
  CullRec r;
  r.lox = r.loy = r.loz = INFINITY; r.hix = r.hiy = r.hiz = -INFINITY; r.scale = 0.0f; r.factor = 0.0f;
  return r;
}

// Leaf j = sorted colliders [kBvhLeaf j, kBvhLeaf (j + 1)) (empty past the last); writes the
// leaf references.
// REFIT: the leaf order is kept (ref holds it) and only bounds and slots are recomputed.
template <bool REFIT>
__global__ void bvh_leaf_kernel(const CullRec* __restrict__ cull, const int* __restrict__ perm, int ns, int na, int n,
                                const SphereRec* __restrict__ sph, const AabbRec* __restrict__ aabb,
                                const ObbRec* __restrict__ obb, CullRec* __restrict__ leaves, int nleaf,
                                uint32_t* __restrict__ ref, float4* __restrict__ slots) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nleaf) return;
  CullRec u = cull_empty();
  // slot (64 B): a = first 16 B, b = next 16 B (b.w = code), c, d = an OBB's local bounds
  //   sphere: a = (cx, cy, cz, r2), b.z = AudioTargetId
  //   AABB:   a = (mn.xyz, mx.x), b.xy = mx.yz, b.z = AudioTargetId
  //   OBB:    a = (c.xyz, q.x), b.xyz = q.yzw, c = (lmn.xyz, lmx.x), d.xy = lmx.yz, d.z = AudioTargetId
  for (int k = j * kBvhLeaf; k < (j + 1) * kBvhLeaf; ++k) {
    float4* sl = slots + 4 * (size_t)k;
    float4 a = make_float4(0, 0, 0, 0), b = a, c = a, d = a;
    int code = -1;
    if (k < n) {
      int g;
      if (REFIT) {
        const uint32_t r = ref[k], t = r >> 30, i = r & 0x3fffffffu;
        g = (int)i + (t == 0 ? 0 : (t == 1 ? ns : ns + na));
      } else {
        g = perm[k];
      }
      cull_union(u, cull[g]);
      if (g < ns) {
        ref[k] = (uint32_t)g;
        const SphereRec r = sph[g];
        a = make_float4(r.cx, r.cy, r.cz, r.r2);
        b.z = __int_as_float(r.tid);
        code = g;
      } else if (g < ns + na) {
        ref[k] = (1u << 30) | (uint32_t)(g - ns);
        const AabbRec r = aabb[g - ns];
        a = make_float4(r.mnx, r.mny, r.mnz, r.mxx);
        b = make_float4(r.mxy, r.mxz, __int_as_float(r.tid), 0.0f);
        code = (1 << 28) | (g - ns);
      } else {
        ref[k] = (2u << 30) | (uint32_t)(g - ns - na);
        const ObbRec r = obb[g - ns - na];
        a = make_float4(r.cx, r.cy, r.cz, r.qx);
        b = make_float4(r.qy, r.qz, r.qw, 0.0f);
        c = make_float4(r.lmnx, r.lmny, r.lmnz, r.lmxx);
        d = make_float4(r.lmxy, r.lmxz, __int_as_float(r.tid), 0.0f);
        code = (2 << 28) | (g - ns - na);
      }
    }
    b.w = __int_as_float(code);
    sl[0] = a; sl[1] = b; sl[2] = c; sl[3] = d;
  }
  leaves[j] = u;
}

// One inner level l (large trees: levels with more nodes than one workgroup handles quickly).
__global__ __launch_bounds__(256) void bvh_level_kernel(CullRec* __restrict__ nodes, int l) {
  const int first = ((1 << (2 * l)) - 1) / 3, cnt = 1 << (2 * l);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cnt) return;
  const int g = first + i;
  CullRec u = cull_empty();
  for (int k = 1; k <= 4; ++k) cull_union(u, nodes[4 * g + k]);
  nodes[g] = u;
}

// Inner levels top_level .. 0, bottom-up, in one workgroup (they hold a third of the leaf count).
__global__ __launch_bounds__(1024) void bvh_upper_kernel(CullRec* __restrict__ nodes, int top_level) {
  for (int l = top_level; l >= 0; --l) {
    const int first = ((1 << (2 * l)) - 1) / 3, cnt = 1 << (2 * l);
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
      const int g = first + i;
      CullRec u = cull_empty();
      for (int k = 1; k <= 4; ++k) cull_union(u, nodes[4 * g + k]);
      nodes[g] = u;
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

int launch_build_bvh(DevScene& sc, const SortBufs& sb, hipStream_t st) {
  const int n = sc.ns + sc.na + sc.no;
  int leaf0 = 0, total = 0;
  const int L = bvh_layout(n, leaf0, total);
  sc.bvh = nullptr; sc.bvh_ref = nullptr; sc.bvh_leaf = nullptr; sc.bvh_levels = 0; sc.bvh_leaf0 = 0;
  if (L == 0 || !sb.bvh || !sb.bvh_ref || !sb.bvh_leaf) return 0;
  hipLaunchKernelGGL(scene_box_kernel, dim3(1), dim3(1024), 0, st, sc.cull, n, sb.box);
  hipLaunchKernelGGL(morton_all_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc.cull, n, sb.box, sb.keys, sb.vals);
  size_t bytes = sb.temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(sb.temp, bytes, sb.keys, sb.keys_s, sb.vals, sb.perm, n, 0, 30, st) != hipSuccess)
    return -1;
  const int nleaf = total - leaf0;
  hipLaunchKernelGGL(bvh_leaf_kernel<false>, dim3((nleaf + 255) / 256), dim3(256), 0, st, sc.cull, sb.perm, sc.ns, sc.na, n,
                     sc.sph, sc.aabb, sc.obb, sb.bvh + leaf0, nleaf, sb.bvh_ref, sb.bvh_leaf);
  launch_bvh_upper(sb.bvh, L, st);
  sc.bvh = sb.bvh; sc.bvh_ref = sb.bvh_ref; sc.bvh_leaf = sb.bvh_leaf; sc.bvh_levels = L; sc.bvh_leaf0 = leaf0;
  return 0;
}

// Colliders moved but their counts did not: keep every order (per-type sorted copies, BVH leaf
// order) and recompute records and bounds in place (4 kernels instead of the 11 of a rebuild).
// Bounds stay exact unions, so the culls stay exact; only their tightness drifts until the next
// rebuild (a count change, or art_scene_bind).
int launch_refit_scene(DevScene& sc, const SortBufs& sb, hipStream_t st) {
  const int n = sc.ns + sc.na + sc.no;
  if (n == 0 || sc.cull_s == nullptr) return launch_sort_scene(sc, sb, st);
  hipLaunchKernelGGL(refit_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sc.ns, sc.na, sc.no, sc.sph, sc.aabb,
                     sc.obb, sc.cull, sb.sph_s, sb.aabb_s, sb.obb_s, sb.cull_s);
  const int nch = (sc.ns + 63) / 64 + (sc.na + 63) / 64 + (sc.no + 63) / 64;
  hipLaunchKernelGGL(chunk_bounds_kernel, dim3(nch), dim3(64), 0, st, sb.cull_s, sc.ns, sc.na, sc.no, sb.chunks);
  if (sc.bvh_levels > 0) {
    const int leaf0 = sc.bvh_leaf0, nleaf = 3 * leaf0 + 1;  // 4^(L-1) leaves
    hipLaunchKernelGGL(bvh_leaf_kernel<true>, dim3((nleaf + 255) / 256), dim3(256), 0, st, sc.cull, (const int*)nullptr,
                       sc.ns, sc.na, n, sc.sph, sc.aabb, sc.obb, sb.bvh + leaf0, nleaf, sb.bvh_ref, sb.bvh_leaf);
    launch_bvh_upper(sb.bvh, sc.bvh_levels, st);
  }
  return 0;
}

}  // namespace art
