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

int launch_sort_scene(DevScene& sc, const SortBufs& sb, hipStream_t st) {
  const int n = sc.ns + sc.na + sc.no;
  sc.nchunks = 0;
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
  return 0;
}

}  // namespace art
