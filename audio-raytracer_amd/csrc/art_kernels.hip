// art_kernels.hip — CDNA4 (gfx950) kernels for the audio ray-tracing hot path.
//
//   prep_kernel      half AoS colliders -> fp32 SoA records (decode + per-collider precompute)
//   raytrace_kernel  AudioRaytracerJobBatched.Execute   (Jobs/AudioRaytracerJobBatched.cs:61-215)
//   permeate_kernel  AudioPermeationJobBatched.Execute  (Jobs/AudioPermeationJobBatched.cs:34-91)
//   reduce_kernel    ProcessAudioDataJob.Execute        (Jobs/ProcessAudioDataJob.cs:32-76)
//                    + DSP parameters                   (AudioSpatializer.cs:58, ReverbDSP.cs:12-13,
//                                                        MuffleDSP.cs:22-26, :38-42)
//
// Mapping: one lane per (fan, ray). All lanes of a wave sweep the collider arrays in the same
// order, so every collider record is wave-uniform and is fetched with scalar loads into SGPRs.
// Any-hit loops (echo / muffle visibility) exit per lane at the first blocker; the wave leaves
// the loop as soon as its last lane has exited (exec mask empty).
//
// Bit-exactness: compiled with -ffp-contract=off, IEEE division/sqrt, f32 denormals on.
// See unity_math.hpp and DESIGN.md §5 for the arguments behind each deviation from a literal
// transcription (hoisted 1/d, per-collider precompute, IEEE minNum/maxNum in sweep loops).
#include <float.h>
#include <hip/hip_runtime.h>

#include "art_device_fns.hpp"
#include "art_frame_math.hpp"

#pragma clang fp contract(off)

namespace art {

// ------------------------------------------------------------------------------------------
// prep: decode colliders once per upload. Every value is computed exactly as the reference
// computes it per access (Center - Size, Radius * Radius, halfQuaternion decode, inverse), so
// hoisting is bit-identical.
// ------------------------------------------------------------------------------------------
__global__ void prep_kernel(const art_sphere* __restrict__ sph, int ns, const art_aabb* __restrict__ aabb, int na,
                            const art_obb* __restrict__ obb, int no, SphereRec* __restrict__ osph,
                            SphereCold* __restrict__ osphc, AabbRec* __restrict__ oaabb, AabbCold* __restrict__ oaabbc,
                            ObbRec* __restrict__ oobb, ObbCold* __restrict__ oobbc, CullRec* __restrict__ cull) {
  const int gi = blockIdx.x * blockDim.x + threadIdx.x;  // global collider order (spheres, AABBs, OBBs)
  int i = gi;
  if (i < ns) { prep_sphere(sph[i], i, gi, osph, osphc, cull); return; }
  i -= ns;
  if (i < na) { prep_aabb(aabb[i], i, gi, oaabb, oaabbc, cull); return; }
  i -= na;
  if (i < no) prep_obb(obb[i], i, gi, oobb, oobbc, cull);
}

// Resident collider store (include/art_colliders.h): each dirty record is written to the
// resident AoS list at its index and decoded in place; the bounds use the synced counts.
__global__ void scatter_prep_kernel(const int* __restrict__ idx_s, const art_sphere* __restrict__ rec_s, int ds,
                                    const int* __restrict__ idx_a, const art_aabb* __restrict__ rec_a, int da,
                                    const int* __restrict__ idx_o, const art_obb* __restrict__ rec_o, int dob,
                                    art_sphere* __restrict__ sph, art_aabb* __restrict__ aabb, art_obb* __restrict__ obb,
                                    int ns, int na, SphereRec* __restrict__ osph, SphereCold* __restrict__ osphc,
                                    AabbRec* __restrict__ oaabb, AabbCold* __restrict__ oaabbc, ObbRec* __restrict__ oobb,
                                    ObbCold* __restrict__ oobbc, CullRec* __restrict__ cull) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < ds) {
    const int i = idx_s[j];
    const art_sphere r = rec_s[j];
    sph[i] = r;
    prep_sphere(r, i, i, osph, osphc, cull);
    return;
  }
  j -= ds;
  if (j < da) {
    const int i = idx_a[j];
    const art_aabb r = rec_a[j];
    aabb[i] = r;
    prep_aabb(r, i, ns + i, oaabb, oaabbc, cull);
    return;
  }
  j -= da;
  if (j < dob) {
    const int i = idx_o[j];
    const art_obb r = rec_o[j];
    obb[i] = r;
    prep_obb(r, i, ns + na + i, oobb, oobbc, cull);
  }
}

// ------------------------------------------------------------------------------------------
// raytrace — AudioRaytracerJobBatched.Execute :61-215. grid = (ray blocks, fans).
// ------------------------------------------------------------------------------------------
template <bool COUNT, bool HITS>
__global__ __launch_bounds__(kRtBlock) void raytrace_kernel(DevScene sc, FrameParams fp, FanLayout L,
                                                            const float* __restrict__ origins, uint8_t* __restrict__ block,
                                                            uint32_t* __restrict__ muffle_acc, DevCounts* counts) {
  __shared__ uint32_t s_muf[kMaxTargets];
  const int fan = blockIdx.y;
  const int ray = blockIdx.x * blockDim.x + threadIdx.x;
  const int T = fp.T;
  for (int t = threadIdx.x; t < T; t += blockDim.x) s_muf[t] = 0;
  // batch slot of this block's rays (batchId = rayStart * TC / R, :63-64)
  const int first_ray = blockIdx.x * blockDim.x;
  const int last_ray = min(first_ray + (int)blockDim.x, fp.R) - 1;
  auto slot_of = [&](int r) { int st = (r / fp.bs) * fp.bs; return (int)(((long long)st * fp.TC) / fp.R); };
  const bool uniform_slot = slot_of(first_ray) == slot_of(last_ray);
  __syncthreads();

  LaneCounts lc = {0, 0, 0};
  uint8_t* fb = block + (size_t)fan * L.stride;
  if (ray < fp.R) {
    uint16_t* echo = reinterpret_cast<uint16_t*>(fb + L.echo_off);
    art_half3* hpo = reinterpret_cast<art_half3*>(fb + L.hit_points_off);
    uint32_t* hid = reinterpret_cast<uint32_t*>(fb + L.hit_ids_off);
    const int H = fp.H;  // <= 32 (validated on the host)
    const int my_slot = slot_of(ray);
    // Reset of this ray's slots (:72-80) under sequential-batch semantics. At TC == 1 every slot
    // is reset and nothing is frozen. frozen bit k: a later batch's reset zeroes slot k after
    // this ray wrote it, so the ray's own write must not land.
    uint32_t frozen = 0;
    {
      const int my_batch = ray / fp.bs;
      const art_half3 z = {0, 0, 0};
      for (int k = 0; k < H; ++k) {
        const int j = ray * H + k;
        bool any_reset;
        const int keep = batch_slot_state(fp, j, my_batch, any_reset);
        if (!keep) frozen |= 1u << k;
        if (!keep || any_reset) {
          echo[j] = 0;
          if (HITS) { hpo[j] = z; hid[j] = ART_HIT_NONE; }
        }
      }
    }
    const vec3 O = load3(origins, fan);
    vec3 o = O;
    vec3 d = load_dir(sc.dirs, ray);
    float life = fp.max_life;
    int hits = 0;
    bool alive = true;

    while (alive) {
      Seg s = make_seg(o, d);
      Hit h = nearest<false, COUNT>(sc, s, lc);
      if (h.type == kNone) break;                       // :200-207
      o = o + d * h.dist;                               // :111
      life -= h.dist;                                   // :112
      hits += 1;                                        // :113
      const int k = hits - 1;
      const int rid = ray * H + k;                      // :115
      const bool live_slot = !((frozen >> k) & 1u);
      if (HITS && live_slot) {                          // :118, :197
        art_half3 p;
        p.x = f32tof16(o.x); p.y = f32tof16(o.y); p.z = f32tof16(o.z);
        hpo[rid] = p;
        hid[rid] = ART_HIT_ID(h.type, h.idx);
      }
      // Echo — :124-145
      vec3 off = o - d * kEps;
      vec3 rdir = normalize(O - off);
      float dist0 = distance(O, o);
      if (visible<false, COUNT>(sc, make_seg(off, rdir), dist0, -1, lc) && live_slot) {
        float em = h.type == kSphere ? sc.sphc[h.idx].echo : (h.type == kAabb ? sc.aabbc[h.idx].echo : sc.obbc[h.idx].echo);
        echo[rid] = f32tof16(dist0 * em);               // Half.Multiply, HalfDataTypesUtility.cs:86-90
      }
      // Muffle — :150-173
      for (int t = 0; t < T; ++t) {
        vec3 tp = load3(sc.targets, t);
        vec3 tdir = normalize(tp - off);
        float dt = distance(off, tp);
        if (dt < fp.max_muffle && visible<true, COUNT>(sc, make_seg(off, tdir), dt, t, lc)) {
          if (uniform_slot) atomicAdd(&s_muf[t], 1u);
          else atomicAdd(&muffle_acc[((size_t)fan * fp.TC + my_slot) * T + t], 1u);
        }
      }
      // Termination / reflection — :179-193, ReflectRay :456-532
      if (hits >= H || life <= 0.0f) {
        alive = false;
      } else {
        vec3 n = mk3(0.0f, 0.0f, 0.0f);
        float absorption = 0.0f;
        if (h.type == kAabb) {
          const AabbCold b = sc.aabbc[h.idx];
          vec3 lp = o - mk3(b.cx, b.cy, b.cz);
          vec3 ap = abs3(lp);
          float dx = b.hx - ap.x, dy = b.hy - ap.y, dz = b.hz - ap.z;
          if (dx < dy && dx < dz) n.x = usign(lp.x);
          else if (dy < dx && dy < dz) n.y = usign(lp.y);
          else n.z = usign(lp.z);
          absorption = b.absorption;
        } else if (h.type == kObb) {
          const ObbRec b = sc.obb[h.idx];
          const ObbCold bc = sc.obbc[h.idx];
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
          const SphereRec c = sc.sph[h.idx];
          n = normalize(o - mk3(c.cx, c.cy, c.cz));
          absorption = sc.sphc[h.idx].absorption;
        }
        d = reflect(d, n);                               // :525
        o = o + d * kEps;                                // :528
        life -= fp.max_life * absorption;                // :531
        if (life < 0.0f) alive = false;                  // :189
      }
    }
    if (HITS) fb[L.hit_counts_off + ray] = (uint8_t)hits;  // :204, :212
  }

  __syncthreads();
  if (uniform_slot) {
    const int slot = slot_of(first_ray);
    for (int t = threadIdx.x; t < T; t += blockDim.x)
      if (s_muf[t]) atomicAdd(&muffle_acc[((size_t)fan * fp.TC + slot) * T + t], s_muf[t]);
  }
  if (COUNT) {
    unsigned long long vs = wave_sum_u32(lc.s), va = wave_sum_u32(lc.a), vo = wave_sum_u32(lc.o);
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&counts->v[0], vs); atomicAdd(&counts->v[1], va); atomicAdd(&counts->v[2], vo);
    }
  }
}

// ------------------------------------------------------------------------------------------
// permeate — AudioPermeationJobBatched.Execute :34-91. grid = (slots TC, fans), 256 threads.
// Each hitting ray OVERWRITES PermeationPowerRemains[slot*T+t] (:85), so a slot's final value is
// the one of the highest-index hitting ray of the last batch that maps to it (App. B Q7). The
// kernel finds that ray by sweeping the batch from its end, then evaluates its T loss rays; the
// per-collider loss terms are computed in parallel and summed serially in reference order.
// ------------------------------------------------------------------------------------------
constexpr int kPermBlock = 256;

// Permeation first hit of one ray (ShootRayCast :101-141, OBB with the inverted stored rotation
// :172-179) with the block's threads over the colliders: each thread keeps the first minimum of its
// colliders (ascending global order, strict <), and a block reduction by (distance, global order)
// gives the reference's first minimum over Sphere, AABB, OBB order. Block-uniform result.
__device__ Hit nearest_block_perm(const DevScene& sc, const Seg& s, int tid, float* s_rd, int* s_ri) {
  const int ctot = sc.ns + sc.na + sc.no;
  float bd = __builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int c = tid; c < ctot; c += kPermBlock) {
    float d;
    bool hit;
    if (c < sc.ns) {
      hit = sphere_test(s, sc.sph[c], d);
    } else if (c < sc.ns + sc.na) {
      hit = aabb_test<false>(s, sc.aabb[c - sc.ns], d);
    } else {
      const int i = c - sc.ns - sc.na;
      hit = obb_test<false>(s, sc.obb[i], inverse_q(sc.obbc[i]), d);
    }
    if (hit && d < bd) { bd = d; bi = c; }
  }
  s_rd[tid] = bd;
  s_ri[tid] = bi;
  __syncthreads();
  for (int st = kPermBlock / 2; st > 0; st >>= 1) {
    if (tid < st) {
      const float d2 = s_rd[tid + st];
      const int i2 = s_ri[tid + st];
      if (d2 < s_rd[tid] || (d2 == s_rd[tid] && i2 < s_ri[tid])) { s_rd[tid] = d2; s_ri[tid] = i2; }
    }
    __syncthreads();
  }
  Hit h;
  h.type = kNone; h.idx = -1; h.dist = s_rd[0];
  const int g = s_ri[0];
  __syncthreads();  // s_rd / s_ri are reused by the next call
  if (g == 0x7fffffff) return h;
  if (g < sc.ns) {
    h.type = kSphere; h.idx = g;
  } else if (g < sc.ns + sc.na) {
    h.type = kAabb; h.idx = g - sc.ns;
    float d; aabb_test<true>(s, sc.aabb[h.idx], d); h.dist = d;  // exact re-evaluation (zero sign)
  } else {
    h.type = kObb; h.idx = g - sc.ns - sc.na;
    float d; obb_test<true>(s, sc.obb[h.idx], inverse_q(sc.obbc[h.idx]), d); h.dist = d;
  }
  if (h.dist == __builtin_huge_valf()) h.type = kNone;  // :140 closestDist != INFINITY
  return h;
}

__global__ __launch_bounds__(kPermBlock) void permeate_kernel(DevScene sc, FrameParams fp, FanLayout L,
                                                              const float* __restrict__ origins, uint8_t* __restrict__ block,
                                                              const int2* __restrict__ slot_batch) {
  __shared__ Hit s_hit;
  __shared__ float s_terms[kPermBlock];
  __shared__ float s_rd[kPermBlock];
  __shared__ int s_ri[kPermBlock];
#ifdef ART_PERM_EMPTY  // measurement-only build (tools/build_variant.sh): bounds what a faster pass could gain
  return;
#endif
  const int fan = blockIdx.y, slot = blockIdx.x, tid = threadIdx.x;
  const int2 br = slot_batch[slot];
  if (br.y <= br.x) return;  // no batch maps to this slot: value stays (stale / uninitialized, Q7)
  const vec3 O = load3(origins, fan);
  LaneCounts lc = {0, 0, 0};

  // Phase 1: highest-index ray in [br.x, br.y) whose first hit exists (ShootRayCast :58). Rays
  // are taken from the end one at a time, each with the block's threads over the colliders
  // (lane = collider); the first ray that hits ends the search, so usually one sweep is needed.
  int found = -1;
  (void)lc;
  for (int ray = br.y - 1; ray >= br.x; --ray) {
    const Hit h = nearest_block_perm(sc, make_seg(O, load_dir(sc.dirs, ray)), tid, s_rd, s_ri);
    if (h.type != kNone) {
      if (tid == 0) s_hit = h;
      __syncthreads();
      found = ray;
      break;
    }
  }

  float* ppr = reinterpret_cast<float*>(block + (size_t)fan * L.stride + L.perm_off);
  const int T = fp.T;
  if (found < 0) {  // reset (:43-46) and no ray hit: zeros
    for (int t = tid; t < T; t += kPermBlock) ppr[slot * T + t] = 0.0f;
    return;
  }
  // Phase 2: T loss rays of the found ray (:61-85)
  const vec3 d = load_dir(sc.dirs, found);
  const vec3 o = O + d * s_hit.dist;
  const int ctot = sc.ns + sc.na + sc.no;
  const int lane = tid & 63, wave = tid >> 6;
  for (int t = 0; t < T; ++t) {
    const vec3 off = o - d * kEps;
    const vec3 tdir = normalize(load3(sc.targets, t) - off);
    const Seg s = make_seg(off, tdir);
    float sum = 0.0f;  // uniform in wave 0
    for (int base = 0; base < ctot; base += kPermBlock) {
      const int c = base + tid;
      float term = 0.0f;
      if (c < sc.ns) {
        const SphereRec r = sc.sph[c];
        if (r.tid != t) term = perm_term_sphere(s, r, sc.sphc[c].density);
      } else if (c < sc.ns + sc.na) {
        const AabbRec r = sc.aabb[c - sc.ns];
        if (r.tid != t)
          term = perm_term_slab(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.mnx, r.mny, r.mnz, r.mxx, r.mxy, r.mxz,
                                sc.aabbc[c - sc.ns].density);
      } else if (c < ctot) {
        const ObbRec r = sc.obb[c - sc.ns - sc.na];
        if (r.tid != t) {
          quat q = stored_q(r);  // RayIntersectsOBBPermeation :294-300 uses the stored rotation
          vec3 lo = qmul(q, s.o - mk3(r.cx, r.cy, r.cz));
          vec3 ld = qmul(q, s.d);
          term = perm_term_slab(lo.x, lo.y, lo.z, 1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z, r.lmnx, r.lmny, r.lmnz, r.lmxx,
                                r.lmxy, r.lmxz, sc.obbc[c - sc.ns - sc.na].density);
        }
      }
      s_terms[tid] = term;
      __syncthreads();
      if (wave == 0) {
        // Serial, in collider order: only non-zero terms change the sum (x + ±0 == x for x != -0,
        // and the running sum starts at +0).
        for (int w = 0; w < kPermBlock / 64; ++w) {
          float v = s_terms[w * 64 + lane];
          unsigned long long m = __ballot(v != 0.0f);
          while (m) {
            int j = __builtin_ctzll(m);
            m &= m - 1;
            sum += __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
          }
        }
      }
      __syncthreads();
    }
    if (tid == 0) ppr[slot * T + t] = (float)fp.R * fp.perm_strength - sum;  // :260
  }
}

// Counting pass for the permeation job (test-count metric only, never timed): every ray runs
// ShootRayCast over all colliders (:58); each hitting ray then runs T loss rays over the
// non-owned colliders (:67-86), whose count the host derives from the number of hitting rays.
__global__ __launch_bounds__(kPermBlock) void perm_count_kernel(DevScene sc, FrameParams fp, const float* __restrict__ origins,
                                                                DevCounts* counts, unsigned long long* nhit) {
  const int fan = blockIdx.y, ray = blockIdx.x * blockDim.x + threadIdx.x;
  LaneCounts lc = {0, 0, 0};
  uint32_t hit = 0;
  if (ray < fp.R) {
    Hit h = nearest<true, true>(sc, make_seg(load3(origins, fan), load_dir(sc.dirs, ray)), lc);
    hit = h.type != kNone;
  }
  unsigned long long vs = wave_sum_u32(lc.s), va = wave_sum_u32(lc.a), vo = wave_sum_u32(lc.o), vh = wave_sum_u32(hit);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&counts->v[3], vs); atomicAdd(&counts->v[4], va); atomicAdd(&counts->v[5], vo);
    atomicAdd(nhit, vh);
  }
}

// ------------------------------------------------------------------------------------------
// reduce — ProcessAudioDataJob.Execute :32-76 + AudioTargetRTSettings ctor + DSP parameters.
// One wave per fan. The echo sum is sequential in index order (App. A.4): non-zero halves are
// added one by one in order; zeros are counted as "returned" (Q4).
// ------------------------------------------------------------------------------------------
// perm_in (host-API frames at TC == 1 without the permeation stage): the caller's permeation
// slots, uploaded with the origins, in place of the block's (which then stay unwritten and are not
// copied back). host_out (host-API frames): the fan's whole result record is also stored into the
// pinned host staging (the frame's D2H copy, done by the kernel that finishes the frame).
#ifndef ART_REDUCE_PACK
#define ART_REDUCE_PACK 1
#endif
__global__ __launch_bounds__(64) void reduce_kernel(DevScene sc, FrameParams fp, FanLayout L, uint8_t* __restrict__ block,
                                                    const uint32_t* __restrict__ muffle_acc,
                                                    const uint8_t* __restrict__ muffle_reset, const float* __restrict__ perm_in,
                                                    uint8_t* __restrict__ host_out) {
  const int fan = blockIdx.x, lane = threadIdx.x;
  uint8_t* fb = block + (size_t)fan * L.stride;
  const int T = fp.T, TC = fp.TC;
  uint16_t* muf = reinterpret_cast<uint16_t*>(fb + L.muffle_off);
  // MuffleRayHits (u16 wrap, :171) from the raytrace accumulators; slots no batch reset keep their value (Q18).
  if (fp.stages & ART_STAGE_RAYTRACE)
    for (int i = lane; i < TC * T; i += 64)
      if (muffle_reset[i / T]) muf[i] = (uint16_t)muffle_acc[(size_t)fan * TC * T + i];
  if (!(fp.stages & ART_STAGE_REDUCE)) return;
  __syncthreads();

  const uint16_t* echo = reinterpret_cast<const uint16_t*>(fb + L.echo_off);
  const int n = fp.R * fp.H;
  // The echo sum (:42-47) must add in index order. Zeros only count as returned, and adding a zero
  // leaves the running sum unchanged (it starts at +0 and a round-to-nearest sum of non-zero terms
  // is never -0), so only the non-zero terms are added: the wave converts a chunk to floats and
  // packs its non-zero ones, in index order, into LDS (coalesced loads, parallel conversion, one
  // ballot per 64 elements), and lane 0 accumulates them from 16-B LDS reads, with no cross-lane
  // step per element. (Round 6: every element was added; the serial chain is now as long as the
  // frame's visible echoes.)
  constexpr int kChunkF = 4096;
  __shared__ float4 s_f4[kChunkF / 4];
  float* s_f = reinterpret_cast<float*>(s_f4);
  float total = 0.0f;
  uint32_t zeros = 0;
  for (int base = 0; base < n; base += kChunkF) {
    const int m = min(kChunkF, n - base);
    int packed = 0;  // wave-uniform: non-zero terms of this chunk so far
    for (int i0 = 0; i0 < m; i0 += 8 * 64) {  // 8 independent loads per lane in flight
      uint16_t h[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + 64 * j + lane;
        h[j] = i < m ? echo[base + i] : (uint16_t)0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + 64 * j + lane;
        const bool in = i < m;
        const float e = f16tof32(h[j]);
        if (ART_REDUCE_PACK) {
          const unsigned long long nz = __ballot(in && e != 0.0f);  // (NaN included)
          if (in && e != 0.0f) s_f[packed + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(nz >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nz, 0u))] = e;
          packed += __popcll(nz);
        } else {
          if (in) s_f[i] = e;
        }
        zeros += __popcll(__ballot(in && e == 0.0f));
      }
    }
    __syncthreads();
    const int mm = ART_REDUCE_PACK ? packed : m;
    if (lane == 0) {  // 8 LDS reads in flight ahead of the 32 dependent adds they feed
      const int m = mm;
      int i = 0;
      for (; i + 32 <= m; i += 32) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = s_f4[(i >> 2) + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) { total += v[j].x; total += v[j].y; total += v[j].z; total += v[j].w; }
      }
      for (; i + 4 <= m; i += 4) {
        const float4 v = s_f4[i >> 2];
        total += v.x; total += v.y; total += v.z; total += v.w;
      }
      for (; i < m; ++i) total += s_f[i];
    }
    __syncthreads();
  }
  total = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, total), 0));
  // echoRayReturnedHits is a float incremented by 1 (exact below 2^24).
  const float returned = (float)zeros;
  const float avg = total / (float)n;
  const float reverbStrength = avg / fp.max_reverb;
  const float reverbVolume = returned / (float)n;

  const float* ppr = perm_in ? perm_in + (size_t)fan * TC * T : reinterpret_cast<const float*>(fb + L.perm_off);
  art_target_settings* st = reinterpret_cast<art_target_settings*>(fb + L.settings_off);
  art_dsp_params* dp = reinterpret_cast<art_dsp_params*>(fb + L.dsp_off);
  for (int t = lane; t < T; t += 64) {
    int hitsum = 0;
    float psum = 0.0f;
    for (int i = 0; i < TC; ++i) { hitsum += muf[T * i + t]; psum += ppr[T * i + t]; }
    float muffle = 1.0f - (float)hitsum / (float)(fp.R * fp.H) * fp.muffle_eff;        // :68
    float perm = psum / (float)fp.R / fp.perm_strength * fp.perm_eff;                  // :69
    muffle = usaturate(muffle - perm);                                                 // :71
    art_target_settings s;
    s.muffle_strength = usaturate(muffle);
    s.reverb_strength = usaturate(reverbStrength);
    s.reverb_volume = usaturate(reverbVolume);
    s.perceived_position[0] = sc.targets[3 * t + 0];
    s.perceived_position[1] = sc.targets[3 * t + 1];
    s.perceived_position[2] = sc.targets[3 * t + 2];
    st[t] = s;
    if ((fp.stages & ART_STAGE_DSP_PARAMS) && L.has_dsp) {
      const float DOUBLE_PI = 2.0f * 3.14159265f;
      art_dsp_params p;
      p.dry_level = ulerp(fp.dl_min, fp.dl_max, s.reverb_strength);
      p.dry_boost = ulerp(fp.db_min, fp.db_max, curve_eval(fp.vol_curve, fp.vol_n, fp.vol_len, s.reverb_volume));
      p.reserved = 0;
      if (s.muffle_strength > 0.0f) {
        float mc = curve_eval(fp.muf_curve, fp.muf_n, fp.muf_len, s.muffle_strength);
        float cutoff = ulerp(fp.mc_max, fp.mc_min, mc);
        float rc = 1.0f / (cutoff * DOUBLE_PI);
        float dt = 1.0f / (float)fp.sample_rate;
        p.muffle_cutoff = cutoff; p.muffle_alpha = dt / (rc + dt); p.muffle_active = 1;
      } else {
        p.muffle_cutoff = 0.0f; p.muffle_alpha = 0.0f; p.muffle_active = 0;
      }
      dp[t] = p;
    }
  }
  if (host_out) {  // the fan's record into the pinned host staging (16-B aligned sections and stride)
    __syncthreads();  // (this wave's settings, DSP and muffle stores above come first)
    const uint4* src = reinterpret_cast<const uint4*>(fb);
    uint4* dst = reinterpret_cast<uint4*>(host_out + (size_t)fan * L.stride);
    for (uint32_t i = (uint32_t)lane; i < L.stride / 16u; i += 64u) dst[i] = src[i];
  }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
void launch_prep(const art_sphere* sph, int ns, const art_aabb* aabb, int na, const art_obb* obb, int no,
                 SphereRec* osph, SphereCold* osphc, AabbRec* oaabb, AabbCold* oaabbc, ObbRec* oobb, ObbCold* oobbc,
                 CullRec* cull, hipStream_t st) {
  int n = ns + na + no;
  if (n == 0) return;
  hipLaunchKernelGGL(prep_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sph, ns, aabb, na, obb, no, osph, osphc, oaabb,
                     oaabbc, oobb, oobbc, cull);
}

// FibonacciDirectionsJobParallel.Execute (Jobs/FibonacciDirectionsJobParallel.cs:15-35), one lane
// per ray. The float operations are the reference's (and art_fibonacci_directions' on the host);
// cos/sin are evaluated in double and rounded to float, which gives the correctly rounded float
// values that the host libm's cosf/sinf return on these arguments (tests/test_dirs_gpu.py).
__global__ void fibonacci_kernel(int count, art_half3* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const float phi = 3.14159265f * (3.0f - sqrtf(5.0f));
  const float y = 1.0f - ((float)i / (float)(count - 1)) * 2.0f;
  const float radius = sqrtf(1.0f - y * y);
  const float theta = phi * (float)i;
  const float x = (float)cos((double)theta) * radius;
  const float z = (float)sin((double)theta) * radius;
  // count == 1 divides 0 by 0. The reference runs on x86, whose default NaN has the sign bit set
  // (half 0xFE00, as the host generator produces); the GPU's is positive, so NaNs are canonicalized.
  auto h16 = [](float v) -> uint16_t { return v != v ? (uint16_t)0xFE00u : f32tof16(v); };
  art_half3 h;
  h.x = h16(x); h.y = h16(y); h.z = h16(z);
  out[i] = h;
}

__global__ void half_range_kernel(uint32_t first, uint32_t count, uint16_t* __restrict__ out) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  out[i] = f32tof16(asfloat(first + (uint32_t)i));  // wraps past 0xFFFFFFFF
}

void launch_half_range(uint32_t first, uint32_t count, uint16_t* out, hipStream_t st) {
  if (count == 0) return;
  const unsigned blocks = (unsigned)(((unsigned long long)count + 255ull) / 256ull);  // no 32-bit wrap near 2^32
  hipLaunchKernelGGL(half_range_kernel, dim3(blocks), dim3(256), 0, st, first, count, out);
}

// The OBB slab's reciprocal (art_device_fns.hpp recip_exact, the product function itself) over a
// range of float bit patterns, for the exhaustive check against IEEE 1.0f / x
// (tests/test_recip_exhaustive.py).
__global__ void recip_range_kernel(uint32_t first, uint32_t count, uint32_t* __restrict__ out) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  out[i] = __float_as_uint(recip_exact(asfloat(first + (uint32_t)i)));  // wraps past 0xFFFFFFFF
}

void launch_recip_range(uint32_t first, uint32_t count, uint32_t* out, hipStream_t st) {
  if (count == 0) return;
  const unsigned blocks = (unsigned)(((unsigned long long)count + 255ull) / 256ull);
  hipLaunchKernelGGL(recip_range_kernel, dim3(blocks), dim3(256), 0, st, first, count, out);
}

void launch_fibonacci(int count, art_half3* out, hipStream_t st) {
  if (count <= 0) return;
  hipLaunchKernelGGL(fibonacci_kernel, dim3((count + 255) / 256), dim3(256), 0, st, count, out);
}

void launch_scatter_prep(const int* idx_s, const art_sphere* rec_s, int ds, const int* idx_a, const art_aabb* rec_a,
                         int da, const int* idx_o, const art_obb* rec_o, int dob, art_sphere* sph, art_aabb* aabb,
                         art_obb* obb, int ns, int na, SphereRec* osph, SphereCold* osphc, AabbRec* oaabb,
                         AabbCold* oaabbc, ObbRec* oobb, ObbCold* oobbc, CullRec* cull, hipStream_t st) {
  const int n = ds + da + dob;
  if (n <= 0) return;
  hipLaunchKernelGGL(scatter_prep_kernel, dim3((n + 255) / 256), dim3(256), 0, st, idx_s, rec_s, ds, idx_a, rec_a, da,
                     idx_o, rec_o, dob, sph, aabb, obb, ns, na, osph, osphc, oaabb, oaabbc, oobb, oobbc, cull);
}

void launch_raytrace(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins, uint8_t* block,
                     uint32_t* muffle_acc, DevCounts* counts, hipStream_t st) {
  if (fp.S == 0) return;
  // Balance the per-fan ray range over ceil(R/256) blocks, rounded to whole waves.
  int nblk = (fp.R + kRtBlock - 1) / kRtBlock;
  int per = (fp.R + nblk - 1) / nblk;
  int threads = ((per + 63) / 64) * 64;
  nblk = (fp.R + threads - 1) / threads;
  dim3 grid(nblk, fp.S), blk(threads);
  if (counts) {
    if (L.has_hits) hipLaunchKernelGGL((raytrace_kernel<true, true>), grid, blk, 0, st, sc, fp, L, origins, block, muffle_acc, counts);
    else hipLaunchKernelGGL((raytrace_kernel<true, false>), grid, blk, 0, st, sc, fp, L, origins, block, muffle_acc, counts);
  } else {
    if (L.has_hits) hipLaunchKernelGGL((raytrace_kernel<false, true>), grid, blk, 0, st, sc, fp, L, origins, block, muffle_acc, counts);
    else hipLaunchKernelGGL((raytrace_kernel<false, false>), grid, blk, 0, st, sc, fp, L, origins, block, muffle_acc, counts);
  }
}

void launch_permeate_sweep(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins, uint8_t* block,
                           const int2* slot_batch, hipStream_t st) {
  if (fp.S == 0) return;
  hipLaunchKernelGGL(permeate_kernel, dim3(fp.TC, fp.S), dim3(kPermBlock), 0, st, sc, fp, L, origins, block, slot_batch);
}

void launch_perm_count(const DevScene& sc, const FrameParams& fp, const float* origins, DevCounts* counts,
                       unsigned long long* nhit, hipStream_t st) {
  if (fp.S == 0) return;
  hipLaunchKernelGGL(perm_count_kernel, dim3((fp.R + kPermBlock - 1) / kPermBlock, fp.S), dim3(kPermBlock), 0, st, sc, fp,
                     origins, counts, nhit);
}

void launch_reduce(const DevScene& sc, const FrameParams& fp, const FanLayout& L, uint8_t* block, const uint32_t* muffle_acc,
                   const uint8_t* muffle_reset, hipStream_t st, const float* perm_in, uint8_t* host_out) {
  if (fp.S == 0) return;
  hipLaunchKernelGGL(reduce_kernel, dim3(fp.S), dim3(64), 0, st, sc, fp, L, block, muffle_acc, muffle_reset, perm_in, host_out);
}

}  // namespace art
