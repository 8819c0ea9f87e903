// art_wavefront.hip — the throughput raytrace path (AudioRaytracerJobBatched.Execute,
// Jobs/AudioRaytracerJobBatched.cs:61-215) as a per-bounce wavefront pipeline.
//
// Per bounce b (the reference's `while (isRayAlive)` loop, :104-208):
//   wf_nearest     ShootRayCast (:108, :225-280) for every live ray. K waves share a group of 64
//                  rays and each sweeps 1/K of every collider array (wave-uniform SMEM records);
//                  the K partial first-minima are merged in LDS by (distance, reference order).
//                  A hit appends the ray's visibility items — the echo ray (:124-145) and every
//                  muffle ray within MaxMuffleHitDistance (:150-173) — to a global item list.
//   wf_visibility  launched once per collider range p = 0..P-1: a persistent grid drains the
//                  list of items not yet blocked through a chip-wide atomic queue. Each wave
//                  rotates through the range's collider chunks in lockstep; a lane holds one item
//                  and leaves when it is blocked (flag byte set) or has seen the whole range
//                  (item forwarded to the next range's list). Any-hit is an OR over colliders,
//                  so testing ranges in sequence gives the reference's verdict, while short
//                  ranges keep the persistent queue balanced and blocked items stop early.
//   wf_finalize    echo write (:142-144), muffle counts (:171), termination and ReflectRay
//                  (:179-193, :456-532); live rays form the next bounce's list.
// Every value is computed with the same arithmetic as the reference-order kernel, so outputs
// are bit-identical to it (and to the oracle); only the schedule differs.
#include "art_device_fns.hpp"
#include "art_wavefront.hpp"

namespace art {

constexpr int kWfU = 4;  // sweep unroll
constexpr int kNoHitCode = 0x7fffffff;
constexpr int kNoOwnerId = 0x7fffffff;  // echo rays skip no collider (AudioTargetId is 16-bit)

__device__ __forceinline__ void wf_chunk_of(int n, int w, int K, int& b, int& e) {
  b = (int)(((long long)n * w) / K);
  e = (int)(((long long)n * (w + 1)) / K);
}

// Sphere test with the square root and the two IEEE divisions only on lanes whose discriminant
// is non-negative (same arithmetic as sphere_test).
__device__ __forceinline__ bool wf_sphere(const Seg& s, const SphereRec& c, float& dist) {
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

// First minimum over this wave's share of the colliders. code = rank << 28 | index with
// rank 0 sphere, 1 AABB, 2 OBB: the reference's global order (Sphere, AABB, OBB loops).
__device__ __forceinline__ void wf_nearest_part(const DevScene& sc, const Seg& s, int w, int K, float& best,
                                                int& code) {
  best = FLT_MAX;
  code = kNoHitCode;
  int b, e;
  wf_chunk_of(sc.ns, w, K, b, e);
  int i = b;
  for (; i + kWfU <= e; i += kWfU) {
    SphereRec c[kWfU];
#pragma unroll
    for (int u = 0; u < kWfU; ++u) c[u] = ldc(sc.sph, wave_uniform(i + u));
#pragma unroll
    for (int u = 0; u < kWfU; ++u) {
      float d;
      if (wf_sphere(s, c[u], d) && d < best) { best = d; code = i + u; }
    }
  }
  for (; i < e; ++i) {
    float d;
    if (wf_sphere(s, ldc(sc.sph, wave_uniform(i)), d) && d < best) { best = d; code = i; }
  }
  wf_chunk_of(sc.na, w, K, b, e);
  i = b;
  for (; i + kWfU <= e; i += kWfU) {
    AabbRec r[kWfU];
#pragma unroll
    for (int u = 0; u < kWfU; ++u) r[u] = ldc(sc.aabb, wave_uniform(i + u));
#pragma unroll
    for (int u = 0; u < kWfU; ++u) {
      float d;
      if (aabb_test<false>(s, r[u], d) && d < best) { best = d; code = (1 << 28) | (i + u); }
    }
  }
  for (; i < e; ++i) {
    float d;
    if (aabb_test<false>(s, ldc(sc.aabb, wave_uniform(i)), d) && d < best) { best = d; code = (1 << 28) | i; }
  }
  wf_chunk_of(sc.no, w, K, b, e);
  for (i = b; i < e; ++i) {
    const ObbRec r = ldc(sc.obb, wave_uniform(i));
    float d;
    if (obb_test<false>(s, r, stored_q(r), d) && d < best) { best = d; code = (2 << 28) | i; }
  }
}

__device__ __forceinline__ int wf_type(int code) {
  const int rank = code >> 28;
  return rank == 0 ? kSphere : (rank == 1 ? kAabb : kObb);
}

__device__ __forceinline__ int wf_slot(const FrameParams& fp, int ray) {  // batchId (:63-64)
  return (int)(((long long)((ray / fp.bs) * fp.bs) * fp.TC) / fp.R);
}

// Ray ended (miss :200-207, or termination :179-193): RayHitResultCounts (:204, :212) and, at
// TC == 1, the reset value 0 in every slot past the last hit (:72-80).
template <bool HITS>
__device__ __forceinline__ void wf_end_ray(const FrameParams& fp, const FanLayout& L, uint8_t* fb, int ray, int hits) {
  if (fp.TC == 1) {
    uint16_t* echo = reinterpret_cast<uint16_t*>(fb + L.echo_off);
    art_half3* hpo = reinterpret_cast<art_half3*>(fb + L.hit_points_off);
    const art_half3 z = {0, 0, 0};
    for (int k = hits; k < fp.H; ++k) {
      echo[ray * fp.H + k] = 0;
      if (HITS) hpo[ray * fp.H + k] = z;
    }
  }
  if (HITS) fb[L.hit_counts_off + ray] = (uint8_t)hits;
}

// ------------------------------------------------------------------------------------------
// wf_nearest — one block = K waves x 64 rays of the bounce's live list.
// ------------------------------------------------------------------------------------------
template <int K, bool HITS>
__global__ __launch_bounds__(64 * K) void wf_nearest(DevScene sc, FrameParams fp, FanLayout L, WfArgs a, int bounce) {
  __shared__ float s_dist[K][64];
  __shared__ int s_code[K][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t n = bounce == 0 ? (uint32_t)(fp.S * fp.R) : a.cnt[bounce].alive_n;
  const uint32_t i0 = blockIdx.x * 64u;
  if (i0 >= n) return;  // uniform per block
  const uint32_t i = i0 + lane;
  const bool valid = i < n;
  const int Q = fp.T + 1;

  int g = 0, fan = 0, ray = 0;
  WfRay st;
  if (bounce == 0) {
    const uint32_t ii = valid ? i : 0u;
    fan = (int)(ii / (uint32_t)fp.R);
    ray = a.ray_order[ii % (uint32_t)fp.R];
    g = fan * fp.R + ray;
    const vec3 O = load3(a.origins, fan);
    const vec3 d = load_dir(sc.dirs, ray);
    st.ox = O.x; st.oy = O.y; st.oz = O.z; st.life = fp.max_life;
    st.dx = d.x; st.dy = d.y; st.dz = d.z; st.dist = 0.0f;
    st.code = kNoHitCode; st.hits = 0; st.active = 0u; st.frozen = 0u;
    // Reset (:72-80) under sequential-batch semantics; at TC == 1 nothing is frozen and the
    // slots are written exactly once later.
    if (valid) {
      uint8_t* fb = a.block + (size_t)fan * L.stride;
      uint16_t* echo = reinterpret_cast<uint16_t*>(fb + L.echo_off);
      art_half3* hpo = reinterpret_cast<art_half3*>(fb + L.hit_points_off);
      const int my_batch = ray / fp.bs;
      const art_half3 z = {0, 0, 0};
      for (int k = 0; k < fp.H; ++k) {
        const int j = ray * fp.H + k;
        bool any_reset;
        const int keep = batch_slot_state(fp, j, my_batch, any_reset);
        if (!keep) st.frozen |= 1u << k;
        if (w == 0 && fp.TC != 1 && (!keep || any_reset)) {
          echo[j] = 0;
          if (HITS) hpo[j] = z;
        }
      }
    }
  } else {
    g = valid ? (int)a.alive_in[i] : 0;
    fan = g / fp.R;
    ray = g - fan * fp.R;
    st = a.rays[g];
  }

  vec3 o = mk3(st.ox, st.oy, st.oz), d = mk3(st.dx, st.dy, st.dz);
  const Seg s = make_seg(o, d);
  float best;
  int code;
  wf_nearest_part(sc, s, w, K, best, code);
  s_dist[w][lane] = best;
  s_code[w][lane] = code;
  __syncthreads();
  float bd = s_dist[0][lane];
  int bc = s_code[0][lane];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    const float dk = s_dist[k][lane];
    const int ck = s_code[k][lane];
    if (dk < bd || (dk == bd && ck < bc)) { bd = dk; bc = ck; }
  }
  if (w != 0) return;  // wave 0 owns the per-ray updates; all its lanes stay for the scan below

  uint32_t active = 0u;
  if (valid) {
    uint8_t* fb = a.block + (size_t)fan * L.stride;
    const bool hit = bc != kNoHitCode;
    if (hit) {
      const int type = wf_type(bc), idx = bc & 0x0fffffff;
      float dist = bd;  // exact (Unity min/max) re-evaluation: a zero distance keeps the reference sign
      if (type == kAabb) aabb_test<true>(s, sc.aabb[idx], dist);
      if (type == kObb) { const ObbRec r = sc.obb[idx]; obb_test<true>(s, r, stored_q(r), dist); }
      o = o + d * dist;      // :111
      st.life -= dist;       // :112
      st.hits += 1;          // :113
      const int k = st.hits - 1;
      if (HITS && !((st.frozen >> k) & 1u)) {  // :118, :197
        art_half3 p;
        p.x = f32tof16(o.x); p.y = f32tof16(o.y); p.z = f32tof16(o.z);
        reinterpret_cast<art_half3*>(fb + L.hit_points_off)[ray * fp.H + k] = p;
      }
      const vec3 off = o - d * kEps;
      active = 1u;  // echo ray (:133)
      for (int t = 0; t < fp.T; ++t)
        if (distance(off, load3(sc.targets, t)) < fp.max_muffle) active |= 2u << t;  // :165-168
      st.ox = o.x; st.oy = o.y; st.oz = o.z;
      st.dist = dist;
      st.code = bc;
    } else {
      st.code = kNoHitCode;
      wf_end_ray<HITS>(fp, L, fb, ray, st.hits);
    }
    st.active = active;
    a.rays[g] = st;
  }

  // append this wave's visibility items query-major (all echo items of the 64 coherent rays, then
  // all items of target 0, ...) as ready-to-sweep segments
  const unsigned long long lt = (1ull << lane) - 1ull;
  int count = 0;
  for (int q = 0; q < Q; ++q) count += __popcll(__ballot((active >> q) & 1u));
  uint32_t base = 0;
  if (lane == 0 && count > 0) base = atomicAdd(&a.cnt[bounce].items_n[0], (uint32_t)count);
  base = __shfl(base, 0, 64);
  const vec3 off = o - d * kEps;  // :124, :158 (o is the hit point)
  for (int q = 0; q < Q; ++q) {
    const bool act = (active >> q) & 1u;
    const unsigned long long m = __ballot(act);
    if (act) {
      vec3 qdir;
      WfItem it;
      if (q == 0) {
        const vec3 O = load3(a.origins, fan);
        qdir = normalize(O - off);                    // :127
        it.maxd = distance(O, o);                     // :130 (un-offset hit point)
        it.owner = kNoOwnerId;
      } else {
        const vec3 tp = load3(sc.targets, q - 1);
        qdir = normalize(tp - off);                   // :162
        it.maxd = distance(off, tp);                  // :165
        it.owner = q - 1;                             // :413, :426, :439
      }
      const Seg g2 = make_seg(off, qdir);
      it.ox = g2.o.x; it.oy = g2.o.y; it.oz = g2.o.z; it.dx = g2.d.x; it.dy = g2.d.y; it.dz = g2.d.z;
      it.ix = g2.inv.x; it.iy = g2.inv.y; it.iz = g2.inv.z; it.a2 = g2.a2; it.a4 = g2.a4;
      it.id = (uint32_t)g * (uint32_t)Q + (uint32_t)q;
      it.pad0 = it.pad1 = 0u;
      a.items[base + (uint32_t)__popcll(m & lt)] = it;
    }
    base += (uint32_t)__popcll(m);
  }
}

// ------------------------------------------------------------------------------------------
// wf_visibility — persistent grid draining the bounce's item list.
// ------------------------------------------------------------------------------------------
struct WfRange {
  int c0, c1;      // chunk range [c0, c1) in the global chunk order
  int cs, ca;      // chunk counts of the sphere and AABB sections (OBB chunks follow)
};

template <typename Rec, typename Test>
__device__ __forceinline__ bool wf_sweep_records(const Rec* recs, int b, int e, bool blocked, bool done, Test test) {
  int i = b;
  for (; i + kWfU <= e; i += kWfU) {
    Rec r[kWfU];
#pragma unroll
    for (int u = 0; u < kWfU; ++u) r[u] = ldc(recs, wave_uniform(i + u));
#pragma unroll
    for (int u = 0; u < kWfU; ++u) blocked |= test(r[u]);
#ifdef ART_WF_INCHUNK_EXIT
    if (__all(blocked || done)) return blocked;
#endif
  }
  for (; i < e; ++i) blocked |= test(ldc(recs, wave_uniform(i)));
  return blocked;
}

__device__ __forceinline__ bool wf_sweep_chunk(const DevScene& sc, const WfRange& rg, int c, const Seg& s, float maxd,
                                               int owner, bool blocked, bool done) {
  if (c < rg.cs) {
    const int b = c * kWfChunk, e = min(b + kWfChunk, sc.ns);
    return wf_sweep_records(sc.sph, b, e, blocked, done, [&](const SphereRec& r) {
      float d;
      return wf_sphere(s, r, d) && d < maxd && r.tid != owner;
    });
  }
  c -= rg.cs;
  if (c < rg.ca) {
    const int b = c * kWfChunk, e = min(b + kWfChunk, sc.na);
    return wf_sweep_records(sc.aabb, b, e, blocked, done, [&](const AabbRec& r) {
      float d;
      return aabb_test<false>(s, r, d) && d < maxd && r.tid != owner;
    });
  }
  c -= rg.ca;
  const int b = c * kWfChunk, e = min(b + kWfChunk, sc.no);
  for (int i = b; i < e; ++i) {
    const ObbRec r = ldc(sc.obb, wave_uniform(i));
    float d;
    blocked |= obb_test<false>(s, r, stored_q(r), d) && d < maxd && r.tid != owner;
    if ((i & 3) == 3 && __all(blocked || done)) return blocked;
  }
  return blocked;
}

__global__ __launch_bounds__(256) void wf_visibility(DevScene sc, FrameParams fp, WfArgs a, int bounce, int part,
                                                     int nparts, WfRange rg) {
  (void)part; (void)nparts;
  const int lane = threadIdx.x & 63;
  const uint32_t n = a.cnt[bounce].items_n[0];
  if (n == 0) return;
  uint32_t* head = &a.cnt[bounce].head[0];
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const unsigned long long lt = (1ull << lane) - 1ull;

  const int nch = rg.c1 - rg.c0;
  int c = rg.c0;
  int left = 0;               // chunks this lane's item still has to see
  uint32_t qlo = 0, qhi = 0;  // this wave's claimed item range (wave-uniform)
  uint32_t item = 0;
  bool busy = false, blocked = false, drained = false;
  Seg s;
  float maxd = 0.0f;
  int owner = kNoOwnerId;
  while (true) {
    // refill free lanes from the wave's range; claim a new range (guided size) when it runs out
    unsigned long long need = __ballot(!busy);
    while (need && !drained) {
      if (qlo >= qhi) {
        uint32_t base = 0, size = 0;
        if (lane == 0) {
          const uint32_t h = __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t rem = h < n ? n - h : 0u;
          size = rem / (4u * nwaves);
          size = size < 64u ? 64u : (size > 2048u ? 2048u : size);
          base = atomicAdd(head, size);
        }
        base = __shfl(base, 0, 64);
        size = __shfl(size, 0, 64);
        if (base >= n) { drained = true; break; }
        qlo = base;
        qhi = min(base + size, n);
      }
      const uint32_t k = (uint32_t)__popcll(need);
      const uint32_t take = min(k, qhi - qlo);
      const uint32_t r = (uint32_t)__popcll(need & lt);
      if (!busy && r < take) {
        const WfItem it = a.items[qlo + r];
        s.o = mk3(it.ox, it.oy, it.oz); s.d = mk3(it.dx, it.dy, it.dz); s.inv = mk3(it.ix, it.iy, it.iz);
        s.a2 = it.a2; s.a4 = it.a4;
        maxd = it.maxd; owner = it.owner; item = it.id;
        busy = true;
        blocked = false;
        left = nch;
      }
      qlo += take;
      need = __ballot(!busy);
    }
    if (__all(!busy)) break;
    blocked = wf_sweep_chunk(sc, rg, c, s, maxd, owner, blocked, !busy);
    if (busy) {
      left -= 1;
      if (blocked) {
        a.flags[item] = 1;  // finalize reads it; an item that saw every chunk unblocked stays 0
        busy = false;
      } else if (left == 0) {
        busy = false;
      }
    }
    c = (c + 1 == rg.c1) ? rg.c0 : c + 1;
  }
}

// ------------------------------------------------------------------------------------------
// wf_finalize — echo, muffle, termination / reflection for the rays of this bounce.
// ------------------------------------------------------------------------------------------
template <bool HITS>
__global__ __launch_bounds__(256) void wf_finalize(DevScene sc, FrameParams fp, FanLayout L, WfArgs a, int bounce) {
  const uint32_t n = bounce == 0 ? (uint32_t)(fp.S * fp.R) : a.cnt[bounce].alive_n;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int Q = fp.T + 1, T = fp.T;
  bool live = false;
  int g = 0, fan = -1, ray = 0;
  if (i < n) {
    if (bounce == 0) {
      fan = (int)(i / (uint32_t)fp.R);
      ray = a.ray_order[i % (uint32_t)fp.R];
      g = fan * fp.R + ray;
    } else {
      g = (int)a.alive_in[i];
      fan = g / fp.R;
      ray = g - fan * fp.R;
    }
  }
  WfRay st;
  st.code = kNoHitCode;
  if (i < n) st = a.rays[g];
  const bool hit = i < n && st.code != kNoHitCode;
  uint32_t clear = 0u;
  if (hit) {
    uint8_t* fb = a.block + (size_t)fan * L.stride;
    uint8_t* fl = a.flags + (size_t)g * Q;
    const int k = st.hits - 1;
    const bool live_slot = !((st.frozen >> k) & 1u);
    const vec3 O = load3(a.origins, fan);
    const vec3 o = mk3(st.ox, st.oy, st.oz);
    vec3 d = mk3(st.dx, st.dy, st.dz);
    const int type = wf_type(st.code), idx = st.code & 0x0fffffff;
    uint16_t* echo = reinterpret_cast<uint16_t*>(fb + L.echo_off);
    if (live_slot) {
      if (!fl[0]) {
        const float em = type == kSphere ? sc.sphc[idx].echo : (type == kAabb ? sc.aabbc[idx].echo : sc.obbc[idx].echo);
        echo[ray * fp.H + k] = f32tof16(distance(O, o) * em);  // :130, :142-144
      } else if (fp.TC == 1) {
        echo[ray * fp.H + k] = 0;  // reset value (:76), written once
      }
    }
    for (int q = 0; q < Q; ++q) {
      if (((st.active >> q) & 1u) && !fl[q]) clear |= 1u << q;
      fl[q] = 0;  // flags start the next bounce cleared
    }
    clear &= ~1u;
    // termination / reflection — :179-193, ReflectRay :456-532
    float life = st.life;
    vec3 oo = o;
    live = true;
    if (st.hits >= fp.H || life <= 0.0f) {
      live = false;
    } else {
      vec3 nrm = mk3(0.0f, 0.0f, 0.0f);
      float absorption = 0.0f;
      if (type == kAabb) {
        const AabbCold b = sc.aabbc[idx];
        vec3 lp = o - mk3(b.cx, b.cy, b.cz);
        vec3 ap = abs3(lp);
        float dx = b.hx - ap.x, dy = b.hy - ap.y, dz = b.hz - ap.z;
        if (dx < dy && dx < dz) nrm.x = usign(lp.x);
        else if (dy < dx && dy < dz) nrm.y = usign(lp.y);
        else nrm.z = usign(lp.z);
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
        nrm = qmul(stored_q(b), ln);
        absorption = bc.absorption;
      } else {
        const SphereRec c = sc.sph[idx];
        nrm = normalize(o - mk3(c.cx, c.cy, c.cz));
        absorption = sc.sphc[idx].absorption;
      }
      d = reflect(d, nrm);
      oo = o + d * kEps;
      life -= fp.max_life * absorption;
      if (life < 0.0f) live = false;
    }
    if (live) {
      st.ox = oo.x; st.oy = oo.y; st.oz = oo.z; st.dx = d.x; st.dy = d.y; st.dz = d.z; st.life = life;
      a.rays[g] = st;
    } else {
      wf_end_ray<HITS>(fp, L, fb, ray, st.hits);
    }
  }
  // muffle counts (:171): one atomic per (wave, target) when the wave's rays share a fan and a slot
  const unsigned long long hm = __ballot(hit);
  const int src = hm ? (int)__builtin_ctzll(hm) : 0;
  const int fan0 = __shfl(fan, src, 64);
  const int slot = hit ? (fp.TC == 1 ? 0 : wf_slot(fp, ray)) : 0;
  const int slot0 = __shfl(slot, src, 64);
  const bool uniform = __all(!hit || (fan == fan0 && slot == slot0));
  for (int t = 0; t < T; ++t) {
    const bool c = (clear >> (t + 1)) & 1u;
    if (uniform) {
      const unsigned long long m = __ballot(c);
      if (m && lane == 0) atomicAdd(&a.muffle_acc[((size_t)fan0 * fp.TC + slot0) * T + t], (uint32_t)__popcll(m));
    } else if (c) {
      atomicAdd(&a.muffle_acc[((size_t)fan * fp.TC + slot) * T + t], 1u);
    }
  }
  // next bounce's live list
  const unsigned long long lm = __ballot(live);
  if (lm) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&a.cnt[bounce + 1].alive_n, (uint32_t)__popcll(lm));
    base = __shfl(base, 0, 64);
    if (live) a.alive_out[base + (uint32_t)__popcll(lm & lt)] = (uint32_t)g;
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
int wf_split(int rays) {
  int K = 1;
  while (K < 8 && (long long)((rays + 63) / 64) * K < 256LL * 24) K *= 2;
  return K;
}

template <int K>
static void launch_nearest_k(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const WfArgs& a, int b,
                             hipStream_t st) {
  const int blocks = (fp.S * fp.R + 63) / 64;
  if (L.has_hits) hipLaunchKernelGGL((wf_nearest<K, true>), dim3(blocks), dim3(64 * K), 0, st, sc, fp, L, a, b);
  else hipLaunchKernelGGL((wf_nearest<K, false>), dim3(blocks), dim3(64 * K), 0, st, sc, fp, L, a, b);
}

int wf_persistent_blocks() {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 2048;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(wf_visibility), 256, 0) != hipSuccess ||
      per <= 0)
    per = 4;
  return cus * per;
}

void wf_launch_bounce(const DevScene& sc, const FrameParams& fp, const FanLayout& L, WfArgs a, int bounce, int nparts,
                      int persistent_blocks, hipStream_t st) {
  // ping-pong live lists: bounce b reads list b&1, writes list (b+1)&1
  a.alive_in = a.alive[bounce & 1];
  a.alive_out = a.alive[(bounce + 1) & 1];
  switch (wf_split(fp.S * fp.R)) {
    case 1: launch_nearest_k<1>(sc, fp, L, a, bounce, st); break;
    case 2: launch_nearest_k<2>(sc, fp, L, a, bounce, st); break;
    case 4: launch_nearest_k<4>(sc, fp, L, a, bounce, st); break;
    default: launch_nearest_k<8>(sc, fp, L, a, bounce, st); break;
  }
  const int cs = (sc.ns + kWfChunk - 1) / kWfChunk, ca = (sc.na + kWfChunk - 1) / kWfChunk,
            co = (sc.no + kWfChunk - 1) / kWfChunk;
  const int nch = cs + ca + co;
  (void)nparts;
  if (nch > 0) {  // with no collider nothing blocks: finalize reads zero flags
    WfRange rg;
    rg.c0 = 0;
    rg.c1 = nch;
    rg.cs = cs;
    rg.ca = ca;
    hipLaunchKernelGGL(wf_visibility, dim3(persistent_blocks), dim3(256), 0, st, sc, fp, a, bounce, 0, 1, rg);
  }
  const int fblocks = (fp.S * fp.R + 255) / 256;
  if (L.has_hits) hipLaunchKernelGGL((wf_finalize<true>), dim3(fblocks), dim3(256), 0, st, sc, fp, L, a, bounce);
  else hipLaunchKernelGGL((wf_finalize<false>), dim3(fblocks), dim3(256), 0, st, sc, fp, L, a, bounce);
}

}  // namespace art
