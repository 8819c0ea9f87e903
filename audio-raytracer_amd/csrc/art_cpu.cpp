// art_cpu.cpp — the CPU backend of the C ABI (art_create with device_mask = 0).
//
// The reference's own execution model on the host: Unity's job system runs
// AudioRaytracerJobBatched / AudioPermeationJobBatched as IJobParallelForBatch over worker threads
// (Audio/AudioRayTracer.cs:191,213), then ProcessAudioDataJob (:237). Here a persistent pool of
// worker threads takes whole fans (one AudioRayTracer job graph each) from an atomic counter; inside
// a fan the batches run in order b = 0, 1, ... (the sequential-batch semantics the device path
// defines for TC > 1), each job in the reference's loop order: colliders in
// Sphere, AABB, OBB order, strict '<', early exits where the reference returns early. Colliders are
// decoded once per frame with the kernels' own decode (art_frame_math.hpp), and every test is the
// kernels' host+device arithmetic (art_device_fns.hpp) with Unity's exact min/max selects, so the
// CPU and GPU backends agree bit for bit by construction and the tests check both against the oracle.
// Test counts (ART_CTX_COUNT_TESTS) are the tests this loop order executes: the metric's numerator.
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "art_cpu.hpp"
#include "art_frame_math.hpp"

namespace art {
namespace {

struct Counts {
  uint64_t v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // art_test_counts order
};

// The decoded scene of one frame (host copy; the caller's arrays may change after art_schedule).
struct Scene {
  std::vector<SphereRec> sph;
  std::vector<SphereCold> sphc;
  std::vector<AabbRec> aabb;
  std::vector<AabbCold> aabbc;
  std::vector<ObbRec> obb;
  std::vector<ObbCold> obbc;
  std::vector<vec3> targets, dirs;
  std::vector<float> vol_curve, muf_curve;
};

struct Frame {
  int R = 0, H = 0, T = 0, TC = 0, bs = 0, nb = 0;
  uint32_t stages = 0;
  float max_life = 0, max_muffle = 0, muffle_eff = 0, perm_strength = 0, perm_eff = 0, max_reverb = 0;
  bool dsp = false;
  float dl_min = 0, dl_max = 0, db_min = 0, db_max = 0, mc_min = 0, mc_max = 0, vol_len = 0, muf_len = 0;
  int sample_rate = 0;
  bool count = false;
};

constexpr int kCpuNone = 0;

// ShootRayCast (AudioRaytracerJobBatched.cs:225-280; PERM: AudioPermeationJobBatched.cs:101-141,
// INFINITY sentinel and the inverted stored rotation :174): first minimum in Sphere, AABB, OBB order.
template <bool PERM>
bool shoot(const Scene& sc, const Seg& s, int& type, int& idx, float& dist, Counts* c) {
  float best = PERM ? __builtin_huge_valf() : FLT_MAX;
  type = kCpuNone;
  idx = -1;
  const int ns = (int)sc.sph.size(), na = (int)sc.aabb.size(), no = (int)sc.obb.size();
  for (int i = 0; i < ns; ++i) {
    float d;
    if (sphere_test(s, sc.sph[(size_t)i], d) && d < best) { best = d; type = kSphere; idx = i; }
  }
  for (int i = 0; i < na; ++i) {
    float d;
    if (aabb_test<true>(s, sc.aabb[(size_t)i], d) && d < best) { best = d; type = kAabb; idx = i; }
  }
  for (int i = 0; i < no; ++i) {
    float d;
    const quat q = PERM ? inverse_q(sc.obbc[(size_t)i]) : stored_q(sc.obb[(size_t)i]);
    if (obb_test<true>(s, sc.obb[(size_t)i], q, d) && d < best) { best = d; type = kObb; idx = i; }
  }
  if (c) {
    c->v[PERM ? 3 : 0] += (uint64_t)ns;
    c->v[PERM ? 4 : 1] += (uint64_t)na;
    c->v[PERM ? 5 : 2] += (uint64_t)no;
  }
  dist = best;
  if (PERM) return best != __builtin_huge_valf();  // :140
  return type != kCpuNone;                         // :279
}

// CanRaySeePoint :365-397 (owner = -1: no skip) / CanRaySeeAudioTarget :405-449 (skip owned).
bool can_see(const Scene& sc, const Seg& s, float maxd, int owner, Counts* c) {
  uint64_t n[3] = {0, 0, 0};
  bool clear = true;
  for (size_t i = 0; clear && i < sc.sph.size(); ++i) {
    if (owner >= 0 && sc.sph[i].tid == owner) continue;
    ++n[0];
    float d;
    if (sphere_test(s, sc.sph[i], d) && d < maxd) clear = false;
  }
  for (size_t i = 0; clear && i < sc.aabb.size(); ++i) {
    if (owner >= 0 && sc.aabb[i].tid == owner) continue;
    ++n[1];
    float d;
    if (aabb_test<true>(s, sc.aabb[i], d) && d < maxd) clear = false;
  }
  for (size_t i = 0; clear && i < sc.obb.size(); ++i) {
    if (owner >= 0 && sc.obb[i].tid == owner) continue;
    ++n[2];
    float d;
    if (obb_test<true>(s, sc.obb[i], stored_q(sc.obb[i]), d) && d < maxd) clear = false;
  }
  if (c) { c->v[0] += n[0]; c->v[1] += n[1]; c->v[2] += n[2]; }
  return clear;
}

float echo_mult(const Scene& sc, int type, int idx) {
  return type == kSphere ? sc.sphc[(size_t)idx].echo : (type == kAabb ? sc.aabbc[(size_t)idx].echo : sc.obbc[(size_t)idx].echo);
}

// ReflectRay :456-532 (Q5: the OBB normal goes through the inverse of the stored inverse rotation).
void reflect_ray(const Scene& sc, int type, int idx, float max_life, vec3& o, vec3& d, float& life) {
  vec3 n = mk3(0.0f, 0.0f, 0.0f);
  float absorption;
  if (type == kAabb) {
    const AabbCold& b = sc.aabbc[(size_t)idx];
    const vec3 lp = o - mk3(b.cx, b.cy, b.cz);
    const vec3 ap = abs3(lp);
    const float dx = b.hx - ap.x, dy = b.hy - ap.y, dz = b.hz - ap.z;
    if (dx < dy && dx < dz) n.x = usign(lp.x);
    else if (dy < dx && dy < dz) n.y = usign(lp.y);
    else n.z = usign(lp.z);
    absorption = b.absorption;
  } else if (type == kObb) {
    const ObbRec& b = sc.obb[(size_t)idx];
    const ObbCold& bc = sc.obbc[(size_t)idx];
    const vec3 lh = qmul(inverse_q(bc), o - mk3(b.cx, b.cy, b.cz));  // :489
    const vec3 ap = abs3(lh);
    const vec3 df = mk3(bc.hx, bc.hy, bc.hz) - ap;
    vec3 ln = mk3(0.0f, 0.0f, 0.0f);
    if (df.x < df.y && df.x < df.z) ln.x = usign(lh.x);
    else if (df.y < df.x && df.y < df.z) ln.y = usign(lh.y);
    else ln.z = usign(lh.z);
    n = qmul(stored_q(b), ln);  // :510
    absorption = bc.absorption;
  } else {
    const SphereRec& c = sc.sph[(size_t)idx];
    n = normalize(o - mk3(c.cx, c.cy, c.cz));  // :516
    absorption = sc.sphc[(size_t)idx].absorption;
  }
  d = reflect(d, n);                // :525
  o = o + d * kEps;                 // :528
  life -= max_life * absorption;    // :531
}

// AudioRaytracerJobBatched.Execute for rays [start, start + cnt) of one fan (:61-215).
void raytrace_batch(const Scene& sc, const Frame& f, const art_fan& fan, int start, int cnt, Counts* c) {
  const int H = f.H, T = f.T;
  const int batch_id = (int)((long long)start * f.TC / f.R);  // :63-64, batchCount = TC
  for (int i = 0; i < cnt * H; ++i) {  // :72-80 (Q1: start + i, not start * H + i)
    fan.echo_ray_distances[start + i] = 0;
    if (fan.ray_hit_points) fan.ray_hit_points[start + i] = art_half3{0, 0, 0};
    if (fan.ray_hit_ids) fan.ray_hit_ids[start + i] = ART_HIT_NONE;
  }
  for (int t = 0; t < T; ++t) fan.muffle_ray_hits[batch_id * T + t] = 0;  // :82-85
  const vec3 O = mk3(fan.origin[0], fan.origin[1], fan.origin[2]);
  for (int ray = start; ray < start + cnt; ++ray) {
    vec3 o = O, d = sc.dirs[(size_t)ray];
    float life = f.max_life;
    int hits = 0;
    for (;;) {  // :104
      int type, idx;
      float dist;
      const Seg s = make_seg(o, d);
      if (!shoot<false>(sc, s, type, idx, dist, c)) break;  // :200-207
      o = o + d * dist;  // :111
      life -= dist;      // :112
      hits += 1;         // :113
      const int rid = ray * H + hits - 1;
      art_half3 result;  // :118
      result.x = f32tof16(o.x); result.y = f32tof16(o.y); result.z = f32tof16(o.z);
      const vec3 off = o - d * kEps;  // :124, :158
      {  // echo :124-145
        const float dist0 = distance(O, o);
        if (can_see(sc, make_seg(off, normalize(O - off)), dist0, -1, c))
          fan.echo_ray_distances[rid] = f32tof16(dist0 * echo_mult(sc, type, idx));
      }
      for (int t = 0; t < T; ++t) {  // muffle :150-173
        const vec3 tp = sc.targets[(size_t)t];
        const float dt = distance(off, tp);
        if (dt < f.max_muffle && can_see(sc, make_seg(off, normalize(tp - off)), dt, t, c))
          fan.muffle_ray_hits[batch_id * T + t] = (uint16_t)(fan.muffle_ray_hits[batch_id * T + t] + 1);  // Q13 wrap
      }
      bool alive = true;
      if (hits >= H || life <= 0.0f) {  // :179-193
        alive = false;
      } else {
        reflect_ray(sc, type, idx, f.max_life, o, d, life);
        if (life < 0.0f) alive = false;
      }
      if (fan.ray_hit_points) fan.ray_hit_points[rid] = result;  // :197
      if (fan.ray_hit_ids) fan.ray_hit_ids[rid] = ART_HIT_ID(type, idx);
      if (!alive) break;
    }
    if (fan.ray_hit_counts) fan.ray_hit_counts[ray] = (uint8_t)hits;  // :204, :212
  }
}

// ShootPermeationRayCast :225-261: loss terms of every non-owned collider, summed in order.
float permeation_loss(const Scene& sc, const Seg& s, int t) {
  float loss = 0.0f;
  for (size_t i = 0; i < sc.sph.size(); ++i)
    if (sc.sph[i].tid != t) loss += perm_term_sphere(s, sc.sph[i], sc.sphc[i].density);
  for (size_t i = 0; i < sc.aabb.size(); ++i) {
    const AabbRec& r = sc.aabb[i];
    if (r.tid != t)
      loss += perm_term_slab(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.mnx, r.mny, r.mnz, r.mxx, r.mxy, r.mxz,
                             sc.aabbc[i].density);
  }
  for (size_t i = 0; i < sc.obb.size(); ++i) {
    const ObbRec& r = sc.obb[i];
    if (r.tid == t) continue;
    const quat q = stored_q(r);  // RayIntersectsOBBPermeation :294-300
    const vec3 lo = qmul(q, s.o - mk3(r.cx, r.cy, r.cz));
    const vec3 ld = qmul(q, s.d);
    loss += perm_term_slab(lo.x, lo.y, lo.z, 1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z, r.lmnx, r.lmny, r.lmnz, r.lmxx, r.lmxy,
                           r.lmxz, sc.obbc[i].density);
  }
  return loss;
}

// AudioPermeationJobBatched.Execute for rays [start, start + cnt) of one fan (:34-91).
void permeate_batch(const Scene& sc, const Frame& f, const art_fan& fan, int start, int cnt, Counts* c) {
  const int T = f.T;
  const int batch_count = (f.TC * T) / cnt / T;                         // :36 (Q7: usually 0)
  const int batch_id = (int)((long long)start * batch_count / f.R);     // :37
  float* ppr = fan.permeation_power_remains;
  for (int t = 0; t < T; ++t) ppr[batch_id * T + t] = 0.0f;             // :43-46
  const vec3 O = mk3(fan.origin[0], fan.origin[1], fan.origin[2]);
  uint64_t nonowned[3] = {0, 0, 0};
  if (c)
    for (int t = 0; t < T; ++t) {
      for (const SphereRec& r : sc.sph) nonowned[0] += r.tid != t;
      for (const AabbRec& r : sc.aabb) nonowned[1] += r.tid != t;
      for (const ObbRec& r : sc.obb) nonowned[2] += r.tid != t;
    }
  for (int ray = start; ray < start + cnt; ++ray) {
    const vec3 d = sc.dirs[(size_t)ray];
    int type, idx;
    float dist;
    if (!shoot<true>(sc, make_seg(O, d), type, idx, dist, c)) continue;  // :58
    const vec3 o = O + d * dist;
    for (int t = 0; t < T; ++t) {  // :67-86
      const vec3 off = o - d * kEps;
      const Seg s = make_seg(off, normalize(sc.targets[(size_t)t] - off));
      ppr[batch_id * T + t] = (float)f.R * f.perm_strength - permeation_loss(sc, s, t);  // :260, :85 (overwrite)
    }
    if (c) { c->v[6] += nonowned[0]; c->v[7] += nonowned[1]; c->v[8] += nonowned[2]; }
  }
}

float curve_at(const std::vector<float>& baked, float length, float time) {
  return curve_eval(baked.data(), (int)baked.size(), length, time);
}

// ProcessAudioDataJob.Execute :32-76 + AudioTargetRTSettings ctor + the DSP-parameter pass.
void reduce_fan(const Scene& sc, const Frame& f, const art_fan& fan) {
  const int T = f.T, n = f.R * f.H;
  float total = 0.0f, returned = 0.0f;
  for (int i = 0; i < n; ++i) {  // :40-48, in order (Q4: a zero counts as returned)
    const float e = f16tof32(fan.echo_ray_distances[i]);
    if (e == 0.0f) returned += 1.0f;
    else total += e;
  }
  const float reverb_strength = total / (float)n / f.max_reverb;  // :49-50
  const float reverb_volume = returned / (float)n;                 // :51
  for (int t = 0; t < T; ++t) {
    int hitsum = 0;
    float psum = 0.0f;
    for (int i = 0; i < f.TC; ++i) { hitsum += fan.muffle_ray_hits[T * i + t]; psum += fan.permeation_power_remains[T * i + t]; }
    float muffle = 1.0f - (float)hitsum / (float)(f.R * f.H) * f.muffle_eff;   // :68
    const float perm = psum / (float)f.R / f.perm_strength * f.perm_eff;       // :69
    muffle = usaturate(muffle - perm);                                          // :71
    art_target_settings s;
    s.muffle_strength = usaturate(muffle);
    s.reverb_strength = usaturate(reverb_strength);
    s.reverb_volume = usaturate(reverb_volume);
    s.perceived_position[0] = sc.targets[(size_t)t].x;
    s.perceived_position[1] = sc.targets[(size_t)t].y;
    s.perceived_position[2] = sc.targets[(size_t)t].z;
    fan.settings[t] = s;
    if (f.dsp && fan.dsp_params) {  // AudioSpatializer.cs:55-59, ReverbDSP.cs:12-13, MuffleDSP.cs:22-26,40-42
      const float DOUBLE_PI = 2.0f * 3.14159265f;
      art_dsp_params p;
      p.dry_level = ulerp(f.dl_min, f.dl_max, s.reverb_strength);
      p.dry_boost = ulerp(f.db_min, f.db_max, curve_at(sc.vol_curve, f.vol_len, s.reverb_volume));
      p.reserved = 0;
      if (s.muffle_strength > 0.0f) {
        const float cutoff = ulerp(f.mc_max, f.mc_min, curve_at(sc.muf_curve, f.muf_len, s.muffle_strength));
        const float rc = 1.0f / (cutoff * DOUBLE_PI);
        const float dt = 1.0f / (float)f.sample_rate;
        p.muffle_cutoff = cutoff; p.muffle_alpha = dt / (rc + dt); p.muffle_active = 1;
      } else {
        p.muffle_cutoff = 0.0f; p.muffle_alpha = 0.0f; p.muffle_active = 0;
      }
      fan.dsp_params[t] = p;
    }
  }
}

void run_fan(const Scene& sc, const Frame& f, const art_fan& fan, Counts* c) {
  for (int b = 0; b < f.nb; ++b) {
    const int start = b * f.bs, cnt = std::min(f.bs, f.R - start);
    if (f.stages & ART_STAGE_RAYTRACE) raytrace_batch(sc, f, fan, start, cnt, c);
    if (f.stages & ART_STAGE_PERMEATE) permeate_batch(sc, f, fan, start, cnt, c);
  }
  if (f.stages & ART_STAGE_REDUCE) reduce_fan(sc, f, fan);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Engine: persistent worker pool; one frame in flight.
// ------------------------------------------------------------------------------------------
struct CpuEngine {
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv_go, cv_done;
  uint64_t generation = 0;
  bool quit = false;
  int running = 0;  // workers still on the current frame
  std::atomic<int> next{0};
  Scene scene;
  Frame frame;
  std::vector<art_fan> fans;
  std::vector<Counts> counts;  // per worker
  std::atomic<bool> done{true};

  explicit CpuEngine(int threads) {
    counts.resize((size_t)threads);
    for (int w = 0; w < threads; ++w) workers.emplace_back([this, w] { loop(w); });
  }
  ~CpuEngine() {
    {
      std::lock_guard<std::mutex> g(mu);
      quit = true;
    }
    cv_go.notify_all();
    for (std::thread& t : workers) t.join();
  }
  void loop(int w) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu);
        cv_go.wait(g, [&] { return quit || generation != seen; });
        if (quit) return;
        seen = generation;
      }
      Counts* c = frame.count ? &counts[(size_t)w] : nullptr;
      for (;;) {
        const int i = next.fetch_add(1);
        if (i >= (int)fans.size()) break;
        run_fan(scene, frame, fans[(size_t)i], c);
      }
      std::lock_guard<std::mutex> g(mu);
      if (--running == 0) {
        done.store(true);
        cv_done.notify_all();
      }
    }
  }
};

CpuEngine* cpu_create(int threads) {
  if (threads <= 0) {
    threads = (int)std::thread::hardware_concurrency();
    if (const char* e = getenv("ART_CPU_THREADS")) threads = atoi(e);
  }
  return new (std::nothrow) CpuEngine(std::max(1, threads));
}

void cpu_destroy(CpuEngine* e) { delete e; }

int cpu_threads(const CpuEngine* e) { return (int)e->workers.size(); }

int cpu_schedule(CpuEngine* e, const art_frame_desc* d, const art_fan* fans, int fan_count, const CpuColliders* resident,
                 bool count) {
  if (!e->done.load()) return ART_E_STATE;
  Scene& sc = e->scene;
  const art_sphere* sph = resident ? resident->sph : d->sphere_colliders;
  const art_aabb* aabb = resident ? resident->aabb : d->aabb_colliders;
  const art_obb* obb = resident ? resident->obb : d->obb_colliders;
  const int ns = resident ? resident->ns : d->sphere_count, na = resident ? resident->na : d->aabb_count,
            no = resident ? resident->no : d->obb_count;
  // the decode of prep_kernel, on the host (inputs are copied before art_schedule returns)
  sc.sph.resize((size_t)ns); sc.sphc.resize((size_t)ns);
  sc.aabb.resize((size_t)na); sc.aabbc.resize((size_t)na);
  sc.obb.resize((size_t)no); sc.obbc.resize((size_t)no);
  std::vector<CullRec> cull((size_t)(ns + na + no) + 1);
  for (int i = 0; i < ns; ++i) prep_sphere(sph[i], i, i, sc.sph.data(), sc.sphc.data(), cull.data());
  for (int i = 0; i < na; ++i) prep_aabb(aabb[i], i, ns + i, sc.aabb.data(), sc.aabbc.data(), cull.data());
  for (int i = 0; i < no; ++i) prep_obb(obb[i], i, ns + na + i, sc.obb.data(), sc.obbc.data(), cull.data());
  const int R = d->ray_count, T = d->audio_target_count;
  sc.dirs.resize((size_t)R);
  for (int i = 0; i < R; ++i) {
    const art_half3 h = d->ray_directions[i];
    sc.dirs[(size_t)i] = mk3(f16tof32(h.x), f16tof32(h.y), f16tof32(h.z));
  }
  sc.targets.resize((size_t)T);
  for (int t = 0; t < T; ++t)
    sc.targets[(size_t)t] = mk3(d->audio_target_positions[3 * t], d->audio_target_positions[3 * t + 1],
                                d->audio_target_positions[3 * t + 2]);
  Frame& f = e->frame;
  f = Frame();
  f.R = R; f.H = d->max_hits_per_ray; f.T = T; f.TC = d->batch_slots; f.bs = d->batch_size;
  f.nb = (R + f.bs - 1) / f.bs;
  f.stages = d->stages;
  f.max_life = d->max_ray_life; f.max_muffle = d->max_muffle_hit_distance; f.muffle_eff = d->muffle_effectiveness;
  f.perm_strength = d->permeation_strength_per_ray; f.perm_eff = d->permeation_effectiveness;
  f.max_reverb = d->max_reverb_distance;
  f.count = count;
  f.dsp = (d->stages & ART_STAGE_DSP_PARAMS) && d->dsp;
  if (f.dsp) {
    const art_dsp_desc* q = d->dsp;
    f.dl_min = q->reverb_dry_level_min; f.dl_max = q->reverb_dry_level_max;
    f.db_min = q->reverb_dry_boost_min; f.db_max = q->reverb_dry_boost_max;
    f.mc_min = q->muffle_cutoff_min; f.mc_max = q->muffle_cutoff_max;
    f.vol_len = q->reverb_volume_curve.length; f.muf_len = q->muffle_curve.length;
    f.sample_rate = q->sample_rate;
    sc.vol_curve.assign(q->reverb_volume_curve.baked, q->reverb_volume_curve.baked + q->reverb_volume_curve.sample_count);
    sc.muf_curve.assign(q->muffle_curve.baked, q->muffle_curve.baked + q->muffle_curve.sample_count);
  }
  e->fans.assign(fans, fans + fan_count);
  for (Counts& c : e->counts) c = Counts();
  {
    std::lock_guard<std::mutex> g(e->mu);
    e->next.store(0);
    e->done.store(false);
    e->running = (int)e->workers.size();
    ++e->generation;
  }
  e->cv_go.notify_all();
  return ART_OK;
}

bool cpu_is_completed(CpuEngine* e) { return e->done.load(); }

void cpu_complete(CpuEngine* e, art_test_counts* out) {
  std::unique_lock<std::mutex> g(e->mu);
  e->cv_done.wait(g, [&] { return e->done.load(); });
  if (out) {
    uint64_t v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (const Counts& c : e->counts)
      for (int k = 0; k < 9; ++k) v[k] += c.v[k];
    out->rt_sphere = v[0]; out->rt_aabb = v[1]; out->rt_obb = v[2];
    out->perm_hit_sphere = v[3]; out->perm_hit_aabb = v[4]; out->perm_hit_obb = v[5];
    out->perm_loss_sphere = v[6]; out->perm_loss_aabb = v[7]; out->perm_loss_obb = v[8];
  }
}

}  // namespace art
