// art_capi.cpp — the C ABI (include/art.h, include/art_device.h) over the HIP kernels.
//
// Replaces the reference's per-frame job scheduling in Audio/AudioRayTracer.cs:161-237:
//   AudioRaytracerJobBatched.Schedule(rayCount, batchSize)           (:191)
//   + AudioPermeationJobBatched.Schedule(rayCount, batchSize)        (:213)
//   + ProcessAudioDataJob.Schedule(handleA), CombineDependencies     (:237)
//   -> art_schedule: H2D of the frame's inputs, prep + raytrace + permeate + reduce kernels on
//      one HIP stream per device, D2H of the packed per-fan result blocks; one event per device.
//   JobHandle.IsCompleted (:95) -> art_is_completed; JobHandle.Complete() (:97) -> art_complete.
// Fans are sharded contiguously over the context's devices (SURVEY.md §8 e); each device holds
// a full copy of the scene. There is no CPU backend: without a HIP device art_create fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/art.h"
#include "../../include/art_device.h"
#include "../../include/art_dsp.h"
#include "../../include/art_colliders.h"
#include "art_cpu.hpp"
#include "art_internal.hpp"
#include "unity_math.hpp"

#include <chrono>
#include <cmath>
#include <csignal>
#include <cstdlib>
#include <execinfo.h>

using namespace art;

// The ABI structs are byte-identical to the C# structs (App. C of SURVEY.md).
static_assert(sizeof(art_half3) == 6, "half3");
static_assert(sizeof(art_aabb) == 20, "ColliderAABBStruct");
static_assert(sizeof(art_obb) == 26, "ColliderOBBStruct");
static_assert(sizeof(art_sphere) == 16, "ColliderSphereStruct");
static_assert(sizeof(art_target_settings) == 24, "AudioTargetRTSettings");
static_assert(sizeof(art_dsp_params) == 24, "art_dsp_params");

namespace {

// ABI major.minor. A struct that grows is a major bump (a caller built against the older header
// would be written past its end). 2.0: art_fan.ray_hit_ids, art_fan_layout.hit_ids_off; 2.1:
// art_exec_counts.cell_entries / muffle_fallback; 2.2: art_exec_counts.bounce_rays; 2.3:
// art_exec_counts.by_kernel (grew from 208 to 328 B), art_kernel_times.nearest_* (32 to 48 B),
// art_debug_leaf_order, ART_CTX_GRAPH removed — a growth 2.3 should have made a major bump; 3.0:
// art_kernel_times per kernel family (kernel_ms / kernel_launches / kernel_marks_dropped, 80 B),
// ART_CTX_TIME_EACH_KERNEL.
constexpr uint32_t kAbiVersion = (3u << 16) | 1u;  // 3.1: ART_CTX_EVENT_EACH_LAUNCH, art_recip_exact_device

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
float art_f16tof32_host(uint16_t h) { return art::f16tof32(h); }

#ifndef ART_CELLS_BESIDE_BVH
#define ART_CELLS_BESIDE_BVH 1
#endif
constexpr bool kCellsBesideBvh = ART_CELLS_BESIDE_BVH != 0;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, std::max<size_t>(n, 256)) != hipSuccess) { p = nullptr; return false; }
    cap = std::max<size_t>(n, 256);
    return true;
  }
  void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    if (hipHostMalloc(&p, std::max<size_t>(n, 256), hipHostMallocDefault) != hipSuccess) { p = nullptr; return false; }
    cap = std::max<size_t>(n, 256);
    return true;
  }
  void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
};

// Scalars of one frame that the kernels need, plus the derived batch tables.
struct Frame {
  int R = 0, H = 0, T = 0, TC = 0, bs = 0, nb = 0;
  int ns = 0, na = 0, no = 0;
  uint32_t stages = 0;
  bool resident = false;               // colliders come from the resident store (art_colliders.h)
  FrameParams fp{};
  FanLayout L{};
  std::vector<int2> slot_batch;        // permeation: [TC] ray range of the last batch writing slot s
  std::vector<uint8_t> muffle_reset;   // raytrace: [TC] 1 if some batch resets slot s
  std::vector<int> ray_order;          // lane slot -> ray index (direction-coherent at TC == 1)
  std::vector<uint8_t> order_dirs;     // the half3 directions ray_order was computed from
  // input staging layout (bytes)
  size_t off_sph = 0, off_aabb = 0, off_obb = 0, off_tgt = 0, off_dirs = 0, off_vol = 0, off_muf = 0, off_tab = 0,
         off_reset = 0, off_order = 0, raw_bytes = 0;
  size_t soa_sph = 0, soa_aabb = 0, soa_obb = 0, soa_sphc = 0, soa_aabbc = 0, soa_obbc = 0, soa_cull = 0, soa_bytes = 0;
  size_t soa_box = 0, soa_keys = 0, soa_keys_s = 0, soa_vals = 0, soa_perm = 0, soa_temp = 0, sort_temp = 0;
  size_t soa_bvh = 0, soa_bvh_ref = 0, soa_bvh_pos = 0, soa_bvh_leaf = 0, soa_kd = 0;
  // muffle candidate lists (art_cells.hip)
  size_t soa_ccount = 0, soa_cstart = 0, soa_ccur = 0, soa_cfar = 0, soa_cok = 0, soa_ctemp = 0, soa_cent = 0, soa_cent_s = 0, soa_ckeys = 0, soa_ctot = 0, soa_cbox = 0, cells_temp = 0,
         soa_cgeo = 0;
  uint32_t cells_cap = 0;
};

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  DevBuf raw, soa, origins, block, acc, counts;
  DevBuf exec;  // executed-work counters (ART_CTX_COUNT_EXECUTED)
  DevBuf cones; // the cell cone table (art_cells.hip), uploaded once
  CellBufs cb{};  // muffle candidate list buffers of the current scene (upload_scene)
  DevBuf pairs; // global visibility pairs of the split raytrace path
  DevBuf dsp;   // per-sample DSP batch (art_dsp_process): samples, offsets, frames, params, states
  // resident collider store (art_colliders.h): AoS lists, decoded records + bounds, sync upload
  DevBuf st_raw, st_soa, st_upd;
  int st_cap[3] = {0, 0, 0};
  DevScene st_sc{};             // collider pointers of the store (counts = last sync)
  bool st_fresh = true;         // capacity (re)allocated: every record must be uploaded
  hipEvent_t st_done = nullptr; // recorded after the last sync's upload + decode (on st_stream)
  hipStream_t st_stream = nullptr;  // the stream the last sync ran on (dv.stream or a device-path launch stream)
  hipEvent_t st_epoch[2] = {nullptr, nullptr};  // after the last sync of an epoch of the update ring
  bool st_epoch_pending[2] = {false, false};
  hipEvent_t launch_done = nullptr;  // after the last art_launch_device frame (caller's stream)
  bool launch_pending = false;       // work on dv.stream waits for it before reusing the scene / buffers
  hipStream_t launch_stream = nullptr;  // the caller's stream of that frame
  bool launch_recorded = false;         // launch_done already recorded after that frame
  uint64_t exec_launches = 0;
  int fan_begin = 0, fan_count = 0;
  size_t in_off = 0;  // art_schedule: this shard's [origins | permeation slots] in the input staging
  DevScene sc{};
  SortBufs sb{};  // buffers of the spatially sorted scene copy (art_bvh.hip), set by upload_scene
  // resident scenes: the sorted copies / BVH in dv.soa were built for store generation sorted_gen
  // (~0: none) with these counts; later frames reuse them (refit when the store changed)
  uint64_t sorted_gen = ~0ull;
  const void* sorted_soa = nullptr;
  int sorted_n[3] = {-1, -1, -1};
  DevScene sorted_sc{};
  // host-API frames: the inputs of the last full upload (bytes, layout key, buffers) and the scene
  // built from them; a frame whose packed inputs are byte-identical skips the H2D copy, the record
  // decode and the BVH build (the Unity caller passes unchanged collider arrays every frame)
  std::vector<uint8_t> last_raw;
  int last_key[10] = {};
  const void* last_raw_p = nullptr;
  const void* last_soa_p = nullptr;
  bool raw_valid = false;
  DevScene last_sc{};
  bool bound = false;
  // side stream of the permeation job: it runs beside the raytrace stage (the reference schedules
  // the two jobs independently, AudioRayTracer.cs:191,213), joined before the reduce job (:237)
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  SideStream echo;  // the echo visibility beside the muffle kernel
  std::vector<hipEvent_t> ev_pool;  // timing events (start/stop pairs)
  std::vector<std::pair<int, size_t>> ev_used;  // (EvKind, pool index of start)
  int marks_dropped = 0;                          // per-kernel marks past the pairs (art_kernel_timing)
};

}  // namespace

struct art_ctx {
  std::vector<Device> devs;        // empty for the CPU backend
  art::CpuEngine* cpu = nullptr;   // art_create(0): the CPU backend (art_cpu.cpp)
  std::vector<uint8_t> cpu_recs[3];  // CPU backend: the resident store's records at the last sync
  std::string err;
  uint32_t flags = 0;
  HostBuf h_in, h_block;
  HostBuf h_dsp;                 // staging of art_dsp_process
  Frame fr;                      // frame of the bound scene / last schedule
  // in-flight frame
  bool inflight = false;
  art_handle handle = 0;
  uint64_t next_handle = 1;
  std::vector<art_fan> fans;
  bool counted = false;
  art_test_counts last_counts{};
  bool has_counts = false;
  std::vector<uint64_t> nonowned;  // per type (s, a, o): sum over targets of non-owned colliders
  // resident collider store: the NextBatch mirror per kind, dirty marks, the last sync's counts
  struct Kind {
    std::vector<uint8_t> recs;      // count * size bytes
    int count = 0;
    std::vector<uint8_t> dirty;     // per record
    std::vector<int> dirty_list;
  } kinds[3];
  int synced[3] = {0, 0, 0};
  bool store_synced = false;
  // the synced records the resident scene's muffle cell lists were built from (cell_still_valid)
  std::vector<uint8_t> cell_base[3];
  bool cell_base_ok = false;
  uint64_t sync_gen = 0;         // bumped by every art_colliders_sync that changed a record
  // audio_target_id of every synced record and their histogram (index = id + 32768), kept
  // incrementally from the dirty records (permeation loss test counts of counting frames)
  std::vector<int16_t> synced_tid[3];
  std::vector<int> tid_hist[3];
  art_collider_sync_stats last_sync{};
  // pinned update images of art_colliders_sync, a ring (sync s uses slot s % kUpdRing): a slot is
  // reused only after the previous epoch's syncs are done (one event per epoch, not per sync)
  static constexpr int kUpdRing = 8;
  HostBuf h_upd[kUpdRing];
  uint64_t upd_seq = 0;
  // Host phases of the Unity-facing frame (ART_HOST_TIMES=1 in the environment at art_create:
  // steady_clock marks in art_schedule / art_complete, means printed by art_destroy to stderr).
  struct HostPhases {
    bool on = false;
    uint64_t frames = 0;
    double us[8] = {};
  } hp;
};

namespace {
// phase names of art_ctx::HostPhases (in the order the frame runs them)
const char* const kHostPhase[8] = {"validate_frame", "pack_inputs", "stage_fans", "upload_scene", "enqueue_copies_kernels",
                                   "complete_wait", "unpack_outputs", "complete_other"};
struct PhaseClock {
  art_ctx::HostPhases* hp;
  std::chrono::steady_clock::time_point t;
  explicit PhaseClock(art_ctx::HostPhases* h) : hp(h && h->on ? h : nullptr) { if (hp) t = std::chrono::steady_clock::now(); }
  void mark(int phase) {
    if (!hp) return;
    const auto n = std::chrono::steady_clock::now();
    hp->us[phase] += std::chrono::duration<double, std::micro>(n - t).count();
    t = n;
  }
};
}  // namespace

namespace {

int fail(art_ctx* c, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(art_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIP_TRY(ctx, expr)                                                                          \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) return fail(ctx, ART_E_DEVICE, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

int validate_desc(art_ctx* c, const art_frame_desc* d) {
  if (!d) return fail(c, ART_E_INVALID, "desc is NULL");
  if (d->ray_count <= 0 || !d->ray_directions) return fail(c, ART_E_INVALID, "ray_count must be > 0 with directions");
  if (d->ray_count > (1 << 20)) return fail(c, ART_E_UNSUPPORTED, "ray_count > 2^20");
  if (d->audio_target_count <= 0 || !d->audio_target_positions)
    return fail(c, ART_E_INVALID, "audio_target_count must be > 0 (the reference skips frames without targets, AudioRayTracer.cs:95)");
  if (d->audio_target_count > kMaxTargets) return fail(c, ART_E_UNSUPPORTED, "audio_target_count > %d", kMaxTargets);
  if (d->max_hits_per_ray <= 0 || d->max_hits_per_ray > 32)
    return fail(c, ART_E_UNSUPPORTED, "max_hits_per_ray must be in [1, 32] (reference maxBounces <= 25, AudioRayTracer.cs:14)");
  if ((long long)d->ray_count * d->max_hits_per_ray > (1 << 24)) return fail(c, ART_E_UNSUPPORTED, "R*H > 2^24");
  if (d->batch_size <= 0 || d->batch_slots <= 0) return fail(c, ART_E_INVALID, "batch_size and batch_slots must be > 0");
  if (d->aabb_count < 0 || d->obb_count < 0 || d->sphere_count < 0) return fail(c, ART_E_INVALID, "negative collider count");
  if ((long long)d->aabb_count + d->obb_count + d->sphere_count > kMaxColliders)
    return fail(c, ART_E_UNSUPPORTED, "more than %lld colliders", kMaxColliders);
  if ((d->aabb_count && !d->aabb_colliders) || (d->obb_count && !d->obb_colliders) || (d->sphere_count && !d->sphere_colliders))
    return fail(c, ART_E_INVALID, "collider pointer is NULL with a non-zero count");
  if (d->stages & ~ART_STAGE_ALL) return fail(c, ART_E_INVALID, "unknown stage bits");
  if (d->stages & ART_STAGE_DSP_PARAMS) {
    if (!d->dsp) return fail(c, ART_E_INVALID, "ART_STAGE_DSP_PARAMS needs desc->dsp");
    if (!(d->stages & ART_STAGE_REDUCE)) return fail(c, ART_E_INVALID, "ART_STAGE_DSP_PARAMS needs ART_STAGE_REDUCE");
    const art_dsp_desc* p = d->dsp;
    if (!p->reverb_volume_curve.baked || p->reverb_volume_curve.sample_count < 2 || !p->muffle_curve.baked ||
        p->muffle_curve.sample_count < 2)
      return fail(c, ART_E_INVALID, "DSP curves need >= 2 baked samples");
    if (p->reverb_volume_curve.sample_count > 4096 || p->muffle_curve.sample_count > 4096)
      return fail(c, ART_E_UNSUPPORTED, "DSP curves > 4096 samples");
  }
  return ART_OK;
}

FanLayout make_layout(const art_frame_desc* d, uint32_t out_flags) {
  FanLayout L{};
  const size_t T = d->audio_target_count, TC = d->batch_slots, RH = (size_t)d->ray_count * d->max_hits_per_ray;
  L.has_dsp = (d->stages & ART_STAGE_DSP_PARAMS) ? 1 : 0;
  L.has_hits = (out_flags & ART_OUT_HIT_RESULTS) ? 1 : 0;
  size_t off = 0;
  L.settings_off = (uint32_t)off; off = align_up(off + T * sizeof(art_target_settings), 16);
  L.dsp_off = (uint32_t)off; off = align_up(off + (L.has_dsp ? T * sizeof(art_dsp_params) : 0), 16);
  L.muffle_off = (uint32_t)off; off = align_up(off + TC * T * 2, 16);
  L.perm_off = (uint32_t)off; off = align_up(off + TC * T * 4, 16);
  L.echo_off = (uint32_t)off; off = align_up(off + RH * 2, 16);
  L.hit_points_off = (uint32_t)off; off = align_up(off + (L.has_hits ? RH * sizeof(art_half3) : 0), 16);
  L.hit_counts_off = (uint32_t)off; off = align_up(off + (L.has_hits ? (size_t)d->ray_count : 0), 16);
  L.hit_ids_off = (uint32_t)off; off = align_up(off + (L.has_hits ? RH * sizeof(uint32_t) : 0), 16);
  L.stride = (uint32_t)off;
  return L;
}

// Direction-coherent visiting order of the rays: octahedral map of each direction, quantised
// to 16 bits per axis, Morton-interleaved, sorted. 64 consecutive slots then cover a compact
// patch of the sphere, so a wave's echo / muffle rays see the same blockers. Only the lane
// assignment changes; every output is written at the ray's own index.
void coherent_order(const art_half3* dirs, int R, std::vector<int>& order) {
  std::vector<std::pair<uint32_t, int>> keys((size_t)R);
  for (int i = 0; i < R; ++i) {
    float x = art_f16tof32_host(dirs[i].x), y = art_f16tof32_host(dirs[i].y), z = art_f16tof32_host(dirs[i].z);
    float n = std::fabs(x) + std::fabs(y) + std::fabs(z);
    float u = 0.0f, v = 0.0f;
    if (n > 0.0f && n == n) {
      x /= n; y /= n; z /= n;
      if (z < 0.0f) {
        float ux = (1.0f - std::fabs(y)) * (x >= 0.0f ? 1.0f : -1.0f);
        float vy = (1.0f - std::fabs(x)) * (y >= 0.0f ? 1.0f : -1.0f);
        u = ux; v = vy;
      } else {
        u = x; v = y;
      }
    }
    auto q = [](float a) {
      float t = (a + 1.0f) * 0.5f * 65535.0f;
      t = t < 0.0f ? 0.0f : (t > 65535.0f ? 65535.0f : t);
      return (uint32_t)t;
    };
    auto spread = [](uint32_t a) {
      a &= 0xFFFFu;
      a = (a | (a << 8)) & 0x00FF00FFu;
      a = (a | (a << 4)) & 0x0F0F0F0Fu;
      a = (a | (a << 2)) & 0x33333333u;
      a = (a | (a << 1)) & 0x55555555u;
      return a;
    };
    keys[(size_t)i] = {spread(q(u)) | (spread(q(v)) << 1), i};
  }
  std::stable_sort(keys.begin(), keys.end(), [](const std::pair<uint32_t, int>& a, const std::pair<uint32_t, int>& b) {
    return a.first < b.first;
  });
  order.resize((size_t)R);
  for (int i = 0; i < R; ++i) order[(size_t)i] = keys[(size_t)i].second;
}

// Cube-map direction cells around a target (art_cells.hip): face f = 2 m + (negative), cell (i, j)
// covers u = v[(m+1)%3] / |v[m]| in [-1 + 2i/G, -1 + 2(i+1)/G] and w = v[(m+2)%3] / |v[m]| likewise
// (art_trace.hip cube_cell). Each cell's cone: the normalised sum of its corner directions and the
// largest angle to a corner (the farthest point of a convex spherical quadrilateral from an inner
// point), plus 1e-4 rad for the rounding of the cell lookup and of this float table.
struct ConeTable {
  CellCone cone[kCells];
  float alpha_max = 0.0f;
  ConeTable() {
    for (int f = 0; f < 6; ++f) {
      const int m = f >> 1;
      const double sg = (f & 1) ? -1.0 : 1.0;
      for (int j = 0; j < kCellG; ++j)
        for (int i = 0; i < kCellG; ++i) {
          double corner[4][3], sum[3] = {0, 0, 0};
          for (int k = 0; k < 4; ++k) {
            const double u = -1.0 + 2.0 * (i + (k & 1)) / kCellG, w = -1.0 + 2.0 * (j + (k >> 1)) / kCellG;
            double d[3];
            d[m] = sg; d[(m + 1) % 3] = u; d[(m + 2) % 3] = w;
            const double nrm = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            for (int a = 0; a < 3; ++a) { corner[k][a] = d[a] / nrm; sum[a] += corner[k][a]; }
          }
          const double sn = std::sqrt(sum[0] * sum[0] + sum[1] * sum[1] + sum[2] * sum[2]);
          for (int a = 0; a < 3; ++a) sum[a] /= sn;
          double alpha = 0.0;
          for (int k = 0; k < 4; ++k) {
            const double c = sum[0] * corner[k][0] + sum[1] * corner[k][1] + sum[2] * corner[k][2];
            alpha = std::max(alpha, std::acos(std::min(1.0, c)));
          }
          alpha += 1e-4;
          CellCone& cc = cone[(f * kCellG + j) * kCellG + i];
          cc.ax = (float)sum[0]; cc.ay = (float)sum[1]; cc.az = (float)sum[2];
          cc.cos_a = (float)std::cos(alpha); cc.sin_a = (float)std::sin(alpha);
          cc.pad0 = cc.pad1 = cc.pad2 = 0.0f;
          alpha_max = std::max(alpha_max, (float)alpha);
        }
    }
  }
};
const ConeTable& cone_table() {
  static const ConeTable t;
  return t;
}

// Frame scalars + batch tables (Audio/AudioRayTracer.cs:161, Jobs/*:63-64, :36-37).
void make_frame(const art_frame_desc* d, uint32_t out_flags, Frame& f, const int* resident_counts = nullptr) {
  // the direction-coherent order of the last frame is kept while its directions stay the same
  // (they are set once at init, AudioRayTracer.cs:72-86): a 3-KB compare instead of the sort
  std::vector<int> last_order;
  std::vector<uint8_t> last_dirs;
  last_order.swap(f.ray_order);
  last_dirs.swap(f.order_dirs);
  f = Frame();
  f.R = d->ray_count; f.H = d->max_hits_per_ray; f.T = d->audio_target_count;
  f.TC = d->batch_slots; f.bs = d->batch_size; f.nb = (f.R + f.bs - 1) / f.bs;
  f.ns = d->sphere_count; f.na = d->aabb_count; f.no = d->obb_count;
  if (resident_counts) {
    f.resident = true;
    f.ns = resident_counts[0]; f.na = resident_counts[1]; f.no = resident_counts[2];
  }
  // collider sections of the staging and record buffers (empty when the store holds them)
  const size_t sn = f.resident ? 0 : (size_t)f.ns, an = f.resident ? 0 : (size_t)f.na, on = f.resident ? 0 : (size_t)f.no;
  f.stages = d->stages;
  f.L = make_layout(d, out_flags);
  f.slot_batch.assign(f.TC, make_int2(0, 0));
  f.muffle_reset.assign(f.TC, 0);
  for (int start = 0; start < f.R; start += f.bs) {
    const int cnt = std::min(f.bs, f.R - start);
    // raytracer: batchCount = MuffleRayHits.Length / T = TC; batchId = start * TC / R
    const long long rid = (long long)start * f.TC / f.R;
    f.muffle_reset[rid] = 1;
    // permeation: batchCount = PPR.Length / totalRays / T (integer division, Q7)
    const int pbc = (f.TC * f.T) / cnt / f.T;
    const long long pid = (long long)start * pbc / f.R;
    f.slot_batch[pid] = make_int2(start, start + cnt);  // later batches overwrite earlier ones
  }
  if (f.TC == 1) {
    const size_t nb = (size_t)f.R * sizeof(art_half3);
    if (last_order.size() == (size_t)f.R && last_dirs.size() == nb && memcmp(last_dirs.data(), d->ray_directions, nb) == 0) {
      f.ray_order.swap(last_order);
      f.order_dirs.swap(last_dirs);
    } else {
      coherent_order(d->ray_directions, f.R, f.ray_order);
      const uint8_t* b = reinterpret_cast<const uint8_t*>(d->ray_directions);
      f.order_dirs.assign(b, b + nb);
    }
  } else {  // per-batch muffle slots: keep rays in index order
    f.ray_order.resize((size_t)f.R);
    for (int i = 0; i < f.R; ++i) f.ray_order[(size_t)i] = i;
  }
  FrameParams& p = f.fp;
  p.R = f.R; p.H = f.H; p.T = f.T; p.TC = f.TC; p.bs = f.bs; p.nb = f.nb;
  p.max_life = d->max_ray_life; p.max_muffle = d->max_muffle_hit_distance;
  p.muffle_eff = d->muffle_effectiveness; p.perm_strength = d->permeation_strength_per_ray;
  p.perm_eff = d->permeation_effectiveness; p.max_reverb = d->max_reverb_distance;
  p.stages = d->stages;
  if ((d->stages & ART_STAGE_DSP_PARAMS) && d->dsp) {
    const art_dsp_desc* q = d->dsp;
    p.dl_min = q->reverb_dry_level_min; p.dl_max = q->reverb_dry_level_max;
    p.db_min = q->reverb_dry_boost_min; p.db_max = q->reverb_dry_boost_max;
    p.mc_min = q->muffle_cutoff_min; p.mc_max = q->muffle_cutoff_max;
    p.vol_n = q->reverb_volume_curve.sample_count; p.vol_len = q->reverb_volume_curve.length;
    p.muf_n = q->muffle_curve.sample_count; p.muf_len = q->muffle_curve.length;
    p.sample_rate = q->sample_rate;
  }
  // input staging layout (16-B aligned sections)
  size_t o = 0;
  f.off_sph = o; o = align_up(o + sn * sizeof(art_sphere), 16);
  f.off_aabb = o; o = align_up(o + an * sizeof(art_aabb), 16);
  f.off_obb = o; o = align_up(o + on * sizeof(art_obb), 16);
  f.off_tgt = o; o = align_up(o + (size_t)f.T * 12, 16);
  f.off_dirs = o; o = align_up(o + (size_t)f.R * sizeof(art_half3), 16);
  f.off_vol = o; o = align_up(o + (size_t)p.vol_n * 4, 16);
  f.off_muf = o; o = align_up(o + (size_t)p.muf_n * 4, 16);
  f.off_tab = o; o = align_up(o + (size_t)f.TC * sizeof(int2), 16);
  f.off_reset = o; o = align_up(o + (size_t)f.TC, 16);
  f.off_order = o; o = align_up(o + (size_t)f.R * 4, 16);
  f.raw_bytes = o;
  size_t s = 0;
  f.soa_sph = s; s = align_up(s + sn * sizeof(SphereRec), 256);
  f.soa_aabb = s; s = align_up(s + an * sizeof(AabbRec), 256);
  f.soa_obb = s; s = align_up(s + on * sizeof(ObbRec), 256);
  f.soa_sphc = s; s = align_up(s + sn * sizeof(SphereCold), 256);
  f.soa_aabbc = s; s = align_up(s + an * sizeof(AabbCold), 256);
  f.soa_obbc = s; s = align_up(s + on * sizeof(ObbCold), 256);
  f.soa_cull = s; s = align_up(s + (sn + an + on) * sizeof(CullRec), 256);
  {  // broad-phase structure (art_bvh.hip)
    const size_t n = (size_t)(f.ns + f.na + f.no);
    f.sort_temp = sort_scene_temp_bytes((int)n);
    f.soa_box = s; s = align_up(s + 6 * sizeof(float), 256);
    f.soa_keys = s; s = align_up(s + n * 4, 256);
    f.soa_keys_s = s; s = align_up(s + n * 4, 256);
    f.soa_vals = s; s = align_up(s + n * 4, 256);
    f.soa_perm = s; s = align_up(s + n * 4, 256);
    f.soa_temp = s; s = align_up(s + f.sort_temp, 256);
    f.soa_bvh = s; s = align_up(s + bvh_node_count((int)n) * sizeof(CullRec), 256);
    f.soa_bvh_ref = s; s = align_up(s + n * 4, 256);
    f.soa_bvh_pos = s; s = align_up(s + n * 4, 256);
    f.soa_bvh_leaf = s; s = align_up(s + bvh_slot_count((int)n) * 64, 256);
    f.soa_kd = s; s = align_up(s + kd_scratch_bytes((int)n), 256);
  }
  {  // muffle candidate lists
    const size_t cells = (size_t)f.T * kCells * 3;  // lists per (target, cell, collider type)
    f.cells_cap = (uint32_t)cells_entry_cap(f.T, f.ns + f.na + f.no);
    f.cells_temp = cells_scan_temp_bytes(f.T, f.cells_cap);
    f.soa_ccount = s; s = align_up(s + (cells + 1) * 4, 256);
    f.soa_cstart = s; s = align_up(s + (cells + 1) * 4, 256);
    f.soa_ccur = s; s = align_up(s + (cells + 1) * 4, 256);
    f.soa_ckeys = s; s = align_up(s + (size_t)f.cells_cap * 8, 256);
    f.soa_cent_s = s; s = align_up(s + (size_t)f.cells_cap * 8, 256);
    f.soa_cfar = s; s = align_up(s + (size_t)f.T * 4, 256);
    f.soa_cok = s; s = align_up(s + (size_t)f.T * 4, 256);
    f.soa_ctot = s; s = align_up(s + (size_t)f.T * 8, 256);
    f.soa_cbox = s; s = align_up(s + sizeof(CullRec), 256);
    f.soa_ctemp = s; s = align_up(s + f.cells_temp, 256);
    f.soa_cent = s; s = align_up(s + (size_t)f.cells_cap * 8, 256);
    f.soa_cgeo = s; s = align_up(s + cells_geo_bytes(f.T, f.ns + f.na + f.no), 256);
  }
  f.soa_bytes = s;
}

void pack_inputs(const art_frame_desc* d, const Frame& f, uint8_t* h) {
  if (!f.resident) {
    if (f.ns) memcpy(h + f.off_sph, d->sphere_colliders, (size_t)f.ns * sizeof(art_sphere));
    if (f.na) memcpy(h + f.off_aabb, d->aabb_colliders, (size_t)f.na * sizeof(art_aabb));
    if (f.no) memcpy(h + f.off_obb, d->obb_colliders, (size_t)f.no * sizeof(art_obb));
  }
  memcpy(h + f.off_tgt, d->audio_target_positions, (size_t)f.T * 12);
  memcpy(h + f.off_dirs, d->ray_directions, (size_t)f.R * sizeof(art_half3));
  if (f.fp.vol_n) memcpy(h + f.off_vol, d->dsp->reverb_volume_curve.baked, (size_t)f.fp.vol_n * 4);
  if (f.fp.muf_n) memcpy(h + f.off_muf, d->dsp->muffle_curve.baked, (size_t)f.fp.muf_n * 4);
  memcpy(h + f.off_tab, f.slot_batch.data(), (size_t)f.TC * sizeof(int2));
  memcpy(h + f.off_reset, f.muffle_reset.data(), (size_t)f.TC);
  memcpy(h + f.off_order, f.ray_order.data(), (size_t)f.R * 4);
}

// An art_launch_device frame still running on the caller's stream reads the scene (records, sorted
// copies, BVH) and uses the context's shared buffers (accumulators, pairs, side streams): work on
// dv.stream that rewrites or reuses them waits for it first.
// The completion event of those frames is recorded only here, when something has to wait for them:
// an event record between frames costs the launch stream ~5 us of GPU idle per frame (kernel trace,
// DESIGN.md §4), so back-to-back frames on one stream record none. The caller's stream of the last
// frame must still exist at the next call that touches the scene (art.h, streams).
// With ART_CTX_EVENT_EACH_LAUNCH the event is recorded by art_launch_device itself (launch_recorded),
// so the caller may destroy or recycle its stream right after the call.
int mark_launch_done(art_ctx* c, Device& dv) {
  if (dv.launch_recorded) return ART_OK;
  if (!dv.launch_done) HIP_TRY(c, hipEventCreateWithFlags(&dv.launch_done, hipEventDisableTiming));
  HIP_TRY(c, hipEventRecord(dv.launch_done, dv.launch_stream));
  dv.launch_recorded = true;
  return ART_OK;
}
int wait_launch(art_ctx* c, Device& dv) {
  if (dv.launch_pending) {
    int rc = mark_launch_done(c, dv);
    if (rc) return rc;
    HIP_TRY(c, hipStreamWaitEvent(dv.stream, dv.launch_done, 0));
    dv.launch_pending = false;
  }
  return ART_OK;
}

// Upload the packed inputs to one device and build its SoA records (async on dv.stream).
// The resident store's records as the muffle cell lists were just built from them (none dirty).
void snapshot_cell_base(art_ctx* c) {
  bool clean = true;
  for (int k = 0; k < 3; ++k) clean &= c->kinds[k].dirty_list.empty();
  for (int k = 0; k < 3; ++k) c->cell_base[k] = c->kinds[k].recs;
  c->cell_base_ok = clean;
}

// The lists built from record `base` still hold record `now` (cell_slack): same extents and owner,
// centre moved by at most half the slack of the base's bounding radius.
bool cell_still_valid(int kind, const uint8_t* now, const uint8_t* base) {
  const size_t ext = kind == 0 ? 2 : 6;  // radius (half) or size (half3), after the centre
  const size_t tid_off = kind == 0 ? offsetof(art_sphere, audio_target_id)
                                   : (kind == 1 ? offsetof(art_aabb, audio_target_id) : offsetof(art_obb, audio_target_id));
  if (memcmp(now + 6, base + 6, ext) != 0 || memcmp(now + tid_off, base + tid_off, 2) != 0) return false;
  uint16_t cn[3], cb[3], e[3] = {0, 0, 0};
  memcpy(cn, now, 6);
  memcpy(cb, base, 6);
  memcpy(e, base + 6, ext);
  float d2 = 0.0f, r2 = 0.0f;
  for (int a = 0; a < 3; ++a) {
    const float dd = art::f16tof32(cn[a]) - art::f16tof32(cb[a]);
    d2 += dd * dd;
    const float ea = art::f16tof32(e[a]);
    r2 += ea * ea;
  }
  const float half = 0.5f * art::cell_slack(std::sqrt(r2)) * 0.999f;
  return std::isfinite(d2) && std::isfinite(r2) && d2 <= half * half;
}

int upload_scene(art_ctx* c, Device& dv, const Frame& f, const uint8_t* h_in) {
  HIP_TRY(c, hipSetDevice(dv.id));
  if (int rc = wait_launch(c, dv)) return rc;
  if (!dv.raw.reserve(f.raw_bytes) || !dv.soa.reserve(f.soa_bytes)) return fail(c, ART_E_NOMEM, "device allocation failed");
  const int key[10] = {f.ns, f.na, f.no, f.T, f.R, f.TC, f.H, f.fp.vol_n, f.fp.muf_n, (int)f.raw_bytes};
  if (!f.resident && dv.raw_valid && dv.last_raw_p == dv.raw.p && dv.last_soa_p == dv.soa.p &&
      memcmp(dv.last_key, key, sizeof key) == 0 && memcmp(dv.last_raw.data(), h_in, f.raw_bytes) == 0) {
    dv.sc = dv.last_sc;  // device records, sorted copies and BVH are those of these same inputs
    dv.bound = true;
    return ART_OK;
  }
  dv.raw_valid = false;
  HIP_TRY(c, hipMemcpyAsync(dv.raw.p, h_in, f.raw_bytes, hipMemcpyHostToDevice, dv.stream));
  uint8_t* raw = static_cast<uint8_t*>(dv.raw.p);
  uint8_t* soa = static_cast<uint8_t*>(dv.soa.p);
  DevScene& sc = dv.sc;
  if (f.resident) {  // records and bounds of the last art_colliders_sync
    sc.sph = dv.st_sc.sph; sc.sphc = dv.st_sc.sphc; sc.ns = dv.st_sc.ns;
    sc.aabb = dv.st_sc.aabb; sc.aabbc = dv.st_sc.aabbc; sc.na = dv.st_sc.na;
    sc.obb = dv.st_sc.obb; sc.obbc = dv.st_sc.obbc; sc.no = dv.st_sc.no;
    sc.cull = dv.st_sc.cull;
  } else {
    launch_prep(reinterpret_cast<const art_sphere*>(raw + f.off_sph), f.ns, reinterpret_cast<const art_aabb*>(raw + f.off_aabb),
                f.na, reinterpret_cast<const art_obb*>(raw + f.off_obb), f.no, reinterpret_cast<SphereRec*>(soa + f.soa_sph),
                reinterpret_cast<SphereCold*>(soa + f.soa_sphc), reinterpret_cast<AabbRec*>(soa + f.soa_aabb),
                reinterpret_cast<AabbCold*>(soa + f.soa_aabbc), reinterpret_cast<ObbRec*>(soa + f.soa_obb),
                reinterpret_cast<ObbCold*>(soa + f.soa_obbc), reinterpret_cast<CullRec*>(soa + f.soa_cull), dv.stream);
    HIP_TRY(c, hipGetLastError());
    sc.sph = reinterpret_cast<const SphereRec*>(soa + f.soa_sph); sc.ns = f.ns;
    sc.aabb = reinterpret_cast<const AabbRec*>(soa + f.soa_aabb); sc.na = f.na;
    sc.obb = reinterpret_cast<const ObbRec*>(soa + f.soa_obb); sc.no = f.no;
    sc.sphc = reinterpret_cast<const SphereCold*>(soa + f.soa_sphc);
    sc.aabbc = reinterpret_cast<const AabbCold*>(soa + f.soa_aabbc);
    sc.obbc = reinterpret_cast<const ObbCold*>(soa + f.soa_obbc);
    sc.cull = reinterpret_cast<const CullRec*>(soa + f.soa_cull);
  }
  sc.targets = reinterpret_cast<const float*>(raw + f.off_tgt); sc.T = f.T;
  sc.dirs = reinterpret_cast<const uint16_t*>(raw + f.off_dirs); sc.R = f.R;
  SortBufs sb;
  sb.box = reinterpret_cast<float*>(soa + f.soa_box);
  sb.keys = reinterpret_cast<uint32_t*>(soa + f.soa_keys); sb.keys_s = reinterpret_cast<uint32_t*>(soa + f.soa_keys_s);
  sb.vals = reinterpret_cast<int*>(soa + f.soa_vals); sb.perm = reinterpret_cast<int*>(soa + f.soa_perm);
  sb.temp = soa + f.soa_temp; sb.temp_bytes = f.sort_temp;
  sb.bvh = bvh_node_count(f.ns + f.na + f.no) ? reinterpret_cast<CullRec*>(soa + f.soa_bvh) : nullptr;
  sb.bvh_ref = reinterpret_cast<uint32_t*>(soa + f.soa_bvh_ref);
  sb.bvh_pos = reinterpret_cast<uint32_t*>(soa + f.soa_bvh_pos);
  sb.bvh_leaf = reinterpret_cast<float4*>(soa + f.soa_bvh_leaf);
  sb.kd = kd_scratch_bytes(f.ns + f.na + f.no) ? soa + f.soa_kd : nullptr;
  sc.bvh = nullptr; sc.bvh_ref = nullptr; sc.bvh_leaf = nullptr; sc.bvh_levels = 0;
  dv.sb = sb;
  // The cell lists need only the decoded colliders and the targets (cells_box_kernel gives their
  // distance bound), the BVH only the colliders: with a rebuilt BVH the lists build on the side
  // stream beside it (its surface-area passes occupy a few CUs for ~70 us), joined before the frame.
  hipStream_t cells_st = dv.stream;
  {
    if (!dv.cones.p) {
      if (!dv.cones.reserve(sizeof(CellCone) * kCells)) return fail(c, ART_E_NOMEM, "device allocation failed");
      HIP_TRY(c, hipMemcpyAsync(dv.cones.p, cone_table().cone, sizeof(CellCone) * kCells, hipMemcpyHostToDevice, dv.stream));
    }
    const bool rebuild = !(f.resident && dv.sorted_gen != ~0ull && dv.sorted_soa == dv.soa.p && dv.sorted_n[0] == f.ns &&
                           dv.sorted_n[1] == f.na && dv.sorted_n[2] == f.no);
    if (rebuild && kCellsBesideBvh && f.cells_cap > 0) {
      if (!dv.side) {
        HIP_TRY(c, hipStreamCreateWithFlags(&dv.side, hipStreamNonBlocking));
        HIP_TRY(c, hipEventCreateWithFlags(&dv.fork, hipEventDisableTiming));
        HIP_TRY(c, hipEventCreateWithFlags(&dv.join, hipEventDisableTiming));
      }
      HIP_TRY(c, hipEventRecord(dv.fork, dv.stream));
      HIP_TRY(c, hipStreamWaitEvent(dv.side, dv.fork, 0));
      cells_st = dv.side;
    }
  }
  auto build_cells = [&]() -> int {
    CellBufs& cb = dv.cb;
    cb.cones = static_cast<const CellCone*>(dv.cones.p);
    cb.alpha_max = cone_table().alpha_max;
    cb.count = reinterpret_cast<uint32_t*>(soa + f.soa_ccount);
    cb.start = reinterpret_cast<uint32_t*>(soa + f.soa_cstart);
    cb.cursor = reinterpret_cast<uint32_t*>(soa + f.soa_ccur);
    cb.far = reinterpret_cast<float*>(soa + f.soa_cfar);
    cb.ok = reinterpret_cast<uint32_t*>(soa + f.soa_cok);
    cb.tcount = reinterpret_cast<unsigned long long*>(soa + f.soa_ctot);
    cb.temp = soa + f.soa_ctemp; cb.temp_bytes = f.cells_temp;
    cb.ent = reinterpret_cast<uint2*>(soa + f.soa_cent);
    cb.ent_s = reinterpret_cast<uint2*>(soa + f.soa_cent_s);
    cb.keys = reinterpret_cast<uint32_t*>(soa + f.soa_ckeys);
    cb.cap = f.cells_cap;
#ifndef ART_CELLS_COMPACT
#define ART_CELLS_COMPACT 1
#endif
    cb.compact = (ART_CELLS_COMPACT && f.ns < (1 << 16) && f.na < (1 << 16) && f.no < (1 << 16)) ? 1u : 0u;  // 4-B entries
    cb.geo = soa + f.soa_cgeo;
    cb.box = reinterpret_cast<CullRec*>(soa + f.soa_cbox);
    if (launch_build_cells(sc, cb, cells_st) != 0) return fail(c, ART_E_DEVICE, "muffle cell lists failed");
    return 0;
  };
  auto build_bvh = [&]() -> int {
    const bool reuse = f.resident && dv.sorted_gen != ~0ull && dv.sorted_soa == dv.soa.p && dv.sorted_n[0] == f.ns &&
                       dv.sorted_n[1] == f.na && dv.sorted_n[2] == f.no;
    if (reuse) {  // same resident colliders (or only moved ones): keep the orders, refit if needed
      const DevScene& o = dv.sorted_sc;
      sc.bvh = o.bvh; sc.bvh_ref = o.bvh_ref; sc.bvh_leaf = o.bvh_leaf;
      sc.bvh_levels = o.bvh_levels; sc.bvh_leaf0 = o.bvh_leaf0;
      if (dv.sorted_gen != c->sync_gen && launch_refit_scene(sc, sb, dv.stream) != 0)
        return fail(c, ART_E_DEVICE, "collider refit failed");
    } else if (launch_sort_scene(sc, sb, dv.stream) != 0) {
      return fail(c, ART_E_DEVICE, "collider sort failed");
    }
    dv.sorted_gen = f.resident ? c->sync_gen : ~0ull;
    dv.sorted_soa = dv.soa.p;
    dv.sorted_n[0] = f.ns; dv.sorted_n[1] = f.na; dv.sorted_n[2] = f.no;
    return 0;
  };
  {  // the BVH's launches first: its first kernels reach the CUs before the lists' wide passes fill them
    int rc = build_bvh();
    if (rc == 0) rc = build_cells();
    if (rc) {  // kernels may already be queued on the side stream: later work on dv.stream waits for them
      if (cells_st != dv.stream && hipEventRecord(dv.join, cells_st) == hipSuccess)
        (void)hipStreamWaitEvent(dv.stream, dv.join, 0);
      return rc;
    }
  }
  if (cells_st != dv.stream) {  // the frame's kernels wait for the lists
    HIP_TRY(c, hipEventRecord(dv.join, cells_st));
    HIP_TRY(c, hipStreamWaitEvent(dv.stream, dv.join, 0));
  }
  {
    dv.sorted_sc = sc;
    if (f.resident) snapshot_cell_base(c);  // the store's synced records (clean unless edited since)
    else c->cell_base_ok = false;
  }
  HIP_TRY(c, hipGetLastError());
  if (!f.resident) {
    dv.last_raw.assign(h_in, h_in + f.raw_bytes);
    memcpy(dv.last_key, key, sizeof key);
    dv.last_raw_p = dv.raw.p;
    dv.last_soa_p = dv.soa.p;
    dv.last_sc = sc;
    dv.raw_valid = true;
  }
  dv.bound = true;
  return ART_OK;
}

// Per-type sum over targets of colliders NOT owned by the target (permeation loss test counts).
void count_nonowned(art_ctx* c, const art_frame_desc* d) {
  c->nonowned.assign(3, 0);
  if (c->flags & ART_CTX_RESIDENT_COLLIDERS) {  // from the last sync's audio_target_id histograms
    for (int k = 0; k < 3; ++k) {
      uint64_t owned = 0;
      if (!c->tid_hist[k].empty())
        for (int t = 0; t < d->audio_target_count && t < 32768; ++t) owned += (uint64_t)c->tid_hist[k][(size_t)t + 32768];
      c->nonowned[k] = (uint64_t)d->audio_target_count * (uint64_t)c->synced[k] - owned;
    }
    return;
  }
  for (int t = 0; t < d->audio_target_count; ++t) {
    uint64_t os = 0, oa = 0, oo = 0;
    for (int i = 0; i < d->sphere_count; ++i) os += d->sphere_colliders[i].audio_target_id == t;
    for (int i = 0; i < d->aabb_count; ++i) oa += d->aabb_colliders[i].audio_target_id == t;
    for (int i = 0; i < d->obb_count; ++i) oo += d->obb_colliders[i].audio_target_id == t;
    c->nonowned[0] += d->sphere_count - os;
    c->nonowned[1] += d->aabb_count - oa;
    c->nonowned[2] += d->obb_count - oo;
  }
}

// ART_CTX_RESIDENT_COLLIDERS: the desc carries no colliders and the store has been synced.
int check_resident(art_ctx* c, const art_frame_desc* d) {
  if (!(c->flags & ART_CTX_RESIDENT_COLLIDERS)) return ART_OK;
  if (d->sphere_count || d->aabb_count || d->obb_count || d->sphere_colliders || d->aabb_colliders || d->obb_colliders)
    return fail(c, ART_E_INVALID, "ART_CTX_RESIDENT_COLLIDERS: the desc's collider arrays must be NULL / 0");
  if (!c->store_synced) return fail(c, ART_E_STATE, "ART_CTX_RESIDENT_COLLIDERS: no art_colliders_sync yet");
  return ART_OK;
}

// What an event pair of Device::ev_used times: a stage of the frame, or one kernel of the raytrace
// stage (kEvKernel0 + MarkKind, ART_CTX_TIME_EACH_KERNEL).
enum EvKind { kEvRaytrace = 0, kEvPermeate = 1, kEvReduce = 2, kEvKernel0 = 3 };

hipEvent_t pool_event(Device& dv, size_t i) {
  while (dv.ev_pool.size() <= i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    dv.ev_pool.push_back(e);
  }
  return dv.ev_pool[i];
}

// Enqueue the kernels of one frame for fan_count fans on stream st.
int enqueue_kernels(art_ctx* c, Device& dv, const Frame& f, const float* d_origins, int fan_count, uint8_t* d_block,
                    hipStream_t st, bool count, const float* perm_in = nullptr, uint8_t* host_out = nullptr) {
  if (fan_count == 0) return ART_OK;
  const bool timing = (c->flags & ART_CTX_TIME_KERNELS) && !count;
  FrameParams fp = f.fp;
  fp.S = fan_count;
  const uint8_t* raw = static_cast<const uint8_t*>(dv.raw.p);
  fp.vol_curve = reinterpret_cast<const float*>(raw + f.off_vol);
  fp.muf_curve = reinterpret_cast<const float*>(raw + f.off_muf);
  const int2* slot_batch = reinterpret_cast<const int2*>(raw + f.off_tab);
  const uint8_t* muffle_reset = raw + f.off_reset;
  const bool fast = (f.stages & ART_STAGE_RAYTRACE) && !count && !(c->flags & ART_CTX_FORCE_REFERENCE_ORDER);
  const size_t acc_per_fan = (size_t)f.TC * f.T;
  // muffle accumulators, then (16-B aligned) the visibility pair counters: cleared by the first
  // nearest_first_kernel of each fast-path chunk, by one memset before the reference-order kernel
  const size_t acc_words = ((size_t)fan_count * acc_per_fan + 3) & ~(size_t)3;
  const size_t acc_bytes = acc_words * sizeof(uint32_t) + 16;  // + 4 pair counters
  if (!dv.acc.reserve(acc_bytes)) return fail(c, ART_E_NOMEM, "device allocation failed");
  uint32_t* acc = static_cast<uint32_t*>(dv.acc.p);
  uint32_t* pair_count = acc + acc_words;
  DevCounts* counts = nullptr;
  unsigned long long* nhit = nullptr;
  if (count) {
    if (!dv.counts.reserve(sizeof(DevCounts) + 16)) return fail(c, ART_E_NOMEM, "device allocation failed");
    counts = static_cast<DevCounts*>(dv.counts.p);
    nhit = reinterpret_cast<unsigned long long*>(static_cast<uint8_t*>(dv.counts.p) + sizeof(DevCounts));
    HIP_TRY(c, hipMemsetAsync(dv.counts.p, 0, sizeof(DevCounts) + 16, st));
  }
  auto tstart = [&](int kind, hipStream_t on) -> size_t {
    size_t i = dv.ev_used.size() * 2;
    hipEvent_t e = pool_event(dv, i);
    pool_event(dv, i + 1);
    if (e) (void)hipEventRecord(e, on);
    dv.ev_used.push_back({kind, i});
    return i;
  };
  auto tstop = [&](size_t i, hipStream_t on) { hipEvent_t e = pool_event(dv, i + 1); if (e) (void)hipEventRecord(e, on); };

  // Everything the stages allocate or create comes first: once the permeation job is forked to the
  // side stream, an early error return would leave it writing the caller's block unjoined.
  // the permeation job over the BVH (art_trace.hip); reference-order and counting frames sweep every
  // collider (art_kernels.hip), an independent implementation the parity tests compare too
  const bool perm_bvh = !count && !(c->flags & ART_CTX_FORCE_REFERENCE_ORDER);
  const int chunk = fast_fans_per_launch(f.R, f.H, f.T, f.TC, f.L.stride);
  if (fast) {
    if ((c->flags & ART_CTX_COUNT_EXECUTED) && !dv.exec.p) {
      if (!dv.exec.reserve(8 * kExecSlots)) return fail(c, ART_E_NOMEM, "device allocation failed");
      HIP_TRY(c, hipMemsetAsync(dv.exec.p, 0, 8 * kExecSlots, st));
    }
    if (!dv.echo.st) {
      HIP_TRY(c, hipStreamCreateWithFlags(&dv.echo.st, hipStreamNonBlocking));
      HIP_TRY(c, hipEventCreateWithFlags(&dv.echo.fork, hipEventDisableTiming));
      HIP_TRY(c, hipEventCreateWithFlags(&dv.echo.join, hipEventDisableTiming));
    }
  }
  if (fast) {
    FrameParams fps = fp;
    fps.S = std::min(fan_count, chunk);
    if (!dv.pairs.reserve(fast_pair_bytes(fps))) return fail(c, ART_E_NOMEM, "device allocation failed");
  }
  // The permeation job (read-only scene and origins, writes only the fans' permeation sections)
  // runs on the side stream concurrently with the raytrace stage, whose kernels leave CUs idle in
  // their tails; the reduce job waits for both. Counting frames stay serial.
  const bool both = (f.stages & ART_STAGE_RAYTRACE) && (f.stages & ART_STAGE_PERMEATE);
  const bool overlap = both && !count;
  if (overlap && !dv.side) {
    HIP_TRY(c, hipStreamCreateWithFlags(&dv.side, hipStreamNonBlocking));
    HIP_TRY(c, hipEventCreateWithFlags(&dv.fork, hipEventDisableTiming));
    HIP_TRY(c, hipEventCreateWithFlags(&dv.join, hipEventDisableTiming));
  }
  unsigned long long* exec_ctr = nullptr;
  if (fast && (c->flags & ART_CTX_COUNT_EXECUTED)) {
    exec_ctr = static_cast<unsigned long long*>(dv.exec.p);
    dv.exec_launches++;
  }

  // The frame's launch sequence on stream st: stage kernels, side-stream forks and joins.
  auto launch = [&](hipStream_t st, hipEvent_t pfork, hipEvent_t pjoin, const SideStream& echo) -> int {
  // an error return after the fork drains the side stream first (the caller may free d_block)
  struct SideDrain {
    hipStream_t side = nullptr;
    ~SideDrain() { if (side) (void)hipStreamSynchronize(side); }
  } drain;
  if (overlap) {
    drain.side = dv.side;
    HIP_TRY(c, hipEventRecord(pfork, st));
    HIP_TRY(c, hipStreamWaitEvent(dv.side, pfork, 0));
    size_t ti = timing ? tstart(kEvPermeate, dv.side) : 0;
    (perm_bvh ? launch_permeate : launch_permeate_sweep)(dv.sc, fp, f.L, d_origins, d_block, slot_batch, dv.side);
    if (timing) tstop(ti, dv.side);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(pjoin, dv.side));
  }

  if (f.stages & ART_STAGE_RAYTRACE) {
    size_t ti = timing ? tstart(kEvRaytrace, st) : 0;
    // The counting variant sweeps colliders in exact reference order per lane (its per-lane
    // test counts are the metric's numerator); the throughput kernel splits the sweep over waves.
    const int* order = reinterpret_cast<const int*>(raw + f.off_order);
    if (!fast) {
      HIP_TRY(c, hipMemsetAsync(acc, 0, acc_bytes, st));
      launch_raytrace(dv.sc, fp, f.L, d_origins, d_block, acc, counts, st);
    } else {
      FrameParams fpx = fp;
      fpx.exec = exec_ctr;
      // The pair arrays index pairs with 32-bit slots (below 2^31) and the echo outputs with 32-bit
      // half offsets into the block: larger frames run as consecutive fan chunks on st (the pair
      // buffer and counters are reused, the muffle accumulators offset per chunk).
      // per-kernel marks (ART_CTX_TIME_EACH_KERNEL): pool pairs after the stage's own, kept for
      // those recorded; a frame has at most 3H + 2 stage kernels per fan chunk
      KernelMarks marks;
      std::vector<hipEvent_t> mev;
      std::vector<int> mkind;
      if (timing && (c->flags & ART_CTX_TIME_EACH_KERNEL)) {
        const size_t base = dv.ev_used.size() * 2;
        marks.cap = (3 * f.H + 2) * ((fan_count + chunk - 1) / chunk);
        for (int k = 0; k < 2 * marks.cap; ++k) {
          hipEvent_t e = pool_event(dv, base + k);
          if (!e) { marks.cap = k / 2; break; }
          mev.push_back(e);
        }
        mkind.assign((size_t)marks.cap, 0);
        marks.ev = mev.data();
        marks.kind = mkind.data();
      }
      for (int b0 = 0; b0 < fan_count; b0 += chunk) {
        FrameParams fpc = fpx;
        fpc.S = std::min(chunk, fan_count - b0);
        launch_raytrace_fast(dv.sc, fpc, f.L, d_origins + 3 * (size_t)b0, d_block + (size_t)b0 * f.L.stride,
                             acc + (size_t)b0 * acc_per_fan, order, dv.pairs.p, pair_count, st, echo,
                             marks.cap ? &marks : nullptr);
      }
      for (int k = 0; k < marks.used; ++k)  // pool index base + 2 k
        dv.ev_used.push_back({kEvKernel0 + mkind[(size_t)k], dv.ev_used.size() * 2});
      dv.marks_dropped += marks.dropped;
    }
    if (timing) tstop(ti, st);
    HIP_TRY(c, hipGetLastError());
  }
  if (overlap) {
    HIP_TRY(c, hipStreamWaitEvent(st, pjoin, 0));
    drain.side = nullptr;  // joined: stream order covers it from here
  }
  if ((f.stages & ART_STAGE_PERMEATE) && !overlap) {
    size_t ti = timing ? tstart(kEvPermeate, st) : 0;
    (perm_bvh ? launch_permeate : launch_permeate_sweep)(dv.sc, fp, f.L, d_origins, d_block, slot_batch, st);
    if (timing) tstop(ti, st);
    HIP_TRY(c, hipGetLastError());
    if (count) {
      launch_perm_count(dv.sc, fp, d_origins, counts, nhit, st);
      HIP_TRY(c, hipGetLastError());
    }
  }
  if (f.stages & (ART_STAGE_RAYTRACE | ART_STAGE_REDUCE)) {
    size_t ti = timing ? tstart(kEvReduce, st) : 0;
    launch_reduce(dv.sc, fp, f.L, d_block, acc, muffle_reset, st, perm_in, (f.stages & ART_STAGE_REDUCE) ? host_out : nullptr);
    if (timing) tstop(ti, st);
    HIP_TRY(c, hipGetLastError());
  }
  return ART_OK;
  };

  return launch(st, dv.fork, dv.join, dv.echo);
}

int read_counts(art_ctx* c, Device& dv, hipStream_t st, art_test_counts* out, bool accumulate) {
  DevCounts h{};
  unsigned long long nhit = 0;
  HIP_TRY(c, hipMemcpyAsync(&h, dv.counts.p, sizeof h, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(&nhit, static_cast<uint8_t*>(dv.counts.p) + sizeof(DevCounts), 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  if (!accumulate) memset(out, 0, sizeof *out);
  out->rt_sphere += h.v[0]; out->rt_aabb += h.v[1]; out->rt_obb += h.v[2];
  out->perm_hit_sphere += h.v[3]; out->perm_hit_aabb += h.v[4]; out->perm_hit_obb += h.v[5];
  if (c->nonowned.size() == 3) {
    out->perm_loss_sphere += nhit * c->nonowned[0];
    out->perm_loss_aabb += nhit * c->nonowned[1];
    out->perm_loss_obb += nhit * c->nonowned[2];
  }
  return ART_OK;
}

bool fan_wants_hits(const art_fan* fans, int n) {
  for (int i = 0; i < n; ++i)
    if (fans[i].ray_hit_points || fans[i].ray_hit_counts || fans[i].ray_hit_ids) return true;
  return false;
}

// JobHandle.Complete (AudioRayTracer.cs:97): the frame's completion event, polled for up to 4 ms
// (a frame takes ~0.1-2 ms: polling wakes the caller within a microsecond or two of the event,
// where a blocking wait adds the runtime's wake-up latency), then waited for. ART_COMPLETE_SPIN=0
// in the environment: always the blocking wait.
hipError_t wait_done(hipEvent_t ev) {
  static const bool spin = [] { const char* e = getenv("ART_COMPLETE_SPIN"); return !(e && e[0] == '0'); }();
  if (spin) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e != hipErrorNotReady) return e;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(4)) break;
    }
  }
  return hipEventSynchronize(ev);
}

// Host-API frames whose slot arrays need no upload (art_schedule): one batch slot (every muffle
// slot is reset by the raytrace stage, the permeation stage rewrites its slot), the raytrace stage
// on, no echo upload, no hit outputs.
bool compact_slots(const Frame& f, bool need_echo) {
  return f.TC == 1 && (f.stages & ART_STAGE_RAYTRACE) && !need_echo && !f.L.has_hits;
}

// One device's share of an art_schedule frame: scene upload, origins and in/out slot arrays H2D,
// kernels, result blocks D2H, completion event (all async on dv.stream).
int enqueue_device_frame(art_ctx* c, Device& dv, const Frame& f, const uint8_t* hin, uint8_t* hb, bool need_echo, bool count,
                         bool inject_failure = false, PhaseClock* pc = nullptr) {
  const FanLayout& L = f.L;
  int rc = upload_scene(c, dv, f, hin);
  if (pc) pc->mark(3);
  if (rc) return rc;
  if (inject_failure) {
    dv.raw_valid = false;  // the scene upload may not have completed: never reuse it
    return fail(c, ART_E_DEVICE, "injected enqueue failure on shard %d (ART_TEST_FAIL_SHARD)", dv.id);
  }
  if (dv.fan_count == 0) { HIP_TRY(c, hipEventRecord(dv.done, dv.stream)); return ART_OK; }
  const size_t bbytes = (size_t)dv.fan_count * L.stride;
  const size_t tcT = (size_t)f.TC * f.T;
  const bool compact = compact_slots(f, need_echo);
  // compact frames: the origins and (without the permeation stage) the caller's permeation slots in
  // one copy; the block's slot sections are written by the kernels (muffle) or not used (permeation)
  const size_t perm_in_off = align_up((size_t)dv.fan_count * 12, 16);
  const bool perm_in = compact && !(f.stages & ART_STAGE_PERMEATE);
  const size_t in_bytes = perm_in ? perm_in_off + (size_t)dv.fan_count * tcT * 4 : (size_t)dv.fan_count * 12;
  if (!dv.origins.reserve(in_bytes) || !dv.block.reserve(bbytes)) return fail(c, ART_E_NOMEM, "device allocation failed");
  uint8_t* hbs = hb + (size_t)dv.fan_begin * L.stride;
  // the shard's origins (and permeation slots), contiguous in the staging (art_schedule)
  HIP_TRY(c, hipMemcpyAsync(dv.origins.p, hin + dv.in_off, in_bytes, hipMemcpyHostToDevice, dv.stream));
  if (need_echo || L.has_hits) {
    HIP_TRY(c, hipMemcpyAsync(dv.block.p, hbs, bbytes, hipMemcpyHostToDevice, dv.stream));
  } else if (!compact) {  // only the muffle + permeation slot arrays (adjacent in the record)
    HIP_TRY(c, hipMemcpy2DAsync(static_cast<uint8_t*>(dv.block.p) + L.muffle_off, L.stride, hbs + L.muffle_off, L.stride,
                                L.echo_off - L.muffle_off, dv.fan_count, hipMemcpyHostToDevice, dv.stream));
  }
  // the reduce kernel stores each fan's record into the pinned staging itself (no D2H copy) when it
  // runs the reduce stage
  const bool direct = (f.stages & ART_STAGE_REDUCE) && !count;
  rc = enqueue_kernels(c, dv, f, static_cast<const float*>(dv.origins.p), dv.fan_count, static_cast<uint8_t*>(dv.block.p),
                       dv.stream, count,
                       perm_in ? reinterpret_cast<const float*>(static_cast<uint8_t*>(dv.origins.p) + perm_in_off) : nullptr,
                       direct ? hbs : nullptr);
  if (rc) return rc;
  if (!direct) HIP_TRY(c, hipMemcpyAsync(hbs, dv.block.p, bbytes, hipMemcpyDeviceToHost, dv.stream));
  HIP_TRY(c, hipEventRecord(dv.done, dv.stream));
  if (pc) pc->mark(4);
  return ART_OK;
}

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

ART_API uint32_t art_version(void) { return kAbiVersion; }

ART_API int art_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Diagnostics: ART_SEGV_TRACE=1 prints the native stack of a fatal signal (glibc backtrace).
static void segv_trace(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  fprintf(stderr, "libart: fatal signal %d, native stack:\n", sig);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static int create_on(const int32_t* ids, int32_t count, art_ctx** out) {
  if (const char* e = getenv("ART_SEGV_TRACE"))
    if (e[0] == '1') { signal(SIGSEGV, segv_trace); signal(SIGABRT, segv_trace); }
  if (!out) return ART_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ART_E_DEVICE;
  if (count <= 0 || count > 64 || !ids) return ART_E_INVALID;
  art_ctx* c = new (std::nothrow) art_ctx();
  if (!c) return ART_E_NOMEM;
  if (const char* e = getenv("ART_HOST_TIMES")) c->hp.on = e[0] == '1';
  for (int32_t k = 0; k < count; ++k) {
    const int i = ids[k];
    Device dv;
    dv.id = i;
    if (i < 0 || i >= n || hipSetDevice(i) != hipSuccess || hipStreamCreateWithFlags(&dv.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&dv.done, hipEventDisableTiming) != hipSuccess) {
      if (dv.stream) (void)hipStreamDestroy(dv.stream);
      art_destroy(c);  // the devices created so far; the failed entry holds nothing
      return ART_E_DEVICE;
    }
    c->devs.push_back(dv);
  }
  *out = c;
  return ART_OK;
}

ART_API int art_create(uint32_t device_mask, art_ctx** out) {
  if (!out) return ART_E_INVALID;
  *out = nullptr;
  if (device_mask == 0) {  // the CPU backend: worker threads, no HIP device needed
    art_ctx* c = new (std::nothrow) art_ctx();
    if (!c) return ART_E_NOMEM;
    c->cpu = art::cpu_create(0);
    if (!c->cpu) { delete c; return ART_E_NOMEM; }
    *out = c;
    return ART_OK;
  }
  int32_t ids[32];
  int32_t k = 0;
  for (int i = 0; i < 32; ++i)
    if (device_mask & (1u << i)) ids[k++] = i;
  return create_on(ids, k, out);
}

ART_API int art_create_on(const int32_t* device_ids, int32_t count, art_ctx** out) {
  return create_on(device_ids, count, out);
}

#ifdef ART_DIAG
void art_diag_dump_impl();
#endif
#ifdef ART_WAVE_TIMES
extern "C" void art_wave_times_dump_impl();
#endif
ART_API void art_destroy(art_ctx* c) {
#ifdef ART_DIAG
  if (c && !c->devs.empty()) art_diag_dump_impl();
#endif
#ifdef ART_WAVE_TIMES
  if (c && !c->devs.empty()) art_wave_times_dump_impl();
#endif
  if (!c) return;
  if (c->hp.on && c->hp.frames) {
    fprintf(stderr, "{\"art_host_phases_us\": {");
    for (int k = 0; k < 8; ++k) fprintf(stderr, "%s\"%s\": %.3f", k ? ", " : "", kHostPhase[k], c->hp.us[k] / (double)c->hp.frames);
    fprintf(stderr, "}, \"frames\": %llu}\n", (unsigned long long)c->hp.frames);
  }
  if (c->cpu) {
    if (c->inflight) art::cpu_complete(c->cpu, nullptr);
    art::cpu_destroy(c->cpu);
  }
  for (Device& dv : c->devs) {
    (void)hipSetDevice(dv.id);
    if (dv.stream) (void)hipStreamSynchronize(dv.stream);
    if (dv.launch_pending) {  // a device frame on the caller's stream: wait for it alone (the stream is valid
                              // until this call, art_device.h); the device-wide wait only if that fails
      if (mark_launch_done(c, dv) != ART_OK || hipEventSynchronize(dv.launch_done) != hipSuccess) (void)hipDeviceSynchronize();
      dv.launch_pending = false;
    }
    dv.raw.release(); dv.soa.release(); dv.origins.release(); dv.block.release(); dv.acc.release(); dv.counts.release();
    dv.exec.release(); dv.pairs.release(); dv.dsp.release(); dv.cones.release();
    dv.st_raw.release(); dv.st_soa.release(); dv.st_upd.release();
    if (dv.st_done) (void)hipEventDestroy(dv.st_done);
    for (hipEvent_t e : dv.st_epoch)
      if (e) (void)hipEventDestroy(e);
    if (dv.launch_done) (void)hipEventDestroy(dv.launch_done);
    for (hipEvent_t e : dv.ev_pool) (void)hipEventDestroy(e);
    if (dv.done) (void)hipEventDestroy(dv.done);
    if (dv.side) (void)hipStreamSynchronize(dv.side);
    if (dv.fork) (void)hipEventDestroy(dv.fork);
    if (dv.join) (void)hipEventDestroy(dv.join);
    if (dv.side) (void)hipStreamDestroy(dv.side);
    if (dv.echo.st) (void)hipStreamSynchronize(dv.echo.st);
    if (dv.echo.fork) (void)hipEventDestroy(dv.echo.fork);
    if (dv.echo.join) (void)hipEventDestroy(dv.echo.join);
    if (dv.echo.st) (void)hipStreamDestroy(dv.echo.st);
    if (dv.stream) (void)hipStreamDestroy(dv.stream);
  }
  c->h_in.release();
  c->h_block.release();
  c->h_dsp.release();
  for (HostBuf& b : c->h_upd) b.release();
  delete c;
}

ART_API const char* art_last_error(const art_ctx* c) { return c ? c->err.c_str() : "null context"; }

// Timing events a device keeps ready once ART_CTX_TIME_KERNELS is first set: the pool grows on the
// host here, before any timed frame, so a timed frame of up to 5 bounces never creates events
// (hipEventCreate inside a caller's timed loop): 6 stage events + 2 (3H + 2) per-kernel events
// (ART_CTX_TIME_EACH_KERNEL) per frame, 64 frames between art_kernel_timing calls.
constexpr size_t kTimingEventsReserve = 64 * (6 + 2 * (3 * 5 + 2));

ART_API int art_set_flags(art_ctx* c, uint32_t flags) {
  if (!c) return ART_E_INVALID;
  if ((flags & ART_CTX_TIME_KERNELS) && !(c->flags & ART_CTX_TIME_KERNELS) && !c->devs.empty()) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (Device& dv : c->devs) {
      (void)hipSetDevice(dv.id);
      (void)pool_event(dv, kTimingEventsReserve - 1);
    }
    (void)hipSetDevice(prev);
  }
  c->flags = flags;
  return ART_OK;
}

ART_API int art_fan_layout_get(const art_frame_desc* d, uint32_t out_flags, art_fan_layout* out) {
  if (!out) return ART_E_INVALID;
  int rc = validate_desc(nullptr, d);
  if (rc) return rc;
  FanLayout L = make_layout(d, out_flags);
  out->stride = L.stride; out->settings_off = L.settings_off; out->dsp_off = L.dsp_off; out->muffle_off = L.muffle_off;
  out->perm_off = L.perm_off; out->echo_off = L.echo_off; out->hit_points_off = L.hit_points_off;
  out->hit_counts_off = L.hit_counts_off;
  out->hit_ids_off = L.hit_ids_off;
  return ART_OK;
}

ART_API int art_schedule(art_ctx* c, const art_frame_desc* d, const art_fan* fans, int32_t fan_count, art_handle* out) {
  if (!c) return ART_E_INVALID;
  if (!out) return fail(c, ART_E_INVALID, "handle pointer is NULL");
  if (c->inflight) return fail(c, ART_E_STATE, "a frame is in flight: call art_complete first (AudioRayTracer.cs:97)");
  int rc = validate_desc(c, d);
  if (rc) return rc;
  if (fan_count < 0 || (fan_count > 0 && !fans)) return fail(c, ART_E_INVALID, "bad fans array");
  rc = check_resident(c, d);
  if (rc) return rc;
  const bool hits = fan_wants_hits(fans, fan_count);
  for (int i = 0; i < fan_count; ++i) {
    const art_fan& f = fans[i];
    if (!f.echo_ray_distances || !f.muffle_ray_hits || !f.permeation_power_remains || !f.settings)
      return fail(c, ART_E_INVALID, "fan %d: echo/muffle/permeation/settings arrays are required", i);
  }
  if (c->cpu) {
    art::CpuColliders rc_{};
    const bool res = (c->flags & ART_CTX_RESIDENT_COLLIDERS) != 0;
    if (res) {
      rc_.sph = reinterpret_cast<const art_sphere*>(c->cpu_recs[0].data()); rc_.ns = c->synced[0];
      rc_.aabb = reinterpret_cast<const art_aabb*>(c->cpu_recs[1].data()); rc_.na = c->synced[1];
      rc_.obb = reinterpret_cast<const art_obb*>(c->cpu_recs[2].data()); rc_.no = c->synced[2];
    }
    const bool count = (c->flags & ART_CTX_COUNT_TESTS) != 0;
    rc = art::cpu_schedule(c->cpu, d, fans, fan_count, res ? &rc_ : nullptr, count);
    if (rc) return fail(c, rc, "CPU backend: schedule failed");
    c->counted = count;
    c->inflight = true;
    c->handle = c->next_handle++;
    *out = c->handle;
    return ART_OK;
  }
  PhaseClock pc(&c->hp);
  Frame& f = c->fr;
  make_frame(d, hits ? ART_OUT_HIT_RESULTS : 0u, f, (c->flags & ART_CTX_RESIDENT_COLLIDERS) ? c->synced : nullptr);
  const FanLayout& L = f.L;
  if (!c->h_in.reserve(f.raw_bytes)) return fail(c, ART_E_NOMEM, "pinned allocation failed");
  const size_t origins_off = align_up(f.raw_bytes, 16);
  if (!c->h_in.reserve(origins_off + (size_t)fan_count * 12)) return fail(c, ART_E_NOMEM, "pinned allocation failed");
  if (!c->h_block.reserve((size_t)fan_count * L.stride)) return fail(c, ART_E_NOMEM, "pinned allocation failed");
  // shard fans over devices
  const int nd = (int)c->devs.size();
  for (int k = 0; k < nd; ++k) {
    Device& dv = c->devs[k];
    dv.fan_begin = (int)((long long)fan_count * k / nd);
    dv.fan_count = (int)((long long)fan_count * (k + 1) / nd) - dv.fan_begin;
  }
  // In/out arrays (the reference's persistent NativeArrays): slots no batch resets keep their
  // contents, so their current values travel to the device with the frame. Compact frames (one
  // batch slot, raytrace stage, no echo upload or hit outputs: every muffle slot is reset) upload
  // no slots, except the permeation slots when the permeation stage does not rewrite them, and
  // those beside the origins (one H2D copy per shard: [origins | permeation slots]).
  const size_t RH = (size_t)f.R * f.H;
  const bool need_echo = f.TC > 1 || !(f.stages & ART_STAGE_RAYTRACE);
  const bool compact = compact_slots(f, need_echo);
  const bool perm_in = compact && !(f.stages & ART_STAGE_PERMEATE);
  const size_t tcT = (size_t)f.TC * f.T;
  size_t in_end = origins_off;
  for (Device& dv : c->devs) {
    dv.in_off = in_end;
    in_end += align_up(align_up((size_t)dv.fan_count * 12, 16) + (perm_in ? (size_t)dv.fan_count * tcT * 4 : 0), 16);
  }
  if (!c->h_in.reserve(in_end)) return fail(c, ART_E_NOMEM, "pinned allocation failed");
  uint8_t* hin = static_cast<uint8_t*>(c->h_in.p);
  uint8_t* hb = static_cast<uint8_t*>(c->h_block.p);
  pc.mark(0);
  pack_inputs(d, f, hin);
  pc.mark(1);
  for (int i = 0, k = 0; i < fan_count; ++i) {
    const art_fan& fn = fans[i];
    while (i >= c->devs[k].fan_begin + c->devs[k].fan_count) ++k;
    const Device& dv = c->devs[k];
    uint8_t* seg = hin + dv.in_off;
    const size_t j = (size_t)(i - dv.fan_begin);
    memcpy(seg + 12 * j, fn.origin, 12);
    if (perm_in) memcpy(seg + align_up((size_t)dv.fan_count * 12, 16) + j * tcT * 4, fn.permeation_power_remains, tcT * 4);
    uint8_t* rec = hb + (size_t)i * L.stride;
    if (!compact) {
      memcpy(rec + L.muffle_off, fn.muffle_ray_hits, tcT * 2);
      memcpy(rec + L.perm_off, fn.permeation_power_remains, tcT * 4);
    }
    if (need_echo) {
      memcpy(rec + L.echo_off, fn.echo_ray_distances, RH * 2);
      if (L.has_hits) {
        if (fn.ray_hit_points) memcpy(rec + L.hit_points_off, fn.ray_hit_points, RH * sizeof(art_half3));
        else memset(rec + L.hit_points_off, 0, RH * sizeof(art_half3));
        if (fn.ray_hit_ids) memcpy(rec + L.hit_ids_off, fn.ray_hit_ids, RH * sizeof(uint32_t));
        else memset(rec + L.hit_ids_off, 0xFF, RH * sizeof(uint32_t));
      }
    }
    if (L.has_hits) {
      if (fn.ray_hit_counts) memcpy(rec + L.hit_counts_off, fn.ray_hit_counts, (size_t)f.R);
      else memset(rec + L.hit_counts_off, 0, (size_t)f.R);
    }
  }
  const bool count = (c->flags & ART_CTX_COUNT_TESTS) != 0;
  if (count) count_nonowned(c, d);
  pc.mark(2);
  // Enqueue per device. An error on device k leaves devices [0, k) (and k itself, partly) with
  // async copies that still read or write the pinned staging: drain every stream before returning,
  // so the next art_schedule can repack h_in / h_block safely.
  // test hook (tests/test_multigpu_gpu.py): shard k's enqueue fails after its scene upload
  const char* fail_env = getenv("ART_TEST_FAIL_SHARD");
  const int fail_shard = fail_env ? atoi(fail_env) : -1;
  for (size_t k = 0; k < c->devs.size(); ++k) {
    Device& dv = c->devs[k];
    rc = enqueue_device_frame(c, dv, f, hin, hb, need_echo, count, (int)k == fail_shard, &pc);
    if (rc) {
      for (Device& e : c->devs) {
        (void)hipSetDevice(e.id);
        (void)hipStreamSynchronize(e.stream);
        if (e.side) (void)hipStreamSynchronize(e.side);  // a forked stage may not have joined
        if (e.echo.st) (void)hipStreamSynchronize(e.echo.st);
      }
      return rc;
    }
  }
  c->fans.assign(fans, fans + fan_count);
  c->counted = count;
  c->inflight = true;
  c->handle = c->next_handle++;
  *out = c->handle;
  return ART_OK;
}

ART_API int art_is_completed(art_ctx* c, art_handle h) {
  if (!c) return ART_E_INVALID;
  if (!c->inflight || h != c->handle) return (h != 0 && h < c->next_handle) ? 1 : fail(c, ART_E_STATE, "unknown handle");
  if (c->cpu) return art::cpu_is_completed(c->cpu) ? 1 : 0;
  for (Device& dv : c->devs) {
    (void)hipSetDevice(dv.id);
    hipError_t e = hipEventQuery(dv.done);
    if (e == hipErrorNotReady) return 0;
    if (e != hipSuccess) return fail(c, ART_E_DEVICE, "hipEventQuery: %s", hipGetErrorString(e));
  }
  return 1;
}

ART_API int art_complete(art_ctx* c, art_handle h) {
  if (!c) return ART_E_INVALID;
  if (!c->inflight || h != c->handle) {
    if (h != 0 && h < c->next_handle) return ART_OK;  // already completed (JobHandle.Complete is idempotent)
    return fail(c, ART_E_STATE, "unknown handle");
  }
  c->inflight = false;
  if (c->cpu) {
    art::cpu_complete(c->cpu, c->counted ? &c->last_counts : nullptr);
    if (c->counted) c->has_counts = true;
    return ART_OK;
  }
  PhaseClock pc(&c->hp);
  for (Device& dv : c->devs) {
    HIP_TRY(c, hipSetDevice(dv.id));
    HIP_TRY(c, wait_done(dv.done));
  }
  pc.mark(5);
  const Frame& f = c->fr;
  const FanLayout& L = f.L;
  const size_t RH = (size_t)f.R * f.H;
  const uint8_t* hb = static_cast<const uint8_t*>(c->h_block.p);
  // compact frames without the permeation stage leave the caller's permeation slots as they are
  const bool perm_back = !(compact_slots(f, f.TC > 1 || !(f.stages & ART_STAGE_RAYTRACE)) && !(f.stages & ART_STAGE_PERMEATE));
  for (size_t i = 0; i < c->fans.size(); ++i) {
    const art_fan& fn = c->fans[i];
    const uint8_t* rec = hb + i * L.stride;
    if (f.stages & ART_STAGE_REDUCE)  // otherwise AudioTargetSettings keep the caller's contents
      memcpy(fn.settings, rec + L.settings_off, (size_t)f.T * sizeof(art_target_settings));
    if (L.has_dsp && fn.dsp_params) memcpy(fn.dsp_params, rec + L.dsp_off, (size_t)f.T * sizeof(art_dsp_params));
    memcpy(fn.muffle_ray_hits, rec + L.muffle_off, (size_t)f.TC * f.T * 2);
    if (perm_back) memcpy(fn.permeation_power_remains, rec + L.perm_off, (size_t)f.TC * f.T * 4);
    memcpy(fn.echo_ray_distances, rec + L.echo_off, RH * 2);
    if (L.has_hits && fn.ray_hit_points) memcpy(fn.ray_hit_points, rec + L.hit_points_off, RH * sizeof(art_half3));
    if (L.has_hits && fn.ray_hit_counts) memcpy(fn.ray_hit_counts, rec + L.hit_counts_off, (size_t)f.R);
    if (L.has_hits && fn.ray_hit_ids) memcpy(fn.ray_hit_ids, rec + L.hit_ids_off, RH * sizeof(uint32_t));
  }
  pc.mark(6);
  if (c->counted) {
    memset(&c->last_counts, 0, sizeof c->last_counts);
    for (Device& dv : c->devs) {
      if (dv.fan_count == 0) continue;
      HIP_TRY(c, hipSetDevice(dv.id));
      int rc = read_counts(c, dv, dv.stream, &c->last_counts, true);
      if (rc) return rc;
    }
    c->has_counts = true;
  }
  pc.mark(7);
  if (c->hp.on) c->hp.frames++;
  return ART_OK;
}

ART_API int art_last_test_counts(art_ctx* c, art_test_counts* out) {
  if (!c || !out) return ART_E_INVALID;
  if (!c->has_counts) return fail(c, ART_E_STATE, "no counted frame yet (set ART_CTX_COUNT_TESTS)");
  *out = c->last_counts;
  return ART_OK;
}

// ---------------------------------------------------------------------------- device-resident
ART_API int art_scene_bind(art_ctx* c, const art_frame_desc* d) {
  if (!c) return ART_E_INVALID;
  if (c->cpu) return fail(c, ART_E_UNSUPPORTED, "%s: the CPU backend (device_mask 0) has the host entry points only", __func__);
  // the in-flight frame's art_complete reads c->fr and its H2D copy may still read c->h_in
  if (c->inflight) return fail(c, ART_E_STATE, "art_scene_bind: a frame is in flight (bind after art_complete)");
  int rc = validate_desc(c, d);
  if (rc) return rc;
  rc = check_resident(c, d);
  if (rc) return rc;
  Frame& f = c->fr;
  make_frame(d, 0u, f, (c->flags & ART_CTX_RESIDENT_COLLIDERS) ? c->synced : nullptr);
  if (!c->h_in.reserve(f.raw_bytes)) return fail(c, ART_E_NOMEM, "pinned allocation failed");
  pack_inputs(d, f, static_cast<uint8_t*>(c->h_in.p));
  count_nonowned(c, d);
  for (Device& dv : c->devs) {
    rc = upload_scene(c, dv, f, static_cast<const uint8_t*>(c->h_in.p));
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(dv.stream));
  }
  return ART_OK;
}

static int launch_common(art_ctx* c, const float* d_origins, int32_t fan_count, void* d_block, uint32_t out_flags,
                         void* stream, bool count, art_test_counts* out) {
  if (!c) return ART_E_INVALID;
  if (c->cpu) return fail(c, ART_E_UNSUPPORTED, "%s: the CPU backend (device_mask 0) has the host entry points only", __func__);
  if (c->inflight) return fail(c, ART_E_STATE, "a frame is in flight (launch after art_complete)");
  if (c->devs.empty() || !c->devs[0].bound) return fail(c, ART_E_STATE, "no scene bound (art_scene_bind)");
  if (fan_count < 0 || (fan_count > 0 && (!d_origins || !d_block))) return fail(c, ART_E_INVALID, "bad device buffers");
  Device& dv = c->devs[0];
  HIP_TRY(c, hipSetDevice(dv.id));
  Frame& f = c->fr;
  // the bound frame's layout is for out_flags = 0; refresh for the requested outputs
  f.L.has_hits = (out_flags & ART_OUT_HIT_RESULTS) ? 1 : 0;
  {
    art_frame_desc tmp{};
    tmp.ray_count = f.R; tmp.max_hits_per_ray = f.H; tmp.audio_target_count = f.T; tmp.batch_slots = f.TC;
    tmp.stages = f.stages;
    f.L = make_layout(&tmp, out_flags);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL is the HIP default stream (torch's default)
  if (f.resident && dv.st_done && st != dv.st_stream) HIP_TRY(c, hipStreamWaitEvent(st, dv.st_done, 0));
  // frames share the context's accumulators and pair buffers: a launch on another stream than the
  // previous one waits for it (on the same stream, stream order already does)
  if (dv.launch_pending && st != dv.launch_stream) {
    int rc = mark_launch_done(c, dv);
    if (rc) return rc;
    HIP_TRY(c, hipStreamWaitEvent(st, dv.launch_done, 0));
  }
  int rc = enqueue_kernels(c, dv, f, d_origins, fan_count, static_cast<uint8_t*>(d_block), st, count);
  if (rc) return rc;
  // the next sync, bind or schedule rewrites the scene or reuses the shared buffers on dv.stream:
  // after this frame (wait_launch records the event on this stream then)
  dv.launch_pending = true;
  dv.launch_stream = st;
  dv.launch_recorded = false;
  if (c->flags & ART_CTX_EVENT_EACH_LAUNCH) {  // opt-in: the caller may drop its stream after this call
    int rc2 = mark_launch_done(c, dv);
    if (rc2) return rc2;
  }
  if (count) return read_counts(c, dv, st, out, false);
  return ART_OK;
}

ART_API int art_launch_device(art_ctx* c, const float* d_origins, int32_t fan_count, void* d_block, uint32_t out_flags,
                              void* stream) {
  return launch_common(c, d_origins, fan_count, d_block, out_flags, stream, false, nullptr);
}

ART_API int art_count_device(art_ctx* c, const float* d_origins, int32_t fan_count, void* d_block, uint32_t out_flags,
                             void* stream, art_test_counts* out) {
  if (!out) return ART_E_INVALID;
  return launch_common(c, d_origins, fan_count, d_block, out_flags, stream, true, out);
}

ART_API int art_fibonacci_directions_device(art_ctx* c, int32_t count, art_half3* d_out, void* stream) {
  if (!c) return ART_E_INVALID;
  if (c->cpu) return fail(c, ART_E_UNSUPPORTED, "%s: the CPU backend (device_mask 0) has the host entry points only", __func__);
  if (count < 0 || (count > 0 && !d_out)) return fail(c, ART_E_INVALID, "art_fibonacci_directions_device: bad arguments");
  if (count == 0) return ART_OK;
  HIP_TRY(c, hipSetDevice(c->devs[0].id));
  launch_fibonacci(count, d_out, static_cast<hipStream_t>(stream));
  HIP_TRY(c, hipGetLastError());
  return ART_OK;
}

ART_API int art_f32tof16_device(art_ctx* c, uint32_t first_bits, uint32_t count, uint16_t* d_out, void* stream) {
  if (!c) return ART_E_INVALID;
  if (c->cpu) return fail(c, ART_E_UNSUPPORTED, "%s: the CPU backend (device_mask 0) has the host entry points only", __func__);
  if (count > 0 && !d_out) return fail(c, ART_E_INVALID, "art_f32tof16_device: d_out is NULL");
  HIP_TRY(c, hipSetDevice(c->devs[0].id));
  launch_half_range(first_bits, count, d_out, static_cast<hipStream_t>(stream));
  HIP_TRY(c, hipGetLastError());
  return ART_OK;
}

ART_API int art_recip_exact_device(art_ctx* c, uint32_t first_bits, uint32_t count, uint32_t* d_out, void* stream) {
  if (!c) return ART_E_INVALID;
  if (c->cpu) return fail(c, ART_E_UNSUPPORTED, "%s: the CPU backend (device_mask 0) has the host entry points only", __func__);
  if (count > 0 && !d_out) return fail(c, ART_E_INVALID, "art_recip_exact_device: d_out is NULL");
  HIP_TRY(c, hipSetDevice(c->devs[0].id));
  launch_recip_range(first_bits, count, d_out, static_cast<hipStream_t>(stream));
  HIP_TRY(c, hipGetLastError());
  return ART_OK;
}

ART_API int art_executed_counts(art_ctx* c, art_exec_counts* out) {
  if (!c || !out) return ART_E_INVALID;
  memset(out, 0, sizeof *out);
  for (Device& dv : c->devs) {
    if (!dv.exec.p) continue;
    HIP_TRY(c, hipSetDevice(dv.id));
    HIP_TRY(c, hipDeviceSynchronize());
    unsigned long long v[kExecSlots] = {};
    HIP_TRY(c, hipMemcpy(v, dv.exec.p, sizeof v, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemset(dv.exec.p, 0, sizeof v));
    for (int k = 0; k < 3; ++k) {  // per kernel family (kExecNearest, kExecEcho, kExecMuffle), then the totals
      const unsigned long long* g = v + kExecNearest + k * kExecGroup;
      out->by_kernel[k].sphere += g[kExecSphere]; out->by_kernel[k].aabb += g[kExecAabb]; out->by_kernel[k].obb += g[kExecObb];
      out->by_kernel[k].cull_box += g[kExecCullBox]; out->by_kernel[k].cell_entries += g[kExecCellEntries];
      out->sphere += g[kExecSphere]; out->aabb += g[kExecAabb]; out->obb += g[kExecObb]; out->cull_box += g[kExecCullBox];
      out->cell_entries += g[kExecCellEntries]; out->muffle_fallback += g[kExecMuffleFallback];
    }
    out->echo_pairs += v[kExecEchoPairs];
    for (int k = 0; k < kExecBounces; ++k) out->bounce_rays[k] += v[kExecBounce0 + k];
    out->launches += dv.exec_launches;
    dv.exec_launches = 0;
  }
  return ART_OK;
}

ART_API int art_debug_leaf_order(art_ctx* c, uint32_t* out, int32_t cap) {
  if (!c || (!out && cap > 0) || cap < 0) return ART_E_INVALID;
  if (c->devs.empty() || !c->devs[0].bound) return ART_E_STATE;
  Device& dv = c->devs[0];
  const int n = dv.sc.ns + dv.sc.na + dv.sc.no;
  if (!dv.sc.bvh_ref || n <= 0) return 0;
  const int m = n < cap ? n : cap;
  HIP_TRY(c, hipSetDevice(dv.id));
  HIP_TRY(c, hipDeviceSynchronize());
  if (m > 0) HIP_TRY(c, hipMemcpy(out, dv.sc.bvh_ref, (size_t)m * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return m;
}

ART_API int art_kernel_timing(art_ctx* c, art_kernel_times* out) {
  if (!c || !out) return ART_E_INVALID;
  memset(out, 0, sizeof *out);
  for (Device& dv : c->devs) {
    HIP_TRY(c, hipSetDevice(dv.id));
    int frames = 0;
    for (auto& u : dv.ev_used) {
      hipEvent_t a = dv.ev_pool[u.second], b = dv.ev_pool[u.second + 1];
      HIP_TRY(c, hipEventSynchronize(b));
      float ms = 0.0f;
      HIP_TRY(c, hipEventElapsedTime(&ms, a, b));
      if (u.first == kEvRaytrace) { out->raytrace_ms += ms; frames++; }
      else if (u.first == kEvPermeate) out->permeate_ms += ms;
      else if (u.first == kEvReduce) out->reduce_ms += ms;
      else if (u.first - kEvKernel0 < kMarkKinds) {
        out->kernel_ms[u.first - kEvKernel0] += ms;
        out->kernel_launches[u.first - kEvKernel0]++;
      }
    }
    dv.ev_used.clear();
    out->launches += frames;
    out->kernel_marks_dropped += dv.marks_dropped;
    dv.marks_dropped = 0;
  }
  return ART_OK;
}

// ---- resident collider store (include/art_colliders.h) ----------------------------------
static const size_t kRecSize[3] = {sizeof(art_sphere), sizeof(art_aabb), sizeof(art_obb)};

ART_API int art_collider_add(art_ctx* c, int32_t kind, const void* rec, int32_t* out_id) {
  if (!c) return ART_E_INVALID;
  if (kind < 0 || kind > 2 || !rec) return fail(c, ART_E_INVALID, "art_collider_add: bad kind or record");
  auto& K = c->kinds[kind];
  if (K.count >= (1 << 24)) return fail(c, ART_E_UNSUPPORTED, "more than 2^24 colliders of one kind");
  const size_t rs = kRecSize[kind];
  K.recs.resize((size_t)(K.count + 1) * rs);
  memcpy(K.recs.data() + (size_t)K.count * rs, rec, rs);
  K.dirty.push_back(1);
  K.dirty_list.push_back(K.count);
  if (out_id) *out_id = K.count;  // AudioColliderId = NextBatch.Length before the add
  K.count++;
  return ART_OK;
}

ART_API int art_collider_set(art_ctx* c, int32_t kind, int32_t id, const void* rec) {
  if (!c) return ART_E_INVALID;
  if (kind < 0 || kind > 2 || !rec) return fail(c, ART_E_INVALID, "art_collider_set: bad kind or record");
  auto& K = c->kinds[kind];
  if (id < 0 || id >= K.count) return fail(c, ART_E_INVALID, "art_collider_set: id %d out of range [0, %d)", id, K.count);
  const size_t rs = kRecSize[kind];
  memcpy(K.recs.data() + (size_t)id * rs, rec, rs);
  if (!K.dirty[(size_t)id]) { K.dirty[(size_t)id] = 1; K.dirty_list.push_back(id); }
  return ART_OK;
}

ART_API int art_collider_set_many(art_ctx* c, int32_t kind, const int32_t* ids, const void* recs, int32_t n) {
  if (!c) return ART_E_INVALID;
  if (kind < 0 || kind > 2 || n < 0 || (n > 0 && (!ids || !recs)))
    return fail(c, ART_E_INVALID, "art_collider_set_many: bad arguments");
  auto& K = c->kinds[kind];
  for (int32_t j = 0; j < n; ++j)  // validate first: all or nothing
    if (ids[j] < 0 || ids[j] >= K.count)
      return fail(c, ART_E_INVALID, "art_collider_set_many: id %d out of range [0, %d)", ids[j], K.count);
  const size_t rs = kRecSize[kind];
  const uint8_t* r = static_cast<const uint8_t*>(recs);
  for (int32_t j = 0; j < n; ++j) {
    const int id = ids[j];
    memcpy(K.recs.data() + (size_t)id * rs, r + (size_t)j * rs, rs);
    if (!K.dirty[(size_t)id]) { K.dirty[(size_t)id] = 1; K.dirty_list.push_back(id); }
  }
  return ART_OK;
}

ART_API int art_collider_remove_swapback(art_ctx* c, int32_t kind, int32_t id) {
  if (!c) return ART_E_INVALID;
  if (kind < 0 || kind > 2) return fail(c, ART_E_INVALID, "art_collider_remove_swapback: bad kind");
  auto& K = c->kinds[kind];
  if (id < 0 || id >= K.count) return ART_OK;  // skipped, as AudioColliderManager.SwapRemove (:92-93)
  const size_t rs = kRecSize[kind];
  const int last = K.count - 1;
  if (id != last) {
    memcpy(K.recs.data() + (size_t)id * rs, K.recs.data() + (size_t)last * rs, rs);
    if (!K.dirty[(size_t)id]) { K.dirty[(size_t)id] = 1; K.dirty_list.push_back(id); }
  }
  K.count = last;
  K.recs.resize((size_t)last * rs);
  K.dirty.resize((size_t)last);
  return ART_OK;
}

ART_API int art_collider_get(art_ctx* c, int32_t kind, int32_t id, void* rec) {
  if (!c) return ART_E_INVALID;
  if (kind < 0 || kind > 2 || !rec) return fail(c, ART_E_INVALID, "art_collider_get: bad kind or record");
  const auto& K = c->kinds[kind];
  if (id < 0 || id >= K.count) return fail(c, ART_E_INVALID, "art_collider_get: id %d out of range [0, %d)", id, K.count);
  memcpy(rec, K.recs.data() + (size_t)id * kRecSize[kind], kRecSize[kind]);
  return ART_OK;
}

ART_API int art_collider_count(art_ctx* c, int32_t kind) {
  if (!c) return ART_E_INVALID;
  if (kind < 0 || kind > 2) return fail(c, ART_E_INVALID, "art_collider_count: bad kind");
  return c->kinds[kind].count;
}

ART_API int art_colliders_clear(art_ctx* c) {
  if (!c) return ART_E_INVALID;
  for (auto& K : c->kinds) {
    K.recs.clear(); K.dirty.clear(); K.dirty_list.clear(); K.count = 0;
  }
  return ART_OK;
}

ART_API int art_colliders_last_sync(art_ctx* c, art_collider_sync_stats* out) {
  if (!c || !out) return ART_E_INVALID;
  *out = c->last_sync;
  return ART_OK;
}

ART_API int art_colliders_sync(art_ctx* c) {
  if (!c) return ART_E_INVALID;
  if (c->inflight) return fail(c, ART_E_STATE, "art_colliders_sync: a frame is in flight (sync after art_complete)");
  const int n[3] = {c->kinds[0].count, c->kinds[1].count, c->kinds[2].count};
  if ((long long)n[0] + n[1] + n[2] > kMaxColliders)
    return fail(c, ART_E_UNSUPPORTED, "art_colliders_sync: more than %lld colliders", kMaxColliders);
  bool counts_changed = !c->store_synced;
  for (int k = 0; k < 3; ++k) counts_changed |= n[k] != c->synced[k];
  // device capacity: grow (x2) and re-upload everything when a list outgrows it
  bool fresh = false;
  for (Device& dv : c->devs) {
    if (n[0] > dv.st_cap[0] || n[1] > dv.st_cap[1] || n[2] > dv.st_cap[2] || !dv.st_raw.p) {
      for (int k = 0; k < 3; ++k) dv.st_cap[k] = std::max({n[k], 2 * dv.st_cap[k], 64});
      dv.st_raw.release();
      dv.st_soa.release();
      dv.st_fresh = true;
    }
    fresh |= dv.st_fresh;
  }
  // dirty records of each kind (all of them after a reallocation), ascending
  std::vector<int> lists[3];
  for (int k = 0; k < 3; ++k) {
    auto& K = c->kinds[k];
    if (fresh) {
      lists[k].resize((size_t)n[k]);
      for (int i = 0; i < n[k]; ++i) lists[k][(size_t)i] = i;
    } else {
      for (int i : K.dirty_list)
        if (i < n[k] && K.dirty[(size_t)i]) lists[k].push_back(i);
      std::sort(lists[k].begin(), lists[k].end());
      lists[k].erase(std::unique(lists[k].begin(), lists[k].end()), lists[k].end());
    }
  }
  // upload image: [idx_s][rec_s][idx_a][rec_a][idx_o][rec_o], 16-B aligned sections
  size_t off_idx[3], off_rec[3], bytes = 0;
  for (int k = 0; k < 3; ++k) {
    off_idx[k] = bytes; bytes = align_up(bytes + lists[k].size() * 4, 16);
    off_rec[k] = bytes; bytes = align_up(bytes + lists[k].size() * kRecSize[k], 16);
  }
  const int nd = (int)(lists[0].size() + lists[1].size() + lists[2].size());
  if (nd || counts_changed) ++c->sync_gen;  // resident frames refit / rebuild their sorted copies
  // the muffle cell lists need a rebuild unless every changed collider stayed within their slack
  bool cells_ok = c->cell_base_ok && !counts_changed && !fresh;
  for (int k = 0; cells_ok && k < 3; ++k) {
    const size_t rs = kRecSize[k];
    if (c->cell_base[k].size() < (size_t)n[k] * rs) { cells_ok = false; break; }
    for (int i : lists[k])
      if (!cell_still_valid(k, c->kinds[k].recs.data() + (size_t)i * rs, c->cell_base[k].data() + (size_t)i * rs)) {
        cells_ok = false;
        break;
      }
  }
  bool cells_rebuilt = false;
  // The update image goes to ring slot seq % kUpdRing. A new epoch reuses the ring: every sync of the
  // previous epoch has finished reading its slot once that epoch's event (recorded after its last
  // sync, on that sync's stream) has completed. Each sync's stream is ordered after the earlier
  // syncs' (a launch on a new stream waits on the old one, a context-stream sync on the launch
  // stream), so that one event covers the whole epoch.
  const uint64_t seq = c->upd_seq++;
  const int slot = (int)(seq % art_ctx::kUpdRing), ep = (int)((seq / art_ctx::kUpdRing) & 1u);
  if (slot == 0)
    for (Device& dv : c->devs)
      if (dv.st_epoch_pending[ep ^ 1]) {
        HIP_TRY(c, hipSetDevice(dv.id));
        HIP_TRY(c, hipEventSynchronize(dv.st_epoch[ep ^ 1]));
        dv.st_epoch_pending[ep ^ 1] = false;
      }
  if (c->cpu) bytes = 0;  // the CPU backend keeps no device copy (it snapshots the lists below)
  if (bytes && !c->h_upd[slot].reserve(bytes)) return fail(c, ART_E_NOMEM, "pinned allocation failed");
  uint8_t* h = static_cast<uint8_t*>(c->h_upd[slot].p);
  for (int k = 0; bytes && k < 3; ++k) {
    const auto& K = c->kinds[k];
    const size_t rs = kRecSize[k];
    for (size_t j = 0; j < lists[k].size(); ++j) {
      const int i = lists[k][j];
      memcpy(h + off_idx[k] + j * 4, &i, 4);
      memcpy(h + off_rec[k] + j * rs, K.recs.data() + (size_t)i * rs, rs);
    }
  }
  for (Device& dv : c->devs) {
    HIP_TRY(c, hipSetDevice(dv.id));
    const int* cap = dv.st_cap;
    const size_t r_s = 0, r_a = align_up((size_t)cap[0] * sizeof(art_sphere), 256),
                 r_o = r_a + align_up((size_t)cap[1] * sizeof(art_aabb), 256),
                 r_end = r_o + align_up((size_t)cap[2] * sizeof(art_obb), 256);
    size_t o = 0;
    const size_t s_sph = o; o = align_up(o + (size_t)cap[0] * sizeof(SphereRec), 256);
    const size_t s_sphc = o; o = align_up(o + (size_t)cap[0] * sizeof(SphereCold), 256);
    const size_t s_aabb = o; o = align_up(o + (size_t)cap[1] * sizeof(AabbRec), 256);
    const size_t s_aabbc = o; o = align_up(o + (size_t)cap[1] * sizeof(AabbCold), 256);
    const size_t s_obb = o; o = align_up(o + (size_t)cap[2] * sizeof(ObbRec), 256);
    const size_t s_obbc = o; o = align_up(o + (size_t)cap[2] * sizeof(ObbCold), 256);
    const size_t s_cull = o; o = align_up(o + (size_t)(cap[0] + cap[1] + cap[2]) * sizeof(CullRec), 256);
    if (!dv.st_raw.reserve(r_end) || !dv.st_soa.reserve(o) || (bytes && !dv.st_upd.reserve(bytes)))
      return fail(c, ART_E_NOMEM, "device allocation failed");
    uint8_t* raw = static_cast<uint8_t*>(dv.st_raw.p);
    uint8_t* soa = static_cast<uint8_t*>(dv.st_soa.p);
    uint8_t* up = static_cast<uint8_t*>(dv.st_upd.p);
    auto* sph = reinterpret_cast<art_sphere*>(raw + r_s);
    auto* aabb = reinterpret_cast<art_aabb*>(raw + r_a);
    auto* obb = reinterpret_cast<art_obb*>(raw + r_o);
    auto* osph = reinterpret_cast<SphereRec*>(soa + s_sph);
    auto* osphc = reinterpret_cast<SphereCold*>(soa + s_sphc);
    auto* oaabb = reinterpret_cast<AabbRec*>(soa + s_aabb);
    auto* oaabbc = reinterpret_cast<AabbCold*>(soa + s_aabbc);
    auto* oobb = reinterpret_cast<ObbRec*>(soa + s_obb);
    auto* oobbc = reinterpret_cast<ObbCold*>(soa + s_obbc);
    auto* cull = reinterpret_cast<CullRec*>(soa + s_cull);
    // Device-path frames still read the records / BVH being rewritten. The sync runs on the stream of
    // the last such frame when its completion is not recorded yet (the stream is valid until this
    // call, art_device.h): stream order puts it after that frame and before the next launch on the
    // same stream, with no cross-stream events (each costs the queue ~5-10 us of idle). Otherwise
    // it runs on the context stream, after the frame's completion event.
    const hipStream_t ss = (dv.launch_pending && !dv.launch_recorded) ? dv.launch_stream : dv.stream;
    if (ss == dv.stream)
      if (int rc = wait_launch(c, dv)) return rc;
    dv.st_stream = ss;
    // moved colliders of a bound resident scene: one launch scatters the records from the pinned image
    // and refits the BVH (launch_sync_refit), below
    const bool refit_follows = nd && dv.bound && c->fr.resident && !counts_changed;
    const bool fused = refit_follows && (long long)n[0] + n[1] + n[2] <= kSyncRefitMax && dv.sc.bvh_levels > 0 && dv.sb.bvh;
    if (nd && !fused) {
      HIP_TRY(c, hipMemcpyAsync(up, h, bytes, hipMemcpyHostToDevice, ss));
      launch_scatter_prep(reinterpret_cast<const int*>(up + off_idx[0]), reinterpret_cast<const art_sphere*>(up + off_rec[0]),
                          (int)lists[0].size(), reinterpret_cast<const int*>(up + off_idx[1]),
                          reinterpret_cast<const art_aabb*>(up + off_rec[1]), (int)lists[1].size(),
                          reinterpret_cast<const int*>(up + off_idx[2]), reinterpret_cast<const art_obb*>(up + off_rec[2]),
                          (int)lists[2].size(), sph, aabb, obb, n[0], n[1], osph, osphc, oaabb, oaabbc, oobb, oobbc, cull,
                          ss);
      HIP_TRY(c, hipGetLastError());
    }
    // a count change moves the bounds of the later kinds (global order spheres, AABBs, OBBs)
    if (counts_changed && !fresh && n[0] + n[1] + n[2] > 0) {
      launch_prep(sph, n[0], aabb, n[1], obb, n[2], osph, osphc, oaabb, oaabbc, oobb, oobbc, cull, ss);
      HIP_TRY(c, hipGetLastError());
    }
    // stream-ordered: frames on ss follow. A sync on the context stream records st_done, which
    // device-path launches on other streams wait on (a refit below records it after its kernels). A
    // sync on the launch stream records nothing (each record costs the queue ~5 us): a launch on
    // another stream waits on that stream's launch_done, work on dv.stream on it through wait_launch.
    if (!dv.st_done) HIP_TRY(c, hipEventCreateWithFlags(&dv.st_done, hipEventDisableTiming));
    const bool lazy = ss != dv.stream;
    if (!refit_follows && !lazy) HIP_TRY(c, hipEventRecord(dv.st_done, ss));
    DevScene& t = dv.st_sc;
    t.sph = osph; t.sphc = osphc; t.ns = n[0];
    t.aabb = oaabb; t.aabbc = oaabbc; t.na = n[1];
    t.obb = oobb; t.obbc = oobbc; t.no = n[2];
    t.cull = cull;
    dv.st_fresh = false;
    if (dv.bound && c->fr.resident) {  // a bound device-resident scene sees the new snapshot
      if (counts_changed) {
        dv.bound = false;  // the sorted copies are sized by count: bind again
      } else {
        dv.sc.sph = t.sph; dv.sc.sphc = t.sphc; dv.sc.ns = t.ns;
        dv.sc.aabb = t.aabb; dv.sc.aabbc = t.aabbc; dv.sc.na = t.na;
        dv.sc.obb = t.obb; dv.sc.obbc = t.obbc; dv.sc.no = t.no;
        dv.sc.cull = t.cull;
        // moved colliders: refit the sorted copies and the BVH in place (device only, no H2D)
        if (nd) {
          if (fused) {
            void* hd = nullptr;  // the pinned image as the device sees it
            HIP_TRY(c, hipHostGetDevicePointer(&hd, h, 0));
            const uint8_t* u = static_cast<const uint8_t*>(hd);
            ScatterArgs a;
            a.idx_s = reinterpret_cast<const int*>(u + off_idx[0]); a.rec_s = reinterpret_cast<const art_sphere*>(u + off_rec[0]);
            a.ds = (int)lists[0].size();
            a.idx_a = reinterpret_cast<const int*>(u + off_idx[1]); a.rec_a = reinterpret_cast<const art_aabb*>(u + off_rec[1]);
            a.da = (int)lists[1].size();
            a.idx_o = reinterpret_cast<const int*>(u + off_idx[2]); a.rec_o = reinterpret_cast<const art_obb*>(u + off_rec[2]);
            a.dob = (int)lists[2].size();
            a.sph = sph; a.aabb = aabb; a.obb = obb; a.ns = n[0]; a.na = n[1];
            a.osph = osph; a.osphc = osphc; a.oaabb = oaabb; a.oaabbc = oaabbc; a.oobb = oobb; a.oobbc = oobbc; a.cull = cull;
            if (!launch_sync_refit(a, dv.sc, dv.sb, ss)) return fail(c, ART_E_DEVICE, "collider sync refit not applicable");
            HIP_TRY(c, hipGetLastError());
          } else if (launch_refit_scene(dv.sc, dv.sb, ss) != 0) {
            (void)hipEventRecord(dv.st_done, ss);
            return fail(c, ART_E_DEVICE, "collider refit failed");
          }
          if (!cells_ok) {
            if (launch_build_cells(dv.sc, dv.cb, ss) != 0) return fail(c, ART_E_DEVICE, "muffle cell lists failed");
            cells_rebuilt = true;
          }
          if (dv.sorted_gen != ~0ull) dv.sorted_gen = c->sync_gen;
          if (!lazy) HIP_TRY(c, hipEventRecord(dv.st_done, ss));  // device-path launches wait for the sort too
        }
      }
    }
    if (slot == art_ctx::kUpdRing - 1) {  // the epoch's last sync: the event that frees the ring
      if (!dv.st_epoch[ep]) HIP_TRY(c, hipEventCreateWithFlags(&dv.st_epoch[ep], hipEventDisableTiming));
      HIP_TRY(c, hipEventRecord(dv.st_epoch[ep], ss));
      dv.st_epoch_pending[ep] = true;
    }
  }
  if (c->fr.resident) { c->fr.ns = n[0]; c->fr.na = n[1]; c->fr.no = n[2]; }
  for (int k = 0; k < 3; ++k) {
    auto& K = c->kinds[k];
    for (int i : K.dirty_list)  // O(changes), not O(colliders)
      if ((size_t)i < K.dirty.size()) K.dirty[(size_t)i] = 0;
    K.dirty_list.clear();
    c->synced[k] = n[k];
    // audio_target_id histogram of the synced records: removed tail, then the dirty records
    auto& tids = c->synced_tid[k];
    auto& hist = c->tid_hist[k];
    if (hist.empty()) hist.assign(65536, 0);
    for (size_t i = (size_t)n[k]; i < tids.size(); ++i) hist[(size_t)(tids[i] + 32768)]--;
    const size_t old_n = tids.size();
    tids.resize((size_t)n[k], 0);
    const size_t rs = kRecSize[k];
    const size_t tid_off = k == 0 ? offsetof(art_sphere, audio_target_id)
                                  : (k == 1 ? offsetof(art_aabb, audio_target_id) : offsetof(art_obb, audio_target_id));
    for (int i : lists[k]) {
      int16_t v;
      memcpy(&v, K.recs.data() + (size_t)i * rs + tid_off, 2);
      if ((size_t)i < old_n) hist[(size_t)(tids[(size_t)i] + 32768)]--;
      tids[(size_t)i] = v;
      hist[(size_t)(v + 32768)]++;
    }
  }
  if (cells_rebuilt) snapshot_cell_base(c);
  else if (!cells_ok) c->cell_base_ok = false;  // the lists (rebuilt at the next bind) no longer hold these records
  if (c->cpu)  // the CPU backend reads the synced snapshot (JobBatch) of each list
    for (int k = 0; k < 3; ++k) c->cpu_recs[k].assign(c->kinds[k].recs.begin(), c->kinds[k].recs.begin() + (size_t)n[k] * kRecSize[k]);
  c->store_synced = true;
  c->last_sync.dirty_records = nd;
  c->last_sync.full_prep = (counts_changed || fresh) ? 1 : 0;
  c->last_sync.reallocated = fresh ? 1 : 0;
  c->last_sync.cells_rebuilt = cells_rebuilt ? 1 : 0;
  c->last_sync.bytes_uploaded = nd ? bytes : 0;
  return ART_OK;
}

// ---- per-sample spatializer DSP (include/art_dsp.h) -------------------------------------
ART_API int art_dsp_source_params_get(const art_spatializer_settings* settings, const art_audio_source* source,
                                      int32_t sample_rate, art_dsp_source_params* out) {
  if (!settings || !source || !out || sample_rate <= 0) return ART_E_INVALID;
  return dsp_source_params(*settings, *source, sample_rate, *out);
}

ART_API int art_dsp_process(art_ctx* c, const art_spatializer_settings* settings, art_audio_source* sources,
                            int32_t count, int32_t sample_rate) {
  if (!c) return ART_E_INVALID;
  if (c->cpu) return fail(c, ART_E_UNSUPPORTED, "%s: the CPU backend (device_mask 0) has the host entry points only", __func__);
  if (!settings || count < 0 || (count > 0 && !sources) || sample_rate <= 0) return fail(c, ART_E_INVALID, "invalid argument");
  if (c->inflight) return fail(c, ART_E_STATE, "a frame is in flight");
  // host: per-buffer scalars; stereo sources with samples go to the device
  std::vector<int> idx;
  std::vector<art_dsp_source_params> params;
  std::vector<long long> offs;
  std::vector<int> frames;
  long long total = 0;  // floats, each source 16-B aligned
  for (int32_t k = 0; k < count; ++k) {
    const art_audio_source& a = sources[k];
    if (a.frames < 0 || (a.frames > 0 && !a.data) || !a.state) return fail(c, ART_E_INVALID, "invalid source %d", k);
    if (a.channels != 2 || a.frames == 0) continue;  // left as is (AudioSpatializer.cs:72)
    art_dsp_source_params p;
    if (dsp_source_params(*settings, a, sample_rate, p) != ART_OK) return fail(c, ART_E_INVALID, "invalid curve");
    idx.push_back(k);
    params.push_back(p);
    offs.push_back(total);
    frames.push_back(a.frames);
    total += ((long long)a.frames * 2 + 3) & ~3LL;
  }
  const size_t n = idx.size();
  if (n == 0) return ART_OK;
  {  // group sources by filter class (muffle x low/high pass) so a wave's chains run one code path
    std::vector<size_t> ord(n);
    for (size_t j = 0; j < n; ++j) ord[j] = j;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return (params[a].flags & 3) < (params[b].flags & 3); });
    std::vector<int> idx2(n);
    std::vector<art_dsp_source_params> params2(n);
    std::vector<int> frames2(n);
    total = 0;
    for (size_t j = 0; j < n; ++j) {
      idx2[j] = idx[ord[j]];
      params2[j] = params[ord[j]];
      frames2[j] = frames[ord[j]];
      offs[j] = total;
      total += ((long long)frames2[j] * 2 + 3) & ~3LL;
    }
    idx.swap(idx2);
    params.swap(params2);
    frames.swap(frames2);
  }
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_data = 0, o_offs = al(o_data + (size_t)total * 4), o_frames = al(o_offs + n * 8),
               o_params = al(o_frames + n * 4), o_state = al(o_params + n * sizeof(art_dsp_source_params)),
               bytes = al(o_state + n * sizeof(art_dsp_state));
  Device& dv = c->devs[0];
  HIP_TRY(c, hipSetDevice(dv.id));
  if (!c->h_dsp.reserve(bytes) || !dv.dsp.reserve(bytes)) return fail(c, ART_E_NOMEM, "allocation failed");
  uint8_t* h = static_cast<uint8_t*>(c->h_dsp.p);
  for (size_t j = 0; j < n; ++j) {
    const art_audio_source& a = sources[idx[j]];
    std::memcpy(h + o_data + offs[j] * 4, a.data, (size_t)a.frames * 8);
    std::memcpy(h + o_state + j * sizeof(art_dsp_state), a.state, sizeof(art_dsp_state));
  }
  std::memcpy(h + o_offs, offs.data(), n * 8);
  std::memcpy(h + o_frames, frames.data(), n * 4);
  std::memcpy(h + o_params, params.data(), n * sizeof(art_dsp_source_params));
  uint8_t* d = static_cast<uint8_t*>(dv.dsp.p);
  HIP_TRY(c, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, dv.stream));
  launch_dsp(reinterpret_cast<float*>(d + o_data), (unsigned long long)total * 4, reinterpret_cast<const long long*>(d + o_offs),
             reinterpret_cast<const int*>(d + o_frames), 0, reinterpret_cast<const art_dsp_source_params*>(d + o_params),
             reinterpret_cast<art_dsp_state*>(d + o_state), (int)n, dv.stream);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipMemcpyAsync(h + o_data, d + o_data, (size_t)total * 4, hipMemcpyDeviceToHost, dv.stream));
  HIP_TRY(c, hipMemcpyAsync(h + o_state, d + o_state, n * sizeof(art_dsp_state), hipMemcpyDeviceToHost, dv.stream));
  HIP_TRY(c, hipStreamSynchronize(dv.stream));
  for (size_t j = 0; j < n; ++j) {
    art_audio_source& a = sources[idx[j]];
    std::memcpy(a.data, h + o_data + offs[j] * 4, (size_t)a.frames * 8);
    std::memcpy(a.state, h + o_state + j * sizeof(art_dsp_state), sizeof(art_dsp_state));
  }
  return ART_OK;
}

ART_API int art_dsp_process_device(art_ctx* c, float* d_data, const art_dsp_source_params* d_params,
                                   art_dsp_state* d_state, int32_t count, int32_t frames, void* stream) {
  if (!c) return ART_E_INVALID;
  if (c->cpu) return fail(c, ART_E_UNSUPPORTED, "%s: the CPU backend (device_mask 0) has the host entry points only", __func__);
  if (count < 0 || frames < 0 || (count > 0 && (!d_data || !d_params || !d_state))) return fail(c, ART_E_INVALID, "invalid argument");
  if (count == 0 || frames == 0) return ART_OK;
  Device& dv = c->devs[0];
  HIP_TRY(c, hipSetDevice(dv.id));
  launch_dsp(d_data, (unsigned long long)count * (unsigned long long)frames * 8ull, nullptr, nullptr, frames, d_params,
             d_state, count, static_cast<hipStream_t>(stream));
  HIP_TRY(c, hipGetLastError());
  return ART_OK;
}

}  // extern "C"
