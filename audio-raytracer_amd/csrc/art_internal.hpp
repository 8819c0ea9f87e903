// art_internal.hpp — device-side records and kernel launch interface (internal to libart.so).
//
// Data layout in HBM (one scene = one contiguous device allocation):
//   SphereRec[ns] | AabbRec[na] | ObbRec[no] | targets float3[T] | dirs half3[R] | curves
// Records are 16-B aligned so the wave-uniform collider loop fetches them with scalar
// (SMEM) loads: every lane of a wave tests the same collider at the same time, so the collider
// lives in SGPRs and costs no VGPRs, LDS traffic or vector-memory bandwidth.
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/art.h"
#include "../../include/art_dsp.h"

namespace art {

constexpr int kMaxTargets = 256;
constexpr int kRtBlock = 256;

enum : int { kNone = 0, kAabb = 1, kObb = 2, kSphere = 3 };  // Enums/ColliderType.cs:4-10

// Hot records hold only what the intersection sweeps read (two records per 64-B line for
// spheres and AABBs); cold records hold what reflection, echo and permeation read per hit.
struct alignas(16) SphereRec {  // 32 B
  float cx, cy, cz, r2;         // r2 = Radius * Radius (AudioRaytracerJobBatched.cs:328)
  int tid, pad0, pad1, pad2;    // AudioTargetId
};
struct alignas(16) SphereCold {  // 16 B
  float density, absorption, echo, pad;
};
struct alignas(16) AabbRec {  // 32 B
  float mnx, mny, mnz;        // Center - halfExtents (:286)
  int tid;
  float mxx, mxy, mxz;        // Center + halfExtents (:287)
  float pad;
};
struct alignas(16) AabbCold {  // 48 B
  float cx, cy, cz, absorption;
  float hx, hy, hz, echo;
  float density, pad0, pad1, pad2;
};
struct alignas(16) ObbRec {  // 64 B
  float cx, cy, cz;
  int tid;
  float qx, qy, qz, qw;        // stored rotation, decoded + normalized (halfQuaternion.cs:34-46)
  float lmnx, lmny, lmnz, pad0;  // float3.zero - halfExtents (:319 -> :286)
  float lmxx, lmxy, lmxz, pad1;  // float3.zero + halfExtents
};
struct alignas(16) ObbCold {  // 48 B
  float iqx, iqy, iqz, iqw;    // inverse(stored) (ReflectRay :489, permeation ShootRayCast :174)
  float hx, hy, hz, echo;
  float absorption, density, pad0, pad1;
};

// Broad-phase bounds of one collider (global order: spheres, AABBs, OBBs). A segment set whose
// bounding box B can be blocked by the collider only if [lo - m, hi + m] overlaps B, with the
// error margin m = factor * (scale + Omax) (Omax bounds |o|_1 + maxd over the set): see
// DESIGN.md §5 (broad phase). fscale = factor * scale, so a test computes m = fscale + factor * Omax
// (one FMA); a node keeps the largest fscale and factor of its colliders. Non-finite colliders get
// infinite bounds (always candidates).
struct alignas(16) CullRec {
  float lox, loy, loz, fscale;
  float hix, hiy, hiz, factor;
};

struct DevScene {
  const SphereRec* sph; const SphereCold* sphc; int ns;
  const AabbRec* aabb; const AabbCold* aabbc; int na;
  const ObbRec* obb; const ObbCold* obbc; int no;
  const float* targets; int T;    // float3[T]
  const uint16_t* dirs; int R;    // half3[R] as 3 x u16
  const CullRec* cull;            // [ns + na + no]
  // BVH over all colliders (art_bvh.hip): a complete 4-ary tree in heap order (root 0, children
  // of node g at 4g + 1 .. 4g + 4) over a spatial order of the bounds' centres, kBvhLeaf colliders
  // per leaf; the leaves are nodes bvh_leaf0 .. bvh_leaf0 + 4^(levels - 1) - 1 (those past the
  // last collider are empty). A node's CullRec is the union of its colliders' bounds with their
  // largest fscale and factor; an empty node is stored at +infinity (lo = hi = +inf, art_bvh.hip cull_stored).
  const CullRec* bvh;
  const uint32_t* bvh_ref;        // [ns + na + no] in leaf order: type rank << 30 | in-type index
  const float4* bvh_leaf;         // [4^(levels-1) * kBvhLeaf] slots in leaf order, 64 B (32 B when the
                                  // scene has no OBBs): the hot record's test fields and the global order
                                  // code (rank << 28 | index; -1: empty slot) in the first 32 B (bvh_leaf_kernel)
  int bvh_levels;                 // 0: no BVH
  int bvh_leaf0;
  // Muffle candidate lists (art_cells.hip): for target t and direction cell c (a
  // cube map of kCellG x kCellG cells per face around the target), the colliders not owned by t
  // whose widened bounding sphere meets cell c's cone; entries (order code, distance from the
  // target to the sphere) at cell_ent[cell_start[(t * kCells + c) * 3 + type] ..), one list per
  // collider type (Sphere, AABB, OBB: muffle_kernel walks them with type-uniform tests), each by
  // ascending near bound. A target whose bound or list
  // overflowed (cell_ok[t] == 0) is tested against every collider instead.
  const uint32_t* cell_start;     // [T * kCells * 3 + 1]
  const uint2* cell_ent;          // [cell_cap]: (code, near bits), each cell's entries by ascending near_key
  const uint32_t* cell_ent32;     // the same lists in 4-B entries (in-type index | near_key << 16), when
  uint32_t cell_compact;          //   cell_compact (every type's count < 2^16)
  const float* cell_far;          // [T]: the segment length the lists were built for
  const uint32_t* cell_ok;        // [T]
  uint32_t cell_cap;
};
// Motion slack of a listed collider (bounding radius r): the cell lists are built for its bounding
// sphere grown by this much, so they stay valid while the collider keeps its extents and owner and
// its centre stays within half of it of where the lists were built; art_colliders_sync then refits
// the BVH and skips the list rebuild. Units are scene units (Unity metres).
#ifndef ART_CELL_SLACK_REL
#define ART_CELL_SLACK_REL 0.1f
#endif
#ifndef ART_CELL_SLACK_ABS
#define ART_CELL_SLACK_ABS 0.2f
#endif
__host__ __device__ inline float cell_slack(float r) { return ART_CELL_SLACK_REL * r + ART_CELL_SLACK_ABS; }
constexpr int kCellG = 32;                   // cells per cube-face axis
constexpr int kCells = 6 * kCellG * kCellG;  // cells per target
// Cell cone (host table, art_capi.cpp): unit axis and cos / sin of the half-angle plus slack.
struct alignas(16) CellCone {
  float ax, ay, az, cos_a;
  float sin_a, pad0, pad1, pad2;
};
constexpr int kBvhLeaf = 4;        // colliders per leaf
constexpr int kBvhMaxLevels = 12;  // up to kBvhLeaf * 4^11 = 2^24 colliders per scene
constexpr int kBvhStack = 3 * (kBvhMaxLevels - 1);  // u32 node ids per traversal stack
constexpr long long kMaxColliders = (long long)kBvhLeaf << (2 * (kBvhMaxLevels - 1));

struct SortBufs {
  float* box;                     // 6 floats
  uint32_t* keys; uint32_t* keys_s; int* vals; int* perm;
  void* temp; size_t temp_bytes;
  CullRec* bvh; uint32_t* bvh_ref;  // BVH nodes (bvh_node_count) and leaf references
  uint32_t* bvh_pos;                // leaf position of each collider (global order): bvh_ref's inverse
  float4* bvh_leaf;                 // leaf slots (bvh_slot_count)
  void* kd;                         // kd leaf-order scratch (kd_scratch_bytes; NULL: Morton order)
};
// per-sample spatializer DSP (art_dsp.hip)
int dsp_source_params(const art_spatializer_settings& st, const art_audio_source& src, int sample_rate,
                      art_dsp_source_params& p);
void launch_dsp(float* data, unsigned long long data_bytes, const long long* offsets, const int* frames_of,
                int frames_all, const art_dsp_source_params* params, art_dsp_state* state, int count, hipStream_t st);

// Dirty records of a resident-store sync (art_colliders_sync): the update image (indices and
// records per kind) and the resident lists and decoded records they are scattered into.
struct ScatterArgs {
  const int* idx_s; const art_sphere* rec_s; int ds;
  const int* idx_a; const art_aabb* rec_a; int da;
  const int* idx_o; const art_obb* rec_o; int dob;
  art_sphere* sph; art_aabb* aabb; art_obb* obb;
  int ns, na;
  SphereRec* osph; SphereCold* osphc; AabbRec* oaabb; AabbCold* oaabbc; ObbRec* oobb; ObbCold* oobbc; CullRec* cull;
};
// Scenes up to this many colliders sync and refit in one workgroup (launch_sync_refit).
constexpr long long kSyncRefitMax = 1 << 16;
// The scatter of a sync's dirty records and the refit of the bound scene's BVH in one launch
// (sc: the bound scene with the store's records); false (nothing launched) for larger scenes or
// scenes without a BVH.
bool launch_sync_refit(const ScatterArgs& a, DevScene& sc, const SortBufs& sb, hipStream_t st);

size_t sort_scene_temp_bytes(int n);
// Spatially sorted copies, chunk bounds and the BVH (art_bvh.hip), built per upload.
int launch_sort_scene(DevScene& sc, const SortBufs& sb, hipStream_t st);
// Node count of the BVH over n colliders (0 when n is 0 or above kMaxColliders), and its build
// (after launch_sort_scene's buffers are free again; same stream).
size_t bvh_node_count(int n);
size_t bvh_slot_count(int n);
size_t kd_scratch_bytes(int n);
int launch_build_bvh(DevScene& sc, const SortBufs& sb, hipStream_t st);
// Colliders moved, counts unchanged: recompute the sorted copies' records, chunk bounds and the
// BVH's bounds and leaf slots in place, keeping every order.
int launch_refit_scene(DevScene& sc, const SortBufs& sb, hipStream_t st);

// Muffle candidate lists (art_cells.hip): built after every scene upload / refit on stream st.
// Sort key of a cell entry's near bound (bits of a float): the top 16 bits of its non-negative
// value (0 for a bound <= 0), monotone in the bound, so a list sorted by it can stop at the first
// key above the segment's key.
__host__ __device__ inline uint32_t near_key(uint32_t near_bits) {
  return (int32_t)near_bits <= 0 ? 0u : near_bits >> 16;
}
struct CellBufs {
  const CellCone* cones;          // [kCells]
  float alpha_max;                // largest cone half-angle (with slack)
  uint32_t* count;                // [T * kCells * 3 + 1] entries per (cell, collider type)
  uint32_t* start;                // [T * kCells * 3 + 1] exclusive scan of count (DevScene::cell_start)
  uint32_t* cursor;               // [T * kCells * 3 + 1] scratch: the 256-counter block sums, then their offsets
  uint2* ent;                     // [cap] in fill order
  uint2* ent_s;                   // [cap] each cell's entries by ascending near bound (DevScene::cell_ent)
  uint32_t compact;               // 4-B entries in the same storage (DevScene::cell_compact)
  uint32_t* keys;                 // [2 * cap] sort keys (near_key) and their sorted copy
  float* far;                     // [T]: distance bound of t's segments
  uint32_t* ok;                   // [T]
  unsigned long long* tcount;     // [T] entries per target (cells_block_sum_kernel), for the capacity check
  uint32_t cap;                   // entry capacity; 0: no lists (cells_enabled false), every muffle ray tests every collider
  void* temp; size_t temp_bytes;  // (unused since round 5: no library scan or sort)
  void* geo;                      // [T * C] per-(target, collider) geometry (cells_geo_bytes)
  CullRec* box;                   // [1] the union of the colliders' bounds (cells_box_kernel: the BVH root's box)
};
size_t cells_scan_temp_bytes(int T, uint32_t cap);
size_t cells_geo_bytes(int T, int C);
bool cells_enabled(int T, int C);
size_t cells_entry_cap(int T, int C);
int launch_build_cells(DevScene& sc, const CellBufs& cb, hipStream_t st);

// Per-fan output block (byte offsets inside one fan's record; fan f starts at f * stride).
struct FanLayout {
  uint32_t stride;
  uint32_t settings_off, dsp_off, muffle_off, perm_off, echo_off, hit_points_off, hit_counts_off, hit_ids_off;
  int has_dsp, has_hits;
};

struct FrameParams {
  int S;          // fans in this launch
  int R, H, T, TC, bs, nb;
  float max_life, max_muffle;
  float muffle_eff, perm_strength, perm_eff, max_reverb;
  uint32_t stages;
  // DSP
  float dl_min, dl_max, db_min, db_max, mc_min, mc_max;
  const float* vol_curve; int vol_n; float vol_len;
  const float* muf_curve; int muf_n; float muf_len;
  int sample_rate;
  unsigned long long* exec;  // executed-work counters (ExecSlot order) or nullptr
};

// Slots of FrameParams::exec (art_exec_counts order). The per-test slots 0..5 are written per
// kernel family at a group offset (nearest traversals, echo traversals, muffle rays); the host
// sums the groups for the totals and reports each group (art_exec_counts.by_kernel).
enum ExecSlot { kExecSphere = 0, kExecAabb = 1, kExecObb = 2, kExecCullBox = 3, kExecCellEntries = 4, kExecMuffleFallback = 5,
                kExecEchoPairs = 6, kExecBounce0 = 8, kExecBounces = 16, kExecNearest = 24, kExecEcho = 32, kExecMuffle = 40,
                kExecGroup = 8, kExecSlots = 48 };

// Device counters for the counting variant, in art_test_counts order.
struct DevCounts { unsigned long long v[9]; };

// --- launchers (art_kernels.hip) ---
void launch_prep(const art_sphere* sph, int ns, const art_aabb* aabb, int na, const art_obb* obb, int no,
                 SphereRec* osph, SphereCold* osphc, AabbRec* oaabb, AabbCold* oaabbc, ObbRec* oobb, ObbCold* oobbc,
                 CullRec* cull, hipStream_t st);
void launch_fibonacci(int count, art_half3* out, hipStream_t st);
void launch_half_range(uint32_t first, uint32_t count, uint16_t* out, hipStream_t st);
void launch_recip_range(uint32_t first, uint32_t count, uint32_t* out, hipStream_t st);
void launch_scatter_prep(const int* idx_s, const art_sphere* rec_s, int ds, const int* idx_a, const art_aabb* rec_a,
                         int da, const int* idx_o, const art_obb* rec_o, int dob, art_sphere* sph, art_aabb* aabb,
                         art_obb* obb, int ns, int na, SphereRec* osph, SphereCold* osphc, AabbRec* oaabb,
                         AabbCold* oaabbc, ObbRec* oobb, ObbCold* oobbc, CullRec* cull, hipStream_t st);
void launch_raytrace(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                     uint8_t* block, uint32_t* muffle_acc, DevCounts* counts, hipStream_t st);
// Bytes of the visibility pair buffer of launch_raytrace_fast for this frame (fp.S fans).
size_t fast_pair_bytes(const FrameParams& fp);
// Fans per launch_raytrace_fast call (32-bit pair slots, accumulator indices and block offsets).
int fast_fans_per_launch(int R, int H, int T, int TC, uint32_t stride);
// The throughput raytrace stage (art_trace.hip): per bounce nearest_first_kernel + path_kernel
// (+ the bounce's echo vis_kernel), then muffle_kernel. Any target count, every DevScene with a BVH
// and cell lists. echo_st (optional, with two events): the echo traversals run there, beside the
// next bounces and the muffle kernel on st, joined at the end.
struct SideStream {
  hipStream_t st = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
// Per-kernel timing marks (ART_CTX_TIME_EACH_KERNEL): an event pair recorded around each kernel of
// the raytrace stage on the stream it is launched on, with its kernel family (art_kernel_times
// kernel_ms order). Marks stop being recorded once the pairs run out (used counts those recorded).
enum MarkKind { kMarkNearest = 0, kMarkEchoMuffle = 1, kMarkEcho = 2, kMarkMuffle = 3, kMarkKinds = 4 };
struct KernelMarks {
  hipEvent_t* ev = nullptr;  // [2 * cap]
  int* kind = nullptr;       // [cap]
  int cap = 0, used = 0;
  int dropped = 0;           // launches that found no pair left (their family's time is then incomplete)
};
void launch_raytrace_fast(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                          uint8_t* block, uint32_t* muffle_acc, const int* ray_order, void* pair_buf,
                          uint32_t* pair_count, hipStream_t st, const SideStream& echo, KernelMarks* marks = nullptr);
void launch_permeate(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                     uint8_t* block, const int2* slot_batch, hipStream_t st);
// (the collider sweep of every loss ray, art_kernels.hip: the reference-order and counting frames)
void launch_permeate_sweep(const DevScene& sc, const FrameParams& fp, const FanLayout& L, const float* origins,
                     uint8_t* block, const int2* slot_batch, hipStream_t st);
void launch_perm_count(const DevScene& sc, const FrameParams& fp, const float* origins, DevCounts* counts,
                       unsigned long long* nhit, hipStream_t st);
void launch_reduce(const DevScene& sc, const FrameParams& fp, const FanLayout& L, uint8_t* block,
                   const uint32_t* muffle_acc, const uint8_t* muffle_reset, hipStream_t st, const float* perm_in = nullptr,
                   uint8_t* host_out = nullptr);

}  // namespace art
