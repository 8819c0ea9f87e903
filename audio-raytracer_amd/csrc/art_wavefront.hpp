// art_wavefront.hpp — device state of the per-bounce wavefront raytrace pipeline
// (art_wavefront.hip). One WfRay per (fan, ray), global ray id g = fan * R + ray.
#pragma once

#include <stdint.h>

#include "art_internal.hpp"

namespace art {

constexpr int kWfParts = 1;   // collider ranges (wf_visibility launches) per bounce
#ifndef ART_WF_CHUNK
#define ART_WF_CHUNK 256
#endif
constexpr int kWfChunk = ART_WF_CHUNK;  // colliders per chunk of the rotating sweep

struct alignas(16) WfRay {  // 48 B
  float ox, oy, oz, life;   // origin; after wf_nearest: the hit point (:111)
  float dx, dy, dz, dist;   // direction; distance of the current hit
  int code;                 // rank << 28 | index of the current hit, 0x7fffffff if none
  int hits;                 // cRayHits (:97)
  uint32_t active;          // bit q: visibility item q exists this bounce (0 echo, t+1 target t)
  uint32_t frozen;          // bit k: echo slot k is reset by a later batch (TC > 1, App. B Q1)
};

// One visibility item: a ready-to-sweep segment (the echo ray :124-130 or a muffle ray :158-165)
// written by wf_nearest, so a refill in wf_visibility is one 64-B load.
struct alignas(16) WfItem {  // 64 B
  float ox, oy, oz, dx;
  float dy, dz, ix, iy;
  float iz, a2, a4, maxd;
  int owner;                 // target whose colliders are skipped, 0x7fffffff for the echo ray
  uint32_t id;               // g * (T + 1) + q
  uint32_t pad0, pad1;
};

struct WfCounters {  // one per bounce (+1), zeroed at frame start
  uint32_t alive_n;                  // rays in this bounce's live list (bounce 0: implicit S*R)
  uint32_t items_n[kWfParts + 1];    // items entering collider range p
  uint32_t head[kWfParts];           // persistent-queue heads
  uint32_t pad[64 - 1 - (kWfParts + 1) - kWfParts];
};

struct WfArgs {
  const float* origins;      // float3[S]
  uint8_t* block;            // packed per-fan records
  uint32_t* muffle_acc;      // [S][TC][T]
  const int* ray_order;      // [R] direction-coherent visiting order
  WfRay* rays;               // [S*R]
  uint32_t* alive[2];        // ping-pong live lists [S*R]
  const uint32_t* alive_in;  // set per bounce
  uint32_t* alive_out;
  WfItem* items;             // [S*R*(T+1)] visibility items of the current bounce
  uint8_t* flags;            // [S*R*(T+1)] blocked flags of the current bounce
  WfCounters* cnt;           // [H+1]
};

int wf_persistent_blocks();
void wf_launch_bounce(const DevScene& sc, const FrameParams& fp, const FanLayout& L, WfArgs a, int bounce, int nparts,
                      int persistent_blocks, hipStream_t st);

}  // namespace art
