// art_cpu.hpp — the CPU backend behind art_create(device_mask = 0) (art_cpu.cpp).
#pragma once

#include "../../include/art.h"

namespace art {

struct CpuEngine;

// Colliders of a resident-store frame (art_colliders.h): the records of the last sync.
struct CpuColliders {
  const art_sphere* sph; int ns;
  const art_aabb* aabb; int na;
  const art_obb* obb; int no;
};

CpuEngine* cpu_create(int threads);  // threads <= 0: ART_CPU_THREADS or the hardware threads
void cpu_destroy(CpuEngine* e);
int cpu_threads(const CpuEngine* e);
// Decode the frame's inputs (copied: the caller may reuse them on return) and start the fans on
// the worker threads; outputs go straight into the caller's fan arrays.
int cpu_schedule(CpuEngine* e, const art_frame_desc* d, const art_fan* fans, int fan_count, const CpuColliders* resident,
                 bool count);
bool cpu_is_completed(CpuEngine* e);
void cpu_complete(CpuEngine* e, art_test_counts* out);  // blocks; out (optional) = the frame's test counts

}  // namespace art
