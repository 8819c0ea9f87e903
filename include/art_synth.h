/*
 * art_synth.h — deterministic synthetic scenes for benchmarks and tests.
 *
 * Input generation only (no hot-path computation): the same bytes feed the GPU path and the
 * CPU oracle. Ray directions follow Jobs/FibonacciDirectionsJobParallel.cs:25-34 (host libm
 * cosf/sinf, Unity f32tof16 rounding); the resulting half bits are the input contract.
 */
#ifndef ART_SYNTH_H
#define ART_SYNTH_H

#include "art.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Which collider type each audio target owns (App. D 6). */
#define ART_OWN_SPHERE 0
#define ART_OWN_AABB 1
#define ART_OWN_OBB 2

typedef struct {
    int32_t sphere_count, aabb_count, obb_count; /* totals, owned colliders included */
    int32_t target_count;                        /* T */
    int32_t fan_count;                           /* S */
    int32_t ray_count;                           /* R */
    int32_t owned_type;                          /* ART_OWN_* */
    uint64_t seed;                               /* 20260206 + config index */
} art_synth_config;

/* Caller allocates: sph[sphere_count], aabb[aabb_count], obb[obb_count], targets[3*T],
 * origins[3*S], dirs[R]. Owned colliders come first in their type array (index t for target t). */
ART_API int art_synth_scene(const art_synth_config* cfg, art_sphere* sph, art_aabb* aabb, art_obb* obb,
                            float* targets, float* origins, art_half3* dirs);

/* Jobs/FibonacciDirectionsJobParallel.cs:15-35 */
ART_API void art_fibonacci_directions(int32_t count, art_half3* out);

/* Unity.Mathematics f32tof16 / f16tof32 (host), exported for bindings and tests. */
ART_API uint16_t art_f32tof16(float x);
ART_API float art_f16tof32(uint16_t h);
/* Bulk host f32tof16 of the float bit patterns first_bits, first_bits + 1, ... (count of them,
 * wrapping past 0xFFFFFFFF): out[i] = art_f32tof16(asfloat(first_bits + i)). */
ART_API void art_f32tof16_range(uint32_t first_bits, uint32_t count, uint16_t* out);

#ifdef __cplusplus
}
#endif
#endif /* ART_SYNTH_H */
