/*
 * art_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, IEEE binary32, no FMA contraction) of the reference's hot path:
 *   Jobs/AudioRaytracerJobBatched.cs, Jobs/AudioPermeationJobBatched.cs, Jobs/ProcessAudioDataJob.cs
 * plus the Unity.Mathematics 1.3.2 primitives they use.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline. The product (libart.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" by the reference — the reference is a Unity/Burst C# project
 * with no tests, no fixtures and no buildable toolchain here. This oracle is
 * pinned by hand-derived known-answer tests (tests/test_oracle_kats.py, SURVEY.md §8c K1–K12).
 */
#ifndef ART_ORACLE_H
#define ART_ORACLE_H

#include <stdint.h>
#include "../include/art.h"
#include "../include/art_dsp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Unity.Mathematics conversions (App. A.1) */
uint16_t or_f32tof16(float x);
void or_f32tof16_range(uint32_t first, uint32_t count, uint16_t* out);
float or_f16tof32(uint16_t h);

/* Jobs/FibonacciDirectionsJobParallel.cs:15-35 (host libm cosf/sinf). */
void or_fibonacci_directions(int32_t count, art_half3* out);

/* Run one frame for fan_count fans, exactly as AudioRayTracer.OnUpdate schedules it
 * (Audio/AudioRayTracer.cs:161-237): per fan, batches Execute(start, min(bs, R-start)) run in
 * ascending order (sequential-batch semantics), raytrace then permeation then reduce (+DSP).
 * threads: worker threads (one task per fan); 0 = 1.  counts may be NULL.
 * Returns 0 or a negative ART_E_* code. */
int or_run_frame(const art_frame_desc* desc, const art_fan* fans, int32_t fan_count,
                 int32_t threads, art_test_counts* counts);

/* Per-sample spatializer DSP (AudioSpatializer.OnAudioFilterRead, SURVEY.md §8 f rank 1). */
int or_dsp_process(const art_spatializer_settings* settings, art_audio_source* sources, int32_t count,
                   int32_t sample_rate);

/* Individual primitives, exposed for known-answer tests. */
int or_ray_intersects_aabb(const float o[3], const float d[3], const float c[3], const float h[3], float* dist);
int or_ray_intersects_sphere(const float o[3], const float d[3], const float c[3], float r, float* dist);
int or_ray_intersects_obb(const float o[3], const float d[3], const float c[3], const float h[3],
                          const float q[4], float* dist);
void or_half_quaternion_value(uint16_t x, uint16_t y, uint16_t z, float q[4]);
void or_quat_inverse(const float q[4], float out[4]);
void or_quat_mul_vec(const float q[4], const float v[3], float out[3]);

#ifdef __cplusplus
}
#endif
#endif
