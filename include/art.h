/*
 * art.h — C ABI of the MI355X-native audio ray tracer (drop-in for the reference's
 * per-frame job graph).
 *
 * Reference surface this replaces (paths relative to "Assets/C# Scripts/" of
 * FirePixel8422/Audio-Raytracer):
 *   - the job parameter blocks  Jobs/AudioRaytracerJobBatched.cs:12-52,
 *                               Jobs/AudioPermeationJobBatched.cs:10-27,
 *                               Jobs/ProcessAudioDataJob.cs:10-28
 *     filled at Audio/AudioRayTracer.cs:163-234               -> art_frame_desc + art_fan
 *   - IJobParallelForBatch.Schedule(rayCount, batchSize)   (AudioRayTracer.cs:191,213)
 *     + IJob.Schedule(handleA) + JobHandle.CombineDependencies (:213,237)
 *                                                            -> art_schedule
 *   - JobHandle.IsCompleted  (AudioRayTracer.cs:95)          -> art_is_completed
 *   - JobHandle.Complete()   (AudioRayTracer.cs:97,244)      -> art_complete
 *
 * All entry points are extern "C", take plain pointers and sizes, and never throw.
 * Return 0 (ART_OK) on success, a negative ART_E_* code on error; art_last_error()
 * gives the message.  art_create(mask != 0) needs the HIP devices it names and fails loudly
 * (ART_E_DEVICE) without them: a GPU context never falls back to the CPU.  art_create(0)
 * selects the CPU backend explicitly (worker threads over fans, the jobs' own loop order;
 * the host entry points of this header and art_colliders.h only).
 */
#ifndef ART_H
#define ART_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define ART_API __attribute__((visibility("default")))
#else
#define ART_API
#endif

/* ------------------------------------------------------------------------------------------
 * Byte layouts.  Identical to the C# structs (LayoutKind.Sequential, 2-byte packing), so a
 * NativeArray<T>.GetUnsafeReadOnlyPtr() can be passed straight through P/Invoke.
 * Every uint16_t "half" field holds IEEE binary16 bits (Unity.Mathematics.half.value).
 * ---------------------------------------------------------------------------------------- */
#pragma pack(push, 2)
/* Unity.Mathematics.half3 (6 B) */
typedef struct { uint16_t x, y, z; } art_half3;

/* DataTypes/Collider Structs/AudioMaterialProperties.cs:10-16 (6 B) */
typedef struct { uint16_t absorption, density, echo; } art_material;

/* DataTypes/Collider Structs/ColliderAABBStruct.cs:10-14 (20 B). size = half-extents. */
typedef struct {
    art_half3 center;
    art_half3 size;
    art_material material;
    int16_t audio_target_id; /* -1 = not owned by an audio target */
} art_aabb;

/* DataTypes/Collider Structs/ColliderOBBStruct.cs:10-24 (26 B).
 * rot_{x,y,z} = halfQuaternion (DataTypes/halfQuaternion.cs:9-11) of the INVERSE rotation
 * (Audio/Colliders/AudioOBBCollider.cs:59), sign-flipped so that w >= 0. */
typedef struct {
    art_half3 center;
    art_half3 size;
    uint16_t rot_x, rot_y, rot_z;
    art_material material;
    int16_t audio_target_id;
} art_obb;

/* DataTypes/Collider Structs/ColliderSphereStruct.cs:10-14 (16 B) */
typedef struct {
    art_half3 center;
    uint16_t radius;
    art_material material;
    int16_t audio_target_id;
} art_sphere;
#pragma pack(pop)

/* DataTypes/AudioTargetRTSettings.cs:11-16 (24 B) */
typedef struct {
    float muffle_strength;
    float reverb_strength;
    float reverb_volume;
    float perceived_position[3];
} art_target_settings;

/* Per-target DSP parameters derived from the settings (config 5's "reverb DSP" pass):
 *   dry_level     = lerp(DryLevel.min, DryLevel.max, ReverbStrength)      AudioSpatializer.cs:58
 *   dry_boost     = lerp(DryBoost.min, DryBoost.max, VolCurve(ReverbVolume))  ReverbDSP.cs:12-13
 *   muffle_cutoff = lerp(Cutoff.max, Cutoff.min, MuffleCurve(MuffleStrength))  MuffleDSP.cs:24-26
 *   muffle_alpha  = dt / (rc + dt), rc = 1/(cutoff*2pi), dt = 1/sampleRate  MuffleDSP.cs:40-42
 *   muffle_active = MuffleStrength > 0  (MuffleDSP.cs:22); cutoff/alpha are 0 when inactive. */
typedef struct {
    float dry_level;
    float dry_boost;
    float muffle_cutoff;
    float muffle_alpha;
    int32_t muffle_active;
    int32_t reserved;
} art_dsp_params; /* 24 B */

/* A baked NativeSampledAnimationCurve (DataTypes/NativeSampledAnimationCurve.cs:22-29; evaluated as :64-89). */
typedef struct {
    const float* baked;   /* float[sample_count] */
    int32_t sample_count; /* >= 2 */
    float length;         /* time of the last key */
} art_curve;

/* Spatializer settings used by the DSP-parameter stage (DataTypes/AudioSpatializerSettings.cs). */
typedef struct {
    float reverb_dry_level_min, reverb_dry_level_max;
    float reverb_dry_boost_min, reverb_dry_boost_max;
    float muffle_cutoff_min, muffle_cutoff_max;
    art_curve reverb_volume_curve;
    art_curve muffle_curve;
    int32_t sample_rate;
} art_dsp_desc;

/* Stage bits (art_frame_desc.stages). RAYTRACE and PERMEATE run concurrently in the reference
 * (AudioRayTracer.cs:191,213); REDUCE (ProcessAudioDataJob) depends on both (:237). */
#define ART_STAGE_RAYTRACE   0x1u
#define ART_STAGE_PERMEATE   0x2u
#define ART_STAGE_REDUCE     0x4u
#define ART_STAGE_DSP_PARAMS 0x8u
#define ART_STAGE_ALL        0xFu

/* Shared, per-frame scene + parameters (one AudioRayTracer's job fields, minus the origin). */
typedef struct {
    const art_half3* ray_directions; int32_t ray_count;           /* R = RayDirections.Length */
    const art_aabb* aabb_colliders; int32_t aabb_count;
    const art_obb* obb_colliders; int32_t obb_count;
    const art_sphere* sphere_colliders; int32_t sphere_count;
    const float* audio_target_positions; int32_t audio_target_count; /* float3[T] */
    float max_ray_life;
    int32_t max_hits_per_ray;                                      /* H = maxBounces + 1 (byte) */
    float max_muffle_hit_distance;
    float muffle_effectiveness;
    float permeation_strength_per_ray;
    float permeation_effectiveness;
    float max_reverb_distance;
    int32_t batch_size;   /* IJobParallelForBatch indicesPerJobCount = max(1, ceil(R/TC)) (AudioRayTracer.cs:161) */
    int32_t batch_slots;  /* TC = MuffleRayHits.Length / T (AudioTargetManager.cs:112-122) */
    uint32_t stages;      /* ART_STAGE_* */
    const art_dsp_desc* dsp; /* required iff stages & ART_STAGE_DSP_PARAMS */
} art_frame_desc;

/* One fan == one AudioRayTracer evaluation: origin in, per-fan arrays out.
 * echo/muffle/permeation arrays are IN/OUT exactly like the reference's persistent
 * NativeArrays: slots no batch resets keep their previous contents (App. B Q1/Q7/Q18 of
 * SURVEY.md; only possible at batch_slots > 1). */
typedef struct {
    float origin[3];                    /* RayOrigin */
    uint16_t* echo_ray_distances;       /* half[R*H]   EchoRayDistances */
    uint16_t* muffle_ray_hits;          /* u16[TC*T]   MuffleRayHits */
    float* permeation_power_remains;    /* f32[TC*T]   PermeationPowerRemains */
    art_target_settings* settings;      /* [T]         AudioTargetSettings */
    art_dsp_params* dsp_params;         /* [T] or NULL */
    art_half3* ray_hit_points;          /* [R*H] or NULL  RayHitResults (editor-only in the reference) */
    uint8_t* ray_hit_counts;            /* [R] or NULL    RayHitResultCounts (editor-only) */
    uint32_t* ray_hit_ids;              /* [R*H] or NULL  (build extension) the collider each hit struck:
                                         * ART_HIT_ID(type, index), written and reset exactly where
                                         * RayHitResults is (:78, :197); ART_HIT_NONE in reset slots */
} art_fan;

/* Hit identity = the (hitColliderType, hitAABB / hitOBB / hitSphere) pair ShootRayCast returns
 * (Jobs/AudioRaytracerJobBatched.cs:225-280): ColliderType (Enums/ColliderType.cs: AABB 1, OBB 2,
 * Sphere 3) in the top two bits, the collider's index in its own array below. */
#define ART_COLLIDER_AABB   1u
#define ART_COLLIDER_OBB    2u
#define ART_COLLIDER_SPHERE 3u
#define ART_HIT_ID(type, index) (((uint32_t)(type) << 30) | (uint32_t)(index))
#define ART_HIT_NONE 0xFFFFFFFFu

/* Number of intersection-routine calls the reference algorithm executes (SURVEY.md §8 d). */
typedef struct {
    uint64_t rt_sphere, rt_aabb, rt_obb;                  /* AudioRaytracerJobBatched: nearest + echo + muffle */
    uint64_t perm_hit_sphere, perm_hit_aabb, perm_hit_obb; /* AudioPermeationJobBatched.ShootRayCast */
    uint64_t perm_loss_sphere, perm_loss_aabb, perm_loss_obb; /* ShootPermeationRayCast */
} art_test_counts;

typedef struct art_ctx art_ctx;
typedef uint64_t art_handle;

/* Error codes */
#define ART_OK             0
#define ART_E_INVALID     -1  /* bad argument / length mismatch */
#define ART_E_DEVICE      -2  /* HIP error or no device */
#define ART_E_UNSUPPORTED -3
#define ART_E_NOMEM       -4
#define ART_E_STATE       -5  /* unknown handle, frame already in flight, ... */

/* device_mask: bit i selects HIP device i; fans are sharded contiguously over the selected
 * devices; fails with ART_E_DEVICE when a selected device is missing.  device_mask 0: the CPU
 * backend (Unity's Burst/CPU job path), ART_CPU_THREADS worker threads (default:
 * the hardware threads); frames run asynchronously between art_schedule and art_complete. */
ART_API int art_create(uint32_t device_mask, art_ctx** out);
ART_API void art_destroy(art_ctx* ctx);
ART_API const char* art_last_error(const art_ctx* ctx);

/* Schedule one frame for fan_count fans. Inputs are copied before this returns (the caller may
 * reuse them); the fans' output arrays must stay valid until art_complete(handle). */
ART_API int art_schedule(art_ctx* ctx, const art_frame_desc* desc, const art_fan* fans,
                         int32_t fan_count, art_handle* out);
/* 1 if done, 0 if still running, <0 on error. */
ART_API int art_is_completed(art_ctx* ctx, art_handle h);
/* Block until done, then write the outputs into the caller's arrays. */
ART_API int art_complete(art_ctx* ctx, art_handle h);

/* Test counts of the last completed frame (requires ART_CTX_COUNT_TESTS). */
#define ART_CTX_COUNT_TESTS 0x1u
ART_API int art_set_flags(art_ctx* ctx, uint32_t flags);
ART_API int art_last_test_counts(art_ctx* ctx, art_test_counts* out);

/* ABI version: major<<16 | minor */
ART_API uint32_t art_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ART_H */
