/*
 * art_colliders.h — device-resident collider store (SURVEY.md §8 f rank 2, the collider upload
 * path on the near side of the ray tracer).
 *
 * Reference (paths relative to "Assets/C# Scripts/"):
 *   NativeJobBatch<T>                       DataTypes/NativeJobBatch.cs:8-56
 *     Add                                   :27-30   (NextBatch.Add)
 *     RemoveAtSwapBack                      :31-34
 *     this[index] set                       :14-18   (an in-place update of NextBatch)
 *     UpdateJobBatch                        :36-50   (memcpy NextBatch -> JobBatch, every frame)
 *   AudioColliderManager.AddColiderToSystem Audio/AudioColliderManager.cs:42-62 (id = NextBatch.Length:
 *                                           Colliders/AudioOBBCollider.cs:18-22, AudioAABBCollider.cs:14-17,
 *                                           AudioSphereCollider.cs:14-17)
 *   AudioColliderManager.SwapRemove         Audio/AudioColliderManager.cs:90-105 (invalid ids skipped)
 *   AudioColliderManager.UpdateColiderInSystem :107-110 (collider[id] = GetBakedColliderStruct(),
 *                                           AudioOBBCollider.cs:23-26)
 *   AudioColliderManager.UpdateJobBatch     :115-122 (called once per frame, AudioRayTracer.cs:155)
 *
 * The reference copies every collider into the job snapshot each frame, and a GPU port of that
 * would upload every collider every frame. Here the context keeps the three collider lists
 * resident in HBM as decoded SoA records. The host side keeps the NextBatch mirror: add / set /
 * remove-at-swap-back touch only the mirror and mark records dirty. art_colliders_sync is
 * UpdateJobBatch: it uploads only the dirty records (one H2D copy) and decodes them on the device
 * (one kernel). With ART_CTX_RESIDENT_COLLIDERS set, art_schedule and art_scene_bind take the
 * colliders from the last sync (the JobBatch snapshot) instead of the desc's arrays.
 *
 * Baking a collider struct from its transform (GetBakedColliderStruct, AudioOBBCollider.cs:31-66)
 * stays with the caller: it uses the engine's transform and quaternion math, and its result (the
 * 20/26/16-byte struct) is the contract.
 */
#ifndef ART_COLLIDERS_H
#define ART_COLLIDERS_H

#include "art.h"

#ifdef __cplusplus
extern "C" {
#endif

/* collider kinds */
#define ART_KIND_SPHERE 0  /* art_sphere (16 B) */
#define ART_KIND_AABB   1  /* art_aabb (20 B) */
#define ART_KIND_OBB    2  /* art_obb (26 B) */

/* art_set_flags bit: frames read the resident store (desc collider arrays must be NULL / 0). */
#define ART_CTX_RESIDENT_COLLIDERS 0x20u

/* NativeJobBatch.Add: appends rec (a struct of the kind) to the kind's list; *out_id = its index
 * (the C# AudioColliderId). */
ART_API int art_collider_add(art_ctx* ctx, int32_t kind, const void* rec, int32_t* out_id);

/* NativeJobBatch[id] = rec (UpdateColiderInSystem). ART_E_INVALID if id is out of range. */
ART_API int art_collider_set(art_ctx* ctx, int32_t kind, int32_t id, const void* rec);

/* n updates of one kind in one call (ids[j] <- recs[j], recs packed back to back); all ids are
 * checked before anything changes. */
ART_API int art_collider_set_many(art_ctx* ctx, int32_t kind, const int32_t* ids, const void* recs, int32_t n);

/* RemoveAtSwapBack(id): the last record moves to id. Like AudioColliderManager.SwapRemove
 * (:92-93), an id out of range is skipped (returns ART_OK, nothing changes). */
ART_API int art_collider_remove_swapback(art_ctx* ctx, int32_t kind, int32_t id);

/* NativeJobBatch[id] get (the mirror, i.e. NextBatch, including unsynced changes). */
ART_API int art_collider_get(art_ctx* ctx, int32_t kind, int32_t id, void* rec);

/* NextBatch.Length of the kind (>= 0), or a negative error code. */
ART_API int art_collider_count(art_ctx* ctx, int32_t kind);

/* Drop every collider of every kind (the lists become empty; the next sync publishes that). */
ART_API int art_colliders_clear(art_ctx* ctx);

/* UpdateJobBatch for the three kinds: publish the mirror to every device of the context.
 * Stream-ordered, not synchronous: the dirty records' upload and decode are enqueued on the
 * context's stream ahead of the next frame (art_launch_device on another stream waits for them).
 * ART_E_STATE while a frame is in flight (the reference syncs after Complete). */
ART_API int art_colliders_sync(art_ctx* ctx);

/* What the last art_colliders_sync moved. */
typedef struct {
    int32_t dirty_records;   /* records uploaded and decoded */
    int32_t full_prep;       /* 1 if a count changed, so every record's bounds were rebuilt on the device */
    int32_t reallocated;     /* 1 if the device capacity grew (every record uploaded) */
    int32_t cells_rebuilt;   /* 1 if the muffle direction-cell lists were rebuilt (a record left its motion slack) */
    uint64_t bytes_uploaded; /* H2D bytes of the sync (indices + records) */
} art_collider_sync_stats;

ART_API int art_colliders_last_sync(art_ctx* ctx, art_collider_sync_stats* out);

#ifdef __cplusplus
}
#endif
#endif /* ART_COLLIDERS_H */
