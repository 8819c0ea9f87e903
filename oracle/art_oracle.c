/*
 * art_oracle.c — TEST INFRASTRUCTURE ONLY (see art_oracle.h).
 *
 * A line-by-line CPU restatement of the reference's audio ray-tracing hot path in plain C.
 * Every function cites the reference file:line it follows. Paths are relative to
 * "/root/reference/Assets/C# Scripts/".
 *
 * Floating point: IEEE binary32 throughout, built with -ffp-contract=off and without
 * -ffast-math, matching Burst's default FloatMode (strict: no contraction, no reassociation,
 * correctly rounded + - * / sqrt).  Unity.Mathematics 1.3.2 primitives are restated in
 * section 1.  The parity contract is defined at TC = 1; for TC > 1 the
 * batches of one fan run in ascending order ("sequential-batch" semantics).
 *
 * Parity is UNPINNED by the reference (no tests/fixtures; Unity/Burst cannot run here); this
 * file is pinned by hand-derived known-answer tests in tests/test_oracle_kats.py.
 */
#include "art_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ========================================================================================
 * 1. Unity.Mathematics 1.3.2 restatement
 * ====================================================================================== */

typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;

static inline uint32_t asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* math.min / math.max (App. A.2): NaN in y returns x. */
static inline float umin(float x, float y) { return (y != y || x < y) ? x : y; }
static inline float umax(float x, float y) { return (y != y || x > y) ? x : y; }
/* math.sign (App. A.2) */
static inline float usign(float x) { return (x > 0.0f ? 1.0f : 0.0f) - (x < 0.0f ? 1.0f : 0.0f); }
/* math.saturate = clamp(x, 0, 1) = max(0, min(1, x)) */
static inline float usaturate(float x) { return umax(0.0f, umin(1.0f, x)); }
/* math.lerp(a, b, s) = a + s * (b - a) */
static inline float ulerp(float a, float b, float s) { return a + s * (b - a); }

/* math.f32tof16 (App. A.1). Round-half-up on bit 12 after truncation; the clamp constant is the
 * float literal 260042752.0f as in the package (it never clamps a finite input; |x| >= 65520 is
 * outside this path's contract). */
uint16_t or_f32tof16(float x)
{
    const int32_t infinity_32 = 255 << 23;
    const uint32_t msk = 0x7FFFF000u;
    uint32_t ux = asuint(x);
    uint32_t uux = ux & msk;
    uint32_t h = (uint32_t)(asuint(umin(asfloat(uux) * 1.92592994e-34f, 260042752.0f)) + 0x1000u) >> 13;
    h = ((int32_t)uux >= infinity_32) ? (((int32_t)uux > infinity_32) ? 0x7e00u : 0x7c00u) : h;
    return (uint16_t)(h | (ux & ~msk) >> 16);
}

/* Bulk form for the exhaustive checks: out[i] = or_f32tof16(asfloat(first + i)). */
void or_f32tof16_range(uint32_t first, uint32_t count, uint16_t* out)
{
    for (uint32_t i = 0; i < count; ++i) out[i] = or_f32tof16(asfloat(first + i));
}

/* math.f16tof32 (exact) */
float or_f16tof32(uint16_t hx)
{
    uint32_t x = hx;
    const uint32_t shifted_exp = (0x7c00u << 13);
    uint32_t uf = (x & 0x7fffu) << 13;
    uint32_t e = uf & shifted_exp;
    uf += (127u - 15u) << 23;
    uf += (e == shifted_exp) ? ((128u - 16u) << 23) : 0u;
    if (e == 0) uf = asuint(asfloat(uf + (1u << 23)) - 6.10351563e-05f);
    uf |= (x & 0x8000u) << 16;
    return asfloat(uf);
}

static inline f3 h3(art_half3 h) { f3 r = { or_f16tof32(h.x), or_f16tof32(h.y), or_f16tof32(h.z) }; return r; }
static inline art_half3 toh3(f3 v) { art_half3 r = { or_f32tof16(v.x), or_f32tof16(v.y), or_f32tof16(v.z) }; return r; }
static inline f3 v3(float x, float y, float z) { f3 r = { x, y, z }; return r; }
static inline f3 add3(f3 a, f3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub3(f3 a, f3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul3(f3 a, f3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 muls(f3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }   /* float3 * float */
static inline f3 smul(float s, f3 a) { return v3(s * a.x, s * a.y, s * a.z); }   /* float * float3 */
static inline f3 abs3(f3 a) { return v3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
static inline f3 min3v(f3 a, f3 b) { return v3(umin(a.x, b.x), umin(a.y, b.y), umin(a.z, b.z)); }
static inline f3 max3v(f3 a, f3 b) { return v3(umax(a.x, b.x), umax(a.y, b.y), umax(a.z, b.z)); }
static inline f3 rcp3(f3 a) { return v3(1.0f / a.x, 1.0f / a.y, 1.0f / a.z); }
/* dot: left to right, no contraction (App. A.3) */
static inline float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float dot4(f4 a, f4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
/* cross(x, y) = (x * y.yzx - x.yzx * y).yzx */
static inline f3 cross3(f3 x, f3 y)
{
    f3 c = v3(x.x * y.y - x.y * y.x, x.y * y.z - x.z * y.y, x.z * y.x - x.x * y.z);
    return v3(c.y, c.z, c.x);
}
/* rsqrt(x) = 1 / sqrt(x); normalize(v) = rsqrt(dot(v, v)) * v */
static inline float ursqrt(float x) { return 1.0f / sqrtf(x); }
static inline f3 normalize3(f3 v) { return smul(ursqrt(dot3(v, v)), v); }
static inline float length3(f3 v) { return sqrtf(dot3(v, v)); }
/* distance(x, y) = length(y - x) */
static inline float distance3(f3 x, f3 y) { return length3(sub3(y, x)); }
/* reflect(i, n) = i - 2f * n * dot(i, n) */
static inline f3 reflect3(f3 i, f3 n) { return sub3(i, muls(smul(2.0f, n), dot3(i, n))); }

/* mul(quaternion q, float3 v): t = 2 * cross(q.xyz, v); v + q.w * t + cross(q.xyz, t) */
static inline f3 qmul(f4 q, f3 v)
{
    f3 qv = v3(q.x, q.y, q.z);
    f3 t = smul(2.0f, cross3(qv, v));
    return add3(add3(v, smul(q.w, t)), cross3(qv, t));
}
/* inverse(q) = rcp(dot(q, q)) * q * (-1, -1, -1, 1) */
static inline f4 qinverse(f4 q)
{
    float r = 1.0f / dot4(q, q);
    f4 o = { (r * q.x) * -1.0f, (r * q.y) * -1.0f, (r * q.z) * -1.0f, (r * q.w) * 1.0f };
    return o;
}
/* normalize(quaternion q) = rsqrt(dot(q, q)) * q */
static inline f4 qnormalize(f4 q)
{
    float r = ursqrt(dot4(q, q));
    f4 o = { r * q.x, r * q.y, r * q.z, r * q.w };
    return o;
}

/* halfQuaternion.QuaternionValue getter — DataTypes/halfQuaternion.cs:34-46 */
static f4 half_quaternion_value(uint16_t hx, uint16_t hy, uint16_t hz)
{
    float xx = or_f16tof32(hx);
    float yy = or_f16tof32(hy);
    float zz = or_f16tof32(hz);
    float wSquared = 1.0f - (xx * xx + yy * yy + zz * zz);
    float w = wSquared > 0.0f ? sqrtf(wSquared) : 0.0f;
    f4 q = { xx, yy, zz, w };
    return qnormalize(q);
}

/* ColliderOBBStruct.Rotation getter — DataTypes/Collider Structs/ColliderOBBStruct.cs:14-21 */
static inline f4 obb_rotation(const art_obb* o) { return half_quaternion_value(o->rot_x, o->rot_y, o->rot_z); }

/* ========================================================================================
 * 2. Counters (SURVEY.md §8 d: one "test" = one call of an intersection routine)
 * ====================================================================================== */
typedef struct {
    uint64_t rt_sphere, rt_aabb, rt_obb;
    uint64_t ph_sphere, ph_aabb, ph_obb;
    uint64_t pl_sphere, pl_aabb, pl_obb;
} counters;

/* ========================================================================================
 * 3. AudioRaytracerJobBatched — Jobs/AudioRaytracerJobBatched.cs
 * ====================================================================================== */

#define EPSILON 0.0001f /* :57 */

enum { CT_NONE = 0, CT_AABB = 1, CT_OBB = 2, CT_SPHERE = 3 }; /* Enums/ColliderType.cs:4-10 */

typedef struct {
    f3 RayOrigin;
    const art_half3* RayDirections; int RayDirectionsLength;
    const art_aabb* AABBColliders; int AABBColliderCount;
    const art_obb* OBBColliders; int OBBColliderCount;
    const art_sphere* SphereColliders; int SphereColliderCount;
    const float* AudioTargetPositions; int TotalAudioTargets;
    float MaxRayLife;
    uint8_t MaxHitsPerRay;
    art_half3* RayHitResults;      /* may be NULL (editor-only) */
    uint8_t* RayHitResultCounts;   /* may be NULL (editor-only) */
    uint32_t* RayHitIds;           /* may be NULL (build extension: ShootRayCast's type << 30 | index) */
    uint16_t* EchoRayDistances;
    uint16_t* MuffleRayHits; int MuffleRayHitsLength;
    float MaxMuffleHitDistance;
    counters* cnt;
} rt_job;

static inline f3 target_pos(const float* p, int t) { return v3(p[3 * t + 0], p[3 * t + 1], p[3 * t + 2]); }

/* RayIntersectsAABB — :284-308 */
static int rt_ray_intersects_aabb(f3 rayOrigin, f3 rayDir, f3 Center, f3 halfExtents, float* distance)
{
    f3 mn = sub3(Center, halfExtents);
    f3 mx = add3(Center, halfExtents);
    f3 invDir = rcp3(rayDir);
    f3 t0 = mul3(sub3(mn, rayOrigin), invDir);
    f3 t1 = mul3(sub3(mx, rayOrigin), invDir);
    f3 tmin = min3v(t0, t1);
    f3 tmax = max3v(t0, t1);
    float tNear = umax(umax(tmin.x, tmin.y), tmin.z);
    float tFar = umin(umin(tmax.x, tmax.y), tmax.z);
    if (tNear > tFar || tFar < 0) { *distance = 0; return 0; }
    *distance = tNear > 0 ? tNear : tFar;
    return 1;
}

/* RayIntersectsOBB — :314-320 (the stored rotation is already the inverse) */
static int rt_ray_intersects_obb(f3 rayOrigin, f3 rayDir, f3 Center, f3 halfExtents, f4 invRotation, float* distance)
{
    f3 localOrigin = qmul(invRotation, sub3(rayOrigin, Center));
    f3 localDir = qmul(invRotation, rayDir);
    return rt_ray_intersects_aabb(localOrigin, localDir, v3(0.0f, 0.0f, 0.0f), halfExtents, distance);
}

/* RayIntersectsSphere — :323-355 */
static int rt_ray_intersects_sphere(f3 rayOrigin, f3 rayDir, f3 Center, float Radius, float* distance)
{
    f3 oc = sub3(rayOrigin, Center);
    float a = dot3(rayDir, rayDir);
    float b = 2.0f * dot3(oc, rayDir);
    float c = dot3(oc, oc) - Radius * Radius;
    float discriminant = b * b - 4.0f * a * c;
    if (discriminant < 0) { *distance = 0; return 0; }
    float sqrtDiscriminant = sqrtf(discriminant);
    float t0 = (-b - sqrtDiscriminant) / (2.0f * a);
    float t1 = (-b + sqrtDiscriminant) / (2.0f * a);
    if (t0 >= 0) { *distance = t0; return 1; }
    else if (t1 >= 0) { *distance = t1; return 1; }
    *distance = 0;
    return 0;
}

typedef struct {
    int type;
    float dist;
    const art_aabb* aabb;
    const art_obb* obb;
    const art_sphere* sphere;
} rt_hit;

/* ShootRayCast — :225-280. Order Sphere, AABB, OBB; strict < keeps the first minimum. */
static int rt_shoot_ray_cast(const rt_job* j, f3 o, f3 d, rt_hit* hit)
{
    float dist;
    hit->dist = 3.40282347e+38f; /* float.MaxValue */
    hit->type = CT_NONE;
    hit->aabb = NULL; hit->obb = NULL; hit->sphere = NULL;
    for (int i = 0; i < j->SphereColliderCount; i++) {
        const art_sphere* s = &j->SphereColliders[i];
        j->cnt->rt_sphere++;
        if (rt_ray_intersects_sphere(o, d, h3(s->center), or_f16tof32(s->radius), &dist) && dist < hit->dist) {
            hit->type = CT_SPHERE; hit->sphere = s; hit->dist = dist;
        }
    }
    for (int i = 0; i < j->AABBColliderCount; i++) {
        const art_aabb* a = &j->AABBColliders[i];
        j->cnt->rt_aabb++;
        if (rt_ray_intersects_aabb(o, d, h3(a->center), h3(a->size), &dist) && dist < hit->dist) {
            hit->type = CT_AABB; hit->aabb = a; hit->dist = dist;
        }
    }
    for (int i = 0; i < j->OBBColliderCount; i++) {
        const art_obb* b = &j->OBBColliders[i];
        j->cnt->rt_obb++;
        if (rt_ray_intersects_obb(o, d, h3(b->center), h3(b->size), obb_rotation(b), &dist) && dist < hit->dist) {
            hit->type = CT_OBB; hit->obb = b; hit->dist = dist;
        }
    }
    return hit->type != CT_NONE;
}

/* The (hitColliderType, collider) pair ShootRayCast returns (:225-280), as ART_HIT_ID: the
 * collider's index is its position in the job's array of that type. */
static uint32_t rt_hit_id(const rt_job* j, const rt_hit* hit)
{
    switch (hit->type) {
    case CT_AABB: return ART_HIT_ID(CT_AABB, (uint32_t)(hit->aabb - j->AABBColliders));
    case CT_OBB: return ART_HIT_ID(CT_OBB, (uint32_t)(hit->obb - j->OBBColliders));
    case CT_SPHERE: return ART_HIT_ID(CT_SPHERE, (uint32_t)(hit->sphere - j->SphereColliders));
    default: return ART_HIT_NONE;
    }
}

/* CanRaySeePoint — :365-397 (echo any-hit, no owner skip) */
static int rt_can_ray_see_point(const rt_job* j, f3 o, f3 d, float distToTarget)
{
    float dist;
    for (int i = 0; i < j->SphereColliderCount; i++) {
        const art_sphere* s = &j->SphereColliders[i];
        j->cnt->rt_sphere++;
        if (rt_ray_intersects_sphere(o, d, h3(s->center), or_f16tof32(s->radius), &dist) && dist < distToTarget) return 0;
    }
    for (int i = 0; i < j->AABBColliderCount; i++) {
        const art_aabb* a = &j->AABBColliders[i];
        j->cnt->rt_aabb++;
        if (rt_ray_intersects_aabb(o, d, h3(a->center), h3(a->size), &dist) && dist < distToTarget) return 0;
    }
    for (int i = 0; i < j->OBBColliderCount; i++) {
        const art_obb* b = &j->OBBColliders[i];
        j->cnt->rt_obb++;
        if (rt_ray_intersects_obb(o, d, h3(b->center), h3(b->size), obb_rotation(b), &dist) && dist < distToTarget) return 0;
    }
    return 1;
}

/* CanRaySeeAudioTarget — :405-449 (muffle any-hit, skips colliders owned by the target) */
static int rt_can_ray_see_audio_target(const rt_job* j, f3 o, f3 d, float distToStartOrigin, int AudioTargetId)
{
    float dist;
    for (int i = 0; i < j->SphereColliderCount; i++) {
        const art_sphere* s = &j->SphereColliders[i];
        if (s->audio_target_id == AudioTargetId) continue;
        j->cnt->rt_sphere++;
        if (rt_ray_intersects_sphere(o, d, h3(s->center), or_f16tof32(s->radius), &dist) && dist < distToStartOrigin) return 0;
    }
    for (int i = 0; i < j->AABBColliderCount; i++) {
        const art_aabb* a = &j->AABBColliders[i];
        if (a->audio_target_id == AudioTargetId) continue;
        j->cnt->rt_aabb++;
        if (rt_ray_intersects_aabb(o, d, h3(a->center), h3(a->size), &dist) && dist < distToStartOrigin) return 0;
    }
    for (int i = 0; i < j->OBBColliderCount; i++) {
        const art_obb* b = &j->OBBColliders[i];
        if (b->audio_target_id == AudioTargetId) continue;
        j->cnt->rt_obb++;
        if (rt_ray_intersects_obb(o, d, h3(b->center), h3(b->size), obb_rotation(b), &dist) && dist < distToStartOrigin) return 0;
    }
    return 1;
}

/* ReflectRay — :456-532 */
static void rt_reflect_ray(const rt_job* j, const rt_hit* hit, f3* cRayOrigin, f3* cRayDir, float* cRayLife)
{
    f3 normal = v3(0.0f, 0.0f, 0.0f);
    float absorption = 0;
    switch (hit->type) {
    case CT_AABB: { /* :463-485 */
        f3 localPoint = sub3(*cRayOrigin, h3(hit->aabb->center));
        f3 absPoint = abs3(localPoint);
        f3 halfExtents = h3(hit->aabb->size);
        normal = v3(0.0f, 0.0f, 0.0f);
        if (halfExtents.x - absPoint.x < halfExtents.y - absPoint.y && halfExtents.x - absPoint.x < halfExtents.z - absPoint.z)
            normal.x = usign(localPoint.x);
        else if (halfExtents.y - absPoint.y < halfExtents.x - absPoint.x && halfExtents.y - absPoint.y < halfExtents.z - absPoint.z)
            normal.y = usign(localPoint.y);
        else
            normal.z = usign(localPoint.z);
        absorption = or_f16tof32(hit->aabb->material.absorption);
        break;
    }
    case CT_OBB: { /* :487-512 — inverse(stored) into local, stored back to world (Q5) */
        f4 rot = obb_rotation(hit->obb);
        f3 localHit = qmul(qinverse(rot), sub3(*cRayOrigin, h3(hit->obb->center)));
        f3 localHalfExtents = h3(hit->obb->size);
        f3 absPointOBB = abs3(localHit);
        f3 deltaToFaceOBB = sub3(localHalfExtents, absPointOBB);
        f3 localNormal = v3(0.0f, 0.0f, 0.0f);
        if (deltaToFaceOBB.x < deltaToFaceOBB.y && deltaToFaceOBB.x < deltaToFaceOBB.z)
            localNormal.x = usign(localHit.x);
        else if (deltaToFaceOBB.y < deltaToFaceOBB.x && deltaToFaceOBB.y < deltaToFaceOBB.z)
            localNormal.y = usign(localHit.y);
        else
            localNormal.z = usign(localHit.z);
        normal = qmul(obb_rotation(hit->obb), localNormal);
        absorption = or_f16tof32(hit->obb->material.absorption);
        break;
    }
    case CT_SPHERE: /* :514-518 */
        normal = normalize3(sub3(*cRayOrigin, h3(hit->sphere->center)));
        absorption = or_f16tof32(hit->sphere->material.absorption);
        break;
    default:
        break;
    }
    *cRayDir = reflect3(*cRayDir, normal);          /* :525 */
    *cRayOrigin = add3(*cRayOrigin, muls(*cRayDir, EPSILON)); /* :528 */
    *cRayLife -= j->MaxRayLife * absorption;        /* :531 */
}

/* Execute — :61-215 */
static void rt_execute(const rt_job* j, int rayStartIndex, int totalRays)
{
    int batchCount = j->MuffleRayHitsLength / j->TotalAudioTargets;     /* :63 */
    int batchId = rayStartIndex * batchCount / j->RayDirectionsLength;  /* :64 */
    f3 cRayOrigin;

    /* :72-80 — reset (index quirk Q1: rayStartIndex + i, not rayStartIndex*H + i) */
    for (int i = 0; i < totalRays * j->MaxHitsPerRay; i++) {
        int rayIndex = rayStartIndex + i;
        j->EchoRayDistances[rayIndex] = 0; /* (half)0 */
        if (j->RayHitResults) { art_half3 z = { 0, 0, 0 }; j->RayHitResults[rayIndex] = z; }
        if (j->RayHitIds) j->RayHitIds[rayIndex] = ART_HIT_NONE;
    }
    /* :82-85 */
    for (int i = 0; i < j->TotalAudioTargets; i++) j->MuffleRayHits[batchId * j->TotalAudioTargets + i] = 0;

    for (int localRayId = 0; localRayId < totalRays; localRayId++) { /* :90 */
        int rayIndex = rayStartIndex + localRayId;
        f3 cRayDir = h3(j->RayDirections[rayIndex]);                  /* :94 */
        cRayOrigin = j->RayOrigin;
        uint8_t cRayHits = 0;
        int rayResultId;
        float cRayLife = j->MaxRayLife;
        int isRayAlive = 1;

        while (isRayAlive) { /* :104 */
            rt_hit hit;
            art_half3 rayResult = { 0, 0, 0 };
            if (rt_shoot_ray_cast(j, cRayOrigin, cRayDir, &hit)) { /* :108 */
                cRayOrigin = add3(cRayOrigin, muls(cRayDir, hit.dist)); /* :111 */
                cRayLife -= hit.dist;
                cRayHits += 1;
                rayResultId = rayIndex * j->MaxHitsPerRay + cRayHits - 1; /* :115 */
                rayResult = toh3(cRayOrigin);                            /* :118 */

                /* Echo — :124-145 */
                f3 offsettedRayHitWorldPoint = sub3(cRayOrigin, muls(cRayDir, EPSILON));
                f3 returnRayDir = normalize3(sub3(j->RayOrigin, offsettedRayHitWorldPoint));
                float distToStartOrigin = distance3(j->RayOrigin, cRayOrigin);
                if (rt_can_ray_see_point(j, offsettedRayHitWorldPoint, returnRayDir, distToStartOrigin)) {
                    uint16_t echoMultiplier;
                    switch (hit.type) {
                    case CT_AABB: echoMultiplier = hit.aabb->material.echo; break;
                    case CT_OBB: echoMultiplier = hit.obb->material.echo; break;
                    case CT_SPHERE: echoMultiplier = hit.sphere->material.echo; break;
                    default: echoMultiplier = 0x3C00; break;
                    }
                    /* Half.Multiply(in float, in float, out half) — Utility/HalfDataTypesUtility.cs:86-90 */
                    j->EchoRayDistances[rayResultId] = or_f32tof16(distToStartOrigin * or_f16tof32(echoMultiplier));
                }

                /* Muffle — :150-173 */
                for (int AudioTargetId = 0; AudioTargetId < j->TotalAudioTargets; AudioTargetId++) {
                    int muffleRayId = batchId * j->TotalAudioTargets + AudioTargetId;
                    offsettedRayHitWorldPoint = sub3(cRayOrigin, muls(cRayDir, EPSILON));
                    f3 audioTargetPosition = target_pos(j->AudioTargetPositions, AudioTargetId);
                    f3 rayToTargetDir = normalize3(sub3(audioTargetPosition, offsettedRayHitWorldPoint));
                    float distToTarget = distance3(offsettedRayHitWorldPoint, audioTargetPosition);
                    if (distToTarget < j->MaxMuffleHitDistance &&
                        rt_can_ray_see_audio_target(j, offsettedRayHitWorldPoint, rayToTargetDir, distToTarget, AudioTargetId)) {
                        j->MuffleRayHits[muffleRayId] = (uint16_t)(j->MuffleRayHits[muffleRayId] + 1);
                    }
                }

                /* Termination — :179-193 */
                if (cRayHits >= j->MaxHitsPerRay || cRayLife <= 0) {
                    isRayAlive = 0;
                } else {
                    rt_reflect_ray(j, &hit, &cRayOrigin, &cRayDir, &cRayLife);
                    if (cRayLife < 0) isRayAlive = 0;
                }
                if (j->RayHitResults) j->RayHitResults[rayResultId] = rayResult; /* :197 */
                if (j->RayHitIds) j->RayHitIds[rayResultId] = rt_hit_id(j, &hit);
            } else {
                if (j->RayHitResultCounts) j->RayHitResultCounts[rayIndex] = cRayHits; /* :204 */
                break;
            }
        }
        if (j->RayHitResultCounts) j->RayHitResultCounts[rayIndex] = cRayHits; /* :212 */
    }
}

/* ========================================================================================
 * 4. AudioPermeationJobBatched — Jobs/AudioPermeationJobBatched.cs
 * ====================================================================================== */

typedef struct {
    f3 RayOrigin;
    const art_half3* RayDirections; int RayDirectionsLength;
    const art_aabb* AABBColliders; int AABBColliderCount;
    const art_obb* OBBColliders; int OBBColliderCount;
    const art_sphere* SphereColliders; int SphereColliderCount;
    const float* AudioTargetPositions; int TotalAudioTargets;
    float PermeationStrengthPerRay;
    float* PermeationPowerRemains; int PermeationPowerRemainsLength;
    counters* cnt;
} perm_job;

/* RayIntersectsOBB — :172-179: applies inverse() to the stored (already inverse) rotation (Q5) */
static int pj_ray_intersects_obb(f3 rayOrigin, f3 rayDir, f3 Center, f3 halfExtents, f4 rotation, float* distance)
{
    f4 invRotation = qinverse(rotation);
    f3 localOrigin = qmul(invRotation, sub3(rayOrigin, Center));
    f3 localDir = qmul(invRotation, rayDir);
    return rt_ray_intersects_aabb(localOrigin, localDir, v3(0.0f, 0.0f, 0.0f), halfExtents, distance);
}

/* ShootRayCast — :101-141 (nearest distance only; INFINITY sentinel, Q9).
 * RayIntersectsAABB :145-169 and RayIntersectsSphere :182-214 are identical to the raytracer's. */
static int pj_shoot_ray_cast(const perm_job* j, f3 o, f3 d, float* closestDist)
{
    float dist;
    *closestDist = INFINITY;
    for (int i = 0; i < j->SphereColliderCount; i++) {
        const art_sphere* s = &j->SphereColliders[i];
        j->cnt->ph_sphere++;
        if (rt_ray_intersects_sphere(o, d, h3(s->center), or_f16tof32(s->radius), &dist) && dist < *closestDist) *closestDist = dist;
    }
    for (int i = 0; i < j->AABBColliderCount; i++) {
        const art_aabb* a = &j->AABBColliders[i];
        j->cnt->ph_aabb++;
        if (rt_ray_intersects_aabb(o, d, h3(a->center), h3(a->size), &dist) && dist < *closestDist) *closestDist = dist;
    }
    for (int i = 0; i < j->OBBColliderCount; i++) {
        const art_obb* b = &j->OBBColliders[i];
        j->cnt->ph_obb++;
        if (pj_ray_intersects_obb(o, d, h3(b->center), h3(b->size), obb_rotation(b), &dist) && dist < *closestDist) *closestDist = dist;
    }
    return *closestDist != INFINITY;
}

/* RayIntersectsAABBPermeation — :265-288 */
static void pj_aabb_permeation(f3 rayOrigin, f3 rayDir, f3 Center, f3 halfExtents, float densityMultiplier, float* total)
{
    f3 mn = sub3(Center, halfExtents);
    f3 mx = add3(Center, halfExtents);
    f3 invDir = rcp3(rayDir);
    f3 t0 = mul3(sub3(mn, rayOrigin), invDir);
    f3 t1 = mul3(sub3(mx, rayOrigin), invDir);
    f3 tmin = min3v(t0, t1);
    f3 tmax = max3v(t0, t1);
    float tEnter = umax(umax(tmin.x, tmin.y), tmin.z);
    float tExit = umin(umin(tmax.x, tmax.y), tmax.z);
    if (tEnter > tExit || tExit < 0.0f) return;
    float enter = umax(tEnter, 0.0f);
    *total += umax(0.0f, tExit - enter) * densityMultiplier;
}

/* RayIntersectsOBBPermeation — :294-300 (stored rotation used directly) */
static void pj_obb_permeation(f3 rayOrigin, f3 rayDir, f3 Center, f3 halfExtents, f4 invRotation, float densityMultiplier, float* total)
{
    f3 localOrigin = qmul(invRotation, sub3(rayOrigin, Center));
    f3 localDir = qmul(invRotation, rayDir);
    pj_aabb_permeation(localOrigin, localDir, v3(0.0f, 0.0f, 0.0f), halfExtents, densityMultiplier, total);
}

/* RayIntersectsSpherePermeation — :303-328 (unit-direction form, Q10) */
static void pj_sphere_permeation(f3 rayOrigin, f3 rayDir, f3 Center, float Radius, float densityMultiplier, float* total)
{
    f3 oc = sub3(rayOrigin, Center);
    float b = dot3(oc, rayDir);
    float c = dot3(oc, oc) - Radius * Radius;
    float discriminant = b * b - c;
    if (discriminant < 0.0f) return;
    float sqrtD = sqrtf(discriminant);
    float tEnter = -b - sqrtD;
    float tExit = -b + sqrtD;
    if (tExit < 0.0f) return;
    float enter = umax(tEnter, 0.0f);
    *total += umax(0.0f, tExit - enter) * densityMultiplier;
}

/* ShootPermeationRayCast — :225-261 (serial over all non-owned colliders, Sphere, AABB, OBB) */
static float pj_shoot_permeation_ray_cast(const perm_job* j, f3 o, f3 d, int AudioTargetId)
{
    float total = 0;
    for (int i = 0; i < j->SphereColliderCount; i++) {
        const art_sphere* s = &j->SphereColliders[i];
        if (s->audio_target_id == AudioTargetId) continue;
        j->cnt->pl_sphere++;
        pj_sphere_permeation(o, d, h3(s->center), or_f16tof32(s->radius), or_f16tof32(s->material.density), &total);
    }
    for (int i = 0; i < j->AABBColliderCount; i++) {
        const art_aabb* a = &j->AABBColliders[i];
        if (a->audio_target_id == AudioTargetId) continue;
        j->cnt->pl_aabb++;
        pj_aabb_permeation(o, d, h3(a->center), h3(a->size), or_f16tof32(a->material.density), &total);
    }
    for (int i = 0; i < j->OBBColliderCount; i++) {
        const art_obb* b = &j->OBBColliders[i];
        if (b->audio_target_id == AudioTargetId) continue;
        j->cnt->pl_obb++;
        pj_obb_permeation(o, d, h3(b->center), h3(b->size), obb_rotation(b), or_f16tof32(b->material.density), &total);
    }
    return (float)j->RayDirectionsLength * j->PermeationStrengthPerRay - total; /* :260 */
}

/* Execute — :34-91 */
static void pj_execute(const perm_job* j, int rayStartIndex, int totalRays)
{
    int batchCount = j->PermeationPowerRemainsLength / totalRays / j->TotalAudioTargets; /* :36 (Q7) */
    int batchId = rayStartIndex * batchCount / j->RayDirectionsLength;                     /* :37 */
    f3 cRayOrigin;
    for (int i = 0; i < j->TotalAudioTargets; i++) j->PermeationPowerRemains[batchId * j->TotalAudioTargets + i] = 0.0f; /* :43-46 */

    for (int localRayId = 0; localRayId < totalRays; localRayId++) {
        int rayIndex = rayStartIndex + localRayId;
        f3 cRayDir = h3(j->RayDirections[rayIndex]);
        cRayOrigin = j->RayOrigin;
        float rayHitDist;
        if (pj_shoot_ray_cast(j, cRayOrigin, cRayDir, &rayHitDist)) { /* :58 */
            cRayOrigin = add3(cRayOrigin, muls(cRayDir, rayHitDist));
            for (int AudioTargetId = 0; AudioTargetId < j->TotalAudioTargets; AudioTargetId++) {
                int permeationRayId = batchId * j->TotalAudioTargets + AudioTargetId;
                f3 offsettedRayHitWorldPoint = sub3(cRayOrigin, muls(cRayDir, EPSILON));
                f3 audioTargetPosition = target_pos(j->AudioTargetPositions, AudioTargetId);
                f3 rayToTargetDir = normalize3(sub3(audioTargetPosition, offsettedRayHitWorldPoint));
                (void)distance3(offsettedRayHitWorldPoint, audioTargetPosition); /* :79, passed but unused */
                j->PermeationPowerRemains[permeationRayId] =
                    pj_shoot_permeation_ray_cast(j, offsettedRayHitWorldPoint, rayToTargetDir, AudioTargetId); /* :82-85 */
            }
        }
    }
}

/* ========================================================================================
 * 5. ProcessAudioDataJob — Jobs/ProcessAudioDataJob.cs:32-76 (+ AudioTargetRTSettings ctor)
 * ====================================================================================== */
static void process_audio_data(const art_frame_desc* d, const art_fan* fan, int TC)
{
    int T = d->audio_target_count;
    int maxBatchSize = (TC * T) / T;                        /* :34 */
    int maxRayHits = d->max_hits_per_ray * d->ray_count;    /* :35 */
    float reverbTotal = 0;
    float echoRayReturnedHits = 0;
    for (int i = 0; i < maxRayHits; i++) {                  /* :40-48 ordered */
        float e = or_f16tof32(fan->echo_ray_distances[i]);
        if (e == 0) { echoRayReturnedHits += 1; continue; }
        reverbTotal += e;
    }
    float avgReverbDist = reverbTotal / (float)maxRayHits;  /* :49 */
    float reverbStrength = avgReverbDist / d->max_reverb_distance;
    float reverbVolume = echoRayReturnedHits / (float)maxRayHits;

    for (int t = 0; t < T; t++) {
        int totalMuffleRayhits = 0;
        float totalPermeationPower = 0;
        for (int i = 0; i < maxBatchSize; i++) {             /* :61-65 */
            totalMuffleRayhits += fan->muffle_ray_hits[T * i + t];
            totalPermeationPower += fan->permeation_power_remains[T * i + t];
        }
        float muffle = 1.0f - (float)totalMuffleRayhits / (float)(d->ray_count * d->max_hits_per_ray) * d->muffle_effectiveness; /* :68 */
        float permeation = totalPermeationPower / (float)d->ray_count / d->permeation_strength_per_ray * d->permeation_effectiveness; /* :69 */
        muffle = usaturate(muffle - permeation);             /* :71 */
        art_target_settings* s = &fan->settings[t];          /* AudioTargetRTSettings.cs:18-24 */
        s->muffle_strength = usaturate(muffle);
        s->reverb_strength = usaturate(reverbStrength);
        s->reverb_volume = usaturate(reverbVolume);
        s->perceived_position[0] = d->audio_target_positions[3 * t + 0];
        s->perceived_position[1] = d->audio_target_positions[3 * t + 1];
        s->perceived_position[2] = d->audio_target_positions[3 * t + 2];
    }
}

/* ========================================================================================
 * 6. DSP parameters (config 5): AudioSpatializer.cs:58, ReverbDSP.cs:12-13, MuffleDSP.cs:22-26 and :38-42,
 *    NativeSampledAnimationCurve.cs:64-89
 * ====================================================================================== */
static float curve_evaluate(const art_curve* c, float time)
{
    float percent = time / c->length;                                            /* :74 */
    int n = c->sample_count;
    float curvePercentage = umax(0.0f, umin((float)(n - 1), percent * (float)(n - 1))); /* :83 clamp */
    int floorIndex = (int)floorf(curvePercentage);                               /* :85-86 */
    int ceilIndex = (int)ceilf(curvePercentage);
    return ulerp(c->baked[floorIndex], c->baked[ceilIndex], curvePercentage - (float)floorIndex); /* :88 */
}

static void dsp_params(const art_dsp_desc* dsp, const art_target_settings* s, art_dsp_params* out)
{
    const float DOUBLE_PI = 2.0f * 3.14159265f; /* MuffleDSP.cs:35, math.PI (float) */
    out->dry_level = ulerp(dsp->reverb_dry_level_min, dsp->reverb_dry_level_max, s->reverb_strength);
    float t = curve_evaluate(&dsp->reverb_volume_curve, s->reverb_volume);
    out->dry_boost = ulerp(dsp->reverb_dry_boost_min, dsp->reverb_dry_boost_max, t);
    out->reserved = 0;
    if (s->muffle_strength > 0.0f) {
        float muffle = curve_evaluate(&dsp->muffle_curve, s->muffle_strength);
        float cutoff = ulerp(dsp->muffle_cutoff_max, dsp->muffle_cutoff_min, muffle);
        float rc = 1.0f / (cutoff * DOUBLE_PI);
        float dt = 1.0f / (float)dsp->sample_rate;
        out->muffle_cutoff = cutoff;
        out->muffle_alpha = dt / (rc + dt);
        out->muffle_active = 1;
    } else {
        out->muffle_cutoff = 0.0f;
        out->muffle_alpha = 0.0f;
        out->muffle_active = 0;
    }
}

/* ========================================================================================
 * 7. Frame orchestration — Audio/AudioRayTracer.cs:161-237, one fan per AudioRayTracer
 * ====================================================================================== */
static int validate(const art_frame_desc* d, const art_fan* fans, int32_t fan_count)
{
    if (!d || (fan_count > 0 && !fans) || fan_count < 0) return ART_E_INVALID;
    if (d->ray_count <= 0 || !d->ray_directions) return ART_E_INVALID;
    if (d->audio_target_count <= 0 || !d->audio_target_positions) return ART_E_INVALID;
    if (d->max_hits_per_ray <= 0 || d->max_hits_per_ray > 255) return ART_E_INVALID;
    if (d->batch_size <= 0 || d->batch_slots <= 0) return ART_E_INVALID;
    if ((d->aabb_count && !d->aabb_colliders) || (d->obb_count && !d->obb_colliders) || (d->sphere_count && !d->sphere_colliders)) return ART_E_INVALID;
    if ((d->stages & ART_STAGE_DSP_PARAMS) && !d->dsp) return ART_E_INVALID;
    return ART_OK;
}

static void run_fan(const art_frame_desc* d, const art_fan* f, counters* cnt)
{
    int R = d->ray_count, T = d->audio_target_count, TC = d->batch_slots, bs = d->batch_size;
    if (d->stages & ART_STAGE_RAYTRACE) {
        rt_job j;
        j.RayOrigin = v3(f->origin[0], f->origin[1], f->origin[2]);
        j.RayDirections = d->ray_directions; j.RayDirectionsLength = R;
        j.AABBColliders = d->aabb_colliders; j.AABBColliderCount = d->aabb_count;
        j.OBBColliders = d->obb_colliders; j.OBBColliderCount = d->obb_count;
        j.SphereColliders = d->sphere_colliders; j.SphereColliderCount = d->sphere_count;
        j.AudioTargetPositions = d->audio_target_positions; j.TotalAudioTargets = T;
        j.MaxRayLife = d->max_ray_life; j.MaxHitsPerRay = (uint8_t)d->max_hits_per_ray;
        j.RayHitResults = f->ray_hit_points; j.RayHitResultCounts = f->ray_hit_counts; j.RayHitIds = f->ray_hit_ids;
        j.EchoRayDistances = f->echo_ray_distances;
        j.MuffleRayHits = f->muffle_ray_hits; j.MuffleRayHitsLength = TC * T;
        j.MaxMuffleHitDistance = d->max_muffle_hit_distance;
        j.cnt = cnt;
        for (int start = 0; start < R; start += bs) rt_execute(&j, start, (R - start) < bs ? (R - start) : bs);
    }
    if (d->stages & ART_STAGE_PERMEATE) {
        perm_job j;
        j.RayOrigin = v3(f->origin[0], f->origin[1], f->origin[2]);
        j.RayDirections = d->ray_directions; j.RayDirectionsLength = R;
        j.AABBColliders = d->aabb_colliders; j.AABBColliderCount = d->aabb_count;
        j.OBBColliders = d->obb_colliders; j.OBBColliderCount = d->obb_count;
        j.SphereColliders = d->sphere_colliders; j.SphereColliderCount = d->sphere_count;
        j.AudioTargetPositions = d->audio_target_positions; j.TotalAudioTargets = T;
        j.PermeationStrengthPerRay = d->permeation_strength_per_ray;
        j.PermeationPowerRemains = f->permeation_power_remains; j.PermeationPowerRemainsLength = TC * T;
        j.cnt = cnt;
        for (int start = 0; start < R; start += bs) pj_execute(&j, start, (R - start) < bs ? (R - start) : bs);
    }
    if (d->stages & ART_STAGE_REDUCE) process_audio_data(d, f, TC);
    if ((d->stages & ART_STAGE_DSP_PARAMS) && f->dsp_params)
        for (int t = 0; t < T; t++) dsp_params(d->dsp, &f->settings[t], &f->dsp_params[t]);
}

typedef struct {
    const art_frame_desc* d;
    const art_fan* fans;
    int32_t fan_count, stride, first;
    counters cnt;
} worker_arg;

static void* worker(void* p)
{
    worker_arg* a = (worker_arg*)p;
    for (int32_t i = a->first; i < a->fan_count; i += a->stride) run_fan(a->d, &a->fans[i], &a->cnt);
    return NULL;
}

int or_run_frame(const art_frame_desc* desc, const art_fan* fans, int32_t fan_count, int32_t threads, art_test_counts* counts)
{
    int rc = validate(desc, fans, fan_count);
    if (rc) return rc;
    if (threads <= 0) threads = 1;
    if (threads > fan_count) threads = fan_count > 0 ? fan_count : 1;
    worker_arg* args = (worker_arg*)calloc((size_t)threads, sizeof(worker_arg));
    pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!args || !tids) { free(args); free(tids); return ART_E_NOMEM; }
    for (int k = 0; k < threads; k++) {
        args[k].d = desc; args[k].fans = fans; args[k].fan_count = fan_count;
        args[k].stride = threads; args[k].first = k;
    }
    if (threads == 1) worker(&args[0]);
    else {
        for (int k = 0; k < threads; k++) pthread_create(&tids[k], NULL, worker, &args[k]);
        for (int k = 0; k < threads; k++) pthread_join(tids[k], NULL);
    }
    if (counts) {
        memset(counts, 0, sizeof(*counts));
        for (int k = 0; k < threads; k++) {
            counts->rt_sphere += args[k].cnt.rt_sphere; counts->rt_aabb += args[k].cnt.rt_aabb; counts->rt_obb += args[k].cnt.rt_obb;
            counts->perm_hit_sphere += args[k].cnt.ph_sphere; counts->perm_hit_aabb += args[k].cnt.ph_aabb; counts->perm_hit_obb += args[k].cnt.ph_obb;
            counts->perm_loss_sphere += args[k].cnt.pl_sphere; counts->perm_loss_aabb += args[k].cnt.pl_aabb; counts->perm_loss_obb += args[k].cnt.pl_obb;
        }
    }
    free(args); free(tids);
    return ART_OK;
}

/* ========================================================================================
 * 8. FibonacciDirectionsJobParallel — Jobs/FibonacciDirectionsJobParallel.cs:15-35
 * ====================================================================================== */
void or_fibonacci_directions(int32_t count, art_half3* out)
{
    for (int32_t i = 0; i < count; i++) {
        float phi = 3.14159265f * (3.0f - sqrtf(5.0f));
        float y = 1.0f - ((float)i / (float)(count - 1)) * 2.0f;
        float radius = sqrtf(1.0f - y * y);
        float theta = phi * (float)i;
        float x = cosf(theta) * radius;
        float z = sinf(theta) * radius;
        out[i] = toh3(v3(x, y, z));
    }
}

/* ========================================================================================
 * 9. Primitive wrappers for known-answer tests
 * ====================================================================================== */
int or_ray_intersects_aabb(const float o[3], const float d[3], const float c[3], const float h[3], float* dist)
{
    return rt_ray_intersects_aabb(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), v3(c[0], c[1], c[2]), v3(h[0], h[1], h[2]), dist);
}
int or_ray_intersects_sphere(const float o[3], const float d[3], const float c[3], float r, float* dist)
{
    return rt_ray_intersects_sphere(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), v3(c[0], c[1], c[2]), r, dist);
}
int or_ray_intersects_obb(const float o[3], const float d[3], const float c[3], const float h[3], const float q[4], float* dist)
{
    f4 qq = { q[0], q[1], q[2], q[3] };
    return rt_ray_intersects_obb(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), v3(c[0], c[1], c[2]), v3(h[0], h[1], h[2]), qq, dist);
}
void or_half_quaternion_value(uint16_t x, uint16_t y, uint16_t z, float q[4])
{
    f4 r = half_quaternion_value(x, y, z);
    q[0] = r.x; q[1] = r.y; q[2] = r.z; q[3] = r.w;
}
void or_quat_inverse(const float q[4], float out[4])
{
    f4 qq = { q[0], q[1], q[2], q[3] };
    f4 r = qinverse(qq);
    out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}
void or_quat_mul_vec(const float q[4], const float v[3], float out[3])
{
    f4 qq = { q[0], q[1], q[2], q[3] };
    f3 r = qmul(qq, v3(v[0], v[1], v[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ========================================================================================
 * 8. Per-sample spatializer DSP (SURVEY.md §8 f rank 1): AudioSpatializer.OnAudioFilterRead
 *    (Audio/AudioTarget/AudioSpatializer.cs:70-87) = MuffleDSP.Process (MuffleDSP.cs:13-32),
 *    ReverbDSP.Process (ReverbDSP.cs:10-24), BinauralDSP.Process (BinauralDSP.cs:15-82), volume.
 *    Literal: per-sample quantities are recomputed inside the loops as the C# does.
 *    BinauralDSP runs in managed code (no [BurstCompile] under Audio/), where Unity.Mathematics'
 *    math.atan2/sin/cos(float) are (float)System.Math.Atan2/Sin/Cos: evaluated in double and
 *    rounded once (BinauralDSP.cs:17,27,32); the host libm's double functions are correctly
 *    rounded for these arguments in practice, .NET's may differ in rare last bits (unpinned).
 * ====================================================================================== */
#define OR_TODEGREES 57.29578f      /* Unity.Mathematics math.degrees factor */
#define OR_TORADIANS 0.0174532924f  /* math.radians factor */

static float or_lowpass(float input, float* prev, float cutoff, float sampleRate) /* MuffleDSP.cs:38-45, BinauralDSP.cs:87-94 */
{
    const float DOUBLE_PI = 2.0f * 3.14159265f;
    float rc = 1.0f / (cutoff * DOUBLE_PI);
    float dt = 1.0f / sampleRate;
    float alpha = dt / (rc + dt);
    *prev += alpha * (input - *prev);
    return *prev;
}

static float or_highpass(float input, float* prevIn, float* prevOut, float cutoff, float sampleRate) /* BinauralDSP.cs:97-106 */
{
    const float DOUBLE_PI = 2.0f * 3.14159265f;
    float rc = 1.0f / (cutoff * DOUBLE_PI);
    float dt = 1.0f / sampleRate;
    float alpha = rc / (rc + dt);
    float output = alpha * (*prevOut + input - *prevIn);
    *prevIn = input;
    *prevOut = output;
    return output;
}

static float uclamp(float x, float a, float b) { return umax(a, umin(b, x)); }

static void or_dsp_source(const art_spatializer_settings* st, art_audio_source* src, int sampleRate)
{
    if (src->channels != 2) return;                                  /* AudioSpatializer.cs:72 */
    float* data = src->data;
    const int len = src->frames * 2;
    art_dsp_state* S = src->state;
    const float sr = (float)sampleRate;
    /* MuffleDSP.Process :13-32 */
    for (int i = 0; i < len; i += 2) {
        float l = data[i], r = data[i + 1];
        if (src->muffle_strength > 0.0f) {                           /* :22 */
            float muffle = curve_evaluate(&st->muffle_curve, src->muffle_strength);       /* :24 */
            float cutoff = ulerp(st->muffle_cutoff_max, st->muffle_cutoff_min, muffle);   /* :26 */
            data[i] = or_lowpass(l, &S->previous_muffle.left, cutoff, sr);                /* :28 */
            data[i + 1] = or_lowpass(r, &S->previous_muffle.right, cutoff, sr);           /* :29 */
        }
    }
    /* ReverbDSP.Process :10-24 */
    {
        float t = curve_evaluate(&st->reverb_volume_curve, src->reverb_volume);           /* :12 */
        float dryBoost = ulerp(st->reverb_dry_boost_min, st->reverb_dry_boost_max, t);    /* :13 */
        for (int i = 0; i < len; i += 2) {
            float l = data[i], r = data[i + 1];
            data[i] = l * dryBoost;
            data[i + 1] = r * dryBoost;
        }
    }
    /* BinauralDSP.Process :15-82 */
    {
        const float* ld = src->local_dir;
        float dist = src->listener_distance;
        /* Unbursted managed code (BinauralDSP.cs has no [BurstCompile]): Unity.Mathematics' float
         * atan2/sin/cos are (float)System.Math.Atan2/Sin/Cos, i.e. double precision rounded once. */
        float azimuth = (float)atan2((double)ld[0], (double)ld[2]) * OR_TODEGREES;        /* :17 */
        float effectivePanStrength = st->pan_strength;                                    /* :19 */
        if (st->distance_based_panning) {                                                 /* :20-24 */
            float distanceFactor = usaturate(dist / st->max_pan_distance);
            effectivePanStrength *= distanceFactor;
        }
        float pan = (float)sin((double)(azimuth * OR_TORADIANS)) * effectivePanStrength; /* :27 */
        float leftGain = sqrtf(0.5f * (1.0f - pan));                                      /* :28 */
        float rightGain = sqrtf(0.5f * (1.0f + pan));                                     /* :29 */
        float frontFactor = umax(0.0f, (float)cos((double)(azimuth * OR_TORADIANS)));    /* :32 */
        float rearAtten = ulerp(1.0f - st->rear_attenuation_strength, 1.0f, frontFactor); /* :33 */
        if (st->distance_based_rear_attenuation) {                                        /* :35-40 */
            float distanceFactor = usaturate(1.0f - (dist / st->max_rear_attenuation_distance));
            rearAtten = uclamp(rearAtten * distanceFactor, 1.0f - st->rear_attenuation_strength, 1.0f);
        }
        float elev = ld[1] <= 0.0f ? ulerp(1.0f, st->low_pass_volume, usaturate(-ld[1]))  /* :43-45 */
                                   : ulerp(1.0f, st->high_pass_volume, usaturate(ld[1]));
        float modL = leftGain * rearAtten * elev;                                         /* :48-50 */
        float modR = rightGain * rearAtten * elev;
        for (int i = 0; i < len; i += 2) {                                                /* :54-81 */
            float pl = data[i] * modL;
            float pr = data[i + 1] * modR;
            if (ld[1] <= 0.0f) {
                float lowPassCutoff = ulerp(st->low_pass_cutoff_min, st->low_pass_cutoff_max, usaturate(-ld[1])) *
                                      (1.0f - 0.5f * usaturate(dist / st->max_elevation_effect_distance)); /* :65 */
                pl = or_lowpass(pl, &S->previous_lp.left, lowPassCutoff, sr);
                pr = or_lowpass(pr, &S->previous_lp.right, lowPassCutoff, sr);
            } else {
                float highPassCutoff = ulerp(st->high_pass_cutoff_min, st->high_pass_cutoff_max, usaturate(ld[1])) *
                                       (1.0f + 0.5f * usaturate(dist / st->max_elevation_effect_distance)); /* :73 */
                pl = or_highpass(pl, &S->previous_input.left, &S->previous_hp.left, highPassCutoff, sr);
                pr = or_highpass(pr, &S->previous_input.right, &S->previous_hp.right, highPassCutoff, sr);
            }
            data[i] = pl;
            data[i + 1] = pr;
        }
    }
    /* volume multiplier, AudioSpatializer.cs:79-86 */
    for (int i = 0; i < len; i += 2) {
        float l = data[i], r = data[i + 1];
        data[i] = l * src->volume_multiplier;
        data[i + 1] = r * src->volume_multiplier;
    }
}

int or_dsp_process(const art_spatializer_settings* settings, art_audio_source* sources, int32_t count, int32_t sample_rate)
{
    if (!settings || (count > 0 && !sources) || count < 0) return ART_E_INVALID;
    for (int32_t k = 0; k < count; ++k) {
        if (sources[k].frames < 0 || (sources[k].frames > 0 && !sources[k].data) || !sources[k].state) return ART_E_INVALID;
        or_dsp_source(settings, &sources[k], sample_rate);
    }
    return ART_OK;
}
