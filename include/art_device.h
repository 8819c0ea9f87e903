/*
 * art_device.h — device-resident extension of the art C ABI.
 *
 * The Unity drop-in surface is art.h (host arrays in, host arrays out). This header adds the
 * entry points a one-process-per-GPU host (bench.py, or a server that keeps scenes resident in
 * HBM and exchanges results with RCCL) needs: bind a scene once, then launch frames whose fan
 * origins and packed per-fan result blocks are DEVICE pointers on a caller-supplied HIP stream.
 *
 * Packed per-fan result block (art_fan_layout): fan f's record starts at f * stride inside the
 * block and holds, at the given byte offsets, exactly the arrays art_fan points to
 * (settings, dsp params, muffle, permeation, echo, hit points, hit counts). One contiguous block
 * per rank is what the multi-GPU path all-gathers (SURVEY.md §8 e).
 */
#ifndef ART_DEVICE_H
#define ART_DEVICE_H

#include "art.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ART_OUT_HIT_RESULTS 0x1u /* also produce ray_hit_points / ray_hit_counts / ray_hit_ids */

typedef struct {
    uint32_t stride;          /* bytes per fan record, multiple of 16 */
    uint32_t settings_off;    /* art_target_settings[T] */
    uint32_t dsp_off;         /* art_dsp_params[T] (valid iff stages & ART_STAGE_DSP_PARAMS) */
    uint32_t muffle_off;      /* uint16_t[TC*T] */
    uint32_t perm_off;        /* float[TC*T] */
    uint32_t echo_off;        /* uint16_t (half) [R*H] */
    uint32_t hit_points_off;  /* art_half3[R*H] (iff ART_OUT_HIT_RESULTS) */
    uint32_t hit_counts_off;  /* uint8_t[R]     (iff ART_OUT_HIT_RESULTS) */
    uint32_t hit_ids_off;     /* uint32_t[R*H]  (iff ART_OUT_HIT_RESULTS): ART_HIT_ID / ART_HIT_NONE */
} art_fan_layout;

/* Kernel families of the raytrace stage (art_kernel_times.kernel_ms order). */
#define ART_KERNEL_NEAREST     0 /* nearest_first_kernel (per bounce; multi-hit frames: the path epilogue folded in) */
#define ART_KERNEL_ECHO_MUFFLE 1 /* echo_muffle_kernel (one-hit frames: echo traversal + muffle rays, one launch) */
#define ART_KERNEL_ECHO        2 /* vis_kernel, the echo any-hit traversal (multi-hit frames: per bounce, side stream) */
#define ART_KERNEL_MUFFLE      3 /* muffle_kernel (multi-hit frames: once, after the last bounce) */

/* ABI 3.0 (80 B; 2.3 had 48 B). */
typedef struct {
    double raytrace_ms, permeate_ms, reduce_ms; /* summed hipEvent durations of the frame's stages */
    int32_t launches;                           /* frames timed */
    int32_t kernel_marks_dropped;               /* ART_CTX_TIME_EACH_KERNEL launches left unmarked (out of event pairs) */
    double kernel_ms[4];                        /* ART_CTX_TIME_EACH_KERNEL: summed durations per ART_KERNEL_* family */
    int32_t kernel_launches[4];                 /*   and the launches timed per family */
} art_kernel_times;

/* Record hipEvents around the stages of every frame of art_launch_device (art_set_flags). An event
 * record costs a few microseconds of GPU idle, so timed frames run slower than untimed ones: time
 * in a pass of its own, outside the frames whose wall time is measured. */
#define ART_CTX_TIME_KERNELS 0x2u
/* With ART_CTX_TIME_KERNELS: also an event pair around each kernel of the raytrace stage, on the
 * stream it runs on (art_kernel_times.kernel_ms). */
#define ART_CTX_TIME_EACH_KERNEL 0x200u
/* Frame outputs from the reference-order raytrace kernel (one ray per lane, every collider in
 * reference order; the kernel the test counts come from) instead of the throughput stage. */
#define ART_CTX_FORCE_REFERENCE_ORDER 0x4u
/* art_launch_device records the frame's completion event on the caller's stream before it returns
 * (ABI 3.1), so the caller may destroy or recycle that stream right after the call. Off by default:
 * the record costs the stream ~5 us of GPU idle per frame, and without it the event is recorded
 * lazily, on that stream, by the next call that has to wait for the frame. */
#define ART_CTX_EVENT_EACH_LAUNCH 0x400u
/* (0x8, 0x40 and 0x80 selected round-1 alternative raytrace implementations; they are gone and
 * the bits are reserved.) */

/* (0x100 selected hipGraph replay of a frame's launch sequence, ABI 2.1-2.2; it measured no faster
 * than direct launches and is gone, the bit is reserved.) */

ART_API int art_fan_layout_get(const art_frame_desc* desc, uint32_t out_flags, art_fan_layout* out);

/* Upload the scene (colliders, directions, targets, curves) to every device of the context and
 * build the device SoA records. Synchronous. Pointers in desc are host pointers. */
ART_API int art_scene_bind(art_ctx* ctx, const art_frame_desc* desc);

/* Enqueue one frame on the context's first device: d_origins = float3[fan_count] (device),
 * d_block = fan_count * stride bytes (device, in/out), stream = the hipStream_t to enqueue on
 * (NULL = the HIP default stream, e.g. torch's default stream). Kernels only; returns without
 * synchronizing and records no event (back-to-back frames run without gaps). The stream must stay
 * valid until the context's next call that touches the scene or its buffers (a bind, sync,
 * schedule, a launch on another stream, or art_destroy), which orders itself after the frame by
 * recording an event on it then; a caller that cannot keep its stream alive that long sets
 * ART_CTX_EVENT_EACH_LAUNCH. */
ART_API int art_launch_device(art_ctx* ctx, const float* d_origins, int32_t fan_count, void* d_block,
                              uint32_t out_flags, void* stream);

/* FibonacciDirectionsJobParallel (Jobs/FibonacciDirectionsJobParallel.cs:15-35) on the device:
 * d_out = half3[count] in HBM, enqueued on `stream`. Equals art_fibonacci_directions (host) bit
 * for bit; directions stay an input of art_frame_desc (the half3 bits are the contract). */
ART_API int art_fibonacci_directions_device(art_ctx* ctx, int32_t count, art_half3* d_out, void* stream);

/* The kernels' f32tof16 (Utility/HalfDataTypesUtility.cs:86-90 -> Unity.Mathematics math.f32tof16)
 * over the float bit patterns first_bits .. first_bits + count - 1 (wrapping), into d_out (HBM,
 * u16[count]) on `stream`: the device conversion every echo, hit point and direction goes through,
 * exposed so it can be checked against the host and the oracle over all 2^32 inputs. */
ART_API int art_f32tof16_device(art_ctx* ctx, uint32_t first_bits, uint32_t count, uint16_t* d_out, void* stream);

/* The OBB slab's reciprocal as the kernels compute it (recip_exact: v_rcp_f32 + one Newton step
 * where the exponent field lies in [3, 251], the IEEE division elsewhere), the bits of 1/x for
 * x = first_bits .. first_bits + count - 1 (wrapping) into d_out (HBM, u32[count]) on `stream`:
 * exposed so the claim that it equals 1.0f / x (RayIntersectsAABB's `1.0f / rayDir`,
 * Jobs/AudioRaytracerJobBatched.cs:289, reached from RayIntersectsOBB :314-320) is checked
 * over all 2^32 inputs. */
ART_API int art_recip_exact_device(art_ctx* ctx, uint32_t first_bits, uint32_t count, uint32_t* d_out, void* stream);

/* Same frame with the test-counting kernels (for the tests/s metric); synchronizes. */
ART_API int art_count_device(art_ctx* ctx, const float* d_origins, int32_t fan_count, void* d_block,
                             uint32_t out_flags, void* stream, art_test_counts* out);

/* Count the work the throughput raytrace kernel actually executes (ART_CTX_COUNT_EXECUTED):
 * exact intersection tests in lane-tests (every wave-level test counts 64, whatever the exec
 * mask), and broad-phase bound tests in lane-evaluations. The tests/s metric counts the tests the
 * reference algorithm executes (art_count_device); this is what the hardware did instead. */
#define ART_CTX_COUNT_EXECUTED 0x10u
typedef struct {
    uint64_t sphere, aabb, obb;      /* exact lane-tests executed */
    uint64_t cull_box;               /* BVH node box tests (lane-evaluations) */
    uint64_t cell_entries;           /* muffle candidate-list entries scanned (lane-evaluations) */
    uint64_t launches;               /* frames counted */
    uint64_t muffle_fallback;        /* muffle rays tested against every collider (no usable cell list) */
    uint64_t echo_pairs;             /* echo rays left to the BVH echo traversal (not decided by the nearest pass) */
    uint64_t bounce_rays[16];        /* live rays the nearest traversal traced per bounce (bounce k, k < 16) */
    /* The first five counters split by kernel family (ABI 2.3): [0] the nearest-hit traversals
     * (nearest_first_kernel), [1] the echo any-hit traversals (vis_kernel, the echo half of
     * echo_muffle_kernel), [2] the muffle rays (muffle_kernel, the muffle half of echo_muffle_kernel).
     * Each field above is the sum of its three entries. */
    struct {
        uint64_t sphere, aabb, obb, cull_box, cell_entries;
    } by_kernel[3];
} art_exec_counts;
/* Executed-work counters since the last call (needs ART_CTX_COUNT_EXECUTED); synchronizes. */
ART_API int art_executed_counts(art_ctx* ctx, art_exec_counts* out);

/* Sum of kernel times since the last call (needs ART_CTX_TIME_KERNELS); synchronizes. */
ART_API int art_kernel_timing(art_ctx* ctx, art_kernel_times* out);

/* Diagnostics (tests): the leaf order of the bound scene's BVH on the context's first device, one
 * reference per leaf slot (type << 30 | in-type index), at most cap of them; returns the number
 * written (the bound scene's collider count when cap allows) or a negative art error. Synchronizes. */
ART_API int art_debug_leaf_order(art_ctx* ctx, uint32_t* out, int32_t cap);

/* Context over an explicit list of HIP devices: fans of every art_schedule are sharded
 * contiguously over the list (one HIP stream, one scene copy and one set of buffers per entry).
 * An id may repeat: art_create_on({0, 0, 0}, 3, &ctx) runs the in-process multi-device split and
 * gather as three shards on three streams of device 0 (how the one-GPU tests exercise it).
 * art_create(mask) is art_create_on over the mask's set bits. */
ART_API int art_create_on(const int32_t* device_ids, int32_t count, art_ctx** out);

/* Number of HIP devices visible (0 when none); never fails. */
ART_API int art_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* ART_DEVICE_H */
