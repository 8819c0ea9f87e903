/*
 * art_dsp.h — per-sample audio DSP of the spatializer (SURVEY.md §8 f rank 1), the direct consumer
 * of the ray tracer's AudioTargetRTSettings.
 *
 * Reference (paths relative to "Assets/C# Scripts/"):
 *   AudioSpatializer.OnAudioFilterRead   Audio/AudioTarget/AudioSpatializer.cs:70-87
 *     muffleDSP.Process                  Audio/AudioTarget/MuffleDSP.cs:13-32, LowPass :38-45
 *     reverbDSP.Process                  Audio/AudioTarget/ReverbDSP.cs:10-24
 *     binauralDSP.Process                Audio/AudioTarget/BinauralDSP.cs:15-82, LowPass :87-94,
 *                                        HighPass :97-106
 *     volume multiplier                  AudioSpatializer.cs:79-86
 *   cached inputs (main thread)          AudioSpatializer.cs:61-67 (local direction, distance)
 *   settings                             DataTypes/AudioSpatializerSettings.cs:4-45
 *   curves                               DataTypes/NativeSampledAnimationCurve.cs:64-89
 *
 * One art_audio_source = one AudioSpatializer's OnAudioFilterRead call: an interleaved buffer
 * processed in place, plus the filter state the C# structs keep between calls. The per-buffer
 * scalars (curve lookups, filter coefficients, binaural gains with atan2/sin/cos) are computed on
 * the host; the per-sample recurrences run on the GPU, one lane per source (both channels).
 */
#ifndef ART_DSP_H
#define ART_DSP_H

#include "art.h"

#ifdef __cplusplus
extern "C" {
#endif

/* StereoFloat (DataTypes/StereoFloat.cs:5-14) */
typedef struct { float left, right; } art_stereo;

/* Filter state of one AudioSpatializer (in/out; zero-initialised like the C# structs). */
typedef struct {
    art_stereo previous_muffle;  /* MuffleDSP.previousMuffle (MuffleDSP.cs:9) */
    art_stereo previous_lp;      /* BinauralDSP.previousLP (BinauralDSP.cs:9) */
    art_stereo previous_hp;      /* BinauralDSP.previousHP (:10) */
    art_stereo previous_input;   /* BinauralDSP.previousInput (:11) */
} art_dsp_state;

/* AudioSpatializerSettings fields the per-sample chain reads (AudioSpatializerSettings.cs:8-45). */
typedef struct {
    float pan_strength;                       /* :8 */
    float rear_attenuation_strength;          /* :12 */
    int32_t distance_based_panning;           /* :15 (bool) */
    float max_pan_distance;                   /* :16 */
    int32_t distance_based_rear_attenuation;  /* :19 (bool) */
    float max_rear_attenuation_distance;      /* :20 */
    float max_elevation_effect_distance;      /* :23 */
    float low_pass_cutoff_min, low_pass_cutoff_max;    /* :26 */
    float low_pass_volume;                    /* :29 */
    float high_pass_cutoff_min, high_pass_cutoff_max;  /* :32 */
    float high_pass_volume;                   /* :35 */
    art_curve muffle_curve;                   /* :38 (baked) */
    float muffle_cutoff_min, muffle_cutoff_max;        /* :39 */
    art_curve reverb_volume_curve;            /* :45 (baked) */
    float reverb_dry_boost_min, reverb_dry_boost_max;  /* :44 */
} art_spatializer_settings;

/* One OnAudioFilterRead call of one AudioSpatializer. */
typedef struct {
    float* data;              /* interleaved samples, frames * channels, processed in place */
    int32_t frames;           /* samples per channel */
    int32_t channels;         /* only 2 is processed (AudioSpatializer.cs:72); others are left as is */
    float muffle_strength;    /* audioTargetSettings.MuffleStrength */
    float reverb_volume;      /* audioTargetSettings.ReverbVolume */
    float local_dir[3];       /* cachedLocalDir (AudioSpatializer.cs:64) */
    float listener_distance;  /* cachedListenerDistance (:66) */
    float volume_multiplier;  /* volumeMultiplier (:18) */
    art_dsp_state* state;     /* in/out */
} art_audio_source;

/* Process count sources (synchronous: buffers and states are updated when this returns). */
ART_API int art_dsp_process(art_ctx* ctx, const art_spatializer_settings* settings, art_audio_source* sources,
                            int32_t count, int32_t sample_rate);

/* Per-buffer scalars of one stereo source, as art_dsp_process derives them on the host. */
typedef struct {
    float muffle_alpha;       /* LowPass alpha of the muffle cutoff (MuffleDSP.cs:40-42) */
    float dry_boost;          /* ReverbDSP.cs:12-13 */
    float gain_left, gain_right;  /* BinauralDSP sampleModification (:48-50) */
    float filter_alpha;       /* low-pass alpha (elevation <= 0) or high-pass alpha (:65-76, :89-101) */
    float volume;             /* volume multiplier */
    int32_t flags;            /* bit 0: muffle active (:22); bit 1: low pass (else high pass) (:63) */
    int32_t reserved;
} art_dsp_source_params;

ART_API int art_dsp_source_params_get(const art_spatializer_settings* settings, const art_audio_source* source,
                                      int32_t sample_rate, art_dsp_source_params* out);

/* Device-resident batch (servers, bench): count stereo sources of `frames` samples each, stored
 * back to back in d_data (float [count][frames][2]); d_params (art_dsp_source_params[count]) and
 * d_state (art_dsp_state[count]) are device arrays. Enqueued on `stream`, not synchronised. */
ART_API int art_dsp_process_device(art_ctx* ctx, float* d_data, const art_dsp_source_params* d_params,
                                   art_dsp_state* d_state, int32_t count, int32_t frames, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ART_DSP_H */
