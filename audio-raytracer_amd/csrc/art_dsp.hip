// art_dsp.hip — per-sample spatializer DSP (include/art_dsp.h; SURVEY.md §8 f rank 1).
//
// AudioSpatializer.OnAudioFilterRead (Audio/AudioTarget/AudioSpatializer.cs:70-87) runs four
// passes over an interleaved stereo buffer: MuffleDSP (MuffleDSP.cs:13-32), ReverbDSP
// (ReverbDSP.cs:10-24), BinauralDSP (BinauralDSP.cs:15-82) and the volume multiplier. Every
// per-sample value of a pass depends only on the same sample's value after the previous pass and
// on the pass's own filter state, so the passes fuse into one loop over samples with identical
// results. The quantities the C# recomputes per sample (curve lookups, cutoffs, filter alphas)
// are constant over a buffer and are computed once on the host with the same float operations
// (art_dsp_source_params_get); the GPU runs the recurrences, one lane per source, both channels
// interleaved (two independent chains per lane).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/art_dsp.h"
#include "art_internal.hpp"

#pragma clang fp contract(off)

namespace art {
namespace {

constexpr int kDspBlock = 256;

// Unity.Mathematics semantics (same definitions as unity_math.hpp, host side)
inline float umin(float x, float y) { return (y != y || x < y) ? x : y; }
inline float umax(float x, float y) { return (y != y || x > y) ? x : y; }
inline float usaturate(float x) { return umax(0.0f, umin(1.0f, x)); }
inline float ulerp(float a, float b, float s) { return a + s * (b - a); }
inline float uclamp(float x, float a, float b) { return umax(a, umin(b, x)); }
constexpr float kToDegrees = 57.29578f;      // math.degrees
constexpr float kToRadians = 0.0174532924f;  // math.radians
constexpr float kDoublePi = 2.0f * 3.14159265f;  // MuffleDSP.cs:35 / BinauralDSP.cs:84

// NativeSampledAnimationCurve.Evaluate (NativeSampledAnimationCurve.cs:64-89)
float curve_eval(const art_curve& c, float time) {
  const float percent = time / c.length;
  const int n = c.sample_count;
  const float cp = umax(0.0f, umin((float)(n - 1), percent * (float)(n - 1)));
  const int fi = (int)std::floor(cp), ci = (int)std::ceil(cp);
  return ulerp(c.baked[fi], c.baked[ci], cp - (float)fi);
}

float lowpass_alpha(float cutoff, float sr) {  // MuffleDSP.cs:40-42, BinauralDSP.cs:89-91
  const float rc = 1.0f / (cutoff * kDoublePi);
  const float dt = 1.0f / sr;
  return dt / (rc + dt);
}
float highpass_alpha(float cutoff, float sr) {  // BinauralDSP.cs:99-101
  const float rc = 1.0f / (cutoff * kDoublePi);
  const float dt = 1.0f / sr;
  return rc / (rc + dt);
}

bool curve_ok(const art_curve& c) { return c.baked && c.sample_count >= 2; }

// One lane per source; both channels. data: this source's interleaved frames.
__global__ __launch_bounds__(kDspBlock) void dsp_kernel(float* __restrict__ data, const long long* __restrict__ offsets,
                                                        const int* __restrict__ frames_of, int frames_all,
                                                        const art_dsp_source_params* __restrict__ params,
                                                        art_dsp_state* __restrict__ state, int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  const art_dsp_source_params p = params[s];
  if (p.flags & 4) return;  // not stereo: left as is (AudioSpatializer.cs:72)
  const int frames = frames_of ? frames_of[s] : frames_all;
  float* d = data + (offsets ? offsets[s] : (long long)s * frames_all * 2);
  art_dsp_state st = state[s];
  const bool muffle = (p.flags & 1) != 0, lp = (p.flags & 2) != 0;
  float pmL = st.previous_muffle.left, pmR = st.previous_muffle.right;
  float plL = st.previous_lp.left, plR = st.previous_lp.right;
  float phL = st.previous_hp.left, phR = st.previous_hp.right;
  float piL = st.previous_input.left, piR = st.previous_input.right;
  auto sample = [&](float& l, float& r) {
    if (muffle) {  // MuffleDSP.LowPass :43-44
      pmL += p.muffle_alpha * (l - pmL); l = pmL;
      pmR += p.muffle_alpha * (r - pmR); r = pmR;
    }
    l = l * p.dry_boost;  // ReverbDSP :21-22
    r = r * p.dry_boost;
    l = l * p.gain_left;  // BinauralDSP :59-60
    r = r * p.gain_right;
    if (lp) {  // LowPass :92-93
      plL += p.filter_alpha * (l - plL); l = plL;
      plR += p.filter_alpha * (r - plR); r = plR;
    } else {   // HighPass :102-105
      const float oL = p.filter_alpha * (phL + l - piL);
      piL = l; phL = oL; l = oL;
      const float oR = p.filter_alpha * (phR + r - piR);
      piR = r; phR = oR; r = oR;
    }
    l = l * p.volume;  // AudioSpatializer.cs:84-85
    r = r * p.volume;
  };
  int i = 0;
  if ((reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    float4* d4 = reinterpret_cast<float4*>(d);
    for (; i + 2 <= frames; i += 2) {
      float4 v = d4[i >> 1];
      sample(v.x, v.y);
      sample(v.z, v.w);
      d4[i >> 1] = v;
    }
  }
  for (; i < frames; ++i) {
    float l = d[2 * i], r = d[2 * i + 1];
    sample(l, r);
    d[2 * i] = l;
    d[2 * i + 1] = r;
  }
  st.previous_muffle.left = pmL; st.previous_muffle.right = pmR;
  st.previous_lp.left = plL; st.previous_lp.right = plR;
  st.previous_hp.left = phL; st.previous_hp.right = phR;
  st.previous_input.left = piL; st.previous_input.right = piR;
  state[s] = st;
}

}  // namespace

// Per-buffer scalars (everything the C# recomputes per sample is constant over the buffer).
int dsp_source_params(const art_spatializer_settings& st, const art_audio_source& src, int sample_rate,
                      art_dsp_source_params& p) {
  std::memset(&p, 0, sizeof p);
  if (src.channels != 2) { p.flags = 4; return ART_OK; }
  if (!curve_ok(st.reverb_volume_curve) || (src.muffle_strength > 0.0f && !curve_ok(st.muffle_curve)))
    return ART_E_INVALID;
  const float sr = (float)sample_rate;
  if (src.muffle_strength > 0.0f) {  // MuffleDSP.cs:22-26
    const float muffle = curve_eval(st.muffle_curve, src.muffle_strength);
    const float cutoff = ulerp(st.muffle_cutoff_max, st.muffle_cutoff_min, muffle);
    p.muffle_alpha = lowpass_alpha(cutoff, sr);
    p.flags |= 1;
  }
  {  // ReverbDSP.cs:12-13
    const float t = curve_eval(st.reverb_volume_curve, src.reverb_volume);
    p.dry_boost = ulerp(st.reverb_dry_boost_min, st.reverb_dry_boost_max, t);
  }
  {  // BinauralDSP.cs:17-50, :65, :73
    const float* ld = src.local_dir;
    const float dist = src.listener_distance;
    const float azimuth = std::atan2(ld[0], ld[2]) * kToDegrees;
    float eps = st.pan_strength;
    if (st.distance_based_panning) eps *= usaturate(dist / st.max_pan_distance);
    const float pan = std::sin(azimuth * kToRadians) * eps;
    const float gl = std::sqrt(0.5f * (1.0f - pan));
    const float gr = std::sqrt(0.5f * (1.0f + pan));
    const float front = umax(0.0f, std::cos(azimuth * kToRadians));
    float rear = ulerp(1.0f - st.rear_attenuation_strength, 1.0f, front);
    if (st.distance_based_rear_attenuation) {
      const float df = usaturate(1.0f - (dist / st.max_rear_attenuation_distance));
      rear = uclamp(rear * df, 1.0f - st.rear_attenuation_strength, 1.0f);
    }
    const float elev = ld[1] <= 0.0f ? ulerp(1.0f, st.low_pass_volume, usaturate(-ld[1]))
                                     : ulerp(1.0f, st.high_pass_volume, usaturate(ld[1]));
    p.gain_left = gl * rear * elev;
    p.gain_right = gr * rear * elev;
    if (ld[1] <= 0.0f) {
      const float c = ulerp(st.low_pass_cutoff_min, st.low_pass_cutoff_max, usaturate(-ld[1])) *
                      (1.0f - 0.5f * usaturate(dist / st.max_elevation_effect_distance));
      p.filter_alpha = lowpass_alpha(c, sr);
      p.flags |= 2;
    } else {
      const float c = ulerp(st.high_pass_cutoff_min, st.high_pass_cutoff_max, usaturate(ld[1])) *
                      (1.0f + 0.5f * usaturate(dist / st.max_elevation_effect_distance));
      p.filter_alpha = highpass_alpha(c, sr);
    }
  }
  p.volume = src.volume_multiplier;
  return ART_OK;
}

void launch_dsp(float* data, const long long* offsets, const int* frames_of, int frames_all,
                const art_dsp_source_params* params, art_dsp_state* state, int count, hipStream_t st) {
  if (count <= 0) return;
  hipLaunchKernelGGL(dsp_kernel, dim3((count + kDspBlock - 1) / kDspBlock), dim3(kDspBlock), 0, st, data, offsets,
                     frames_of, frames_all, params, state, count);
}

}  // namespace art
