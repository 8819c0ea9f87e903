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
#include <cstdint>
#include <cstdlib>
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

// ---- tiled kernel: one lane per (source, channel), tiles transposed through LDS -------------
//
// The recurrences are serial over frames, so a lane owns one channel chain. The buffers are
// [source][frame][L,R]: a wave reads a tile of kTF frames of its kTS sources with coalesced 8-B
// loads (one instruction covers 256 contiguous bytes of two sources), transposes it through LDS,
// runs the chains out of LDS, and writes the tile back the same way. The next tile's loads are in
// flight while the current one is processed.
#ifndef ART_DSP_TF
#define ART_DSP_TF 64
#endif
constexpr int kTS = 32;              // sources per wave (lane = 2 * source + channel)
constexpr int kTF = ART_DSP_TF;      // frames per tile (64; 32 measured slower on large batches)
constexpr int kSPI = 64 / kTF;       // sources covered by one load instruction
static_assert(kTF == 32 || kTF == 64, "tile width");
constexpr int kRow = 2 * kTF + 2;    // floats per LDS row: bank (2 s + c + 2 n) mod 32 is distinct per half-wave
constexpr int kLoads = kTS * kTF / 64;  // float2 loads per lane per tile

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

struct Chain {
  float pm, pl, ph, pi;  // previousMuffle, previousLP, previousHP, previousInput of this channel
};

// M: bit 0 muffle, bit 1 low pass (fixed for the wave); M == 4: per-lane selects (exact: every
// selected value is computed with the same operations as in the fixed variants).
template <int M>
__device__ __forceinline__ float step(float x, const art_dsp_source_params& p, float gain, bool mf, bool lp,
                                      Chain& c) {
  if constexpr (M == 4) {
    const float m = c.pm + p.muffle_alpha * (x - c.pm);
    x = mf ? m : x;
    c.pm = mf ? m : c.pm;
  } else if constexpr (M & 1) {
    c.pm = c.pm + p.muffle_alpha * (x - c.pm);  // MuffleDSP.LowPass :43-44
    x = c.pm;
  }
  x = x * p.dry_boost;  // ReverbDSP :21-22
  x = x * gain;         // BinauralDSP :59-60
  if constexpr (M == 4) {
    const float l = c.pl + p.filter_alpha * (x - c.pl);
    const float h = p.filter_alpha * (c.ph + x - c.pi);
    c.pl = lp ? l : c.pl;
    c.ph = lp ? c.ph : h;
    c.pi = lp ? c.pi : x;
    x = lp ? l : h;
  } else if constexpr (M & 2) {
    c.pl = c.pl + p.filter_alpha * (x - c.pl);  // LowPass :92-93
    x = c.pl;
  } else {
    const float h = p.filter_alpha * (c.ph + x - c.pi);  // HighPass :102-105
    c.pi = x;
    c.ph = h;
    x = h;
  }
  return x * p.volume;  // AudioSpatializer.cs:84-85
}

template <int M>
__device__ __forceinline__ void run_tile(float* row, int n, const art_dsp_source_params& p, float gain, bool mf,
                                         bool lp, Chain& c) {
  if (n == kTF) {
    float x[kTF];
#pragma unroll
    for (int k = 0; k < kTF; ++k) x[k] = row[2 * k];
#pragma unroll
    for (int k = 0; k < kTF; ++k) x[k] = step<M>(x[k], p, gain, mf, lp, c);
#pragma unroll
    for (int k = 0; k < kTF; ++k) row[2 * k] = x[k];
  } else {
    for (int k = 0; k < n; ++k) row[2 * k] = step<M>(row[2 * k], p, gain, mf, lp, c);
  }
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ __launch_bounds__(64) void dsp_tiled_kernel(float* __restrict__ data, const long long* __restrict__ offsets,
                                                       const int* __restrict__ frames_of, int frames_all,
                                                       const art_dsp_source_params* __restrict__ params,
                                                       art_dsp_state* __restrict__ state, int count,
                                                       uint32_t nbytes) {
  __shared__ float tile[kTS * kRow];
  const int lane = threadIdx.x;
  const int s0 = blockIdx.x * kTS;
  const int sl = lane >> 1, ch = lane & 1;
  const int s = s0 + sl;
  art_dsp_source_params p{};
  int my_frames = 0;
  Chain c{};
  if (s < count) {
    p = params[s];
    if (!(p.flags & 4)) {
      my_frames = frames_of ? frames_of[s] : frames_all;
      const float* sv = reinterpret_cast<const float*>(state + s);
      c.pm = sv[0 + ch]; c.pl = sv[2 + ch]; c.ph = sv[4 + ch]; c.pi = sv[6 + ch];
    }
  }
  const bool mf = (p.flags & 1) != 0, lp = (p.flags & 2) != 0;
  const float gain = ch ? p.gain_right : p.gain_left;
  const int cls = my_frames > 0 ? (p.flags & 3) : -1;
  const int fmax = wave_max_i(my_frames);
  if (fmax == 0) return;
  const uint64_t b0 = __ballot(cls == 0), b1 = __ballot(cls == 1), b2 = __ballot(cls == 2), b3 = __ballot(cls == 3);
  const bool generic = (b0 != 0) + (b1 != 0) + (b2 != 0) + (b3 != 0) >= 3;

  // loader view: item i of this lane is frame lane % kTF of local source kSPI * i + lane / kTF.
  // Buffer loads/stores with the hardware range check: an item past its source's frames gets the
  // offset nbytes (loads 0, store dropped), so the transfers are branch-free and the wait for the
  // next tile's loads does not also wait for this tile's stores.
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(data, 0, (int)nbytes, 0x00020000);
  const int lf = lane & (kTF - 1);
  // per-source frames and byte offset come from the source's channel-0 lane (no dependent loads)
  const long long my_off = my_frames > 0 ? (offsets ? offsets[s] : (long long)s * frames_all * 2) : 0;
  const int my_ob = (int)(uint32_t)(my_off * 4);
  uint32_t obase[kLoads];
  int lfr[kLoads];
#pragma unroll
  for (int i = 0; i < kLoads; ++i) {
    const int src_lane = 2 * (kSPI * i + lane / kTF);
    lfr[i] = __shfl(my_frames, src_lane, 64);
    obase[i] = (uint32_t)__shfl(my_ob, src_lane, 64);
  }
  u32x2 pre[kLoads];
  auto voff = [&](int i, int t) -> uint32_t {
    const int f = t * kTF + lf;
    return f < lfr[i] ? obase[i] + (uint32_t)f * 8u : nbytes;
  };
  auto load = [&](int t) {
#pragma unroll
    for (int i = 0; i < kLoads; ++i) pre[i] = __builtin_amdgcn_raw_buffer_load_b64(rs, voff(i, t), 0, 0);
  };
  const int ntiles = (fmax + kTF - 1) / kTF;
  float* row = tile + sl * kRow + ch;
  load(0);
  // 16 out-of-range stores (dropped by the range check): the loop is then entered with the same
  // memory-op order as its back edge (loads, then stores), so the wait for the prefetched tile at
  // the loop head leaves the previous tile's stores in flight (vmcnt(16), not vmcnt(0))
#pragma unroll
  for (int i = 0; i < kLoads; ++i) __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, rs, nbytes + 16u * i, 0, 0);
  for (int t = 0; t < ntiles; ++t) {
#pragma unroll
    for (int i = 0; i < kLoads; ++i)
      *reinterpret_cast<u32x2*>(tile + (kSPI * i + lane / kTF) * kRow + 2 * lf) = pre[i];
    __syncthreads();
    load(t + 1);  // past the last tile every offset is out of range: loads 0, no branch
    const int n = min(max(my_frames - t * kTF, 0), kTF);
    if (generic) {
      run_tile<4>(row, n, p, gain, mf, lp, c);
    } else {
      if (b0 && cls == 0) run_tile<0>(row, n, p, gain, mf, lp, c);
      if (b1 && cls == 1) run_tile<1>(row, n, p, gain, mf, lp, c);
      if (b2 && cls == 2) run_tile<2>(row, n, p, gain, mf, lp, c);
      if (b3 && cls == 3) run_tile<3>(row, n, p, gain, mf, lp, c);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kLoads; ++i) {
      const u32x2 v = *reinterpret_cast<const u32x2*>(tile + (kSPI * i + lane / kTF) * kRow + 2 * lf);
      __builtin_amdgcn_raw_buffer_store_b64(v, rs, voff(i, t), 0, 0);
    }
    __syncthreads();
  }
  if (my_frames > 0) {
    float* sv = reinterpret_cast<float*>(state + s);
    sv[0 + ch] = c.pm; sv[2 + ch] = c.pl; sv[4 + ch] = c.ph; sv[6 + ch] = c.pi;
  }
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
    // BinauralDSP.Process runs unbursted on the audio thread (no [BurstCompile] under Audio/), so
    // Unity.Mathematics' atan2 / sin / cos are (float)System.Math.Atan2/Sin/Cos: double precision,
    // rounded once to float.
    const float azimuth = (float)std::atan2((double)ld[0], (double)ld[2]) * kToDegrees;
    float eps = st.pan_strength;
    if (st.distance_based_panning) eps *= usaturate(dist / st.max_pan_distance);
    const float pan = (float)std::sin((double)(azimuth * kToRadians)) * eps;
    const float gl = std::sqrt(0.5f * (1.0f - pan));
    const float gr = std::sqrt(0.5f * (1.0f + pan));
    const float front = umax(0.0f, (float)std::cos((double)(azimuth * kToRadians)));
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

void launch_dsp(float* data, unsigned long long data_bytes, const long long* offsets, const int* frames_of,
                int frames_all, const art_dsp_source_params* params, art_dsp_state* state, int count, hipStream_t st) {
  if (count <= 0) return;
  static const int mode = [] {  // ART_DSP_KERNEL=lane: one lane per source, direct loads (A/B only)
    const char* e = std::getenv("ART_DSP_KERNEL");
    return e && !std::strcmp(e, "lane") ? 1 : 0;
  }();
  // the tiled kernel's 8-B buffer ops need an 8-B aligned base (every source offset is an even
  // float count) and 32-bit byte offsets
  const bool aligned = (reinterpret_cast<uintptr_t>(data) & 7) == 0;
  if (mode == 0 && aligned && data_bytes < 0x7fffffffULL) {
    hipLaunchKernelGGL(dsp_tiled_kernel, dim3((count + kTS - 1) / kTS), dim3(64), 0, st, data, offsets, frames_of,
                       frames_all, params, state, count, (uint32_t)data_bytes);
  } else {
    hipLaunchKernelGGL(dsp_kernel, dim3((count + kDspBlock - 1) / kDspBlock), dim3(kDspBlock), 0, st, data, offsets,
                       frames_of, frames_all, params, state, count);
  }
}

}  // namespace art
