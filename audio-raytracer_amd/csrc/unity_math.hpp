// unity_math.hpp — bit-exact Unity.Mathematics 1.3.2 arithmetic for HIP device (and host) code.
//
// Semantics restated from SURVEY.md App. A (the package is not vendored in the reference; its
// call sites are e.g. Jobs/AudioRaytracerJobBatched.cs:127,130,162,165,294-298,316-317,473-525,
// DataTypes/halfQuaternion.cs:42,45, Jobs/ProcessAudioDataJob.cs:71).
//
// Rules that keep device results bit-identical to the strict-IEEE CPU path:
//   * this translation unit is compiled with -ffp-contract=off (and the pragma below): no FMA;
//   * f32 denormals are preserved (never -fgpu-flush-denormals-to-zero);
//   * '/' and sqrtf stay correctly rounded (hipcc default);
//   * f32tof16 is Unity's round-half-up algorithm, never v_cvt_f16_f32 (RNE);
//   * math.min/max are the explicit NaN-aware selects (umin/umax), except where a caller has
//     proven the IEEE minNum/maxNum form equivalent (see fmin_ieee below).
#pragma once

#include <stdint.h>

#pragma clang fp contract(off)

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define ART_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define ART_HD inline
#endif

namespace art {

ART_HD uint32_t asuint(float f) { return __builtin_bit_cast(uint32_t, f); }
ART_HD float asfloat(uint32_t u) { return __builtin_bit_cast(float, u); }
ART_HD bool ufinite(float x) { return (asuint(x) & 0x7F800000u) != 0x7F800000u; }  // isfinite on host and device

// math.min / math.max: isnan(y) || x < y ? x : y   (App. A.2)
ART_HD float umin(float x, float y) { return (y != y || x < y) ? x : y; }
ART_HD float umax(float x, float y) { return (y != y || x > y) ? x : y; }
ART_HD float usign(float x) { return (x > 0.0f ? 1.0f : 0.0f) - (x < 0.0f ? 1.0f : 0.0f); }
ART_HD float usaturate(float x) { return umax(0.0f, umin(1.0f, x)); }
ART_HD float ulerp(float a, float b, float s) { return a + s * (b - a); }

// IEEE minNum/maxNum (v_min_f32 / v_max_f32 in IEEE mode): identical to umin/umax on every input
// except that a {+0,-0} pair may return the other zero. Used only where the sign of a zero result
// provably cannot reach an output (any-hit comparisons, permeation loss terms, nearest-hit
// ordering) — see DESIGN.md "min/max".
ART_HD float fmin_ieee(float x, float y) { return __builtin_fminf(x, y); }
ART_HD float fmax_ieee(float x, float y) { return __builtin_fmaxf(x, y); }

// math.f32tof16 (App. A.1): truncate bits 0-11, round half up on bit 12; subnormal halves via an
// f32 multiply into the f32-denormal range (double rounding, needs f32 denormals).
ART_HD uint16_t f32tof16(float x) {
  const int32_t infinity_32 = 255 << 23;
  const uint32_t msk = 0x7FFFF000u;
  uint32_t ux = asuint(x);
  uint32_t uux = ux & msk;
  uint32_t h = (uint32_t)(asuint(umin(asfloat(uux) * 1.92592994e-34f, 260042752.0f)) + 0x1000u) >> 13;
  h = ((int32_t)uux >= infinity_32) ? (((int32_t)uux > infinity_32) ? 0x7e00u : 0x7c00u) : h;
  return (uint16_t)(h | (ux & ~msk) >> 16);
}

// math.f16tof32 (exact, NaN payload preserved)
ART_HD float f16tof32(uint16_t hx) {
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

struct vec3 { float x, y, z; };
struct quat { float x, y, z, w; };

ART_HD vec3 mk3(float x, float y, float z) { vec3 r; r.x = x; r.y = y; r.z = z; return r; }
ART_HD vec3 operator+(vec3 a, vec3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
ART_HD vec3 operator-(vec3 a, vec3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
ART_HD vec3 operator*(vec3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
ART_HD vec3 operator*(float s, vec3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
// dot: left to right, two roundings per add, no contraction (App. A.3)
ART_HD float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
ART_HD float dot(quat a, quat b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
// cross(x, y) = (x * y.yzx - x.yzx * y).yzx
ART_HD vec3 cross(vec3 x, vec3 y) {
  return mk3(x.y * y.z - x.z * y.y, x.z * y.x - x.x * y.z, x.x * y.y - x.y * y.x);
}
ART_HD float rsqrt_u(float x) { return 1.0f / sqrtf(x); }
ART_HD vec3 normalize(vec3 v) { return rsqrt_u(dot(v, v)) * v; }
ART_HD float length(vec3 v) { return sqrtf(dot(v, v)); }
ART_HD float distance(vec3 x, vec3 y) { return length(y - x); }
ART_HD vec3 reflect(vec3 i, vec3 n) { return i - (2.0f * n) * dot(i, n); }
ART_HD vec3 abs3(vec3 a) { return mk3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }

// mul(quaternion q, vec3 v) = v + q.w * t + cross(q.xyz, t), t = 2 * cross(q.xyz, v)
ART_HD vec3 qmul(quat q, vec3 v) {
  vec3 qv = mk3(q.x, q.y, q.z);
  vec3 t = 2.0f * cross(qv, v);
  return (v + q.w * t) + cross(qv, t);
}
// inverse(q) = rcp(dot(q,q)) * q * (-1,-1,-1,1)
ART_HD quat qinverse(quat q) {
  float r = 1.0f / dot(q, q);
  quat o;
  o.x = (r * q.x) * -1.0f; o.y = (r * q.y) * -1.0f; o.z = (r * q.z) * -1.0f; o.w = (r * q.w) * 1.0f;
  return o;
}
ART_HD quat qnormalize(quat q) {
  float r = rsqrt_u(dot(q, q));
  quat o; o.x = r * q.x; o.y = r * q.y; o.z = r * q.z; o.w = r * q.w;
  return o;
}
// halfQuaternion.QuaternionValue — DataTypes/halfQuaternion.cs:34-46
ART_HD quat half_quaternion_value(uint16_t hx, uint16_t hy, uint16_t hz) {
  float xx = f16tof32(hx), yy = f16tof32(hy), zz = f16tof32(hz);
  float wSquared = 1.0f - (xx * xx + yy * yy + zz * zz);
  float w = wSquared > 0.0f ? sqrtf(wSquared) : 0.0f;
  quat q; q.x = xx; q.y = yy; q.z = zz; q.w = w;
  return qnormalize(q);
}

}  // namespace art
