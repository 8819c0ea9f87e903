// art_synth.cpp — deterministic synthetic scenes. Input generation only.
//
// RNG: splitmix64. U[a,b) = a + (b - a) * ((u >> 40) * 2^-24) in fp32.
// Box half-width L = round(40 * (C / 4096)^(1/3)). Colliders: centers U[-L, L)^3, sizes
// U[0.25, 2.5), quantised with Unity f32tof16. OBBs store halfQuaternion(inverse(q)) of a
// uniform (Shoemake) rotation q, as Audio/Colliders/AudioOBBCollider.cs:59 and
// DataTypes/halfQuaternion.cs:47-61 do. Materials: the four shipped presets
// (Assets/ScriptableObjects/AudioMaterials/*.asset:17-21). Each target owns one collider at its
// position (first in its type array). Fan origins U[-L/2, L/2)^3, rejected inside any collider.
#include <cmath>
#include <cstring>

#include "../../include/art_synth.h"
#include "unity_math.hpp"

using namespace art;

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  float u01() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }
  float uniform(float a, float b) { return a + (b - a) * u01(); }
};

// {absorption, density, echo} half bits: Concrete, Echo, Steel, Wood
const art_material kMaterials[4] = {
    {0x3400, 0x3C00, 0x3C00}, {0x0000, 0x4500, 0x4200}, {0x0000, 0x3C00, 0x3C00}, {0x0000, 0x4500, 0x3C00}};
const art_material kDefaultMaterial = {0x0000, 0x3C00, 0x3C00};  // AudioMaterialProperties.Default

art_half3 h3(float x, float y, float z) {
  art_half3 r;
  r.x = f32tof16(x); r.y = f32tof16(y); r.z = f32tof16(z);
  return r;
}

bool inside_sphere(const art_sphere& s, const float p[3]) {
  float dx = p[0] - f16tof32(s.center.x), dy = p[1] - f16tof32(s.center.y), dz = p[2] - f16tof32(s.center.z);
  float r = f16tof32(s.radius);
  return dx * dx + dy * dy + dz * dz <= r * r;
}
bool inside_box(float lx, float ly, float lz, art_half3 size) {
  return std::fabs(lx) <= f16tof32(size.x) && std::fabs(ly) <= f16tof32(size.y) && std::fabs(lz) <= f16tof32(size.z);
}
bool inside_aabb(const art_aabb& a, const float p[3]) {
  return inside_box(p[0] - f16tof32(a.center.x), p[1] - f16tof32(a.center.y), p[2] - f16tof32(a.center.z), a.size);
}
bool inside_obb(const art_obb& b, const float p[3]) {
  quat q = half_quaternion_value(b.rot_x, b.rot_y, b.rot_z);  // stored = world-to-local rotation
  vec3 l = qmul(q, mk3(p[0] - f16tof32(b.center.x), p[1] - f16tof32(b.center.y), p[2] - f16tof32(b.center.z)));
  return inside_box(l.x, l.y, l.z, b.size);
}

}  // namespace

extern "C" {

ART_API uint16_t art_f32tof16(float x) { return f32tof16(x); }
ART_API float art_f16tof32(uint16_t h) { return f16tof32(h); }
ART_API void art_f32tof16_range(uint32_t first_bits, uint32_t count, uint16_t* out) {
  for (uint32_t i = 0; i < count; ++i) out[i] = f32tof16(asfloat(first_bits + i));
}

// FibonacciDirectionsJobParallel.Execute (Jobs/FibonacciDirectionsJobParallel.cs:15-35). cos/sin are
// evaluated in double and rounded to float (the correctly rounded float values), exactly as
// fibonacci_kernel does on the device, so host and device directions are identical; glibc's
// cosf/sinf (the oracle's) differ from them in a few arguments per million.
ART_API void art_fibonacci_directions(int32_t count, art_half3* out) {
  for (int32_t i = 0; i < count; ++i) {
    float phi = 3.14159265f * (3.0f - std::sqrt(5.0f));
    float y = 1.0f - ((float)i / (float)(count - 1)) * 2.0f;
    float radius = std::sqrt(1.0f - y * y);
    float theta = phi * (float)i;
    float x = (float)std::cos((double)theta) * radius;
    float z = (float)std::sin((double)theta) * radius;
    out[i] = h3(x, y, z);
  }
}

ART_API int art_synth_scene(const art_synth_config* cfg, art_sphere* sph, art_aabb* aabb, art_obb* obb, float* targets,
                            float* origins, art_half3* dirs) {
  if (!cfg || cfg->target_count <= 0 || cfg->ray_count <= 0 || cfg->fan_count < 0) return ART_E_INVALID;
  const int ns = cfg->sphere_count, na = cfg->aabb_count, no = cfg->obb_count, T = cfg->target_count;
  const int owned_n = cfg->owned_type == ART_OWN_SPHERE ? ns : (cfg->owned_type == ART_OWN_AABB ? na : no);
  if (ns < 0 || na < 0 || no < 0 || owned_n < T) return ART_E_INVALID;
  if ((ns && !sph) || (na && !aabb) || (no && !obb) || !targets || (cfg->fan_count && !origins) || !dirs) return ART_E_INVALID;
  const int C = ns + na + no;
  const float L = (float)std::llround(40.0 * std::cbrt((double)C / 4096.0));
  Rng rng{cfg->seed};

  for (int t = 0; t < T; ++t)
    for (int k = 0; k < 3; ++k) targets[3 * t + k] = rng.uniform(-L / 2, L / 2);

  // owned colliders (App. D 6)
  for (int t = 0; t < T; ++t) {
    art_half3 c = h3(targets[3 * t], targets[3 * t + 1], targets[3 * t + 2]);
    if (cfg->owned_type == ART_OWN_SPHERE) {
      sph[t].center = c; sph[t].radius = f32tof16(0.5f); sph[t].material = kDefaultMaterial; sph[t].audio_target_id = (int16_t)t;
    } else if (cfg->owned_type == ART_OWN_AABB) {
      aabb[t].center = c; aabb[t].size = h3(0.5f, 0.5f, 0.5f); aabb[t].material = kDefaultMaterial;
      aabb[t].audio_target_id = (int16_t)t;
    } else {
      obb[t].center = c; obb[t].size = h3(0.5f, 0.5f, 0.5f); obb[t].rot_x = obb[t].rot_y = obb[t].rot_z = 0;
      obb[t].material = kDefaultMaterial; obb[t].audio_target_id = (int16_t)t;
    }
  }
  const int s0 = cfg->owned_type == ART_OWN_SPHERE ? T : 0;
  const int a0 = cfg->owned_type == ART_OWN_AABB ? T : 0;
  const int o0 = cfg->owned_type == ART_OWN_OBB ? T : 0;
  for (int i = s0; i < ns; ++i) {
    float x = rng.uniform(-L, L), y = rng.uniform(-L, L), z = rng.uniform(-L, L);
    sph[i].center = h3(x, y, z);
    sph[i].radius = f32tof16(rng.uniform(0.25f, 2.5f));
    sph[i].material = kMaterials[rng.next() >> 62];
    sph[i].audio_target_id = -1;
  }
  for (int i = a0; i < na; ++i) {
    float x = rng.uniform(-L, L), y = rng.uniform(-L, L), z = rng.uniform(-L, L);
    aabb[i].center = h3(x, y, z);
    float hx = rng.uniform(0.25f, 2.5f), hy = rng.uniform(0.25f, 2.5f), hz = rng.uniform(0.25f, 2.5f);
    aabb[i].size = h3(hx, hy, hz);
    aabb[i].material = kMaterials[rng.next() >> 62];
    aabb[i].audio_target_id = -1;
  }
  for (int i = o0; i < no; ++i) {
    float x = rng.uniform(-L, L), y = rng.uniform(-L, L), z = rng.uniform(-L, L);
    obb[i].center = h3(x, y, z);
    float hx = rng.uniform(0.25f, 2.5f), hy = rng.uniform(0.25f, 2.5f), hz = rng.uniform(0.25f, 2.5f);
    obb[i].size = h3(hx, hy, hz);
    // Shoemake uniform rotation
    float u1 = rng.u01(), u2 = rng.u01(), u3 = rng.u01();
    const float two_pi = 6.28318531f;
    quat q;
    q.x = std::sqrt(1.0f - u1) * std::sin(two_pi * u2);
    q.y = std::sqrt(1.0f - u1) * std::cos(two_pi * u2);
    q.z = std::sqrt(u1) * std::sin(two_pi * u3);
    q.w = std::sqrt(u1) * std::cos(two_pi * u3);
    quat qi = qinverse(q);  // AudioOBBCollider.cs:59
    if (qi.w < 0.0f) { qi.x = -qi.x; qi.y = -qi.y; qi.z = -qi.z; }  // halfQuaternion.cs:50-55
    obb[i].rot_x = f32tof16(qi.x); obb[i].rot_y = f32tof16(qi.y); obb[i].rot_z = f32tof16(qi.z);
    obb[i].material = kMaterials[rng.next() >> 62];
    obb[i].audio_target_id = -1;
  }
  // fan origins, rejection-sampled outside every collider
  for (int s = 0; s < cfg->fan_count; ++s) {
    float p[3];
    for (int attempt = 0; attempt < 10000; ++attempt) {
      for (int k = 0; k < 3; ++k) p[k] = rng.uniform(-L / 2, L / 2);
      bool in = false;
      for (int i = 0; i < ns && !in; ++i) in = inside_sphere(sph[i], p);
      for (int i = 0; i < na && !in; ++i) in = inside_aabb(aabb[i], p);
      for (int i = 0; i < no && !in; ++i) in = inside_obb(obb[i], p);
      if (!in) break;
    }
    memcpy(origins + 3 * s, p, 12);
  }
  art_fibonacci_directions(cfg->ray_count, dirs);
  return ART_OK;
}

}  // extern "C"
