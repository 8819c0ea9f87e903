// Host check of sphere_test_1div against sphere_test (art_device_fns.hpp): the same verdict and
// distance bits on random, scaled and adversarial inputs (run by tests/test_sphere_1div.py).
//   g++ -O2 -std=c++17 -ffp-contract=off -I audio-raytracer_amd/csrc tools/check_sphere_1div.cpp
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "art_device_fns.hpp"

using namespace art;

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 4000000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  const float specials[] = {0.0f, -0.0f, 1e-45f, -1e-45f, 2.8e-45f, 1e-38f, 1.0f, 2.0f, 0.5f, 1e30f, -1e30f,
                            INFINITY, -INFINITY, NAN, 3.4e38f, 1e-20f};
  long bad = 0, hits = 0;
  for (long i = 0; i < n; ++i) {
    Seg s;
    SphereRec c;
    const int mode = (int)(i % 8);
    float sc = std::pow(10.0f, (float)((int)(rng() % 13) - 6));
    vec3 o = mk3(u(rng) * sc, u(rng) * sc, u(rng) * sc);
    vec3 d = mk3(u(rng), u(rng), u(rng));
    if (mode == 1) d = d * std::pow(10.0f, (float)((int)(rng() % 41) - 20));    // unnormalized directions
    if (mode == 2) d = mk3(specials[rng() % 16], u(rng), specials[rng() % 16]);  // special components
    if (mode != 1 && mode != 2) { const float l = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z); if (l > 0) d = d * (1.0f / l); }
    s = make_seg(o, d);
    c.cx = o.x + u(rng) * sc; c.cy = o.y + u(rng) * sc; c.cz = o.z + u(rng) * sc;
    c.r2 = std::fabs(u(rng)) * sc * sc;
    if (mode == 3) {  // origin on the sphere: tiny numerators
      c.cx = o.x; c.cy = o.y; c.cz = o.z + 1.0f; c.r2 = 1.0f;
      s = make_seg(mk3(o.x, o.y, o.z + from_bits(bits(1.0f) ^ (uint32_t)(rng() & 7))), mk3(0.0f, 0.0f, 1.0f));
    }
    if (mode == 4) {  // denormal-scale geometry
      const float t = 1e-43f;
      s = make_seg(mk3(u(rng) * t, u(rng) * t, u(rng) * t), d);
      c.cx = u(rng) * t; c.cy = u(rng) * t; c.cz = u(rng) * t; c.r2 = 0.0f;
    }
    if (mode == 5) s.a2 = from_bits((uint32_t)(rng() & 0xffffffffu));  // arbitrary a2 bit patterns
    float d0 = 0.0f, d1 = 0.0f;
    const bool h0 = sphere_test(s, c, d0);
    const bool h1 = sphere_test_1div(s, c, d1);
    if (h0) ++hits;
    if (h0 != h1 || (h0 && bits(d0) != bits(d1))) {
      if (++bad <= 10)
        printf("mismatch %ld: h %d/%d dist %a/%a a2 %a\n", i, (int)h0, (int)h1, d0, d1, s.a2);
    }
  }
  // the quotient selection alone, on raw bit patterns (tiny and denormal numerators around a2)
  long bad2 = 0;
  for (long i = 0; i < n; ++i) {
    uint32_t b0 = (uint32_t)rng(), b1 = (uint32_t)rng(), ba = (uint32_t)rng();
    if (i % 4 == 1) { b0 = (b0 & 0x8000000fu); }                     // +-tiny denormal numerators
    if (i % 4 == 2) { ba = (ba & 0x807fffffu) | ((uint32_t)(120 + rng() % 30) << 23); b0 = 0x80000000u | (b0 & 0x3ffu); }
    if (i % 4 == 3) { ba = 0x40000000u; b0 = 0x80000001u; }          // a2 = 2, n0 = -2^-149: a tie to -0
    const float n0 = from_bits(b0), n1 = from_bits(b1), a2 = from_bits(ba);
    const float t0 = n0 / a2, t1 = n1 / a2;
    const bool h0 = t0 >= 0.0f || t1 >= 0.0f;
    const float d0 = t0 >= 0.0f ? t0 : t1;
    float d1;
    const bool h1 = sphere_pick_1div(n0, n1, a2, d1);
    if (h0 != h1 || bits(d0) != bits(d1)) {
      if (++bad2 <= 10) printf("pick mismatch: n0 %a n1 %a a2 %a: %d/%d %a/%a\n", n0, n1, a2, (int)h0, (int)h1, d0, d1);
    }
  }
  bad += bad2;
  printf("cases %ld hits %ld mismatches %ld (quotient selection %ld)\n", n, hits, bad, bad2);
  return bad ? 1 : 0;
}
