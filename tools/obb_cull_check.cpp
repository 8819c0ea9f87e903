// Host check of the OBB broad-phase bounds (art_frame_math.hpp prep_obb):
// for random OBB records (half-precision centres, sizes and half-quaternions, as the C# structs
// carry them) and rays aimed at their corners, edges and faces, every hit the exact OBB tests report
// (the raytrace cast's stored rotation, the permeation first hit's inverse rotation) must be found
// by the node test on the collider's bounds with a QUARTER of its margin: the box is entered, at an
// entry distance not past the reported distance. Prints the case count and the failures.
//   hipcc -x hip -O2 -std=c++17 -ffp-contract=off -Iinclude -Iaudio-raytracer_amd/csrc \
//       tools/obb_cull_check.cpp -o /tmp/obb_cull_check && /tmp/obb_cull_check [cases]
#include <cstdio>
#include <cstdlib>
#include <random>

#include "art_frame_math.hpp"

using namespace art;

static bool node_hit(const Seg& s, const CullRec& r, float om, float frac, float& en) {
  const float m = frac * (r.factor * om + r.fscale);
  float tn, tf;
  const bool h = slab<false>(s.o.x, s.o.y, s.o.z, s.inv.x, s.inv.y, s.inv.z, r.lox - m, r.loy - m, r.loz - m, r.hix + m,
                             r.hiy + m, r.hiz + m, tn, tf);
  en = fmaxf(tn, 0.0f);
  return h;
}

int main(int argc, char** argv) {
  const long long cases = argc > 1 ? atoll(argv[1]) : 2000000;
  const float frac = argc > 2 ? (float)atof(argv[2]) : 0.25f;  // share of the margin the node test keeps
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  long long hits = 0, bad = 0, tight = 0;
  for (long long k = 0; k < cases; ++k) {
    const float scale = k % 3 == 0 ? 4.0f : (k % 3 == 1 ? 60.0f : 3000.0f);  // coordinate magnitudes
    art_obb b{};
    b.center = {f32tof16(u(rng) * scale), f32tof16(u(rng) * scale), f32tof16(u(rng) * scale)};
    const float aniso = k % 5 == 0 ? 200.0f : 1.0f;  // flat or long boxes too
    b.size = {f32tof16(0.05f + 2.5f * fabsf(u(rng)) * aniso), f32tof16(0.05f + 2.5f * fabsf(u(rng))),
              f32tof16(0.05f + 2.5f * fabsf(u(rng)))};
    b.rot_x = f32tof16(u(rng)); b.rot_y = f32tof16(u(rng) * 0.7f); b.rot_z = f32tof16(u(rng) * 0.5f);
    if (k % 7 == 0) b.rot_x = b.rot_y = 0;  // near-axis-aligned rotations
    ObbRec r;
    ObbCold c;
    CullRec cr;
    prep_obb(b, 0, 0, &r, &c, &cr);
    // world-space target on the box surface: local point on a face / edge / corner, mapped back
    const float lx = (k & 1) ? c.hx : -c.hx;
    const float ly = u(rng) * c.hy * (k % 4 == 0 ? 1.0f : 1.0001f);
    const float lz = (k % 6 < 2) ? ((k & 2) ? c.hz : -c.hz) : u(rng) * c.hz;
    const quat qs = stored_q(r), qi = inverse_q(c);
    const bool perm = (k % 2) == 1;  // which rotation maps world -> local for this case
    // local -> world is the other rotation
    const vec3 lw = qmul(perm ? qs : qi, mk3(lx, ly, lz));
    const vec3 P = mk3(r.cx + lw.x, r.cy + lw.y, r.cz + lw.z);
    const float dist0 = 0.5f + 80.0f * fabsf(u(rng)) * (k % 11 == 0 ? 30.0f : 1.0f);
    vec3 dir = mk3(u(rng), u(rng), u(rng));
    const float dl = sqrtf(dot(dir, dir));
    if (!(dl > 1e-3f)) continue;
    dir = mk3(dir.x / dl, dir.y / dl, dir.z / dl);
    const vec3 o = mk3(P.x - dir.x * dist0, P.y - dir.y * dist0, P.z - dir.z * dist0);
    // aim at P (grazing the face / edge / corner)
    const vec3 d0 = mk3(P.x - o.x, P.y - o.y, P.z - o.z);
    const float n0 = sqrtf(dot(d0, d0));
    const vec3 d = mk3(d0.x / n0, d0.y / n0, d0.z / n0);
    const Seg s = make_seg(o, d);
    float dist;
    const bool hit = obb_test<false>(s, r, perm ? qi : qs, dist);
    if (!hit || !(dist >= 0.0f) || !(dist < FLT_MAX)) continue;
    ++hits;
    const float om = fabsf(o.x) + fabsf(o.y) + fabsf(o.z);
    float en;
    const bool h = node_hit(s, cr, om, frac, en);
    if (!h || en > dist) {
      if (++bad <= 8)
        printf("FAIL case %lld perm %d dist %.9g entry %.9g h %d box (%g %g %g)-(%g %g %g)\n", k, (int)perm, dist, en, (int)h,
               cr.lox, cr.loy, cr.loz, cr.hix, cr.hiy, cr.hiz);
    }
    // the bounds are tighter than round 3's cube of half-width 1.001 |h|_1
    const float rho = (fabsf(c.hx) + fabsf(c.hy) + fabsf(c.hz)) * 1.001f;
    if (cr.hix - r.cx < rho * 0.999f || cr.hiy - r.cy < rho * 0.999f || cr.hiz - r.cz < rho * 0.999f) ++tight;
  }
  printf("obb cull check: %lld cases, %lld reported hits, %lld failures, %lld tighter than the cube\n", cases, hits, bad, tight);
  return bad ? 1 : 0;
}
