// fast_margin.h — the per-ray margins of the certified walk's box test
// (DESIGN.md §4b), shared by the gfx950 kernel and host analysis tools.
//
// For a child box holding triangles whose hit_triangle arithmetic
// (compute_dynamic_ray.comp:105-129) may accept a hit at computed t_c, the
// forward error bound of that float arithmetic gives:
//   * the real ray point at the exact parameter t_e lies within Delta of the
//     box (the barycentric error times the edge length, plus the roundings of
//     s = o - v0 and of e1 = v1 - v0, e2 = v2 - v0);
//   * |t_c - t_e| <= E_t and t_e <= Te.
// Inflating the box by r = Delta + rho (rho covers the slab test's own
// rounding) makes the computed slab test pass with t_enter <= t_c + E_t, so a
// child whose inflated t_enter exceeds closest_t + m (m >= E_t) holds no
// triangle that could still be reported.  All the bounds scale with 1/|det|;
// |det| is bounded below by the child's normal cone (|det| = |d.(e1 x e2)|),
// or by the shader's own |det| >= 1e-5 cut-off when the cone allows grazing.
#pragma once
#include <cmath>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rtamd {
namespace fast {

// kdet = sqrt(2) gamma_5 (1 + 4u): |delta det| <= kdet emax^2 and
// |delta numerator| <= kdet S2 emax (u, v) or kdet S2 emax^2 (t).
constexpr float kDetK = 4.2150e-7f;
constexpr float kG2 = 1.19210e-7f * 1.0001f;   // gamma_2 (u = 2^-24)
constexpr float kG3 = 1.78814e-7f * 1.0001f;   // gamma_3
constexpr float kU = 5.9604645e-8f;
constexpr float kDetFloor = 9.99e-6f;          // |det_c| >= 1e-5f for a valid hit (:110)

// Returns false when no bound holds (never cull).  lo/hi: child box; ax, ca,
// sa, a2min, emax: fast_bvh.h ChildBox; ulscene = 1.01 u max|coordinate|.
RT_HD bool child_margins(float lox, float loy, float loz, float hix, float hiy, float hiz,
                         float axx, float axy, float axz, float ca, float sa, float a2min, float emax,
                         float ox, float oy, float oz, float dx, float dy, float dz, float ulscene,
                         float& r, float& m) {
    const float sx = fmaxf(fabsf(lox - ox), fabsf(hix - ox));
    const float sy = fmaxf(fabsf(loy - oy), fabsf(hiy - oy));
    const float sz = fmaxf(fabsf(loz - oz), fabsf(hiz - oz));
    const float sinf_ = fmaxf(fmaxf(sx, sy), sz) * 1.000001f;
    const float s2 = sqrtf((sx * sx + sy * sy) + sz * sz) * 1.000001f;
    // lower bound of |cos| between the d line and every normal line of the cone
    const float cd = fmaxf(fabsf((dx * axx + dy * axy) + dz * axz) - 1e-6f, 0.0f);
    const float sd = sqrtf(fmaxf(1.0f - cd * cd, 0.0f) + 4.0f * kU) + 1e-6f;
    const float cb = cd * ca - sd * sa - 2e-6f;
    const float b = kDetK * emax * emax;
    const float dlb = fmaxf(kDetFloor, a2min * cb * (1.0f - 5.0f * kU) - b);
    if (!(b <= 0.5f * dlb)) return false;
    const float inv = (1.0f / (dlb - b)) * 1.000001f;
    const float eu = (kDetK * s2 * emax + b + kG2 * dlb) * inv;                // barycentric error
    const float delta = 1.01f * (2.0f * emax * eu + 2.0f * kU * emax + kU * sinf_);
    const float te = (s2 + 1.7321f * delta) * (1.0f + 4.0f * kU);             // bound on t_e
    const float et = ((b * (s2 + te)) / dlb + kG2 * te) * 1.0001f;              // |t_c - t_e|
    const float rho = 1.05f * (et + 2.0f * kG3 * (te + et + 1.0f));
    r = 1.001f * (delta + rho) + ulscene;
    m = 1.02f * et;
    return true;
}

}  // namespace fast
}  // namespace rtamd
