// rt_planar_filter.h -- conservative f32 pre-test of Quad::hit / Triangle::hit
// (shapes/quad.rs:71-102, shapes/triangle.rs:69-98), host and device.
//
// The exact f64 test the kernel runs (planar_t) computes
//     denom = n.d,  t = (D - n.o) / denom,  hv = o + t d - Q,
//     alpha = w.(hv x v),  beta = w.(u x hv)
// and accepts t in [tmin, c] with alpha, beta in [0, 1] (and alpha + beta <= 1
// for a triangle).  With num = D - n.o and the triple-product identities
// w.(h x v) = h.(v x w), w.(u x h) = h.(w x u), alpha * denom and
// beta * denom are division-free:
//     Xa = denom * (o - Q).a + num * d.a,    a = v x w
//     Xb = denom * (o - Q).b + num * d.b,    b = w x u
// so, with s = sign(denom), the exact test's conditions read
//     t >= 0:          s num >= 0            t <= c:  s num <= c |denom|
//     alpha in [0,1]:  0 <= s Xa <= |denom|  (beta, alpha + beta likewise).
// This filter evaluates them in f32 from f32 copies of the ray and of the
// primitive (PlanarF, 64 B instead of the 128-B f64 record) and rejects a
// primitive only when a condition fails by more than a forward error bound:
// every quantity is a short sum of products of the inputs, so with u = 2^-24
// and the magnitudes Ro = |o|_1, Rd = |d|_1, Sq = |Q|_1, |D|, Sa = |a|_1,
// Sb = |b|_1 (|n|_1 <= sqrt 3):
//     |denom~ - denom| <= 5u   * 2 Rd
//     |num~   - num|   <= 7u   * (|D| + 2 Ro)
//     |Xa~    - Xa|    <= 13u  * Sa Rd (4 Ro + 2 Sq + |D|)     (Xb with Sb)
// counting the f64 -> f32 roundings of every input (1u each), the
// subtraction o - Q and the dot products (gamma_3).  The kernel uses
// C u = 2^-19 (32u) times the cruder magnitudes below, which also covers the
// f32 rounding of the bounds themselves and the f64 test's own rounding
// (2^-53-relative: alpha from a rounded t and p).  A primitive with
// |denom~| <= its error bound (grazing, sign uncertain) or any non-finite
// value is never rejected.  tests/cpp/planar_prop.cpp checks the filter
// against the exact f64 test on millions of random and adversarial rays and
// primitives (edges, vertices, grazing rays, near-parallel planes, tiny and
// huge scales): no exact hit is ever rejected.
#pragma once
#include <cmath>
#include <cstdint>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define RT_PF_HD __host__ __device__ __forceinline__
#else
#define RT_PF_HD inline
#endif

namespace rtk {

struct alignas(16) PlanarF {
    float n[3], D;   // unit normal and parm_d (quad.rs:34-36), f32
    float q[3], g;   // anchor Q; g = 8 |Q|_1 + 2 |D| rounded up
    float a[3], sa;  // a = v x w (the f64 cross, rounded), sa = |a|_1 rounded up
    float b[3], sb;  // b = w x u, sb = |b|_1 rounded up
};
static_assert(sizeof(PlanarF) == 64, "PlanarF must be 64 B (4 dwordx4)");

// The ray's f32 copy: o, d rounded to nearest; ro8 >= 8 |o|_1, rd >= |d|_1.
struct PRayF {
    float o[3], d[3];
    float ro8, rd;
};

RT_PF_HD PRayF make_prayf(const double o[3], const double d[3]) {
    PRayF R;
    float so = 0.0f, sd = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        R.o[k] = (float)o[k];
        R.d[k] = (float)d[k];
        so += fabsf(R.o[k]);
        sd += fabsf(R.d[k]);
    }
    // the f32 sums are within 3u of the sums of the rounded values, which are
    // within 1u of |o|_1 / |d|_1: scale up by 2^-20 more than that
    R.ro8 = 8.0f * so * 1.0000010f;
    R.rd = sd * 1.0000010f;
    return R;
}

// true: the exact test over t in [tmin >= 0, c <= c_f] certainly misses.
RT_PF_HD bool planar_reject(const PlanarF& P, const PRayF& R, float c_f, bool tri) {
    constexpr float CU = 1.9073486328125e-06f;  // 2^-19
    const float den = P.n[0] * R.d[0] + P.n[1] * R.d[1] + P.n[2] * R.d[2];
    const float num = P.D - (P.n[0] * R.o[0] + P.n[1] * R.o[1] + P.n[2] * R.o[2]);
    const float h0 = R.o[0] - P.q[0], h1 = R.o[1] - P.q[1], h2 = R.o[2] - P.q[2];
    const float A0 = h0 * P.a[0] + h1 * P.a[1] + h2 * P.a[2];
    const float A1 = R.d[0] * P.a[0] + R.d[1] * P.a[1] + R.d[2] * P.a[2];
    const float B0 = h0 * P.b[0] + h1 * P.b[1] + h2 * P.b[2];
    const float B1 = R.d[0] * P.b[0] + R.d[1] * P.b[1] + R.d[2] * P.b[2];
    const float Xa = den * A0 + num * A1;
    const float Xb = den * B0 + num * B1;
    const float mag = R.ro8 + P.g;      // >= 8 Ro + 8 Sq + 2 |D|
    const float K = CU * R.rd * mag;
    const float Ea = K * P.sa + 1e-35f, Eb = K * P.sb + 1e-35f;
    const float Eden = CU * 2.0f * R.rd + 1e-35f;
    const float Enum = CU * mag + 1e-35f;
    const float aden = fabsf(den);
    const float sgn = den < 0.0f ? -1.0f : 1.0f;
    const float ns = sgn * num, xa = sgn * Xa, xb = sgn * Xb;
    const float hi = aden + Eden;
    // every rejecting comparison is false on a NaN: non-finite input keeps the primitive
    const bool sure = aden > Eden;
    const bool behind = ns < -Enum;                      // t < 0 <= tmin
    const bool beyond = ns - Enum > c_f * hi;            // t > c_f >= c
    const bool a_out = xa < -Ea || xa - Ea > hi;         // alpha outside [0, 1]
    const bool b_out = xb < -Eb || xb - Eb > hi;         // beta outside [0, 1]
    const bool ab_out = tri && (xa + xb) - (Ea + Eb) > hi;  // alpha + beta > 1
    return sure && (behind || beyond || a_out || b_out || ab_out);
}

}  // namespace rtk
