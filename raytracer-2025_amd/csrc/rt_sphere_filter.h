// rt_sphere_filter.h -- the basic tier's conservative f32 sphere test.
//
// Host and device: the kernel (rt_kernel.hip visit4) runs it, and the CPU
// property test (tests/test_filter_cpu.py, tests/filter_prop.cpp) checks it
// against the exact f64 Sphere::hit (sphere.rs:77-108) on random and
// adversarial rays.
//
// Reference algorithm (sphere.rs:77-96): oc = c - o, a = |d|^2, h = d.oc,
// cc = |oc|^2 - r^2, disc = h^2 - a cc; hit at the near root (h - sqrt(disc))/a
// if it lies in [t_min, t_max], else at the far root.  The filter evaluates
// the same quantities in f32 from inputs rounded to nearest.  With u = 2^-24
// and G = |c|_1 + r + |o|_1, which bounds every magnitude involved:
//   |h - h*| <= 6.2u |d| G,  |cc - cc*| <= 10.4u G^2,  |disc - disc*| <= 31u a G^2
// (standard forward error bounds of the dot products and the final fma); the
// filter uses 32u |d| G, 32u G^2 and 128u a G^2.  The f64 evaluation the
// reference (and the exact test) does is orders of magnitude closer to the
// real values, so:
//  - disc < -bound: the exact test sees disc < 0 (miss);
//  - origin certainly outside (cc > 0) and h certainly < 0: both roots < 0;
//  - origin outside, h > 0: the near root is >= cc / 2h (product of the roots
//    cc/a, sum 2h/a), so cc_lo > 2 h_hi t gives near root > t; with t = the
//    walk's bound c_f no hit closer than c_f is possible; with t = 1e-8 (x1.05)
//    the near root certainly passes t_min;
//  - disc certainly > 0 and the near root certainly >= t_min: the exact test
//    returns a t <= near root <= h/a (<= hh * ia, rounded up), a bound of the
//    closest hit the walk may cull with.  (A bound from the far root as well
//    -- rays inside a glass sphere -- culled more but cost C2 +7 % in VALU:
//    measured, not kept.)
#pragma once
#include <cmath>

#include "rt_slab.h"  // rcp_f32, RT_RCP_F32

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rtk {

// Per-ray f32 data of the filter.
struct SphF {
    float o[3], d[3];
    float a;    // |d|^2
    float gr;   // |o|_1 rounded up
    float ka;   // 2^-17 a: discriminant error bound per G^2
    float ehd;  // 2^-19 |d|: error bound of h per G
    float ia;   // 1/a rounded up (with margin)
};

RT_HD SphF make_sphf(const double o[3], const double d[3]) {
    SphF F;
    for (int k = 0; k < 3; ++k) {
        F.o[k] = (float)o[k];
        F.d[k] = (float)d[k];
    }
    F.a = fmaf(F.d[2], F.d[2], fmaf(F.d[1], F.d[1], F.d[0] * F.d[0]));
    F.gr = (fabsf(F.o[0]) + fabsf(F.o[1]) + fabsf(F.o[2])) * (1.0f + 0x1p-20f);
    F.ka = F.a * 0x1p-17f;
#if RT_RCP_F32 == 2
    // the hardware square root and reciprocal (1 ulp): ehd's 2^-19 is five
    // times the 6.2u bound it scales, and ia's margin of 2^-19 is 16 ulps
#if defined(__HIP_DEVICE_COMPILE__)
    F.ehd = __builtin_amdgcn_sqrtf(F.a) * 0x1p-19f;
#else
    F.ehd = std::sqrt(F.a) * 0x1p-19f;
#endif
    F.ia = rcp_f32(F.a) * (1.0f + 0x1p-19f);
#else
    F.ehd = sqrtf(F.a) * 0x1p-19f;
    F.ia = (1.0f / F.a) * (1.0f + 0x1p-19f);
#endif
    return F;
}

// One sphere {c, r} with g = |c|_1 + r rounded up (the node's record, as
// rth::bvh4_convert writes it), against the ray F and the walk's f32 bound c_f
// of the closest t.  Returns false when the exact test is certain not to give
// a hit closer than c_f (and for is_sph = false: a slot that holds no sphere);
// lowers c_f when it is certain to give one.
RT_HD bool sphere_filter(float cx, float cy, float cz, float r, float g, const SphF& F, float& c_f, bool is_sph) {
    const float ocx = cx - F.o[0], ocy = cy - F.o[1], ocz = cz - F.o[2];
    const float h = fmaf(F.d[2], ocz, fmaf(F.d[1], ocy, F.d[0] * ocx));
    const float q = fmaf(ocz, ocz, fmaf(ocy, ocy, ocx * ocx));
    const float cc = fmaf(-r, r, q);
    const float disc = fmaf(h, h, -(F.a * cc));
    const float G = g + F.gr, G2 = G * G;
    const float m = F.ka * G2;
    const float eh = F.ehd * G;
    const float hh = h + eh;                    // >= h*
    const float clo = fmaf(-0x1p-19f, G2, cc);  // <= cc*
    const bool outside = clo > 0.0f;            // origin certainly outside: roots of one sign
    const bool miss = disc < -m || (outside && (hh < 0.0f || clo > 2.0004f * hh * c_f));
    const bool sure = outside && disc > m && h > eh && clo > 2.1e-8f * hh;
    c_f = (is_sph && !miss && sure) ? fminf(c_f, hh * F.ia) : c_f;
    return is_sph && !miss;
}

}  // namespace rtk
