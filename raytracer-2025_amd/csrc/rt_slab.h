// rt_slab.h -- the conservative f32 box test every kernel tier walks with.
//
// Host and device: the kernel (rt_kernel.hip) runs it, and the CPU property
// test (tests/test_slab_cpu.py, tests/cpp/slab_prop.cpp) checks it against the
// slab test of aabb.rs:62-78 evaluated in extended precision.
//
// aabb.rs:62-78: per axis t0 = (lo - o) / d, t1 = (hi - o) / d, the interval
// [min, max] of the two intersected with the ray's [t_min, t_max]; a hit when
// the result is not empty (inclusive).  Here in f32, made conservative --
// whenever the exact test on the exact box admits part of [t_min, c], this one
// does too:
//  - boxes are stored rounded outward (rth flatten / bvh4_convert);
//  - the origin's f32 rounding (and the rounding of o * idf) is absorbed by
//    widening the slab by pad = 2^-22 |o| per axis in space (RayF::nlo/nhi);
//  - the fma and 1/d roundings (relative, < 3u) by widening the t-interval
//    by 2^-22 |t| (REL);
//  - 1/d is clamped to |.| <= 2^60 so a zero direction component gives huge
//    finite t (the reference's +-inf) instead of inf - inf = NaN.
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rtk {

#ifndef RT_SLAB_FOLD
#define RT_SLAB_FOLD 1
#endif
// 1/d of the f32 ray: 2 = the hardware reciprocal (below; C2 -1.3 % kernel
// time against 1, C4 +-0, A/B at 128 spp, RMSE 0), 1 = the correctly rounded
// f32 quotient of d rounded to f32, 0 = the f64 quotient rounded once
#ifndef RT_RCP_F32
#define RT_RCP_F32 2
#endif

// RT_RCP_F32 == 2: 1/x as the hardware reciprocal (v_rcp_f32, within 1 ulp
// of 1/x: the correctly rounded quotient or its neighbour) instead of the
// ~10-instruction IEEE division.  Host builds (the CPU property tests) cannot
// run v_rcp_f32, so they take the correctly rounded quotient moved one ulp in
// the direction RT_RCP_EMU (+1 up, -1 down, 0 none): the tests run both, which
// covers whatever the hardware returns.  (Results below 2^-126 may flush to
// zero on the device: |d| >= 2^126 does not occur for a ray direction.)
#ifndef RT_RCP_EMU
#define RT_RCP_EMU 0
#endif
RT_HD float rcp_f32(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    const float q = 1.0f / x;
    return RT_RCP_EMU > 0 ? std::nextafter(q, __builtin_huge_valf())
                          : RT_RCP_EMU < 0 ? std::nextafter(q, -__builtin_huge_valf()) : q;
#endif
}

#if RT_SLAB_FOLD
// The t-interval widening folded into the ray: the plane distances of the
// near planes (lo when 1/d > 0) are scaled by 1 - 2^-21, those of the far
// planes by 1 + 2^-21, so the box's entry is moved earlier and its exit later
// by that relative amount whenever they are positive -- the only case where
// they decide a hit (a negative entry is clamped to t_min, a negative exit
// misses either way).  The scalings' own roundings are covered by the doubled
// widths: pad = 2^-21 |o| in space, 2^-21 relative in t.
struct RayF {
    float idl[3], idh[3];  // 1/d scaled for the lo and hi planes
    float nlo[3];          // -(o + pad) * idl  (lo planes moved outward)
    float nhi[3];          // -(o - pad) * idh  (hi planes moved outward)
};

RT_HD RayF make_rayf(const double o[3], const double d[3]) {
    RayF R;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#if RT_RCP_F32 == 2
        // d rounded to f32, then the hardware reciprocal: < 2.01u relative,
        // common to both plane distances of the axis (a relative error of t,
        // inside the 2^-21 widening with the other roundings; the CPU test
        // holds it there with the quotient moved an ulp either way)
        float f = rcp_f32((float)d[k]);
#elif RT_RCP_F32
        // d rounded to f32, then the correctly rounded f32 quotient: < 1.01u
        // relative (the f64 quotient rounded once: 0.5u).  The error is
        // common to both plane distances of the axis, a relative error of t,
        // inside the 2^-21 widening with the other roundings.
        float f = 1.0f / (float)d[k];
#else
        float f = (float)(1.0 / d[k]);
#endif
        if (!(fabsf(f) <= 1.152921504606847e18f)) f = copysignf(1.152921504606847e18f, f);
        const float of = (float)o[k];
        const float pad = fabsf(of) * 4.76837158203125e-07f + 1e-30f;  // 2^-21 |o|
        constexpr float SHRINK = 1.0f - 4.76837158203125e-07f, GROW = 1.0f + 4.76837158203125e-07f;
        const float sl = f > 0.0f ? SHRINK : GROW, sh = f > 0.0f ? GROW : SHRINK;
        R.idl[k] = f * sl;
        R.idh[k] = f * sh;
        R.nlo[k] = -((of + pad) * f) * sl;
        R.nhi[k] = -((of - pad) * f) * sh;
    }
    return R;
}
#else
struct RayF {
    float idf[3];  // 1/d
    float nlo[3];  // -(o + pad) * idf  (lo planes moved outward)
    float nhi[3];  // -(o - pad) * idf  (hi planes moved outward)
};

RT_HD RayF make_rayf(const double o[3], const double d[3]) {
    RayF R;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double id = 1.0 / d[k];
        float f = (float)id;
        if (!(fabsf(f) <= 1.152921504606847e18f)) f = copysignf(1.152921504606847e18f, (float)id);
        const float of = (float)o[k];
        const float pad = fabsf(of) * 2.384185791015625e-07f + 1e-30f;
        R.idf[k] = f;
        R.nlo[k] = -((of + pad) * f);
        R.nhi[k] = -((of - pad) * f);
    }
    return R;
}
#endif

// f32 not above x (round to nearest, then one ulp down when that rounded up)
RT_HD float f32_down(double x) {
    float f = (float)x;
    if ((double)f > x) {
        union {
            float f;
            uint32_t u;
        } b{f};
        b.u = (f > 0.0f) ? b.u - 1u : (f == 0.0f ? 0x80000001u : b.u + 1u);
        f = b.f;
    }
    return f;
}

// Entry distance (clamped to t_min) and hit of box [lo, hi] for t in [tmin_f, c_f].
RT_HD bool slab_f(const float* lo, const float* hi, const RayF& R, float tmin_f, float c_f, float& entry) {
#if RT_SLAB_FOLD
    const float tlx = fmaf(lo[0], R.idl[0], R.nlo[0]), thx = fmaf(hi[0], R.idh[0], R.nhi[0]);
    const float tly = fmaf(lo[1], R.idl[1], R.nlo[1]), thy = fmaf(hi[1], R.idh[1], R.nhi[1]);
    const float tlz = fmaf(lo[2], R.idl[2], R.nlo[2]), thz = fmaf(hi[2], R.idh[2], R.nhi[2]);
    entry = fmaxf(fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fminf(tlz, thz)), tmin_f);
    return entry <= fminf(fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fmaxf(tlz, thz)), c_f);
#else
    const float tlx = fmaf(lo[0], R.idf[0], R.nlo[0]), thx = fmaf(hi[0], R.idf[0], R.nhi[0]);
    const float tly = fmaf(lo[1], R.idf[1], R.nlo[1]), thy = fmaf(hi[1], R.idf[1], R.nhi[1]);
    const float tlz = fmaf(lo[2], R.idf[2], R.nlo[2]), thz = fmaf(hi[2], R.idf[2], R.nhi[2]);
    const float nr = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fminf(tlz, thz));
    const float fr = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fmaxf(tlz, thz));
    constexpr float REL = 2.384185791015625e-07f;  // 2^-22
    entry = fmaxf(fmaf(-fabsf(nr), REL, nr), tmin_f);
    return entry <= fminf(fmaf(fabsf(fr), REL, fr), c_f);
#endif
}

}  // namespace rtk
