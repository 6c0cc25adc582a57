// rt_math.h -- f64 vector math and the render RNG for the gfx950 kernel.
//
// Arithmetic follows the reference's expression order (src/utils/vec3.rs):
// Div<f64> multiplies by the reciprocal (vec3.rs:226-232), dot/cross/length
// as written there.  The RNG is the contract of oracle/rng_contract.hpp,
// restated here for the device (Philox4x32-10, Random123 constants).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_crmath.h"

namespace rtk {

constexpr double PI = 3.14159265358979323846264338327950288;

struct D3 {
    double x, y, z;
};
__device__ __forceinline__ D3 d3(double x, double y, double z) { return D3{x, y, z}; }
__device__ __forceinline__ D3 operator+(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ D3 operator-(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ D3 operator*(D3 a, D3 b) { return d3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ D3 operator*(double s, D3 v) { return d3(s * v.x, s * v.y, s * v.z); }
__device__ __forceinline__ D3 operator-(D3 a) { return d3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ D3 operator/(D3 a, D3 b) { return d3(a.x / b.x, a.y / b.y, a.z / b.z); }
__device__ __forceinline__ D3 divs(D3 v, double s) { return (1.0 / s) * v; }
__device__ __forceinline__ double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ D3 cross(D3 a, D3 b) {
    return d3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// f64 square root, the same double as sqrt(x) (IEEE, correctly rounded).
// LLVM lowers sqrt to v_rsq_f64 and two Newton-Raphson corrections on x scaled
// by 2^256 when x < 2^-767, and then selects x itself for +-0 and +inf.  For x in
// [2^-767, inf) the scale is 2^0 and the select keeps the Newton result, so that
// sequence without them is the same instructions on the same values.
// RT_FAST_SQRT takes it when every active lane's x is in that range (a
// wave-uniform branch), else sqrt(x) for the wave: C2 -1.1 % kernel time, C4
// -0.15 %, C5 +-0 (A/B, RMSE 0: profiles/r06/ab_fast_sqrt_c*.json; bit-equal to
// IEEE sqrt on every binade and on mixed waves, tests/test_sqrt_gpu.py).
#ifndef RT_FAST_SQRT
#define RT_FAST_SQRT 1
#endif
__device__ __forceinline__ double k_sqrt(double x) {
#if RT_FAST_SQRT
    if (__builtin_expect(__ballot(!(x >= 0x1p-767 && x < __builtin_huge_val())) == 0ull, 1)) {
        const double y = __builtin_amdgcn_rsq(x);
        double g = x * y, h = y * 0.5;
        const double r = __builtin_fma(-h, g, 0.5);
        g = __builtin_fma(g, r, g);
        h = __builtin_fma(h, r, h);
        double d = __builtin_fma(-g, g, x);
        g = __builtin_fma(d, h, g);
        d = __builtin_fma(-g, g, x);
        return __builtin_fma(d, h, g);
    }
#endif
    return sqrt(x);
}
__device__ __forceinline__ double len2(D3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ double len(D3 a) { return k_sqrt(len2(a)); }
__device__ __forceinline__ bool finite3(D3 v) { return isfinite(v.x) && isfinite(v.y) && isfinite(v.z); }
// UnitVec3::from_vec3 (vec3.rs:299-306): v / |v|, ok = all finite
__device__ __forceinline__ D3 unit(D3 v, bool& ok) {
    D3 u = divs(v, len(v));
    ok = finite3(u);
    return u;
}
// vec3.rs:71-73
__device__ __forceinline__ D3 reflect(D3 v, D3 n) { return v - (2.0 * dot(v, n)) * n; }
__device__ __forceinline__ D3 mat3(const double* m, D3 v) {
    return d3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
              m[6] * v.x + m[7] * v.y + m[8] * v.z);
}

// ---------------------------------------------------------------- libm
// The transcendentals of the path: correctly rounded (rt_crmath.h), so that
// they agree with glibc -- what Rust's f64::sin / cos / ln / acos / atan2 call
// -- wherever glibc is correctly rounded (~99.9 % of arguments); RT_CRMATH=0
// selects ROCm's ocml (A/B only: it differs from glibc by an ulp far more
// often, tests/test_crmath_gpu.py).
#ifndef RT_CRMATH
#define RT_CRMATH 1
#endif
__device__ __forceinline__ double k_sin(double x) { return RT_CRMATH ? rtcr::sin(x) : ::sin(x); }
__device__ __forceinline__ double k_log(double x) { return RT_CRMATH ? rtcr::log(x) : ::log(x); }
__device__ __forceinline__ double k_acos(double x) { return RT_CRMATH ? rtcr::acos(x) : ::acos(x); }
__device__ __forceinline__ double k_atan2(double y, double x) { return RT_CRMATH ? rtcr::atan2(y, x) : ::atan2(y, x); }
__device__ __forceinline__ void k_sincos(double x, double* s, double* c) {
    if (RT_CRMATH)
        rtcr::sincos(x, s, c);
    else
        ::sincos(x, s, c);
}
// sin / cos of 2.0 * PI * xi for a unit draw xi (every sincos of the path):
// the same doubles as k_sincos(2.0 * PI * xi), the argument's range known
// (rtcr::sincos_2pi); RT_SC2PI=0 evaluates k_sincos (A/B only)
#ifndef RT_SC2PI
#define RT_SC2PI 1
#endif
__device__ __forceinline__ void k_sincos_2pi(double xi, double* s, double* c) {
    if (RT_CRMATH && RT_SC2PI)
        rtcr::sincos_2pi(xi, s, c);
    else
        k_sincos(2.0 * PI * xi, s, c);
}

// ---------------------------------------------------------------- RNG
__device__ __forceinline__ void philox4x32_10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                              uint32_t k1) {
#pragma unroll
    for (int round = 0; round < 10; ++round) {
        if (round > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // one v_mad_u64_u32 per 32x32->64 product (not a mul_lo + mul_hi pair)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
}
__device__ __forceinline__ double u64_unit(uint32_t lo, uint32_t hi) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    return (double)(v >> 11) * (1.0 / 9007199254740992.0);
}

// Keyed per-path stream (oracle/rng_contract.hpp): draw `slot` of path vertex
// `vertex` of sample (pixel, sample).  Draws of one vertex come in pairs from
// one Philox block; the odd half is cached.
struct Rng {
    uint32_t k0, k1, pixel, sample, vertex, slot;
    uint32_t c_lo, c_hi;
    __device__ __forceinline__ void begin(uint32_t v) {
        vertex = v;
        slot = 0;
    }
    __device__ __forceinline__ double next(uint32_t& overflow) {
        if (slot >= 16u) {
            overflow = 1;
            slot = 0;
        }
        double r;
        if ((slot & 1u) == 0u) {
            uint32_t c0 = vertex * 8u + (slot >> 1), c1 = pixel, c2 = sample, c3 = 0u;
            philox4x32_10(c0, c1, c2, c3, k0, k1);
            c_lo = c2;
            c_hi = c3;
            r = u64_unit(c0, c1);
        } else {
            r = u64_unit(c_lo, c_hi);
        }
        ++slot;
        return r;
    }
    // draws 2p and 2p + 1 of vertex v (one Philox block), as next() would
    // return them at slots 2p and 2p + 1; the stream position is not moved
    __device__ __forceinline__ void pair(uint32_t v, uint32_t p, double& a, double& b) const {
        uint32_t c0 = v * 8u + p, c1 = pixel, c2 = sample, c3 = 0u;
        philox4x32_10(c0, c1, c2, c3, k0, k1);
        a = u64_unit(c0, c1);
        b = u64_unit(c2, c3);
    }
    __device__ __forceinline__ double medium(uint32_t id) const {
        uint32_t c0 = vertex, c1 = pixel, c2 = sample, c3 = 1u + id;
        philox4x32_10(c0, c1, c2, c3, k0, k1);
        return u64_unit(c0, c1);
    }
};

}  // namespace rtk
