// rt_qnode.h -- 8-bit quantized child boxes of a 4-wide BVH node (DNode4Q),
// host encoder and the decode the kernel runs; one source for both so that
// tests/test_qnode_cpu.py checks the exact arithmetic the device does.
//
// Decode: bound = fmaf(q, 2^(e - 127), origin) -- q * 2^k is exact (8-bit q,
// power-of-two scale), so the one rounding is the fused add; IEEE fmaf gives
// the same bits on host and device.  Encode: for each child and axis, the
// largest q whose decoded value is <= the child's lower bound and the
// smallest whose decoded value is >= its upper bound (rounding is monotone in
// q, so a short search from the estimate finds them); q = 0 decodes to origin
// (<= every lower bound) and q = 255 to at least the union's upper bound (the
// scale is a power of two >= extent / 255), so both always exist.  The
// decoded box therefore contains the child's f32 box (itself rounded outward
// from the f64 box), and the conservative slab test of rt_slab.h applied to
// it admits every hit the exact box would.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define RTQ_FN __host__ __device__ inline
#else
#define RTQ_FN inline
#endif

namespace rtk {

RTQ_FN float qnode_scale(uint32_t exps, int axis) {
    const uint32_t e = (exps >> (8 * axis)) & 0xffu;
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(e << 23);
#else
    const uint32_t b = e << 23;
    float f;
    memcpy(&f, &b, 4);
    return f;
#endif
}
RTQ_FN float qnode_decode(float origin, float scale, uint32_t q) {
    return fmaf((float)q, scale, origin);
}

}  // namespace rtk

#if !defined(__HIP_DEVICE_COMPILE__)
#include <cmath>
namespace rth {
// One node's quantized children, as DNode4Q stores them (rt_layout.h).
struct QNode {
    float origin[3];
    uint32_t exps, qlo[3], qhi[3];
};
// Quantizes one node's children (lo[a][i], hi[a][i] f32, ref[i]; empty slots
// 0 = REF_NONE).  False when a bound is not finite or the extent needs a
// scale beyond 2^100 (the caller keeps the f32 node format for the world).
inline bool qnode_encode(const float lo[3][4], const float hi[3][4], const uint32_t ref[4], QNode& out) {
    out = QNode{};
    bool any = false;
    for (int i = 0; i < 4; ++i) any |= ref[i] != 0u;
    for (int a = 0; a < 3; ++a) {
        float ulo = INFINITY, uhi = -INFINITY;
        for (int i = 0; i < 4; ++i) {
            if (ref[i] == 0u) continue;
            if (!std::isfinite(lo[a][i]) || !std::isfinite(hi[a][i])) return false;
            ulo = std::fmin(ulo, lo[a][i]);
            uhi = std::fmax(uhi, hi[a][i]);
        }
        if (!any) ulo = uhi = 0.0f;
        out.origin[a] = ulo;
        // the smallest power of two >= extent / 255 (extent rounded up in f64)
        const double ext = ((double)uhi - (double)ulo) * (1.0 + 0x1p-50);
        int e = -100;
        while (std::ldexp(255.0, e) < ext) ++e;
        if (e > 100) return false;
        const float s = std::ldexp(1.0f, e);
        uint32_t qlo = 0, qhi = 0;
        for (int i = 0; i < 4; ++i) {
            uint32_t ql = 255, qh = 0;  // empty slot: inverted
            if (ref[i] != 0u) {
                double t = std::floor(((double)lo[a][i] - ulo) / s);
                int q = t < 0 ? 0 : (t > 255 ? 255 : (int)t);
                while (q > 0 && rtk::qnode_decode(ulo, s, (uint32_t)q) > lo[a][i]) --q;
                while (q < 255 && rtk::qnode_decode(ulo, s, (uint32_t)q + 1) <= lo[a][i]) ++q;
                if (rtk::qnode_decode(ulo, s, (uint32_t)q) > lo[a][i]) return false;
                ql = (uint32_t)q;
                t = std::ceil(((double)hi[a][i] - ulo) / s);
                q = t < 0 ? 0 : (t > 255 ? 255 : (int)t);
                while (q < 255 && rtk::qnode_decode(ulo, s, (uint32_t)q) < hi[a][i]) ++q;
                while (q > 0 && rtk::qnode_decode(ulo, s, (uint32_t)q - 1) >= hi[a][i]) --q;
                if (rtk::qnode_decode(ulo, s, (uint32_t)q) < hi[a][i]) return false;
                qh = (uint32_t)q;
            }
            qlo |= ql << (8 * i);
            qhi |= qh << (8 * i);
        }
        out.exps |= (uint32_t)(e + 127) << (8 * a);
        out.qlo[a] = qlo;
        out.qhi[a] = qhi;
    }
    return true;
}
}  // namespace rth
#endif
