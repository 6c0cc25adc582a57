// TEST HARNESS: the 8-bit quantized child boxes of the mesh / full tiers'
// 4-wide nodes (raytracer-2025_amd/csrc/rt_qnode.h, DNode4Q): for random and
// adversarial nodes -- children at every scale from 1e-6 to 1e6, far from
// the origin, negative, flat (zero extent), identical, one child spanning the
// node, empty slots -- the decoded box (fmaf(q, scale, origin), the kernel's
// arithmetic) must contain each child's f32 box on every axis.  Also:
// non-finite bounds are refused.
// Prints "nodes children violations mean_slack"; exits 1 on any violation.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../raytracer-2025_amd/csrc/rt_qnode.h"

int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 200000;
    std::mt19937_64 g(argc > 2 ? atoll(argv[2]) : 1);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long children = 0, bad = 0;
    double slack = 0.0;
    for (long n = 0; n < N; ++n) {
        float lo[3][4], hi[3][4];
        uint32_t ref[4];
        const double scale = std::pow(10.0, -6.0 + 12.0 * U(g));
        const double center = (U(g) < 0.3 ? 0.0 : (U(g) - 0.5) * std::pow(10.0, 6.0 * U(g)));
        const int mode = (int)(U(g) * 6);
        for (int i = 0; i < 4; ++i) {
            ref[i] = (U(g) < 0.15 && i > 0) ? 0u : (uint32_t)(i + 1);
            for (int a = 0; a < 3; ++a) {
                double c = center + (U(g) - 0.5) * scale, h = U(g) * scale * 0.5;
                if (mode == 1) h = 0.0;                                 // flat children
                if (mode == 2) c = center, h = scale;                   // identical
                if (mode == 3 && i == 0) c = center, h = scale * 4.0;   // one spans the node
                if (mode == 4) h *= 1e-7;                               // tiny next to the node
                float l = (float)(c - h), u = (float)(c + h);
                if ((double)l > c - h) l = std::nextafter(l, -INFINITY);
                if ((double)u < c + h) u = std::nextafter(u, INFINITY);
                if (mode == 5 && a == 1) l = u = (float)c;              // exactly flat axis
                lo[a][i] = l;
                hi[a][i] = u;
            }
        }
        rth::QNode q;
        if (!rth::qnode_encode(lo, hi, ref, q)) {
            printf("encode refused a finite node\n");
            return 1;
        }
        for (int i = 0; i < 4; ++i) {
            for (int a = 0; a < 3; ++a) {
                const float s = rtk::qnode_scale(q.exps, a);
                const float dl = rtk::qnode_decode(q.origin[a], s, (q.qlo[a] >> (8 * i)) & 0xffu);
                const float dh = rtk::qnode_decode(q.origin[a], s, (q.qhi[a] >> (8 * i)) & 0xffu);
                if (ref[i] == 0u) continue;  // masked by its REF_NONE in the kernel
                ++children;
                if (!(dl <= lo[a][i] && dh >= hi[a][i])) {
                    if (bad < 5) printf("violation: [%a, %a] decoded [%a, %a]\n", lo[a][i], hi[a][i], dl, dh);
                    ++bad;
                }
                const double ext = (double)hi[a][i] - lo[a][i];
                slack += ((double)dh - dl - ext) / (std::ldexp(255.0, (int)((q.exps >> (8 * a)) & 0xffu) - 127));
            }
        }
    }
    float lo[3][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}}, hi[3][4] = {{1, 1, 1, 1}, {1, 1, 1, 1}, {1, 1, 1, 1}};
    const uint32_t ref[4] = {1, 2, 3, 4};
    hi[1][2] = INFINITY;
    rth::QNode q;
    if (rth::qnode_encode(lo, hi, ref, q)) {
        printf("encode accepted an infinite bound\n");
        return 1;
    }
    printf("%ld %ld %ld %.4f\n", N, children, bad, slack / (double)(children ? children : 1));
    return bad ? 1 : 0;
}
