// TEST HARNESS: property test of the kernel's conservative f32 slab test
// (raytracer-2025_amd/csrc/rt_slab.h) against aabb.rs:62-78 evaluated in
// long double on the exact box: whenever the exact test admits part of
// [t_min, c] (by more than a relative 1e-12, so long double's own rounding
// cannot decide), the f32 test on the box rounded outward, with t_min rounded
// down and c rounded up, must admit it too.  Random and adversarial rays and
// boxes: origins on faces, edges and corners, grazing rays along a face,
// zero direction components, flat boxes, boxes far from the origin, tiny and
// huge boxes, c right at the box entry.
// Prints "cases exact_hits f32_hits violations"; exits 1 on any violation.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../raytracer-2025_amd/csrc/rt_slab.h"

typedef long double LD;

static float down(double x) { return rtk::f32_down(x); }
static float up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}

// aabb.rs:62-78 in long double: 1 when [tmin, c] meets the box by a margin,
// 0 when it misses by a margin, -1 when too close to call
static int exact(const double lo[3], const double hi[3], const double o[3], const double d[3], double tmin, double c) {
    LD a = tmin, b = c;
    for (int k = 0; k < 3; ++k) {
        const LD inv = 1.0L / (LD)d[k];
        LD t0 = ((LD)lo[k] - (LD)o[k]) * inv, t1 = ((LD)hi[k] - (LD)o[k]) * inv;
        if (std::isnan((double)t0) || std::isnan((double)t1)) return -1;  // o on a plane with d = 0
        const LD mn = t0 < t1 ? t0 : t1, mx = t0 < t1 ? t1 : t0;
        if (mn > a) a = mn;
        if (mx < b) b = mx;
    }
    const LD scale = std::fabs((double)a) + std::fabs((double)b) + 1e-300L;
    if (b - a > 1e-12L * scale) return 1;
    if (b - a < -1e-12L * scale) return 0;
    return -1;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 2000000;
    std::mt19937_64 rng(argc > 2 ? std::atoll(argv[2]) : 2025);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long hits = 0, fhits = 0, bad = 0;
    for (long i = 0; i < n; ++i) {
        double lo[3], hi[3], o[3], d[3];
        const double scale = std::exp(std::log(1e-4) + U(rng) * std::log(1e7));  // box size 1e-4 .. 1e3
        const double off = (U(rng) < 0.3) ? 1e4 * (U(rng) - 0.5) : 20 * (U(rng) - 0.5);
        for (int k = 0; k < 3; ++k) {
            const double c = off + 10 * (U(rng) - 0.5);
            const double w = (U(rng) < 0.1) ? 0.0 : scale * U(rng);  // flat boxes too
            lo[k] = c - w;
            hi[k] = c + w;
        }
        // origin: outside, on a face, on an edge or corner, inside, or remote
        // (a camera near the world origin, the box up to 1e4 away)
        const int ok = (int)(U(rng) * 5);
        for (int k = 0; k < 3; ++k) {
            if (ok == 0) o[k] = lo[k] + (hi[k] - lo[k]) * (3 * U(rng) - 1) + (U(rng) - 0.5) * 10 * scale;
            else if (ok == 4) o[k] = 20 * (U(rng) - 0.5);
            else if (ok == 2) o[k] = U(rng) < 0.5 ? lo[k] : hi[k];
            else o[k] = lo[k] + (hi[k] - lo[k]) * U(rng);
        }
        if (ok == 1) {
            const int k = (int)(U(rng) * 3);
            o[k] = U(rng) < 0.5 ? lo[k] : hi[k];
        }
        // direction: at a random point of the box (or its boundary), random, or
        // grazing along a face; zero components sometimes
        const int dk = (int)(U(rng) * 3);
        if (dk == 0) {
            // a boundary point nudged by 1e-11 .. 1e-5 of the box size, so
            // the exact gap is where f32 rounding decides
            const double nudge = std::exp(std::log(1e-11) + U(rng) * std::log(1e6)) * (U(rng) - 0.5) * (scale + 1e-3);
            for (int k = 0; k < 3; ++k) {
                const double u = U(rng);
                const double p = U(rng) < 0.5 ? (u < 0.5 ? lo[k] : hi[k]) + nudge * (U(rng) - 0.5)
                                              : lo[k] + (hi[k] - lo[k]) * u;
                d[k] = p - o[k];
            }
        } else {
            for (int k = 0; k < 3; ++k) d[k] = U(rng) - 0.5;
        }
        if (dk == 2) d[(int)(U(rng) * 3)] = 0.0;
        const double len = std::exp(std::log(1e-3) + U(rng) * std::log(1e6));
        for (int k = 0; k < 3; ++k) d[k] *= len;
        if (d[0] == 0 && d[1] == 0 && d[2] == 0) continue;
        const double tmin = 1e-8;
        double c = INFINITY;
        const int ck = (int)(U(rng) * 3);
        if (ck == 1) c = std::exp(std::log(1e-6) + U(rng) * std::log(1e12));
        const int ex0 = exact(lo, hi, o, d, tmin, INFINITY);
        if (ck == 2 && ex0 == 1) {  // c right at the entry distance
            LD a = tmin;
            for (int k = 0; k < 3; ++k) {
                const LD inv = 1.0L / (LD)d[k];
                LD t0 = ((LD)lo[k] - (LD)o[k]) * inv, t1 = ((LD)hi[k] - (LD)o[k]) * inv;
                const LD mn = t0 < t1 ? t0 : t1;
                if (mn > a) a = mn;
            }
            c = (double)(a * (1.0L + 1e-9L));
        }
        const int ex = exact(lo, hi, o, d, tmin, c);
        if (ex < 0) continue;
        float flo[3], fhi[3];
        for (int k = 0; k < 3; ++k) {
            flo[k] = down(lo[k]);
            fhi[k] = up(hi[k]);
        }
        const rtk::RayF R = rtk::make_rayf(o, d);
        float entry;
        const bool f = rtk::slab_f(flo, fhi, R, rtk::f32_down(tmin), up(c), entry);
        hits += ex;
        fhits += f;
        if (ex == 1 && !f) {
            if (bad < 10)
                std::printf("VIOLATION origin %d dir %d c %d: lo=(%.17g %.17g %.17g) hi=(%.17g %.17g %.17g) "
                            "o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) c=%.17g\n",
                            ok, dk, ck, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], o[0], o[1], o[2], d[0], d[1], d[2], c);
            ++bad;
        }
    }
    std::printf("%ld %ld %ld %ld\n", n, hits, fhits, bad);
    return bad ? 1 : 0;
}
