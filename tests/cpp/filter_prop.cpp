// TEST HARNESS: property test of the basic tier's conservative f32 sphere
// filter (raytracer-2025_amd/csrc/rt_sphere_filter.h) against the exact f64
// test (sphere_exact.cpp) on random and adversarial (ray, sphere, bound)
// triples.  For every triple, with t = the exact accepted root over
// [1e-8, inf) (none = miss):
//   (a) filter rejects             => t is none or t > c_f (the bound it got)
//   (b) filter lowers c_f to c_f'  => t exists and t <= c_f'
//   (c) c_f' <= c_f always
// Prints "cases rejected lowered violations" and exits 1 on any violation.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../raytracer-2025_amd/csrc/rt_sphere_filter.h"

extern "C" double exact_sphere_t(const double c[3], double r, const double o[3], const double d[3], double tmin,
                                 double tmax);

static float round_up_f(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 2000000;
    std::mt19937_64 rng(argc > 2 ? std::atoll(argv[2]) : 2025);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto unit = [&](double v[3]) {
        double z = 1 - 2 * U(rng), r = std::sqrt(std::fmax(0.0, 1 - z * z)), p = 2 * M_PI * U(rng);
        v[0] = r * std::cos(p);
        v[1] = r * std::sin(p);
        v[2] = z;
    };
    long rejected = 0, lowered = 0, bad = 0;
    for (long i = 0; i < n; ++i) {
        // sphere: book-1 small / big / ground, tiny, far away
        double c[3], r;
        const int kind = (int)(U(rng) * 6);
        if (kind == 0) { c[0] = 0; c[1] = -1000; c[2] = 0; r = 1000; }
        else if (kind == 1) { c[0] = -11 + 22 * U(rng); c[1] = 0.2; c[2] = -11 + 22 * U(rng); r = 0.2; }
        else if (kind == 2) { c[0] = 4 * (int)(U(rng) * 3) - 4; c[1] = 1; c[2] = 0; r = 1; }
        else if (kind == 3) { c[0] = 1e4 * (U(rng) - 0.5); c[1] = 1e4 * (U(rng) - 0.5); c[2] = 1e3 * U(rng); r = 1e-3 + U(rng); }
        else if (kind == 4) { c[0] = U(rng); c[1] = U(rng); c[2] = U(rng); r = 1e-3 * (1 + U(rng)); }
        else { c[0] = 100 * (U(rng) - 0.5); c[1] = 50 * U(rng); c[2] = 100 * (U(rng) - 0.5); r = 50 * U(rng) + 0.01; }
        // ray: origin on this sphere's surface (self-intersection regime), near
        // it, at the book-1 camera, or anywhere; direction random, tangent to
        // the sphere at its origin, or aimed at the sphere's rim
        double o[3], d[3], nrm[3];
        unit(nrm);
        const int ok = (int)(U(rng) * 5);
        const double lift = ok == 1 ? (U(rng) - 0.5) * 1e-6 * r : 0.0;
        if (ok <= 1) for (int k = 0; k < 3; ++k) o[k] = c[k] + (r + lift) * nrm[k];
        else if (ok == 2) { o[0] = 13; o[1] = 2; o[2] = 3; }
        else if (ok == 4) {  // inside: anywhere from the center to a hair below the surface
            const double f = U(rng) < 0.5 ? U(rng) : 1.0 - std::exp(std::log(1e-12) + U(rng) * std::log(1e10));
            for (int k = 0; k < 3; ++k) o[k] = c[k] + f * r * nrm[k];
        }
        else for (int k = 0; k < 3; ++k) o[k] = c[k] + (U(rng) - 0.5) * 40 * (r + 1);
        const int dk = (int)(U(rng) * 3);
        unit(d);
        if (dk == 1 && ok <= 1) {  // tangent at the origin's surface point
            const double dn = d[0] * nrm[0] + d[1] * nrm[1] + d[2] * nrm[2];
            for (int k = 0; k < 3; ++k) d[k] -= dn * nrm[k];
            for (int k = 0; k < 3; ++k) d[k] += (U(rng) - 0.5) * 1e-7 * nrm[k];
        } else if (dk == 2) {      // aim at a point of the rim as seen from o
            double t[3];
            unit(t);
            double p[3];
            for (int k = 0; k < 3; ++k) p[k] = c[k] + r * (1 + (U(rng) - 0.5) * 1e-6) * t[k];
            for (int k = 0; k < 3; ++k) d[k] = p[k] - o[k];
        }
        const double len = std::exp(std::log(1e-2) + U(rng) * std::log(1e4));  // |d| in [0.01, 100]
        for (int k = 0; k < 3; ++k) d[k] *= len;
        const double tx = exact_sphere_t(c, r, o, d, 1e-8, INFINITY);
        // the walk's bound: none, random, or right at the exact root
        float cf = INFINITY;
        const int bk = (int)(U(rng) * 4);
        if (bk == 1) cf = (float)(std::exp(std::log(1e-6) + U(rng) * std::log(1e10)));
        else if (bk >= 2 && tx >= 0) cf = (float)(tx * (1.0 + (U(rng) - 0.5) * 1e-5));
        const rtk::SphF F = rtk::make_sphf(o, d);
        const float cx = (float)c[0], cy = (float)c[1], cz = (float)c[2], rf = (float)r;
        const float g = round_up_f(std::fabs((double)cx) + std::fabs((double)cy) + std::fabs((double)cz) + std::fabs((double)rf));
        float cf2 = cf;
        const bool keep = rtk::sphere_filter(cx, cy, cz, rf, g, F, cf2, true);
        bool ok_case = cf2 <= cf || (std::isnan(cf) && std::isnan(cf2));
        if (!keep) {
            ++rejected;
            ok_case = ok_case && (tx < 0 || tx > (double)cf);
        }
        if (cf2 < cf) {
            ++lowered;
            ok_case = ok_case && tx >= 0 && tx <= (double)cf2;
        }
        if (!ok_case) {
            if (bad < 10)
                std::printf("VIOLATION kind %d origin %d dir %d bound %d: c=(%.17g %.17g %.17g) r=%.17g o=(%.17g %.17g %.17g) "
                            "d=(%.17g %.17g %.17g) exact t=%.17g cf=%.9g -> keep %d cf'=%.9g\n",
                            kind, ok, dk, bk, c[0], c[1], c[2], r, o[0], o[1], o[2], d[0], d[1], d[2], tx, cf, keep, cf2);
            ++bad;
        }
    }
    std::printf("%ld %ld %ld %ld\n", n, rejected, lowered, bad);
    return bad ? 1 : 0;
}
