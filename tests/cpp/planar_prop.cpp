// TEST HARNESS: property test of the conservative f32 quad / triangle filter
// (raytracer-2025_amd/csrc/rt_planar_filter.h) against the exact f64 test the
// kernel runs after it (planar_t: quad.rs:71-102 / triangle.rs:69-98 as
// written, f64, no contraction) on random and adversarial (ray, primitive,
// bound) triples.  For each: exact = accepted t over [1e-8, c] or none.
//   filter rejects  =>  exact is none
// Prints "cases rejected violations" and exits 1 on any violation.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../raytracer-2025_amd/csrc/rt_planar_filter.h"

struct V {
    double x, y, z;
};
static V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V operator*(double s, V a) { return {s * a.x, s * a.y, s * a.z}; }
static double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static double l1(V a) { return std::fabs(a.x) + std::fabs(a.y) + std::fabs(a.z); }

struct Prim {  // Quad::new / Triangle::new (quad.rs:30-47)
    V Q, u, v, n, w;
    double D;
};
static Prim make(V Q, V u, V v) {
    Prim p;
    p.Q = Q, p.u = u, p.v = v;
    V nn = cross(u, v);
    const double len = std::sqrt(dot(nn, nn));
    p.n = (1.0 / len) * nn;
    p.D = dot(p.n, Q);
    p.w = (1.0 / dot(nn, nn)) * nn;
    return p;
}

// the kernel's planar_t (rt_kernel.hip), f64
static bool exact(const Prim& P, bool tri, V o, V d, double tmin, double tmax, double& t) {
    const double denom = dot(P.n, d);
    if (std::fabs(denom) < 1e-8) return false;
    const double tt = (P.D - dot(P.n, o)) / denom;
    if (!(tt >= tmin && tt <= tmax)) return false;
    const V hv = (o + tt * d) - P.Q;
    const double alpha = dot(P.w, cross(hv, P.v));
    const double beta = dot(P.w, cross(P.u, hv));
    if (!(alpha >= 0.0 && alpha <= 1.0 && beta >= 0.0 && beta <= 1.0)) return false;
    if (tri) {
        const double ab = alpha + beta;
        if (!(ab >= 0.0 && ab <= 1.0)) return false;
    }
    t = tt;
    return true;
}

static float round_up_f(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}

// rth::flatten's PlanarF (rt_scene.cpp)
static rtk::PlanarF make_f(const Prim& P) {
    rtk::PlanarF F;
    const V a = cross(P.v, P.w), b = cross(P.w, P.u);
    F.n[0] = (float)P.n.x, F.n[1] = (float)P.n.y, F.n[2] = (float)P.n.z, F.D = (float)P.D;
    F.q[0] = (float)P.Q.x, F.q[1] = (float)P.Q.y, F.q[2] = (float)P.Q.z;
    F.g = round_up_f(8.0 * l1(P.Q) + 2.0 * std::fabs(P.D));
    F.a[0] = (float)a.x, F.a[1] = (float)a.y, F.a[2] = (float)a.z, F.sa = round_up_f(l1(a));
    F.b[0] = (float)b.x, F.b[1] = (float)b.y, F.b[2] = (float)b.z, F.sb = round_up_f(l1(b));
    return F;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 2000000;
    std::mt19937_64 rng(argc > 2 ? std::atoll(argv[2]) : 2025);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto unit = [&]() {
        double z = 1 - 2 * U(rng), r = std::sqrt(std::fmax(0.0, 1 - z * z)), p = 2 * M_PI * U(rng);
        return V{r * std::cos(p), r * std::sin(p), z};
    };
    long rejected = 0, bad = 0, hits = 0;
    for (long i = 0; i < n; ++i) {
        // primitive: Cornell walls (axis-aligned, 555), a rotated box face,
        // terrain-size triangles, tiny, huge, far from the origin, slivers
        const int kind = (int)(U(rng) * 7);
        double scale = 1.0;
        V Q, u, v;
        if (kind == 0) {
            const int ax = (int)(U(rng) * 3);
            Q = {0, 0, 0};
            u = ax == 0 ? V{0, 555, 0} : V{555, 0, 0};
            v = ax == 2 ? V{0, 555, 0} : V{0, 0, 555};
            if (U(rng) < 0.5) Q = {555 * (double)(ax == 0), 555 * (double)(ax == 1), 555 * (double)(ax == 2)};
            scale = 555;
        } else if (kind == 1) {
            const V e1 = unit(), e2 = unit();
            Q = {265 + 100 * U(rng), 330 * U(rng), 295 + 100 * U(rng)};
            u = 165.0 * e1;
            v = 165.0 * cross(e1, e2);
            scale = 400;
        } else if (kind == 2) {
            Q = {8 * U(rng) - 4, 0.5 * U(rng), 8 * U(rng) - 4};
            u = 0.0113 * unit();
            v = 0.0113 * unit();
            scale = 5;
        } else if (kind == 3) {
            Q = {1e-4 * U(rng), 1e-4 * U(rng), 1e-4 * U(rng)};
            u = 1e-5 * unit();
            v = 1e-5 * unit();
            scale = 1e-4;
        } else if (kind == 4) {
            Q = {1e4 * (U(rng) - 0.5), 1e4 * (U(rng) - 0.5), 1e4 * (U(rng) - 0.5)};
            u = 3e3 * unit();
            v = 3e3 * unit();
            scale = 1e4;
        } else if (kind == 5) {  // far from the origin, small
            Q = {3000 + U(rng), -2000 + U(rng), 1500 + U(rng)};
            u = 0.5 * unit();
            v = 0.5 * unit();
            scale = 4000;
        } else {  // sliver
            const V e = unit();
            Q = {U(rng), U(rng), U(rng)};
            u = e;
            v = e + 1e-4 * unit();
            scale = 2;
        }
        const V nn = cross(u, v);
        if (!(dot(nn, nn) > 0)) continue;
        const Prim P = make(Q, u, v);
        const bool tri = U(rng) < 0.5;
        // the ray: at a random / edge / vertex / interior point of the
        // primitive, nudged off it by 1e-12 .. 1e-5 (relative); origin random,
        // on the plane, or near; direction toward the target, grazing, or random
        const double a0 = U(rng), b0 = U(rng);
        double al = a0, be = b0;
        const int pk = (int)(U(rng) * 5);
        const double eps = std::exp(std::log(1e-12) + U(rng) * std::log(1e7)) * (U(rng) < 0.5 ? -1 : 1);
        if (pk == 1) al = eps;                                   // near edge alpha = 0
        else if (pk == 2) al = 1 + eps;                          // near alpha = 1
        else if (pk == 3) { al = eps; be = (U(rng) < 0.5 ? 0 : 1) + eps; }  // near a vertex
        else if (pk == 4 && tri) { al = a0; be = 1 - a0 + eps; }  // near the hypotenuse
        const V target = (P.Q + al * P.u) + be * P.v;
        V o;
        const int ok = (int)(U(rng) * 4);
        if (ok == 0) o = target + (scale * 2.0) * unit();
        else if (ok == 1) o = (P.Q + U(rng) * P.u) + U(rng) * P.v;  // on the plane
        else if (ok == 2) o = ((P.Q + U(rng) * P.u) + U(rng) * P.v) + (scale * 1e-6 * (U(rng) - 0.5)) * P.n;
        else o = V{scale * 4 * (U(rng) - 0.5), scale * 4 * (U(rng) - 0.5), scale * 4 * (U(rng) - 0.5)};
        V d;
        const int dk = (int)(U(rng) * 3);
        if (dk == 0) d = target - o;
        else if (dk == 1) {  // grazing: in the plane, tilted by a hair
            V r = unit();
            r = r - dot(r, P.n) * P.n;
            d = r + (std::exp(std::log(1e-9) + U(rng) * std::log(1e8)) * (U(rng) < 0.5 ? -1 : 1)) * P.n;
        } else d = unit();
        const double len = std::exp(std::log(1e-2) + U(rng) * std::log(1e4));
        const double dl = std::sqrt(dot(d, d));
        if (!(dl > 0)) continue;
        d = (len / dl) * d;
        // the walk's closest t: none, random, or right at the exact t
        double tfull;
        const bool hit_full = exact(P, tri, o, d, 1e-8, INFINITY, tfull);
        double c = INFINITY;
        const int bk = (int)(U(rng) * 4);
        if (bk == 1) c = std::exp(std::log(1e-6) + U(rng) * std::log(1e10));
        else if (bk >= 2 && hit_full) c = tfull * (1.0 + (bk == 2 ? 0.0 : (U(rng) - 0.5) * 1e-6));
        const float c_f = round_up_f(c);
        double t;
        const bool ex = exact(P, tri, o, d, 1e-8, c, t);
        hits += ex;
        const double oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z};
        const rtk::PRayF R = rtk::make_prayf(oa, da);
        const bool rej = rtk::planar_reject(make_f(P), R, c_f, tri);
        rejected += rej;
        if (rej && ex) {
            if (bad < 10)
                std::printf("VIOLATION kind %d tri %d point %d origin %d dir %d bound %d: Q=(%.17g %.17g %.17g) "
                            "u=(%.17g %.17g %.17g) v=(%.17g %.17g %.17g) o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) "
                            "c=%.17g t=%.17g\n",
                            kind, tri, pk, ok, dk, bk, Q.x, Q.y, Q.z, u.x, u.y, u.z, v.x, v.y, v.z, o.x, o.y, o.z, d.x,
                            d.y, d.z, c, t);
            ++bad;
        }
    }
    std::printf("hits %ld\n%ld %ld %ld\n", hits, n, rejected, bad);
    return bad ? 1 : 0;
}
