// crmath_check.cpp -- CPU check of rt_crmath.h (tests/test_crmath_cpu.py).
//
// For each function and argument family: rtcr::f(x) against the correctly
// rounded value (libquadmath's 113-bit result rounded to double), and glibc's
// f(x) against the same -- the rate at which glibc itself is not correctly
// rounded is the floor of any device / host disagreement after the switch.
// Also counts how often the slow path ran.  Prints one JSON object.
//
//   g++ -O2 -std=c++17 -ffp-contract=off crmath_check.cpp -lquadmath -o crmath_check
//   ./crmath_check [n_per_family] [dump.bin]
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

static unsigned long long g_slow = 0;
#define RTCR_SLOW_COUNTER g_slow
#include "../../raytracer-2025_amd/csrc/rt_crmath.h"

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64() {  // splitmix64
    uint64_t z = (s_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01() { return (double)(next_u64() >> 11) * 0x1p-53; }  // the path's draw

struct Tally {
    std::string name;
    long n = 0, cr_bad = 0, glibc_bad = 0, cr_ne_glibc = 0;
    unsigned long long slow = 0;
    double first_bad = 0.0, first_bad_y = 0.0;
};

static bool same(double a, double b) { return (a == b && signbit(a) == signbit(b)) || (a != a && b != b); }

template <class F, class G, class R>
static void run(Tally& t, const std::vector<double>& xs, const std::vector<double>& ys, F cr, G glibc, R ref) {
    const unsigned long long s0 = g_slow;
    for (size_t i = 0; i < xs.size(); ++i) {
        const double x = xs[i], y = ys.empty() ? 0.0 : ys[i];
        const double a = cr(x, y), g = glibc(x, y), r = ref(x, y);
        ++t.n;
        if (!same(a, r)) {
            if (!t.cr_bad) t.first_bad = x, t.first_bad_y = y;
            ++t.cr_bad;
        }
        if (!same(g, r)) ++t.glibc_bad;
        if (!same(a, g)) ++t.cr_ne_glibc;
    }
    t.slow += g_slow - s0;
}

int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 200000;
    std::vector<Tally> out;
    auto fam = [&](const char* name) -> Tally& {
        out.push_back(Tally{});
        out.back().name = name;
        return out.back();
    };
    const double PI = 3.14159265358979323846;
    std::vector<double> none;

    // ---- sin / cos: the path's 2 pi xi, wide ranges, hard spots, huge
    auto sin_c = [](double x, double) { return rtcr::sin(x); };
    auto sin_g = [](double x, double) { return sin(x); };
    auto sin_q = [](double x, double) { return (double)sinq((__float128)x); };
    auto cos_c = [](double x, double) { return rtcr::cos(x); };
    auto cos_g = [](double x, double) { return cos(x); };
    auto cos_q = [](double x, double) { return (double)cosq((__float128)x); };
    auto sc_s = [](double x, double) { double s, c; rtcr::sincos(x, &s, &c); return s; };
    auto sc_c = [](double x, double) { double s, c; rtcr::sincos(x, &s, &c); return c; };
    std::vector<double> a_path, a_wide, a_log, a_hard, a_huge;
    for (long i = 0; i < N; ++i) a_path.push_back(2.0 * PI * u01());
    for (long i = 0; i < N; ++i) a_wide.push_back((u01() * 2.0 - 1.0) * 2e4);
    for (long i = 0; i < N; ++i) a_log.push_back((u01() < 0.5 ? -1 : 1) * pow(10.0, -20.0 + 26.0 * u01()));
    for (long i = 0; i < N; ++i) {  // a few ulps around k pi/128 and k pi/2
        const long k = (long)(u01() * 4096.0) - 2048;
        const double c = (u01() < 0.5 ? (double)k * PI / 128.0 : (double)(k / 32) * PI / 2.0);
        double x = c;
        const int steps = (int)(u01() * 64.0) - 32;
        for (int s = 0; s < (steps < 0 ? -steps : steps); ++s) x = nextafter(x, steps < 0 ? -1e300 : 1e300);
        a_hard.push_back(x);
    }
    for (long i = 0; i < N / 4; ++i) a_huge.push_back((u01() < 0.5 ? -1 : 1) * pow(2.0, 20.0 + 1000.0 * u01()));
    a_huge.push_back(0x1.6ac5b262ca1ffp+849);  // classic hard reductions
    a_huge.push_back(0x1.6a09e667f3bcdp+0);
    a_huge.push_back(6381956970095103.0 * pow(2.0, 797));
    a_huge.push_back(5261692873635770.0 * pow(2.0, 499));
    a_hard.push_back(PI);
    a_hard.push_back(2 * PI);
    a_hard.push_back(PI / 2);
    a_hard.push_back(0.0);
    a_hard.push_back(-0.0);
    a_hard.push_back(1e-300);
    a_hard.push_back(0x1p-1074);
    struct {
        const char* n;
        std::vector<double>* v;
    } sets[] = {{"path_2pi_xi", &a_path}, {"wide_2e4", &a_wide}, {"log_uniform", &a_log}, {"near_k_pi_128", &a_hard},
                {"huge", &a_huge}};
    for (auto& s : sets) {
        run(fam((std::string("sin/") + s.n).c_str()), *s.v, none, sin_c, sin_g, sin_q);
        run(fam((std::string("cos/") + s.n).c_str()), *s.v, none, cos_c, cos_g, cos_q);
        run(fam((std::string("sincos.sin/") + s.n).c_str()), *s.v, none, sc_s, sin_g, sin_q);
        run(fam((std::string("sincos.cos/") + s.n).c_str()), *s.v, none, sc_c, cos_g, cos_q);
    }

    // ---- sincos_2pi(xi) = sincos(2 pi xi): the path's draws, and xi stepped
    // ulp by ulp around k / 256 (x next to k pi/128, every k of the range)
    auto s2_s = [](double xi, double) { double s, c; rtcr::sincos_2pi(xi, &s, &c); return s; };
    auto s2_c = [](double xi, double) { double s, c; rtcr::sincos_2pi(xi, &s, &c); return c; };
    auto s2_sg = [PI](double xi, double) { return sin(2.0 * PI * xi); };
    auto s2_cg = [PI](double xi, double) { return cos(2.0 * PI * xi); };
    auto s2_sq = [PI](double xi, double) { return (double)sinq((__float128)(2.0 * PI * xi)); };
    auto s2_cq = [PI](double xi, double) { return (double)cosq((__float128)(2.0 * PI * xi)); };
    std::vector<double> x_path, x_hard;
    for (long i = 0; i < N; ++i) x_path.push_back(u01());
    for (double v : {0.0, 1.0, 0.5, 0.25, 0.75, 0x1p-53, 1.0 - 0x1p-53, 0.125}) x_path.push_back(v);
    for (int k = 0; k <= 256; ++k) {
        const double c = k / 256.0;
        for (int st = -40; st <= 40; ++st) {
            double xi = c;
            for (int j = 0; j < (st < 0 ? -st : st); ++j) xi = nextafter(xi, st < 0 ? -1.0 : 2.0);
            if (xi >= 0.0 && xi <= 1.0) x_hard.push_back(xi);
        }
    }
    run(fam("sincos_2pi.sin/path_xi"), x_path, none, s2_s, s2_sg, s2_sq);
    run(fam("sincos_2pi.cos/path_xi"), x_path, none, s2_c, s2_cg, s2_cq);
    run(fam("sincos_2pi.sin/near_k_over_256"), x_hard, none, s2_s, s2_sg, s2_sq);
    run(fam("sincos_2pi.cos/near_k_over_256"), x_hard, none, s2_c, s2_cg, s2_cq);

    // ---- log: the media's ln xi, wide, near 1, subnormal, specials
    auto log_c = [](double x, double) { return rtcr::log(x); };
    auto log_g = [](double x, double) { return log(x); };
    auto log_q = [](double x, double) { return (double)logq((__float128)x); };
    std::vector<double> l_path, l_wide, l_one;
    for (long i = 0; i < N; ++i) l_path.push_back(u01());
    for (long i = 0; i < N; ++i) l_wide.push_back(pow(2.0, -1074.0 + 2097.0 * u01()));
    for (long i = 0; i < N; ++i) l_one.push_back(1.0 + (u01() - 0.5) * (u01() < 0.5 ? 0x1p-6 : 0x1p-30));
    for (double v : {0.0, -0.0, 1.0, 2.0, 0.5, -1.0, 1e-310, 0x1p-1074, 1.7976931348623157e308}) l_path.push_back(v);
    l_path.push_back(__builtin_inf());
    l_path.push_back(__builtin_nan(""));
    run(fam("log/path_xi"), l_path, none, log_c, log_g, log_q);
    run(fam("log/wide"), l_wide, none, log_c, log_g, log_q);
    run(fam("log/near_1"), l_one, none, log_c, log_g, log_q);

    // ---- acos: -n.y of unit normals, near +-1, specials
    auto acos_c = [](double x, double) { return rtcr::acos(x); };
    auto acos_g = [](double x, double) { return acos(x); };
    auto acos_q = [](double x, double) { return (double)acosq((__float128)x); };
    std::vector<double> c_path, c_edge;
    for (long i = 0; i < N; ++i) c_path.push_back(u01() * 2.0 - 1.0);
    for (long i = 0; i < N; ++i) {
        const double d = pow(10.0, -16.0 + 15.0 * u01());
        c_edge.push_back(u01() < 0.5 ? 1.0 - d : -1.0 + d);
    }
    for (double v : {1.0, -1.0, 0.0, -0.0, 0.5, -0.5, 1.0000000000000002, -1.0000000000000002}) c_edge.push_back(v);
    run(fam("acos/uniform"), c_path, none, acos_c, acos_g, acos_q);
    run(fam("acos/near_pm1"), c_edge, none, acos_c, acos_g, acos_q);

    // ---- atan2: sphere-uv style (-n.z, n.x), wide magnitudes, axes
    auto at_c = [](double y, double x) { return rtcr::atan2(y, x); };
    auto at_g = [](double y, double x) { return atan2(y, x); };
    auto at_q = [](double y, double x) { return (double)atan2q((__float128)y, (__float128)x); };
    std::vector<double> ty, tx, wy, wx;
    for (long i = 0; i < N; ++i) ty.push_back(u01() * 2.0 - 1.0), tx.push_back(u01() * 2.0 - 1.0);
    for (long i = 0; i < N; ++i) {
        wy.push_back((u01() < 0.5 ? -1 : 1) * pow(2.0, -1000.0 + 2000.0 * u01()));
        wx.push_back((u01() < 0.5 ? -1 : 1) * pow(2.0, -1000.0 + 2000.0 * u01()));
    }
    const double sp[] = {0.0, -0.0, 1.0, -1.0, __builtin_inf(), -__builtin_inf(), 1e-300, -1e300};
    for (double a : sp)
        for (double b : sp) ty.push_back(a), tx.push_back(b);
    run(fam("atan2/unit_square"), ty, tx, at_c, at_g, at_q);
    run(fam("atan2/wide"), wy, wx, at_c, at_g, at_q);

    printf("{\"families\": [");
    for (size_t i = 0; i < out.size(); ++i) {
        const Tally& t = out[i];
        printf("%s{\"name\": \"%s\", \"n\": %ld, \"cr_not_correctly_rounded\": %ld, \"glibc_not_correctly_rounded\": %ld, "
               "\"cr_ne_glibc\": %ld, \"slow_path\": %llu, \"first_bad\": [\"%a\", \"%a\"]}",
               i ? ", " : "", t.name.c_str(), t.n, t.cr_bad, t.glibc_bad, t.cr_ne_glibc, t.slow, t.first_bad,
               t.first_bad_y);
    }
    printf("]}\n");
    return 0;
}
