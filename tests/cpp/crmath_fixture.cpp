// crmath_fixture.cpp -- writes the argument sets of tests/golden/crmath_args.npz
// (scripts/gen_crmath_fixture.py): for each family, the arguments the path
// feeds the function, glibc's result (what Rust's f64 functions return on
// Linux) and the correctly rounded result (libquadmath's 113-bit value
// rounded to double).  Raw little-endian doubles on stdout, per family:
//   fn code, n, a[n], b[n], glibc[n], cr[n]
//   g++ -O2 -std=c++17 -ffp-contract=off crmath_fixture.cpp -lquadmath -lm
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

static uint64_t s_state = 0x243F6A8885A308D3ull;
static uint64_t next_u64() {  // splitmix64
    uint64_t z = (s_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01() { return (double)(next_u64() >> 11) * 0x1p-53; }

static void emit(double fn, const std::vector<double>& a, const std::vector<double>& b, const std::vector<double>& g,
                 const std::vector<double>& c) {
    const double n = (double)a.size();
    fwrite(&fn, 8, 1, stdout);
    fwrite(&n, 8, 1, stdout);
    fwrite(a.data(), 8, a.size(), stdout);
    fwrite(b.data(), 8, b.size(), stdout);
    fwrite(g.data(), 8, g.size(), stdout);
    fwrite(c.data(), 8, c.size(), stdout);
}

int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 16384;
    const double PI = 3.14159265358979323846;
    // fn codes as rt_math_selftest: 0 sin, 1 cos, 2/3 sincos, 4 log, 5 acos, 6 atan2, 7 sqrt
    for (int fam = 0; fam < 9; ++fam) {
        std::vector<double> a, b, g, c;
        int fn = 0;
        for (long i = 0; i < N; ++i) {
            double x = 0, y = 0, gv = 0, cv = 0;
            switch (fam) {
                case 0:  // sin(2 pi xi): Metal / cosine-PDF / light-sphere draws (vec3.rs:313-343)
                case 1:  // cos(2 pi xi)
                    x = 2.0 * PI * u01();
                    fn = fam;
                    gv = fam == 0 ? sin(x) : cos(x);
                    cv = fam == 0 ? (double)sinq(x) : (double)cosq(x);
                    break;
                case 2:  // sin of NoiseTexture's scale * p.z + 10 turb (texture.rs:191-196)
                case 3:
                    x = (u01() * 2.0 - 1.0) * 2000.0;
                    fn = fam - 2;
                    gv = fn == 0 ? sin(x) : cos(x);
                    cv = fn == 0 ? (double)sinq(x) : (double)cosq(x);
                    break;
                case 4:  // ln xi: ConstantMedium's free flight (volume.rs:58)
                    x = u01();
                    fn = 4;
                    gv = log(x);
                    cv = (double)logq(x);
                    break;
                case 5:  // acos(-n.y): sphere / environment uv (sphere.rs:53-61)
                    x = u01() < 0.9 ? u01() * 2.0 - 1.0 : (u01() < 0.5 ? 1.0 : -1.0) * (1.0 - pow(10.0, -15.0 * u01()));
                    fn = 5;
                    gv = acos(x);
                    cv = (double)acosq(x);
                    break;
                case 6: {  // atan2(-n.z, n.x) of unit vectors (sphere.rs:53-61, environment.rs:14-24)
                    const double t = 2.0 * PI * u01(), z = 2.0 * u01() - 1.0, r = sqrt(1.0 - z * z);
                    x = -(r * sin(t));
                    y = r * cos(t);
                    fn = 6;
                    gv = atan2(x, y);
                    cv = (double)atan2q(x, y);
                    break;
                }
                case 7:  // sqrt: every square root of the path
                    x = u01() * pow(10.0, 12.0 * u01() - 6.0);
                    fn = 7;
                    gv = sqrt(x);
                    cv = (double)sqrtq(x);
                    break;
                default:  // sin(2 pi xi) through sincos
                    x = 2.0 * PI * u01();
                    fn = 2;
                    gv = sin(x);
                    cv = (double)sinq(x);
                    break;
            }
            a.push_back(x);
            b.push_back(y);
            g.push_back(gv);
            c.push_back(cv);
        }
        emit((double)fn, a, b, g, c);
    }
    return 0;
}
