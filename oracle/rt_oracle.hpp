// oracle/rt_oracle.hpp -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement (C++17, IEEE f64, -ffp-contract=off) of the reference render
// path of caidj0/Raytracer-2025 (Rust, /root/reference).  It is the parity
// checker for the gfx950 kernel and the "port" CPU baseline of bench.py.  It is
// never linked into, loaded by, or called from the product library.
//
// Every type below restates one reference type; each function cites the
// reference file:line it follows.  The structure is deliberately the
// reference's: trait objects (virtual classes), a recursive ray_color, BVH
// built by longest-axis / sort-by-min / median split, Hittables tested with the
// full interval and min_by(t).  Only the RNG differs (see rng_contract.hpp).
//
// Parity pins: the reference's own unit tests (vec3.rs, ray.rs, aabb.rs,
// quaternion.rs, sphere.rs) are restated in oracle/kat_reference_tests.cpp and
// run by tests/test_oracle_kat.py; Philox is pinned by the Random123 KATs.
#pragma once
#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "rng_contract.hpp"
#ifdef ORC_CRMATH
// liboracle_cr.so only: the render path's libm calls go to the kernel's
// correctly rounded functions instead of glibc, so that a GPU-vs-oracle
// comparison isolates everything but libm (tests/test_parity_gpu.py: RMSE 0,
// no diverged sums).  The default liboracle.so calls glibc, as Rust's f64
// functions do on Linux.
#include "../raytracer-2025_amd/csrc/rt_crmath.h"
#endif

namespace orc {

// The path's transcendentals (vec3.rs:63-69, 313-343; sphere.rs:53-61;
// environment.rs:14-24; volume.rs:58; texture.rs:191-196)
namespace m {
#ifdef ORC_CRMATH
inline double sin(double x) { return rtcr::sin(x); }
inline double cos(double x) { return rtcr::cos(x); }
inline double log(double x) { return rtcr::log(x); }
inline double acos(double x) { return rtcr::acos(x); }
inline double atan2(double y, double x) { return rtcr::atan2(y, x); }
#else
inline double sin(double x) { return std::sin(x); }
inline double cos(double x) { return std::cos(x); }
inline double log(double x) { return std::log(x); }
inline double acos(double x) { return std::acos(x); }
inline double atan2(double y, double x) { return std::atan2(y, x); }
#endif
}  // namespace m

constexpr double PI = 3.14159265358979323846264338327950288;
constexpr double INF = std::numeric_limits<double>::infinity();

// A reference panic!/assert!/expect failure.  The C API turns it into an error
// code (the reference aborts the process).
struct Panic : std::runtime_error {
    explicit Panic(const std::string& m) : std::runtime_error(m) {}
};

// ---------------------------------------------------------------- Vec3
// src/utils/vec3.rs:13-304
struct Vec3 {
    double e[3];
    constexpr Vec3() : e{0.0, 0.0, 0.0} {}
    constexpr Vec3(double x, double y, double z) : e{x, y, z} {}
    double x() const { return e[0]; }
    double y() const { return e[1]; }
    double z() const { return e[2]; }
    double operator[](int i) const { return e[i]; }
    double& operator[](int i) { return e[i]; }
    // vec3.rs:94-96
    double length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
    // vec3.rs:103-105
    double length() const { return std::sqrt(length_squared()); }
    // vec3.rs:107-109
    double dot(const Vec3& r) const { return e[0] * r.e[0] + e[1] * r.e[1] + e[2] * r.e[2]; }
    // vec3.rs:111-117
    Vec3 cross(const Vec3& r) const {
        return Vec3(e[1] * r.e[2] - e[2] * r.e[1], e[2] * r.e[0] - e[0] * r.e[2], e[0] * r.e[1] - e[1] * r.e[0]);
    }
    // vec3.rs:71-73  self - 2*(self.n)*n
    Vec3 reflect(const Vec3& n) const;
    Vec3 operator-() const { return Vec3(-e[0], -e[1], -e[2]); }
    Vec3& operator+=(const Vec3& r) {
        e[0] += r.e[0];
        e[1] += r.e[1];
        e[2] += r.e[2];
        return *this;
    }
    bool operator==(const Vec3& r) const { return e[0] == r.e[0] && e[1] == r.e[1] && e[2] == r.e[2]; }
    bool any_nan() const { return std::isnan(e[0]) || std::isnan(e[1]) || std::isnan(e[2]); }
};
using Point3 = Vec3;
using Color = Vec3;

inline Vec3 operator+(const Vec3& a, const Vec3& b) { return Vec3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline Vec3 operator-(const Vec3& a, const Vec3& b) { return Vec3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline Vec3 operator*(const Vec3& a, const Vec3& b) { return Vec3(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
inline Vec3 operator/(const Vec3& a, const Vec3& b) { return Vec3(a.e[0] / b.e[0], a.e[1] / b.e[1], a.e[2] / b.e[2]); }
// vec3.rs:140-146 / 156-162
inline Vec3 operator*(double s, const Vec3& v) { return Vec3(s * v.e[0], s * v.e[1], s * v.e[2]); }
inline Vec3 operator*(const Vec3& v, double s) { return Vec3(v.e[0] * s, v.e[1] * s, v.e[2] * s); }
// vec3.rs:226-232: Div<f64> is `1.0 / rhs * self`
inline Vec3 operator/(const Vec3& v, double s) { return (1.0 / s) * v; }
inline Vec3 Vec3::reflect(const Vec3& n) const { return *this - (2.0 * this->dot(n)) * n; }

// vec3.rs:299-306 UnitVec3::from_vec3: v / |v|, None unless every component finite
inline std::optional<Vec3> from_vec3(const Vec3& v) {
    Vec3 u = v / v.length();
    if (std::isfinite(u.e[0]) && std::isfinite(u.e[1]) && std::isfinite(u.e[2])) return u;
    return std::nullopt;
}
inline Vec3 expect_unit(const Vec3& v, const char* what) {
    auto u = from_vec3(v);
    if (!u) throw Panic(what);
    return *u;
}

// ---------------------------------------------------------------- Random
// src/utils/random.rs:5-27 -- thread-local facade.  The per-path keyed stream
// replaces ThreadRng (rng_contract.hpp).
struct PathRng {
    uint64_t seed = 0;
    uint32_t pixel = 0, sample = 0, vertex = 0, slot = 0;
    void begin_vertex(uint32_t v) {
        vertex = v;
        slot = 0;
    }
    double next() {
        if (slot >= 16) throw Panic("rng slot overflow (>16 draws in one path vertex)");
        return rng_main(seed, pixel, sample, vertex, slot++);
    }
    double medium(uint32_t id) const { return rng_medium(seed, pixel, sample, vertex, id); }
};

PathRng*& current_rng();  // thread-local slot, rt_oracle.cpp

struct Random {
    // random.rs:12-14
    static double f64() {
        PathRng* r = current_rng();
        if (!r) throw Panic("Random::f64 outside a render path");
        return r->next();
    }
    // random.rs:16-18  (rand's UniformFloat restated as lo + (hi-lo)*xi)
    static double random_range(double lo, double hi) { return lo + (hi - lo) * f64(); }
    // random.rs:24-26 / hits.rs:71 choose: uniform index in [0, n)
    static size_t index(size_t n) {
        size_t k = (size_t)(f64() * (double)n);
        return k < n ? k : n - 1;
    }
};

// vec3.rs:63-69
inline Vec3 random_in_unit_disk() {
    double theta = Random::random_range(0.0, 2.0 * PI);
    double r = std::sqrt(Random::f64());
    return Vec3(r * m::cos(theta), r * m::sin(theta), 0.0);
}
// vec3.rs:313-322
inline Vec3 random_unit_vector() {
    double r1 = Random::f64();
    double r2 = Random::f64();
    double x = m::cos(2.0 * PI * r1) * 2.0 * std::sqrt(r2 * (1.0 - r2));
    double y = m::sin(2.0 * PI * r1) * 2.0 * std::sqrt(r2 * (1.0 - r2));
    double z = 1.0 - 2.0 * r2;
    return Vec3(x, y, z);
}
// vec3.rs:333-343 (y-up)
inline Vec3 random_cosine_direction() {
    double r1 = Random::f64();
    double r2 = Random::f64();
    double phi = 2.0 * PI * r1;
    double x = m::sin(phi) * std::sqrt(r2);
    double y = std::sqrt(1.0 - r2);
    double z = m::cos(phi) * std::sqrt(r2);
    return Vec3(x, y, z);
}
// vec3.rs:345-354
inline std::optional<Vec3> refract(const Vec3& uv, const Vec3& n, double eta) {
    double cos_theta = std::fmin((-uv).dot(n), 1.0);
    Vec3 out_perp = eta * (uv + cos_theta * n);
    double par_len = std::sqrt(1.0 - out_perp.length_squared());
    if (std::isnan(par_len)) return std::nullopt;
    Vec3 out_par = -par_len * n;
    return out_perp + out_par;
}

// ---------------------------------------------------------------- Interval
// src/utils/interval.rs:4-77
struct Interval {
    double min = 0.0, max = 0.0;
    Interval() = default;
    static Interval make(double a, double b) {  // interval.rs:10-15 (f64::min/max)
        Interval i;
        i.min = std::fmin(a, b);
        i.max = std::fmax(a, b);
        return i;
    }
    static Interval range(double a, double b) {  // interval.rs:17-22
        Interval i;
        i.min = a;
        i.max = b;
        return i;
    }
    Interval expand(double delta) const {  // interval.rs:28-34
        double padding = delta / 2.0;
        return range(min - padding, max + padding);
    }
    double size() const { return std::fmax(max - min, 0.0); }  // interval.rs:44-46
    std::optional<Interval> intersect(const Interval& r) const {  // interval.rs:48-56
        double mx = std::fmin(max, r.max);
        double mn = std::fmax(min, r.min);
        if (mn <= mx) return range(mn, mx);
        return std::nullopt;
    }
    Interval unite(const Interval& r) const { return range(std::fmin(min, r.min), std::fmax(max, r.max)); }
    bool contains(double x) const { return x >= min && x <= max; }  // interval.rs:65-67
    static Interval empty() { return range(INF, -INF); }
    static Interval universe() { return range(-INF, INF); }
    bool operator==(const Interval& o) const { return min == o.min && max == o.max; }
};

// ---------------------------------------------------------------- Ray
// src/utils/ray.rs:4-42
struct Ray {
    Point3 orig;
    Vec3 dir;
    double time = 0.0;
    Ray() = default;
    Ray(const Point3& o, const Vec3& d, double t = 0.0) : orig(o), dir(d), time(t) {}
    Point3 at(double t) const { return orig + t * dir; }
};

// ---------------------------------------------------------------- AABB
// src/aabb.rs:10-127
struct AABB {
    Interval x = Interval(), y = Interval(), z = Interval();
    AABB() = default;
    static AABB raw(const Interval& a, const Interval& b, const Interval& c) {
        AABB r;
        r.x = a;
        r.y = b;
        r.z = c;
        return r;
    }
    AABB pad_to_minimums() const {  // aabb.rs:43-51
        const double DELTA = 0.0001;
        auto pad = [&](const Interval& t) { return t.size() < DELTA ? t.expand(DELTA) : t; };
        return raw(pad(x), pad(y), pad(z));
    }
    static AABB make(const Interval& a, const Interval& b, const Interval& c) { return raw(a, b, c).pad_to_minimums(); }
    static AABB from_points(const Point3& a, const Point3& b) {  // aabb.rs:21-28
        return raw(Interval::make(a[0], b[0]), Interval::make(a[1], b[1]), Interval::make(a[2], b[2])).pad_to_minimums();
    }
    const Interval& axis_interval(int n) const {  // aabb.rs:53-60
        switch (n) {
            case 0: return x;
            case 1: return y;
            case 2: return z;
            default: throw Panic("The index of axis should between 0 and 2!");
        }
    }
    std::array<Point3, 8> all_points() const {  // aabb.rs:30-41
        return {Point3(x.min, y.min, z.min), Point3(x.min, y.min, z.max), Point3(x.min, y.max, z.min),
                Point3(x.min, y.max, z.max), Point3(x.max, y.min, z.min), Point3(x.max, y.min, z.max),
                Point3(x.max, y.max, z.min), Point3(x.max, y.max, z.max)};
    }
    bool hit(const Ray& r, Interval ray_t) const;  // aabb.rs:62-78
    int longest_axis() const {                      // aabb.rs:80-92
        double lx = x.size(), ly = y.size(), lz = z.size();
        if (lx > ly) return lx > lz ? 0 : 2;
        return ly > lz ? 1 : 2;
    }
    AABB unite(const AABB& r) const { return raw(x.unite(r.x), y.unite(r.y), z.unite(r.z)); }  // aabb.rs:94-100
    static AABB empty() { return raw(Interval::empty(), Interval::empty(), Interval::empty()); }
    static AABB universe() { return raw(Interval::universe(), Interval::universe(), Interval::universe()); }
};

// ---------------------------------------------------------------- Quaternion
// src/utils/quaternion.rs:5-104
struct Quaternion {
    double w = 1.0, x = 0.0, y = 0.0, z = 0.0;
    static Quaternion identity() { return Quaternion{1.0, 0.0, 0.0, 0.0}; }
    static Quaternion from_euler(double yaw, double pitch, double roll);  // quaternion.rs:23-38
    static Quaternion from_axis_angle(const Vec3& axis, double deg);     // quaternion.rs:40-53
    void to_euler(double& yaw, double& pitch, double& roll) const;        // quaternion.rs:55-70
    Quaternion conjugate() const { return Quaternion{w, -x, -y, -z}; }
    Quaternion operator*(const Quaternion& r) const {  // quaternion.rs:94-103
        return Quaternion{w * r.w - x * r.x - y * r.y - z * r.z, w * r.x + x * r.w + y * r.z - z * r.y,
                          w * r.y - x * r.z + y * r.w + z * r.x, w * r.z + x * r.y - y * r.x + z * r.w};
    }
    Vec3 rotate_vector(const Vec3& v) const {  // quaternion.rs:72-82
        Quaternion qv{0.0, v.x(), v.y(), v.z()};
        Quaternion res = (*this * qv) * conjugate();
        return Vec3(res.x, res.y, res.z);
    }
};

// ---------------------------------------------------------------- ONB
// src/utils/onb.rs:3-45
struct ONB {
    Vec3 axis[3];
    explicit ONB(const Vec3& n) {
        Vec3 a = std::fabs(n.x()) > 0.9 ? Vec3(0.0, 1.0, 0.0) : Vec3(1.0, 0.0, 0.0);
        Vec3 u = expect_unit(n.cross(a), "ONB u normalize");
        Vec3 w = u.cross(n);
        axis[0] = u;
        axis[1] = n;
        axis[2] = w;
    }
    const Vec3& v() const { return axis[1]; }
    Vec3 onb_to_world(const Vec3& v) const { return v[0] * axis[0] + v[1] * axis[1] + v[2] * axis[2]; }
};

// ---------------------------------------------------------------- Work counters
// Instrumentation for SURVEY §8(d) algorithmic work per sample (not in the
// reference).  Thread-local, summed by the renderer.
struct WorkCounts {
    uint64_t camera_rays = 0, ray_color_calls = 0, bvh_node_tests = 0, sphere_tests = 0, sphere_disc_ok = 0,
             sphere_records = 0, quad_tests = 0, tri_tests = 0, planar_records = 0, lambert = 0, metal = 0,
             dielectric = 0, isotropic = 0, sky_miss = 0, medium_tests = 0, light_pdf = 0, transform_tests = 0,
             emitted = 0;
    void add(const WorkCounts& o) {
        const uint64_t* s = &o.camera_rays;
        uint64_t* d = &camera_rays;
        for (size_t i = 0; i < sizeof(WorkCounts) / sizeof(uint64_t); ++i) d[i] += s[i];
    }
};
WorkCounts& work();
// The counting build (liboracle.so: scripts/work_counts.py, the tests) bumps a
// thread-local counter at every node test, primitive test and scatter; the
// timed CPU baseline (liboracle_fast.so, bench.py's cpu_baseline) is built
// with -DORC_NO_COUNTS, so none of those TLS accesses is in the measured work.
#ifdef ORC_NO_COUNTS
#define ORC_COUNT(field) ((void)0)
#else
#define ORC_COUNT(field) (++::orc::work().field)
#endif

// ---------------------------------------------------------------- Textures
// src/texture.rs:5-7
struct Texture {
    virtual ~Texture() = default;
    virtual Color value(double u, double v, const Point3& p) const = 0;
};
struct SolidColor : Texture {  // texture.rs:10-36
    Color albedo;
    explicit SolidColor(const Color& c) : albedo(c) {}
    Color value(double, double, const Point3&) const override { return albedo; }
};
struct CheckerTexture : Texture {  // texture.rs:39-73
    double inv_scale;
    std::shared_ptr<Texture> even, odd;
    CheckerTexture(double scale, std::shared_ptr<Texture> e, std::shared_ptr<Texture> o)
        : inv_scale(1.0 / scale), even(std::move(e)), odd(std::move(o)) {}
    Color value(double u, double v, const Point3& p) const override {
        int32_t xi = (int32_t)std::floor(inv_scale * p.x());
        int32_t yi = (int32_t)std::floor(inv_scale * p.y());
        int32_t zi = (int32_t)std::floor(inv_scale * p.z());
        bool is_even = ((xi + yi + zi) % 2) == 0;
        return is_even ? even->value(u, v, p) : odd->value(u, v, p);
    }
};
// Book-1 sky: the reference has no book-1 sky gradient, so the
// build defines it as a user Texture plugged into Camera.background
// (camera.rs:50, environment.rs:14-24).  p is the normalised ray direction.
struct SkyGradient : Texture {
    Color horizon, zenith;
    SkyGradient(const Color& h, const Color& z) : horizon(h), zenith(z) {}
    Color value(double, double, const Point3& p) const override {
        double a = 0.5 * (p.y() + 1.0);
        return (1.0 - a) * horizon + a * zenith;
    }
};
// texture.rs:76-174 + utils/image.rs:10-82.  Pixels are supplied decoded to
// linear RGBA f32 (the decode happens in the caller); w==h==0 is the "file
// missing" image: value -> cyan (texture.rs:167-169).
struct ImageTexture : Texture {
    int w = 0, h = 0;
    std::vector<float> rgba;
    bool linear_interp = false;
    std::array<float, 4> pixel_data(int64_t x, int64_t y) const {  // image.rs:63-82 (clamp)
        if (h == 0) return {1.0f, 0.0f, 1.0f, 1.0f};
        x = std::clamp<int64_t>(x, 0, w - 1);
        y = std::clamp<int64_t>(y, 0, h - 1);
        const float* p = &rgba[((size_t)y * w + x) * 4];
        return {p[0], p[1], p[2], p[3]};
    }
    static double abs_fract(double x) { return x - std::floor(x); }
    std::array<float, 4> get_pixel(double u, double v) const {
        u = abs_fract(u);
        v = 1.0 - abs_fract(v);
        if (!linear_interp) {  // texture.rs:109-118
            uint32_t i = (uint32_t)(u * (double)w);
            uint32_t j = (uint32_t)(v * (double)h);
            return pixel_data(i, j);
        }
        double x = u * (double)w - 0.5, y = v * (double)h - 0.5;  // texture.rs:120-153
        uint32_t x0 = (uint32_t)std::fmax(std::floor(x), 0.0);
        uint32_t y0 = (uint32_t)std::fmax(std::floor(y), 0.0);
        uint32_t x1 = std::min<uint32_t>(x0 + 1, (uint32_t)w - 1);
        uint32_t y1 = std::min<uint32_t>(y0 + 1, (uint32_t)h - 1);
        double dx = x - (double)x0, dy = y - (double)y0;
        auto p00 = pixel_data(x0, y0), p10 = pixel_data(x1, y0), p01 = pixel_data(x0, y1), p11 = pixel_data(x1, y1);
        std::array<float, 4> r{};
        for (int i = 0; i < 4; ++i) {
            float v0 = p00[i] * (1.0f - (float)dx) + p10[i] * (float)dx;
            float v1 = p01[i] * (1.0f - (float)dx) + p11[i] * (float)dx;
            r[i] = v0 * (1.0f - (float)dy) + v1 * (float)dy;
        }
        return r;
    }
    Color value(double u, double v, const Point3&) const override {
        if (h == 0) return Color(0.0, 1.0, 1.0);
        auto p = get_pixel(u, v);
        return Color((double)p[0], (double)p[1], (double)p[2]);
    }
    double alpha(double u, double v) const {  // texture.rs:99-106
        if (h == 0) return 1.0;
        return (double)get_pixel(u, v)[3];
    }
};
// src/utils/perlin.rs:8-108; tables from SplitMix64(seed) in the reference's draw order.
struct Perlin {
    Vec3 randvec[256];
    int perm_x[256], perm_y[256], perm_z[256];
    explicit Perlin(uint64_t seed);
    double noise(const Point3& p) const;
    double turb(const Point3& p, int depth) const;
};
struct NoiseTexture : Texture {  // texture.rs:177-196
    Perlin noise;
    double scale;
    NoiseTexture(double s, uint64_t seed) : noise(seed), scale(s) {}
    Color value(double, double, const Point3& p) const override {
        return Color(0.5, 0.5, 0.5) * (1.0 + m::sin(scale * p.z() + 10.0 * noise.turb(p, 7)));
    }
};

// ---------------------------------------------------------------- Hit record
struct Material;
// src/hit.rs:11-43
struct HitRecord {
    Point3 p;
    Vec3 normal;
    const Material* mat = nullptr;
    double t = 0.0, u = 0.0, v = 0.0;
    bool front_face = false;
    static HitRecord make(const Point3& p, const Vec3& n, const Material* m, double t, double u, double v,
                          const Ray& r_in) {
        HitRecord h;
        h.front_face = r_in.dir.dot(n) < 0.0;
        h.p = p;
        h.normal = h.front_face ? n : -n;
        h.mat = m;
        h.t = t;
        h.u = u;
        h.v = v;
        return h;
    }
};

// ---------------------------------------------------------------- PDFs
// src/pdf.rs:13-16
struct PDF {
    virtual ~PDF() = default;
    virtual std::pair<Color, double> value(const Vec3& direction) const = 0;
    virtual std::optional<Vec3> generate() const = 0;
};
struct SpherePDF : PDF {  // pdf.rs:18-34
    Color attenuation;
    explicit SpherePDF(const Color& a) : attenuation(a) {}
    std::pair<Color, double> value(const Vec3&) const override {
        return {attenuation / (4.0 * PI), 1.0 / (4.0 * PI)};
    }
    std::optional<Vec3> generate() const override { return random_unit_vector(); }
};
struct CosinePDF : PDF {  // pdf.rs:36-64
    Color attenuation;
    ONB uvw;
    CosinePDF(const Color& a, const Vec3& w) : attenuation(a), uvw(w) {}
    std::pair<Color, double> value(const Vec3& direction) const override {
        auto u = from_vec3(direction);
        if (!u) throw Panic("CosinePDF::value unwrap on non-normalizable direction");
        double c = u->dot(uvw.v());
        double pdf = std::fmax(0.0, c / PI);
        Color brdf = attenuation * std::fmax(c, 0.0) / PI;
        return {brdf, pdf};
    }
    std::optional<Vec3> generate() const override { return uvw.onb_to_world(random_cosine_direction()); }
};
struct Hittable;
struct HittablePDF : PDF {  // pdf.rs:66-88
    const Hittable* objects;
    Point3 origin;
    HittablePDF(const Hittable* o, const Point3& p) : objects(o), origin(p) {}
    std::pair<Color, double> value(const Vec3& direction) const override;
    std::optional<Vec3> generate() const override;
};
struct MixturePDF : PDF {  // pdf.rs:90-120
    const PDF* p0;
    const PDF* p1;
    MixturePDF(const PDF* a, const PDF* b) : p0(a), p1(b) {}
    std::pair<Color, double> value(const Vec3& direction) const override {
        auto [att, v0] = p0->value(direction);
        auto v1 = p1->value(direction).second;
        if (v0 == 0.0 && v1 == 0.0) throw Panic("MixturePDF: both pdf values are 0");
        return {att, v0 * 0.5 + v1 * 0.5};
    }
    std::optional<Vec3> generate() const override {
        if (Random::f64() < 0.5) return p0->generate();
        return p1->generate();
    }
};

// ---------------------------------------------------------------- Materials
// src/material.rs:18-34
struct ScatterRecord {
    std::unique_ptr<PDF> pdf;  // ScatterRecord::PDF
    Color attenuation;         // ScatterRecord::Ray
    Ray ray;
    bool is_pdf() const { return (bool)pdf; }
};
struct Material {
    virtual ~Material() = default;
    virtual std::optional<ScatterRecord> scatter(const Ray&, const HitRecord&) const { return std::nullopt; }
    virtual Color emitted(const Ray&, const HitRecord&) const { return Color(); }
};
inline ScatterRecord pdf_record(std::unique_ptr<PDF> p) {
    ScatterRecord s;
    s.pdf = std::move(p);
    return s;
}
inline ScatterRecord ray_record(const Color& a, const Ray& r) {
    ScatterRecord s;
    s.attenuation = a;
    s.ray = r;
    return s;
}
struct EmptyMaterial : Material {  // material.rs:36-47
    std::optional<ScatterRecord> scatter(const Ray&, const HitRecord& rec) const override {
        return pdf_record(std::make_unique<CosinePDF>(Color(0.75, 0.75, 0.75), rec.normal));
    }
};
struct Lambertian : Material {  // material.rs:49-66
    std::shared_ptr<Texture> texture;
    explicit Lambertian(std::shared_ptr<Texture> t) : texture(std::move(t)) {}
    std::optional<ScatterRecord> scatter(const Ray&, const HitRecord& rec) const override {
        ORC_COUNT(lambert);
        Color albedo = texture->value(rec.u, rec.v, rec.p);
        return pdf_record(std::make_unique<CosinePDF>(albedo, rec.normal));
    }
};
struct Metal : Material {  // material.rs:68-95
    Color albedo;
    double fuzz;
    Metal(const Color& a, double f) : albedo(a), fuzz(std::clamp(f, 0.0, 1.0)) {}
    std::optional<ScatterRecord> scatter(const Ray& r_in, const HitRecord& rec) const override {
        ORC_COUNT(metal);
        auto ud = from_vec3(r_in.dir);
        if (!ud) return std::nullopt;
        Vec3 raw_reflected = ud->reflect(rec.normal);
        auto rr = from_vec3(raw_reflected);
        if (!rr) return std::nullopt;
        Vec3 reflected = *rr + fuzz * random_unit_vector();
        return ray_record(albedo, Ray(rec.p, reflected, r_in.time));
    }
};
struct Dielectric : Material {  // material.rs:97-144
    std::shared_ptr<Texture> attenuation;
    double refraction_index;
    Dielectric(std::shared_ptr<Texture> t, double ior) : attenuation(std::move(t)), refraction_index(ior) {}
    static double reflectance(double cosine, double ri) {  // material.rs:110-114 (powi(5) = x*(x^2)^2)
        double r0 = (1.0 - ri) / (1.0 + ri);
        double r0sq = r0 * r0;
        double x = 1.0 - cosine;
        double x2 = x * x;
        double x5 = x * (x2 * x2);
        return r0sq + (1.0 - r0sq) * x5;
    }
    std::optional<ScatterRecord> scatter(const Ray& r_in, const HitRecord& rec) const override {
        ORC_COUNT(dielectric);
        double ri = rec.front_face ? 1.0 / refraction_index : refraction_index;
        Vec3 ud = expect_unit(r_in.dir, "Dielectric unwrap");
        double cos_theta = std::fmin((-ud).dot(rec.normal), 1.0);
        double sin_theta = std::sqrt(1.0 - cos_theta * cos_theta);
        bool cannot_refract = ri * sin_theta > 1.0;
        Vec3 direction;
        if (cannot_refract || reflectance(cos_theta, ri) > Random::f64()) {
            direction = ud.reflect(rec.normal);
        } else {
            auto d = refract(ud, rec.normal, ri);
            if (!d) throw Panic("Dielectric refract unwrap");
            direction = *d;
        }
        return ray_record(attenuation->value(rec.u, rec.v, rec.p), Ray(rec.p, direction, r_in.time));
    }
};
struct DiffuseLight : Material {  // material.rs:146-186
    std::shared_ptr<Texture> texture;
    std::shared_ptr<Material> material;
    explicit DiffuseLight(std::shared_ptr<Texture> t, std::shared_ptr<Material> m = nullptr)
        : texture(std::move(t)), material(std::move(m)) {}
    Color emitted(const Ray& ray, const HitRecord& rec) const override {
        Color self_emit = texture->value(rec.u, rec.v, rec.p);
        Color mat_emit = material ? material->emitted(ray, rec) : Color();
        return self_emit + mat_emit;
    }
    std::optional<ScatterRecord> scatter(const Ray& r_in, const HitRecord& rec) const override {
        if (material) return material->scatter(r_in, rec);
        return std::nullopt;
    }
};
struct Isotropic : Material {  // material.rs:188-207
    std::shared_ptr<Texture> texture;
    explicit Isotropic(std::shared_ptr<Texture> t) : texture(std::move(t)) {}
    std::optional<ScatterRecord> scatter(const Ray&, const HitRecord& rec) const override {
        ORC_COUNT(isotropic);
        Color albedo = texture->value(rec.u, rec.v, rec.p);
        return pdf_record(std::make_unique<SpherePDF>(albedo));
    }
};
struct Transparent : Material {  // material.rs:209-218
    std::optional<ScatterRecord> scatter(const Ray& r_in, const HitRecord& rec) const override {
        return ray_record(Color(1.0, 1.0, 1.0), Ray(rec.p, r_in.dir, r_in.time));
    }
};
struct Mix : Material {  // material.rs:220-268: Mix::new (constant) or Mix::from_image (alpha)
    std::shared_ptr<Material> mat1, mat2;
    double ratio;
    std::shared_ptr<ImageTexture> ratio_tex;  // Mix::from_image (material.rs:235-247), else null
    Mix(std::shared_ptr<Material> a, std::shared_ptr<Material> b, double r)
        : mat1(std::move(a)), mat2(std::move(b)), ratio(r) {}
    Mix(std::shared_ptr<Material> a, std::shared_ptr<Material> b, std::shared_ptr<ImageTexture> t)
        : mat1(std::move(a)), mat2(std::move(b)), ratio(0.0), ratio_tex(std::move(t)) {}
    double get_ratio(const HitRecord& rec) const {  // material.rs:249-251
        return ratio_tex ? ratio_tex->alpha(rec.u, rec.v) : ratio;
    }
    std::optional<ScatterRecord> scatter(const Ray& r_in, const HitRecord& rec) const override {
        const double r = get_ratio(rec);
        if (Random::f64() > r) return mat1->scatter(r_in, rec);
        return mat2->scatter(r_in, rec);
    }
    Color emitted(const Ray& r_in, const HitRecord& rec) const override {
        const double r = get_ratio(rec);
        return mat1->emitted(r_in, rec) * (1.0 - r) + mat2->emitted(r_in, rec) * r;
    }
};

// shapes/obj.rs:20-81 -- the per-triangle wrapper of an OBJ mesh (no normal
// map: normal_tex = None).  remap_record replaces the normal by the normalised
// barycentric mix of the vertex normals (not face-flipped) and (u, v) by the
// interpolated texture coordinates; p, t, front_face are kept.
struct RemappedMaterial : Material {
    std::shared_ptr<Material> material;
    Vec3 tex_ori, tex_u, tex_v;  // z = 0 (get_two_values, obj.rs:112-115)
    std::optional<Vec3> u_vec, v_vec;
    Vec3 normal[3];
    std::shared_ptr<Texture> normal_tex;  // None = null
    HitRecord remap_record(const HitRecord& rec) const {
        Vec3 tex_coord = tex_ori + rec.u * tex_u + rec.v * tex_v;
        Vec3 n = expect_unit((1.0 - rec.u - rec.v) * normal[0] + rec.u * normal[1] + rec.v * normal[2],
                             "called `Option::unwrap()` on a `None` value (obj.rs:40)");
        if (normal_tex) {
            Vec3 normal_color = normal_tex->value(tex_coord.e[0], tex_coord.e[1], rec.p);
            normal_color = normal_color * 2.0 - Vec3(1.0, 1.0, 1.0);
            if (!u_vec || !v_vec) throw Panic("called `Option::unwrap()` on a `None` value (obj.rs:47)");
            Vec3 normal_raw = *u_vec * normal_color.e[0] + *v_vec * normal_color.e[1] + n * normal_color.e[2];
            n = expect_unit(normal_raw, "The mapped normal can't normalized!");
        }
        HitRecord h = rec;
        h.normal = n;
        h.u = tex_coord.e[0];
        h.v = tex_coord.e[1];
        return h;
    }
    std::optional<ScatterRecord> scatter(const Ray& r_in, const HitRecord& rec) const override {
        return material->scatter(r_in, remap_record(rec));
    }
    Color emitted(const Ray& r_in, const HitRecord& rec) const override {
        return material->emitted(r_in, remap_record(rec));
    }
};

// ---------------------------------------------------------------- Hittables
// src/hit.rs:46-60
struct Hittable {
    virtual ~Hittable() = default;
    virtual std::optional<HitRecord> hit(const Ray& r, const Interval& interval) const = 0;
    virtual const AABB& bounding_box() const = 0;
    virtual double pdf_value(const Point3&, const Vec3&) const { throw Panic("pdf_value: unimplemented!()"); }
    virtual Vec3 random(const Point3&) const { throw Panic("random: unimplemented!()"); }
};
using HittablePtr = std::unique_ptr<Hittable>;

struct Hittables : Hittable {  // src/hits.rs:9-76
    std::vector<HittablePtr> objects;
    AABB bbox = AABB();  // Default::default() -> all-zero intervals (hits.rs:9)
    void add(HittablePtr o) {  // hits.rs:27-30
        bbox = bbox.unite(o->bounding_box());
        objects.push_back(std::move(o));
    }
    std::optional<HitRecord> hit(const Ray& r, const Interval& interval) const override;
    const AABB& bounding_box() const override { return bbox; }
    double pdf_value(const Point3& o, const Vec3& d) const override;
    Vec3 random(const Point3& o) const override;
};

struct BVH : Hittable {  // src/bvh.rs:5-90
    HittablePtr left, right;
    AABB bbox;
    static std::unique_ptr<BVH> from_vec(std::vector<HittablePtr> objects);
    std::optional<HitRecord> hit(const Ray& r, const Interval& interval) const override;
    const AABB& bounding_box() const override { return bbox; }
};

struct Sphere : Hittable {  // src/shapes/sphere.rs:17-145
    Ray center;
    double radius;
    std::shared_ptr<Material> mat;
    AABB bbox;
    Sphere(const Point3& c, double r, std::shared_ptr<Material> m);
    Sphere(const Point3& c1, const Point3& c2, double r, std::shared_ptr<Material> m);
    static void get_sphere_uv(const Vec3& p, double& u, double& v);
    std::optional<HitRecord> hit(const Ray& r, const Interval& interval) const override;
    const AABB& bounding_box() const override { return bbox; }
    double pdf_value(const Point3& o, const Vec3& d) const override;
    Vec3 random(const Point3& o) const override;
};

struct Planar : Hittable {  // Quad (shapes/quad.rs:17-126), Triangle (shapes/triangle.rs:16-129)
    Point3 anchor;
    Vec3 u, v, w, normal;
    double parm_d = 0.0, area = 0.0;
    std::shared_ptr<Material> mat;
    AABB bbox;
    bool triangle = false;
    std::optional<HitRecord> hit(const Ray& r, const Interval& interval) const override;
    const AABB& bounding_box() const override { return bbox; }
    double pdf_value(const Point3& o, const Vec3& d) const override;
    Vec3 random(const Point3& o) const override;
};
std::unique_ptr<Planar> make_quad(const Point3& q, const Vec3& u, const Vec3& v, std::shared_ptr<Material> m);
std::unique_ptr<Planar> make_triangle(const Point3& a, const Vec3& u, const Vec3& v, std::shared_ptr<Material> m);
std::unique_ptr<Hittables> build_box(const Point3& a, const Point3& b, std::shared_ptr<Material> m);

struct Transform : Hittable {  // src/shapes.rs:23-133
    HittablePtr object;
    Vec3 offset;
    Quaternion quaternion;
    Vec3 scale;
    AABB bbox;
    Transform(HittablePtr o, const Vec3& off, const Quaternion& q, const Vec3& s);
    Vec3 transform(const Vec3& v) const { return quaternion.rotate_vector(v * scale) + offset; }
    Vec3 detransform(const Vec3& v) const { return quaternion.conjugate().rotate_vector(v - offset) / scale; }
    std::optional<HitRecord> hit(const Ray& r, const Interval& interval) const override;
    const AABB& bounding_box() const override { return bbox; }
    double pdf_value(const Point3& o, const Vec3& d) const override;
    Vec3 random(const Point3& o) const override;
};

struct ConstantMedium : Hittable {  // src/volume.rs:16-78
    HittablePtr boundary;
    double neg_inv_density;
    std::unique_ptr<Isotropic> phase_function;
    uint32_t medium_id;
    ConstantMedium(HittablePtr b, double density, std::shared_ptr<Texture> tex, uint32_t id)
        : boundary(std::move(b)), neg_inv_density(-1.0 / density),
          phase_function(std::make_unique<Isotropic>(std::move(tex))), medium_id(id) {}
    std::optional<HitRecord> hit(const Ray& r, const Interval& interval) const override;
    const AABB& bounding_box() const override { return boundary->bounding_box(); }
};

// ---------------------------------------------------------------- Camera
// src/camera.rs:45-325
// ---------------------------------------------------------------- OBJ (tobj restated, rt_oracle_obj.cpp)
struct ObjMaterial {  // tobj::Material, the fields obj.rs:212-345 reads
    std::string name;
    bool has_diffuse = false, has_optical_density = false, has_dissolve = false;
    Vec3 diffuse;
    double optical_density = 0.0, dissolve = 1.0;
    std::string diffuse_texture, normal_texture, dissolve_texture;
    std::map<std::string, std::string> unknown_param;
};
struct ObjModel {  // tobj::Model / Mesh (single_index)
    std::string name;
    int material_id = -1;  // None
    std::vector<double> positions, texcoords, normals;
    std::vector<uint32_t> indices;
};
struct ObjFile {
    std::vector<ObjModel> models;
    std::vector<ObjMaterial> materials;
    bool materials_ok = true;
};
ObjFile load_obj_file(const std::string& path);

enum class ToonMap { None = 0, ACES = 1 };
struct Camera {
    double aspect_ratio = 1.0;
    uint32_t image_width = 100;
    size_t samples_per_pixel = 10;
    uint32_t max_depth = 10;
    std::shared_ptr<Texture> background;  // Environment{texture}; null = SolidColor(BLACK)
    double vertical_fov_in_degrees = 90.0;
    Point3 look_from = Point3(0, 0, 0), look_at = Point3(0, 0, -1);
    Vec3 vec_up = Vec3(0, 1, 0);
    double defocus_angle_in_degrees = 0.0, focus_distance = 10.0;
    ToonMap toon_map = ToonMap::None;

    uint32_t image_height = 0, sqrt_spp = 0;
    double recip_sqrt_spp = 0.0, pixel_sample_scale = 0.0;
    Point3 center, pixel00_loc;
    Vec3 pixel_delta_u, pixel_delta_v, axis_u, axis_v, axis_w, defocus_disk_u, defocus_disk_v;

    void initialize();
    Ray get_ray(uint32_t i, uint32_t j, uint32_t s_i, uint32_t s_j) const;
    Color background_value(const Ray& r) const;
    Color ray_color(const Ray& r, uint32_t depth, const Hittable& world, const Hittable* lights) const;
};

// color.rs:14-36
Color aces_tonemap(const Color& c);
void to_rgb(const Color& c, ToonMap tm, uint8_t out[3]);

// Renders the frame; linear (pixel_color * pixel_sample_scale) as f64 into
// `linear` (rows*W*3) and the u8 sRGB image into `srgb` (optional).
struct RenderResult {
    uint32_t width = 0, height = 0, rows = 0;
    WorkCounts counts;
    double seconds = 0.0;
};
// Rows y = row_offset + k*row_stride only, written compact (k-th row at k).
// partials (optional, test tooling): the sum over s_j of ray_color for each
// (pixel, stratum row s_i), [rows*W][sqrt_spp][3] -- the GPU's per-item sums.
RenderResult render(Camera& cam, const Hittable& world, const Hittable* lights, uint64_t seed, int threads,
                    std::vector<double>& linear, std::vector<uint8_t>* srgb, uint32_t row_offset = 0,
                    uint32_t row_stride = 1, std::vector<double>* partials = nullptr);

}  // namespace orc
