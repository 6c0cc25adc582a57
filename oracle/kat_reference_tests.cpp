// oracle/kat_reference_tests.cpp -- TEST INFRASTRUCTURE ONLY.
//
// The reference's own unit tests (all 34 inline #[cfg(test)] tests of
// src/utils/vec3.rs, src/utils/ray.rs, src/utils/quaternion.rs, src/aabb.rs and
// src/shapes/sphere.rs), restated against the oracle, plus the Random123
// Philox4x32-10 known-answer vectors that pin the RNG contract.  These are the
// only golden vectors the reference holds for this path.
// Prints one "PASS name" / "FAIL name" line per test; exit code = #failures.
#include <cstdio>
#include <sstream>

#include "rt_oracle.hpp"

using namespace orc;

static int g_fail = 0;
#define CHECK(name, cond)                                                   \
    do {                                                                    \
        bool ok_ = (cond);                                                  \
        std::printf("%s %s\n", ok_ ? "PASS" : "FAIL", name);                \
        if (!ok_) ++g_fail;                                                 \
    } while (0)

static bool approx(double a, double b, double eps) { return std::fabs(a - b) < eps; }

// Rust's `{}` Display for f64 prints the shortest round-trip repr.
static std::string rust_display(const Vec3& v) {
    std::ostringstream os;
    os.precision(17);
    auto shortest = [](double x) {
        char buf[64];
        for (int p = 1; p <= 17; ++p) {
            std::snprintf(buf, sizeof buf, "%.*g", p, x);
            if (std::strtod(buf, nullptr) == x) break;
        }
        return std::string(buf);
    };
    return shortest(v[0]) + " " + shortest(v[1]) + " " + shortest(v[2]);
}

int main() {
    // ---- vec3.rs:462-580 (16 tests)
    {
        Vec3 v(1.0, 2.0, 3.0);
        CHECK("vec3::test_new_and_getters", v.x() == 1.0 && v.y() == 2.0 && v.z() == 3.0);
    }
    {
        Vec3 v(1.0, 2.0, 3.0);
        bool ok = v[0] == 1.0 && v[1] == 2.0 && v[2] == 3.0;
        v[0] = 4.0;
        v[1] = 5.0;
        v[2] = 6.0;
        ok = ok && v[0] == 4.0 && v[1] == 5.0 && v[2] == 6.0;
        CHECK("vec3::test_indexing", ok);
    }
    CHECK("vec3::test_negation", -Vec3(1.0, -2.0, 3.0) == Vec3(-1.0, 2.0, -3.0));
    CHECK("vec3::test_add", Vec3(1, 2, 3) + Vec3(4, 5, 6) == Vec3(5, 7, 9));
    {
        Vec3 a(1, 2, 3);
        a += Vec3(4, 5, 6);
        CHECK("vec3::test_add_assign", a == Vec3(5, 7, 9));
    }
    CHECK("vec3::test_sub", Vec3(1, 2, 3) - Vec3(4, 5, 6) == Vec3(-3, -3, -3));
    CHECK("vec3::test_mul_scalar", Vec3(1, 2, 3) * 2.0 == Vec3(2, 4, 6) && 2.0 * Vec3(1, 2, 3) == Vec3(2, 4, 6));
    {
        Vec3 a(1, 2, 3);
        a = a * 2.0;  // MulAssign<f64>
        CHECK("vec3::test_mul_assign_scalar", a == Vec3(2, 4, 6));
    }
    CHECK("vec3::test_mul_vec", Vec3(1, 2, 3) * Vec3(4, 5, 6) == Vec3(4, 10, 18));
    CHECK("vec3::test_div_scalar", Vec3(2, 4, 6) / 2.0 == Vec3(1, 2, 3));
    {
        Vec3 a(2, 4, 6);
        a = (1.0 / 2.0) * a;  // DivAssign: *self *= 1.0 / rhs
        CHECK("vec3::test_div_assign_scalar", a == Vec3(1, 2, 3));
    }
    {
        Vec3 v(3, 4, 0);
        CHECK("vec3::test_length", v.length_squared() == 25.0 && v.length() == 5.0);
    }
    CHECK("vec3::test_dot_product", Vec3(1, 2, 3).dot(Vec3(4, 5, 6)) == 32.0);
    CHECK("vec3::test_cross_product", Vec3(1, 2, 3).cross(Vec3(4, 5, 6)) == Vec3(-3, 6, -3));
    {
        auto u = from_vec3(Vec3(0, 5, 0));
        auto e = from_vec3(Vec3(0, 1, 0));
        CHECK("vec3::test_unit_vector", u && e && *u == *e && std::fabs(u->length() - 1.0) < 2.220446049250313e-16);
    }
    CHECK("vec3::test_display", rust_display(Vec3(1.1, 2.2, 3.3)) == "1.1 2.2 3.3");

    // ---- ray.rs:48-71 (3 tests)
    {
        Ray r(Point3(1, 2, 3), Vec3(4, 5, 6));
        CHECK("ray::test_new_ray", r.orig == Point3(1, 2, 3) && r.dir == Vec3(4, 5, 6));
        CHECK("ray::test_ray_at", r.at(2.0) == Point3(9, 12, 15));
        Ray d;
        CHECK("ray::test_default_ray", d.orig == Point3() && d.dir == Vec3());
    }

    // ---- quaternion.rs:114-183 (6 tests)
    {
        Quaternion q = Quaternion::identity();
        CHECK("quaternion::test_identity_quaternion", q.w == 1.0 && q.x == 0.0 && q.y == 0.0 && q.z == 0.0);
    }
    {
        Quaternion q = Quaternion::from_euler(1.0, 0.5, -0.3);
        double y, p, r;
        q.to_euler(y, p, r);
        CHECK("quaternion::test_from_euler_and_to_euler",
              approx(y, 1.0, 1e-10) && approx(p, 0.5, 1e-10) && approx(r, -0.3, 1e-10));
    }
    {
        Quaternion q = Quaternion::from_axis_angle(Vec3(1, 0, 0), 90.0);
        Vec3 r = q.rotate_vector(Vec3(0, 1, 0));
        CHECK("quaternion::test_from_axis_angle_90deg_x",
              approx(r.x(), 0, 1e-10) && approx(r.y(), 0, 1e-10) && approx(r.z(), 1, 1e-10));
    }
    {
        Quaternion q1 = Quaternion::from_axis_angle(Vec3(0, 0, 1), 90.0);
        Quaternion q2 = Quaternion::from_axis_angle(Vec3(1, 0, 0), 90.0);
        Vec3 r = (q1 * q2).rotate_vector(Vec3(0, 0, 1));
        CHECK("quaternion::test_quaternion_multiplication",
              approx(r.x(), 1, 1e-10) && approx(r.y(), 0, 1e-10) && approx(r.z(), 0, 1e-10));
    }
    {
        Quaternion q{1, 2, 3, 4};
        Quaternion c = q.conjugate();
        CHECK("quaternion::test_conjugate", c.w == 1 && c.x == -2 && c.y == -3 && c.z == -4);
    }
    {
        Vec3 v(1, 2, 3);
        Vec3 r = Quaternion::identity().rotate_vector(v);
        CHECK("quaternion::test_rotate_vector_identity",
              approx(r.x(), 1, 1e-10) && approx(r.y(), 2, 1e-10) && approx(r.z(), 3, 1e-10));
    }

    // ---- aabb.rs:180-261 (8 tests)
    {
        Interval x = Interval::make(1, 2), y = Interval::make(3, 4), z = Interval::make(5, 6);
        AABB b = AABB::make(x, y, z);
        CHECK("aabb::test_new_and_axis_interval", b.axis_interval(0) == x && b.axis_interval(1) == y && b.axis_interval(2) == z);
    }
    {
        bool panicked = false;
        try {
            AABB().axis_interval(3);
        } catch (const Panic&) {
            panicked = true;
        }
        CHECK("aabb::test_axis_interval_panic", panicked);
    }
    {
        AABB b = AABB::from_points(Point3(1, 2, 3), Point3(4, 5, 6));
        CHECK("aabb::test_from_points", b.x.min == 1 && b.x.max == 4 && b.y.min == 2 && b.y.max == 5 && b.z.min == 3 && b.z.max == 6);
    }
    {
        AABB b = AABB::from_points(Point3(0, 0, 0), Point3(1, 1, 1));
        CHECK("aabb::test_hit_inside", b.hit(Ray(Point3(0.5, 0.5, -1), Vec3(0, 0, 1)), Interval::make(0, 100)));
        CHECK("aabb::test_hit_outside", !b.hit(Ray(Point3(2, 2, 2), Vec3(1, 0, 0)), Interval::make(0, 100)));
    }
    CHECK("aabb::test_longest_axis", AABB::from_points(Point3(0, 0, 0), Point3(2, 1, 1)).longest_axis() == 0 &&
                                         AABB::from_points(Point3(0, 0, 0), Point3(1, 3, 1)).longest_axis() == 1 &&
                                         AABB::from_points(Point3(0, 0, 0), Point3(1, 1, 4)).longest_axis() == 2);
    {
        AABB u = AABB::from_points(Point3(0, 0, 0), Point3(1, 1, 1)).unite(AABB::from_points(Point3(1, 1, 1), Point3(2, 2, 2)));
        CHECK("aabb::test_union", u.x.min == 0 && u.x.max == 2 && u.y.min == 0 && u.y.max == 2 && u.z.min == 0 && u.z.max == 2);
    }
    {
        AABB u = AABB::universe();
        CHECK("aabb::test_empty_and_universe", u.x.contains(0.0) && u.y.contains(1e10) && u.z.contains(-1e10));
    }

    // ---- sphere.rs:151-170 (1 test, 6 points)
    {
        struct {
            Vec3 p;
            double u, v;
        } pts[] = {{Vec3(1, 0, 0), 0.5, 0.5},  {Vec3(-1, 0, 0), 0.0, 0.5}, {Vec3(0, 1, 0), 0.5, 1.0},
                   {Vec3(0, -1, 0), 0.5, 0.0}, {Vec3(0, 0, 1), 0.25, 0.5}, {Vec3(0, 0, -1), 0.75, 0.5}};
        bool ok = true;
        for (auto& t : pts) {
            double u, v;
            Sphere::get_sphere_uv(t.p, u, v);
            ok = ok && u == t.u && v == t.v;
        }
        CHECK("sphere::test_sphere_uv", ok);
    }

    // ---- Random123 Philox4x32-10 known-answer vectors (kat_vectors, philox4x32_10)
    {
        struct {
            uint32_t ctr[4], key[2], out[4];
        } kats[] = {
            {{0, 0, 0, 0}, {0, 0}, {0x6627e8d5u, 0xe169c58du, 0xbc57ac4cu, 0x9b00dbd8u}},
            {{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}, {0xffffffffu, 0xffffffffu},
             {0x408f276du, 0x41c83b0eu, 0xa20bc7c6u, 0x6d5451fdu}},
            {{0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u}, {0xa4093822u, 0x299f31d0u},
             {0xd16cfe09u, 0x94fdccebu, 0x5001e420u, 0x24126ea1u}},
        };
        bool ok = true;
        for (auto& k : kats) {
            uint32_t o[4];
            philox4x32_10(k.ctr, k.key, o);
            ok = ok && o[0] == k.out[0] && o[1] == k.out[1] && o[2] == k.out[2] && o[3] == k.out[3];
        }
        CHECK("rng::philox4x32_10_random123_kat", ok);
    }
    std::printf("%d failures\n", g_fail);
    return g_fail;
}
