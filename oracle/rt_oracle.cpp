// oracle/rt_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see rt_oracle.hpp header).
#include "rt_oracle.hpp"

#include <chrono>
#include <thread>

namespace orc {

PathRng*& current_rng() {
    static thread_local PathRng* r = nullptr;
    return r;
}
WorkCounts& work() {
    static thread_local WorkCounts w;
    return w;
}

// ---------------------------------------------------------------- AABB
// aabb.rs:62-78
bool AABB::hit(const Ray& r, Interval ray_t) const {
    for (int axis = 0; axis < 3; ++axis) {
        const Interval& ax = axis_interval(axis);
        double adinv = 1.0 / r.dir[axis];
        double t0 = (ax.min - r.orig[axis]) * adinv;
        double t1 = (ax.max - r.orig[axis]) * adinv;
        auto next = ray_t.intersect(Interval::make(t0, t1));
        if (!next) return false;
        ray_t = *next;
    }
    return true;
}

// ---------------------------------------------------------------- Quaternion
// quaternion.rs:23-38
Quaternion Quaternion::from_euler(double yaw, double pitch, double roll) {
    double cy = std::cos(0.5 * yaw), sy = std::sin(0.5 * yaw);
    double cp = std::cos(0.5 * pitch), sp = std::sin(0.5 * pitch);
    double cr = std::cos(0.5 * roll), sr = std::sin(0.5 * roll);
    return Quaternion{cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                      cr * cp * sy - sr * sp * cy};
}
// quaternion.rs:40-53
Quaternion Quaternion::from_axis_angle(const Vec3& axis, double deg) {
    double half = deg * (PI / 180.0) * 0.5;  // f64::to_radians = self * (PI/180)
    double s = std::sin(half), c = std::cos(half);
    Vec3 a = expect_unit(axis, "Quaternion axis unwrap");
    return Quaternion{c, a.x() * s, a.y() * s, a.z() * s};
}
// quaternion.rs:55-70
void Quaternion::to_euler(double& yaw, double& pitch, double& roll) const {
    double sinr_cosp = 2.0 * (w * x + y * z);
    double cosr_cosp = 1.0 - 2.0 * (x * x + y * y);
    roll = std::atan2(sinr_cosp, cosr_cosp);
    double sinp = 2.0 * (w * y - z * x);
    pitch = std::fabs(sinp) >= 1.0 ? std::copysign(PI / 2.0, sinp) : std::asin(sinp);
    double siny_cosp = 2.0 * (w * z + x * y);
    double cosy_cosp = 1.0 - 2.0 * (y * y + z * z);
    yaw = std::atan2(siny_cosp, cosy_cosp);
}

// ---------------------------------------------------------------- Perlin
// perlin.rs:16-36 (Default): 256 random_unit_vector (2 draws each), then three
// permutations, each a Fisher-Yates from the top with usize(0..=i).
Perlin::Perlin(uint64_t seed) {
    SplitMix64 g(seed);
    for (int i = 0; i < 256; ++i) {
        double r1 = g.next_f64(), r2 = g.next_f64();
        // host-side construction: glibc in both builds, as the product library's scene builder
        double x = std::cos(2.0 * PI * r1) * 2.0 * std::sqrt(r2 * (1.0 - r2));
        double y = std::sin(2.0 * PI * r1) * 2.0 * std::sqrt(r2 * (1.0 - r2));
        double z = 1.0 - 2.0 * r2;
        randvec[i] = Vec3(x, y, z);
    }
    int* perms[3] = {perm_x, perm_y, perm_z};
    for (int* p : perms) {
        for (int i = 0; i < 256; ++i) p[i] = i;
        for (int i = 255; i >= 1; --i) {
            int target = (int)(g.next_f64() * (double)(i + 1));
            if (target > i) target = i;
            std::swap(p[i], p[target]);
        }
    }
}
// perlin.rs:40-58 + 74-89
double Perlin::noise(const Point3& p) const {
    int64_t i = (int64_t)std::floor(p.x()), j = (int64_t)std::floor(p.y()), k = (int64_t)std::floor(p.z());
    double u = p.x() - std::floor(p.x()), v = p.y() - std::floor(p.y()), w = p.z() - std::floor(p.z());
    double uu = u * u * (3.0 - 2.0 * u), vv = v * v * (3.0 - 2.0 * v), ww = w * w * (3.0 - 2.0 * w);
    double accum = 0.0;
    for (int di = 0; di < 2; ++di)
        for (int dj = 0; dj < 2; ++dj)
            for (int dk = 0; dk < 2; ++dk) {
                const Vec3& c = randvec[perm_x[(size_t)(i + di) & 255] ^ perm_y[(size_t)(j + dj) & 255] ^
                                        perm_z[(size_t)(k + dk) & 255]];
                Vec3 weight_v(u - di, v - dj, w - dk);
                accum += (di * uu + (1 - di) * (1.0 - uu)) * (dj * vv + (1 - dj) * (1.0 - vv)) *
                         (dk * ww + (1 - dk) * (1.0 - ww)) * c.dot(weight_v);
            }
    return accum;
}
// perlin.rs:60-72
double Perlin::turb(const Point3& p, int depth) const {
    double accum = 0.0, weight = 1.0;
    Point3 tp = p;
    for (int i = 0; i < depth; ++i) {
        accum += weight * noise(tp);
        tp = 2.0 * tp;
        weight = 0.5 * weight;
    }
    return std::fabs(accum);
}

// ---------------------------------------------------------------- PDFs
// pdf.rs:77-87
std::pair<Color, double> HittablePDF::value(const Vec3& direction) const {
    ORC_COUNT(light_pdf);
    return {Color(), objects->pdf_value(origin, direction)};
}
std::optional<Vec3> HittablePDF::generate() const { return objects->random(origin); }

// ---------------------------------------------------------------- Hittables
// hits.rs:34-46: every object with the unchanged interval, min_by(t) (first minimum)
std::optional<HitRecord> Hittables::hit(const Ray& r, const Interval& interval) const {
    std::optional<HitRecord> best;
    for (const auto& o : objects) {
        auto rec = o->hit(r, interval);
        if (!rec) continue;
        if (!best) {
            best = rec;
            continue;
        }
        if (std::isnan(rec->t) || std::isnan(best->t)) throw Panic("The length of ray should not be NaN!");
        if (rec->t < best->t) best = rec;
    }
    return best;
}
// hits.rs:52-67
double Hittables::pdf_value(const Point3& o, const Vec3& d) const {
    double sum = 0.0;
    for (const auto& ob : objects) sum += ob->pdf_value(o, d);
    double ret = sum / (double)objects.size();
    if (std::isnan(ret)) throw Panic("The sum of pdf is NaN!");
    return ret;
}
// hits.rs:69-75
Vec3 Hittables::random(const Point3& o) const {
    if (objects.empty()) throw Panic("The collection of objects is empty!");
    return objects[Random::index(objects.size())]->random(o);
}

// ---------------------------------------------------------------- BVH
// bvh.rs:16-46 (+ box_compare 48-54: total_cmp on bbox.axis_interval(axis).min)
static bool total_less(double a, double b) {
    int64_t ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    ia ^= (int64_t)(((uint64_t)(ia >> 63)) >> 1);
    ib ^= (int64_t)(((uint64_t)(ib >> 63)) >> 1);
    return ia < ib;
}
std::unique_ptr<BVH> BVH::from_vec(std::vector<HittablePtr> objects) {
    auto node = std::make_unique<BVH>();
    AABB bbox = AABB::empty();
    for (const auto& o : objects) bbox = bbox.unite(o->bounding_box());
    int axis = bbox.longest_axis();
    size_t len = objects.size();
    if (len == 0) throw Panic("BVH node must contain at least one object");
    if (len == 1) {
        node->left = std::move(objects[0]);
    } else if (len == 2) {
        node->left = std::move(objects[0]);
        node->right = std::move(objects[1]);
    } else {
        // Rust slice::sort_by is stable
        std::stable_sort(objects.begin(), objects.end(), [axis](const HittablePtr& a, const HittablePtr& b) {
            return total_less(a->bounding_box().axis_interval(axis).min, b->bounding_box().axis_interval(axis).min);
        });
        size_t mid = len / 2;
        std::vector<HittablePtr> right_vec, left_vec;
        for (size_t i = 0; i < mid; ++i) left_vec.push_back(std::move(objects[i]));
        for (size_t i = mid; i < len; ++i) right_vec.push_back(std::move(objects[i]));
        node->left = BVH::from_vec(std::move(left_vec));
        node->right = BVH::from_vec(std::move(right_vec));
    }
    node->bbox = bbox;
    return node;
}
// bvh.rs:57-85
std::optional<HitRecord> BVH::hit(const Ray& r, const Interval& interval) const {
    ORC_COUNT(bvh_node_tests);
    if (!bbox.hit(r, interval)) return std::nullopt;
    std::optional<HitRecord> hit_left;
    double closest_so_far = interval.max;
    if (left) {
        hit_left = left->hit(r, interval);
        if (hit_left) closest_so_far = hit_left->t;
    }
    std::optional<HitRecord> hit_right;
    if (right) hit_right = right->hit(r, Interval::make(interval.min, closest_so_far));
    return hit_right ? hit_right : hit_left;
}

// ---------------------------------------------------------------- Sphere
// sphere.rs:25-35
Sphere::Sphere(const Point3& c, double r, std::shared_ptr<Material> m)
    : center(c, Vec3(0, 0, 0)), radius(std::fmax(0.0, r)), mat(std::move(m)) {
    Vec3 rvec(r, r, r);
    bbox = AABB::from_points(c - rvec, c + rvec);
}
// sphere.rs:37-51
Sphere::Sphere(const Point3& c1, const Point3& c2, double r, std::shared_ptr<Material> m)
    : center(c1, c2 - c1), radius(std::fmax(0.0, r)), mat(std::move(m)) {
    Vec3 rvec(r, r, r);
    AABB box1 = AABB::from_points(center.at(0.0) - rvec, center.at(0.0) + rvec);
    AABB box2 = AABB::from_points(center.at(1.0) - rvec, center.at(1.0) + rvec);
    bbox = box1.unite(box2);
}
// sphere.rs:53-61
void Sphere::get_sphere_uv(const Vec3& p, double& u, double& v) {
    double theta = m::acos(-p.y());
    double phi = m::atan2(-p.z(), p.x()) + PI;
    u = phi / (2.0 * PI);
    v = theta / PI;
}
// sphere.rs:77-108
std::optional<HitRecord> Sphere::hit(const Ray& r, const Interval& interval) const {
    ORC_COUNT(sphere_tests);
    Point3 current_center = center.at(r.time);
    Vec3 oc = current_center - r.orig;
    double a = r.dir.length_squared();
    double h = r.dir.dot(oc);
    double c = oc.length_squared() - radius * radius;
    double discriminant = h * h - a * c;
    if (discriminant < 0.0) return std::nullopt;
    ORC_COUNT(sphere_disc_ok);
    double sqrtd = std::sqrt(discriminant);
    double root = (h - sqrtd) / a;
    if (!interval.contains(root)) {
        root = (h + sqrtd) / a;
        if (!interval.contains(root)) return std::nullopt;
    }
    ORC_COUNT(sphere_records);
    Point3 p = r.at(root);
    Vec3 outward_normal = (p - current_center) / radius;
    double u, v;
    get_sphere_uv(outward_normal, u, v);
    return HitRecord::make(p, outward_normal, mat.get(), root, u, v, r);
}
// sphere.rs:114-132
double Sphere::pdf_value(const Point3& o, const Vec3& d) const {
    if (!hit(Ray(o, d), Interval::make(1e-8, INF))) return 0.0;
    double dist_squared = (center.at(0.0) - o).length_squared();
    double cos_theta_max = std::sqrt(1.0 - radius * radius / dist_squared);
    if (std::isnan(cos_theta_max)) return 1.0 / (4.0 * PI);
    double solid_angle = 2.0 * PI * (1.0 - cos_theta_max);
    return 1.0 / solid_angle;
}
// sphere.rs:134-144 + random_to_sphere 63-74
Vec3 Sphere::random(const Point3& o) const {
    Vec3 direction = center.at(0.0) - o;
    double distance_squared = direction.length_squared();
    ONB uvw(expect_unit(direction, "The direction should be normalizable!"));
    double r1 = Random::f64();
    double r2 = Random::f64();
    double y = 1.0 + r2 * (std::sqrt(1.0 - radius * radius / distance_squared) - 1.0);
    double phi = 2.0 * PI * r1;
    double x = m::cos(phi) * std::sqrt(1.0 - y * y);
    double z = m::sin(phi) * std::sqrt(1.0 - y * y);
    return expect_unit(uvw.onb_to_world(Vec3(x, y, z)), "sphere random unwrap");
}

// ---------------------------------------------------------------- Quad / Triangle
// quad.rs:30-47
std::unique_ptr<Planar> make_quad(const Point3& q, const Vec3& u, const Vec3& v, std::shared_ptr<Material> m) {
    auto s = std::make_unique<Planar>();
    Vec3 n = u.cross(v);
    s->normal = expect_unit(n, "The length of normal should be normalizable!");
    s->parm_d = s->normal.dot(q);
    s->w = n / n.length_squared();
    s->area = n.length();
    s->anchor = q;
    s->u = u;
    s->v = v;
    s->mat = std::move(m);
    // quad.rs:50-55
    AABB d1 = AABB::from_points(q, q + u + v);
    AABB d2 = AABB::from_points(q + u, q + v);
    s->bbox = d1.unite(d2);
    s->triangle = false;
    return s;
}
// triangle.rs:28-46 (None when degenerate)
std::unique_ptr<Planar> make_triangle(const Point3& a, const Vec3& u, const Vec3& v, std::shared_ptr<Material> m) {
    Vec3 n = u.cross(v);
    auto normal = from_vec3(n);
    if (!normal) return nullptr;
    auto s = std::make_unique<Planar>();
    s->normal = *normal;
    s->parm_d = s->normal.dot(a);
    s->w = n / n.length_squared();
    s->area = n.length() / 2.0;
    s->anchor = a;
    s->u = u;
    s->v = v;
    s->mat = std::move(m);
    // triangle.rs:49-54
    AABB b1 = AABB::from_points(a, a + u);
    AABB b2 = AABB::from_points(a, a + v);
    s->bbox = b1.unite(b2);
    s->triangle = true;
    return s;
}
// quad.rs:71-102 / triangle.rs:69-98
std::optional<HitRecord> Planar::hit(const Ray& r, const Interval& interval) const {
    if (triangle)
        ORC_COUNT(tri_tests);
    else
        ORC_COUNT(quad_tests);
    double denom = normal.dot(r.dir);
    if (std::fabs(denom) < 1e-8) return std::nullopt;
    double t = (parm_d - normal.dot(r.orig)) / denom;
    if (!interval.contains(t)) return std::nullopt;
    Point3 intersection = r.at(t);
    Vec3 hv = intersection - anchor;
    double alpha = w.dot(hv.cross(v));
    double beta = w.dot(u.cross(hv));
    const Interval unit = Interval::make(0.0, 1.0);
    if (triangle) {  // triangle.rs:57-65
        if (!(unit.contains(alpha) && unit.contains(beta) && unit.contains(alpha + beta))) return std::nullopt;
    } else {  // quad.rs:57-67
        if (!unit.contains(alpha) || !unit.contains(beta)) return std::nullopt;
    }
    ORC_COUNT(planar_records);
    return HitRecord::make(intersection, normal, mat.get(), t, alpha, beta, r);
}
// quad.rs:108-120 / triangle.rs:108-120
double Planar::pdf_value(const Point3& o, const Vec3& d) const {
    auto rec = hit(Ray(o, d), Interval::make(1e-8, INF));
    if (!rec) return 0.0;
    double distance_squared = rec->t * rec->t * d.length_squared();
    double cosine = std::fabs(d.dot(rec->normal) / d.length());
    return distance_squared / (cosine * area);
}
// quad.rs:122-125 / triangle.rs:117-128
Vec3 Planar::random(const Point3& o) const {
    double a = Random::f64();
    double b = Random::f64();
    if (triangle && a + b > 1.0) {
        double na = 1.0 - b, nb = 1.0 - a;
        a = na;
        b = nb;
    }
    Point3 p = anchor + (a * u) + (b * v);
    return expect_unit(p - o, "planar random unwrap");
}
// quad.rs:128-189
std::unique_ptr<Hittables> build_box(const Point3& a, const Point3& b, std::shared_ptr<Material> m) {
    auto sides = std::make_unique<Hittables>();
    Point3 mn(std::fmin(a.x(), b.x()), std::fmin(a.y(), b.y()), std::fmin(a.z(), b.z()));
    Point3 mx(std::fmax(a.x(), b.x()), std::fmax(a.y(), b.y()), std::fmax(a.z(), b.z()));
    Vec3 dx(mx.x() - mn.x(), 0.0, 0.0), dy(0.0, mx.y() - mn.y(), 0.0), dz(0.0, 0.0, mx.z() - mn.z());
    sides->add(make_quad(Point3(mn.x(), mn.y(), mx.z()), dx, dy, m));
    sides->add(make_quad(Point3(mx.x(), mn.y(), mx.z()), -dz, dy, m));
    sides->add(make_quad(Point3(mx.x(), mn.y(), mn.z()), -dx, dy, m));
    sides->add(make_quad(Point3(mn.x(), mn.y(), mn.z()), dz, dy, m));
    sides->add(make_quad(Point3(mn.x(), mx.y(), mx.z()), dx, -dz, m));
    sides->add(make_quad(Point3(mn.x(), mn.y(), mn.z()), dx, dz, m));
    return sides;
}

// ---------------------------------------------------------------- Transform
// shapes.rs:31-72
Transform::Transform(HittablePtr o, const Vec3& off, const Quaternion& q, const Vec3& s)
    : object(std::move(o)), offset(off), quaternion(q), scale(s) {
    auto pts = object->bounding_box().all_points();
    Vec3 mn(INF, INF, INF), mx(-INF, -INF, -INF);
    for (const auto& p0 : pts) {
        Vec3 p = transform(p0);
        mn = Vec3(std::fmin(mn.x(), p.x()), std::fmin(mn.y(), p.y()), std::fmin(mn.z(), p.z()));
        mx = Vec3(std::fmax(mx.x(), p.x()), std::fmax(mx.y(), p.y()), std::fmax(mx.z(), p.z()));
    }
    bbox = AABB::from_points(mn, mx);
}
// shapes.rs:87-111
std::optional<HitRecord> Transform::hit(const Ray& r, const Interval& interval) const {
    ORC_COUNT(transform_tests);
    Point3 to = r.at(1.0);
    Point3 lo = detransform(r.orig);
    Point3 lt = detransform(to);
    Ray local(lo, lt - lo, r.time);
    auto rec = object->hit(local, interval);
    if (!rec) return std::nullopt;
    rec->p = transform(rec->p);
    rec->normal = expect_unit(quaternion.rotate_vector(rec->normal / scale),
                              "The transformed normal can't be normalized!");
    return rec;
}
// shapes.rs:117-123
double Transform::pdf_value(const Point3& o, const Vec3& d) const {
    Point3 lo = detransform(o);
    Point3 lt = detransform(o + d);
    return object->pdf_value(lo, lt - lo);
}
// shapes.rs:125-132
Vec3 Transform::random(const Point3& o) const {
    Point3 lo = detransform(o);
    Vec3 ld = object->random(lo);
    Point3 world_to = transform(lo + ld);
    return expect_unit(world_to - o, "Random direction can't be normalized!");
}

// ---------------------------------------------------------------- ConstantMedium
// volume.rs:37-73
std::optional<HitRecord> ConstantMedium::hit(const Ray& r, const Interval& interval) const {
    ORC_COUNT(medium_tests);
    auto rec1 = boundary->hit(r, Interval::universe());
    if (!rec1) return std::nullopt;
    auto rec2 = boundary->hit(r, Interval::make(rec1->t + 0.0001, INF));
    if (!rec2) return std::nullopt;
    double t1 = rec1->t, t2 = rec2->t;
    if (t1 < interval.min) t1 = interval.min;  // clamp_min_assign
    if (t2 > interval.max) t2 = interval.max;  // clamp_max_assign
    if (t1 >= t2) return std::nullopt;
    if (t1 < 0.0) t1 = 0.0;
    double ray_length = r.dir.length();
    double distance_inside_boundary = (t2 - t1) * ray_length;
    PathRng* rng = current_rng();
    if (!rng) throw Panic("medium outside a render path");
    double hit_distance = neg_inv_density * m::log(rng->medium(medium_id));
    if (hit_distance > distance_inside_boundary) return std::nullopt;
    double t = t1 + hit_distance / ray_length;
    Point3 p = r.at(t);
    return HitRecord::make(p, Vec3(1.0, 0.0, 0.0), phase_function.get(), t, 0.0, 0.0, r);
}

// ---------------------------------------------------------------- Camera
// camera.rs:204-245
void Camera::initialize() {
    image_height = (uint32_t)((double)image_width / aspect_ratio);
    if (image_height < 1) image_height = 1;
    sqrt_spp = (uint32_t)std::sqrt((double)samples_per_pixel);
    pixel_sample_scale = 1.0 / (double)(sqrt_spp * sqrt_spp);
    recip_sqrt_spp = 1.0 / (double)sqrt_spp;
    center = look_from;
    double theta = vertical_fov_in_degrees * (PI / 180.0);
    double h = std::tan(theta / 2.0);
    double viewport_height = 2.0 * h * focus_distance;
    double viewport_width = viewport_height * ((double)image_width / (double)image_height);
    axis_w = expect_unit(look_from - look_at, "Camera axis w should be normalizable!");
    axis_u = expect_unit(vec_up.cross(axis_w), "Camera axis u should be normalizable!");
    axis_v = axis_w.cross(axis_u);
    Vec3 viewport_u = viewport_width * axis_u;
    Vec3 viewport_v = viewport_height * (-axis_v);
    pixel_delta_u = viewport_u / (double)image_width;
    pixel_delta_v = viewport_v / (double)image_height;
    Point3 viewport_upper_left = center - focus_distance * axis_w - viewport_u / 2.0 - viewport_v / 2.0;
    pixel00_loc = viewport_upper_left + 0.5 * (pixel_delta_u + pixel_delta_v);
    double defocus_radius = focus_distance * std::tan((defocus_angle_in_degrees / 2.0) * (PI / 180.0));
    defocus_disk_u = axis_u * defocus_radius;
    defocus_disk_v = axis_v * defocus_radius;
}
// camera.rs:247-273
Ray Camera::get_ray(uint32_t i, uint32_t j, uint32_t s_i, uint32_t s_j) const {
    ORC_COUNT(camera_rays);
    double px = (((double)s_i + Random::f64()) * recip_sqrt_spp) - 0.5;
    double py = (((double)s_j + Random::f64()) * recip_sqrt_spp) - 0.5;
    Point3 pixel_sample = pixel00_loc + (((double)i + px) * pixel_delta_u) + (((double)j + py) * pixel_delta_v);
    Point3 ray_origin;
    if (defocus_angle_in_degrees <= 0.0) {
        ray_origin = center;
    } else {
        Vec3 p = random_in_unit_disk();
        ray_origin = center + (p[0] * defocus_disk_u) + (p[1] * defocus_disk_v);
    }
    Vec3 ray_direction = pixel_sample - ray_origin;
    double ray_time = Random::f64();
    return Ray(ray_origin, ray_direction, ray_time);
}
// environment.rs:14-24
Color Camera::background_value(const Ray& r) const {
    Vec3 p = expect_unit(r.dir, "The direction can't be normalized!");
    double theta = m::acos(-p.y());
    double phi = PI - m::atan2(-p.z(), p.x());
    double u = phi / (2.0 * PI);
    double v = theta / PI;
    if (!background) return Color();
    return background->value(u, v, p);
}
// camera.rs:275-325
Color Camera::ray_color(const Ray& r, uint32_t depth, const Hittable& world, const Hittable* lights) const {
    if (depth == 0) return Color();
    ORC_COUNT(ray_color_calls);
    current_rng()->begin_vertex(max_depth - depth + 1);
    auto rec = world.hit(r, Interval::range(1e-8, INF));
    if (!rec) {
        ORC_COUNT(sky_miss);
        return background_value(r);
    }
    ORC_COUNT(emitted);
    Color color_from_emission = rec->mat->emitted(r, *rec);
    auto sr = rec->mat->scatter(r, *rec);
    if (!sr) return color_from_emission;
    Color color_from_scatter;
    if (sr->is_pdf()) {
        std::unique_ptr<HittablePDF> light_ptr;
        std::unique_ptr<MixturePDF> mixed;
        const PDF* mixed_pdf = sr->pdf.get();
        if (lights) {
            light_ptr = std::make_unique<HittablePDF>(lights, rec->p);
            mixed = std::make_unique<MixturePDF>(sr->pdf.get(), light_ptr.get());
            mixed_pdf = mixed.get();
        }
        auto gen = mixed_pdf->generate();
        if (gen) {
            Ray scattered(rec->p, *gen, r.time);
            auto [albedo_x_pscatter, pdf_value] = mixed_pdf->value(scattered.dir);
            if (pdf_value == 0.0) throw Panic("assert_ne!(pdf_value, 0.0)");
            Color sample_color = ray_color(scattered, depth - 1, world, lights);
            color_from_scatter = (albedo_x_pscatter * sample_color) / pdf_value;
        }
    } else {
        color_from_scatter = sr->attenuation * ray_color(sr->ray, depth - 1, world, lights);
    }
    Color ret = color_from_emission + color_from_scatter;
    if (ret.any_nan()) throw Panic("ray_color returned NaN");
    return ret;
}

// color.rs:14-25
Color aces_tonemap(const Color& c) {
    const double A = 2.51, C = 2.43;
    const Vec3 B(0.03, 0.03, 0.03), D(0.59, 0.59, 0.59), E(0.14, 0.14, 0.14);
    Vec3 m = (c * (A * c + B)) / (c * (C * c + D) + E);
    return Vec3(std::clamp(m[0], 0.0, 1.0), std::clamp(m[1], 0.0, 1.0), std::clamp(m[2], 0.0, 1.0));
}
// color.rs:27-36 -- palette Srgb::from_linear (IEC 61966-2-1 OETF) then f64 -> u8
// (round, clamp).  palette is absent here: restated from the standard (parity unpinned).
void to_rgb(const Color& c, ToonMap tm, uint8_t out[3]) {
    if (c.any_nan()) throw Panic("to_rgb NaN");
    Color m = tm == ToonMap::ACES ? aces_tonemap(c) : c;
    for (int i = 0; i < 3; ++i) {
        double x = m[i];
        double s = x <= 0.0031308 ? 12.92 * x : 1.055 * std::pow(x, 1.0 / 2.4) - 0.055;
        double q = std::round(s * 255.0);
        out[i] = (uint8_t)std::clamp(q, 0.0, 255.0);
    }
}

// camera.rs:161-202 -- rayon par_bridge over pixels restated as a dynamic
// pixel-chunk queue over `threads` std::threads.
RenderResult render(Camera& cam, const Hittable& world, const Hittable* lights, uint64_t seed, int threads,
                    std::vector<double>& linear, std::vector<uint8_t>* srgb, uint32_t row_offset, uint32_t row_stride,
                    std::vector<double>* partials) {
    cam.initialize();
    const uint32_t W = cam.image_width, H = cam.image_height;
    if (row_stride < 1) row_stride = 1;
    const uint32_t rows = row_offset >= H ? 0 : (H - row_offset + row_stride - 1) / row_stride;
    linear.assign((size_t)W * rows * 3, 0.0);
    if (srgb) srgb->assign((size_t)W * rows * 3, 0);
    if (partials) partials->assign((size_t)W * rows * cam.sqrt_spp * 3, 0.0);
    std::atomic<uint64_t> next{0};
    const uint64_t end = (uint64_t)rows * W;
    std::vector<WorkCounts> per_thread(threads > 0 ? threads : 1);
    std::vector<std::string> errors(per_thread.size());
    auto t0 = std::chrono::steady_clock::now();
    auto worker = [&](int tid) {
        work() = WorkCounts();
        PathRng rng;
        rng.seed = seed;
        current_rng() = &rng;
        try {
            for (;;) {
                uint64_t first = next.fetch_add(16);
                if (first >= end) break;
                uint64_t last = std::min<uint64_t>(first + 16, end);
                for (uint64_t k = first; k < last; ++k) {
                    uint32_t i = (uint32_t)(k % W), j = row_offset + (uint32_t)(k / W) * row_stride;
                    uint64_t pix = (uint64_t)j * W + i;
                    Color pixel_color;
                    for (uint32_t s_i = 0; s_i < cam.sqrt_spp; ++s_i) {
                        Color row_sum;
                        for (uint32_t s_j = 0; s_j < cam.sqrt_spp; ++s_j) {
                            rng.pixel = (uint32_t)pix;
                            rng.sample = s_i * cam.sqrt_spp + s_j;
                            rng.begin_vertex(0);
                            Ray r = cam.get_ray(i, j, s_i, s_j);
                            const Color c = cam.ray_color(r, cam.max_depth, world, lights);
                            pixel_color += c;
                            if (partials) row_sum += c;
                        }
                        if (partials) {
                            double* pd = &(*partials)[(k * cam.sqrt_spp + s_i) * 3];
                            pd[0] = row_sum[0];
                            pd[1] = row_sum[1];
                            pd[2] = row_sum[2];
                        }
                    }
                    Color pc = pixel_color * cam.pixel_sample_scale;
                    double* dst = &linear[k * 3];
                    dst[0] = pc[0];
                    dst[1] = pc[1];
                    dst[2] = pc[2];
                    if (srgb) to_rgb(pc, cam.toon_map, &(*srgb)[k * 3]);
                }
            }
        } catch (const std::exception& e) {
            errors[tid] = e.what();
            next.store(end);
        }
        current_rng() = nullptr;
        per_thread[tid] = work();
    };
    std::vector<std::thread> pool;
    for (size_t t = 1; t < per_thread.size(); ++t) pool.emplace_back(worker, (int)t);
    worker(0);
    for (auto& t : pool) t.join();
    RenderResult res;
    res.width = W;
    res.height = H;
    res.rows = rows;
    res.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (auto& w : per_thread) res.counts.add(w);
    for (auto& e : errors)
        if (!e.empty()) throw Panic(e);
    return res;
}

}  // namespace orc
