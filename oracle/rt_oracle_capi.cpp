// oracle/rt_oracle_capi.cpp -- TEST INFRASTRUCTURE ONLY.
//
// The C ABI of include/rt_mi355x.h implemented by the CPU oracle under the
// prefix `orc_` (liboracle.so), so tests can build one scene description on
// both the gfx950 library and the oracle and compare the images.
#include <cstdio>
#include <fstream>
#include <sstream>
#include <mutex>
#include <thread>

#include "../include/rt_mi355x.h"
#include "rt_oracle.hpp"
#include "orc_png.hpp"

using namespace orc;

namespace {
thread_local std::string g_err;

int32_t fail(int32_t code, const std::string& msg) {
    g_err = msg;
    return code;
}
Vec3 v3(const double* p) { return Vec3(p[0], p[1], p[2]); }

}  // namespace

struct rt_scene {
    std::vector<std::shared_ptr<Texture>> tex;
    std::vector<std::shared_ptr<Material>> mat;
    std::vector<HittablePtr> obj;  // null after a move
    std::vector<bool> moved;
    uint32_t next_medium_id = 0;

    int32_t add_obj(HittablePtr p) {
        obj.push_back(std::move(p));
        moved.push_back(false);
        return (int32_t)obj.size() - 1;
    }
    bool tex_ok(int32_t t) const { return t >= 0 && (size_t)t < tex.size(); }
    bool mat_ok(int32_t m) const { return m >= 0 && (size_t)m < mat.size(); }
    int32_t check_obj(int32_t o) const {
        if (o < 0 || (size_t)o >= obj.size()) return fail(RT_EHANDLE, "unknown object handle");
        if (moved[o]) return fail(RT_EMOVED, "object handle already moved");
        return RT_OK;
    }
    HittablePtr take(int32_t o) {
        moved[o] = true;
        return std::move(obj[o]);
    }
};

#define GUARD_BEGIN try {
#define GUARD_END                                          \
    }                                                      \
    catch (const Panic& p) {                               \
        return fail(RT_EPANIC, p.what());                  \
    }                                                      \
    catch (const std::bad_alloc&) {                        \
        return fail(RT_ENOMEM, "out of memory");           \
    }                                                      \
    catch (const std::exception& e) {                      \
        return fail(RT_EINVAL, e.what());                  \
    }

extern "C" {

int32_t orc_abi_version(void) { return RT_ABI_VERSION; }
const char* orc_last_error(void) { return g_err.c_str(); }
rt_scene* orc_scene_create(void) { return new rt_scene(); }
void orc_scene_destroy(rt_scene* s) { delete s; }

int32_t orc_tex_solid(rt_scene* s, const double rgb[3]) {
    if (!s || !rgb) return fail(RT_EINVAL, "null");
    s->tex.push_back(std::make_shared<SolidColor>(v3(rgb)));
    return (int32_t)s->tex.size() - 1;
}
int32_t orc_tex_checker(rt_scene* s, double scale, int32_t even, int32_t odd) {
    if (!s) return fail(RT_EINVAL, "null");
    if (!s->tex_ok(even) || !s->tex_ok(odd)) return fail(RT_EHANDLE, "unknown texture");
    s->tex.push_back(std::make_shared<CheckerTexture>(scale, s->tex[even], s->tex[odd]));
    return (int32_t)s->tex.size() - 1;
}
int32_t orc_tex_image(rt_scene* s, uint32_t w, uint32_t h, const float* rgba, int32_t linear) {
    if (!s) return fail(RT_EINVAL, "null");
    if ((w == 0) != (h == 0)) return fail(RT_EINVAL, "image must have both dimensions or none");
    if (w && !rgba) return fail(RT_EINVAL, "null pixels");
    auto t = std::make_shared<ImageTexture>();
    t->w = (int)w;
    t->h = (int)h;
    t->linear_interp = linear != 0;
    if (w) t->rgba.assign(rgba, rgba + (size_t)w * h * 4);
    s->tex.push_back(t);
    return (int32_t)s->tex.size() - 1;
}
// Image::new(path, raw) + pixel_data's colour handling (utils/image.rs:21-82)
// with the oracle's own PNG reader (orc_png.hpp): a file that cannot be
// opened or decoded is Image::EMPTY (0 x 0: cyan), a file that is not a PNG
// is refused (the product library refuses it too: RT_EUNSUPPORTED).
static bool orc_load_image(const std::string& path, bool raw, uint32_t& w, uint32_t& h, std::vector<float>& px) {
    const orcpng::Result r = orcpng::decode_file(path, w, h, px);
    if (r == orcpng::NOT_PNG) return false;
    if (r == orcpng::DECODED && !raw)
        for (size_t i = 0; i < px.size(); i += 4)
            for (int c = 0; c < 3; ++c) px[i + c] = orcpng::eotf(px[i + c]);
    return true;
}
// ImageTexture::new / new_raw_image from a file
int32_t orc_tex_image_file(rt_scene* s, const char* path, int32_t raw, int32_t linear) {
    if (!s || !path) return fail(RT_EINVAL, "null");
    uint32_t w = 0, h = 0;
    std::vector<float> px;
    if (!orc_load_image(path, raw != 0, w, h, px)) return fail(RT_EUNSUPPORTED, std::string(path) + ": not a PNG");
    return orc_tex_image(s, w, h, px.empty() ? nullptr : px.data(), linear);
}
int32_t orc_tex_noise(rt_scene* s, double scale, uint64_t seed) {
    if (!s) return fail(RT_EINVAL, "null");
    s->tex.push_back(std::make_shared<NoiseTexture>(scale, seed));
    return (int32_t)s->tex.size() - 1;
}
int32_t orc_tex_sky_gradient(rt_scene* s, const double horizon[3], const double zenith[3]) {
    if (!s || !horizon || !zenith) return fail(RT_EINVAL, "null");
    s->tex.push_back(std::make_shared<SkyGradient>(v3(horizon), v3(zenith)));
    return (int32_t)s->tex.size() - 1;
}

static int32_t push_mat(rt_scene* s, std::shared_ptr<Material> m) {
    s->mat.push_back(std::move(m));
    return (int32_t)s->mat.size() - 1;
}
int32_t orc_mat_empty(rt_scene* s) { return s ? push_mat(s, std::make_shared<EmptyMaterial>()) : fail(RT_EINVAL, "null"); }
int32_t orc_mat_lambertian(rt_scene* s, int32_t tex) {
    if (!s) return fail(RT_EINVAL, "null");
    if (!s->tex_ok(tex)) return fail(RT_EHANDLE, "unknown texture");
    return push_mat(s, std::make_shared<Lambertian>(s->tex[tex]));
}
int32_t orc_mat_metal(rt_scene* s, const double albedo[3], double fuzz) {
    if (!s || !albedo) return fail(RT_EINVAL, "null");
    return push_mat(s, std::make_shared<Metal>(v3(albedo), fuzz));
}
int32_t orc_mat_dielectric(rt_scene* s, int32_t tex, double ior) {
    if (!s) return fail(RT_EINVAL, "null");
    if (!s->tex_ok(tex)) return fail(RT_EHANDLE, "unknown texture");
    return push_mat(s, std::make_shared<Dielectric>(s->tex[tex], ior));
}
int32_t orc_mat_diffuse_light(rt_scene* s, int32_t tex, int32_t inner) {
    if (!s) return fail(RT_EINVAL, "null");
    if (!s->tex_ok(tex)) return fail(RT_EHANDLE, "unknown texture");
    if (inner != -1 && !s->mat_ok(inner)) return fail(RT_EHANDLE, "unknown material");
    return push_mat(s, std::make_shared<DiffuseLight>(s->tex[tex], inner == -1 ? nullptr : s->mat[inner]));
}
int32_t orc_mat_isotropic(rt_scene* s, int32_t tex) {
    if (!s) return fail(RT_EINVAL, "null");
    if (!s->tex_ok(tex)) return fail(RT_EHANDLE, "unknown texture");
    return push_mat(s, std::make_shared<Isotropic>(s->tex[tex]));
}
int32_t orc_mat_transparent(rt_scene* s) { return s ? push_mat(s, std::make_shared<Transparent>()) : fail(RT_EINVAL, "null"); }
int32_t orc_mat_mix(rt_scene* s, int32_t m1, int32_t m2, double ratio) {
    if (!s) return fail(RT_EINVAL, "null");
    if (!s->mat_ok(m1) || !s->mat_ok(m2)) return fail(RT_EHANDLE, "unknown material");
    return push_mat(s, std::make_shared<Mix>(s->mat[m1], s->mat[m2], ratio));
}

int32_t orc_mat_mix_image(rt_scene* s, int32_t m1, int32_t m2, int32_t tex) {
    if (!s) return fail(RT_EINVAL, "null");
    if (!s->mat_ok(m1) || !s->mat_ok(m2)) return fail(RT_EHANDLE, "unknown material");
    auto it = s->tex_ok(tex) ? std::dynamic_pointer_cast<ImageTexture>(s->tex[tex]) : nullptr;
    if (!it) return fail(RT_EHANDLE, "Mix::from_image takes an ImageTexture");
    return push_mat(s, std::make_shared<Mix>(s->mat[m1], s->mat[m2], it));
}

int32_t orc_sphere(rt_scene* s, const double c[3], double r, int32_t mat) {
    if (!s || !c) return fail(RT_EINVAL, "null");
    if (!s->mat_ok(mat)) return fail(RT_EHANDLE, "unknown material");
    return s->add_obj(std::make_unique<Sphere>(v3(c), r, s->mat[mat]));
}
int32_t orc_sphere_moving(rt_scene* s, const double c1[3], const double c2[3], double r, int32_t mat) {
    if (!s || !c1 || !c2) return fail(RT_EINVAL, "null");
    if (!s->mat_ok(mat)) return fail(RT_EHANDLE, "unknown material");
    return s->add_obj(std::make_unique<Sphere>(v3(c1), v3(c2), r, s->mat[mat]));
}
int32_t orc_quad(rt_scene* s, const double q[3], const double u[3], const double v[3], int32_t mat) {
    if (!s || !q || !u || !v) return fail(RT_EINVAL, "null");
    if (!s->mat_ok(mat)) return fail(RT_EHANDLE, "unknown material");
    GUARD_BEGIN
    return s->add_obj(make_quad(v3(q), v3(u), v3(v), s->mat[mat]));
    GUARD_END
}
int32_t orc_triangle(rt_scene* s, const double a[3], const double u[3], const double v[3], int32_t mat) {
    if (!s || !a || !u || !v) return fail(RT_EINVAL, "null");
    if (!s->mat_ok(mat)) return fail(RT_EHANDLE, "unknown material");
    auto t = make_triangle(v3(a), v3(u), v3(v), s->mat[mat]);
    if (!t) return fail(RT_EDEGENERATE, "degenerate triangle (Triangle::new -> None)");
    return s->add_obj(std::move(t));
}
int32_t orc_hittables_new(rt_scene* s) {
    if (!s) return fail(RT_EINVAL, "null");
    return s->add_obj(std::make_unique<Hittables>());
}
int32_t orc_hittables_add(rt_scene* s, int32_t list, int32_t object) {
    if (!s) return fail(RT_EINVAL, "null");
    int32_t rc;
    if ((rc = s->check_obj(list)) != RT_OK) return rc;
    if ((rc = s->check_obj(object)) != RT_OK) return rc;
    if (list == object) return fail(RT_EINVAL, "cannot add a list to itself");
    auto* l = dynamic_cast<Hittables*>(s->obj[list].get());
    if (!l) return fail(RT_EHANDLE, "not a Hittables object");
    l->add(s->take(object));
    return RT_OK;
}
int32_t orc_bvh_new(rt_scene* s, int32_t list) {
    if (!s) return fail(RT_EINVAL, "null");
    int32_t rc;
    if ((rc = s->check_obj(list)) != RT_OK) return rc;
    auto* l = dynamic_cast<Hittables*>(s->obj[list].get());
    if (!l) return fail(RT_EHANDLE, "not a Hittables object");
    GUARD_BEGIN
    auto owned = s->take(list);
    auto objs = std::move(static_cast<Hittables*>(owned.get())->objects);
    return s->add_obj(BVH::from_vec(std::move(objs)));
    GUARD_END
}
int32_t orc_build_box(rt_scene* s, const double a[3], const double b[3], int32_t mat) {
    if (!s || !a || !b) return fail(RT_EINVAL, "null");
    if (!s->mat_ok(mat)) return fail(RT_EHANDLE, "unknown material");
    GUARD_BEGIN
    return s->add_obj(build_box(v3(a), v3(b), s->mat[mat]));
    GUARD_END
}
int32_t orc_transform_new(rt_scene* s, int32_t object, const double* off, const double* q, const double* sc) {
    if (!s) return fail(RT_EINVAL, "null");
    int32_t rc;
    if ((rc = s->check_obj(object)) != RT_OK) return rc;
    Quaternion quat = q ? Quaternion{q[0], q[1], q[2], q[3]} : Quaternion::identity();
    return s->add_obj(std::make_unique<Transform>(s->take(object), off ? v3(off) : Vec3(0, 0, 0), quat,
                                                  sc ? v3(sc) : Vec3(1, 1, 1)));
}
int32_t orc_constant_medium_new(rt_scene* s, int32_t boundary, double density, int32_t tex) {
    if (!s) return fail(RT_EINVAL, "null");
    int32_t rc;
    if ((rc = s->check_obj(boundary)) != RT_OK) return rc;
    if (!s->tex_ok(tex)) return fail(RT_EHANDLE, "unknown texture");
    return s->add_obj(std::make_unique<ConstantMedium>(s->take(boundary), density, s->tex[tex], s->next_medium_id++));
}

// Wavefont::new (shapes/obj.rs:117-134), load_materials (212-345), load_object (137-194)
int32_t orc_wavefront_load(rt_scene* s, const char* obj_path, int32_t vanilla) {
    if (!s || !obj_path) return fail(RT_EINVAL, "null");
    GUARD_BEGIN
    ObjFile f = load_obj_file(obj_path);
    const std::string path(obj_path);
    const size_t slash = path.rfind('/');
    const std::string prefix = slash == std::string::npos ? "." : path.substr(0, slash);
    auto parse_f64 = [](const std::string& v, double& out) {  // str::parse::<f64>
        if (v.empty()) return false;
        char* end = nullptr;
        out = std::strtod(v.c_str(), &end);
        return *end == 0;
    };
    auto param = [&](const ObjMaterial& m, const char* k, double def) {
        auto it = m.unknown_param.find(k);
        double x;
        return (it != m.unknown_param.end() && parse_f64(it->second, x)) ? x : def;
    };
    auto values = [&](const std::string& v) {
        std::vector<double> out;
        std::istringstream is(v);
        std::string w;
        double x;
        while (is >> w)
            if (parse_f64(w, x)) out.push_back(x);
        return out;
    };
    auto transparent = std::make_shared<Transparent>();
    std::vector<std::shared_ptr<Material>> mats;
    std::vector<std::shared_ptr<Texture>> normals;
    // ImageTexture::new(prefix/file) (texture.rs:82-88) / new_raw_image (90-97)
    std::string img_err;
    auto image = [&](const std::string& file, bool raw) -> std::shared_ptr<ImageTexture> {
        auto t = std::make_shared<ImageTexture>();
        uint32_t w = 0, h = 0;
        if (!orc_load_image(prefix + "/" + file, raw, w, h, t->rgba)) {
            img_err = prefix + "/" + file + ": not a PNG";
            return nullptr;
        }
        t->w = (int)w;
        t->h = (int)h;  // 0 x 0: missing -> cyan (texture.rs:167-169)
        t->linear_interp = raw;
        return t;
    };
    for (const ObjMaterial& m : f.materials) {
        std::shared_ptr<Texture> base;
        if (!m.diffuse_texture.empty()) {
            base = image(m.diffuse_texture, false);
            if (!base) return fail(RT_EUNSUPPORTED, img_err);
        } else if (m.has_diffuse) {
            base = std::make_shared<SolidColor>(m.diffuse);
        } else {
            throw Panic("The material should at least have one diffuse!");
        }
        const double roughness = param(m, "Pr", 0.5), metallic = param(m, "Pm", 0.0);
        const double ior = m.has_optical_density ? m.optical_density : 1.45;
        double spec_trans = 0.0;
        auto tf = m.unknown_param.find("Tf");
        if (tf != m.unknown_param.end()) {
            std::vector<double> v = values(tf->second);
            double sum = 0.0;
            for (double x : v) sum += x;
            spec_trans = sum / (double)v.size();
        }
        std::shared_ptr<Material> mat;
        if (vanilla && metallic == 1.0)
            mat = std::make_shared<Metal>(base->value(0.0, 0.0, Vec3(0, 0, 0)), roughness);
        else if (vanilla && spec_trans == 1.0)
            mat = std::make_shared<Dielectric>(base, ior);
        else
            return fail(RT_EUNSUPPORTED, "Disney BSDF materials are not supported");
        auto ke = m.unknown_param.find("Ke");
        if (ke != m.unknown_param.end()) {
            std::vector<double> v = values(ke->second);
            if (v.size() == 3) mat = std::make_shared<DiffuseLight>(std::make_shared<SolidColor>(Vec3(v[0], v[1], v[2])), mat);
        }
        auto mke = m.unknown_param.find("map_Ke");
        if (mke != m.unknown_param.end()) {  // obj.rs:319-323
            auto et = image(mke->second, false);
            if (!et) return fail(RT_EUNSUPPORTED, img_err);
            mat = std::make_shared<DiffuseLight>(et, mat);
        }
        if (!m.dissolve_texture.empty()) {  // obj.rs:325-332
            auto dt = image(m.dissolve_texture, false);
            if (!dt) return fail(RT_EUNSUPPORTED, img_err);
            mat = std::make_shared<Mix>(transparent, mat, dt);
        }
        if (m.has_dissolve && m.dissolve < 1.0) mat = std::make_shared<Mix>(transparent, mat, m.dissolve);
        mats.push_back(mat);
        std::shared_ptr<Texture> ntex;  // obj.rs:324-343
        if (!m.normal_texture.empty()) {
            std::string fname = m.normal_texture;
            if (fname.rfind("-bm", 0) == 0) {
                std::istringstream is(fname.substr(3));
                std::string w, last;
                while (is >> w) last = w;
                if (!last.empty()) fname = last;
            }
            ntex = image(fname, true);  // new_raw_image: raw, linear interpolation
            if (!ntex) return fail(RT_EUNSUPPORTED, img_err);
        }
        normals.push_back(ntex);
    }
    auto objs = std::make_unique<Hittables>();
    auto empty = std::make_shared<EmptyMaterial>();
    const size_t n = std::min(f.models.size(), f.materials.size());  // objects.iter().zip(normals.iter())
    for (size_t mi = 0; mi < n; ++mi) {
        const ObjModel& o = f.models[mi];
        std::vector<HittablePtr> v;
        auto three = [](const std::vector<double>& a, uint32_t i) {
            if ((size_t)i * 3 + 2 >= a.size()) throw Panic("index out of bounds (obj.rs:107-110)");
            return Vec3(a[i * 3], a[i * 3 + 1], a[i * 3 + 2]);
        };
        auto two = [](const std::vector<double>& a, uint32_t i) {
            if ((size_t)i * 2 + 1 >= a.size()) throw Panic("index out of bounds (obj.rs:112-115)");
            return Vec3(a[i * 2], a[i * 2 + 1], 0.0);
        };
        for (size_t k = 0; k + 2 < o.indices.size(); k += 3) {
            const uint32_t i0 = o.indices[k], i1 = o.indices[k + 1], i2 = o.indices[k + 2];
            const Vec3 p1 = three(o.positions, i0), p2 = three(o.positions, i1), p3 = three(o.positions, i2);
            const Vec3 t1 = two(o.texcoords, i0), t2 = two(o.texcoords, i1), t3 = two(o.texcoords, i2);
            auto rm = std::make_shared<RemappedMaterial>();
            rm->material = o.material_id >= 0 ? mats[o.material_id] : empty;
            rm->tex_ori = t1;
            rm->tex_u = t2 - t1;
            rm->tex_v = t3 - t1;
            rm->normal[0] = three(o.normals, i0);
            rm->normal[1] = three(o.normals, i1);
            rm->normal[2] = three(o.normals, i2);
            rm->normal_tex = normals[mi];
            {  // uv_local_to_world (obj.rs:196-210)
                const Vec3 tu = rm->tex_u, tv = rm->tex_v, wu = p2 - p1, wv = p3 - p1;
                const double ua = tv.e[1] / (-tu.e[1] * tv.e[0] + tu.e[0] * tv.e[1]);
                const double ub = tu.e[1] / (tu.e[1] * tv.e[0] - tu.e[0] * tv.e[1]);
                const double va = tv.e[0] / (tu.e[1] * tv.e[0] - tu.e[0] * tv.e[1]);
                const double vb = tu.e[0] / (-tu.e[1] * tv.e[0] + tu.e[0] * tv.e[1]);
                rm->u_vec = from_vec3(wu * ua + wv * ub);
                rm->v_vec = from_vec3(wu * va + wv * vb);
            }
            auto tri = make_triangle(p1, p2 - p1, p3 - p1, rm);
            if (tri) v.push_back(std::move(tri));
        }
        if (!v.empty()) objs->add(BVH::from_vec(std::move(v)));
    }
    return s->add_obj(std::move(objs));
    GUARD_END
}

int32_t orc_quat_from_axis_angle(const double axis[3], double deg, double out[4]) {
    GUARD_BEGIN
    Quaternion q = Quaternion::from_axis_angle(v3(axis), deg);
    out[0] = q.w;
    out[1] = q.x;
    out[2] = q.y;
    out[3] = q.z;
    return RT_OK;
    GUARD_END
}
void orc_quat_from_euler(double yaw, double pitch, double roll, double out[4]) {
    Quaternion q = Quaternion::from_euler(yaw, pitch, roll);
    out[0] = q.w;
    out[1] = q.x;
    out[2] = q.y;
    out[3] = q.z;
}

void orc_camera_default(rt_camera* c) {
    std::memset(c, 0, sizeof(*c));
    c->aspect_ratio = 1.0;
    c->image_width = 100;
    c->samples_per_pixel = 10;
    c->max_depth = 10;
    c->background_tex = -1;
    c->vertical_fov_in_degrees = 90.0;
    c->look_at[2] = -1.0;
    c->vec_up[1] = 1.0;
    c->focus_distance = 10.0;
}
uint32_t orc_camera_image_height(const rt_camera* c) {
    uint32_t h = (uint32_t)((double)c->image_width / c->aspect_ratio);
    return h < 1 ? 1 : h;
}
void orc_render_opts_default(rt_render_opts* o) {
    std::memset(o, 0, sizeof(*o));
    o->struct_size = sizeof(*o);
    o->seed = 1;
    o->row_stride = 1;
}
uint32_t orc_shard_rows(const rt_camera* c, const rt_render_opts* o) {
    uint32_t H = orc_camera_image_height(c);
    uint32_t stride = (o && o->row_stride > 1) ? o->row_stride : 1;
    uint32_t off = o ? o->row_offset : 0;
    if (off >= H) return 0;
    return (H - off + stride - 1) / stride;
}

// Oracle-only extras for tests and the CPU baseline: f64 output and the
// instrumented work counts of SURVEY §8(d).
int32_t orc_render_f64(rt_scene* s, int32_t world, int32_t lights, const rt_camera* c, const rt_render_opts* o,
                       double* out_linear, uint8_t* out_srgb, rt_stats* stats, uint64_t* work_counts) {
    if (!s || !c) return fail(RT_EINVAL, "null");
    int32_t rc;
    if ((rc = s->check_obj(world)) != RT_OK) return rc;
    if (lights != -1 && (rc = s->check_obj(lights)) != RT_OK) return rc;
    if (c->background_tex != -1 && !s->tex_ok(c->background_tex)) return fail(RT_EHANDLE, "unknown background");
    if (c->image_width == 0 || !(c->aspect_ratio > 0)) return fail(RT_EINVAL, "bad image size");
    GUARD_BEGIN
    Camera cam;
    cam.aspect_ratio = c->aspect_ratio;
    cam.image_width = c->image_width;
    cam.samples_per_pixel = c->samples_per_pixel;
    cam.max_depth = c->max_depth;
    cam.background = c->background_tex == -1 ? nullptr : s->tex[c->background_tex];
    cam.vertical_fov_in_degrees = c->vertical_fov_in_degrees;
    cam.look_from = v3(c->look_from);
    cam.look_at = v3(c->look_at);
    cam.vec_up = v3(c->vec_up);
    cam.defocus_angle_in_degrees = c->defocus_angle_in_degrees;
    cam.focus_distance = c->focus_distance;
    cam.toon_map = c->toon_map == 1 ? ToonMap::ACES : ToonMap::None;
    int threads = (o && o->threads) ? (int)o->threads : (int)std::thread::hardware_concurrency();
    if (threads < 1) threads = 1;
    std::vector<double> lin;
    std::vector<uint8_t> srgb;
    RenderResult res = render(cam, *s->obj[world], lights == -1 ? nullptr : s->obj[lights].get(), o ? o->seed : 1,
                              threads, lin, out_srgb ? &srgb : nullptr, o ? o->row_offset : 0,
                              (o && o->row_stride > 1) ? o->row_stride : 1);
    if (out_linear && !lin.empty()) std::memcpy(out_linear, lin.data(), lin.size() * sizeof(double));
    if (out_srgb && !srgb.empty()) std::memcpy(out_srgb, srgb.data(), srgb.size());
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->samples = (uint64_t)res.rows * res.width * (uint64_t)cam.sqrt_spp * cam.sqrt_spp;
        stats->rays = res.counts.ray_color_calls;
        stats->render_ms = res.seconds * 1e3;
    }
    if (work_counts) std::memcpy(work_counts, &res.counts, sizeof(WorkCounts));
    return RT_OK;
    GUARD_END
}
// Test tooling: the per-(pixel, stratum row) f64 sums (as rt_render_partials_get).
int32_t orc_render_partials(rt_scene* s, int32_t world, int32_t lights, const rt_camera* c, const rt_render_opts* o,
                            double* partials, rt_stats* stats) {
    if (!s || !c || !partials) return fail(RT_EINVAL, "null");
    int32_t rc;
    if ((rc = s->check_obj(world)) != RT_OK) return rc;
    if (lights != -1 && (rc = s->check_obj(lights)) != RT_OK) return rc;
    if (c->background_tex != -1 && !s->tex_ok(c->background_tex)) return fail(RT_EHANDLE, "unknown background");
    if (c->image_width == 0 || !(c->aspect_ratio > 0)) return fail(RT_EINVAL, "bad image size");
    GUARD_BEGIN
    Camera cam;
    cam.aspect_ratio = c->aspect_ratio;
    cam.image_width = c->image_width;
    cam.samples_per_pixel = c->samples_per_pixel;
    cam.max_depth = c->max_depth;
    cam.background = c->background_tex == -1 ? nullptr : s->tex[c->background_tex];
    cam.vertical_fov_in_degrees = c->vertical_fov_in_degrees;
    cam.look_from = v3(c->look_from);
    cam.look_at = v3(c->look_at);
    cam.vec_up = v3(c->vec_up);
    cam.defocus_angle_in_degrees = c->defocus_angle_in_degrees;
    cam.focus_distance = c->focus_distance;
    int threads = (o && o->threads) ? (int)o->threads : (int)std::thread::hardware_concurrency();
    if (threads < 1) threads = 1;
    std::vector<double> lin, part;
    RenderResult res = render(cam, *s->obj[world], lights == -1 ? nullptr : s->obj[lights].get(), o ? o->seed : 1,
                              threads, lin, nullptr, o ? o->row_offset : 0,
                              (o && o->row_stride > 1) ? o->row_stride : 1, &part);
    if (!part.empty()) std::memcpy(partials, part.data(), part.size() * sizeof(double));
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->samples = (uint64_t)res.rows * res.width * (uint64_t)cam.sqrt_spp * cam.sqrt_spp;
        stats->rays = res.counts.ray_color_calls;
        stats->render_ms = res.seconds * 1e3;
    }
    return RT_OK;
    GUARD_END
}
uint32_t orc_work_count_fields(void) { return sizeof(WorkCounts) / sizeof(uint64_t); }

int32_t orc_render(rt_scene* s, int32_t world, int32_t lights, const rt_camera* c, const rt_render_opts* o,
                   float* out_linear, uint8_t* out_srgb, rt_stats* stats) {
    if (!c) return fail(RT_EINVAL, "null");
    const size_t n = (size_t)orc_shard_rows(c, o) * c->image_width * 3;
    std::vector<double> lin(n);
    int32_t rc = orc_render_f64(s, world, lights, c, o, lin.data(), out_srgb, stats, nullptr);
    if (rc != RT_OK) return rc;
    if (out_linear)
        for (size_t i = 0; i < n; ++i) out_linear[i] = (float)lin[i];
    return RT_OK;
}

}  // extern "C"
