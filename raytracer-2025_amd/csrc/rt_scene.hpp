// rt_scene.hpp -- host-side world model of librt_mi355x.so.
//
// Objects mirror the reference constructors (shapes/*.rs, hits.rs, bvh.rs,
// volume.rs) as tagged records instead of trait objects; their bounding boxes
// and the reference BVH topology are computed exactly as the reference does
// (aabb.rs, bvh.rs:16-46, shapes.rs:49-72).  `flatten` turns one (world,
// lights) pair into the device layout of rt_layout.h; by default it rebuilds
// every BVH with a binned SAH over the same objects (tight boxes), keeping the
// reference topology only on request (RT_FLAG_REFERENCE_BVH).
#pragma once
#include <cmath>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "rt_layout.h"

namespace rth {

struct V3 {
    double x = 0, y = 0, z = 0;
    V3() = default;
    V3(double a, double b, double c) : x(a), y(b), z(c) {}
    explicit V3(const double* p) : x(p[0]), y(p[1]), z(p[2]) {}
    double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(V3 a, V3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(V3 a, V3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 operator/(V3 a, V3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline V3 operator*(double s, V3 v) { return V3(s * v.x, s * v.y, s * v.z); }
inline V3 operator-(V3 a) { return V3(-a.x, -a.y, -a.z); }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline double length(V3 a) { return std::sqrt(dot(a, a)); }
inline V3 div(V3 v, double s) { return (1.0 / s) * v; }  // vec3.rs:226-232
inline bool finite(V3 v) { return std::isfinite(v.x) && std::isfinite(v.y) && std::isfinite(v.z); }

// interval.rs / aabb.rs restated for construction-time boxes
struct Iv {
    double lo = 0, hi = 0;
};
struct Box3 {
    Iv a[3];  // Default: all [0,0] (aabb.rs:9 derive(Default))
    static Box3 empty();
    static Box3 from_points(V3 p, V3 q);  // aabb.rs:21-28 (+ pad 43-51)
    Box3 unite(const Box3& o) const;      // aabb.rs:94-100
    int longest_axis() const;             // aabb.rs:80-92
};

struct Quat {
    double w = 1, x = 0, y = 0, z = 0;
    Quat operator*(const Quat& r) const;  // quaternion.rs:94-103
    Quat conj() const { return Quat{w, -x, -y, -z}; }
    V3 rotate(V3 v) const;                // quaternion.rs:72-82
};

enum ObjKind { O_SPHERE, O_MSPHERE, O_QUAD, O_TRI, O_LIST, O_BVH, O_XFORM, O_MEDIUM };

struct Obj {
    ObjKind kind;
    Box3 bbox;
    bool moved = false;
    bool hidden = false;  // internal BVH node
    // sphere
    V3 c1, cdir;
    double radius = 0;
    int mat = -1;
    // planar
    V3 anchor, u, v, w, normal;
    double D = 0, area = 0;
    // OBJ triangle: RemappedMaterial (obj.rs:20-29)
    bool remap = false;
    V3 rn[3];
    double tex_ori[2] = {0, 0}, tex_u[2] = {0, 0}, tex_v[2] = {0, 0};
    int normal_tex = -1;  // RemappedMaterial::normal_tex (raw image texture), -1 = None
    bool uv_ok = false;   // u_vec / v_vec are Some
    V3 u_vec, v_vec;
    // list / bvh / transform / medium
    std::vector<int> children;
    int left = -1, right = -1, child = -1;
    V3 offset, scale;
    Quat q;
    double neg_inv_density = 0;
    int phase_mat = -1;
    uint32_t medium_id = 0;
};

struct TexRec {
    int type;
    double color[3] = {0, 0, 0}, color2[3] = {0, 0, 0};
    double scale = 0;
    int even = -1, odd = -1;
    uint32_t w = 0, h = 0;
    int linear = 0;
    size_t texel_offset = 0;
    int perlin = -1;
};
struct MatRec {
    int type;
    int tex = -1, inner = -1, inner2 = -1;
    double albedo[3] = {0, 0, 0};
    double param = 0;
};

// Flattened world on the host, ready to upload as one blob.
struct HostWorld {
    std::vector<rtk::DNode> nodes;
    std::vector<rtk::DNode4> nodes4;  // basic tier (bvh4_basic); mesh / full tiers before bvh4_quantize
    std::vector<double4> spheres;
    std::vector<int32_t> sphere_mat;
    std::vector<double> sphere_rinv;  // 1.0 / radius, the factor of sphere.rs:99's (p - c) / radius
    std::vector<double4> msph_center, msph_dir;
    std::vector<int32_t> msph_mat;
    std::vector<rtk::DPlanar> planars;
    std::vector<rtk::PlanarF> planars_f;  // parallel to planars
    std::vector<double> planar_area;
    std::vector<int32_t> planar_mat;
    std::vector<int32_t> planar_remap;
    std::vector<rtk::DRemap> remaps;
    std::vector<rtk::DRemapNM> remap_nm;  // parallel to remaps when any normal map is used
    std::vector<uint32_t> list_children;
    std::vector<rtk::DBoxF> list_boxes;  // parallel to list_children
    std::vector<rtk::DXform> xforms;
    std::vector<rtk::DMedium> media;
    std::vector<rtk::DMaterial> materials;
    std::vector<rtk::DTexture> textures;
    std::vector<float> texels;
    std::vector<rtk::DPerlin> perlin;
    uint32_t world_root = 0, lights_root = 0;
    uint32_t stack_need = 0;
    uint32_t features = 0;
    size_t n_prims = 0;
    size_t n_bvh_leaves = 0;
};

struct RenderState;  // rt_render.cpp: per-device worlds and work buffers

}  // namespace rth

struct rt_scene {
    std::vector<rth::Obj> objs;
    std::vector<rth::TexRec> texs;
    std::vector<rth::MatRec> mats;
    std::vector<float> texels;
    std::vector<rtk::DPerlin> perlins;
    uint32_t next_medium_id = 0;
    uint64_t generation = 0;  // bumped by every mutation; invalidates the device cache
    // device-side cache and the last render's state (rt_render.cpp)
    rth::RenderState* rs = nullptr;
};

namespace rth {
int32_t set_error(int32_t code, const std::string& msg);
// Flattens (world, lights) of scene s; lights = -1 for None.  Returns RT_OK or an RT_E* code.
// reference_bvh: keep the reference's BVH topology (bvh.rs:16-46) instead of
// the binned-SAH rebuild (closest-hit results agree up to exact t ties).
int32_t flatten(const rt_scene* s, int32_t world, int32_t lights, int32_t background_tex, bool reference_bvh,
                HostWorld& out);
// Collapses every two-box BVH into 4-wide nodes (hw.nodes4; sphere children as
// filter records when filter_spheres, the basic tier), rewrites the K_BVH refs
// to index nodes4 and recomputes stack_need.  Returns the new stack_need (hw is
// unchanged when it exceeds max_need), or UINT32_MAX (hw unchanged) when the
// tree would have more than max_nodes nodes.
uint32_t bvh4_convert(HostWorld& hw, uint32_t max_need, bool filter_spheres, size_t max_nodes = SIZE_MAX);
void destroy_render_state(RenderState* r);
}  // namespace rth
