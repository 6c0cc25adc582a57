// rt_layout.h -- the flattened world as it lives in HBM.
//
// The reference world is a tree of Box<dyn Hittable> (src/hit.rs:46) walked by
// recursive virtual calls (Hittables::hit hits.rs:34, BVH::hit bvh.rs:57,
// Transform::hit shapes.rs:88, ConstantMedium::hit volume.rs:37).  Here it is
// one read-only blob of typed arrays, and every edge of the tree is a 32-bit
// `ref` = kind (top 4 bits) | index (low 28 bits), walked by an explicit
// per-lane stack (rt_kernel.hip).
//
// Layout choices (DESIGN.md "Data layout in HBM"):
//  - a BVH node is one record holding what is needed to test every child
//    (DNode4: four f32 boxes component-major + four refs, 112 B = 7 dwordx4
//    loads): one traversal step of a lane reads one record, never scattered
//    SoA streams (rays are incoherent after the first bounce);
//  - hot geometry is split from cold attributes: spheres are a double4
//    {center, radius} stream with materials in a separate int stream (read
//    only for the closest hit); planar primitives keep the 16 doubles the hit
//    test reads in one 128-B record and area/material apart;
//  - materials/textures are small tables read once per bounce.
#pragma once
#include "rt_planar_filter.h"
#include <hip/hip_runtime.h>
#include <stdint.h>

// Device code reads the world through global-address-space pointers so loads
// are global_load (vmcnt only), never flat_load (which also holds lgkmcnt and
// so serialises with the LDS traversal stack).
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_GLOBAL __attribute__((address_space(1)))
#define RT_LDS __attribute__((address_space(3)))
#else
#define RT_GLOBAL
#define RT_LDS
#endif

namespace rtk {

enum RefKind : uint32_t {
    K_NONE = 0,
    K_BVH = 1,
    K_LIST = 2,      // index = position in list_children (iterator form)
    K_SPHERE = 3,
    K_MSPHERE = 4,   // moving sphere (Sphere::new_with_motion)
    K_QUAD = 5,
    K_TRI = 6,
    K_XFORM = 7,
    K_MEDIUM = 8,
    K_POPXF = 9,     // traversal-stack marker: leave a Transform's frame
};

__host__ __device__ inline uint32_t make_ref(uint32_t kind, uint32_t index) { return (kind << 28) | index; }
__host__ __device__ inline uint32_t ref_kind(uint32_t r) { return r >> 28; }
__host__ __device__ inline uint32_t ref_index(uint32_t r) { return r & 0x0FFFFFFFu; }
constexpr uint32_t REF_NONE = 0u;

// BVH node (bvh.rs:5-9 re-laid out): the parent carries what is needed to
// test each child, so one node visit is one 80-B record:
//  - a child that is a sphere stores the sphere itself (f64 center, radius:
//    the exact data Sphere::hit reads, sphere.rs:77-108), tested directly --
//    no box test, no dependent load;
//  - any other child stores its AABB as f32 rounded outward (lo down, hi up);
//    the slab test is made conservative (rt_kernel.hip slab_f), so every hit
//    the reference's exact-box f64 test admits is admitted.
// c1 may be REF_NONE (a BVH over one object, bvh.rs:25).
struct alignas(16) DNodeSlot {
    union {
        struct {
            float lo[3], hi[3];
            uint32_t pad[2];
        } box;
        double sphere[4];  // {cx, cy, cz, r}
    };
};
struct alignas(16) DNode {
    DNodeSlot slot[2];
    uint32_t c0, c1;
    uint32_t pad[2];
};
static_assert(sizeof(DNode) == 80, "DNode must be 80 B (5 dwordx4)");

// Basic-tier 4-wide BVH node (rth::bvh4_basic): up to four children, their
// f32 boxes (rounded outward) stored component-major so one dwordx4 holds one
// bound of all four.  A sphere child keeps the sphere filter's record in its
// box slots instead: lo = center, hi.x = radius, hi.y = g = |c|_1 + r rounded
// up (rt_sphere_filter.h), all rounded to nearest but g.
struct alignas(16) DNode4 {
    float lo[3][4], hi[3][4];
    uint32_t ref[4];  // REF_NONE for an unused slot
};
static_assert(sizeof(DNode4) == 112, "DNode4 must be 112 B (7 dwordx4)");

// f32 box of one list element (list_boxes, parallel to list_children),
// rounded outward: the flat tier tests it before the element itself.  run:
// for a quad / triangle element, the number n (<= RT_PLANAR_RUN_MAX) of
// planar elements from this one on whose planar indices follow each other,
// with bit 8 + k set when element k of the run is a triangle (0 otherwise).
constexpr uint32_t RT_PLANAR_RUN_MAX = 8;
struct alignas(16) DBoxF {
    float lo[3], hi[3];
    uint32_t run, pad;
};
static_assert(sizeof(DBoxF) == 32, "DBoxF must be 32 B (2 dwordx4)");

// Planar: quad.rs:17-27 / triangle.rs:16-26 hot fields, packed in 128 B:
// f[0..3) unit normal, f[3] parm_d, f[4..7) anchor, f[7..10) u, f[10..13) v,
// f[13..16) w = n / |n|^2.
struct alignas(16) DPlanar {
    double f[16];
};

// RemappedMaterial (shapes/obj.rs:20-29) of an OBJ triangle, applied to the
// closest hit's record before shading: vertex normals n0..n2 (9 doubles),
// tex_ori, tex_u, tex_v (2 each, z = 0 in the reference's Vec3).
struct alignas(16) DRemap {
    double n[9];
    double tex_ori[2], tex_u[2], tex_v[2];
    int32_t normal_tex;  // -1 = no normal map; else texture id (remap_nm holds the frame)
    int32_t uv_ok;       // uv_local_to_world gave Some(u_vec), Some(v_vec)
};
static_assert(sizeof(DRemap) == 128, "DRemap must be 128 B");
// The tangent frame of a normal-mapped OBJ triangle (obj.rs:44-50, 196-210).
struct alignas(16) DRemapNM {
    double u_vec[3], v_vec[3];
};

// Transform (shapes.rs:23-29): the quaternion itself -- the kernel rotates
// with Quaternion::rotate_vector's two products (quaternion.rs:72-103) in the
// reference's operation order, so a transformed ray has the reference's bits
// (a 3x3 matrix form is the same rotation but not the same roundings).
struct alignas(16) DXform {
    double off[3];
    double scale[3];
    double q[4];  // w, x, y, z
    uint32_t child;
    uint32_t flags;  // XF_UNIT_SCALE: scale is exactly (1, 1, 1)
};
constexpr uint32_t XF_UNIT_SCALE = 1;

constexpr uint32_t RT_MED_PLANAR_MAX = 6;  // elements of a one-pass medium boundary (build_box: 6)

// ConstantMedium (volume.rs:16-20)
struct alignas(16) DMedium {
    double neg_inv_density;
    uint32_t boundary;
    int32_t phase_mat;
    uint32_t medium_id;
    // > 0: the boundary is planar_n quads / triangles stored consecutively at
    // planars[planar_first ..] (build_box's six quads), inside at most two
    // Transforms, tested in one pass (rt_kernel.hip medium_hit); 0: any other
    // boundary, walked twice
    uint32_t planar_n;
    uint32_t planar_first;
    uint32_t tri_mask;  // bit k: element k is a triangle
    uint32_t bxf_n;     // Transforms around those elements (outermost first)
    uint32_t bxf[2];
    uint32_t bsphere;   // > 0: the boundary is spheres[bsphere - 1] (inside bxf), one pass too
    uint32_t pad;
};

enum MatType : int32_t {
    M_LAMBERTIAN = 0,
    M_METAL = 1,
    M_DIELECTRIC = 2,
    M_DIFFUSE_LIGHT = 3,
    M_ISOTROPIC = 4,
    M_EMPTY = 5,
    M_TRANSPARENT = 6,
    M_MIX = 7,
};

// material.rs: one record per Arc<dyn Material>
struct alignas(16) DMaterial {
    int32_t type;
    int32_t tex;       // albedo / attenuation / emission texture
    int32_t inner;     // DiffuseLight inner material, Mix mat1
    int32_t inner2;    // Mix mat2
    double albedo[3];  // Metal albedo; the solid texture's colour (MF_SOLID)
    double fuzz;       // Metal fuzz (clamped), Dielectric ior, Mix ratio
    uint32_t flags;    // MF_*
    uint32_t pad[3];
};
// MF_SOLID: tex is a SolidColor, whose colour albedo holds (not for Metal)
enum : uint32_t { MF_NEEDS_UV = 1u, MF_EMISSIVE = 2u, MF_SOLID = 4u };

enum TexType : int32_t {
    T_SOLID = 0,
    T_CHECKER = 1,
    T_IMAGE = 2,
    T_NOISE = 3,
    T_SKY = 4,
};

struct alignas(16) DTexture {
    int32_t type;
    int32_t a, b;        // checker even/odd; image width/height
    int32_t c;           // image linear-interp flag
    double color[3];     // solid / sky horizon
    double color2[3];    // sky zenith
    double scale;        // checker inv_scale; noise scale
    uint64_t data;       // image: float offset into texels; noise: index into perlin tables
    uint32_t needs_uv, pad;
};

// perlin.rs:8-13
struct alignas(16) DPerlin {
    double randvec[256][3];
    int32_t perm[3][256];
};

// Everything the kernel reads about the world, as device pointers.
struct SceneView {
    const RT_GLOBAL DNode* nodes;
    const RT_GLOBAL DNode4* nodes4;          // 4-wide nodes: K_BVH refs index these
    const RT_GLOBAL double4* spheres;        // {cx, cy, cz, r}
    const RT_GLOBAL int32_t* sphere_mat;
    const RT_GLOBAL double* sphere_rinv;     // 1.0 / r, rounded as the kernel's division would
    const RT_GLOBAL double4* msph_center;    // moving: {c1.x, c1.y, c1.z, r}
    const RT_GLOBAL double4* msph_dir;       // {c2-c1, 0}
    const RT_GLOBAL int32_t* msph_mat;
    const RT_GLOBAL DPlanar* planars;        // quads then triangles share the record
    const RT_GLOBAL PlanarF* planars_f;      // their f32 pre-test records (rt_planar_filter.h)
    const RT_GLOBAL double* planar_area;
    const RT_GLOBAL int32_t* planar_mat;
    const RT_GLOBAL int32_t* planar_remap;   // index into remaps, -1 = plain Triangle/Quad
    const RT_GLOBAL DRemap* remaps;
    const RT_GLOBAL DRemapNM* remap_nm;
    const RT_GLOBAL uint32_t* list_children;  // runs of refs, each run terminated by REF_NONE
    const RT_GLOBAL DBoxF* list_boxes;        // the f32 box of each list_children entry (flat tier)
    const RT_GLOBAL DXform* xforms;
    const RT_GLOBAL DMedium* media;
    const RT_GLOBAL DMaterial* materials;
    const RT_GLOBAL DTexture* textures;
    const RT_GLOBAL float* texels;
    const RT_GLOBAL DPerlin* perlin;
    uint32_t world_root;
    uint32_t lights_root;  // REF_NONE = lights: None
    int32_t background_tex;  // -1 = black
    // background_tex's kind when it is a sky gradient (BG_SKY), with its two
    // colours copied here: the miss reads them with the launch parameters
    // (scalar loads) instead of two dependent vector loads of the texture
    // table in every wave iteration with a miss
    int32_t bg_kind;
    double bg_c0[3], bg_c1[3];  // BG_SKY: DTexture::color, color2
    uint32_t stack_need;     // max traversal stack entries (host-computed)
    uint32_t features;       // F_* of everything reachable from world/lights
    uint32_t n_nodes4;       // entries of nodes4
    uint32_t n_perlin;       // entries of perlin (the full tiers copy the first into LDS)
    // records each ref kind indexes (K_BVH: nodes4 or the two-box nodes,
    // K_LIST: list_children, K_QUAD / K_TRI: planars, ...): the check build
    // (make check, -DRT_CHECK) verifies every decoded ref against it
    uint32_t n_ref[16];
};

enum : int32_t { BG_NONE = 0, BG_SKY = 1, BG_OTHER = 2 };

// Scene features; the launcher picks the smallest kernel tier covering them.
enum : uint32_t {
    F_XFORM = 1u,
    F_MEDIUM = 2u,
    F_PLANAR = 4u,
    F_MSPHERE = 8u,
    F_LIGHTS = 16u,
    F_TEXFULL = 32u,  // image / noise textures
    F_MATFULL = 64u,  // DiffuseLight, Isotropic, Transparent, Mix
    F_REMAP = 128u,   // OBJ triangles with RemappedMaterial
    F_GENERAL = 512u,  // tier FULL_GL: lights beyond a flat list of static primitives, nested
                       // DiffuseLight / Mix wrappers, Mix::from_image ratios
    F_NORMALMAP = 256u,  // ... with a normal map (full tier: image textures)
};

}  // namespace rtk
