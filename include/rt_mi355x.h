/* include/rt_mi355x.h -- C ABI of librt_mi355x.so, the MI355X (gfx950) render
 * path for caidj0/Raytracer-2025.
 *
 * The reference path is `Camera::render(&mut self, world: &dyn Hittable,
 * lights: Option<&dyn Hittable>) -> RgbImage` (src/camera.rs:161) over the
 * plugin traits Hittable (src/hit.rs:46-60), Material (src/material.rs:23-34),
 * Texture (src/texture.rs:5-7) and PDF (src/pdf.rs:13-16).  Rust trait objects
 * cannot cross a C boundary, so the world is described by constructor calls
 * that mirror the reference constructors one-to-one (each cited below), and is
 * flattened once into device arrays at the first rt_render that uses it.
 *
 * Conventions
 *  - Every constructor returns a handle >= 0 or a negative RT_E* code; the
 *    message of the last failure on this thread is rt_last_error().
 *  - Handles are per scene and per kind (texture / material / object).
 *    Textures and materials are shared (Arc in the reference): a handle may be
 *    used any number of times.  Objects are owned (Box<dyn Hittable>): passing
 *    an object to rt_hittables_add / rt_bvh_new / rt_transform_new /
 *    rt_constant_medium_new moves it, and a moved handle is RT_EMOVED
 *    afterwards (the Rust compiler rejects such reuse).
 *  - Reference panics (assert!, expect, unwrap, unimplemented!) become
 *    RT_EPANIC with a message; the library never aborts the process.
 *  - Not thread-safe per scene: calls on one scene are serialised by the
 *    caller.  Different scenes may be used from different threads, also
 *    when they render on the same device list or through the same rt_comm:
 *    the frame gathers of such renders are enqueued one whole RCCL group
 *    at a time.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 3

enum rt_status {
    RT_OK = 0,
    RT_EINVAL = -1,       /* bad argument (null pointer, non-finite, out of range) */
    RT_EHANDLE = -2,      /* unknown handle or wrong kind */
    RT_EMOVED = -3,       /* object handle already moved into another object */
    RT_EDEGENERATE = -4,  /* Triangle::new returned None (triangle.rs:29-31) */
    RT_EPANIC = -5,       /* a reference panic condition was hit (message in rt_last_error) */
    RT_EUNSUPPORTED = -6, /* construct valid in the reference but not on this path yet */
    RT_EDEVICE = -7,      /* HIP runtime error, or no gfx950 device */
    RT_ENOMEM = -8,       /* host or device allocation failed */
    RT_ESTACK = -9        /* world deeper than the kernel's traversal stack */
};

typedef struct rt_scene rt_scene;

int32_t rt_abi_version(void);
const char* rt_last_error(void);
rt_scene* rt_scene_create(void);
void rt_scene_destroy(rt_scene* s);

/* ---- Textures (src/texture.rs) ------------------------------------------ */
/* SolidColor::new (texture.rs:14-16) */
int32_t rt_tex_solid(rt_scene* s, const double rgb[3]);
/* CheckerTexture::new (texture.rs:46-56) */
int32_t rt_tex_checker(rt_scene* s, double scale, int32_t even_tex, int32_t odd_tex);
/* ImageTexture::new / new_raw_image (texture.rs:82-97): pixels already decoded
 * to linear RGBA f32, row 0 = top (image.rs:63-82).  width == height == 0 is a
 * missing file: value() is cyan (texture.rs:167-169).  linear_interp selects
 * ImageInterpMethod::Linear (new_raw_image) instead of None. */
int32_t rt_tex_image(rt_scene* s, uint32_t width, uint32_t height, const float* rgba, int32_t linear_interp);
/* ImageTexture::new / new_raw_image (texture.rs:82-97) with the file path
 * given directly (the reference joins RTW_IMAGES or ./assets, image.rs:21-46):
 * the format comes from the extension as ImageReader::open takes it; the
 * library decodes PNG, JPEG and Radiance HDR (rt_image.hpp: the image crate's
 * into_rgba32f, then the sRGB EOTF unless raw or HDR, image.rs:63-82).  A file
 * that is missing, has no image extension, fails to decode or whose decoded
 * buffer would pass the image crate's default 512 MiB allocation limit
 * (ImageReader::decode reserves it first) is the reference's Image::EMPTY
 * (cyan); another image format (GIF, EXR, ...), a CMYK / arithmetic-coded /
 * 12-bit JPEG, or a file within the crate's limit but past this library's
 * 2^28 pixels is RT_EUNSUPPORTED.  raw != 0: no sRGB
 * conversion (new_raw_image); linear_interp selects ImageInterpMethod::Linear. */
int32_t rt_tex_image_file(rt_scene* s, const char* path, int32_t raw, int32_t linear_interp);
/* NoiseTexture::new (texture.rs:183-188).  Perlin tables are drawn from
 * SplitMix64(seed) in the order of perlin.rs:16-36. */
int32_t rt_tex_noise(rt_scene* s, double scale, uint64_t seed);
/* Book-1 sky: a user Texture for Camera.background (camera.rs:50) with
 * value(u,v,p) = (1-a)*horizon + a*zenith, a = (p.y+1)/2, p = unit direction
 * (environment.rs:14-24).  Not a reference type: the reference has no book-1
 * sky, so the build defines it through the Texture trait. */
int32_t rt_tex_sky_gradient(rt_scene* s, const double horizon[3], const double zenith[3]);

/* ---- Materials (src/material.rs) ---------------------------------------- */
int32_t rt_mat_empty(rt_scene* s);                                         /* EmptyMaterial 36-47 */
int32_t rt_mat_lambertian(rt_scene* s, int32_t tex);                       /* Lambertian::new 53-57 */
int32_t rt_mat_metal(rt_scene* s, const double albedo[3], double fuzz);   /* Metal::new 73-80 */
int32_t rt_mat_dielectric(rt_scene* s, int32_t tex, double ior);          /* Dielectric::new 103-108 */
/* DiffuseLight::new / new_with_material (152-169); inner_mat -1 = None */
int32_t rt_mat_diffuse_light(rt_scene* s, int32_t tex, int32_t inner_mat);
int32_t rt_mat_isotropic(rt_scene* s, int32_t tex);                        /* Isotropic::new 193-197 */
int32_t rt_mat_transparent(rt_scene* s);                                   /* Transparent 209-218 */
int32_t rt_mat_mix(rt_scene* s, int32_t mat1, int32_t mat2, double ratio); /* Mix::new 227-233 */
/* Mix::from_image (material.rs:235-247): ratio = the image texture's alpha at
 * (u, v) (ImageTexture::alpha, texture.rs:99-106: 1 for a missing image) */
int32_t rt_mat_mix_image(rt_scene* s, int32_t mat1, int32_t mat2, int32_t image_tex);

/* ---- Hittables ------------------------------------------------------------ */
/* Sphere::new (shapes/sphere.rs:25-35) */
int32_t rt_sphere(rt_scene* s, const double center[3], double radius, int32_t mat);
/* Sphere::new_with_motion (shapes/sphere.rs:37-51) */
int32_t rt_sphere_moving(rt_scene* s, const double center1[3], const double center2[3], double radius, int32_t mat);
/* Quad::new (shapes/quad.rs:30-47) */
int32_t rt_quad(rt_scene* s, const double anchor[3], const double u[3], const double v[3], int32_t mat);
/* Triangle::new (shapes/triangle.rs:28-46); RT_EDEGENERATE where it returns None */
int32_t rt_triangle(rt_scene* s, const double anchor[3], const double u[3], const double v[3], int32_t mat);
/* Hittables::default (hits.rs:9) -- an empty list object */
int32_t rt_hittables_new(rt_scene* s);
/* Hittables::add (hits.rs:27-30); moves `object` */
int32_t rt_hittables_add(rt_scene* s, int32_t list, int32_t object);
/* BVH::new(Hittables) (bvh.rs:12-46); moves `list`.  The reference topology is
 * built; rendering rebuilds it with a binned SAH unless RT_FLAG_REFERENCE_BVH. */
int32_t rt_bvh_new(rt_scene* s, int32_t list);
/* build_box (shapes/quad.rs:128-189); returns a Hittables object */
int32_t rt_build_box(rt_scene* s, const double a[3], const double b[3], int32_t mat);
/* Transform::new (shapes.rs:31-47); moves `object`; null pointers = None
 * (offset 0, identity quaternion (w,x,y,z), scale 1) */
int32_t rt_transform_new(rt_scene* s, int32_t object, const double* offset3, const double* quat_wxyz, const double* scale3);
/* ConstantMedium::new_with_tex (volume.rs:23-33); moves `boundary` */
int32_t rt_constant_medium_new(rt_scene* s, int32_t boundary, double density, int32_t tex);
/* Wavefont::new (shapes/obj.rs:117-134) with the OBJ path given directly (the
 * reference joins RTW_OBJS or ./assets, prefix and file name, obj.rs:86-115;
 * MTL and map_* paths resolve against the OBJ's directory).  tobj
 * GPU_LOAD_OPTIONS semantics; one BVH per loaded model, each triangle under a
 * RemappedMaterial (vertex normals + texture coordinates, obj.rs:20-81).
 * vanilla != 0: Metal / Dielectric from Pm / Tf (obj.rs:289-298); image maps
 * (map_Kd, map_Ke, map_d, map_Bump / normal) are decoded as rt_tex_image_file
 * does (obj.rs:212-345: map_d -> Mix::from_image(Transparent, mat)); Disney
 * materials -> RT_EUNSUPPORTED.  Returns a Hittables object (possibly empty). */
int32_t rt_wavefront_load(rt_scene* s, const char* obj_path, int32_t vanilla);

/* Quaternion::from_axis_angle / from_euler (utils/quaternion.rs:23-53), host helpers */
int32_t rt_quat_from_axis_angle(const double axis[3], double angle_degrees, double out_wxyz[4]);
void rt_quat_from_euler(double yaw, double pitch, double roll, double out_wxyz[4]);

/* ---- Camera (src/camera.rs:45-61 pub fields) ------------------------------ */
typedef struct rt_camera {
    double aspect_ratio;
    uint32_t image_width;
    uint32_t samples_per_pixel; /* traced samples = floor(sqrt(spp))^2 (camera.rs:212) */
    uint32_t max_depth;
    int32_t background_tex; /* Environment texture; -1 = SolidColor(BLACK) (camera.rs:83-85) */
    double vertical_fov_in_degrees;
    double look_from[3];
    double look_at[3];
    double vec_up[3];
    double defocus_angle_in_degrees;
    double focus_distance;
    int32_t toon_map; /* 0 = ToonMap::None, 1 = ToonMap::ACES (utils/color.rs:8-11) */
    int32_t reserved;
} rt_camera;

/* Camera::default (camera.rs:76-104) */
void rt_camera_default(rt_camera* cam);
/* Camera::initilize's image_height (camera.rs:205-210) */
uint32_t rt_camera_image_height(const rt_camera* cam);

typedef struct rt_comm rt_comm;

typedef struct rt_render_opts {
    /* sizeof(rt_render_opts) of the caller's header, set by
     * rt_render_opts_default: the library reads a field only when the
     * caller's struct holds it, and refuses (RT_EINVAL) a size smaller than
     * ABI version 3's -- fields are only ever appended. */
    uint32_t struct_size;
    uint32_t reserved0;
    uint64_t seed;       /* render RNG key (oracle/rng_contract.hpp) */
    uint32_t row_offset; /* shard: render rows y = row_offset + k*row_stride */
    uint32_t row_stride; /* 0 or 1 = every row */
    uint32_t threads;    /* CPU implementations only; 0 = all cores */
    uint32_t flags;      /* RT_FLAG_* */
    void* stream;        /* hipStream_t for rt_render_device (of devices[0] when n_devices > 1); NULL = default */
    /* In-process multi-GPU (replaces the rayon pool, camera.rs:178-197):
     * n_devices > 1 renders the shard's rows interleaved over the HIP devices
     * devices[0..n_devices) -- part k takes the shard rows k, k + n, k + 2n,
     * ... -- one host thread per device (world flatten shared, one upload per
     * device), and gathers the parts onto devices[0] over RCCL (ncclSend /
     * ncclRecv in one group; peer copies when a device repeats in the list).
     * 0 or 1 = the calling thread's current device only. */
    uint32_t n_devices;
    uint32_t reserved;
    const int32_t* devices;
    /* Multi-process (one process per GPU): a communicator from rt_comm_init.
     * Rank r renders the shard rows r, r + nranks, ... on its current device;
     * rank 0 receives the whole shard (RCCL gather), other ranks' outputs are
     * not written.  Exclusive with n_devices > 1. */
    rt_comm* comm;
} rt_render_opts;

/* Keep the reference BVH topology (bvh.rs:16-46: longest axis, sort by box
 * min, median split) instead of the default binned-SAH rebuild of every BVH.
 * Closest-hit results agree up to exact ties in t; used for A/B measurement. */
#define RT_FLAG_REFERENCE_BVH 1u

void rt_render_opts_default(rt_render_opts* opts);

typedef struct rt_stats {
    uint64_t samples;         /* traced camera samples (pixels x floor(sqrt(spp))^2), all devices of this call */
    uint64_t rays;            /* ray_color calls that reached world.hit */
    uint64_t panics;          /* reference assert/expect conditions (NaN, zero pdf, ...) */
    uint64_t n_devices;       /* devices that rendered (1 per rank with a comm) */
    double render_ms;         /* wall time of the call (host) */
    double kernel_ms;         /* device time of the path-tracing kernel (HIP events), max over devices */
    double flatten_ms;        /* world flatten + upload, 0 when cached */
    double gather_ms;         /* device time of the framebuffer gather on devices[0] / rank 0, 0 without one */
} rt_stats;

/* Camera::render(&world, lights) (camera.rs:161-202).  world: object handle;
 * lights: object handle or -1 (None).  Writes the shard's rows, compact and
 * row-major (y down), as linear RGB f32 = pixel_color * pixel_sample_scale
 * (camera.rs:193) to out_linear_rgb (rows x W x 3, may be NULL) and as sRGB u8
 * = Color::to_rgb (utils/color.rs:27-36) to out_srgb (may be NULL).  Blocking.
 * Objects passed here are borrowed, not moved. */
int32_t rt_render(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam, const rt_render_opts* opts,
                  float* out_linear_rgb, uint8_t* out_srgb, rt_stats* stats);

/* What rt_render would upload for (world, lights): host-only, no device needed. */
typedef struct rt_world_info {
    uint64_t device_bytes;    /* size of the flattened world blob */
    uint32_t bvh_nodes;       /* two-box BVH nodes */
    uint32_t primitives;      /* spheres + moving spheres + quads + triangles */
    uint32_t bvh_leaves;      /* objects under BVHs */
    uint32_t stack_need;      /* traversal-stack entries one lane needs */
    uint32_t kernel_tier;     /* 0 = spheres/BVH/basic materials, 1 = + quads/triangles/OBJ, 2 = full */
    uint32_t features;        /* F_* bits (rt_layout.h) */
} rt_world_info;
int32_t rt_world_info_get(rt_scene* s, int32_t world, int32_t lights, int32_t background_tex, uint32_t flags,
                          rt_world_info* out);

/* Number of rows a shard renders (rows of the compact output). */
uint32_t rt_shard_rows(const rt_camera* cam, const rt_render_opts* opts);

/* Device-resident variant: out_linear_rgb_device is a gfx950 device pointer
 * (rows x W x 3 f32; on devices[0] when n_devices > 1; may be NULL on comm
 * ranks other than 0).  Enqueued on opts->stream and returns without waiting;
 * stats (if given) are filled by rt_render_device_wait.  Renders on one scene
 * are ordered: a call's device work starts after the previous call's on the
 * same device has finished (its stream waits on that call's completion
 * event), because they share the scene's per-device work buffers. */
int32_t rt_render_device(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam,
                         const rt_render_opts* opts, float* out_linear_rgb_device);
/* Waits for the last rt_render_device on this scene and reports its stats
 * (an earlier call's stats are superseded by a later call's). */
int32_t rt_render_device_wait(rt_scene* s, rt_stats* stats);
/* How the last render on this scene brought its parts to devices[0] / rank 0
 * (the transfer rt_stats.gather_ms times; the replacement of rayon's join of
 * the pixel iterator, camera.rs:178-197): RT_GATHER_NONE (one part, nothing
 * gathered), RT_GATHER_RCCL_COMM (one ncclSend / ncclRecv group over an
 * rt_comm_init communicator), RT_GATHER_RCCL_DEVICES (one group over the
 * ncclCommInitAll communicators of a device list), RT_GATHER_PEER_COPY
 * (hipMemcpyPeerAsync: a device listed twice, or librccl absent); < 0 when
 * nothing was rendered on the scene. */
#define RT_GATHER_NONE 0
#define RT_GATHER_RCCL_COMM 1
#define RT_GATHER_RCCL_DEVICES 2
#define RT_GATHER_PEER_COPY 3
int32_t rt_render_gather_mode(const rt_scene* s);

/* Test hook (parity tooling, not part of the reference surface): the f64 sum
 * of each (pixel, stratum row s_i) of the last single-device render on this
 * scene -- Sum over s_j of ray_color (camera.rs:183-192) before the 1/spp
 * scale -- laid out [rows x W][sqrt_spp][3].  n_values must equal
 * rows * W * sqrt_spp * 3.  Waits for the render. */
int32_t rt_render_partials_get(rt_scene* s, double* out, uint64_t n_values);

/* Test hook (parity tooling, not part of the reference surface): n calls of
 * one f64 function on the current gfx950 device, from host arrays a (and b)
 * into out.  fn: 0 sin, 1 cos, 2 sincos's sin, 3 sincos's cos, 4 log (ln),
 * 5 acos, 6 atan2(a, b), 7 sqrt, 8 / 9 sin / cos of 2 pi a (a a unit draw,
 * the path's sincos_2pi).  impl 0: the functions the render kernel
 * calls (rt_crmath.h: correctly rounded, in place of Rust's f64::sin / cos /
 * ln / acos / atan2 = glibc's); impl 1: ROCm's device libm (ocml).  Blocking. */
int32_t rt_math_selftest(int32_t fn, int32_t impl, const double* a, const double* b, double* out, uint64_t n);

/* Test hook (host only, not part of the reference surface): builds
 * BVH::from_vec (bvh.rs:16-46) over the children of `list` twice, on copies
 * of the scene -- the parallel builder rt_bvh_new uses and the plain serial
 * recursion -- and returns 1 when the two give the same nodes (ids, children,
 * boxes bit for bit), 0 when they differ, < 0 on a bad argument.  The scene
 * is not modified. */
int32_t rt_bvh_selftest(rt_scene* s, int32_t list);
/* Test hook (host only): flattens (world, lights, background) for rt_render
 * twice -- the binned-SAH rebuild with both halves of large nodes built at
 * once, and serially -- and returns 1 when the flattened worlds agree (nodes,
 * lists, primitives, roots, stack need: bit for bit), 0 when not, < 0 on an
 * error.  The scene is not modified. */
int32_t rt_world_selftest(rt_scene* s, int32_t world, int32_t lights, int32_t background_tex);

/* ---- Multi-process communicator (RCCL) -------------------------------------- */
#define RT_COMM_ID_BYTES 128
/* ncclGetUniqueId: call on rank 0 and hand the bytes to every rank. */
int32_t rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
/* ncclCommInitRank on the calling thread's current HIP device; NULL on failure
 * (rt_last_error). */
rt_comm* rt_comm_init(const uint8_t id[RT_COMM_ID_BYTES], int32_t nranks, int32_t rank);
void rt_comm_destroy(rt_comm* comm);

/* ---- Output stage ---------------------------------------------------------- */
/* Color::to_rgb (utils/color.rs:27-36) of a device-resident linear framebuffer
 * (n_values f32 -> u8, toon_map 0 = None, 1 = ACES), enqueued on `stream`.
 * rt_render's out_srgb is the same conversion made from the f64 pixel sums. */
int32_t rt_to_rgb_device(const float* linear_device, uint8_t* srgb_device, uint64_t n_values, int32_t toon_map,
                         void* stream);
/* img.save(path) with std::fs::create_dir_all of its parent (main.rs:39-47):
 * 8-bit RGB PNG, row-major, y down. */
int32_t rt_write_png(const char* path, uint32_t width, uint32_t height, const uint8_t* rgb);
/* Camera::from_json (camera.rs:119-159) with the path given directly (the
 * reference looks in RTW_IMAGES, then ./assets): the CameraParams fields
 * (camera.rs:33-43) over rt_camera_default; a missing field or a malformed
 * file is RT_EINVAL (the reference's Err). */
int32_t rt_camera_from_json(const char* path, rt_camera* cam);

#ifdef __cplusplus
}
#endif
#endif /* RT_MI355X_H */
