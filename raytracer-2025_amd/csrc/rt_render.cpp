// rt_render.cpp -- render half of the C ABI: Camera::initilize on the host,
// world upload (one device blob per scene, cached until the scene changes),
// and the blocking / stream-ordered render entry points.
#include <chrono>
#include <cstring>
#include <mutex>

#include "../../include/rt_mi355x.h"
#include "rt_kernel.h"
#include "rt_scene.hpp"

namespace rth {

struct DeviceWorld {
    int device = -1;
    int32_t world = -1, lights = -1, background = -1;
    uint64_t generation = ~0ull;
    char* blob = nullptr;
    size_t blob_bytes = 0;
    rtk::SceneView view{};
    size_t n_prims = 0;
    // frame work buffers (grow-only)
    uint32_t* queue = nullptr;
    unsigned long long* stats = nullptr;
    void* params = nullptr;
    double* partial = nullptr;
    size_t partial_bytes = 0;
    float* out = nullptr;
    size_t out_bytes = 0;
    uint8_t* srgb = nullptr;  // to_rgb bytes of the host-path render
    size_t srgb_bytes = 0;
    void* stack_ovf = nullptr;  // mesh tier: traversal-stack entries beyond the LDS part
    size_t stack_ovf_bytes = 0;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    // last async render
    bool pending = false;
    uint64_t pending_samples = 0;
    double pending_flatten_ms = 0;
    std::chrono::steady_clock::time_point pending_t0;
    int grid[rtk::N_TIERS] = {};
    int tier = 1;
    int cus = 0;
    bool reference_bvh = false;
    hipStream_t pending_stream = nullptr;
};

void destroy_device_world(DeviceWorld* d) {
    if (!d) return;
    if (d->blob) (void)hipFree(d->blob);
    if (d->queue) (void)hipFree(d->queue);
    if (d->stats) (void)hipFree(d->stats);
    if (d->params) (void)hipFree(d->params);
    if (d->partial) (void)hipFree(d->partial);
    if (d->out) (void)hipFree(d->out);
    if (d->stack_ovf) (void)hipFree(d->stack_ovf);
    if (d->srgb) (void)hipFree(d->srgb);
    if (d->ev_start) (void)hipEventDestroy(d->ev_start);
    if (d->ev_stop) (void)hipEventDestroy(d->ev_stop);
    delete d;
}

// The kernel tier for a flattened world, with the tier's node format applied:
// the basic and mesh tiers walk 4-wide BVH nodes; a world whose 4-wide nodes
// would need more stack than the tier holds moves up a tier (the basic tier's
// LDS stack -> the mesh tier -> the full tier, whose walk has no fallback:
// -1 with RT_ESTACK set).
static int prepare_tier(HostWorld& hw) {
    int tier = rtk_tier_for(hw.features, hw.stack_need);
    // the basic tier queues sphere indices as 16-bit LDS entries
    if (tier == rtk::TIER_BASIC && hw.spheres.size() > 65536) tier = rtk::TIER_MESH;
    // the basic tier's kernel reads every 4-wide node from its LDS copy
    if (tier == rtk::TIER_BASIC && rtk_basic_bvh4() &&
        bvh4_convert(hw, RT_STACK_BASIC, true, RT_NODE_LDS_BYTES / sizeof(rtk::DNode4)) > RT_STACK_BASIC)
        tier = rtk::TIER_MESH;
    if (tier == rtk::TIER_MESH && rtk_mesh_bvh4() && bvh4_convert(hw, RT_STACK_MAX, false) > RT_STACK_MAX)
        tier = rtk::TIER_FULL;
    if (tier == rtk::TIER_FULL && hw.nodes.empty()) return rtk::TIER_FULL_FLAT;
    if (tier == rtk::TIER_FULL && rtk_full_bvh4()) {
        const uint32_t need = bvh4_convert(hw, RT_STACK_MAX, false);
        if (need > RT_STACK_MAX) {
            set_error(RT_ESTACK, "world needs " + std::to_string(need) + " traversal-stack entries, kernel has " +
                                     std::to_string(RT_STACK_MAX));
            return -1;
        }
    }
    return tier;
}

static int32_t hip_fail(hipError_t e, const char* what) {
    return set_error(RT_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
static size_t put(std::vector<char>& blob, const std::vector<T>& v) {
    size_t off = (blob.size() + 255) & ~(size_t)255;
    blob.resize(off + v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

// Checks there is a gfx950 device and binds the scene's device world to it,
// flattening + uploading when (world, lights, background, scene) changed.
static int32_t prepare(rt_scene* s, int32_t world, int32_t lights, int32_t bg, bool reference_bvh, double& flatten_ms) {
    flatten_ms = 0;
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice (no HIP device)");
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(RT_EDEVICE, std::string("librt_mi355x.so needs a gfx950 device, found ") + prop.gcnArchName);
    DeviceWorld* d = s->dev;
    if (d && d->device != dev) {
        destroy_device_world(d);
        s->dev = d = nullptr;
    }
    if (!d) {
        d = new DeviceWorld();
        d->device = dev;
        s->dev = d;
        if ((e = hipMalloc(&d->queue, 256)) != hipSuccess) return hip_fail(e, "hipMalloc queue");
        if ((e = hipMalloc(&d->stats, 256)) != hipSuccess) return hip_fail(e, "hipMalloc stats");
        if ((e = hipMalloc(&d->params, rtk_params_bytes())) != hipSuccess) return hip_fail(e, "hipMalloc params");
        if ((e = hipEventCreate(&d->ev_start)) != hipSuccess) return hip_fail(e, "hipEventCreate");
        if ((e = hipEventCreate(&d->ev_stop)) != hipSuccess) return hip_fail(e, "hipEventCreate");
        for (int t = 0; t < rtk::N_TIERS; ++t) {
            int bpc = 0;
            if ((e = (hipError_t)rtk_path_kernel_occupancy(t, &bpc)) != hipSuccess) return hip_fail(e, "occupancy query");
            if (bpc < 1) bpc = 1;
            d->grid[t] = bpc * prop.multiProcessorCount;
        }
        d->cus = prop.multiProcessorCount;
    }
    if (d->blob && d->world == world && d->lights == lights && d->background == bg && d->generation == s->generation &&
        d->reference_bvh == reference_bvh)
        return RT_OK;
    auto t0 = std::chrono::steady_clock::now();
    HostWorld hw;
    int32_t rc = flatten(s, world, lights, bg, reference_bvh, hw);
    if (rc != RT_OK) return rc;
    const int tier = prepare_tier(hw);
    if (tier < 0) return RT_ESTACK;
    const uint32_t stack_cap = rtk_stack_entries(tier);
    if (hw.stack_need > stack_cap)
        return set_error(RT_ESTACK, "world needs " + std::to_string(hw.stack_need) + " traversal-stack entries, kernel has " +
                                        std::to_string(stack_cap));
    const uint32_t lds_entries = rtk::lds_stack_entries(tier);
    if (hw.stack_need > lds_entries) {
        const size_t need = (size_t)(hw.stack_need - lds_entries) * d->grid[tier] * RT_BLOCK * sizeof(uint64_t);
        if (need > d->stack_ovf_bytes) {
            if (d->stack_ovf) (void)hipFree(d->stack_ovf);
            d->stack_ovf = nullptr;
            d->stack_ovf_bytes = 0;
            if ((e = hipMalloc(&d->stack_ovf, need)) != hipSuccess) return hip_fail(e, "hipMalloc stack overflow");
            d->stack_ovf_bytes = need;
        }
    }
    std::vector<char> blob;
    size_t o_nodes = put(blob, hw.nodes), o_n4 = put(blob, hw.nodes4), o_sph = put(blob, hw.spheres), o_sphm = put(blob, hw.sphere_mat),
           o_msc = put(blob, hw.msph_center), o_msd = put(blob, hw.msph_dir), o_msm = put(blob, hw.msph_mat),
           o_pl = put(blob, hw.planars), o_pla = put(blob, hw.planar_area), o_plm = put(blob, hw.planar_mat),
           o_plr = put(blob, hw.planar_remap), o_rm = put(blob, hw.remaps),
           o_rnm = put(blob, (hw.features & rtk::F_NORMALMAP) ? hw.remap_nm : std::vector<rtk::DRemapNM>()),
           o_lc = put(blob, hw.list_children), o_xf = put(blob, hw.xforms), o_md = put(blob, hw.media),
           o_mat = put(blob, hw.materials), o_tex = put(blob, hw.textures), o_tx = put(blob, hw.texels),
           o_per = put(blob, hw.perlin);
    if (d->blob) {
        (void)hipFree(d->blob);
        d->blob = nullptr;
    }
    if ((e = hipMalloc(&d->blob, blob.size() + 256)) != hipSuccess) return hip_fail(e, "hipMalloc world");
    if ((e = hipMemcpy(d->blob, blob.data(), blob.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy world");
    char* b = d->blob;
    rtk::SceneView& v = d->view;
    v.nodes = (const rtk::DNode*)(b + o_nodes);
    v.nodes4 = (const rtk::DNode4*)(b + o_n4);
    v.spheres = (const double4*)(b + o_sph);
    v.sphere_mat = (const int32_t*)(b + o_sphm);
    v.msph_center = (const double4*)(b + o_msc);
    v.msph_dir = (const double4*)(b + o_msd);
    v.msph_mat = (const int32_t*)(b + o_msm);
    v.planars = (const rtk::DPlanar*)(b + o_pl);
    v.planar_area = (const double*)(b + o_pla);
    v.planar_mat = (const int32_t*)(b + o_plm);
    v.planar_remap = (const int32_t*)(b + o_plr);
    v.remaps = (const rtk::DRemap*)(b + o_rm);
    v.remap_nm = (const rtk::DRemapNM*)(b + o_rnm);
    v.list_children = (const uint32_t*)(b + o_lc);
    v.xforms = (const rtk::DXform*)(b + o_xf);
    v.media = (const rtk::DMedium*)(b + o_md);
    v.materials = (const rtk::DMaterial*)(b + o_mat);
    v.textures = (const rtk::DTexture*)(b + o_tex);
    v.texels = (const float*)(b + o_tx);
    v.perlin = (const rtk::DPerlin*)(b + o_per);
    v.world_root = hw.world_root;
    v.lights_root = hw.lights_root;
    v.background_tex = bg;
    v.stack_need = hw.stack_need;
    v.features = hw.features;
    v.n_nodes4 = (uint32_t)hw.nodes4.size();
    d->tier = tier;
    d->reference_bvh = reference_bvh;
    d->blob_bytes = blob.size();
    d->n_prims = hw.n_prims;
    d->world = world;
    d->lights = lights;
    d->background = bg;
    d->generation = s->generation;
    flatten_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

// Camera::initilize (camera.rs:204-245)
static int32_t init_frame(const rt_camera* c, const rt_render_opts* o, rtk_frame_desc& f) {
    if (!c) return set_error(RT_EINVAL, "null camera");
    if (c->image_width == 0 || !(c->aspect_ratio > 0)) return set_error(RT_EINVAL, "bad image size");
    const double PI = 3.14159265358979323846;
    const uint32_t W = c->image_width, H = rt_camera_image_height(c);
    std::memset(&f, 0, sizeof f);
    f.W = W;
    f.row_stride = (o && o->row_stride > 1) ? o->row_stride : 1;
    f.row_offset = o ? o->row_offset : 0;
    f.rows = rt_shard_rows(c, o);
    f.S = (uint32_t)std::sqrt((double)c->samples_per_pixel);
    f.max_depth = c->max_depth;
    f.seed = o ? o->seed : 1;
    f.pixel_sample_scale = 1.0 / (double)(f.S * f.S);
    f.recip_sqrt_spp = 1.0 / (double)f.S;
    if ((uint64_t)W * f.rows * f.S >= 0xFFF00000ull) return set_error(RT_EINVAL, "frame too large for one launch");
    V3 from(c->look_from), at(c->look_at), up(c->vec_up);
    double theta = c->vertical_fov_in_degrees * (PI / 180.0);
    double h = std::tan(theta / 2.0);
    double vh = 2.0 * h * c->focus_distance;
    double vw = vh * ((double)W / (double)H);
    V3 w = div(from - at, length(from - at));
    if (!finite(w)) return set_error(RT_EPANIC, "Camera axis w should be normalizable!");
    V3 uc = cross(up, w);
    V3 u = div(uc, length(uc));
    if (!finite(u)) return set_error(RT_EPANIC, "Camera axis u should be normalizable!");
    V3 v = cross(w, u);
    V3 vu = vw * u, vv = vh * (-v);
    V3 du = div(vu, (double)W), dv = div(vv, (double)H);
    V3 ul = ((from - c->focus_distance * w) - div(vu, 2.0)) - div(vv, 2.0);
    V3 p00 = ul + 0.5 * (du + dv);
    double radius = c->focus_distance * std::tan((c->defocus_angle_in_degrees / 2.0) * (PI / 180.0));
    V3 disk_u = radius * u, disk_v = radius * v;
    auto cp = [](double* dst, V3 x) {
        dst[0] = x.x;
        dst[1] = x.y;
        dst[2] = x.z;
    };
    cp(f.center, from);
    cp(f.pixel00, p00);
    cp(f.du, du);
    cp(f.dv, dv);
    cp(f.disk_u, disk_u);
    cp(f.disk_v, disk_v);
    f.defocus = c->defocus_angle_in_degrees > 0.0 ? 1 : 0;
    return RT_OK;
}

static int32_t ensure_buffers(DeviceWorld* d, const rtk_frame_desc& f, bool need_out) {
    hipError_t e;
    size_t pb = (size_t)f.W * f.rows * f.S * 3 * sizeof(double);
    if (pb > d->partial_bytes) {
        if (d->partial) (void)hipFree(d->partial);
        d->partial = nullptr;
        d->partial_bytes = 0;
        if ((e = hipMalloc(&d->partial, pb)) != hipSuccess) return hip_fail(e, "hipMalloc partial sums");
        d->partial_bytes = pb;
    }
    size_t ob = (size_t)f.W * f.rows * 3 * sizeof(float);
    if (need_out && ob > d->out_bytes) {
        if (d->out) (void)hipFree(d->out);
        d->out = nullptr;
        d->out_bytes = 0;
        if ((e = hipMalloc(&d->out, ob)) != hipSuccess) return hip_fail(e, "hipMalloc output");
        d->out_bytes = ob;
    }
    return RT_OK;
}

static int32_t launch(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam, const rt_render_opts* opts,
                      float* dev_out, hipStream_t stream, bool want_srgb = false) {
    if (!s) return set_error(RT_EINVAL, "null scene");
    if (world < 0 || (size_t)world >= s->objs.size() || s->objs[world].hidden)
        return set_error(RT_EHANDLE, "unknown world handle");
    if (s->objs[world].moved) return set_error(RT_EMOVED, "world handle was moved");
    if (lights != -1) {
        if (lights < 0 || (size_t)lights >= s->objs.size() || s->objs[lights].hidden)
            return set_error(RT_EHANDLE, "unknown lights handle");
        if (s->objs[lights].moved) return set_error(RT_EMOVED, "lights handle was moved");
    }
    rtk_frame_desc f;
    int32_t rc = init_frame(cam, opts, f);
    if (rc != RT_OK) return rc;
    if (cam->background_tex != -1 && (cam->background_tex < 0 || (size_t)cam->background_tex >= s->texs.size()))
        return set_error(RT_EHANDLE, "unknown background texture");
    double flatten_ms = 0;
    const bool reference_bvh = opts && (opts->flags & RT_FLAG_REFERENCE_BVH);
    if ((rc = prepare(s, world, lights, cam->background_tex, reference_bvh, flatten_ms)) != RT_OK) return rc;
    DeviceWorld* d = s->dev;
    if ((rc = ensure_buffers(d, f, dev_out == nullptr)) != RT_OK) return rc;
    hipError_t e = hipMemsetAsync(d->stats, 0, 2 * sizeof(unsigned long long), stream);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync stats");
    f.ev_start = d->ev_start;
    f.ev_stop = d->ev_stop;
    d->pending_t0 = std::chrono::steady_clock::now();
    d->pending_stream = stream;
    float* out = dev_out ? dev_out : d->out;
    const bool run = f.rows > 0 && f.max_depth > 0;
    if (run) {
        uint8_t* srgb = nullptr;
        if (want_srgb) {
            const size_t nb = (size_t)f.W * f.rows * 3;
            if (nb > d->srgb_bytes) {
                if (d->srgb) (void)hipFree(d->srgb);
                d->srgb = nullptr;
                d->srgb_bytes = 0;
                if ((e = hipMalloc(&d->srgb, nb)) != hipSuccess) return hip_fail(e, "hipMalloc srgb");
                d->srgb_bytes = nb;
            }
            srgb = d->srgb;
        }
        e = rtk_launch_frame(&d->view, &f, d->queue, d->partial, d->stats, out, srgb, cam->toon_map, stream, d->tier,
                             d->grid[d->tier], d->params, d->stack_ovf);
        if (e != hipSuccess) return hip_fail(e, "kernel launch");
    } else if (f.rows > 0) {
        // max_depth == 0: every ray_color returns BLACK (camera.rs:282-284)
        e = hipMemsetAsync(out, 0, (size_t)f.W * f.rows * 3 * sizeof(float), stream);
        if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync output");
    }
    d->pending = run;
    d->pending_samples = (uint64_t)f.W * f.rows * f.S * f.S;
    d->pending_flatten_ms = flatten_ms;
    return RT_OK;
}

static int32_t wait(rt_scene* s, rt_stats* st) {
    DeviceWorld* d = s ? s->dev : nullptr;
    if (st) std::memset(st, 0, sizeof(*st));
    if (!d) return set_error(RT_EINVAL, "nothing rendered on this scene");
    hipError_t e = hipStreamSynchronize(d->pending_stream);
    if (e != hipSuccess) return hip_fail(e, "render (stream synchronize)");
    unsigned long long h[2] = {0, 0};
    if ((e = hipMemcpy(h, d->stats, sizeof h, hipMemcpyDeviceToHost)) != hipSuccess) return hip_fail(e, "stats copy");
    float ms = 0;
    if (d->pending) (void)hipEventElapsedTime(&ms, d->ev_start, d->ev_stop);
    if (st) {
        st->samples = d->pending_samples;
        st->rays = h[0];
        st->panics = h[1];
        st->kernel_ms = ms;
        st->flatten_ms = d->pending_flatten_ms;
        st->render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d->pending_t0).count();
    }
    d->pending = false;
    if (h[1]) return set_error(RT_EPANIC, std::to_string(h[1]) + " path(s) hit a reference panic condition "
                                                                "(NaN radiance, zero pdf, non-normalizable vector)");
    return RT_OK;
}

}  // namespace rth

using namespace rth;

extern "C" {

int32_t rt_render_device(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam, const rt_render_opts* opts,
                         float* out_dev) {
    if (!out_dev) return set_error(RT_EINVAL, "null device output");
    try {
        return launch(s, world, lights, cam, opts, out_dev, opts ? (hipStream_t)opts->stream : nullptr);
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
}

int32_t rt_world_info_get(rt_scene* s, int32_t world, int32_t lights, int32_t bg, uint32_t flags, rt_world_info* out) {
    if (!s || !out) return set_error(RT_EINVAL, "null argument");
    if (world < 0 || (size_t)world >= s->objs.size() || s->objs[world].hidden)
        return set_error(RT_EHANDLE, "unknown world handle");
    try {
        HostWorld hw;
        int32_t rc = flatten(s, world, lights, bg, (flags & RT_FLAG_REFERENCE_BVH) != 0, hw);
        if (rc != RT_OK) return rc;
        std::vector<char> blob;
        put(blob, hw.nodes), put(blob, hw.spheres), put(blob, hw.sphere_mat), put(blob, hw.msph_center),
            put(blob, hw.msph_dir), put(blob, hw.msph_mat), put(blob, hw.planars), put(blob, hw.planar_area),
            put(blob, hw.planar_mat), put(blob, hw.list_children), put(blob, hw.xforms), put(blob, hw.media),
            put(blob, hw.materials), put(blob, hw.textures), put(blob, hw.texels), put(blob, hw.perlin);
        out->device_bytes = blob.size();
        out->bvh_nodes = (uint32_t)hw.nodes.size();
        out->primitives = (uint32_t)hw.n_prims;
        out->bvh_leaves = (uint32_t)hw.n_bvh_leaves;
        const int tier = prepare_tier(hw);
        if (tier < 0) return RT_ESTACK;
        if (!hw.nodes4.empty()) out->bvh_nodes = (uint32_t)hw.nodes4.size();
        out->stack_need = hw.stack_need;
        out->kernel_tier = (uint32_t)tier;
        out->features = hw.features;
        return RT_OK;
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
}

int32_t rt_render_device_wait(rt_scene* s, rt_stats* st) {
    return wait(s, st);
}

int32_t rt_to_rgb_device(const float* lin_dev, uint8_t* srgb_dev, uint64_t n_values, int32_t toon_map, void* stream) {
    if (n_values && (!lin_dev || !srgb_dev)) return set_error(RT_EINVAL, "null argument");
    hipError_t e = rtk_launch_to_rgb(lin_dev, srgb_dev, n_values, toon_map, (hipStream_t)stream);
    return e == hipSuccess ? RT_OK : hip_fail(e, "to_rgb launch");
}

int32_t rt_render(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam, const rt_render_opts* opts,
                  float* out_lin, uint8_t* out_srgb, rt_stats* st) {
    try {
        hipStream_t stream = opts ? (hipStream_t)opts->stream : nullptr;
        const uint32_t rows = rt_shard_rows(cam, opts);
        const size_t n = (size_t)cam->image_width * rows * 3;
        const bool srgb_dev = out_srgb && cam->max_depth > 0;  // else every pixel is BLACK -> 0
        int32_t rc = launch(s, world, lights, cam, opts, nullptr, stream, srgb_dev);
        if (rc != RT_OK) return rc;
        DeviceWorld* d = s->dev;
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail(e, "render");
        if (n && out_lin && (e = hipMemcpy(out_lin, d->out, n * sizeof(float), hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "hipMemcpy output");
        if (n && out_srgb) {
            if (srgb_dev) {
                if ((e = hipMemcpy(out_srgb, d->srgb, n, hipMemcpyDeviceToHost)) != hipSuccess)
                    return hip_fail(e, "hipMemcpy srgb");
            } else {
                std::memset(out_srgb, 0, n);
            }
        }
        return wait(s, st);
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
}

}  // extern "C"
