// rt_render.cpp -- render half of the C ABI: Camera::initilize on the host,
// world upload (one device blob per scene and device, cached until the scene
// changes), the blocking / stream-ordered render entry points, and the
// multi-GPU row split with its one framebuffer gather (RCCL over xGMI).
//
// The reference renders with rayon over pixels (camera.rs:178-197).  Here a
// render is split into parts, one per device: part k of n takes the shard's
// rows k, k + n, ... (row interleave, so sky and ground rows balance) and
// renders them with the persistent path kernel of its device.  With n > 1 the
// parts' compact rows are gathered onto the root device (devices[0], or comm
// rank 0) by ncclSend / ncclRecv in one group and re-interleaved there by one
// small kernel -- the only exchange of the frame.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <map>
#include <thread>

#include <rccl/rccl.h>

#include "../../include/rt_mi355x.h"
#include "rt_kernel.h"
#include "rt_scene.hpp"

// ---------------------------------------------------------------------------- RCCL
// librccl is opened on first use (a single-GPU render never loads it).
// Check build only (make check, -DRT_CHECK): RT_RCCL_LIB names another library
// with librccl's point-to-point ABI instead -- the test-only stand-in
// tests/cpp/fake_rccl.cpp, with which one process on one GPU runs the
// nranks > 1 gathers (tests/test_gather_standin_gpu.py).  The product library
// reads no such variable: it opens librccl and nothing else.  Each library is
// opened once; a communicator keeps the API it was made with.
namespace {
struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

RcclApi& rccl() {
    static std::mutex m;
    static std::map<std::string, RcclApi*>* apis = new std::map<std::string, RcclApi*>();  // never freed
#ifdef RT_CHECK
    const char* env = std::getenv("RT_RCCL_LIB");
    const std::string path = env ? env : "";
#else
    const std::string path;
#endif
    std::lock_guard<std::mutex> lk(m);
    auto it = apis->find(path);
    if (it != apis->end()) return *it->second;
    RcclApi* ap = new RcclApi();
    (*apis)[path] = ap;
    RcclApi& a = *ap;
    void* h = nullptr;
    if (!path.empty()) {
        h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    } else {
        h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    }
    if (!h) {
        const char* e = dlerror();
        a.err = "cannot load " + (path.empty() ? std::string("librccl") : path) + ": " + (e ? e : "?");
        return a;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        if (!fn) {
            all = false;
            a.err = std::string("librccl lacks ") + name;
        }
    };
    sym(a.get_unique_id, "ncclGetUniqueId");
    sym(a.comm_init_rank, "ncclCommInitRank");
    sym(a.comm_init_all, "ncclCommInitAll");
    sym(a.comm_destroy, "ncclCommDestroy");
    sym(a.send, "ncclSend");
    sym(a.recv, "ncclRecv");
    sym(a.group_start, "ncclGroupStart");
    sym(a.group_end, "ncclGroupEnd");
    sym(a.error_string, "ncclGetErrorString");
    a.ok = all;
    return a;
}
}  // namespace

struct rt_comm {
    RcclApi* api = nullptr;  // the library the communicator was made with
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = -1;
    // held from ncclGroupStart to ncclGroupEnd: two scenes gathering through
    // one communicator from two threads enqueue their groups one after the
    // other, never interleaved (RCCL matches a communicator's sends and
    // receives in enqueue order)
    std::mutex group;
};

namespace rth {

// The calling thread's current device, restored on scope exit: the library
// switches devices for the parts and the gather but leaves the caller's as it was.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

struct DeviceWorld {
    int device = -1;
    int32_t world = -1, lights = -1, background = -1;
    uint64_t generation = ~0ull;
    bool reference_bvh = false;
    char* blob = nullptr;
    size_t blob_bytes = 0;
    rtk::SceneView view{};
    int tier = 1;
    int grid[rtk::N_TIERS] = {};
    int cus = 0;
    // frame work buffers (grow-only)
    uint32_t* queue = nullptr;
    unsigned long long* stats = nullptr;
    void* params = nullptr;
    double* partial = nullptr;
    size_t partial_bytes = 0;
    float* out = nullptr;  // the part's compact rows when they are not written to the caller's buffer
    size_t out_bytes = 0;
    uint8_t* srgb = nullptr;  // to_rgb bytes of the host-path render
    size_t srgb_bytes = 0;
    void* stack_ovf = nullptr;  // mesh / full tiers: traversal-stack entries beyond the LDS part
    size_t stack_ovf_bytes = 0;
    hipStream_t own_stream = nullptr;  // for parts that do not run on the caller's stream
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    hipEvent_t ev_done = nullptr;  // after the slot's last device work (orders the next render)
    bool done_recorded = false;
    // the last render on this slot
    bool ran = false;  // the path kernel ran (ev_start / ev_stop are valid)
    uint64_t samples = 0;
    uint32_t W = 0, rows = 0, S = 0, parts = 1, whole_rows = 0, parts2 = 1, fine_row = 0;
    hipStream_t last_stream = nullptr;
};

struct RenderState {
    std::vector<DeviceWorld*> slots;  // slot k renders part k; slot 0 also serves single-device renders
    // gather buffers on the root device
    int root_device = -1;
    float* staging = nullptr;
    size_t staging_bytes = 0;
    uint8_t* staging_srgb = nullptr;  // the parts' to_rgb bytes, gathered like their f32 rows
    size_t staging_srgb_bytes = 0;
    float* full = nullptr;  // gathered frame of a host-buffer render
    size_t full_bytes = 0;
    uint8_t* full_srgb = nullptr;
    size_t full_srgb_bytes = 0;
    hipEvent_t g_start = nullptr, g_stop = nullptr;
    bool g_recorded = false;
    // ncclCommInitAll communicators of the last device list with distinct devices
    std::vector<int> comm_devices;
    std::shared_ptr<struct CommSet> comm_set;
    // the last render
    int n_parts = 0;
    bool gathered = false;
    int gather_mode = RT_GATHER_NONE;  // rt_render_gather_mode
    bool pending = false;
    bool is_root = true;
    hipStream_t root_stream = nullptr;
    double flatten_ms = 0;
    std::chrono::steady_clock::time_point t0;
};

static void destroy_device_world(DeviceWorld* d) {
    if (!d) return;
    if (d->device >= 0) (void)hipSetDevice(d->device);
    if (d->own_stream) (void)hipStreamSynchronize(d->own_stream);
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
    if (d->ev_done) (void)hipEventDestroy(d->ev_done);
    if (d->own_stream) (void)hipStreamDestroy(d->own_stream);
    delete d;
}

static void free_root_buffers(RenderState* r) {
    if (r->root_device >= 0) (void)hipSetDevice(r->root_device);
    if (r->staging) (void)hipFree(r->staging);
    if (r->staging_srgb) (void)hipFree(r->staging_srgb);
    if (r->full) (void)hipFree(r->full);
    if (r->full_srgb) (void)hipFree(r->full_srgb);
    if (r->g_start) (void)hipEventDestroy(r->g_start);
    if (r->g_stop) (void)hipEventDestroy(r->g_stop);
    r->staging = r->full = nullptr;
    r->full_srgb = r->staging_srgb = nullptr;
    r->staging_bytes = r->full_bytes = r->full_srgb_bytes = r->staging_srgb_bytes = 0;
    r->g_start = r->g_stop = nullptr;
    r->g_recorded = false;
    r->root_device = -1;
}

// ncclCommInitAll communicators are process-wide, one set per device list,
// shared by every scene that renders on that list and kept until the process
// exits: building a set is slow, and scenes (or calls) that alternate device
// lists would otherwise rebuild them each time.  A set is used by one gather
// at a time: the gather holds the set's `group` lock from ncclGroupStart to
// ncclGroupEnd, so that scenes rendering on the same device list from
// different threads (rt_mi355x.h: different scenes may be used from
// different threads) enqueue whole groups one after the other -- RCCL matches
// a communicator's sends and receives in enqueue order, and interleaved
// groups could hang or swap two scenes' rows.
struct CommSet {
    std::mutex group;
    RcclApi* api = nullptr;
    std::vector<ncclComm_t> comms;
};
struct CommCache {
    std::mutex m;  // the map only
    std::map<std::pair<RcclApi*, std::vector<int>>, std::shared_ptr<CommSet>> sets;
};
static CommCache& comm_cache() {
    static CommCache* c = new CommCache();  // never destroyed: RCCL may already be torn down at exit
    return *c;
}
static int32_t nccl_fail(const RcclApi& nc, ncclResult_t e, const char* what);
static int32_t acquire_comms(RenderState* r, RcclApi& nc, const std::vector<int>& devs) {
    if (r->comm_devices == devs && r->comm_set && r->comm_set->api == &nc) return RT_OK;
    CommCache& cc = comm_cache();
    std::lock_guard<std::mutex> lk(cc.m);
    const auto key = std::make_pair(&nc, devs);
    auto it = cc.sets.find(key);
    if (it == cc.sets.end()) {
        auto set = std::make_shared<CommSet>();
        set->api = &nc;
        set->comms.assign(devs.size(), nullptr);
        const ncclResult_t ne = nc.comm_init_all(set->comms.data(), (int)devs.size(), devs.data());
        if (ne != ncclSuccess) return nccl_fail(nc, ne, "ncclCommInitAll");
        it = cc.sets.emplace(key, std::move(set)).first;
    }
    r->comm_set = it->second;
    r->comm_devices = devs;
    return RT_OK;
}
static void destroy_comms(RenderState* r) {  // the scene lets go of its cached set
    r->comm_set.reset();
    r->comm_devices.clear();
}

void destroy_render_state(RenderState* r) {
    if (!r) return;
    DeviceGuard g;
    (void)hipDeviceSynchronize();
    destroy_comms(r);
    for (DeviceWorld* d : r->slots) destroy_device_world(d);
    free_root_buffers(r);
    delete r;
}

// The kernel tier for a flattened world, with the tier's node format applied:
// the basic and mesh tiers walk 4-wide BVH nodes; a world whose 4-wide nodes
// would need more stack than the tier holds moves up a tier (the basic tier's
// LDS stack -> the mesh tier -> the full tier, whose walk has no fallback:
// -1 with RT_ESTACK set).
static int prepare_tier(HostWorld& hw) {
    int tier = rtk_tier_for(hw.features, hw.stack_need);
    // the basic tier's walk words hold 15-bit sphere indices (rt_kernel.hip bword)
    if (tier == rtk::TIER_BASIC && hw.spheres.size() > 32768) tier = rtk::TIER_MESH;
    // and its 4-B stack entries hold 15-bit node / list indices
    if (tier == rtk::TIER_BASIC && hw.list_children.size() >= 32768) tier = rtk::TIER_MESH;
    // the basic tier's kernel reads every 4-wide node from its LDS copy
    if (tier == rtk::TIER_BASIC && rtk_basic_bvh4() &&
        bvh4_convert(hw, RT_STACK_BASIC, true, RT_NODE_LDS_BYTES / sizeof(rtk::DNode4)) > RT_STACK_BASIC)
        tier = rtk::TIER_MESH;
    if (tier == rtk::TIER_MESH && rtk_mesh_bvh4() && bvh4_convert(hw, RT_STACK_MAX, false) > RT_STACK_MAX)
        tier = rtk::TIER_FULL;
    if (tier == rtk::TIER_FULL && hw.nodes.empty()) return rtk::TIER_FULL_FLAT;
    if (rtk::tier_full_bvh(tier) && rtk_full_bvh4()) {
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

// The world of one render flattened once on the host and shared by every
// device that needs an upload (built by the first part that needs it).
struct FlatWorld {
    std::mutex m;
    bool done = false;
    int32_t rc = RT_OK;
    std::string err;
    double ms = 0;
    int tier = 1;
    uint32_t stack_need = 0;
    std::vector<char> blob;
    rtk::SceneView rel{};  // SceneView with byte offsets into blob instead of pointers
    size_t n_prims = 0;
};

static int32_t build_flat(rt_scene* s, int32_t world, int32_t lights, int32_t bg, bool reference_bvh, FlatWorld& fw) {
    std::lock_guard<std::mutex> lk(fw.m);
    if (fw.done) {
        if (fw.rc != RT_OK) set_error(fw.rc, fw.err);
        return fw.rc;
    }
    fw.done = true;
    auto t0 = std::chrono::steady_clock::now();
    HostWorld hw;
    int32_t rc = flatten(s, world, lights, bg, reference_bvh, hw);
    int tier = rc == RT_OK ? prepare_tier(hw) : -1;
    if (rc == RT_OK && tier < 0) rc = RT_ESTACK;
#ifdef RT_CHECK
    // check build only: RT_CHECK_INJECT=1 makes every node slot that names a
    // primitive name a record past its array -- the kind of fault the check
    // is for (a bad relayout once did this silently); tests/test_check_gpu.py
    // expects the render to report it
    if (rc == RT_OK && std::getenv("RT_CHECK_INJECT") && std::getenv("RT_CHECK_INJECT")[0] == '1') {
        for (rtk::DNode4& nd : hw.nodes4)
            for (int k = 0; k < 4; ++k) {
                const uint32_t kind = rtk::ref_kind(nd.ref[k]);
                const size_t n = kind == rtk::K_SPHERE ? hw.spheres.size()
                                 : (kind == rtk::K_QUAD || kind == rtk::K_TRI) ? hw.planars.size() : 0;
                if (n) nd.ref[k] = rtk::make_ref(kind, (uint32_t)n + rtk::ref_index(nd.ref[k]));
            }
    }
#endif
    if (rc == RT_OK) {
        const uint32_t stack_cap = rtk_stack_entries(tier);
        if (hw.stack_need > stack_cap)
            rc = set_error(RT_ESTACK, "world needs " + std::to_string(hw.stack_need) +
                                          " traversal-stack entries, kernel has " + std::to_string(stack_cap));
    }
    if (rc != RT_OK) {
        fw.rc = rc;
        fw.err = rt_last_error();
        return rc;
    }
    std::vector<char>& blob = fw.blob;
    auto off = [](size_t o) { return (uintptr_t)o; };
    rtk::SceneView& v = fw.rel;
    v.nodes = (const rtk::DNode*)off(put(blob, hw.nodes));
    v.nodes4 = (const rtk::DNode4*)off(put(blob, hw.nodes4));
    v.spheres = (const double4*)off(put(blob, hw.spheres));
    v.sphere_mat = (const int32_t*)off(put(blob, hw.sphere_mat));
    v.sphere_rinv = (const double*)off(put(blob, hw.sphere_rinv));
    v.msph_center = (const double4*)off(put(blob, hw.msph_center));
    v.msph_dir = (const double4*)off(put(blob, hw.msph_dir));
    v.msph_mat = (const int32_t*)off(put(blob, hw.msph_mat));
    v.planars = (const rtk::DPlanar*)off(put(blob, hw.planars));
    v.planars_f = (const rtk::PlanarF*)off(put(blob, hw.planars_f));
    v.planar_area = (const double*)off(put(blob, hw.planar_area));
    v.planar_mat = (const int32_t*)off(put(blob, hw.planar_mat));
    v.planar_remap = (const int32_t*)off(put(blob, hw.planar_remap));
    v.remaps = (const rtk::DRemap*)off(put(blob, hw.remaps));
    v.remap_nm = (const rtk::DRemapNM*)off(
        put(blob, (hw.features & rtk::F_NORMALMAP) ? hw.remap_nm : std::vector<rtk::DRemapNM>()));
    v.list_children = (const uint32_t*)off(put(blob, hw.list_children));
    v.list_boxes = (const rtk::DBoxF*)off(put(blob, hw.list_boxes));
    v.xforms = (const rtk::DXform*)off(put(blob, hw.xforms));
    v.media = (const rtk::DMedium*)off(put(blob, hw.media));
    v.materials = (const rtk::DMaterial*)off(put(blob, hw.materials));
    v.textures = (const rtk::DTexture*)off(put(blob, hw.textures));
    v.texels = (const float*)off(put(blob, hw.texels));
    v.perlin = (const rtk::DPerlin*)off(put(blob, hw.perlin));
    // the mesh tier reads 128 B from any record's address (rt_kernel.hip
    // unified_load): slack past the last array
    blob.resize(((blob.size() + 255) & ~(size_t)255) + 256, 0);
    v.world_root = hw.world_root;
    v.lights_root = hw.lights_root;
    v.background_tex = bg;
    v.bg_kind = rtk::BG_NONE;
    std::memset(v.bg_c0, 0, sizeof v.bg_c0);
    std::memset(v.bg_c1, 0, sizeof v.bg_c1);
    if (bg >= 0 && (size_t)bg < hw.textures.size()) {
        const rtk::DTexture& t = hw.textures[bg];
        v.bg_kind = t.type == rtk::T_SKY ? rtk::BG_SKY : rtk::BG_OTHER;
        if (v.bg_kind == rtk::BG_SKY)
            for (int k = 0; k < 3; ++k) v.bg_c0[k] = t.color[k], v.bg_c1[k] = t.color2[k];
    }
    v.stack_need = hw.stack_need;
    v.features = hw.features;
    v.n_nodes4 = (uint32_t)hw.nodes4.size();
    v.n_perlin = (uint32_t)hw.perlin.size();
    std::memset(v.n_ref, 0, sizeof v.n_ref);
    v.n_ref[rtk::K_BVH] = (uint32_t)std::max(hw.nodes4.size(), hw.nodes.size());
    v.n_ref[rtk::K_LIST] = (uint32_t)hw.list_children.size();
    v.n_ref[rtk::K_SPHERE] = (uint32_t)hw.spheres.size();
    v.n_ref[rtk::K_MSPHERE] = (uint32_t)hw.msph_center.size();
    v.n_ref[rtk::K_QUAD] = v.n_ref[rtk::K_TRI] = (uint32_t)hw.planars.size();
    v.n_ref[rtk::K_XFORM] = (uint32_t)hw.xforms.size();
    v.n_ref[rtk::K_MEDIUM] = (uint32_t)hw.media.size();
    v.n_ref[rtk::K_POPXF] = 1;  // the marker's index is 0
    fw.tier = tier;
    fw.stack_need = hw.stack_need;
    fw.n_prims = hw.n_prims;
    fw.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

// A slot's device world on `device` (the thread's current device), created on
// first use (work buffers, events, stream, the grid of each tier).
static int32_t slot_for(RenderState* r, size_t k, int device, DeviceWorld*& out) {
    DeviceWorld* d = r->slots[k];
    if (d && d->device != device) {
        destroy_device_world(d);
        r->slots[k] = d = nullptr;
        (void)hipSetDevice(device);
    }
    if (d) {
        out = d;
        return RT_OK;
    }
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(RT_EDEVICE, std::string("librt_mi355x.so needs a gfx950 device, found ") + prop.gcnArchName);
    d = new DeviceWorld();
    d->device = device;
    r->slots[k] = d;
    if ((e = hipMalloc(&d->queue, 256)) != hipSuccess) return hip_fail(e, "hipMalloc queue");
    if ((e = hipMalloc(&d->stats, 256)) != hipSuccess) return hip_fail(e, "hipMalloc stats");
    if ((e = hipMalloc(&d->params, rtk_params_bytes())) != hipSuccess) return hip_fail(e, "hipMalloc params");
    if ((e = hipEventCreate(&d->ev_start)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    if ((e = hipEventCreate(&d->ev_stop)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&d->ev_done, hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e, "hipEventCreate");
    if ((e = hipStreamCreateWithFlags(&d->own_stream, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(e, "hipStreamCreate");
    for (int t = 0; t < rtk::N_TIERS; ++t) {
        int bpc = 0;
        if ((e = (hipError_t)rtk_path_kernel_occupancy(t, &bpc)) != hipSuccess) return hip_fail(e, "occupancy query");
        if (bpc < 1) bpc = 1;
        d->grid[t] = bpc * prop.multiProcessorCount;
    }
    d->cus = prop.multiProcessorCount;
    out = d;
    return RT_OK;
}

// Uploads the world to the slot's device unless it already holds this
// (world, lights, background, scene generation, topology).
static int32_t upload_world(rt_scene* s, DeviceWorld* d, int32_t world, int32_t lights, int32_t bg, bool reference_bvh,
                            FlatWorld& fw, double& flatten_ms) {
    flatten_ms = 0;
    if (d->blob && d->world == world && d->lights == lights && d->background == bg && d->generation == s->generation &&
        d->reference_bvh == reference_bvh)
        return RT_OK;
    auto t0 = std::chrono::steady_clock::now();
    int32_t rc = build_flat(s, world, lights, bg, reference_bvh, fw);
    if (rc != RT_OK) return rc;
    hipError_t e;
    const uint32_t lds_entries = rtk::lds_stack_entries(fw.tier);
    if (fw.stack_need > lds_entries) {
        const int blocks = d->grid[fw.tier];
        const size_t need = (size_t)(fw.stack_need - lds_entries) * blocks * RT_BLOCK * sizeof(uint64_t);
        if (need > d->stack_ovf_bytes) {
            if (d->stack_ovf) (void)hipFree(d->stack_ovf);
            d->stack_ovf = nullptr;
            d->stack_ovf_bytes = 0;
            if ((e = hipMalloc(&d->stack_ovf, need)) != hipSuccess) return hip_fail(e, "hipMalloc stack overflow");
            d->stack_ovf_bytes = need;
        }
    }
    if (d->blob) {
        (void)hipFree(d->blob);
        d->blob = nullptr;
    }
    d->world = -1;  // invalid until the upload completes
    if ((e = hipMalloc(&d->blob, fw.blob.size() + 256)) != hipSuccess) return hip_fail(e, "hipMalloc world");
    if ((e = hipMemcpy(d->blob, fw.blob.data(), fw.blob.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy world");
    char* b = d->blob;
    rtk::SceneView v = fw.rel;
    auto fix = [b](auto& p) { p = reinterpret_cast<std::remove_reference_t<decltype(p)>>(b + (uintptr_t)p); };
    fix(v.nodes), fix(v.nodes4), fix(v.spheres), fix(v.sphere_mat), fix(v.sphere_rinv), fix(v.msph_center), fix(v.msph_dir),
        fix(v.msph_mat), fix(v.planars), fix(v.planars_f), fix(v.planar_area), fix(v.planar_mat), fix(v.planar_remap), fix(v.remaps),
        fix(v.remap_nm), fix(v.list_children), fix(v.list_boxes), fix(v.xforms), fix(v.media), fix(v.materials), fix(v.textures),
        fix(v.texels), fix(v.perlin);
    d->view = v;
    d->tier = fw.tier;
    d->reference_bvh = reference_bvh;
    d->blob_bytes = fw.blob.size();
    d->world = world;
    d->lights = lights;
    d->background = bg;
    d->generation = s->generation;
    flatten_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

// Camera::initilize (camera.rs:204-245) for the rows y = row_offset + k * row_stride
static int32_t init_frame(const rt_camera* c, uint64_t seed, uint32_t row_offset, uint32_t row_stride,
                          rtk_frame_desc& f) {
    if (!c) return set_error(RT_EINVAL, "null camera");
    if (c->image_width == 0 || !(c->aspect_ratio > 0)) return set_error(RT_EINVAL, "bad image size");
    const double PI = 3.14159265358979323846;
    const uint32_t W = c->image_width, H = rt_camera_image_height(c);
    std::memset(&f, 0, sizeof f);
    f.W = W;
    f.row_stride = row_stride > 1 ? row_stride : 1;
    f.row_offset = row_offset;
    f.rows = row_offset >= H ? 0 : (H - row_offset + f.row_stride - 1) / f.row_stride;
    f.S = (uint32_t)std::sqrt((double)c->samples_per_pixel);
    f.max_depth = c->max_depth;
    f.seed = seed;
    f.pixel_sample_scale = 1.0 / (double)(f.S * f.S);
    f.recip_sqrt_spp = 1.0 / (double)f.S;
    if ((uint64_t)W * f.rows * f.S >= 0xFFF00000ull) return set_error(RT_EINVAL, "frame too large for one launch");
    if (W >= (1u << 20)) return set_error(RT_EINVAL, "image_width must be below 2^20");
    if (f.S >= (1u << 16)) return set_error(RT_EINVAL, "samples_per_pixel must be below 2^32");
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

static int32_t grow(void** p, size_t& have, size_t need, const char* what) {
    if (need <= have) return RT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    have = 0;
    hipError_t e = hipMalloc(p, need);
    if (e != hipSuccess) return hip_fail(e, what);
    have = need;
    return RT_OK;
}

// One part of a render: rows row_offset + k * row_stride on one device.
struct Part {
    size_t slot = 0;
    int device = -1;
    uint32_t row_offset = 0, row_stride = 1;
    bool user_stream = false;  // part 0 runs on the caller's stream (NULL = the default stream)
    hipStream_t stream = nullptr;
    float* out = nullptr;  // nullptr: the slot's own buffer
    bool want_srgb = false;
    // results
    DeviceWorld* d = nullptr;
    float* out_used = nullptr;
    uint32_t rows = 0;
    int32_t rc = RT_OK;
    std::string err;
    double flatten_ms = 0;
};

// A tuning knob from the environment (A/B runs), else its default.
static uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    char* end = nullptr;
    const unsigned long x = std::strtoul(v, &end, 10);
    return (end && *end == 0 && x <= 0xFFFFFFFFul) ? (uint32_t)x : dflt;
}

// Runs on the part's host thread: device world, buffers, kernel launch.
static void run_part(rt_scene* s, RenderState* r, int32_t world, int32_t lights, const rt_camera* cam, uint64_t seed,
                     bool reference_bvh, FlatWorld& fw, Part& p) {
    auto fail = [&](int32_t rc) {
        p.rc = rc;
        p.err = rt_last_error();
    };
    hipError_t e = hipSetDevice(p.device);
    if (e != hipSuccess) return fail(hip_fail(e, "hipSetDevice"));
    int32_t rc = slot_for(r, p.slot, p.device, p.d);
    if (rc != RT_OK) return fail(rc);
    DeviceWorld* d = p.d;
    if (!p.user_stream) p.stream = d->own_stream;
    if ((rc = upload_world(s, d, world, lights, cam->background_tex, reference_bvh, fw, p.flatten_ms)) != RT_OK)
        return fail(rc);
    rtk_frame_desc f;
    if ((rc = init_frame(cam, seed, p.row_offset, p.row_stride, f)) != RT_OK) return fail(rc);
    p.rows = f.rows;
    // The stratum rows of the frame's last RT_TAIL_PERMILLE / 1000 image rows
    // (half; the mesh tier 0.65: C4 frame -0.5 % and worst 1/8 shard -2.3 %
    // against half, profiles/r05/tail_sweep_c4.jsonl -- for C2 and C3 a longer
    // tail costs the one-GPU frame 0.2-0.4 %) go out in parts of about
    // RT_PART_SAMPLES (4; the mesh tier 2) samples, every other
    // row as one queue entry (rtk_row_parts, rtk_tail_rows; decided on the
    // whole frame, so shards and device counts sum rows alike): a launch ends
    // on short queue entries, since each shard's tail rows are its last.
    // One f64 sum per queue entry: the part-sum buffer (held per scene and
    // device slot, grow-only, freed with the scene) is one sum per stratum
    // row plus the tail's extra parts, those within RT_PART_BUDGET_MB (4 GiB)
    // and 1/64 of the device's memory.  A device that cannot allocate it
    // renders whole rows only (parts = 1): the same samples, the tail rows'
    // f64 sums then in one run instead of part sums added in order (~1 ulp).
    // (DESIGN.md §4 "Tail rows": C2 at a tail of 1/4, 1/2 and the whole frame.)
    const uint32_t H = rt_camera_image_height(cam);
    uint64_t budget = (uint64_t)env_u32("RT_PART_BUDGET_MB", 4096) << 20;
    size_t mem_free = 0, mem_total = 0;
    if (hipMemGetInfo(&mem_free, &mem_total) == hipSuccess && mem_total) budget = std::min<uint64_t>(budget, mem_total / 64);
    // The tail's last RT_FINE_PERMILLE / 1000 image rows (3 %) go out in
    // parts of about RT_FINE_SAMPLES (1) samples: what is in flight when the
    // queue runs dry is then one sample a lane, not a 4-sample part
    // (DESIGN.md §4 "Fine rows").  The mesh tier's tail parts are 2 samples:
    // its samples are long (dependent global loads per walk step), C4's 1/8
    // shard 25.5 -> 24.5 ms and frame -1 %; C2 keeps 4 (its shard +2 % at 2).
    f.parts = rtk_row_parts(f.S, env_u32("RT_PART_SAMPLES", d->tier == rtk::TIER_MESH ? 2 : 4));
    f.parts2 = rtk_row_parts(f.S, env_u32("RT_FINE_SAMPLES", 1));
    uint32_t tail = 0, fine = 0;
    rtk_tail_split(f.W, H, f.S, f.parts, f.parts2, budget, env_u32("RT_TAIL_PERMILLE", d->tier == rtk::TIER_MESH ? 650 : 500),
                   env_u32("RT_FINE_PERMILLE", 30), &tail, &fine);
    if (tail == 0) f.parts = 1;
    if (fine == 0) f.parts2 = f.parts;
    // the shard's rows above the tail (image rows row_offset + r * row_stride
    // < H - tail), and above the fine rows
    f.whole_rows = rtk_shard_whole_rows(H, tail, f.row_offset, f.row_stride, f.rows);
    f.fine_row = rtk_shard_whole_rows(H, fine, f.row_offset, f.row_stride, f.rows);
    // guided chunks of at least 64 entries, one per lane of the wave (DESIGN §4
    // "Tail rows": C2 -0.4 % frame, -2.3 % worst 1/8 shard; C3 -0.3 %; C4 +-0)
    f.chunk_min = env_u32("RT_CHUNK_MIN", 64);
    f.chunk_cap = env_u32("RT_CHUNK_CAP", 0);  // A/B knobs (0: the kernel's defaults)
    f.guide = env_u32("RT_CHUNK_GUIDE", 0);
    f.chunk_min_whole = env_u32("RT_CHUNK_MIN_WHOLE", 0);
    auto part_sums = [&f]() {
        const size_t fr = std::max(f.fine_row, f.whole_rows);
        return ((size_t)f.W * f.whole_rows * f.S + (size_t)f.W * (fr - f.whole_rows) * f.S * f.parts +
                (size_t)f.W * (f.rows - fr) * f.S * f.parts2) *
               3 * sizeof(double);
    };
    rc = grow((void**)&d->partial, d->partial_bytes, part_sums(), "hipMalloc partial sums");
    if (rc != RT_OK && f.parts > 1) {
        (void)hipGetLastError();
        f.parts = f.parts2 = 1;
        f.whole_rows = f.fine_row = f.rows;
        rc = grow((void**)&d->partial, d->partial_bytes, part_sums(), "hipMalloc partial sums (whole rows)");
    }
    if (rc != RT_OK) return fail(rc);
    if (!p.out &&
        (rc = grow((void**)&d->out, d->out_bytes, (size_t)f.W * f.rows * 3 * sizeof(float), "hipMalloc output")) != RT_OK)
        return fail(rc);
    uint8_t* srgb = nullptr;
    if (p.want_srgb) {
        if ((rc = grow((void**)&d->srgb, d->srgb_bytes, (size_t)f.W * f.rows * 3, "hipMalloc srgb")) != RT_OK)
            return fail(rc);
        srgb = d->srgb;
    }
    // order after the previous render's use of this slot's buffers, and after
    // the gather that read them
    if (d->done_recorded && (e = hipStreamWaitEvent(p.stream, d->ev_done, 0)) != hipSuccess)
        return fail(hip_fail(e, "hipStreamWaitEvent"));
    if (r->g_recorded && (e = hipStreamWaitEvent(p.stream, r->g_stop, 0)) != hipSuccess)
        return fail(hip_fail(e, "hipStreamWaitEvent"));
    if ((e = hipMemsetAsync(d->stats, 0, 2 * sizeof(unsigned long long), p.stream)) != hipSuccess)
        return fail(hip_fail(e, "hipMemsetAsync stats"));
    f.ev_start = d->ev_start;
    f.ev_stop = d->ev_stop;
    float* out = p.out ? p.out : d->out;
    p.out_used = out;
    const bool run = f.rows > 0 && f.max_depth > 0;
    if (run) {
        e = rtk_launch_frame(&d->view, &f, d->queue, d->partial, d->stats, out, srgb, cam->toon_map, p.stream, d->tier,
                             d->grid[d->tier], d->params, d->stack_ovf);
        if (e != hipSuccess) return fail(hip_fail(e, "kernel launch"));
    } else if (f.rows > 0) {
        // max_depth == 0: every ray_color returns BLACK (camera.rs:282-284)
        if ((e = hipMemsetAsync(out, 0, (size_t)f.W * f.rows * 3 * sizeof(float), p.stream)) != hipSuccess)
            return fail(hip_fail(e, "hipMemsetAsync output"));
        if (srgb && (e = hipMemsetAsync(srgb, 0, (size_t)f.W * f.rows * 3, p.stream)) != hipSuccess)
            return fail(hip_fail(e, "hipMemsetAsync srgb"));
    }
    if ((e = hipEventRecord(d->ev_done, p.stream)) != hipSuccess) return fail(hip_fail(e, "hipEventRecord"));
    d->done_recorded = true;
    d->ran = run;
    d->samples = (uint64_t)f.W * f.rows * f.S * f.S;
    d->W = f.W;
    d->rows = f.rows;
    d->S = f.S;
    d->parts = f.parts;
    d->whole_rows = f.parts > 1 ? f.whole_rows : f.rows;
    d->parts2 = f.parts > 1 ? f.parts2 : 1u;
    d->fine_row = f.parts > 1 ? std::max(f.fine_row, d->whole_rows) : f.rows;
    d->last_stream = p.stream;
}

static int32_t nccl_fail(const RcclApi& nc, ncclResult_t e, const char* what) {
    return set_error(RT_EDEVICE, std::string(what) + ": " + nc.error_string(e));
}

// Root-side buffers of a gather on the current (root) device.
static int32_t root_buffers(RenderState* r, int device, size_t staging_bytes, size_t full_bytes, size_t srgb_bytes) {
    if (r->root_device != device) {
        free_root_buffers(r);
        (void)hipSetDevice(device);
        r->root_device = device;
    }
    hipError_t e;
    if (!r->g_start && (e = hipEventCreate(&r->g_start)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    if (!r->g_stop && (e = hipEventCreate(&r->g_stop)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    int32_t rc;
    if ((rc = grow((void**)&r->staging, r->staging_bytes, staging_bytes, "hipMalloc gather staging")) != RT_OK) return rc;
    if ((rc = grow((void**)&r->full, r->full_bytes, full_bytes, "hipMalloc gathered frame")) != RT_OK) return rc;
    if ((rc = grow((void**)&r->full_srgb, r->full_srgb_bytes, srgb_bytes, "hipMalloc gathered srgb")) != RT_OK)
        return rc;
    const size_t srgb_staging = srgb_bytes ? staging_bytes / sizeof(float) : 0;
    if ((rc = grow((void**)&r->staging_srgb, r->staging_srgb_bytes, srgb_staging, "hipMalloc gather srgb staging")) !=
        RT_OK)
        return rc;
    return RT_OK;
}

// Rows of part k of n of a shard with `rows` compact rows (rows k, k+n, ...).
static inline uint32_t part_rows(uint32_t rows, uint32_t k, uint32_t n) { return k >= rows ? 0 : (rows - k + n - 1) / n; }

static int32_t validate(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam) {
    if (!s) return set_error(RT_EINVAL, "null scene");
    if (!cam) return set_error(RT_EINVAL, "null camera");
    if (world < 0 || (size_t)world >= s->objs.size() || s->objs[world].hidden)
        return set_error(RT_EHANDLE, "unknown world handle");
    if (s->objs[world].moved) return set_error(RT_EMOVED, "world handle was moved");
    if (lights != -1) {
        if (lights < 0 || (size_t)lights >= s->objs.size() || s->objs[lights].hidden)
            return set_error(RT_EHANDLE, "unknown lights handle");
        if (s->objs[lights].moved) return set_error(RT_EMOVED, "lights handle was moved");
    }
    if (cam->background_tex != -1 && (cam->background_tex < 0 || (size_t)cam->background_tex >= s->texs.size()))
        return set_error(RT_EHANDLE, "unknown background texture");
    return RT_OK;
}

// Enqueues one render (all parts, and the gather when there is more than one
// part).  dev_out: the caller's device buffer (root), or nullptr for the
// library's own (rt_render).  On return the render's state is in s->rs.
static int32_t launch(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam, const rt_render_opts* opts,
                      float* dev_out, bool host_call, bool want_srgb) {
    int32_t rc = validate(s, world, lights, cam);
    if (rc != RT_OK) return rc;
    if (opts && opts->struct_size < sizeof(rt_render_opts))  // ABI 3 holds every field read below
        return set_error(RT_EINVAL, "rt_render_opts.struct_size is " + std::to_string(opts->struct_size) +
                                        ", ABI version 3 needs " + std::to_string(sizeof(rt_render_opts)) +
                                        ": initialise the options with rt_render_opts_default");
    const uint64_t seed = opts ? opts->seed : 1;
    const uint32_t off = opts ? opts->row_offset : 0;
    const uint32_t stride = (opts && opts->row_stride > 1) ? opts->row_stride : 1;
    rtk_frame_desc f_all;
    if ((rc = init_frame(cam, seed, off, stride, f_all)) != RT_OK) return rc;
    rt_comm* comm = opts ? opts->comm : nullptr;
    const uint32_t nd = (opts && opts->n_devices > 1) ? opts->n_devices : 1;
    if (comm && nd > 1) return set_error(RT_EINVAL, "opts.comm and opts.n_devices > 1 are exclusive");
    if (nd > 1 && !opts->devices) return set_error(RT_EINVAL, "n_devices > 1 without a device list");
    if (comm && (comm->rank < 0 || comm->rank >= comm->nranks)) return set_error(RT_EINVAL, "bad communicator");
    const bool reference_bvh = opts && (opts->flags & RT_FLAG_REFERENCE_BVH);
    hipStream_t user_stream = opts ? (hipStream_t)opts->stream : nullptr;
    // every rank of a host-buffer render sends its to_rgb bytes (the root's
    // out_srgb decides nothing the other ranks could see)
    if (comm && host_call) want_srgb = true;

    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice (no HIP device)");
    if (comm && comm->device != cur) return set_error(RT_EINVAL, "communicator belongs to another device");
    if (!s->rs) s->rs = new RenderState();
    RenderState* r = s->rs;
    DeviceGuard guard;

    const uint32_t n_parts = comm ? (uint32_t)comm->nranks : nd;
    // with a communicator the frame always goes through the RCCL group (a
    // one-rank communicator sends to itself), so every rank count runs one path
    const bool gather = n_parts > 1 || comm;
    const bool is_root = !comm || comm->rank == 0;
    std::vector<Part> parts(comm ? 1 : nd);
    for (size_t i = 0; i < parts.size(); ++i) {
        Part& p = parts[i];
        const uint32_t k = comm ? (uint32_t)comm->rank : (uint32_t)i;
        p.slot = i;
        p.device = comm ? cur : (nd > 1 ? opts->devices[i] : cur);
        p.row_offset = off + k * stride;
        p.row_stride = stride * n_parts;
        p.user_stream = i == 0;
        p.stream = (i == 0) ? user_stream : nullptr;
        p.out = gather ? nullptr : dev_out;  // gathered parts render into the slot's buffer
        // every part makes its rows' to_rgb bytes from the f64 pixel sums, as
        // the reference converts its f64 colour (color.rs:27-36); a gathered
        // frame's bytes are those parts' bytes, not a conversion of its f32
        // values, so they do not depend on the device count
        p.want_srgb = want_srgb;
    }
    if (r->slots.size() < parts.size()) r->slots.resize(parts.size(), nullptr);
    FlatWorld fw;
    r->pending = false;
    r->t0 = std::chrono::steady_clock::now();
    if (parts.size() == 1) {
        run_part(s, r, world, lights, cam, seed, reference_bvh, fw, parts[0]);
    } else {
        // one host thread per device: uploads and launches proceed in parallel
        std::vector<std::thread> th;
        for (size_t i = 1; i < parts.size(); ++i)
            th.emplace_back(run_part, s, r, world, lights, cam, seed, reference_bvh, std::ref(fw), std::ref(parts[i]));
        run_part(s, r, world, lights, cam, seed, reference_bvh, fw, parts[0]);
        for (auto& t : th) t.join();
    }
    // On any failure after the parts started: wait for the parts that did
    // enqueue work (their buffers may be reused right away), and leave the
    // scene in the "nothing rendered" state, not the previous render's.
    auto abort_render = [&](int32_t code) {
        const std::string msg = rt_last_error();
        for (Part& p : parts)
            if (p.d && p.d->device >= 0 && hipSetDevice(p.d->device) == hipSuccess)
                (void)hipStreamSynchronize(p.stream);  // own stream, or the caller's (NULL: the default stream)
        r->n_parts = 0;
        r->pending = false;
        r->gathered = false;
        r->gather_mode = RT_GATHER_NONE;
        return set_error(code, msg);
    };
    double flatten_ms = 0;
    for (Part& p : parts) {
        if (p.rc != RT_OK) {
            set_error(p.rc, p.err);
            return abort_render(p.rc);
        }
        flatten_ms = std::max(flatten_ms, p.flatten_ms);
    }
    r->n_parts = (int)parts.size();
    r->gathered = gather;
    r->gather_mode = RT_GATHER_NONE;
    r->is_root = is_root;
    r->flatten_ms = flatten_ms;
    r->root_stream = parts[0].stream;
    if (gather) {
        // ---- the framebuffer gather onto the root (one RCCL group)
        Part& root = parts[0];
        const uint32_t W = f_all.W, rows = f_all.rows;
        const size_t slice = (size_t)part_rows(rows, 0, n_parts) * W * 3;  // part 0 has the most rows
        const size_t row_floats = (size_t)W * 3;
        // a communicator's own library; a device list's, the current one
        RcclApi& nc = comm ? *comm->api : rccl();
        if ((e = hipSetDevice(root.device)) != hipSuccess) return abort_render(hip_fail(e, "hipSetDevice"));
        hipStream_t rs = root.stream;
        if (is_root) {
            const size_t full = (dev_out ? 0 : rows * row_floats * sizeof(float));
            const size_t srgb = want_srgb ? rows * row_floats : 0;
            if ((rc = root_buffers(r, root.device, n_parts * slice * sizeof(float), full, srgb)) != RT_OK) return abort_render(rc);
            if ((e = hipEventRecord(r->g_start, rs)) != hipSuccess) return abort_render(hip_fail(e, "hipEventRecord"));
        }
        bool distinct = true;
        for (uint32_t i = 0; i < nd && !comm; ++i)
            for (uint32_t j = i + 1; j < nd; ++j) distinct = distinct && opts->devices[i] != opts->devices[j];
#ifdef RT_CHECK
        // check build only: RT_CHECK_RCCL_DUPS=1 sends a device list with a
        // repeated device through the RCCL group too (real RCCL refuses two
        // ranks on one device; the test stand-in of RT_RCCL_LIB accepts them),
        // so the one-GPU box runs the distinct-device gather's sends,
        // receives and slice offsets (tests/test_gather_standin_gpu.py)
        if (!comm && std::getenv("RT_CHECK_RCCL_DUPS") && std::getenv("RT_CHECK_RCCL_DUPS")[0] == '1') distinct = true;
#endif
        if (comm) {
            if (!nc.ok) return abort_render(set_error(RT_EDEVICE, nc.err));
            r->gather_mode = RT_GATHER_RCCL_COMM;
            std::lock_guard<std::mutex> glk(comm->group);  // the whole group, enqueued at once
            ncclResult_t ne = nc.group_start();
            if (ne == ncclSuccess)
                ne = nc.send(root.out_used, (size_t)root.rows * row_floats, ncclFloat32, 0, comm->comm, rs);
            if (ne == ncclSuccess && want_srgb)
                ne = nc.send(root.d->srgb, (size_t)root.rows * row_floats, ncclUint8, 0, comm->comm, rs);
            if (ne == ncclSuccess && is_root)
                for (uint32_t q = 0; q < n_parts && ne == ncclSuccess; ++q) {
                    const size_t n_q = (size_t)part_rows(rows, q, n_parts) * row_floats;
                    ne = nc.recv(r->staging + q * slice, n_q, ncclFloat32, (int)q, comm->comm, rs);
                    if (ne == ncclSuccess && want_srgb)
                        ne = nc.recv(r->staging_srgb + q * slice, n_q, ncclUint8, (int)q, comm->comm, rs);
                }
            const ncclResult_t ge = nc.group_end();
            if (ne != ncclSuccess) return abort_render(nccl_fail(nc, ne, "ncclSend/ncclRecv"));
            if (ge != ncclSuccess) return abort_render(nccl_fail(nc, ge, "ncclGroupEnd"));
        } else if (distinct && nc.ok) {
            const std::vector<int> devs(opts->devices, opts->devices + nd);
            if ((rc = acquire_comms(r, nc, devs)) != RT_OK) return abort_render(rc);
            CommSet& cs = *r->comm_set;
            r->gather_mode = RT_GATHER_RCCL_DEVICES;
            std::lock_guard<std::mutex> glk(cs.group);  // the whole group, enqueued at once
            ncclResult_t ne = nc.group_start();
            for (uint32_t k = 0; k < nd && ne == ncclSuccess; ++k) {
                ne = nc.send(parts[k].out_used, (size_t)parts[k].rows * row_floats, ncclFloat32, 0, cs.comms[k],
                             parts[k].stream);
                if (ne == ncclSuccess && want_srgb)
                    ne = nc.send(parts[k].d->srgb, (size_t)parts[k].rows * row_floats, ncclUint8, 0, cs.comms[k],
                                 parts[k].stream);
            }
            for (uint32_t k = 0; k < nd && ne == ncclSuccess; ++k) {
                ne = nc.recv(r->staging + k * slice, (size_t)parts[k].rows * row_floats, ncclFloat32, (int)k,
                             cs.comms[0], rs);
                if (ne == ncclSuccess && want_srgb)
                    ne = nc.recv(r->staging_srgb + k * slice, (size_t)parts[k].rows * row_floats, ncclUint8, (int)k,
                                 cs.comms[0], rs);
            }
            const ncclResult_t ge = nc.group_end();
            if (ne != ncclSuccess) return abort_render(nccl_fail(nc, ne, "ncclSend/ncclRecv"));
            if (ge != ncclSuccess) return abort_render(nccl_fail(nc, ge, "ncclGroupEnd"));
        } else {
            // a device listed twice (one communicator per device is all RCCL
            // allows) or no librccl: peer copies onto the root
            r->gather_mode = RT_GATHER_PEER_COPY;
            for (uint32_t k = 0; k < nd; ++k) {
                if (!parts[k].rows) continue;
                if ((e = hipStreamWaitEvent(rs, parts[k].d->ev_done, 0)) != hipSuccess)
                    return abort_render(hip_fail(e, "hipStreamWaitEvent"));
                if ((e = hipMemcpyPeerAsync(r->staging + k * slice, root.device, parts[k].out_used, parts[k].device,
                                            (size_t)parts[k].rows * row_floats * sizeof(float), rs)) != hipSuccess)
                    return abort_render(hip_fail(e, "hipMemcpyPeerAsync"));
                if (want_srgb &&
                    (e = hipMemcpyPeerAsync(r->staging_srgb + k * slice, root.device, parts[k].d->srgb, parts[k].device,
                                            (size_t)parts[k].rows * row_floats, rs)) != hipSuccess)
                    return abort_render(hip_fail(e, "hipMemcpyPeerAsync srgb"));
            }
        }
        if (is_root) {
            float* frame = dev_out ? dev_out : r->full;
            if ((e = rtk_launch_deinterleave(r->staging, slice, frame, rows, W, n_parts, rs)) != hipSuccess)
                return abort_render(hip_fail(e, "deinterleave launch"));
            if (want_srgb &&
                (e = rtk_launch_deinterleave_u8(r->staging_srgb, slice, r->full_srgb, rows, W, n_parts, rs)) != hipSuccess)
                return abort_render(hip_fail(e, "deinterleave launch"));
            if ((e = hipEventRecord(r->g_stop, rs)) != hipSuccess) return abort_render(hip_fail(e, "hipEventRecord"));
            r->g_recorded = true;
        }
        // the root's slot is reused only after the gather read it
        if ((e = hipEventRecord(root.d->ev_done, rs)) != hipSuccess) return abort_render(hip_fail(e, "hipEventRecord"));
    }
    r->pending = true;
    return RT_OK;
}

// check build only (make check): the kernel's count of decoded refs past
// their arrays on the current device (rt_kernel.hip ref_idx); absent from
// the product library
extern "C" __attribute__((weak)) int rtk_check_read(unsigned long long* out, int reset);

static int32_t wait(rt_scene* s, rt_stats* st) {
    RenderState* r = s ? s->rs : nullptr;
    if (st) std::memset(st, 0, sizeof(*st));
    if (!r || r->n_parts == 0) return set_error(RT_EINVAL, "nothing rendered on this scene");
    DeviceGuard guard;
    uint64_t rays = 0, panics = 0, samples = 0;
    double kernel_ms = 0;
    hipError_t e;
    for (int k = 0; k < r->n_parts; ++k) {
        DeviceWorld* d = r->slots[k];
        (void)hipSetDevice(d->device);
        if ((e = hipStreamSynchronize(d->last_stream)) != hipSuccess) return hip_fail(e, "render (stream synchronize)");
        unsigned long long h[2] = {0, 0};
        if ((e = hipMemcpy(h, d->stats, sizeof h, hipMemcpyDeviceToHost)) != hipSuccess) return hip_fail(e, "stats copy");
        rays += h[0];
        panics += h[1];
        if (rtk_check_read) {
            unsigned long long c[2] = {0, 0};
            if ((e = (hipError_t)rtk_check_read(c, 1)) != hipSuccess) return hip_fail(e, "check counters");
            if (c[0]) {
                const uint32_t bad = (uint32_t)c[1];
                r->pending = false;
                return set_error(RT_EPANIC, "check build: " + std::to_string(c[0]) +
                                                " decoded ref(s) past their array (first: kind " +
                                                std::to_string(rtk::ref_kind(bad)) + ", index " +
                                                std::to_string(rtk::ref_index(bad)) + ")");
            }
        }
        samples += d->samples;
        float ms = 0;
        if (d->ran) (void)hipEventElapsedTime(&ms, d->ev_start, d->ev_stop);
        kernel_ms = std::max(kernel_ms, (double)ms);
    }
    float gms = 0;
    if (r->gathered && r->is_root) {
        (void)hipSetDevice(r->root_device);
        if ((e = hipStreamSynchronize(r->root_stream)) != hipSuccess) return hip_fail(e, "gather (stream synchronize)");
        (void)hipEventElapsedTime(&gms, r->g_start, r->g_stop);
    }
    if (st) {
        st->samples = samples;
        st->rays = rays;
        st->panics = panics;
        st->n_devices = (uint64_t)r->n_parts;
        st->kernel_ms = kernel_ms;
        st->flatten_ms = r->flatten_ms;
        st->gather_ms = gms;
        st->render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r->t0).count();
    }
    r->pending = false;
    if (panics) return set_error(RT_EPANIC, std::to_string(panics) + " path(s) hit a reference panic condition "
                                                                     "(NaN radiance, zero pdf, non-normalizable vector)");
    return RT_OK;
}

}  // namespace rth

using namespace rth;

extern "C" {

int32_t rt_render_device(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam, const rt_render_opts* opts,
                         float* out_dev) {
    const bool root = !(opts && opts->comm) || opts->comm->rank == 0;
    if (!out_dev && root) return set_error(RT_EINVAL, "null device output");
    try {
        return launch(s, world, lights, cam, opts, out_dev, false, false);
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
        put(blob, hw.nodes), put(blob, hw.spheres), put(blob, hw.sphere_mat), put(blob, hw.sphere_rinv),
            put(blob, hw.msph_center),
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

int32_t rt_render_gather_mode(const rt_scene* s) {
    const RenderState* r = s ? s->rs : nullptr;
    if (!r || r->n_parts == 0) return set_error(RT_EINVAL, "nothing rendered on this scene");
    return r->gather_mode;
}

int32_t rt_render_partials_get(rt_scene* s, double* out, uint64_t n_values) {
    RenderState* r = s ? s->rs : nullptr;
    if (!r || r->n_parts != 1 || r->gathered || !r->slots[0])
        return set_error(RT_EINVAL, "no single-device render on this scene");
    DeviceWorld* d = r->slots[0];
    const uint64_t n = (uint64_t)d->W * d->rows * d->S * 3;
    if (n_values != n) return set_error(RT_EINVAL, "n_values must be rows * W * sqrt_spp * 3 = " + std::to_string(n));
    if (!d->ran) return set_error(RT_EINVAL, "the last render traced no samples");
    if (n && !out) return set_error(RT_EINVAL, "null output");
    DeviceGuard guard;
    (void)hipSetDevice(d->device);
    hipError_t e = hipStreamSynchronize(d->last_stream);
    if (e != hipSuccess) return hip_fail(e, "render (stream synchronize)");
    // device slots in queue order (rtk::Frame): one per stratum row of the
    // whole rows, `parts` per stratum row of the tail rows, `parts2` per
    // stratum row of the fine rows; a tail row's sum = its part sums added in
    // part order, as rt_reduce_kernel adds them
    const uint64_t npix = (uint64_t)d->W * d->rows, whole_px = (uint64_t)d->W * d->whole_rows;
    const uint64_t fine_px = (uint64_t)d->W * d->fine_row;
    const uint64_t fine_first = whole_px * d->S + (fine_px - whole_px) * d->S * d->parts;
    const uint64_t slots = fine_first + (npix - fine_px) * d->S * d->parts2;
    std::vector<double> buf;
    try {
        buf.resize(slots * 3);
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
    if (n && (e = hipMemcpy(buf.data(), d->partial, buf.size() * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "hipMemcpy partials");
    for (uint64_t pix = 0; pix < npix; ++pix) {
        const bool whole = pix < whole_px, fine = pix >= fine_px;
        const uint32_t np = whole ? 1u : (fine ? d->parts2 : d->parts);
        const double* px = buf.data() + (whole ? pix * d->S
                                         : fine ? fine_first + (pix - fine_px) * d->S * np
                                                : whole_px * d->S + (pix - whole_px) * d->S * np) * 3;
        for (uint32_t si = 0; si < d->S; ++si)
            for (int c = 0; c < 3; ++c) {
                const double* src = px + (uint64_t)si * np * 3 + c;
                double sum = src[0];
                for (uint32_t j = 1; j < np; ++j) sum += src[j * 3];
                out[(pix * d->S + si) * 3 + c] = sum;
            }
    }
    return RT_OK;
}

int32_t rt_to_rgb_device(const float* lin_dev, uint8_t* srgb_dev, uint64_t n_values, int32_t toon_map, void* stream) {
    if (n_values && (!lin_dev || !srgb_dev)) return set_error(RT_EINVAL, "null argument");
    hipError_t e = rtk_launch_to_rgb(lin_dev, srgb_dev, n_values, toon_map, (hipStream_t)stream);
    return e == hipSuccess ? RT_OK : hip_fail(e, "to_rgb launch");
}

int32_t rt_math_selftest(int32_t fn, int32_t impl, const double* a, const double* b, double* out, uint64_t n) {
    if (fn < 0 || fn > 9 || impl < 0 || impl > 1) return set_error(RT_EINVAL, "unknown function or implementation");
    if (n && (!a || !out || (fn == 6 && !b))) return set_error(RT_EINVAL, "null argument");
    if (n == 0) return RT_OK;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, dev)) != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(RT_EDEVICE, std::string("librt_mi355x.so needs a gfx950 device, found ") + prop.gcnArchName);
    double* d = nullptr;
    const size_t bytes = n * sizeof(double);
    if ((e = hipMalloc(&d, bytes * 3)) != hipSuccess) return hip_fail(e, "hipMalloc");
    int32_t rc = RT_OK;
    if ((e = hipMemcpy(d, a, bytes, hipMemcpyHostToDevice)) != hipSuccess ||
        (b && (e = hipMemcpy(d + n, b, bytes, hipMemcpyHostToDevice)) != hipSuccess) ||
        (e = rtk_launch_math(fn, impl, d, b ? d + n : nullptr, d + 2 * n, n, nullptr)) != hipSuccess ||
        (e = hipMemcpy(out, d + 2 * n, bytes, hipMemcpyDeviceToHost)) != hipSuccess)
        rc = hip_fail(e, "math self-test");
    (void)hipFree(d);
    return rc;
}

int32_t rt_render(rt_scene* s, int32_t world, int32_t lights, const rt_camera* cam, const rt_render_opts* opts,
                  float* out_lin, uint8_t* out_srgb, rt_stats* st) {
    if (!cam) return set_error(RT_EINVAL, "null camera");
    try {
        const uint32_t rows = rt_shard_rows(cam, opts);
        const size_t n = (size_t)cam->image_width * rows * 3;
        const bool srgb_dev = out_srgb && cam->max_depth > 0;  // else every pixel is BLACK -> 0
        int32_t rc = launch(s, world, lights, cam, opts, nullptr, true, out_srgb != nullptr);
        if (rc != RT_OK) return rc;
        RenderState* r = s->rs;
        rc = wait(s, st);
        if (rc != RT_OK && rc != RT_EPANIC) return rc;
        if (!r->is_root) return rc;
        DeviceGuard guard;
        hipError_t e;
        const float* lin = r->gathered ? r->full : r->slots[0]->out;
        const uint8_t* sb = r->gathered ? r->full_srgb : r->slots[0]->srgb;
        (void)hipSetDevice(r->gathered ? r->root_device : r->slots[0]->device);
        if (n && out_lin && (e = hipMemcpy(out_lin, lin, n * sizeof(float), hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "hipMemcpy output");
        if (n && out_srgb) {
            if (srgb_dev || r->gathered) {
                if ((e = hipMemcpy(out_srgb, sb, n, hipMemcpyDeviceToHost)) != hipSuccess)
                    return hip_fail(e, "hipMemcpy srgb");
            } else {
                std::memset(out_srgb, 0, n);
            }
        }
        return rc;
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
}

int32_t rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]) {
    if (!id) return set_error(RT_EINVAL, "null id");
    RcclApi& nc = rccl();
    if (!nc.ok) return set_error(RT_EDEVICE, nc.err);
    ncclUniqueId u;
    ncclResult_t e = nc.get_unique_id(&u);
    if (e != ncclSuccess) return nccl_fail(nc, e, "ncclGetUniqueId");
    static_assert(sizeof(u) == RT_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof u);
    return RT_OK;
}

rt_comm* rt_comm_init(const uint8_t id[RT_COMM_ID_BYTES], int32_t nranks, int32_t rank) {
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) {
        set_error(RT_EINVAL, "bad communicator arguments");
        return nullptr;
    }
    RcclApi& nc = rccl();
    if (!nc.ok) {
        set_error(RT_EDEVICE, nc.err);
        return nullptr;
    }
    int dev = -1;
    hipError_t he = hipGetDevice(&dev);
    if (he != hipSuccess) {
        hip_fail(he, "hipGetDevice");
        return nullptr;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    rt_comm* c = new rt_comm();
    c->api = &nc;
    ncclResult_t e = nc.comm_init_rank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) {
        nccl_fail(nc, e, "ncclCommInitRank");
        delete c;
        return nullptr;
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = dev;
    return c;
}

void rt_comm_destroy(rt_comm* c) {
    if (!c) return;
    if (c->comm && c->api && c->api->ok) (void)c->api->comm_destroy(c->comm);
    delete c;
}

}  // extern "C"
