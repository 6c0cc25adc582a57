// tests/cpp/launcher_tsan.cpp -- TEST HARNESS: the launcher's concurrent host
// code (rt_render.cpp) under ThreadSanitizer, on the stub device layer of
// tests/cpp/hip_stub.cpp (no GPU), with the RCCL stand-in of
// tests/cpp/fake_rccl.cpp loaded through RT_RCCL_LIB (this build compiles
// rt_render.cpp with -DRT_CHECK, as the check library is).  This replaces the
// safety rayon's pool gives the reference (camera.rs:178-197) for the code
// that first runs concurrently on an 8-GPU node:
//   - a device list of N distinct devices (ncclCommInitAll, one send /
//     receive group; run_part threads sharing one FlatWorld), N = 2, 3, 8,
//     twice (the cached communicator set);
//   - a device list with a repeat (peer copies onto the root);
//   - N communicator ranks on N host threads (rt_comm_init: ncclCommInitRank
//     on one unique id), N = 2, 3, 8;
//   - two scenes gathering over the same device list from two threads at
//     once (the set's group lock), and the same with two communicator sets;
//   - rt_render_device + rt_render_device_wait on a caller stream (NULL).
// Every gathered frame is checked row by row against the stub kernel's
// pixel function: a row of the wrong part, a missing part or a torn copy is a
// failure.  Mode "planted" reads a device output before rt_render_device_wait
// -- a race TSan must report (the harness's proof that it can).
// Usage: launcher_tsan <fake_rccl.so> [planted]; prints "ok <frames>".
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_mi355x.h"

extern "C" float stub_value(uint32_t y, uint32_t x, uint32_t c);
extern "C" uint8_t stub_byte(uint32_t y, uint32_t x, uint32_t c);
extern "C" int hipSetDevice(int);
extern "C" int hipMalloc(void**, size_t);
extern "C" int hipFree(void*);

static int g_frames = 0;
static std::mutex* g_lock = new std::mutex();

#define CHECK(c)                                                                               \
    do {                                                                                       \
        if (!(c)) {                                                                            \
            std::fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, rt_last_error()); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

struct World {
    rt_scene* s = nullptr;
    int32_t world = -1;
    rt_camera cam{};
};

static World make_world(uint32_t W, uint32_t spp) {
    World w;
    w.s = rt_scene_create();
    CHECK(w.s);
    const double grey[3] = {0.5, 0.5, 0.5};
    const int32_t mat = rt_mat_lambertian(w.s, rt_tex_solid(w.s, grey));
    const int32_t list = rt_hittables_new(w.s);
    for (int i = 0; i < 40; ++i) {
        const double c[3] = {(double)(i % 7) - 3.0, 0.2 * (i % 3), -1.0 - (double)(i / 7)};
        CHECK(rt_hittables_add(w.s, list, rt_sphere(w.s, c, 0.2, mat)) == 0);
    }
    w.world = rt_bvh_new(w.s, list);
    CHECK(w.world >= 0);
    rt_camera_default(&w.cam);
    w.cam.image_width = W;
    w.cam.aspect_ratio = 16.0 / 9.0;
    w.cam.samples_per_pixel = spp;
    w.cam.max_depth = 8;
    return w;
}

static void check_frame(const rt_camera& cam, const float* lin, const uint8_t* srgb) {
    const uint32_t W = cam.image_width, H = rt_camera_image_height(&cam);
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x)
            for (uint32_t c = 0; c < 3; ++c) {
                const size_t i = ((size_t)y * W + x) * 3 + c;
                if (lin[i] != stub_value(y, x, c) || (srgb && srgb[i] != stub_byte(y, x, c))) {
                    std::fprintf(stderr, "FAIL pixel (%u, %u, %u): %g / %u\n", y, x, c, (double)lin[i],
                                 srgb ? srgb[i] : 0u);
                    std::exit(1);
                }
            }
    std::lock_guard<std::mutex> lk(*g_lock);
    ++g_frames;
}

static void render_devices(World& w, const std::vector<int32_t>& devs, int expect_mode) {
    const uint32_t W = w.cam.image_width, H = rt_camera_image_height(&w.cam);
    std::vector<float> lin((size_t)W * H * 3);
    std::vector<uint8_t> srgb(lin.size());
    rt_render_opts o;
    rt_render_opts_default(&o);
    o.n_devices = (uint32_t)devs.size();
    o.devices = devs.data();
    rt_stats st;
    CHECK(rt_render(w.s, w.world, -1, &w.cam, &o, lin.data(), srgb.data(), &st) == 0);
    CHECK(st.n_devices == devs.size());
    CHECK(rt_render_gather_mode(w.s) == expect_mode);
    check_frame(w.cam, lin.data(), srgb.data());
}

static void render_ranks(int n, uint32_t W) {
    uint8_t id[RT_COMM_ID_BYTES];
    CHECK(rt_comm_unique_id(id) == 0);
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            CHECK(hipSetDevice(r % 8) == 0);
            rt_comm* c = rt_comm_init(id, n, r);
            CHECK(c);
            World w = make_world(W, 4);
            const uint32_t H = rt_camera_image_height(&w.cam);
            std::vector<float> lin((size_t)W * H * 3, -1.0f);
            std::vector<uint8_t> srgb(lin.size());
            for (int frame = 0; frame < 2; ++frame) {
                rt_render_opts o;
                rt_render_opts_default(&o);
                o.comm = c;
                CHECK(rt_render(w.s, w.world, -1, &w.cam, &o, lin.data(), srgb.data(), nullptr) == 0);
                CHECK(rt_render_gather_mode(w.s) == RT_GATHER_RCCL_COMM);
                if (r == 0) check_frame(w.cam, lin.data(), srgb.data());
            }
            rt_scene_destroy(w.s);
            rt_comm_destroy(c);
        });
    for (auto& t : th) t.join();
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: launcher_tsan <fake_rccl.so> [planted]\n");
        return 2;
    }
    setenv("RT_RCCL_LIB", argv[1], 1);
    const bool planted = argc > 2 && std::strcmp(argv[2], "planted") == 0;
    if (planted) {
        // a device output read on the host before rt_render_device_wait: the
        // stub kernel writes it on its stream's thread
        World w = make_world(48, 4);
        const uint32_t H = rt_camera_image_height(&w.cam);
        float* out = nullptr;
        CHECK(hipMalloc((void**)&out, (size_t)48 * H * 3 * sizeof(float)) == 0);
        rt_render_opts o;
        rt_render_opts_default(&o);
        CHECK(rt_render_device(w.s, w.world, -1, &w.cam, &o, out) == 0);
        volatile float v = out[0];  // the planted race
        (void)v;
        CHECK(rt_render_device_wait(w.s, nullptr) == 0);
        hipFree(out);
        rt_scene_destroy(w.s);
        std::printf("planted done\n");
        return 0;
    }
    // device lists with distinct devices: ncclCommInitAll + one group
    for (int n : {2, 3, 8}) {
        World w = make_world(40 + n, 9);
        std::vector<int32_t> devs;
        for (int k = 0; k < n; ++k) devs.push_back(k);
        render_devices(w, devs, RT_GATHER_RCCL_DEVICES);
        render_devices(w, devs, RT_GATHER_RCCL_DEVICES);  // the cached set, the slots' second frame
        rt_scene_destroy(w.s);
    }
    {  // a repeated device: peer copies
        World w = make_world(36, 4);
        render_devices(w, {0, 1, 0}, RT_GATHER_PEER_COPY);
        rt_scene_destroy(w.s);
    }
    // communicator ranks, one host thread each
    for (int n : {2, 3, 8}) render_ranks(n, 32 + n);
    {  // two scenes gathering at once over one device list, and over two lists
        for (int lists = 1; lists <= 2; ++lists) {
            std::vector<std::thread> th;
            for (int k = 0; k < 2; ++k)
                th.emplace_back([k, lists] {
                    World w = make_world(44, 4);
                    std::vector<int32_t> devs = (lists == 2 && k == 1) ? std::vector<int32_t>{4, 5, 6, 7}
                                                                       : std::vector<int32_t>{0, 1, 2, 3};
                    for (int f = 0; f < 3; ++f) render_devices(w, devs, RT_GATHER_RCCL_DEVICES);
                    rt_scene_destroy(w.s);
                });
            for (auto& t : th) t.join();
        }
    }
    {  // stream-ordered render into a device buffer, then the wait
        World w = make_world(40, 4);
        const uint32_t H = rt_camera_image_height(&w.cam);
        float* out = nullptr;
        CHECK(hipMalloc((void**)&out, (size_t)40 * H * 3 * sizeof(float)) == 0);
        rt_render_opts o;
        rt_render_opts_default(&o);
        for (int f = 0; f < 2; ++f) {
            CHECK(rt_render_device(w.s, w.world, -1, &w.cam, &o, out) == 0);
            CHECK(rt_render_device_wait(w.s, nullptr) == 0);
            check_frame(w.cam, out, nullptr);
        }
        hipFree(out);
        rt_scene_destroy(w.s);
    }
    std::printf("ok %d\n", g_frames);
    return 0;
}
