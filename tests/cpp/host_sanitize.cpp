// tests/cpp/host_sanitize.cpp -- TEST-ONLY driver of the host code under
// AddressSanitizer + UBSan or ThreadSanitizer (tests/test_sanitize_cpu.py).
//
// Built twice, against the C ABI:
//   -DPRODUCT: the product's host objects (rt_scene.cpp -- BVH::from_vec's
//     parallel builder, the flatten with its parallel binned SAH, the
//     selftests --, rt_obj.cpp -- the in-place OBJ / MTL parser --,
//     rt_output.cpp -- PNG writer, Camera::from_json), compiled with the
//     sanitizer; the device half of the library (rt_render.cpp, the kernels)
//     is not linked: two stubs below stand in for what the host objects call;
//   -DORACLE: the CPU oracle (oracle/*.cpp) with the same calls (orc_ prefix)
//     plus a multithreaded render of a book-1-style world (C1-shaped).
//
//   host_sanitize <obj path> <png out dir> <render threads> <render spp> [oob | race]
// (oob / race: a deliberate heap overflow / data race first -- the test's
// proof that the build is instrumented and the sanitizer aborts)
// Prints one line per check and exits non-zero on the first failure; the
// sanitizers abort on their own findings (-fno-sanitize-recover).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/rt_mi355x.h"

#ifdef ORACLE
#define API(f) orc_##f
extern "C" {
decltype(rt_scene_create) orc_scene_create;
decltype(rt_scene_destroy) orc_scene_destroy;
decltype(rt_last_error) orc_last_error;
decltype(rt_tex_solid) orc_tex_solid;
decltype(rt_tex_sky_gradient) orc_tex_sky_gradient;
decltype(rt_mat_lambertian) orc_mat_lambertian;
decltype(rt_mat_metal) orc_mat_metal;
decltype(rt_mat_dielectric) orc_mat_dielectric;
decltype(rt_sphere) orc_sphere;
decltype(rt_hittables_new) orc_hittables_new;
decltype(rt_hittables_add) orc_hittables_add;
decltype(rt_bvh_new) orc_bvh_new;
decltype(rt_wavefront_load) orc_wavefront_load;
decltype(rt_camera_default) orc_camera_default;
decltype(rt_camera_image_height) orc_camera_image_height;
decltype(rt_render_opts_default) orc_render_opts_default;
decltype(rt_render) orc_render;
}
#else
#define API(f) rt_##f
// what rt_scene.cpp calls in the device half of the library (not linked here)
namespace rth {
struct RenderState;
void destroy_render_state(RenderState*) {}
}  // namespace rth
extern "C" int rtk_planar_filter(void) { return 0; }  // the product's RT_PLANAR_FILTER default
#endif

static int fails = 0;
static void check(bool ok, const char* what) {
    std::printf("%s %s\n", ok ? "ok  " : "FAIL", what);
    if (!ok) {
        std::printf("     last error: %s\n", API(last_error)() ? API(last_error)() : "");
        ++fails;
    }
}

// SplitMix64, for the world's layout only
static uint64_t g_sm = 2025;
static double rnd() {
    uint64_t z = (g_sm += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (double)((z ^ (z >> 31)) >> 11) * 0x1.0p-53;
}

// book-1's final scene shape (main.rs random spheres): ground, a grid of
// small spheres of the three materials, three big spheres, under one BVH
static int32_t spheres_list(rt_scene* s, int grid) {
    const int32_t list = API(hittables_new)(s);
    const double g[3] = {0.5, 0.5, 0.5};
    const double ground[3] = {0, -1000, 0};
    API(hittables_add)(s, list, API(sphere)(s, ground, 1000.0, API(mat_lambertian)(s, API(tex_solid)(s, g))));
    for (int a = -grid; a < grid; ++a)
        for (int b = -grid; b < grid; ++b) {
            const double c[3] = {a + 0.9 * rnd(), 0.2, b + 0.9 * rnd()};
            const double m = rnd();
            int32_t mat;
            if (m < 0.8) {
                const double alb[3] = {rnd() * rnd(), rnd() * rnd(), rnd() * rnd()};
                mat = API(mat_lambertian)(s, API(tex_solid)(s, alb));
            } else if (m < 0.95) {
                const double alb[3] = {0.5 + rnd() / 2, 0.5 + rnd() / 2, 0.5 + rnd() / 2};
                mat = API(mat_metal)(s, alb, rnd() / 2);
            } else {
                const double w[3] = {1, 1, 1};
                mat = API(mat_dielectric)(s, API(tex_solid)(s, w), 1.5);
            }
            API(hittables_add)(s, list, API(sphere)(s, c, 0.2, mat));
        }
    const double p1[3] = {0, 1, 0}, p2[3] = {-4, 1, 0}, p3[3] = {4, 1, 0}, w[3] = {1, 1, 1};
    const double a2[3] = {0.4, 0.2, 0.1}, a3[3] = {0.7, 0.6, 0.5};
    API(hittables_add)(s, list, API(sphere)(s, p1, 1.0, API(mat_dielectric)(s, API(tex_solid)(s, w), 1.5)));
    API(hittables_add)(s, list, API(sphere)(s, p2, 1.0, API(mat_lambertian)(s, API(tex_solid)(s, a2))));
    API(hittables_add)(s, list, API(sphere)(s, p3, 1.0, API(mat_metal)(s, a3, 0.0)));
    return list;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s <obj> <out dir> <threads> <spp>\n", argv[0]);
        return 2;
    }
    const std::string obj = argv[1], out_dir = argv[2];
    const uint32_t threads = (uint32_t)std::atoi(argv[3]), spp = (uint32_t)std::atoi(argv[4]);
    if (argc > 5 && !std::strcmp(argv[5], "oob")) {
        std::vector<int> v(4, 1);
        volatile int x = v.data()[v.size()];  // one past the end
        std::printf("read %d\n", x);
    }
    if (argc > 5 && !std::strcmp(argv[5], "race")) {
        static int shared = 0;
        std::thread a([] { for (int i = 0; i < 100000; ++i) ++*(volatile int*)&shared; });
        std::thread b([] { for (int i = 0; i < 100000; ++i) ++*(volatile int*)&shared; });
        a.join();
        b.join();
        std::printf("shared %d\n", shared);
    }
    rt_scene* s = API(scene_create)();
    const double hz[3] = {1, 1, 1}, zn[3] = {0.5, 0.7, 1.0};
    const int32_t sky = API(tex_sky_gradient)(s, hz, zn);

    // the book-1 world: 11 x 11 grid -> 489 spheres (C1 / C2's world shape)
    const int32_t list = spheres_list(s, 11);
#ifdef PRODUCT
    check(rt_bvh_selftest(s, list) == 1, "BVH::from_vec, parallel builder == serial (489 spheres)");
    // a list past the parallel builder's threshold (16384 objects)
    const int32_t big = spheres_list(s, 75);  // 22 504 spheres
    check(rt_bvh_selftest(s, big) == 1, "BVH::from_vec, parallel builder == serial (22 504 spheres)");
#endif
    const int32_t bvh = API(bvh_new)(s, list);
    check(bvh >= 0, "BVH::new over the book-1 list");
    const int32_t world = API(hittables_new)(s);
    API(hittables_add)(s, world, bvh);
#ifdef PRODUCT
    check(rt_world_selftest(s, world, -1, sky) == 1, "flatten, parallel SAH == serial (book-1 world)");
#endif

    // the OBJ terrain through the OBJ / MTL parser
    const int32_t mesh = API(wavefront_load)(s, obj.c_str(), 1);  // vanilla MTL (Pm metals), as the C4 loader
    check(mesh >= 0, "Wavefont::new on the terrain OBJ");
    if (mesh >= 0) {
        const int32_t w2 = API(hittables_new)(s);
        API(hittables_add)(s, w2, mesh);
        const double c[3] = {0, 1, 0};
        const double alb[3] = {0.8, 0.3, 0.3};
        API(hittables_add)(s, w2, API(sphere)(s, c, 0.5, API(mat_metal)(s, alb, 0.1)));
#ifdef PRODUCT
        check(rt_world_selftest(s, w2, -1, sky) == 1, "flatten, parallel SAH == serial (terrain world)");
#endif
    }

#ifdef PRODUCT
    // the output stage: PNG writer (with create_dir_all) and Camera::from_json
    {
        std::vector<uint8_t> img(37 * 23 * 3);
        for (size_t i = 0; i < img.size(); ++i) img[i] = (uint8_t)(i * 7);
        const std::string png = out_dir + "/nested/dir/out.png";
        check(rt_write_png(png.c_str(), 37, 23, img.data()) == RT_OK, "img.save (PNG writer)");
        const std::string js = out_dir + "/camera.json";
        FILE* f = std::fopen(js.c_str(), "w");
        std::fputs("{\"aspect_ratio\": 1.5, \"image_width\": 64, \"vertical_fov_in_degrees\": 30.0,"
                   " \"look_from\": [1, 2, 3], \"look_at\": [0, 0, 0], \"vec_up\": [0, 1, 0],"
                   " \"defocus_angle_in_degrees\": 0.5, \"focus_distance\": 4.0}", f);
        std::fclose(f);
        rt_camera cam;
        check(rt_camera_from_json(js.c_str(), &cam) == RT_OK && cam.image_width == 64, "Camera::from_json");
        const std::string bad = out_dir + "/bad.json";
        f = std::fopen(bad.c_str(), "w");
        std::fputs("{\"aspect_ratio\": 1.5, \"image_width\": ", f);
        std::fclose(f);
        check(rt_camera_from_json(bad.c_str(), &cam) != RT_OK, "Camera::from_json rejects a truncated file");
    }
#endif
#ifdef ORACLE
    // one C1-shaped render (book-1 world, 400 x 225, defocus) on `threads` threads
    {
        rt_camera cam;
        orc_camera_default(&cam);
        cam.aspect_ratio = 16.0 / 9.0;
        cam.image_width = 400;
        cam.samples_per_pixel = spp;
        cam.max_depth = 50;
        cam.background_tex = sky;
        cam.vertical_fov_in_degrees = 20.0;
        const double from[3] = {13, 2, 3}, at[3] = {0, 0, 0};
        for (int k = 0; k < 3; ++k) cam.look_from[k] = from[k], cam.look_at[k] = at[k];
        cam.defocus_angle_in_degrees = 0.6;
        cam.focus_distance = 10.0;
        rt_render_opts opts;
        orc_render_opts_default(&opts);
        opts.threads = threads;
        const uint32_t H = orc_camera_image_height(&cam);
        std::vector<float> lin((size_t)H * cam.image_width * 3);
        std::vector<uint8_t> srgb(lin.size());
        rt_stats st;
        const int32_t rc = orc_render(s, world, -1, &cam, &opts, lin.data(), srgb.data(), &st);
        bool finite = true;
        for (float v : lin) finite = finite && std::isfinite(v);
        check(rc == RT_OK && finite && st.samples == (uint64_t)H * cam.image_width * (uint64_t)std::floor(std::sqrt(spp)) *
                                                       (uint64_t)std::floor(std::sqrt(spp)),
              "multithreaded oracle render of the book-1 world (400 x 225)");
    }
#endif
    API(scene_destroy)(s);
    std::printf("%s\n", fails ? "FAILED" : "PASSED");
    return fails ? 1 : 0;
}
