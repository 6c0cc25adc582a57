// rt_kernel.hip -- the persistent-threads f64 path-tracing megakernel for gfx950.
//
// One launch renders one frame (or one shard of rows) of Camera::render
// (src/camera.rs:161-202).  Work item = (pixel, stratum row s_i): the lane
// traces the sqrt_spp samples s_j of that row (camera.rs:183-192) one after
// another and stores their f64 sum; rt_reduce sums the rows of a pixel in s_i
// order and scales by pixel_sample_scale (camera.rs:193).
//
// ray_color's recursion (camera.rs:275-325) is run as a loop that carries a
// path throughput `beta` and radiance `L`; a lane whose path ends starts the
// next sample of its row at once, and a lane whose row ends takes the next row
// from a device-wide counter.  Refills are aggregated per wave: __ballot of the
// lanes that need work, one atomicAdd by the first of them, and each lane's
// slot from its mbcnt rank -- the wave64 prefix-sum compaction that keeps all
// 64 lanes tracing until the queue is empty.
//
// world.hit (hits.rs:34, bvh.rs:57, shapes.rs:88, volume.rs:37) is an explicit
// depth-first walk over the flattened world (rt_layout.h) with a per-lane stack
// in LDS, laid out [depth][lane] so a wave's pushes/pops hit 64 distinct banks.
#include <hip/hip_runtime.h>

#include "rt_crmath.h"
#include "rt_kernel.h"
#include "rt_math.h"
#include "rt_slab.h"
#include "rt_sphere_filter.h"
#include "rt_plan.h"

namespace rtk {

// Basic tier: 4-wide BVH nodes (rth::bvh4_convert), sphere children through
// the f32 filter (rt_sphere_filter.h) into a per-lane LDS queue of exact tests
// (visit4); 0 = two-box nodes with inline f64 sphere tests.
#ifndef RT_BVH4
#define RT_BVH4 1
#endif
#ifndef RT_PEND_CAP
#define RT_PEND_CAP 8  // queued sphere tests per lane (LDS, 2 B each: sphere index < 65536)
#endif
// Mesh tier: 4-wide BVH nodes with every child boxed (visit4_boxes).
#ifndef RT_MESH_BVH4
#define RT_MESH_BVH4 1
#endif
// Full tier: the same boxed 4-wide nodes, for the walk and the medium boundary walks.
#ifndef RT_FULL_BVH4
#define RT_FULL_BVH4 1
#endif

// Diagnostic build (-DRT_DIAG, librt_mi355x_diag.so only): per-wave cycle
// stamps and per-lane work counters, summed into g_diag.  The product build
// compiles all of it away.
struct Diag {
#ifdef RT_DIAG
    unsigned long long cyc_refill = 0, cyc_trace = 0, cyc_shade = 0, cyc_media = 0;
    // basic / mesh tiers' unified loop: the parts of cyc_refill after the walk
    unsigned long long cyc_miss = 0, cyc_queue = 0, cyc_draws = 0;
    unsigned long long wave_trace_iters = 0, lane_trace_iters = 0, node_visits = 0, sphere_tests = 0, main_iters = 0;
    unsigned long long load_cyc = 0, loads = 0;  // -DRT_DIAG_LOADLAT: node-load latency (first active lane)
    unsigned long long pops = 0, pop_reads = 0;  // basic tier: pops and the stack entries they read
    unsigned long long big_tests = 0, big_hits = 0;  // basic tier: exact tests of spheres with r > 100 (and hits)
    // mesh / full tiers' unified walk-step loads: wave steps, steps whose
    // active lanes all read one record (of them node records), active lanes,
    // lanes reading the first active lane's record
    unsigned long long u_steps = 0, u_uniform = 0, u_uniform_node = 0, u_active = 0, u_same = 0;
    // ... steps whose active lanes all read nodes of the top 5 / 21 / 85 / 341
    // (rth::bvh4_convert numbers the top levels first, breadth-first), and
    // node reads of lanes at those nodes (lane counts)
    unsigned long long u_top[4] = {0, 0, 0, 0}, l_top[4] = {0, 0, 0, 0}, l_node = 0;
    // full tiers' shading rounds: rounds, lanes shaded, distinct shading
    // classes per round (miss, Lambertian by texture kind, Metal, Dielectric,
    // light, Isotropic, other) -- the branches a round executes one after the
    // other whatever the order of its lanes
    unsigned long long sh_rounds = 0, sh_lanes = 0, sh_classes = 0;
    // basic tier: wave iterations with no lane able to walk a node (pure
    // sphere rounds), and the lanes with a queued sphere in them
    unsigned long long pure_rounds = 0, pure_lanes = 0, pure_max_pn = 0;
    // ... per shading class (the 11 above): rounds in which it is present,
    // and its lanes
    unsigned long long cls_rounds[11] = {}, cls_lanes[11] = {};
#endif
};
#ifdef RT_DIAG
constexpr int RT_DIAG_N = 61;
__device__ unsigned long long g_diag[RT_DIAG_N];
#define RT_DIAG_ONLY(x) x
#else
#define RT_DIAG_ONLY(x)
#endif
// ISA attribution build only (scripts/isa_phases.py, -DRT_ISA_MARKS): an
// assembler comment at each phase boundary of the basic tier's loop, so that
// the static instruction mix of every phase can be read off the ISA
#ifdef RT_ISA_MARKS
#define RT_ISA_MARK(name) asm volatile(";@@phase " name)
#else
#define RT_ISA_MARK(name)
#endif

#ifdef RT_WAVE_TRACE
// trace build: per lane of the grid, {start, end (s_memrealtime, 100 MHz),
// queue entries taken, rays traced, time / queue entry / rays so far at the
// lane's last refill, s_memtime ticks from start to end} (scripts/lane_trace.py)
constexpr uint32_t RT_TRACE_LANES = 1u << 19, RT_TRACE_W = 12;
__device__ unsigned long long g_lane_trace[RT_TRACE_LANES * RT_TRACE_W];
// ... and the rays begun per 0.25 ms of the launch (each wave's own clock
// from its start; one atomic per wave and bucket): the launch's throughput
// over time -- its ramp, steady state and drain
constexpr uint32_t RT_HIST_N = 1024, RT_HIST_TICKS = 25000;  // s_memrealtime: 100 MHz
__device__ unsigned long long g_ray_hist[RT_HIST_N];
struct RayHist {
    unsigned long long t0;
    uint32_t bucket = 0, count = 0;
    // beg: the lanes of the wave beginning a ray now (wave-uniform)
    __device__ __forceinline__ void add(unsigned long long beg) {
        const uint32_t b = min((uint32_t)((__builtin_amdgcn_s_memrealtime() - t0) / RT_HIST_TICKS), RT_HIST_N - 1);
        if (b != bucket) {
            flush();
            bucket = b;
        }
        count += (uint32_t)__popcll(beg);
    }
    __device__ __forceinline__ void flush() {
        if (count && __lane_id() == (uint32_t)(__ffsll((long long)__ballot(true)) - 1))
            atomicAdd(&g_ray_hist[bucket], (unsigned long long)count);
        count = 0;
    }
};
#endif

struct Ray {
    D3 o, d;
    double time;
};

struct Frame {
    uint32_t W, rows, row_offset, row_stride;
    uint32_t S;  // sqrt_spp
    uint32_t max_depth;
    uint32_t key0, key1;
    uint32_t total_items;
    // Work queue (item = launch pixel * S + s_i, a stratum row): the shard's
    // first whole_items items -- the pixels of its rows above the frame's
    // tail rows (rtk_tail_rows) -- are one entry each, a whole row of S
    // samples; every later item is `parts` entries of part_len consecutive
    // samples s_j (the last part the rest), so that the last entries of a
    // launch are short: a whole row of a pixel whose paths bounce 40 times
    // inside a glass sphere is ~10 ms of one wave (scripts/lane_trace.py).
    // The frame's last `fine` rows (rtk_tail_split) go out in finer parts
    // still -- parts2 entries of part_len2 samples, from queue entry fine_q0
    // and item fine_item0 on -- so that what is in flight when the queue
    // runs dry is about one sample a lane: a 1/8 row shard of C4 drained for
    // ~3 ms after its last 4-sample part was handed out (lane_trace_c4.json).
    // Entry q writes its f64 sum to partial slot q (queue order: the lanes
    // of a wave take consecutive entries, so their 24-B sums fill whole L2
    // lines), and the reduce adds a tail row's parts in part order.
    uint32_t parts, part_len, queue_total, whole_items;
    uint32_t parts2, part_len2, fine_q0, fine_item0;
    uint32_t static_entries;  // 64 per wave of the grid: their first pools, taken without the counter
    uint32_t chunk_min;  // smallest guided chunk (queue entries per atomic)
    uint32_t chunk_cap;  // largest guided chunk
    uint32_t chunk_min_whole;  // smallest guided chunk while whole-row entries are left
    // 1/parts, 1/S, 1/W rounded up (udiv_inv), and 1/(waves of the grid x
    // RT_QUEUE_GUIDE): the queue-entry decode without integer divisions
    double inv_parts, inv_parts2, inv_S, inv_W;
    float inv_guide;
    // samples per entry of each region and their reciprocals: the guided
    // chunk is the work left in samples / (waves x guide), in the entries of
    // the region the pool starts in
    float S_f, part_len_f, part_len2_f, inv_S_f, inv_part_len_f, inv_part_len2_f;
    uint32_t defocus;
    double recip_sqrt_spp, pixel_sample_scale;
    D3 center, pixel00, du, dv, disk_u, disk_v;
};

// ------------------------------------------------------------------ check build
// make check (-DRT_CHECK, librt_mi355x_check.so): every ref the walk, the
// hit record and the lights decode is checked against the count of its
// kind's array (SceneView::n_ref); a ref past its array is counted in
// g_check (the host's wait() turns a nonzero count into an error naming the
// first bad ref) and read as index 0, so the run itself stays in bounds.
// The product build compiles the check away.
#ifdef RT_CHECK
__device__ unsigned long long g_check[2];
__device__ __noinline__ void check_fail(uint32_t ref) {
    atomicAdd(&g_check[0], 1ull);
    atomicCAS(&g_check[1], 0ull, (1ull << 32) | ref);
}
#endif
__device__ __forceinline__ uint32_t ref_idx(const SceneView& S, uint32_t ref) {
    const uint32_t i = ref_index(ref);
#ifdef RT_CHECK
    const uint32_t k = ref_kind(ref);
    if (k != K_NONE && i >= S.n_ref[k]) {
        check_fail(ref);
        return 0u;
    }
#endif
    return i;
}
// a planar run's last record (DBoxF::run) must lie inside planars too
__device__ __forceinline__ void check_run(const SceneView& S, uint32_t first, uint32_t n) {
#ifdef RT_CHECK
    if (n && first + n > S.n_ref[K_QUAD]) check_fail(make_ref(K_QUAD, first + n - 1));
#endif
}

// n / d for n < 2^32, d < 2^20, from inv = 1/d rounded up: n * inv is at least
// the quotient's integer part when d divides n (a representable product,
// rounded to nearest, cannot fall below it) and below the next integer
// otherwise (the excess n * 2^-52 / d stays under 1/d): three f64 / convert
// instructions instead of a ~25-instruction integer division expansion.
__device__ __forceinline__ uint32_t udiv_inv(uint32_t n, double inv) { return (uint32_t)((double)n * inv); }

// ------------------------------------------------------------------ textures
// texture.rs: SolidColor 33-36, CheckerTexture 60-73, ImageTexture 165-174,
// NoiseTexture 191-196 (+ perlin.rs), book-1 sky.
#ifndef RT_PERLIN_LDS
#define RT_PERLIN_LDS 1
#endif
// Full tiers: the block's LDS copy of the world's first Perlin table (9 KiB,
// copied at launch), read by NoiseTexture instead of global memory: the
// marble's 7 octaves are 14 dependent table reads per shade, and a shading
// batch with one marble hit waits for all of them.
__shared__ DPerlin g_perlin_lds;

template <class PP>
__device__ double perlin_noise(PP P, D3 p) {
    const double fx = floor(p.x), fy = floor(p.y), fz = floor(p.z);
    const int64_t i = (int64_t)fx, j = (int64_t)fy, k = (int64_t)fz;
    const double u = p.x - fx, v = p.y - fy, w = p.z - fz;
    const double uu = u * u * (3.0 - 2.0 * u), vv = v * v * (3.0 - 2.0 * v), ww = w * w * (3.0 - 2.0 * w);
    double accum = 0.0;
    for (int di = 0; di < 2; ++di)
        for (int dj = 0; dj < 2; ++dj)
            for (int dk = 0; dk < 2; ++dk) {
                const int idx = P->perm[0][(uint64_t)(i + di) & 255] ^ P->perm[1][(uint64_t)(j + dj) & 255] ^
                                P->perm[2][(uint64_t)(k + dk) & 255];
                const D3 c = d3(P->randvec[idx][0], P->randvec[idx][1], P->randvec[idx][2]);
                const D3 wv = d3(u - di, v - dj, w - dk);
                accum += (di * uu + (1 - di) * (1.0 - uu)) * (dj * vv + (1 - dj) * (1.0 - vv)) *
                         (dk * ww + (1 - dk) * (1.0 - ww)) * dot(c, wv);
            }
    return accum;
}

__device__ void image_pixel(const SceneView& S, const DTexture& t, int64_t x, int64_t y, float out[4]) {
    x = x < 0 ? 0 : (x > t.a - 1 ? t.a - 1 : x);
    y = y < 0 ? 0 : (y > t.b - 1 ? t.b - 1 : y);
    const RT_GLOBAL float* px = S.texels + t.data + ((uint64_t)y * t.a + x) * 4;
    out[0] = px[0];
    out[1] = px[1];
    out[2] = px[2];
    out[3] = px[3];
}

// ImageTexture::get_pixel (texture.rs:109-158): nearest or bilinear, u / v
// wrapped by x - floor(x), v flipped; t.b != 0 (a loaded image)
__device__ __forceinline__ void image_rgba(const SceneView& S, const DTexture& t, double u, double v, float px[4]) {
    const double uu = u - floor(u);
    const double vv = 1.0 - (v - floor(v));
    if (!t.c) {
        const uint32_t i = (uint32_t)(uu * (double)t.a), j = (uint32_t)(vv * (double)t.b);
        image_pixel(S, t, i, j, px);
        return;
    }
    const double x = uu * (double)t.a - 0.5, y = vv * (double)t.b - 0.5;
    const uint32_t x0 = (uint32_t)fmax(floor(x), 0.0), y0 = (uint32_t)fmax(floor(y), 0.0);
    const uint32_t x1 = min(x0 + 1, (uint32_t)t.a - 1), y1 = min(y0 + 1, (uint32_t)t.b - 1);
    const float dx = (float)(x - (double)x0), dy = (float)(y - (double)y0);
    float p00[4], p10[4], p01[4], p11[4];
    image_pixel(S, t, x0, y0, p00);
    image_pixel(S, t, x1, y0, p10);
    image_pixel(S, t, x0, y1, p01);
    image_pixel(S, t, x1, y1, p11);
    for (int c = 0; c < 4; ++c) {
        const float v0 = p00[c] * (1.0f - dx) + p10[c] * dx;
        const float v1 = p01[c] * (1.0f - dx) + p11[c] * dx;
        px[c] = v0 * (1.0f - dy) + v1 * dy;
    }
}
// ImageTexture::alpha (texture.rs:99-106): 1 for a missing image
__device__ __forceinline__ double tex_alpha(const SceneView& S, int tid, double u, double v) {
    const DTexture& t = S.textures[tid];
    if (t.b == 0) return 1.0;
    float px[4];
    image_rgba(S, t, u, v, px);
    return (double)px[3];
}

#ifndef RT_BG_PARAMS
// 1: the basic and mesh tiers' miss under a sky gradient reads its colours
// from the launch parameters (SceneView::bg_c0 / bg_c1); 0: from the texture
// table (A/B only)
#define RT_BG_PARAMS 1
#endif
// the sky gradient (rt_tex_sky_gradient, include/rt_mi355x.h) at the unit direction's y
__device__ __forceinline__ D3 sky_value(const double* c0, const double* c1, double py) {
    const double a = 0.5 * (py + 1.0);
    return (1.0 - a) * d3(c0[0], c0[1], c0[2]) + a * d3(c1[0], c1[1], c1[2]);
}
__device__ __forceinline__ D3 sky_value(const DTexture& t, double py) { return sky_value(t.color, t.color2, py); }

template <bool FULL, bool PL = false>  // PL: NoiseTexture reads the LDS copy of the first Perlin table
__device__ D3 tex_value(const SceneView& S, int tid, double u, double v, D3 p) {
    for (int guard = 0; guard < 16; ++guard) {
        const DTexture& t = S.textures[tid];
        switch (t.type) {
            case T_SOLID: return d3(t.color[0], t.color[1], t.color[2]);
            case T_SKY: return sky_value(t, p.y);
            case T_CHECKER: {
                const int32_t xi = (int32_t)floor(t.scale * p.x), yi = (int32_t)floor(t.scale * p.y),
                              zi = (int32_t)floor(t.scale * p.z);
                tid = ((xi + yi + zi) % 2 == 0) ? t.a : t.b;
                continue;
            }
            default: break;
        }
        if constexpr (FULL) {
          switch (t.type) {
            case T_IMAGE: {
                if (t.b == 0) return d3(0.0, 1.0, 1.0);  // texture.rs:167-169
                float px[4];
                image_rgba(S, t, u, v, px);
                return d3(px[0], px[1], px[2]);
            }
            case T_NOISE: {
                const bool lds = PL && t.data == 0;
                double accum = 0.0, weight = 1.0;
                D3 tp = p;
                for (int o = 0; o < 7; ++o) {
                    accum += weight * (lds ? perlin_noise((const RT_LDS DPerlin*)&g_perlin_lds, tp)
                                           : perlin_noise(S.perlin + t.data, tp));
                    tp = 2.0 * tp;
                    weight = 0.5 * weight;
                }
                const double turb = fabs(accum);
                return (1.0 + k_sin(t.scale * p.z + 10.0 * turb)) * d3(0.5, 0.5, 0.5);
            }
            default: break;
          }
        }
        return d3(0.0, 0.0, 0.0);
    }
    return d3(0.0, 0.0, 0.0);
}

// ------------------------------------------------------------------ geometry tests
__device__ __forceinline__ RayF make_rayf(const Ray& r) {
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    return make_rayf(o, d);
}

// sphere.rs:77-96 -- t of the accepted root, or false
__device__ __forceinline__ bool sphere_t(D3 c, double radius, const Ray& r, double a, double tmin, double tmax,
                                         double& t) {
    const D3 oc = c - r.o;
    const double h = dot(r.d, oc);
    const double cc = len2(oc) - radius * radius;
    const double disc = h * h - a * cc;
    if (disc < 0.0) return false;
    const double sq = k_sqrt(disc);
    double root = (h - sq) / a;
    if (!(root >= tmin && root <= tmax)) {
        root = (h + sq) / a;
        if (!(root >= tmin && root <= tmax)) return false;
    }
    t = root;
    return true;
}

// num / a for a ray's a = |d|^2 with the correctly rounded inva = 1/a computed
// once per ray: q = num*inva is within 1 ulp, the FMA residual is exact, and
// the corrected quotient is the correctly rounded num / a (Markstein) -- the
// value sphere.rs:88-92's division gives, for 3 instructions instead of 10.
__device__ __forceinline__ double div_a(double num, double a, double inva) {
    const double q = num * inva;
    const double r = fma(-q, a, num);
    return fma(r, inva, q);
}
__device__ __forceinline__ bool sphere_t_inv(D3 c, double radius, const Ray& r, double a, double inva, double tmin,
                                             double tmax, double& t) {
    const D3 oc = c - r.o;
    const double h = dot(r.d, oc);
    const double cc = len2(oc) - radius * radius;
    const double disc = h * h - a * cc;
    if (disc < 0.0) return false;
    const double sq = k_sqrt(disc);
    double root = div_a(h - sq, a, inva);
    if (!(root >= tmin && root <= tmax)) {
        root = div_a(h + sq, a, inva);
        if (!(root >= tmin && root <= tmax)) return false;
    }
    t = root;
    return true;
}

// quad.rs:71-102 / triangle.rs:69-98 on the record's values: unit normal n,
// parm_d D, anchor Q, edges u / v, w = n / |n|^2
__device__ __forceinline__ bool planar_t_v(const D3 n, const double D, const D3 Q, const D3 u, const D3 v, const D3 w,
                                           bool tri, const Ray& r, double tmin, double tmax, double& t) {
    const double denom = dot(n, r.d);
    if (fabs(denom) < 1e-8) return false;
    const double num = D - dot(n, r.o);
    const double tt = num / denom;
    if (!(tt >= tmin && tt <= tmax)) return false;
    const D3 hv = (r.o + tt * r.d) - Q;
    const double alpha = dot(w, cross(hv, v));
    const double beta = dot(w, cross(u, hv));
    if (!(alpha >= 0.0 && alpha <= 1.0 && beta >= 0.0 && beta <= 1.0)) return false;
    if (tri) {
        const double ab = alpha + beta;
        if (!(ab >= 0.0 && ab <= 1.0)) return false;
    }
    t = tt;
    return true;
}
// quad.rs:71-102 / triangle.rs:69-98
__device__ __forceinline__ bool planar_t(const DPlanar& P, bool tri, const Ray& r, double tmin, double tmax,
                                         double& t) {
    return planar_t_v(d3(P.f[0], P.f[1], P.f[2]), P.f[3], d3(P.f[4], P.f[5], P.f[6]), d3(P.f[7], P.f[8], P.f[9]),
                      d3(P.f[10], P.f[11], P.f[12]), d3(P.f[13], P.f[14], P.f[15]), tri, r, tmin, tmax, t);
}

#ifndef RT_PLANAR_FILTER
// 1: quads / triangles take the f32 pre-test (rt_planar_filter.h) before
// planar_t.  Measured slower (A/B at 128 spp, min of 4: C4 +13 %, C5 +5 %,
// C3 +2 %): a triangle reached through a hit box is rarely ruled out, and a
// flat-tier quad's f32 test costs about what the f64 one does.  Kept as an
// option with its CPU property test (tests/test_planar_filter_cpu.py).
#define RT_PLANAR_FILTER 0
#endif
// planar_t behind the conservative f32 pre-test: the f64 record is read and
// tested only when the f32 test cannot rule the primitive out.  The
// pre-test's "behind the origin" rejection needs tmin >= 0 (a medium
// boundary walk starts at -inf).
__device__ __forceinline__ bool planar_t_filtered(const SceneView& S, uint32_t idx, bool tri, const Ray& r,
                                                  double tmin, double tmax, float tmax_f, double& t) {
    if constexpr (RT_PLANAR_FILTER) {
        const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
        if (tmin >= 0.0 && planar_reject(S.planars_f[idx], make_prayf(o, d), tmax_f, tri)) return false;
    }
    return planar_t(S.planars[idx], tri, r, tmin, tmax, t);
}

// Quaternion::rotate_vector (quaternion.rs:72-82): (q * (0, v)) * conj(q)
// with Mul (quaternion.rs:94-103) term by term in the reference's order; the
// products with qv.w = 0 are exact zeros, so a + 0*b is a and those terms
// are left out without changing a bit.
__device__ __forceinline__ D3 quat_rotate(double w, double x, double y, double z, D3 v) {
    const double pw = ((-(x * v.x)) - y * v.y) - z * v.z;
    const double px = (w * v.x + y * v.z) - z * v.y;
    const double py = (w * v.y - x * v.z) + z * v.x;
    const double pz = (w * v.z + x * v.y) - y * v.x;
    const double cx = -x, cy = -y, cz = -z;  // conjugate
    return d3(((pw * cx + px * w) + py * cz) - pz * cy, ((pw * cy - px * cz) + py * w) + pz * cx,
              ((pw * cz + px * cy) - py * cx) + pz * w);
}
// Transform::detransform (shapes.rs:80-84): conj(q).rotate_vector(v - offset) / scale
// 1: a Transform whose scale is exactly (1, 1, 1) (the reference's `None`,
// every Transform of C3 and C5) skips the three f64 divisions: x / 1.0 is x,
// bit for bit, NaN, infinities and signed zeros included
__device__ __forceinline__ D3 xf_in(const DXform& X, D3 v) {
    const D3 p = quat_rotate(X.q[0], -X.q[1], -X.q[2], -X.q[3], v - d3(X.off[0], X.off[1], X.off[2]));
    if (X.flags & XF_UNIT_SCALE) return p;
    return p / d3(X.scale[0], X.scale[1], X.scale[2]);
}
// Transform::transform (shapes.rs:74-78): q.rotate_vector(v * scale) + offset
__device__ __forceinline__ D3 xf_out(const DXform& X, D3 v) {
    return quat_rotate(X.q[0], X.q[1], X.q[2], X.q[3], v * d3(X.scale[0], X.scale[1], X.scale[2])) +
           d3(X.off[0], X.off[1], X.off[2]);
}
// shapes.rs:93-99 local ray
__device__ __forceinline__ Ray xf_ray(const DXform& X, const Ray& r) {
    const D3 lo = xf_in(X, r.o);
    const D3 lt = xf_in(X, r.o + 1.0 * r.d);
    return Ray{lo, lt - lo, r.time};
}

// The Transforms entered on the way to a hit, innermost last.  Two named
// fields, not an array: a dynamically indexed private array is placed in
// scratch memory by the compiler.
struct XfIds {
    uint32_t a = 0, b = 0;
    __device__ __forceinline__ uint32_t get(uint32_t k) const { return k == 0 ? a : b; }
    __device__ __forceinline__ void set(uint32_t k, uint32_t v) {
        if (k == 0)
            a = v;
        else
            b = v;
    }
};

struct HitInfo {
    double t;
    uint32_t ref;
    uint32_t nxf;
    XfIds xf;
};

// The per-lane traversal stack: entry k of lane l at stk[k * RT_BLOCK] (the
// pointer is already offset by the lane), {ref, entry distance as f32 rounded
// down} -- one ds_write_b64 / ds_read_b64 per push / pop, 64 distinct banks
// per half-wave.  With OVF, entries k >= CAP (deep triangle BVHs) live in the
// lane's column of a global overflow buffer, [k - CAP][lane of the grid], so
// the LDS part stays small enough for 4 blocks per CU.
template <uint32_t CAP, bool OVF, uint32_t BLK>
struct StackT {
    RT_LDS uint2* base;  // explicitly LDS: a select against ovf must not become a flat pointer
    RT_GLOBAL uint2* ovf;
    uint32_t stride;
    // The overflow side moves the entry as one 64-bit word and the LDS side
    // as a uint2: different instructions, so the optimizer cannot merge the
    // two accesses into one through a phi of flat pointers (which also hit a
    // gfx950 code-generation error on an LDS-to-flat cast in the flat tier).
    __device__ __forceinline__ void push(uint32_t sp, uint32_t ref, float t) {
        if (OVF && sp >= CAP)
            reinterpret_cast<RT_GLOBAL unsigned long long*>(ovf)[(sp - CAP) * stride] =
                ((unsigned long long)__float_as_uint(t) << 32) | ref;
        else
            base[sp * BLK] = make_uint2(ref, __float_as_uint(t));
    }
    __device__ __forceinline__ uint2 at(uint32_t sp) const {
        if (OVF && sp >= CAP) {
            const unsigned long long v = reinterpret_cast<const RT_GLOBAL unsigned long long*>(ovf)[(sp - CAP) * stride];
            return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
        }
        return base[sp * BLK];
    }
};
// Basic tier: 4-B entries -- a list flag and a 15-bit node / list
// index, and the upper 16 bits of the entry distance (a positive f32 cut to
// 16 bits is rounded down: the cull stays conservative; -inf stays -inf).
// The block's stack takes half the LDS; the rest parks walk state.
template <uint32_t CAP, uint32_t BLK>
struct StackB4 {
    RT_LDS uint32_t* base;
    __device__ __forceinline__ void push(uint32_t sp, uint32_t ref, float t) {
        const uint32_t r16 = (ref_kind(ref) == K_LIST ? 0x8000u : 0u) | (ref_index(ref) & 0x7fffu);
        base[sp * BLK] = (r16 << 16) | (__float_as_uint(t) >> 16);
    }
    __device__ __forceinline__ uint2 at(uint32_t sp) const {
        const uint32_t e = base[sp * BLK], r16 = e >> 16;
        return make_uint2(make_ref((r16 & 0x8000u) ? K_LIST : K_BVH, r16 & 0x7fffu), e << 16);
    }
    // The 4-wide basic tier's walk keeps its refs as "words" (bword): a
    // box child's 16-bit stack code in the upper half -- push is one byte
    // permute with the entry distance, pop one mask
    __device__ __forceinline__ void push_w(uint32_t sp, uint32_t word, float t) {
        base[sp * BLK] = __builtin_amdgcn_perm(word, __float_as_uint(t), 0x07060302u);
    }
    __device__ __forceinline__ uint2 at_w(uint32_t sp) const {
        const uint32_t e = base[sp * BLK];
        return make_uint2(e & 0xffff0000u, e << 16);
    }
};
// Basic-tier walk words (the 4-wide walk's cur, stack entries and the ref
// row of the block's LDS node copy): 0 = none; a node = (index + 1) << 16;
// a list position = (0x8000 | index) << 16; a sphere = 0x8000 | index (low
// half).  So a box child is word > 0xffff, a sphere child has a nonzero low
// half, and the upper half is the stack entry's ref code as it stands.
// Indices: nodes < 0x7fff (the LDS copy holds 658), lists < 0x8000 and
// spheres < 0x8000 (rt_render.cpp prepare_tier).
__device__ __forceinline__ uint32_t bword(const SceneView& S, uint32_t ref) {
    const uint32_t k = ref_kind(ref), i = ref_idx(S, ref);
    return k == K_BVH ? (i + 1u) << 16 : k == K_LIST ? (0x8000u | i) << 16 : k == K_SPHERE ? (0x8000u | i) : 0u;
}
template <class Stack>
__device__ __forceinline__ uint32_t pop_w(const Stack& stk, uint32_t& sp, float c_f) {
    while (sp > 0) {
        --sp;
        const uint2 e = stk.at_w(sp);
        if (__uint_as_float(e.y) <= c_f) return e.x;
    }
    return 0u;
}
template <int TIER, bool B4 = TIER == TIER_BASIC>
struct StackSel {
    using type = StackT<lds_stack_entries(TIER), TIER != TIER_BASIC, TIER == TIER_BASIC ? RT_BLOCK_BASIC : RT_BLOCK>;
};
template <int TIER>
struct StackSel<TIER, true> {
    using type = StackB4<lds_stack_entries(TIER), RT_BLOCK_BASIC>;
};
template <int TIER>
using StackFor = typename StackSel<TIER>::type;

// Closest-hit state of one traversal: t and its f32 upper bound.
struct Closest {
    double c;
    float c_f;
    // c_f = (float)t plus at least one ulp: an upper bound of t in two
    // instructions (|f| * 2^-23 >= 1 ulp of f, and (float)t is within half an
    // ulp), where the exact round-up takes a compare-and-step sequence.
    __device__ __forceinline__ void set(double t) {
        c = t;
        const float f = (float)t;
        c_f = fmaf(fabsf(f), 1.1920928955078125e-07f, f);
    }
    // a hit t <= c found while c_f may already be a tighter bound (sphere filter)
    __device__ __forceinline__ void lower(double t) {
        c = t;
        const float f = (float)t;
        c_f = fminf(c_f, fmaf(fabsf(f), 1.1920928955078125e-07f, f));
    }
};

// One BVH node visit (one 80-B record): a sphere child is intersected right
// here from the data in its slot (sphere.rs:77-108); other children get the
// f32 slab test, and the hit ones are walked near-first with the farther one
// pushed with its entry distance.
template <class Stack, class OnHit>
__device__ __forceinline__ uint32_t visit_node(const SceneView& S, uint32_t idx, const Ray& r, const RayF& rf,
                                               double a, double inva, double tmin, float tmin_f, Closest& cl,
                                               Stack& stk, uint32_t& sp, OnHit&& on_hit) {
    const RT_GLOBAL float4* np = reinterpret_cast<const RT_GLOBAL float4*>(S.nodes + idx);
    const float4 q0 = np[0], q1 = np[1], q2 = np[2], q3 = np[3], q4 = np[4];
    const uint32_t c0 = __float_as_uint(q4.x), c1 = __float_as_uint(q4.y);
    bool h0 = false, h1 = false;
    float e0 = 0.0f, e1 = 0.0f;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t ch = k ? c1 : c0;
        const float4 qa = k ? q2 : q0, qb = k ? q3 : q1;
        bool& hk = k ? h1 : h0;
        float& ek = k ? e1 : e0;
        if (ch == REF_NONE) continue;
        if (ref_kind(ch) == K_SPHERE) {
            const double cx = __hiloint2double(__float_as_int(qa.y), __float_as_int(qa.x));
            const double cy = __hiloint2double(__float_as_int(qa.w), __float_as_int(qa.z));
            const double cz = __hiloint2double(__float_as_int(qb.y), __float_as_int(qb.x));
            const double rr = __hiloint2double(__float_as_int(qb.w), __float_as_int(qb.z));
            double t;
            if (sphere_t_inv(d3(cx, cy, cz), rr, r, a, inva, tmin, cl.c, t)) {
                cl.set(t);
                on_hit(ch, t);
            }
        } else {
            const float lo[3] = {qa.x, qa.y, qa.z}, hi[3] = {qa.w, qb.x, qb.y};
            hk = slab_f(lo, hi, rf, tmin_f, cl.c_f, ek);
        }
    }
    h0 = h0 && e0 <= cl.c_f;
    h1 = h1 && e1 <= cl.c_f;
    if (h0 && h1) {
        const bool first0 = e0 <= e1;
        stk.push(sp++, first0 ? c1 : c0, first0 ? e1 : e0);
        return first0 ? c0 : c1;
    }
    return h0 ? c0 : (h1 ? c1 : REF_NONE);
}

// Pops until an entry whose box can still hold a hit closer than c.
template <class Stack>
__device__ __forceinline__ uint32_t pop(const Stack& stk, uint32_t& sp, uint32_t sp0, float c_f) {
    while (sp > sp0) {
        --sp;
        const uint2 e = stk.at(sp);
        if (__uint_as_float(e.y) <= c_f) return e.x;
    }
    return REF_NONE;
}

constexpr float NO_CULL = -__builtin_huge_valf();
// The flat tier tests the f32 box of a compound list element (a Transform, a
// ConstantMedium, a nested list) before entering it, with the ray's f32 form
// made on the spot: a ray that misses the box skips the element's whole
// walk -- for C3's smoke box the two boundary walks of media_phase.  (Testing
// every element's box, primitives included, with the f32 ray parked in LDS
// was 4.6 % slower: a wall's box test costs what its exact test does.)
template <int TIER>
constexpr bool flat_boxes() { return TIER == TIER_FULL_FLAT; }
template <int TIER>
constexpr bool unified_load() {
    return (TIER == TIER_MESH && RT_MESH_BVH4) || (tier_full_bvh(TIER) && RT_FULL_BVH4);
}
// the two doubles of a float4 read from a double record
__device__ __forceinline__ double f4_lo(float4 q) { return __hiloint2double(__float_as_int(q.y), __float_as_int(q.x)); }
__device__ __forceinline__ double f4_hi(float4 q) { return __hiloint2double(__float_as_int(q.w), __float_as_int(q.z)); }
template <int TIER>
constexpr bool flat_runs() { return TIER == TIER_FULL_FLAT; }

// The flat tier's list step tests an element's f32 box (list_boxes, rounded
// outward; the conservative slab of rt_slab.h) before the element: a ray
// that misses the box within [tmin, c] cannot hit the element closer than c
// (for a ConstantMedium: cannot enter its boundary there), so skipping it
// keeps the list's closest hit -- the role a BVH node's boxes play, without
// the BVH code.
__device__ __forceinline__ bool list_box_hit(const SceneView& S, uint32_t li, const RayF& rf, float tmin_f,
                                             float c_f) {
    const RT_GLOBAL float4* bp = reinterpret_cast<const RT_GLOBAL float4*>(S.list_boxes + li);
    const float4 b0 = bp[0], b1 = bp[1];
    const float lo[3] = {b0.x, b0.y, b0.z}, hi[3] = {b0.w, b1.x, b1.y};
    float e;
    return slab_f(lo, hi, rf, tmin_f, c_f, e);
}

// Closest t of a medium boundary (no media inside, no records) -- the two
// boundary.hit calls of volume.rs:44-48.
template <bool BVH, class Stack>
__device__ bool boundary_t(const SceneView& S, uint32_t root, const Ray& r0, double tmin, double tmax, Stack& stk,
                           uint32_t sp0, double& tbest) {
    Ray r = r0;
    RayF rf = make_rayf(r);
    double a = len2(r.d), inva = 1.0 / a;
    XfIds xfs;
    uint32_t nxf = 0;
    uint32_t sp = sp0;
    uint32_t cur = root;
    const float tmin_f = f32_down(tmin);
    Closest cl;
    cl.set(tmax);
    bool found = false;
    auto on_hit = [&](uint32_t, double) { found = true; };
    for (;;) {
        if (cur == REF_NONE) {
            cur = pop(stk, sp, sp0, cl.c_f);
            if (cur == REF_NONE) break;
        }
        uint32_t after = REF_NONE;  // as trace_step: a primitive list element is tested in the list step
        if (ref_kind(cur) == K_LIST) {
            const uint32_t li = ref_idx(S, cur);
            const uint32_t child = S.list_children[li];
            cur = REF_NONE;
            if (child == REF_NONE) continue;
            const uint32_t nxt = S.list_children[li + 1] != REF_NONE ? make_ref(K_LIST, li + 1) : REF_NONE;
            const uint32_t ck = ref_kind(child);
            if (ck == K_SPHERE || ck == K_QUAD || ck == K_TRI || ck == K_MSPHERE) {
                cur = child;
                after = nxt;
            } else {
                if (nxt != REF_NONE) stk.push(sp++, nxt, NO_CULL);
                cur = child;
                continue;
            }
        }
        const uint32_t kind = ref_kind(cur), idx = ref_idx(S, cur);
        cur = REF_NONE;
        double t;
        switch (kind) {
            case K_BVH:
                if constexpr (!BVH)
                    break;
                else if constexpr (RT_FULL_BVH4)
                    cur = visit4_boxes(S, idx, rf, tmin_f, cl.c_f, stk, sp);
                else
                    cur = visit_node(S, idx, r, rf, a, inva, tmin, tmin_f, cl, stk, sp, on_hit);
                break;
            case K_SPHERE: {
                const double4 s = S.spheres[idx];
                if (sphere_t_inv(d3(s.x, s.y, s.z), s.w, r, a, inva, tmin, cl.c, t)) {
                    cl.set(t);
                    found = true;
                }
                break;
            }
            case K_MSPHERE: {
                const double4 s = S.msph_center[idx], m = S.msph_dir[idx];
                const D3 cc = d3(s.x, s.y, s.z) + r.time * d3(m.x, m.y, m.z);
                if (sphere_t_inv(cc, s.w, r, a, inva, tmin, cl.c, t)) {
                    cl.set(t);
                    found = true;
                }
                break;
            }
            case K_QUAD:
            case K_TRI:
                if (planar_t_filtered(S, idx, kind == K_TRI, r, tmin, cl.c, cl.c_f, t)) {
                    cl.set(t);
                    found = true;
                }
                break;
            case K_XFORM: {
                const DXform& X = S.xforms[idx];
                stk.push(sp++, make_ref(K_POPXF, 0), NO_CULL);
                xfs.set(nxf++, idx);
                r = xf_ray(X, r);
                rf = make_rayf(r);
                a = len2(r.d);
                inva = 1.0 / a;
                cur = X.child;
                break;
            }
            case K_POPXF: {
                --nxf;
                r = r0;
                for (uint32_t k = 0; k < nxf; ++k) r = xf_ray(S.xforms[xfs.get(k)], r);
                rf = make_rayf(r);
                a = len2(r.d);
                inva = 1.0 / a;
                break;
            }
            default: break;
        }
        if (after != REF_NONE) cur = after;
    }
    tbest = cl.c;
    return found;
}

// ConstantMedium::hit (volume.rs:37-73) of medium idx for ray r in the
// medium's frame, interval [tmin, tmax]: the two boundary hits are one
// boundary walk run twice (one copy of the walk in the code).
// The two boundary hits of a boundary made of one sphere or of planar_n
// consecutive quads / triangles (rt_scene.cpp planar_boundary) in one pass.  A
// planar test's t and inside decision do not depend on the interval (quad.rs:
// 71-102: the interval only accepts or rejects the t already computed), so
// each element is tested once over (-inf, inf) and its t kept; the first hit
// is the least t (Hittables::hit, hits.rs:34-46), the second the least t >=
// t1 + 0.0001 -- the values and decisions of the two walks of volume.rs:44-48,
// without the list walk and with one planar test per element instead of two.
__device__ __forceinline__ bool boundary_onepass(const SceneView& S, const DMedium& M, const Ray& r0, double& t1,
                                                double& t2) {
    const double NINF = -__builtin_huge_val(), PINF = __builtin_huge_val();
    Ray r = r0;  // into the frame of the Transforms around the elements, as the walk does
    for (uint32_t j = 0; j < M.bxf_n; ++j) r = xf_ray(S.xforms[j == 0 ? M.bxf[0] : M.bxf[1]], r);
    if (M.bsphere) {
        // sphere.rs:77-92 over (-inf, inf), then over [t1 + 0.0001, inf):
        // the same roots, chosen by each interval as sphere_t_inv chooses
        const double4 s4 = S.spheres[M.bsphere - 1];
        const double a = len2(r.d), inva = 1.0 / a;
        const D3 oc = d3(s4.x, s4.y, s4.z) - r.o;
        const double h = dot(r.d, oc);
        const double cc = len2(oc) - s4.w * s4.w;
        const double disc = h * h - a * cc;
        if (disc < 0.0) return false;
        const double sq = k_sqrt(disc);
        const double rn = div_a(h - sq, a, inva), rf = div_a(h + sq, a, inva);
        auto pick = [&](double lo, double& t) {
            if (rn >= lo && rn <= PINF) t = rn;
            else if (rf >= lo && rf <= PINF) t = rf;
            else return false;
            return true;
        };
        if (!pick(NINF, t1)) return false;
        return pick(fmin(t1 + 0.0001, PINF), t2);
    }
    double tv[RT_MED_PLANAR_MAX];
    bool any = false;
    t1 = PINF;
#pragma unroll
    for (uint32_t k = 0; k < RT_MED_PLANAR_MAX; ++k) {
        tv[k] = __builtin_nan("");
        double tt;
        if (k < M.planar_n && planar_t(S.planars[M.planar_first + k], (M.tri_mask >> k) & 1u, r, NINF, PINF, tt)) {
            tv[k] = tt;
            t1 = any ? fmin(t1, tt) : tt;
            any = true;
        }
    }
    if (!any) return false;
    const double lo = fmin(t1 + 0.0001, PINF);
    any = false;
    t2 = PINF;
#pragma unroll
    for (uint32_t k = 0; k < RT_MED_PLANAR_MAX; ++k) {
        if (tv[k] >= lo && tv[k] <= PINF) {  // NaN (no hit) fails both
            t2 = any ? fmin(t2, tv[k]) : tv[k];
            any = true;
        }
    }
    return any;
}

template <bool BVH, class Stack>
__device__ __forceinline__ bool medium_hit(const SceneView& S, uint32_t idx, const Ray& r, double tmin, double tmax,
                                           Stack& stk, uint32_t sp0, const Rng& rng, double& t) {
    const DMedium M = S.media[idx];
    const double NINF = -__builtin_huge_val(), PINF = __builtin_huge_val();
    double t1 = 0.0, t2 = 0.0, lo = NINF;
    if (M.planar_n || M.bsphere) {
        if (!boundary_onepass(S, M, r, t1, t2)) return false;
    } else {
#pragma nounroll
        for (int pass = 0; pass < 2; ++pass) {
            double tb;
            if (!boundary_t<BVH>(S, M.boundary, r, lo, PINF, stk, sp0, tb)) return false;
            if (pass == 0) {
                t1 = tb;
                lo = fmin(t1 + 0.0001, PINF);
            } else {
                t2 = tb;
            }
        }
    }
    if (t1 < tmin) t1 = tmin;
    if (t2 > tmax) t2 = tmax;
    if (t1 >= t2) return false;
    if (t1 < 0.0) t1 = 0.0;
    const double ray_length = len(r.d);
    const double inside = (t2 - t1) * ray_length;
    const double hd = M.neg_inv_density * k_log(rng.medium(M.medium_id));
    if (hd > inside) return false;
    t = t1 + hd / ray_length;  // volume.rs:65
    return t <= tmax;
}

// world.hit(r, [1e-8, inf)) (camera.rs:286) as a depth-first walk with one
// running closest t.  Lists are walked in order with the interval shrunk to
// the best hit so far (hits.rs:34-46 tests every child with the full interval
// and keeps the first minimum: the same closest hit up to exact t ties).
//
// The walk is resumable: Trav holds its whole state, trace_step advances it by
// one stack entry, so a lane whose walk ends can be shaded and handed its next
// ray while the other lanes of its wave keep walking (rt_path_kernel).
template <int TIER>
struct Trav {
    Ray r;  // the ray in the frame of the innermost Transform entered (FULL only)
    RayF rf;
    double a, inva;  // |d|^2 and its correctly rounded reciprocal
    Closest cl;
    uint32_t cur, sp, nxf;
    XfIds xfs;
    bool found;
    HitInfo hit;
    uint32_t nmed;  // FULL: media met by the walk, tested after it (media_phase)
    SphF sf;        // BASIC (4-wide): the sphere filter's per-ray f32 data
    uint32_t pn;    // and the number of spheres queued for the exact test
};

template <int TIER>
__device__ __forceinline__ void trace_begin(const SceneView& S, const Ray& wr, Trav<TIER>& T) {
    T.r = wr;
    T.rf = make_rayf(wr);
    T.a = len2(wr.d);
    T.inva = 1.0 / T.a;
    T.cl.c = __builtin_huge_val();
    T.cl.c_f = __builtin_huge_valf();
    T.cur = S.world_root;
    T.sp = 0;
    T.nxf = 0;
    T.found = false;
    T.hit.nxf = 0;
    T.nmed = 0;
    if constexpr (TIER == TIER_BASIC && RT_BVH4) {
        const double o[3] = {wr.o.x, wr.o.y, wr.o.z}, d[3] = {wr.d.x, wr.d.y, wr.d.z};
        T.sf = make_sphf(o, d);
        T.pn = 0;
        T.cur = bword(S, S.world_root);  // the 4-wide walk's cur is a walk word
    }
}

// Mesh tier with shading batches: the same 8 words; the f32
// ray, |d|^2 and its reciprocal are made again from the world ray on resume.
template <class Park>
__device__ __forceinline__ void trace_park(const Trav<TIER_MESH>& T, Park pk) {
    constexpr uint32_t B = RT_BLOCK;
    const uint64_t c = (uint64_t)__double_as_longlong(T.cl.c), ht = (uint64_t)__double_as_longlong(T.hit.t);
    pk[0 * B] = T.cur;
    pk[1 * B] = T.sp | ((uint32_t)T.found << 16);
    pk[2 * B] = (uint32_t)c;
    pk[3 * B] = (uint32_t)(c >> 32);
    pk[4 * B] = __float_as_uint(T.cl.c_f);
    pk[5 * B] = (uint32_t)ht;
    pk[6 * B] = (uint32_t)(ht >> 32);
    pk[7 * B] = T.hit.ref;
}
template <class Park>
__device__ __forceinline__ void trace_unpark(const Ray& wr, Trav<TIER_MESH>& T, Park pk) {
    constexpr uint32_t B = RT_BLOCK;
    T.cur = pk[0 * B];
    const uint32_t w = pk[1 * B];
    T.sp = w & 0xffffu;
    T.found = (w >> 16) & 1u;
    T.cl.c = __hiloint2double((int)pk[3 * B], (int)pk[2 * B]);
    T.cl.c_f = __uint_as_float(pk[4 * B]);
    T.hit.t = __hiloint2double((int)pk[6 * B], (int)pk[5 * B]);
    T.hit.ref = pk[7 * B];
    T.rf = make_rayf(wr);
    T.a = len2(wr.d);
    T.inva = 1.0 / T.a;
}
// Basic tier with shading batches: a carried-over walk's state is parked in
// LDS across the shading round as four 8-byte rows -- {cur, sp | pn | found},
// c, {c_f, hit ref}, hit t: two ds_write2st64_b64 / ds_read2st64_b64 a park
// and a resume, not four of the 4-byte kind (C2 -0.2 %, A/B at 128 spp, 5
// reps, RMSE 0: profiles/r05/ab_park64_c2_128spp.json).  The ray-derived
// fields are made again on resume (trace_ray_fields), as for a new walk.
__device__ __forceinline__ void trace_park2(const Trav<TIER_BASIC>& T, RT_LDS uint2* pk) {
    constexpr uint32_t B = RT_BLOCK_BASIC;
    const uint64_t c = (uint64_t)__double_as_longlong(T.cl.c), ht = (uint64_t)__double_as_longlong(T.hit.t);
    pk[0 * B] = make_uint2(T.cur, T.sp | (T.pn << 8) | ((uint32_t)T.found << 16));
    pk[1 * B] = make_uint2((uint32_t)c, (uint32_t)(c >> 32));
    pk[2 * B] = make_uint2(__float_as_uint(T.cl.c_f), T.hit.ref);
    pk[3 * B] = make_uint2((uint32_t)ht, (uint32_t)(ht >> 32));
}
__device__ __forceinline__ void trace_unpark_state2(Trav<TIER_BASIC>& T, const RT_LDS uint2* pk) {
    constexpr uint32_t B = RT_BLOCK_BASIC;
    const uint2 w0 = pk[0 * B], w1 = pk[1 * B], w2 = pk[2 * B], w3 = pk[3 * B];
    T.cur = w0.x;
    T.sp = w0.y & 0xffu;
    T.pn = (w0.y >> 8) & 0xffu;
    T.found = (w0.y >> 16) & 1u;
    T.cl.c = __hiloint2double((int)w1.y, (int)w1.x);
    T.cl.c_f = __uint_as_float(w2.x);
    T.hit.ref = w2.y;
    T.hit.t = __hiloint2double((int)w3.y, (int)w3.x);
}
__device__ __forceinline__ void trace_ray_fields(const Ray& wr, Trav<TIER_BASIC>& T) {
    T.rf = make_rayf(wr);
    T.a = len2(wr.d);
    T.inva = 1.0 / T.a;
    const double o[3] = {wr.o.x, wr.o.y, wr.o.z}, d[3] = {wr.d.x, wr.d.y, wr.d.z};
    T.sf = make_sphf(o, d);
}
// The world-frame ray as the walk reads it: a register copy, or (full-flat
// tier) the lane's LDS copy, read only where a walk step
// needs it (leaving a Transform, the media phase) so that it holds no
// registers across the walk.
struct RayReg {
    const Ray& r;
    __device__ __forceinline__ Ray get() const { return r; }
};
struct RayLds {
    const RT_LDS double* p;  // 7 doubles, RT_BLOCK apart: o, d, time
    __device__ __forceinline__ Ray get() const {
        Ray r;
        r.o = d3(p[0 * RT_BLOCK], p[1 * RT_BLOCK], p[2 * RT_BLOCK]);
        r.d = d3(p[3 * RT_BLOCK], p[4 * RT_BLOCK], p[5 * RT_BLOCK]);
        r.time = p[6 * RT_BLOCK];
        return r;
    }
};
__device__ __forceinline__ RayReg world_ray(const Ray& r) { return RayReg{r}; }
__device__ __forceinline__ const RayLds& world_ray(const RayLds& r) { return r; }

// A lane's media queue (full tiers) in the lane rows of the LDS arena:
// entry k = {medium, nxf, xf a, xf b} in rows 2k and 2k + 1 (uint2, RT_BLOCK
// apart), so that it shares the one per-lane base address of the stack and
// the parked path state (rt_path_kernel's lane arena)
struct MedQ {
    RT_LDS uint2* p;
    __device__ __forceinline__ void set(uint32_t k, uint4 v) const {
        p[(2 * k) * RT_BLOCK] = make_uint2(v.x, v.y);
        p[(2 * k + 1) * RT_BLOCK] = make_uint2(v.z, v.w);
    }
    __device__ __forceinline__ uint4 get(uint32_t k) const {
        const uint2 a = p[(2 * k) * RT_BLOCK], b = p[(2 * k + 1) * RT_BLOCK];
        return make_uint4(a.x, a.y, b.x, b.y);
    }
};

// One stack entry of the walk; false when the walk is over (T.found, T.hit hold the result).
template <int TIER, class WR>
__device__ __forceinline__ bool trace_step(const SceneView& S, const WR& wrr, Trav<TIER>& T, StackFor<TIER>& stk,
                                           const Rng& rng, MedQ med, Diag& dg) {
    const auto wq = world_ray(wrr);
    constexpr bool FULL = tier_full(TIER);
    constexpr double tmin = 1e-8;
    const float tmin_f = f32_down(tmin);
    if (T.cur == REF_NONE) {
        T.cur = pop(stk, T.sp, 0, T.cl.c_f);
        if (T.cur == REF_NONE) return false;
    }
    const Ray& r = FULL ? T.r : wq.get();
    uint32_t cur = T.cur;
    T.cur = REF_NONE;
    auto record = [&](uint32_t ref, double tt) {
        T.found = true;
        T.hit.t = tt;
        T.hit.ref = ref;
        if constexpr (FULL) {
            T.hit.nxf = T.nxf;
            T.hit.xf = T.xfs;
        }
    };
    // A list step whose element is a primitive tests it right here and goes
    // on with the next element (no stack round trip, one step per element);
    // a compound element (BVH, Transform, medium, list) is walked next with
    // the rest of the list pushed.
    uint32_t after = REF_NONE;
    if (ref_kind(cur) == K_LIST) {
        const uint32_t li = ref_idx(S, cur);
        const uint32_t child = S.list_children[li];
        if (child == REF_NONE) return true;  // empty list
        if constexpr (flat_runs<TIER>()) {
            // the flat tier tests a run of planar elements (the Cornell walls,
            // a box's six faces) in one step, in list order, each against the
            // closest t so far -- what the run's single steps do
            const uint32_t ck0 = ref_kind(child);
            if (ck0 == K_QUAD || ck0 == K_TRI) {
                const uint32_t run = S.list_boxes[li].run, n = run & 0xffu, first = ref_idx(S, child);
                check_run(S, first, n);
                RT_DIAG_ONLY(dg.sphere_tests += n;)
                for (uint32_t k = 0; k < n; ++k) {
                    const bool tri = (run >> (8u + k)) & 1u;
                    double tt;
                    if (planar_t_filtered(S, first + k, tri, r, tmin, T.cl.c, T.cl.c_f, tt)) {
                        T.cl.set(tt);
                        record(make_ref(tri ? K_TRI : K_QUAD, first + k), tt);
                    }
                }
                T.cur = S.list_children[li + n] != REF_NONE ? make_ref(K_LIST, li + n) : REF_NONE;
                return true;
            }
        }
        const uint32_t nxt = S.list_children[li + 1] != REF_NONE ? make_ref(K_LIST, li + 1) : REF_NONE;
        if constexpr (flat_boxes<TIER>()) {
            const uint32_t ck = ref_kind(child);
            if (ck != K_SPHERE && ck != K_QUAD && ck != K_TRI && ck != K_MSPHERE) {
                const bool in_box = list_box_hit(S, li, make_rayf(r), tmin_f, T.cl.c_f);
                // a ConstantMedium element whose box the ray meets is queued
                // for the media phase right here (K_MEDIUM below), without a
                // step of its own and the pop of the rest of the list
                const bool queue = in_box && ck == K_MEDIUM && T.nmed < RT_MEDIA_CAP;
                if (queue) {
                    med.set(T.nmed, make_uint4(ref_idx(S, child), T.nxf, T.xfs.a, T.xfs.b));
                    ++T.nmed;
                }
                if (!in_box || queue) {
                    T.cur = nxt;
                    return true;
                }
            }
        }
        const uint32_t ck = ref_kind(child);
        if (ck == K_SPHERE || ck == K_QUAD || ck == K_TRI || (FULL && ck == K_MSPHERE)) {
            cur = child;
            after = nxt;
        } else {
            if (nxt != REF_NONE) stk.push(T.sp++, nxt, NO_CULL);
            T.cur = child;
            return true;
        }
    }
    const uint32_t kind = ref_kind(cur), idx = ref_idx(S, cur);
    const uint32_t this_ref = cur;
    double t;
    bool got = false;
    RT_DIAG_ONLY(if (kind == K_BVH) ++dg.node_visits; if (kind == K_SPHERE || kind == K_TRI || kind == K_QUAD) ++dg.sphere_tests;)
    if (unified_load<TIER>() && (kind == K_BVH || kind == K_SPHERE || kind == K_TRI || kind == K_QUAD)) {
        // One load for the step's record, whatever it is: a node's 7 rows, a
        // quad's / triangle's 128 B, a sphere's 32 B, read as 8 dwordx4 from
        // the record's address (the world blob is padded past every array).
        // In a wave whose lanes hold nodes and primitives both, the node
        // visit and the primitive test then wait on one memory latency, not
        // one after the other.
        const bool planar = kind == K_TRI || kind == K_QUAD;
        // (the array addresses as values, selected: a select between the
        // SceneView's members made the compiler index a scratch copy of it)
        const uint64_t a_node = (uint64_t)S.nodes4, a_planar = (uint64_t)S.planars, a_sphere = (uint64_t)S.spheres;
        uint64_t addr = a_node;
        uint32_t stride = 0u;
        if (kind == K_BVH) stride = (uint32_t)sizeof(DNode4);
        if (planar) addr = a_planar, stride = (uint32_t)sizeof(DPlanar);
        if (kind == K_SPHERE) addr = a_sphere, stride = (uint32_t)sizeof(double4);
        const RT_GLOBAL float4* q = reinterpret_cast<const RT_GLOBAL float4*>(addr + (uint64_t)idx * stride);
#ifdef RT_DIAG
        {  // how often a wave's lanes read one record (the scalar-load case)
            const uint64_t ra = addr + (uint64_t)idx * stride;
            const uint32_t lo = (uint32_t)ra, hi = (uint32_t)(ra >> 32);
            const bool same = lo == __builtin_amdgcn_readfirstlane(lo) && hi == __builtin_amdgcn_readfirstlane(hi);
            const unsigned long long act = __ballot(true), sm = __ballot(same);
            if (__lane_id() == (uint32_t)(__ffsll((long long)act) - 1)) {
                ++dg.u_steps;
                dg.u_active += (unsigned long long)__popcll(act);
                dg.u_same += (unsigned long long)__popcll(sm);
                if (sm == act) {
                    ++dg.u_uniform;
                    if (kind == K_BVH) ++dg.u_uniform_node;
                }
            }
            constexpr uint32_t TOPK[4] = {5u, 21u, 85u, 341u};
            if (kind == K_BVH) ++dg.l_node;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool top = kind == K_BVH && idx < TOPK[k];
                if (top) ++dg.l_top[k];
                if (__ballot(top) == act && __lane_id() == (uint32_t)(__ffsll((long long)act) - 1)) ++dg.u_top[k];
            }
        }
#endif
        // rows 0-3 hold a sphere (2) and half a planar record; the rest
        // only for the lanes whose record has them
        const float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
        float4 q4 = make_float4(0.f, 0.f, 0.f, 0.f), q5 = q4, q6 = q4, q7 = q4;
        if (planar || kind == K_BVH) q4 = q[4], q5 = q[5], q6 = q[6];
        if (planar) q7 = q[7];
        if (kind == K_BVH) {
            T.cur = visit4_boxes_rows(q0, q1, q2, q3, q4, q5, q6, T.rf, tmin_f, T.cl.c_f, stk, T.sp);
        } else if (kind == K_SPHERE) {
            got = sphere_t_inv(d3(f4_lo(q0), f4_hi(q0), f4_lo(q1)), f4_hi(q1), r, T.a, T.inva, tmin, T.cl.c, t);
        } else if (planar) {
            got = planar_t_v(d3(f4_lo(q0), f4_hi(q0), f4_lo(q1)), f4_hi(q1), d3(f4_lo(q2), f4_hi(q2), f4_lo(q3)),
                             d3(f4_hi(q3), f4_lo(q4), f4_hi(q4)), d3(f4_lo(q5), f4_hi(q5), f4_lo(q6)),
                             d3(f4_hi(q6), f4_lo(q7), f4_hi(q7)), kind == K_TRI, r, tmin, T.cl.c, t);
        }
        if (got) {
            T.cl.set(t);
            record(this_ref, t);
        }
        if (after != REF_NONE) T.cur = after;
        return true;
    }
    if (TIER != TIER_FULL_FLAT && kind == K_BVH) {
        if constexpr ((TIER == TIER_MESH && RT_MESH_BVH4) || (tier_full_bvh(TIER) && RT_FULL_BVH4))
            T.cur = visit4_boxes(S, idx, T.rf, tmin_f, T.cl.c_f, stk, T.sp);
        else
            T.cur = visit_node(S, idx, r, T.rf, T.a, T.inva, tmin, tmin_f, T.cl, stk, T.sp, record);
    } else if (kind == K_SPHERE) {
        const double4 sp4 = S.spheres[idx];
        got = sphere_t_inv(d3(sp4.x, sp4.y, sp4.z), sp4.w, r, T.a, T.inva, tmin, T.cl.c, t);
    } else if constexpr (TIER == TIER_MESH) {
        if (kind == K_TRI || kind == K_QUAD) got = planar_t_filtered(S, idx, kind == K_TRI, r, tmin, T.cl.c, T.cl.c_f, t);
    } else if constexpr (FULL) {
        switch (kind) {
            case K_MSPHERE: {
                const double4 s4 = S.msph_center[idx], m = S.msph_dir[idx];
                const D3 cc = d3(s4.x, s4.y, s4.z) + r.time * d3(m.x, m.y, m.z);
                got = sphere_t_inv(cc, s4.w, r, T.a, T.inva, tmin, T.cl.c, t);
                break;
            }
            case K_QUAD:
            case K_TRI: got = planar_t_filtered(S, idx, kind == K_TRI, r, tmin, T.cl.c, T.cl.c_f, t); break;
            case K_XFORM: {
                const DXform& X = S.xforms[idx];
                stk.push(T.sp++, make_ref(K_POPXF, 0), NO_CULL);
                T.xfs.set(T.nxf++, idx);
                T.r = xf_ray(X, T.r);
                T.rf = make_rayf(T.r);
                T.a = len2(T.r.d);
                T.inva = 1.0 / T.a;
                T.cur = X.child;
                break;
            }
            case K_POPXF: {
                --T.nxf;
                T.r = wq.get();
                for (uint32_t k = 0; k < T.nxf; ++k) T.r = xf_ray(S.xforms[T.xfs.get(k)], T.r);
                T.rf = make_rayf(T.r);
                T.a = len2(T.r.d);
                T.inva = 1.0 / T.a;
                break;
            }
            case K_MEDIUM: {
                // volume.rs:37-73.  The medium's hit is independent of the
                // other objects but for the interval's upper end, so it is
                // queued (with the Transforms around it) and tested after the
                // walk against the walk's closest t (media_phase); only a
                // lane whose queue is full tests it here.
                if (T.nmed < RT_MEDIA_CAP) {
                    med.set(T.nmed, make_uint4(idx, T.nxf, T.xfs.a, T.xfs.b));
                    ++T.nmed;
                } else {
                    got = medium_hit<TIER != TIER_FULL_FLAT>(S, idx, r, tmin, T.cl.c, stk, T.sp, rng, t);
                }
                break;
            }
            default: break;
        }
    }
    if (got) {
        T.cl.set(t);
        record(this_ref, t);
    }
    if (after != REF_NONE) T.cur = after;
    return true;
}

// The queued media of a finished walk (FULL tier), each in its own frame,
// against the walk's closest t; the walk's stack is free again.
template <int TIER, class WR>
__device__ __forceinline__ void media_phase(const SceneView& S, const WR& wrr, Trav<TIER>& T, StackFor<TIER>& stk,
                                            const Rng& rng, MedQ med) {
    const auto wq = world_ray(wrr);
    for (uint32_t k = 0; k < T.nmed; ++k) {
        const uint4 e = med.get(k);
        Ray r = wq.get();
        for (uint32_t j = 0; j < e.y; ++j) r = xf_ray(S.xforms[j == 0 ? e.z : e.w], r);
        double t;
        if (medium_hit<TIER != TIER_FULL_FLAT>(S, e.x, r, 1e-8, T.cl.c, stk, 0, rng, t)) {
            T.cl.set(t);
            T.found = true;
            T.hit.t = t;
            T.hit.ref = make_ref(K_MEDIUM, e.x);
            T.hit.nxf = e.y;
            T.hit.xf.a = e.z;
            T.hit.xf.b = e.w;
        }
    }
    T.nmed = 0;
}

// ------------------------------------------------------------------ basic tier: sphere rounds
#ifndef RT_DEFER_THRESH
#define RT_DEFER_THRESH 48  // lanes with a queued sphere that trigger a sphere round
#endif
// ... or 3/4 of the lanes still in the walk, when fewer than 64 are; and any
// one of them when at most RT_DEFER_THIN are: a wave thinned out at the end
// of a launch tests its queued spheres at once instead of walking on with an
// unbounded walk (a ray trapped in a glass sphere queues the sphere it starts
// on at every bounce: its origin is on the surface, so the filter can bound
// nothing).  Measured within noise on the whole frame and on the 1/8 shard:
// the slow last waves of the lane trace were the exit atomics' (the kernel's
// end), not this.
#ifndef RT_DEFER_THIN
#define RT_DEFER_THIN 16
#endif

// ------------------------------------------------------------------ basic tier: 4-wide BVH
// One visit of a DNode4: the sphere children's f32 filter (queued into the
// lane's LDS queue, pq[k * RT_BLOCK_BASIC], when the exact test must run), then the
// four slab tests; the hit boxes are sorted by entry distance, the nearest is
// walked next and the others pushed farthest first.
struct Node4Rows {
    float4 lx, ly, lz, hx, hy, hz, rq;
};
constexpr uint32_t NODE_LDS_CAP = RT_NODE_LDS_BYTES / sizeof(DNode4);
constexpr uint32_t NODE_LDS_CAP_BATCH = RT_NODE_LDS_BATCH_BYTES / sizeof(DNode4);
// The node rows from the block's LDS copy: the launcher gives the basic tier
// only worlds whose whole 4-wide tree fits it (NODE_LDS_CAP nodes: about 900
// spheres; larger sphere worlds run the mesh tier).  A per-wave
// fallback to global reads for larger trees cost 88 B/lane of scratch at the
// 128-VGPR budget.
__device__ __forceinline__ Node4Rows load_node4(const RT_LDS float4* nl, uint32_t idx) {
    const RT_LDS float4* np = nl + idx * 7u;
    return Node4Rows{np[0], np[1], np[2], np[3], np[4], np[5], np[6]};
}
#ifndef RT_SPHERE_RINV
#define RT_SPHERE_RINV 1  // basic / mesh tiers: a static sphere's 1.0 / r from the flatten, not divided per hit
#endif
// visit4 on node rows already loaded; the ref row holds walk words (bword)
template <class Stack>
__device__ __forceinline__ uint32_t visit4_rows(const SceneView& S, const Node4Rows& nr, const RayF& rf, const SphF& sf, float tmin_f,
                                                float& c_f, Stack& stk, uint32_t& sp, RT_LDS uint16_t* pq, uint32_t& pn) {
    const float4 lx = nr.lx, ly = nr.ly, lz = nr.lz, hx = nr.hx, hy = nr.hy, hz = nr.hz, rq = nr.rq;
    const float LX[4] = {lx.x, lx.y, lx.z, lx.w}, LY[4] = {ly.x, ly.y, ly.z, ly.w}, LZ[4] = {lz.x, lz.y, lz.z, lz.w};
    const float HX[4] = {hx.x, hx.y, hx.z, hx.w}, HY[4] = {hy.x, hy.y, hy.z, hy.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
    const uint32_t R[4] = {__float_as_uint(rq.x), __float_as_uint(rq.y), __float_as_uint(rq.z), __float_as_uint(rq.w)};
    constexpr float INF = __builtin_huge_valf();
    float key[4];
    uint32_t ref[4];
    // per slot, the filter / slab only when some lane has a sphere / a box
    // there: the flatten puts a node's spheres in its low slots and its empty
    // slots last (rth::bvh4_convert), and most leaf-level nodes hold 2-3 spheres
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bool sph = (uint16_t)R[i] != 0;
        if (__ballot(sph)) {
            if (sphere_filter(LX[i], LY[i], LZ[i], HX[i], HY[i], sf, c_f, sph)) {
                pq[pn * RT_BLOCK_BASIC] = (uint16_t)(R[i] & 0x7fffu);
                ++pn;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool box = R[i] > 0xffffu;
        key[i] = INF;
        ref[i] = R[i];
        if (__ballot(box)) {
            const float lo[3] = {LX[i], LY[i], LZ[i]}, hi[3] = {HX[i], HY[i], HZ[i]};
            float e;
            const bool h = slab_f(lo, hi, rf, tmin_f, c_f, e) && box;
            key[i] = h ? e : INF;
        }
    }
    // no lane of the wave hit a box child (nodes of spheres only, or every
    // box missed): nothing to sort or push (C2 -0.65 %, A/B at 128 spp, 5
    // reps, RMSE 0; a two-slot network when no lane has a box in slots 0 and
    // 1 was +1.9 %)
    if (!__ballot(fminf(fminf(key[0], key[1]), fminf(key[2], key[3])) < INF)) return 0u;
    auto cs = [&](int a, int b) {  // compare-exchange: key[a] <= key[b] afterwards
        const bool sw = key[b] < key[a];
        const float ka = key[a], kb = key[b];
        const uint32_t ra = ref[a], rb = ref[b];
        key[a] = sw ? kb : ka;
        key[b] = sw ? ka : kb;
        ref[a] = sw ? rb : ra;
        ref[b] = sw ? ra : rb;
    };
    cs(0, 1);
    cs(2, 3);
    cs(0, 2);
    cs(1, 3);
    cs(1, 2);
    if (key[3] < INF) stk.push_w(sp++, ref[3], key[3]);
    if (key[2] < INF) stk.push_w(sp++, ref[2], key[2]);
    if (key[1] < INF) stk.push_w(sp++, ref[1], key[1]);
    return key[0] < INF ? ref[0] : 0u;
}

// One visit of a DNode4 whose children all carry boxes (mesh tier): four slab
// tests, the hit children sorted by entry distance, the nearest walked next
// and the others pushed farthest first -- primitives included, so a triangle
// is tested (planar_t) when the walk reaches it, in distance order.
template <class Stack>
__device__ __forceinline__ uint32_t visit4_core(const float LX[4], const float LY[4], const float LZ[4],
                                                const float HX[4], const float HY[4], const float HZ[4],
                                                const uint32_t R[4], const RayF& rf, float tmin_f, float c_f,
                                                Stack& stk, uint32_t& sp);
template <class Stack>
__device__ __forceinline__ uint32_t visit4_boxes_rows(const float4 lx, const float4 ly, const float4 lz,
                                                      const float4 hx, const float4 hy, const float4 hz,
                                                      const float4 rq, const RayF& rf, float tmin_f, float c_f,
                                                      Stack& stk, uint32_t& sp) {
    const float LX[4] = {lx.x, lx.y, lx.z, lx.w}, LY[4] = {ly.x, ly.y, ly.z, ly.w}, LZ[4] = {lz.x, lz.y, lz.z, lz.w};
    const float HX[4] = {hx.x, hx.y, hx.z, hx.w}, HY[4] = {hy.x, hy.y, hy.z, hy.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
    const uint32_t R[4] = {__float_as_uint(rq.x), __float_as_uint(rq.y), __float_as_uint(rq.z), __float_as_uint(rq.w)};
    return visit4_core(LX, LY, LZ, HX, HY, HZ, R, rf, tmin_f, c_f, stk, sp);
}
template <class Stack>
__device__ __forceinline__ uint32_t visit4_boxes(const SceneView& S, uint32_t idx, const RayF& rf, float tmin_f,
                                                 float c_f, Stack& stk, uint32_t& sp) {
    const RT_GLOBAL float4* np = reinterpret_cast<const RT_GLOBAL float4*>(S.nodes4 + idx);
    return visit4_boxes_rows(np[0], np[1], np[2], np[3], np[4], np[5], np[6], rf, tmin_f, c_f, stk, sp);
}
template <class Stack>
__device__ __forceinline__ uint32_t visit4_core(const float LX[4], const float LY[4], const float LZ[4],
                                                const float HX[4], const float HY[4], const float HZ[4],
                                                const uint32_t R[4], const RayF& rf, float tmin_f, float c_f,
                                                Stack& stk, uint32_t& sp) {
    constexpr float INF = __builtin_huge_valf();
    float key[4];
    uint32_t ref[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float lo[3] = {LX[i], LY[i], LZ[i]}, hi[3] = {HX[i], HY[i], HZ[i]};
        float e;
        const bool h = slab_f(lo, hi, rf, tmin_f, c_f, e) && R[i] != REF_NONE;
        key[i] = h ? e : INF;
        ref[i] = R[i];
    }
    auto cs = [&](int a, int b) {
        const bool sw = key[b] < key[a];
        const float ka = key[a], kb = key[b];
        const uint32_t ra = ref[a], rb = ref[b];
        key[a] = sw ? kb : ka;
        key[b] = sw ? ka : kb;
        ref[a] = sw ? rb : ra;
        ref[b] = sw ? ra : rb;
    };
    cs(0, 1);
    cs(2, 3);
    cs(0, 2);
    cs(1, 3);
    cs(1, 2);
    if (key[3] < INF) stk.push(sp++, ref[3], key[3]);
    if (key[2] < INF) stk.push(sp++, ref[2], key[2]);
    if (key[1] < INF) stk.push(sp++, ref[1], key[1]);
    return key[0] < INF ? ref[0] : REF_NONE;
}

// world.hit for the basic tier over 4-wide nodes, one wave iteration per call:
// a node round (f32 only) for lanes with room in their queue, then a sphere
// round -- each lane with a queued sphere tests one exactly in f64
// (sphere.rs:77-108) -- when 48 lanes have one queued or none can walk on.  A
// lane whose queue is full waits for that before walking on.  Returns false
// when the lane's walk and queue are both done; same closest hit as
// trace_step's walk (A/B renders: RMSE 0).
template <class Stack>
__device__ __forceinline__ bool trace4_step(const SceneView& S, const Ray& r, Trav<TIER_BASIC>& T, Stack& stk,
                                            RT_LDS uint16_t* pq, const RT_LDS float4* nl, Diag& dg) {
    constexpr double tmin = 1e-8;
    const float tmin_f = f32_down(tmin);
    constexpr uint32_t ROOM = RT_PEND_CAP - 4;  // a visit queues at most 4
    RT_DIAG_ONLY(if (__lane_id() == (uint32_t)(__ffsll((long long)__ballot(true)) - 1)) ++dg.wave_trace_iters;)
    uint32_t pn = T.pn;
    // The sphere round is decided on the state before this step's node
    // round and its sphere load issued first, ahead of the node's seven LDS
    // reads; its f64 test comes after the node visit, by when the load has
    // landed.
    const bool can = (T.cur != 0u || T.sp > 0) && pn <= ROOM;
    const unsigned long long mw0 = __ballot(can);
    const unsigned long long mp0 = __ballot(pn > 0);
    const uint32_t in_walk = (uint32_t)__popcll(__ballot(true));
    const uint32_t thresh =
        in_walk <= RT_DEFER_THIN ? 1u : min((uint32_t)RT_DEFER_THRESH, (in_walk * 3u + 3u) / 4u);
    const bool round = (mw0 == 0 || (uint32_t)__popcll(mp0) >= thresh) && pn > 0;
#ifdef RT_DIAG
    if (mw0 == 0 && __lane_id() == (uint32_t)(__ffsll((long long)__ballot(true)) - 1)) {
        ++dg.pure_rounds;
        dg.pure_lanes += (unsigned long long)__popcll(mp0);
    }
    if (mw0 == 0) {  // the most spheres any lane of the wave still has queued
        uint32_t mx = 0;
        for (uint32_t k = 1; k <= RT_PEND_CAP; ++k) mx += __ballot(pn >= k) != 0ull ? 1u : 0u;
        if (__lane_id() == (uint32_t)(__ffsll((long long)__ballot(true)) - 1)) dg.pure_max_pn += mx;
    }
#endif
    // the loads are unconditional (a lane without a round / a node reads
    // entry 0, cache-hot) so that no branch stands between them and their
    // waits: the sphere test then waits for its own load only
    const uint32_t top = pn > 0 ? pn - 1 : 0;
    const uint32_t sidx = pq[top * RT_BLOCK_BASIC];
    pn -= round ? 1u : 0u;
    const double4 s4 = S.spheres[round ? sidx : 0u];
    uint32_t cur = REF_NONE;
    if (can) {
        RT_DIAG_ONLY(++dg.lane_trace_iters;)
#ifdef RT_DIAG
        if (T.cur == 0u) {
            const uint32_t sp_before = T.sp;
            T.cur = pop_w(stk, T.sp, T.cl.c_f);
            ++dg.pops;
            dg.pop_reads += sp_before - T.sp;
        }
#else
        if (T.cur == 0u) T.cur = pop_w(stk, T.sp, T.cl.c_f);
#endif
        cur = T.cur;
        T.cur = 0u;
    }
    // cur is a walk word (bword): a node, a list position or a sphere
    const uint32_t r16 = cur >> 16;
    const bool node = r16 - 1u < 0x7fffu;  // 1 ..= 0x7fff
    const Node4Rows rows = load_node4(nl - 7, node ? r16 : 1u);

    if (__ballot(!node && cur != 0u)) {  // lists, standalone spheres (none in C2)
        if (r16 >= 0x8000u) {  // a list position
            const uint32_t li = r16 & 0x7fffu;
            const uint32_t child = S.list_children[li];
            if (child != REF_NONE) {
                if (S.list_children[li + 1] != REF_NONE) stk.push_w(T.sp++, (0x8000u | (li + 1)) << 16, NO_CULL);
                T.cur = bword(S, child);
            }
        } else {  // a sphere element of a list: queued for its exact test
            pq[pn * RT_BLOCK_BASIC] = (uint16_t)(cur & 0x7fffu);
            ++pn;
        }
    }
    if (node) {
        RT_ISA_MARK("walk_visit");
        RT_DIAG_ONLY(++dg.node_visits;)
        T.cur = visit4_rows(S, rows, T.rf, T.sf, tmin_f, T.cl.c_f, stk, T.sp, pq, pn);
    }
    // the sphere round's f64 test after the node visit: the visit's LDS rows
    // arrive before the sphere's global load, and the test then finds it
    // there (C2 -0.2 %, profiles/r05/ab_round_late_c2_128spp.json; the
    // visit culls against the closest t before this test, which only makes
    // it cull less, never wrongly)
    if (round) {  // sphere round (sphere.rs:77-108)
        RT_ISA_MARK("walk_sphere");
        RT_DIAG_ONLY(++dg.sphere_tests;)
        double t;
        RT_DIAG_ONLY(if (s4.w > 100.0) ++dg.big_tests;)
        if (sphere_t_inv(d3(s4.x, s4.y, s4.z), s4.w, r, T.a, T.inva, tmin, T.cl.c, t)) {
            RT_DIAG_ONLY(if (s4.w > 100.0) ++dg.big_hits;)
            T.cl.lower(t);
            T.found = true;
            T.hit.t = t;
            T.hit.ref = make_ref(K_SPHERE, sidx);
        }
    }
    RT_ISA_MARK("walk_tail");
    T.pn = pn;
    return T.cur != 0u || T.sp > 0 || pn > 0;
}

// ------------------------------------------------------------------ hit record
struct Rec {
    D3 p, n;
    double u, v;
    int mat;
    bool front;
};

// HitRecord::new (hit.rs:24-43) of the recorded closest hit, in the frame of
// its innermost Transform, then carried out through the chain (shapes.rs:104-108).
template <int TIER>
__device__ Rec make_record(const SceneView& S, const Ray& wr, const HitInfo& h, bool& panic) {
    constexpr bool FULL = tier_full(TIER), PLANAR = TIER >= TIER_MESH;
    Ray r = wr;
    if constexpr (FULL)
        for (uint32_t k = 0; k < h.nxf; ++k) r = xf_ray(S.xforms[h.xf.get(k)], r);
    const uint32_t kind = ref_kind(h.ref), idx = ref_idx(S, h.ref);
    Rec rec;
    rec.u = 0.0;
    rec.v = 0.0;
    const D3 p = r.o + h.t * r.d;
    D3 outward;
    if (!PLANAR || kind == K_SPHERE || kind == K_MSPHERE) {
        D3 c;
        double rinv;  // sphere.rs:99: (p - c) / radius = (1.0 / radius) * (p - c) (vec3.rs:225-227)
        if (!FULL || kind == K_SPHERE) {
            const double4 s = S.spheres[idx];
            c = d3(s.x, s.y, s.z);
            // basic / mesh tiers: the host's 1.0 / r, the same double (C2 -0.5 %);
            // the full tiers divide (C5 +1.0 % with the load: A/B, RMSE 0)
            rinv = (RT_SPHERE_RINV && !FULL) ? S.sphere_rinv[idx] : 1.0 / s.w;
            rec.mat = S.sphere_mat[idx];
        } else {
            const double4 s = S.msph_center[idx], m = S.msph_dir[idx];
            c = d3(s.x, s.y, s.z) + r.time * d3(m.x, m.y, m.z);
            rinv = 1.0 / s.w;
            rec.mat = S.msph_mat[idx];
        }
        outward = rinv * (p - c);
        if (S.materials[rec.mat].flags & MF_NEEDS_UV) {
            // sphere.rs:53-61
            const double theta = k_acos(-outward.y);
            const double phi = k_atan2(-outward.z, outward.x) + PI;
            rec.u = phi / (2.0 * PI);
            rec.v = theta / PI;
        }
    } else if (kind == K_QUAD || kind == K_TRI) {
        const DPlanar& P = S.planars[idx];
        outward = d3(P.f[0], P.f[1], P.f[2]);
        rec.mat = S.planar_mat[idx];
        // (u, v) = (alpha, beta) of quad.rs:93-99, for a texture that reads
        // them or an OBJ triangle's RemappedMaterial (obj.rs:32-62); nothing
        // else looks at them (full tiers: C3 -1.3 %, C5 -2 %; the mesh tier's
        // OBJ triangles always need them)
        if (!FULL || (S.materials[rec.mat].flags & MF_NEEDS_UV) ||
            (PLANAR && kind == K_TRI && S.planar_remap[idx] >= 0)) {
            const D3 hv = p - d3(P.f[4], P.f[5], P.f[6]);
            const D3 u = d3(P.f[7], P.f[8], P.f[9]), v = d3(P.f[10], P.f[11], P.f[12]), w = d3(P.f[13], P.f[14], P.f[15]);
            rec.u = dot(w, cross(hv, v));
            rec.v = dot(w, cross(u, hv));
        }
    } else {  // K_MEDIUM (volume.rs:67-72)
        outward = d3(1.0, 0.0, 0.0);
        rec.mat = S.media[idx].phase_mat;
    }
    rec.front = dot(r.d, outward) < 0.0;
    rec.n = rec.front ? outward : -outward;
    rec.p = p;
    if constexpr (FULL) {
        for (int k = (int)h.nxf - 1; k >= 0; --k) {
            const DXform& X = S.xforms[h.xf.get(k)];
            rec.p = xf_out(X, rec.p);
            bool ok;
            rec.n = unit(quat_rotate(X.q[0], X.q[1], X.q[2], X.q[3], rec.n / d3(X.scale[0], X.scale[1], X.scale[2])), ok);
        }
    }
    if constexpr (PLANAR) {
        // RemappedMaterial::remap_record (obj.rs:32-62), no normal map: applied to
        // the record every material of an OBJ triangle sees (scatter and emitted)
        if (kind == K_TRI) {
            const int32_t ri = S.planar_remap[idx];
            if (ri >= 0) {
                const DRemap& R = S.remaps[ri];
                const double u = rec.u, v = rec.v;
                const double tu = (R.tex_ori[0] + u * R.tex_u[0]) + v * R.tex_v[0];
                const double tv = (R.tex_ori[1] + u * R.tex_u[1]) + v * R.tex_v[1];
                const double w0 = (1.0 - u) - v;
                const D3 nm = ((w0 * d3(R.n[0], R.n[1], R.n[2])) + (u * d3(R.n[3], R.n[4], R.n[5]))) +
                              (v * d3(R.n[6], R.n[7], R.n[8]));
                bool ok;
                rec.n = unit(nm, ok);
                if (!ok) panic = true;  // .unwrap() (obj.rs:40)
                if constexpr (FULL) {
                    if (R.normal_tex >= 0) {  // obj.rs:42-51
                        if (!R.uv_ok) panic = true;  // u_vec.unwrap()
                        const DRemapNM& F = S.remap_nm[ri];
                        const D3 c = tex_value<FULL>(S, R.normal_tex, tu, tv, rec.p);
                        const D3 nc = 2.0 * c - d3(1.0, 1.0, 1.0);
                        const D3 raw = ((nc.x * d3(F.u_vec[0], F.u_vec[1], F.u_vec[2])) +
                                        (nc.y * d3(F.v_vec[0], F.v_vec[1], F.v_vec[2]))) + (nc.z * rec.n);
                        bool ok2;
                        rec.n = unit(raw, ok2);
                        if (!ok2) panic = true;  // "The mapped normal can't normalized!"
                    }
                }
                rec.u = tu;
                rec.v = tv;
            }
        }
    }
    return rec;
}

// ------------------------------------------------------------------ lights (pdf.rs:66-88)
__device__ double light_pdf_one(const SceneView& S, uint32_t ref, D3 o, D3 d) {
    const uint32_t kind = ref_kind(ref), idx = ref_idx(S, ref);
    const Ray r{o, d, 0.0};
    double t;
    if (kind == K_QUAD || kind == K_TRI) {  // quad.rs:108-120
        const DPlanar& P = S.planars[idx];
        if (!planar_t(P, kind == K_TRI, r, 1e-8, __builtin_huge_val(), t)) return 0.0;
        const D3 n = d3(P.f[0], P.f[1], P.f[2]);
        const D3 rn = dot(d, n) < 0.0 ? n : -n;
        const double distance_squared = t * t * len2(d);
        const double cosine = fabs(dot(d, rn) / len(d));
        return distance_squared / (cosine * S.planar_area[idx]);
    }
    if (kind == K_SPHERE) {  // sphere.rs:114-132
        const double4 s = S.spheres[idx];
        if (!sphere_t(d3(s.x, s.y, s.z), s.w, r, len2(d), 1e-8, __builtin_huge_val(), t)) return 0.0;
        const double dist_squared = len2(d3(s.x, s.y, s.z) - o);
        const double ctm = k_sqrt(1.0 - s.w * s.w / dist_squared);
        if (isnan(ctm)) return 1.0 / (4.0 * PI);
        return 1.0 / (2.0 * PI * (1.0 - ctm));
    }
    return 0.0;
}
__device__ double light_pdf(const SceneView& S, D3 o, D3 d) {
    const uint32_t root = S.lights_root;
    if (ref_kind(root) != K_LIST) return light_pdf_one(S, root, o, d);
    double sum = 0.0;  // hits.rs:52-67
    uint32_t n = 0;
    for (uint32_t i = ref_idx(S, root); S.list_children[i] != REF_NONE; ++i, ++n) sum += light_pdf_one(S, S.list_children[i], o, d);
    return sum / (double)n;
}
__device__ __forceinline__ D3 onb_world(D3 n, D3 v, bool& ok) {  // onb.rs:8-21, 34-38
    const D3 a = fabs(n.x) > 0.9 ? d3(0.0, 1.0, 0.0) : d3(1.0, 0.0, 0.0);
    const D3 u = unit(cross(n, a), ok);
    const D3 w = cross(u, n);
    return v.x * u + v.y * n + v.z * w;
}
// Quad / Triangle / Sphere::random (quad.rs:122-125, triangle.rs:117-128, sphere.rs:134-144)
__device__ __forceinline__ D3 light_random_one(const SceneView& S, uint32_t ref, D3 o, Rng& rng, uint32_t& ovf,
                                               bool& ok) {
    const uint32_t kind = ref_kind(ref), idx = ref_idx(S, ref);
    if (kind == K_QUAD || kind == K_TRI) {  // quad.rs:122-125, triangle.rs:117-128
        const DPlanar& P = S.planars[idx];
        double a = rng.next(ovf);
        double b = rng.next(ovf);
        if (kind == K_TRI && a + b > 1.0) {
            const double na = 1.0 - b, nb = 1.0 - a;
            a = na;
            b = nb;
        }
        const D3 p = d3(P.f[4], P.f[5], P.f[6]) + (a * d3(P.f[7], P.f[8], P.f[9])) + (b * d3(P.f[10], P.f[11], P.f[12]));
        return unit(p - o, ok);
    }
    // sphere.rs:134-144
    const double4 s = S.spheres[idx];
    const D3 direction = d3(s.x, s.y, s.z) - o;
    const double distance_squared = len2(direction);
    bool ok1, ok2;
    const D3 nd = unit(direction, ok1);
    const double r1 = rng.next(ovf), r2 = rng.next(ovf);
    const double y = 1.0 + r2 * (k_sqrt(1.0 - s.w * s.w / distance_squared) - 1.0);
    double sphi, cphi;
    k_sincos_2pi(r1, &sphi, &cphi);  // phi = 2.0 * PI * r1
    const double x = cphi * k_sqrt(1.0 - y * y), z = sphi * k_sqrt(1.0 - y * y);
    const D3 wv = onb_world(nd, d3(x, y, z), ok2);
    bool ok3;
    const D3 res = unit(wv, ok3);
    ok = ok1 && ok2 && ok3;
    return res;
}
__device__ D3 light_random(const SceneView& S, D3 o, Rng& rng, uint32_t& ovf, bool& ok) {
    uint32_t ref = S.lights_root;
    if (ref_kind(ref) == K_LIST) {  // hits.rs:69-75 choose
        uint32_t n = 0;
        for (uint32_t i = ref_idx(S, ref); S.list_children[i] != REF_NONE; ++i) ++n;
        uint32_t k = (uint32_t)(rng.next(ovf) * (double)n);
        if (k >= n) k = n - 1;
        ref = S.list_children[ref_index(ref) + k];
    }
    return light_random_one(S, ref, o, rng, ovf, ok);
}

// ---- general lights (tier FULL_GL): any tree of Hittables lists and
// Transforms over spheres (static or moving: pdf_value / random use the
// center at time 0, sphere.rs:114-144), quads and triangles.
// Hittables::pdf_value averages its children's values in order
// (hits.rs:52-67); Hittables::random draws one child (hits.rs:69-75);
// Transform maps the origin and direction into its frame and the sampled
// point back out (shapes.rs:117-132).  The tree is walked by compile-time
// recursion over its depth (the flattener rejects deeper trees), as a
// reference call chain would.
constexpr int RT_LIGHT_DEPTH = 4;  // list / Transform levels of a lights tree (rt_scene.cpp light_tree_ok)

__device__ double light_pdf_leaf(const SceneView& S, uint32_t ref, D3 o, D3 d) {
    if (ref_kind(ref) != K_MSPHERE) return light_pdf_one(S, ref, o, d);
    const double4 s = S.msph_center[ref_idx(S, ref)];  // Ray::new: time 0 (ray.rs:11-17) -> center.at(0)
    const Ray r{o, d, 0.0};
    double t;
    if (!sphere_t(d3(s.x, s.y, s.z), s.w, r, len2(d), 1e-8, __builtin_huge_val(), t)) return 0.0;
    const double dist_squared = len2(d3(s.x, s.y, s.z) - o);
    const double ctm = k_sqrt(1.0 - s.w * s.w / dist_squared);
    if (isnan(ctm)) return 1.0 / (4.0 * PI);
    return 1.0 / (2.0 * PI * (1.0 - ctm));
}

template <int D>
__device__ double light_pdf_tree(const SceneView& S, uint32_t ref, D3 o, D3 d, bool& panic) {
    const uint32_t kind = ref_kind(ref), idx = ref_idx(S, ref);
    if constexpr (D > 0) {
        if (kind == K_LIST) {  // hits.rs:52-67
            double sum = 0.0;
            uint32_t n = 0;
            for (uint32_t i = idx; S.list_children[i] != REF_NONE; ++i, ++n)
                sum += light_pdf_tree<D - 1>(S, S.list_children[i], o, d, panic);
            const double ret = sum / (double)n;
            if (isnan(ret)) panic = true;  // "The sum of pdf is NaN!"
            return ret;
        }
        if (kind == K_XFORM) {  // shapes.rs:117-123
            const DXform& X = S.xforms[idx];
            const D3 lo = xf_in(X, o);
            const D3 lt = xf_in(X, o + d);
            return light_pdf_tree<D - 1>(S, X.child, lo, lt - lo, panic);
        }
    }
    return light_pdf_leaf(S, ref, o, d);
}

template <int D>
__device__ D3 light_random_tree(const SceneView& S, uint32_t ref, D3 o, Rng& rng, uint32_t& ovf, bool& ok) {
    const uint32_t kind = ref_kind(ref), idx = ref_idx(S, ref);
    if constexpr (D > 0) {
        if (kind == K_LIST) {  // hits.rs:69-75 choose
            uint32_t n = 0;
            for (uint32_t i = idx; S.list_children[i] != REF_NONE; ++i) ++n;
            uint32_t k = (uint32_t)(rng.next(ovf) * (double)n);
            if (k >= n) k = n - 1;
            return light_random_tree<D - 1>(S, S.list_children[idx + k], o, rng, ovf, ok);
        }
        if (kind == K_XFORM) {  // shapes.rs:125-132
            const DXform& X = S.xforms[idx];
            const D3 lo = xf_in(X, o);
            const D3 ld = light_random_tree<D - 1>(S, X.child, lo, rng, ovf, ok);
            const D3 world_to = xf_out(X, lo + ld);
            bool ok2;
            const D3 res = unit(world_to - o, ok2);  // "Random direction can't be normalized!"
            ok = ok && ok2;
            return res;
        }
    }
    if (kind == K_MSPHERE) {  // sphere.rs:134-144 with center.at(0)
        const double4 s = S.msph_center[idx];
        const D3 direction = d3(s.x, s.y, s.z) - o;
        const double distance_squared = len2(direction);
        bool ok1, ok2, ok3;
        const D3 nd = unit(direction, ok1);
        const double r1 = rng.next(ovf), r2 = rng.next(ovf);
        const double y = 1.0 + r2 * (k_sqrt(1.0 - s.w * s.w / distance_squared) - 1.0);
        double sphi, cphi;
        k_sincos_2pi(r1, &sphi, &cphi);  // phi = 2.0 * PI * r1
        const double x = cphi * k_sqrt(1.0 - y * y), z = sphi * k_sqrt(1.0 - y * y);
        const D3 res = unit(onb_world(nd, d3(x, y, z), ok2), ok3);
        ok = ok1 && ok2 && ok3;
        return res;
    }
    return light_random_one(S, ref, o, rng, ovf, ok);
}

// A material's texture value; a SolidColor's colour comes with the material
// record (MF_SOLID, set by the flatten), one dependent load fewer.
template <bool FULL, bool PL = false>
__device__ __forceinline__ D3 mat_tex(const SceneView& S, const DMaterial& M, double u, double v, D3 p) {
    if (M.flags & MF_SOLID) return d3(M.albedo[0], M.albedo[1], M.albedo[2]);
    return tex_value<FULL, PL>(S, M.tex, u, v, p);
}

// vec3.rs:313-322
__device__ __forceinline__ D3 random_unit_vector(Rng& rng, uint32_t& ovf) {
    const double r1 = rng.next(ovf), r2 = rng.next(ovf);
    double sn, cs;
    k_sincos_2pi(r1, &sn, &cs);
    const double s = k_sqrt(r2 * (1.0 - r2));
    return d3(cs * 2.0 * s, sn * 2.0 * s, 1.0 - 2.0 * r2);
}

// Basic / mesh tiers: the draws of one path vertex that every scattering
// material there takes -- slots 0 and 1 of the vertex (one Philox block) and
// cos / sin(2 pi xi0) (Lambertian's cosine direction and Metal's
// random_unit_vector, vec3.rs:313-343; Dielectric's Schlick draw is xi0) --
// made once per wave iteration by the main loop, shared with the camera rays
// of the lanes that start a sample there (random_in_unit_disk's theta is
// 2 pi xi too, vec3.rs:63-69): one Philox block and one sincos per lane and
// iteration instead of a shading set and a camera set.
struct Draws {
    double xi0, xi1, sn, cs;
};
// The basic tier's main loop shares the draws.  A/B (RMSE 0): C2 -1.3 % (64
// spp) / -1.8 % (128 spp) kernel time; the mesh tier +3.3 % on C4 (64 spp,
// round 4: the loop's extra live state spills 44 B/lane) and +1.0 % in round
// 5 (28 B/lane), so it keeps the loop of the full tiers.

// ---- general materials (tier FULL_GL): DiffuseLight / Mix wrappers nested
// up to RT_MAT_DEPTH levels (rt_scene.cpp checks), Mix::from_image ratios.
constexpr int RT_MAT_DEPTH = 4;
// Mix::get_ratio (material.rs:249-251): the constant, or the image's alpha
__device__ __forceinline__ double mix_ratio(const SceneView& S, const DMaterial& M, double u, double v) {
    return M.tex >= 0 ? tex_alpha(S, M.tex, u, v) : M.fuzz;
}
// Material::emitted of a wrapper tree: DiffuseLight = its texture + the
// wrapped material's emission (material.rs:171-178), Mix = mat1 * (1 - r) +
// mat2 * r (material.rs:262-266), anything else BLACK
template <int D>
__device__ D3 emitted_tree(const SceneView& S, int mid, double u, double v, D3 p) {
    const DMaterial& M = S.materials[mid];
    if (M.type == M_DIFFUSE_LIGHT) {
        const D3 self = mat_tex<true, RT_PERLIN_LDS>(S, M, u, v, p);
        D3 inner = d3(0.0, 0.0, 0.0);
        if constexpr (D > 0)
            if (M.inner >= 0) inner = emitted_tree<D - 1>(S, M.inner, u, v, p);
        return self + inner;
    }
    if constexpr (D > 0) {
        if (M.type == M_MIX) {
            const double r = mix_ratio(S, M, u, v);
            return ((1.0 - r) * emitted_tree<D - 1>(S, M.inner, u, v, p)) + (r * emitted_tree<D - 1>(S, M.inner2, u, v, p));
        }
    }
    return d3(0.0, 0.0, 0.0);
}

// ------------------------------------------------------------------ one ray_color level
// camera.rs:275-325 at path vertex `vertex`; updates (ray, beta, L).  Returns
// true when the path ends here (miss, no scatter, panic).
// Deferred shading classes (full BVH tier, A/B lever): a lane whose hit is
// a plain Lambertian with a texture kind in RT_SHADE_DEFER_TEX_MASK (a bit per
// T_*) skips a shading round while fewer than RT_SHADE_DEFER_K such lanes are
// ready, other lanes still walk, and the wave has deferred fewer than
// RT_SHADE_DEFER_WAIT rounds in a row.  It keeps its hit, its RNG state and its
// path and is shaded in a later round, with the same doubles (nothing it
// computes depends on when).  0: off -- measured on C5 (64 spp, 4 reps, the
// tier's product flags, RMSE 0): +0.5 % to +1.6 % kernel time, the noise
// class's share of rounds 38 % -> 22 % but VALU exec density unchanged
// (0.3383) and walk lane efficiency 0.628 -> 0.611
// (profiles/r06/ab_shade_defer_t2flags_c5_64spp.json, density_c5_t2*.json).
#ifndef RT_SHADE_DEFER
#define RT_SHADE_DEFER 0
#endif
#ifndef RT_SHADE_DEFER_TEX_MASK
#define RT_SHADE_DEFER_TEX_MASK (1u << T_NOISE)
#endif
#ifndef RT_SHADE_DEFER_K
#define RT_SHADE_DEFER_K 12
#endif
#ifndef RT_SHADE_DEFER_WAIT
#define RT_SHADE_DEFER_WAIT 3
#endif
// RT_SHADE_DEFER: the hit's material is a plain (non-emissive) Lambertian whose
// texture kind is in RT_SHADE_DEFER_TEX_MASK
__device__ __forceinline__ bool shade_deferrable(const SceneView& S, uint32_t ref) {
    const uint32_t k = ref_kind(ref), i = ref_index(ref);
    const int32_t m = k == K_SPHERE ? S.sphere_mat[i] : k == K_MSPHERE ? S.msph_mat[i]
                    : (k == K_QUAD || k == K_TRI) ? S.planar_mat[i] : -1;
    if (m < 0) return false;
    const DMaterial& M = S.materials[m];
    if (M.type != M_LAMBERTIAN || (M.flags & (MF_SOLID | MF_EMISSIVE))) return false;
    return ((RT_SHADE_DEFER_TEX_MASK >> S.textures[M.tex].type) & 1u) != 0u;
}

template <int TIER>
__device__ __forceinline__ bool shade(const SceneView& S, Ray& ray, D3& beta, D3& L, Rng& rng, bool hit_any,
                                      const HitInfo& h, bool& panic, const Draws& Dr = Draws{}) {
    constexpr bool FULL = tier_full(TIER);
    constexpr bool PL = tier_full_bvh(TIER) && RT_PERLIN_LDS;  // the block holds the LDS copy of the first Perlin table (the flat tier's LDS is full)
    uint32_t ovf = 0;
    if (!hit_any) {
        // miss: Environment::value (environment.rs:14-24)
        if constexpr (TIER == TIER_BASIC) {
            // (C2 -1.4 %, profiles/r05/ab_sky_y_c2_128spp.json; the mesh tier
            // measured +0.4 % on C4 with it and keeps unit())
            // Basic tier under a sky gradient (the world's background
            // is wave-uniform: a scalar branch): the gradient reads the unit
            // direction's y only, so only that component is made, as unit()
            // makes it: (1 / l) * d.y (vec3.rs:225-232, rt_math.h divs).
            // `ok` is the same as unit()'s finite3 of the three products:
            // with l = |d| not NaN and not 0 and every component finite,
            // 1 / l is finite (a nonzero l is >= sqrt(5e-324) ~ 2e-162) and
            // each (1 / l) * d_i is finite (|d_i| <= l, or l = inf over
            // finite components: 0); l = 0 or NaN, or an infinite component
            // (0 * inf), gives a NaN (tests/test_miss_unit_cpu.py)
            // The gradient's colours come with the launch parameters
            // (SceneView::bg_c0 / bg_c1), not from the texture table.
            if (RT_BG_PARAMS ? S.bg_kind == BG_SKY
                             : (S.background_tex >= 0 && S.textures[S.background_tex].type == T_SKY)) {
                const double l = len(ray.d);
                if (isnan(l) || l == 0.0 || !finite3(ray.d)) panic = true;
                L = L + beta * (RT_BG_PARAMS ? sky_value(S.bg_c0, S.bg_c1, (1.0 / l) * ray.d.y)
                                             : sky_value(S.textures[S.background_tex], (1.0 / l) * ray.d.y));
                return true;
            }
        }
        if (RT_BG_PARAMS && !FULL && S.bg_kind == BG_SKY) {  // the mesh tier: unit(), the gradient from the launch parameters
            bool ok;
            const D3 p = unit(ray.d, ok);
            if (!ok) panic = true;
            L = L + beta * sky_value(S.bg_c0, S.bg_c1, p.y);
            return true;
        }
        if (S.background_tex >= 0) {
            bool ok;
            const D3 p = unit(ray.d, ok);
            if (!ok) panic = true;
            double u = 0.0, v = 0.0;
            if (FULL && S.textures[S.background_tex].needs_uv) {
                const double theta = k_acos(-p.y);
                const double phi = PI - k_atan2(-p.z, p.x);
                u = phi / (2.0 * PI);
                v = theta / PI;
            }
            L = L + beta * tex_value<FULL, PL>(S, S.background_tex, u, v, p);
        }
        return true;
    }
    const Rec rec = make_record<TIER>(S, ray, h, panic);
    if (panic) return true;
    DMaterial M = S.materials[rec.mat];
    // Basic / mesh tiers: every scattering material draws slot 0 (and 1) of
    // this vertex first, and Lambertian and Metal both turn the first draw
    // into cos/sin(2 pi r1) (vec3.rs:313-322, 333-343): the main loop's Draws.
    constexpr bool HOIST = !FULL;
    const double xi0 = Dr.xi0, xi1 = Dr.xi1, sn0 = Dr.sn, cs0 = Dr.cs;
    if constexpr (TIER == TIER_FULL_GL) {
        if (M.flags & MF_EMISSIVE) L = L + beta * emitted_tree<RT_MAT_DEPTH>(S, rec.mat, rec.u, rec.v, rec.p);
        // the wrappers' scatter: DiffuseLight -> its material or None, Mix -> one draw (material.rs:180-185, 254-260)
        for (int k = 0; k < RT_MAT_DEPTH && (M.type == M_DIFFUSE_LIGHT || M.type == M_MIX); ++k) {
            if (M.type == M_DIFFUSE_LIGHT) {
                if (M.inner < 0) return true;
                M = S.materials[M.inner];
            } else {
                M = S.materials[rng.next(ovf) > mix_ratio(S, M, rec.u, rec.v) ? M.inner : M.inner2];
            }
        }
        if (M.type == M_DIFFUSE_LIGHT) return true;  // a plain light at the last level
    } else if constexpr (FULL) {
        // emitted (material.rs:30-33, 171-178, 262-266)
        if (M.flags & MF_EMISSIVE) {
            D3 em;
            if (M.type == M_DIFFUSE_LIGHT) {
                em = mat_tex<FULL, PL>(S, M, rec.u, rec.v, rec.p);
            } else {  // Mix of non-wrapping materials (flatten checks)
                const DMaterial& A = S.materials[M.inner];
                const DMaterial& B = S.materials[M.inner2];
                const D3 ea = A.type == M_DIFFUSE_LIGHT ? mat_tex<FULL, PL>(S, A, rec.u, rec.v, rec.p) : d3(0, 0, 0);
                const D3 eb = B.type == M_DIFFUSE_LIGHT ? mat_tex<FULL, PL>(S, B, rec.u, rec.v, rec.p) : d3(0, 0, 0);
                em = ((1.0 - M.fuzz) * ea) + (M.fuzz * eb);
            }
            L = L + beta * em;
        }
        // wrappers: DiffuseLight(inner) scatters as inner (material.rs:180-185); Mix draws (254-260)
        if (M.type == M_DIFFUSE_LIGHT) {
            if (M.inner < 0) return true;
            M = S.materials[M.inner];
        }
        if (M.type == M_MIX) {
            M = S.materials[rng.next(ovf) > M.fuzz ? M.inner : M.inner2];
            if (M.type == M_DIFFUSE_LIGHT) return true;
        }
    }
    const D3 n = rec.n;
    int pdf_kind = -1;  // 0 cosine, 1 sphere
    D3 albedo = d3(0, 0, 0);
    switch (M.type) {
        case M_LAMBERTIAN:  // material.rs:60-65
            albedo = mat_tex<FULL, PL>(S, M, rec.u, rec.v, rec.p);
            pdf_kind = 0;
            break;
        case M_EMPTY:  // material.rs:41-46
            albedo = d3(0.75, 0.75, 0.75);
            pdf_kind = 0;
            break;
        case M_METAL: {  // material.rs:82-95
            bool ok1, ok2;
            const D3 ud = unit(ray.d, ok1);
            if (!ok1) return true;
            const D3 rr = unit(reflect(ud, n), ok2);
            if (!ok2) return true;
            D3 ruv;
            if constexpr (!HOIST) {
                ruv = random_unit_vector(rng, ovf);
            } else {
                const double s = k_sqrt(xi1 * (1.0 - xi1));
                ruv = d3(cs0 * 2.0 * s, sn0 * 2.0 * s, 1.0 - 2.0 * xi1);
            }
            beta = beta * d3(M.albedo[0], M.albedo[1], M.albedo[2]);
            ray = Ray{rec.p, rr + (M.fuzz * ruv), ray.time};
            break;
        }
        case M_DIELECTRIC: {  // material.rs:117-143
            const double ri = rec.front ? 1.0 / M.fuzz : M.fuzz;
            bool ok;
            const D3 ud = unit(ray.d, ok);
            if (!ok) panic = true;
            const double cos_theta = fmin(dot(-ud, n), 1.0);
            const double sin_theta = k_sqrt(1.0 - cos_theta * cos_theta);
            bool do_reflect = ri * sin_theta > 1.0;
            if (!do_reflect) {  // Schlick (material.rs:110-114); the draw only when refraction is possible
                const double r0 = (1.0 - ri) / (1.0 + ri);
                const double r0sq = r0 * r0;
                const double x = 1.0 - cos_theta;
                const double x2 = x * x;
                do_reflect = r0sq + (1.0 - r0sq) * (x * (x2 * x2)) > (HOIST ? xi0 : rng.next(ovf));
            }
            D3 dir;
            if (do_reflect) {
                dir = reflect(ud, n);
            } else {  // vec3.rs:345-354
                const D3 perp = ri * (ud + cos_theta * n);
                const double pl = k_sqrt(1.0 - len2(perp));
                if (isnan(pl)) panic = true;
                dir = perp + (-pl * n);
            }
            beta = beta * mat_tex<FULL, PL>(S, M, rec.u, rec.v, rec.p);
            ray = Ray{rec.p, dir, ray.time};
            break;
        }
        default:
            if constexpr (FULL) {
                if (M.type == M_ISOTROPIC) {  // material.rs:199-206
                    albedo = mat_tex<FULL, PL>(S, M, rec.u, rec.v, rec.p);
                    pdf_kind = 1;
                    break;
                }
                if (M.type == M_TRANSPARENT) {  // material.rs:211-217
                    ray = Ray{rec.p, ray.d, ray.time};
                    break;
                }
            }
            return true;
    }
    if (pdf_kind >= 0) {
        // PDF branch (camera.rs:297-316)
        const bool use_lights = FULL && S.lights_root != REF_NONE;
        bool from_material = true;
        if (use_lights) from_material = rng.next(ovf) < 0.5;  // MixturePDF::generate (pdf.rs:113-119)
        D3 dir;
        bool ok = true;
        if (from_material) {
            if (!FULL || pdf_kind == 0) {  // CosinePDF::generate (pdf.rs:59-63), vec3.rs:333-343
                double r2 = xi1, sn = sn0, cs = cs0;
                if constexpr (!HOIST) {
                    const double r1 = rng.next(ovf);
                    r2 = rng.next(ovf);
                    k_sincos_2pi(r1, &sn, &cs);
                }
                const double sr2 = k_sqrt(r2);
                dir = onb_world(n, d3(sn * sr2, k_sqrt(1.0 - r2), cs * sr2), ok);
            } else {
                dir = random_unit_vector(rng, ovf);
            }
        } else {
            if constexpr (TIER == TIER_FULL_GL)
                dir = light_random_tree<RT_LIGHT_DEPTH>(S, S.lights_root, rec.p, rng, ovf, ok);
            else
                dir = light_random(S, rec.p, rng, ovf, ok);
        }
        if (!ok) panic = true;
        // value (pdf.rs:22-28, 50-57, 101-111)
        D3 f;
        double pdf;
        if (!FULL || pdf_kind == 0) {
            bool okd;
            const D3 ud = unit(dir, okd);
            if (!okd) panic = true;
            const double ct = dot(ud, n);
            pdf = fmax(0.0, ct / PI);
            const double cp = fmax(ct, 0.0);
            f = divs(albedo * d3(cp, cp, cp), PI);
        } else {
            pdf = 1.0 / (4.0 * PI);
            f = divs(albedo, 4.0 * PI);
        }
        if (use_lights) {
            double pdf1;
            if constexpr (TIER == TIER_FULL_GL)
                pdf1 = light_pdf_tree<RT_LIGHT_DEPTH>(S, S.lights_root, rec.p, dir, panic);
            else
                pdf1 = light_pdf(S, rec.p, dir);
            if (isnan(pdf1)) panic = true;
            if (pdf == 0.0 && pdf1 == 0.0) panic = true;
            pdf = pdf * 0.5 + pdf1 * 0.5;
        }
        if (pdf == 0.0) panic = true;  // camera.rs:309
        beta = beta * divs(f, pdf);
        ray = Ray{rec.p, dir, ray.time};
    }
    if (ovf) panic = true;
    return panic;
}

// ------------------------------------------------------------------ basic tier: one hit, merged
#ifndef RT_SHADE_MERGED
// 1: the basic tier shades a hit with shade_hit_basic (below), 0: with shade
// (A/B only)
#define RT_SHADE_MERGED 1
#endif
// shade() for a hit in the basic tier (camera.rs:286-316; Lambertian /
// EmptyMaterial, Metal, Dielectric: material.rs:41-143, onb.rs:8-38,
// pdf.rs:50-63), with the three scatter codes' square roots and divisions
// merged.  As one switch, a wave whose shading batch holds all three
// classes ran every class's unit vectors, square roots and divisions one
// after the other (10 square roots and 9 divisions); here each stage is one
// square root or division that every lane runs on its own class's operand:
//   A  unit(cross(n, a)) (Lambertian's ONB)  |  unit(r_in.direction) (Metal, Dielectric)
//   B1 sqrt(r2)  |  sqrt(r2 (1 - r2)) (random_unit_vector)  |  sin_theta
//   B2 sqrt(1 - r2) (Lambertian)
//   C  unit(direction) (Lambertian)  |  unit(reflect) (Metal);  1 / ior (Dielectric, front face)
//   D1 cos_theta / PI (Lambertian pdf)  |  r0 = (1 - ri) / (1 + ri) (Dielectric, Schlick)
//   D2 1 / pdf (Lambertian);  E  the refracted ray's sqrt (Dielectric)
// Every lane computes exactly the operations of its class, in the
// reference's order (the same doubles as shade()); only the instructions
// are shared.  Returns true when the path ends (panic: a reference panic
// condition).
__device__ __forceinline__ bool shade_hit_basic(const SceneView& S, Ray& ray, D3& beta, const HitInfo& h, bool& panic,
                                                const Draws& Dr) {
    const Rec rec = make_record<TIER_BASIC>(S, ray, h, panic);
    if (panic) return true;
    const DMaterial M = S.materials[rec.mat];
    constexpr int LAMB = 0, METAL = 1, DIEL = 2;
    const int cls = (M.type == M_LAMBERTIAN || M.type == M_EMPTY) ? LAMB
                  : M.type == M_METAL ? METAL : M.type == M_DIELECTRIC ? DIEL : 3;
    if (cls == 3) return true;  // (no other material reaches the basic tier)
    const D3 n = rec.n;
    const double xi0 = Dr.xi0, xi1 = Dr.xi1, sn0 = Dr.sn, cs0 = Dr.cs;
    // the albedo (Lambertian, material.rs:60-65) or attenuation (Dielectric, :141)
    D3 tex = d3(0.75, 0.75, 0.75);  // EmptyMaterial (material.rs:41-46)
    if (M.type == M_LAMBERTIAN || cls == DIEL) tex = mat_tex<false, false>(S, M, rec.u, rec.v, rec.p);
    // ---- A
    D3 vA = ray.d;
    if (cls == LAMB) {  // onb.rs:8-21
        const D3 a = fabs(n.x) > 0.9 ? d3(0.0, 1.0, 0.0) : d3(1.0, 0.0, 0.0);
        vA = cross(n, a);
    }
    bool okA;
    const D3 uA = unit(vA, okA);
    if (!okA) {
        if (cls == METAL) return true;  // material.rs:83: r_in.direction not normalizable -> None
        panic = true;                   // onb.rs / material.rs:120: .expect
    }
    // ---- B1, B2
    double cosd = 0.0, xB1 = xi1;  // Lambertian: r2 (vec3.rs:333-343)
    if (cls == METAL) xB1 = xi1 * (1.0 - xi1);  // vec3.rs:313-322
    if (cls == DIEL) {                          // material.rs:121-122
        cosd = fmin(dot(-uA, n), 1.0);
        xB1 = 1.0 - cosd * cosd;
    }
    const double sB1 = k_sqrt(xB1);
    double sB2 = 0.0;
    if (cls == LAMB) sB2 = k_sqrt(1.0 - xi1);
    // ---- C
    D3 vC = ray.d;
    if (cls == LAMB) {  // onb_world: v.x u + v.y n + v.z w (onb.rs:34-38)
        const D3 w = cross(uA, n);
        const D3 v = d3(sn0 * sB1, sB2, cs0 * sB1);
        vC = v.x * uA + v.y * n + v.z * w;
    } else if (cls == METAL) {
        vC = reflect(uA, n);
    }
    const double lC = len(vC);
    const double qC = 1.0 / (cls == DIEL ? M.fuzz : lC);  // unit(): (1 / |v|) v; Dielectric: 1 / ior
    const D3 uC = qC * vC;
    const bool okC = finite3(uC);
    if (cls == METAL) {  // material.rs:82-95
        if (!okC) return true;
        const double s = sB1;
        const D3 ruv = d3(cs0 * 2.0 * s, sn0 * 2.0 * s, 1.0 - 2.0 * xi1);
        beta = beta * d3(M.albedo[0], M.albedo[1], M.albedo[2]);
        ray = Ray{rec.p, uC + (M.fuzz * ruv), ray.time};
        return panic;
    }
    // ---- D1
    double ct = 0.0, ri = 0.0;
    bool refl = false;
    if (cls == LAMB) {
        if (!okC) panic = true;  // pdf.rs:22-28 (the direction's unit)
        ct = dot(uC, n);
    } else {  // Dielectric: ri (material.rs:118), total internal reflection (:123)
        ri = rec.front ? qC : M.fuzz;
        refl = ri * sB1 > 1.0;
    }
    const double qD1 = (cls == LAMB ? ct : 1.0 - ri) / (cls == LAMB ? PI : 1.0 + ri);
    if (cls == LAMB) {  // pdf.rs:50-57, camera.rs:305-316
        const double pdf = fmax(0.0, qD1);
        const double cp = fmax(ct, 0.0);
        const D3 f = divs(tex * d3(cp, cp, cp), PI);
        if (pdf == 0.0) panic = true;  // camera.rs:309
        beta = beta * divs(f, pdf);
        ray = Ray{rec.p, vC, ray.time};
        return panic;
    }
    // Dielectric: Schlick (material.rs:110-114), the draw only when refraction is possible
    if (!refl) {
        const double r0 = qD1;
        const double r0sq = r0 * r0;
        const double x = 1.0 - cosd;
        const double x2 = x * x;
        refl = r0sq + (1.0 - r0sq) * (x * (x2 * x2)) > xi0;
    }
    D3 dir;
    if (refl) {
        dir = reflect(uA, n);
    } else {  // vec3.rs:345-354
        const D3 perp = ri * (uA + cosd * n);
        const double pl = k_sqrt(1.0 - len2(perp));
        if (isnan(pl)) panic = true;
        dir = perp + (-pl * n);
    }
    beta = beta * tex;
    ray = Ray{rec.p, dir, ray.time};
    return panic;
}

// ------------------------------------------------------------------ the kernel
#ifndef RT_BASIC_WAVES
#define RT_BASIC_WAVES 4  // waves per SIMD the basic tier is register-allocated for
#endif
#ifndef RT_FULL_WAVES
#define RT_FULL_WAVES 2  // full tier (C5): 2 waves without spills, shading in batches of 56 (below)
#endif
#ifndef RT_FLAT_WAVES
#define RT_FLAT_WAVES 3  // FULL_FLAT
#endif
// Lanes of a wave that must have finished their walk before it shades (64 =
// all).  Trace-heavy worlds (deep triangle BVHs) gain from shading in batches;
// for C2 the shading divergence of small batches costs more than the walks
// gain (A/B in DESIGN.md).
#ifndef RT_SHADE_BATCH_BASIC
// basic tier over a tree of at most NODE_LDS_CAP_BATCH nodes (C1 / C2: 241):
// shading in 56-lane batches, the carried-over walks parked in LDS (32 KiB
// taken from the node copy).  Round 5, with the shared-draws loop: C2 -2.3 %
// kernel time against whole-wave shading (A/B at 128 spp, RMSE 0; round 2's
// loop had measured +1.7 %).  Larger trees (up to NODE_LDS_CAP) run the
// whole-wave variant of the tier (rt_path_kernel<TIER_BASIC, true>).
#define RT_SHADE_BATCH_BASIC 56
#endif
#ifndef RT_SHADE_BATCH_MESH
#define RT_SHADE_BATCH_MESH 48
#endif
#ifndef RT_SHADE_BATCH_FULL
// C5 walks are uneven (37 % lane efficiency with whole-wave shading): at 2
// waves/SIMD the 256-VGPR budget holds the walk state across a shading batch
// without spills, C5 -12 % against 3 waves / whole-wave shading; at 3 waves
// batches spill 372 B/lane and cost +65 %
#define RT_SHADE_BATCH_FULL 56
#endif
#ifndef RT_SHADE_BATCH_FLAT
#define RT_SHADE_BATCH_FLAT 64
#endif
#ifndef RT_QUEUE_CHUNK
// most entries a wave takes per queue atomic, with chunks shrinking as
// left / (waves x RT_QUEUE_GUIDE): 512 / 16 against 256 / 8 -- half the
// counter's atomics early, smaller pools late -- C2 186.3 -> 185.0 ms frame
// and 1/8 shard 24.8 -> 24.4, C4 188.6 -> 186.2 and 29.8 -> 26.7, C3 +-0.5 %
// (A/B, 2 interleaved reps each; 512 at guide 8: C2 frame -1.1 % but shard
// +11 %; 512 / 32 and 1024 / 32: C2 shard +4-5 %)
#define RT_QUEUE_CHUNK 512
#endif
#ifndef RT_QUEUE_CHUNK_MESH
// the mesh tier's cap, a knob: its rounds are long (a dependent global load
// per walk step) and a large pool can outlive the queue by milliseconds, but
// smaller caps cost the whole frame in counter contention (at guide 8, cap
// 128: C4 frame +2 %, 1/8 shard 30.0 -> 27.3 ms; 64: +6 %, 27.2 ms)
#define RT_QUEUE_CHUNK_MESH RT_QUEUE_CHUNK
#endif
#ifndef RT_QUEUE_GUIDE
#define RT_QUEUE_GUIDE 16  // guided chunks: left / (waves * GUIDE), 0 = fixed RT_QUEUE_CHUNK
#endif
#ifndef RT_MESH_WAVES
#define RT_MESH_WAVES 4  // beats 2 waves (164.7 vs 263.8 ms, C4 64 spp) and 3 / 5 waves (+16 % / +12 %)
#endif

// Queue entry q -> its stratum-row item and samples [s_j, s_end) (Frame:
// whole rows, then parts, then the fine parts of the frame's last rows).
__device__ __forceinline__ void queue_entry(const Frame& F, uint32_t q, uint32_t& item, uint32_t& s_j,
                                            uint32_t& s_end) {
    const bool whole = q < F.whole_items, fine = q >= F.fine_q0;
    const uint32_t qt = whole ? 0u : q - (fine ? F.fine_q0 : F.whole_items);  // (udiv_inv wants n < 2^32 in range)
    const uint32_t np = fine ? F.parts2 : F.parts, pl = fine ? F.part_len2 : F.part_len;
    const uint32_t it = udiv_inv(qt, fine ? F.inv_parts2 : F.inv_parts), part = qt - it * np;
    item = whole ? q : (fine ? F.fine_item0 : F.whole_items) + it;
    s_j = whole ? 0u : part * pl;
    s_end = whole ? F.S : min(F.S, s_j + pl);
}
// The guided chunk of a wave whose pool ends at pool_end: about 1/GUIDE of
// the samples left (as last seen) per wave of the grid, in the entries of
// the region the next pool starts in; never below what the wave's lanes need
// now (n lanes, avail entries in the pool), nor below Frame::chunk_min.
__device__ __forceinline__ uint32_t guided_chunk(const Frame& F, uint32_t pool_end, uint32_t avail, uint32_t n) {
    const uint32_t whole_left = F.whole_items > pool_end ? F.whole_items - pool_end : 0u;
    const uint32_t p0 = max(pool_end, F.whole_items), part_left = F.fine_q0 > p0 ? F.fine_q0 - p0 : 0u;
    const uint32_t f0 = max(pool_end, F.fine_q0), fine_left = F.queue_total > f0 ? F.queue_total - f0 : 0u;
    const float g = ((float)whole_left * F.S_f + (float)part_left * F.part_len_f + (float)fine_left * F.part_len2_f) *
                    F.inv_guide;
    const float inv_per = whole_left ? F.inv_S_f : (part_left ? F.inv_part_len_f : F.inv_part_len2_f);
    const uint32_t chunk = min((uint32_t)(g * inv_per), F.chunk_cap);
    return max(max(chunk, whole_left ? F.chunk_min_whole : F.chunk_min), avail < n ? n - avail : 0u);
}

// Launch parameters live in device memory and are read where they are used
// (scalar loads), not pinned in SGPRs for the life of the kernel.
struct KParams {
    SceneView S;
    Frame F;
    uint32_t* queue;
    double* partial;  // [queue_total][3]: the f64 sum of each queue entry's samples
    unsigned long long* stats;
    RT_GLOBAL uint2* stack_ovf;  // mesh / full tiers: [stack_need - LDS entries][grid * RT_BLOCK]
};

template <int TIER>
__device__ __forceinline__ StackFor<TIER> make_stack(RT_LDS uint2* s8, RT_LDS uint32_t* s4, RT_GLOBAL uint2* ovf,
                                                     uint32_t stride) {
    if constexpr (TIER == TIER_BASIC)
        return StackFor<TIER>{s4};
    else
        return StackFor<TIER>{s8, ovf, stride};
}
constexpr uint32_t RT_PARK_WORDS = 8;

// WIDE (basic tier only): the variant for trees of NODE_LDS_CAP_BATCH +
// 1 .. NODE_LDS_CAP nodes -- the whole LDS node copy, whole-wave shading, no
// park area.
template <int TIER, bool WIDE = false>
__global__ void __launch_bounds__(TIER == TIER_BASIC ? RT_BLOCK_BASIC : RT_BLOCK, TIER == TIER_FULL_FLAT ? RT_FLAT_WAVES : tier_full_bvh(TIER) ? RT_FULL_WAVES : (TIER == TIER_MESH ? RT_MESH_WAVES : RT_BASIC_WAVES))
    rt_path_kernel(const KParams* __restrict__ P) {
    static_assert(!WIDE || TIER == TIER_BASIC, "the wide variant is the basic tier's");
    constexpr int BASIC_BATCH = WIDE ? 64 : RT_SHADE_BATCH_BASIC;
    constexpr uint32_t NODE_CAP = WIDE ? NODE_LDS_CAP : NODE_LDS_CAP_BATCH;
    // The params block is read-only for the launch: scalar loads, hoisted.
    const SceneView S = P->S;
    const Frame& F = P->F;
    uint32_t* queue = P->queue;
    constexpr int STACK = lds_stack_entries(TIER);
    constexpr uint32_t BLK = TIER == TIER_BASIC ? RT_BLOCK_BASIC : RT_BLOCK;
    constexpr bool B4 = TIER == TIER_BASIC;
    // The lane arena (all tiers but the basic one): one uint2 row per lane and
    // row, RT_BLOCK apart -- the stack's rows, then (full tiers) the media
    // queue's (MedQ), then (full-flat tier) the parked path state's -- so
    // that every per-lane LDS access is one base address (threadIdx.x * 8)
    // plus a constant in the instruction's offset field, not a base VGPR per
    // array held across the path loop
    constexpr bool LDS_STATE = TIER == TIER_FULL_FLAT;
    constexpr bool PARK_RAY = LDS_STATE;  // + the world ray (7 doubles)
    constexpr uint32_t R_MED = B4 ? 0u : (uint32_t)STACK;
    constexpr uint32_t R_PST = R_MED + (tier_full(TIER) ? 2u * RT_MEDIA_CAP : 0u);
    constexpr uint32_t R_PIT = R_PST + (LDS_STATE ? (PARK_RAY ? 16u : 9u) : 0u);
    constexpr uint32_t R_END = R_PIT + (LDS_STATE ? 2u : 0u);
    __shared__ uint2 lane_lds[B4 ? 1 : R_END * BLK];
    __shared__ uint32_t stack4_lds[B4 ? STACK * BLK : 1];
    RT_LDS uint2* const lrow = (RT_LDS uint2*)(lane_lds + threadIdx.x);
    const MedQ med{lrow + R_MED * BLK};
    __shared__ uint16_t pend_lds[TIER == TIER_BASIC && RT_BVH4 ? RT_PEND_CAP * BLK : 1];
    RT_LDS uint16_t* pq = (RT_LDS uint16_t*)(pend_lds + threadIdx.x);
    StackFor<TIER> stk = make_stack<TIER>(lrow, (RT_LDS uint32_t*)(stack4_lds + threadIdx.x),
                                          P->stack_ovf + (uint64_t)blockIdx.x * BLK + threadIdx.x, gridDim.x * BLK);
    // Basic tier with shading batches: the walk state of a lane whose walk
    // carries over a shading round is parked here across it (RT_PARK_WORDS
    // words: cur, sp | pn | found, c, c_f, hit t, hit ref), so that the
    // shading code does not hold it in registers.
    constexpr bool PARK = (TIER == TIER_BASIC && BASIC_BATCH < 64) ||
                          (TIER == TIER_MESH && RT_SHADE_BATCH_MESH < 64);
    __shared__ __attribute__((aligned(16))) uint32_t park_lds[PARK ? RT_PARK_WORDS * BLK : 1];
    RT_LDS uint32_t* pk = (RT_LDS uint32_t*)(park_lds + threadIdx.x);
    RT_LDS uint2* pk2 = (RT_LDS uint2*)park_lds + threadIdx.x;  // basic tier: 8-byte rows (trace_park2)
    // Basic tier: the block's copy of the world's 4-wide nodes (the whole tree:
    // 241 nodes for C1/C2), read by every node visit instead of global memory.
    __shared__ float4 node_lds[TIER == TIER_BASIC && RT_BVH4 ? NODE_CAP * 7 : 1];
    if constexpr (TIER == TIER_BASIC && RT_BVH4) {
        const uint32_t n_lds = min(S.n_nodes4, NODE_CAP);  // == n_nodes4 (launcher: rtk_launch_frame)
        const RT_GLOBAL float4* src = reinterpret_cast<const RT_GLOBAL float4*>(S.nodes4);
        for (uint32_t k = threadIdx.x; k < n_lds * 7u; k += BLK) {
            float4 v = src[k];
            if (k % 7u == 6u) {  // the ref row: walk words (bword)
                v.x = __uint_as_float(bword(S, __float_as_uint(v.x)));
                v.y = __uint_as_float(bword(S, __float_as_uint(v.y)));
                v.z = __uint_as_float(bword(S, __float_as_uint(v.z)));
                v.w = __uint_as_float(bword(S, __float_as_uint(v.w)));
            }
            node_lds[k] = v;
        }
        __syncthreads();
    }
    if constexpr (tier_full_bvh(TIER) && RT_PERLIN_LDS) {
        if (S.n_perlin > 0) {
            const RT_GLOBAL float4* src = reinterpret_cast<const RT_GLOBAL float4*>(S.perlin);
            RT_LDS float4* dst = (RT_LDS float4*)&g_perlin_lds;
            for (uint32_t k = threadIdx.x; k < sizeof(DPerlin) / 16; k += BLK) dst[k] = src[k];
            __syncthreads();
        }
    }
    // Full-flat tier: the path state the walk never reads (beta, L, acc, the
    // item's fields) is parked in LDS across the walk, so that its registers
    // are free there instead of spilled to scratch around it.
    RT_LDS double* const pst = (RT_LDS double*)(lrow + R_PST * BLK);
    RT_LDS uint2* const pit = lrow + R_PIT * BLK;
    // ... and the queue entry's running sum and part-sum slot stay there for
    // the whole entry (pst rows 6-8, pit row 1 .y): read at the sample's end
    // only, they hold no registers through the shading code
    constexpr bool ACC_LDS = LDS_STATE;

    Rng rng;
    rng.k0 = F.key0;
    rng.k1 = F.key1;
    // the lane's queue entry: stratum row s_i of pixel rng.pixel (= py * W +
    // px), samples s_j ..< s_end (sie = s_i | s_end << 16: S < 2^16),
    // partial-sum slot `slot` -- few registers across the path loop
    uint32_t slot = 0, s_j = 0, sie = 0;
    bool need = true;
    bool in_path = false;
    // defined from the start: the basic tier's walk-field set-up reads it for
    // lanes without a path too (values never used; no indeterminate read)
    Ray ray{};
    D3 beta = d3(1, 1, 1), L = d3(0, 0, 0), acc = d3(0, 0, 0);
    uint32_t vertex = 0;
    uint32_t n_rays = 0, n_panics = 0;

    // wave-uniform: the queue entries this wave holds.  Wave w starts with the
    // 64 entries [64 w, 64 w + 64) -- no atomic at launch: 4096 waves taking
    // their first chunk from one counter at once waited up to 2.9 ms for it
    // (scripts/lone_wave.py) -- and the counter hands out entries from
    // Frame::static_entries on.  `dry`: an atomic of this wave has passed the
    // end of the queue, so none will hand out entries any more -- lanes that
    // need one leave without another atomic (the drain's waves waited ~70 us
    // a round on the counter the whole grid hammered).
    uint32_t pool_next = (blockIdx.x * (BLK / 64) + threadIdx.x / 64) * 64u, pool_end = pool_next + 64u;
    bool dry = false;
    Diag dg;
    Trav<TIER> T;
    bool walking = false;
    // RT_SHADE_DEFER (full BVH tier): this lane's finished walk waits for a later
    // shading round; the wave's count of rounds deferred in a row
    constexpr bool DEFER = RT_SHADE_DEFER && TIER == TIER_FULL;
    bool deferred = false;
    uint32_t defer_rounds = 0;
#ifdef RT_WAVE_TRACE
    const uint32_t trace_lane = blockIdx.x * BLK + threadIdx.x;
    const unsigned long long trace_t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long trace_c0 = __builtin_amdgcn_s_memtime();
    uint32_t trace_items = 0, trace_q = 0, trace_rays = 0, trace_steps = 0, trace_steps_q = 0;
    // the wave's queue atomics: count and the ticks from issue to return
    // (wave-uniform; every lane holds the wave's value)
    unsigned long long trace_atomic_ticks = 0, trace_atomic_first = 0;
    uint32_t trace_atomics = 0;
    RayHist hist;
    hist.t0 = trace_t0;  // (an s_memrealtime: one value per wave)
    unsigned long long trace_tq = trace_t0;
#endif
    // ---- refill: the lanes that need a queue entry take one (false: the
    // queue is done and this lane leaves the loop)
    auto refill = [&]() -> bool {
        // wave-aggregated dequeue of stratum rows.  The wave takes
        // RT_QUEUE_CHUNK items per atomic into a wave-uniform pool and hands them
        // to its lanes in rank order: one contended atomic per chunk, not one per
        // main-loop iteration (every iteration some lane of the wave needs work).
        const unsigned long long mask = __ballot(need);
        if (mask) {
            const uint32_t n = (uint32_t)__popcll(mask);
            const uint32_t avail = pool_end - pool_next;
            uint32_t fresh = 0;
            // guided chunk: about 1/GUIDE of the items left (as last seen) per
            // wave of the grid, so the last chunks are small and waves finish
            // together; never below what the wave's lanes need now, nor below
            // Frame::chunk_min.  Near the end a wave takes only what its lanes
            // need: a pool held by a slow wave (deep glass paths) is work the
            // idle waves cannot take (scripts/lane_trace.py).
            // (the chunk in the entries it takes: a pool of whole rows taken
            // as the tail starts is no larger in samples than the tail's
            // pools -- it would outlast them)
            const uint32_t chunk = RT_QUEUE_GUIDE ? guided_chunk(F, pool_end, avail, n) : (uint32_t)RT_QUEUE_CHUNK;
            // the lane's rank among the needy lanes (the leader: rank 0 with
            // need); the leader's atomic result is read with v_readlane -- no
            // lane id held across the loop, no ds_bpermute
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
            if (avail < n) {
                if (!dry) {
                    const uint32_t leader = __ffsll((long long)mask) - 1;
#ifdef RT_WAVE_TRACE
                    const unsigned long long ta = __builtin_amdgcn_s_memrealtime();
#endif
                    if (need && rank == 0) fresh = atomicAdd(queue, chunk);
                    fresh = __builtin_amdgcn_readlane(fresh, leader) + F.static_entries;
#ifdef RT_WAVE_TRACE
                    {
                        const unsigned long long tb = __builtin_amdgcn_s_memrealtime();
                        trace_atomic_ticks += tb - ta;
                        if (trace_atomics++ == 0) trace_atomic_first = tb - trace_t0;
                    }
#endif
                    dry = fresh + chunk >= F.queue_total;
                } else {
                    fresh = F.queue_total;  // past the end: the needy lanes leave
                }
            }
            const uint32_t old_next = pool_next;
            if (avail < n) {
                pool_next = fresh + (n - avail);
                pool_end = fresh + chunk;
            } else {
                pool_next += n;
            }
            if (need) {
                const uint32_t q = rank < avail ? old_next + rank : fresh + (rank - avail);
                if (q >= F.queue_total) return false;
                need = false;
#ifdef RT_WAVE_TRACE
                ++trace_items;
                trace_q = q;
                trace_rays = n_rays;
                trace_steps_q = trace_steps;
                trace_tq = __builtin_amdgcn_s_memrealtime();
#endif
                uint32_t item, s_end;
                queue_entry(F, q, item, s_j, s_end);
                acc = d3(0, 0, 0);
                const uint32_t pl = udiv_inv(item, F.inv_S), s_i = item - pl * F.S;
                sie = s_i | (s_end << 16);
                slot = q;
                const uint32_t prow = udiv_inv(pl, F.inv_W);
                rng.pixel = (F.row_offset + prow * F.row_stride) * F.W + (pl - prow * F.W);
            }
        }
        return true;
    };
    // ---- the end of a lane's sample (camera.rs:193's sum, in s_j order): its
    // radiance joins the entry's sum; the entry's last sample writes the sum
    auto finish_sample = [&]() {
        if (isnan(L.x) || isnan(L.y) || isnan(L.z)) {  // camera.rs:323
            ++n_panics;
            L = d3(0, 0, 0);
        }
        acc = acc + L;
        ++s_j;
        if (s_j == (sie >> 16)) {
#ifndef RT_MEASURE_NOSTORE
            double* dst = P->partial + (uint64_t)slot * 3;
            dst[0] = acc.x;
            dst[1] = acc.y;
            dst[2] = acc.z;
#endif
            need = true;
        }
    };
    if constexpr (TIER == TIER_BASIC) {
        // Basic / mesh tiers: a lane's iteration is walk -> (miss: the sample
        // ends) -> refill -> draws -> shade or a new sample's camera ray, so
        // that the one Philox block and sincos of the iteration's Draws serve
        // both (struct Draws).  A lane whose path ends in shading (depth,
        // panic, no scatter) starts its next sample one iteration later.
        bool no_path = true;  // the lane starts a sample at its next post-walk stage
        constexpr int BATCH = TIER == TIER_BASIC ? BASIC_BATCH : RT_SHADE_BATCH_MESH;
        // ---- Camera::get_ray (camera.rs:247-273), vertex 0, from the iteration's draws
        auto camera_ray = [&](const Draws& Dr) {
            const uint32_t s_i = sie & 0xFFFFu, py = udiv_inv(rng.pixel, F.inv_W), px = rng.pixel - py * F.W;
            double xi0 = Dr.xi0, xi1 = Dr.xi1;
            D3 origin = F.center;
            if (F.defocus) {  // vec3.rs:63-69: theta = 2 pi Dr.xi0, r = sqrt(Dr.xi1)
#ifndef RT_MEASURE_NOCAMPAIR
                rng.pair(0u, 0u, xi0, xi1);
#endif
                const double rr = k_sqrt(Dr.xi1);
                origin = (F.center + ((rr * Dr.cs) * F.disk_u)) + ((rr * Dr.sn) * F.disk_v);
            }
            const double ox = (((double)s_i + xi0) * F.recip_sqrt_spp) - 0.5;
            const double oy = (((double)s_j + xi1) * F.recip_sqrt_spp) - 0.5;
            const D3 ps = (F.pixel00 + (((double)px + ox) * F.du)) + (((double)py + oy) * F.dv);
            ray.o = origin;
            ray.d = ps - origin;
            ray.time = 0.0;  // read only by moving spheres (full tiers): its draw is skipped
            beta = d3(1, 1, 1);
            L = d3(0, 0, 0);
            vertex = 1;
            no_path = false;
        };
        for (;;) {
            RT_DIAG_ONLY(const unsigned long long t_loop0 = __builtin_amdgcn_s_memtime(); ++dg.main_iters;)
            RT_ISA_MARK("fields");
#ifdef RT_WAVE_TRACE
            hist.add(__ballot(!no_path && !walking));
#endif
            if constexpr (TIER == TIER_BASIC && PARK) {
                // a new walk and a walk carried over the last shading round
                // make the same ray-derived fields: once, for both (as two
                // branches the wave ran that code twice in most rounds: C2
                // -0.7 %, profiles/r05/ab_shared_rayfields_c2_128spp.json).
                // A lane with no path (it starts its sample after this walk
                // phase) sets up the walk state too, which it does not walk:
                // the state is then defined on every path into the walk, so
                // that the compiler need not keep the last walk's values live
                // through the shading code (C2 -1.6 %: 28 B/lane of scratch
                // -> none, 128 -> 124 VGPRs; ab_define_t_c2_128spp.json)
                trace_ray_fields(ray, T);
                if (!walking) {
                    T.cl.c = __builtin_huge_val();
                    T.cl.c_f = __builtin_huge_valf();
                    T.sp = 0;
                    T.found = false;
                    T.pn = 0;
                    T.nxf = 0;
                    T.hit.nxf = 0;
                    T.nmed = 0;
                    T.cur = bword(S, S.world_root);
                    if (!no_path) {
                        rng.begin(vertex);
                        ++n_rays;
                        walking = true;
                    }
                } else {
                    trace_unpark_state2(T, pk2);
                }
            } else if (!no_path && !walking) {  // the whole-wave variant: every walk ends in the walk phase
                rng.begin(vertex);
                ++n_rays;
                trace_begin<TIER>(S, ray, T);
                walking = true;
            }
            RT_DIAG_ONLY(const unsigned long long t_b0 = __builtin_amdgcn_s_memtime(); dg.cyc_refill += t_b0 - t_loop0;)
            RT_ISA_MARK("walk");
            auto step = [&]() -> bool {
                if constexpr (TIER == TIER_BASIC && RT_BVH4) {
                    return trace4_step(S, ray, T, stk, pq, (const RT_LDS float4*)node_lds, dg);
                } else {
                    RT_DIAG_ONLY(if (__lane_id() == (uint32_t)(__ffsll((long long)__ballot(true)) - 1)) ++dg.wave_trace_iters; ++dg.lane_trace_iters;)
                    return trace_step<TIER>(S, ray, T, stk, rng, med, dg);
                }
            };
            if constexpr (BATCH >= 64) {
#ifdef RT_WAVE_TRACE
                while (walking) walking = step(), ++trace_steps;
#else
                while (walking) walking = step();
#endif
            } else {
                const unsigned long long active = __ballot(true);
                for (;;) {
                    if (walking) walking = step();
                    const unsigned long long w = __ballot(walking);
                    if (w == 0 || __popcll(active & ~w) >= BATCH) break;
                }
            }
            RT_DIAG_ONLY(const unsigned long long t_b1 = __builtin_amdgcn_s_memtime(); dg.cyc_trace += t_b1 - t_b0;)
            // a walk that carries over this shading round is parked;
            // the lane skips the rest of the iteration but for the refill,
            // which every lane of the wave runs: the queue pool (pool_next,
            // pool_end, dry) is wave-uniform state and must be updated in
            // uniform control flow, or a parked lane would keep a stale copy
            RT_ISA_MARK("park");
            const bool carry = BATCH < 64 && walking;
            if constexpr (PARK) {
                if (carry) trace_park2(T, pk2);
            }
            // ---- this lane's walk is over, or it has no path
            bool cam = no_path;
            if (!carry && !no_path && !T.found) {  // a miss: Environment::value, and the sample ends
                RT_ISA_MARK("miss");
#ifndef RT_MEASURE_NOSKY
                bool panic = false;
                shade<TIER>(S, ray, beta, L, rng, false, T.hit, panic);
                if (panic) ++n_panics;
#endif
                finish_sample();
                cam = true;
            }
            RT_DIAG_ONLY(const unsigned long long t_m = __builtin_amdgcn_s_memtime(); dg.cyc_miss += t_m - t_b1;)
            RT_ISA_MARK("refill");
            if (!refill()) break;
            RT_DIAG_ONLY(const unsigned long long t_q = __builtin_amdgcn_s_memtime(); dg.cyc_queue += t_q - t_m;)
            if (carry) continue;
            // the iteration's draws: a hit's (vertex, slots 0 and 1) or a new
            // sample's camera draws (vertex 0: theta and r of the defocus disk
            // at slots 2 and 3, else the pixel offsets at slots 0 and 1)
            RT_ISA_MARK("draws");
            if (cam) rng.sample = (sie & 0xFFFFu) * F.S + s_j;
            Draws Dr;
            rng.pair(cam ? 0u : vertex, (cam && F.defocus) ? 1u : 0u, Dr.xi0, Dr.xi1);
            k_sincos_2pi(Dr.xi0, &Dr.sn, &Dr.cs);
            RT_DIAG_ONLY(const unsigned long long t_d = __builtin_amdgcn_s_memtime(); dg.cyc_refill += t_d - t_b1;
                         dg.cyc_draws += t_d - t_q;)
            if (!cam) {
                RT_ISA_MARK("shade");
                // ---- one ray_color level (camera.rs:275-325) at depth max_depth - vertex + 1
                rng.begin(vertex);
                rng.slot = 2;  // slots 0 and 1 are Dr
                bool panic = false;
                bool end_path;
                if constexpr (TIER == TIER_BASIC && RT_SHADE_MERGED && !WIDE)  // (the wide variant spills 76 B/lane with it)
                    end_path = shade_hit_basic(S, ray, beta, T.hit, panic, Dr);
                else
                    end_path = shade<TIER>(S, ray, beta, L, rng, true, T.hit, panic, Dr);
                if (panic) {
                    ++n_panics;
                    end_path = true;
                }
                if (!end_path) {
                    ++vertex;
                    if (vertex > F.max_depth) end_path = true;  // depth == 0 -> BLACK (camera.rs:282-284)
                }
                if (end_path) {
                    finish_sample();
                    no_path = true;
                }
                RT_DIAG_ONLY(dg.cyc_shade += __builtin_amdgcn_s_memtime() - t_d;)
            } else {
                RT_ISA_MARK("camera");
                camera_ray(Dr);
                RT_DIAG_ONLY(dg.cyc_refill += __builtin_amdgcn_s_memtime() - t_d;)
            }
        }
    } else {
    for (;;) {
        RT_DIAG_ONLY(const unsigned long long t_loop0 = __builtin_amdgcn_s_memtime(); ++dg.main_iters;)
        // ---- refill: wave-aggregated dequeue of stratum rows.  The wave takes
        // RT_QUEUE_CHUNK items per atomic into a wave-uniform pool and hands them
        // to its lanes in rank order: one contended atomic per chunk, not one per
        // main-loop iteration (every iteration some lane of the wave needs work).
        const unsigned long long mask = __ballot(need);
        if (mask) {
            const uint32_t n = (uint32_t)__popcll(mask);
            const uint32_t avail = pool_end - pool_next;
            uint32_t fresh = 0;
            // guided chunk: about 1/GUIDE of the items left (as last seen) per
            // wave of the grid, so the last chunks are small and waves finish
            // together; never below what the wave's lanes need now, nor below
            // Frame::chunk_min.  Near the end a wave takes only what its lanes
            // need: a pool held by a slow wave (deep glass paths) is work the
            // idle waves cannot take (scripts/lane_trace.py).
            // (the chunk in the entries it takes: a pool of whole rows taken
            // as the tail starts is no larger in samples than the tail's
            // pools -- it would outlast them)
            const uint32_t chunk = RT_QUEUE_GUIDE ? guided_chunk(F, pool_end, avail, n) : (uint32_t)RT_QUEUE_CHUNK;
            // the lane's rank among the needy lanes (the leader: rank 0 with
            // need); the leader's atomic result is read with v_readlane -- no
            // lane id held across the loop, no ds_bpermute
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
            if (avail < n) {
                if (!dry) {
                    const uint32_t leader = __ffsll((long long)mask) - 1;
#ifdef RT_WAVE_TRACE
                    const unsigned long long ta = __builtin_amdgcn_s_memrealtime();
#endif
                    if (need && rank == 0) fresh = atomicAdd(queue, chunk);
                    fresh = __builtin_amdgcn_readlane(fresh, leader) + F.static_entries;
#ifdef RT_WAVE_TRACE
                    {
                        const unsigned long long tb = __builtin_amdgcn_s_memrealtime();
                        trace_atomic_ticks += tb - ta;
                        if (trace_atomics++ == 0) trace_atomic_first = tb - trace_t0;
                    }
#endif
                    dry = fresh + chunk >= F.queue_total;
                } else {
                    fresh = F.queue_total;  // past the end: the needy lanes leave
                }
            }
            const uint32_t old_next = pool_next;
            if (avail < n) {
                pool_next = fresh + (n - avail);
                pool_end = fresh + chunk;
            } else {
                pool_next += n;
            }
            if (need) {
                const uint32_t q = rank < avail ? old_next + rank : fresh + (rank - avail);
                if (q >= F.queue_total) break;
                need = false;
#ifdef RT_WAVE_TRACE
                ++trace_items;
                trace_q = q;
                trace_rays = n_rays;
                trace_steps_q = trace_steps;
                trace_tq = __builtin_amdgcn_s_memrealtime();
#endif
                uint32_t item, s_end;
                queue_entry(F, q, item, s_j, s_end);
                if constexpr (ACC_LDS)  // the entry's sum lives in LDS (flat tier)
                    pst[6 * RT_BLOCK] = 0.0, pst[7 * RT_BLOCK] = 0.0, pst[8 * RT_BLOCK] = 0.0;
                else
                    acc = d3(0, 0, 0);
                const uint32_t pl = udiv_inv(item, F.inv_S), s_i = item - pl * F.S;
                sie = s_i | (s_end << 16);
                if constexpr (ACC_LDS)
                    pit[BLK].y = q;
                else
                    slot = q;
                const uint32_t prow = udiv_inv(pl, F.inv_W);
                rng.pixel = (F.row_offset + prow * F.row_stride) * F.W + (pl - prow * F.W);
            }
        }
        if (!in_path) {
            // ---- Camera::get_ray (camera.rs:247-273), vertex 0
            const uint32_t s_i = sie & 0xFFFFu, py = udiv_inv(rng.pixel, F.inv_W), px = rng.pixel - py * F.W;
            rng.sample = s_i * F.S + s_j;
            rng.begin(0);
            uint32_t ovf = 0;
            const double xi0 = rng.next(ovf), xi1 = rng.next(ovf);
            const double ox = (((double)s_i + xi0) * F.recip_sqrt_spp) - 0.5;
            const double oy = (((double)s_j + xi1) * F.recip_sqrt_spp) - 0.5;
            const D3 ps = (F.pixel00 + (((double)px + ox) * F.du)) + (((double)py + oy) * F.dv);
            D3 origin = F.center;
            if (F.defocus) {
                const double xt = rng.next(ovf);  // theta = 0.0 + (2.0 * PI - 0.0) * xt = 2.0 * PI * xt (vec3.rs:63-69)
                const double rr = k_sqrt(rng.next(ovf));
                double sn, cs;
                k_sincos_2pi(xt, &sn, &cs);
                origin = (F.center + ((rr * cs) * F.disk_u)) + ((rr * sn) * F.disk_v);
            }
            ray.o = origin;
            ray.d = ps - origin;
            // the ray's time (vertex 0's last draw) is read only by moving
            // spheres, which only the full tiers hold: the basic and mesh
            // tiers skip its Philox block (no other draw depends on it)
            ray.time = tier_full(TIER) ? rng.next(ovf) : 0.0;
            beta = d3(1, 1, 1);
            L = d3(0, 0, 0);
            vertex = 1;
            in_path = true;
        }

        // ---- one ray_color level (camera.rs:275-325) at depth max_depth - vertex + 1:
        // world.hit as a resumable walk.  The wave walks until RT_SHADE_BATCH of its
        // lanes have finished (or none walks any more); those are shaded and get
        // their next ray while the unfinished walks carry over to the next round,
        // so short walks do not idle behind the longest one of the wave.
#ifdef RT_WAVE_TRACE
        hist.add(__ballot(!walking));
#endif
        if (!walking && !(DEFER && deferred)) {
            rng.begin(vertex);
            ++n_rays;
            trace_begin<TIER>(S, ray, T);
            walking = true;
        } else if constexpr (PARK) {
            trace_unpark(ray, T, pk);  // a walk carried over the last shading round
        }
        RT_DIAG_ONLY(const unsigned long long t_b0 = __builtin_amdgcn_s_memtime(); dg.cyc_refill += t_b0 - t_loop0;)
        constexpr int BATCH = TIER == TIER_BASIC ? BASIC_BATCH
                            : TIER == TIER_MESH ? RT_SHADE_BATCH_MESH
                            : TIER == TIER_FULL ? RT_SHADE_BATCH_FULL : RT_SHADE_BATCH_FLAT;
        auto step = [&]() -> bool {
            if constexpr (TIER == TIER_BASIC && RT_BVH4) {
                return trace4_step(S, ray, T, stk, pq, (const RT_LDS float4*)node_lds, dg);
            } else {
                // every step call of the lane (the basic tier counts its own)
                RT_DIAG_ONLY(if (__lane_id() == (uint32_t)(__ffsll((long long)__ballot(true)) - 1)) ++dg.wave_trace_iters; ++dg.lane_trace_iters;)
                if constexpr (PARK_RAY)
                    return trace_step<TIER>(S, RayLds{pst + 9 * RT_BLOCK}, T, stk, rng, med, dg);
                else
                    return trace_step<TIER>(S, ray, T, stk, rng, med, dg);
            }
        };
        if constexpr (BATCH >= 64) {  // the whole wave finishes its walks, then shades
            if constexpr (LDS_STATE) {
                pst[0 * RT_BLOCK] = beta.x, pst[1 * RT_BLOCK] = beta.y, pst[2 * RT_BLOCK] = beta.z;
                pst[3 * RT_BLOCK] = L.x, pst[4 * RT_BLOCK] = L.y, pst[5 * RT_BLOCK] = L.z;
                pit[0] = make_uint2(sie, s_j);
                if constexpr (PARK_RAY) {
                    pst[9 * RT_BLOCK] = ray.o.x, pst[10 * RT_BLOCK] = ray.o.y, pst[11 * RT_BLOCK] = ray.o.z;
                    pst[12 * RT_BLOCK] = ray.d.x, pst[13 * RT_BLOCK] = ray.d.y, pst[14 * RT_BLOCK] = ray.d.z;
                    pst[15 * RT_BLOCK] = ray.time;
                }
            }
#ifdef RT_WAVE_TRACE
            while (walking) walking = step(), ++trace_steps;
#else
            while (walking) walking = step();
#endif
            RT_DIAG_ONLY(const unsigned long long t_m0 = __builtin_amdgcn_s_memtime();)
            if constexpr (PARK_RAY)
                media_phase<TIER>(S, RayLds{pst + 9 * RT_BLOCK}, T, stk, rng, med);
            else if constexpr (tier_full(TIER))
                media_phase<TIER>(S, ray, T, stk, rng, med);
            RT_DIAG_ONLY(dg.cyc_media += __builtin_amdgcn_s_memtime() - t_m0;)
            if constexpr (LDS_STATE) {
                if constexpr (PARK_RAY) ray = RayLds{pst + 9 * RT_BLOCK}.get();
                beta = d3(pst[0 * RT_BLOCK], pst[1 * RT_BLOCK], pst[2 * RT_BLOCK]);
                L = d3(pst[3 * RT_BLOCK], pst[4 * RT_BLOCK], pst[5 * RT_BLOCK]);
                const uint2 it = pit[0];
                sie = it.x, s_j = it.y;
            }
        } else {
            const unsigned long long active = __ballot(true);
            for (;;) {
                if (walking) walking = step();
                const unsigned long long w = __ballot(walking);
                if (w == 0 || __popcll(active & ~w) >= BATCH) break;
            }
        }
        RT_DIAG_ONLY(const unsigned long long t_b1 = __builtin_amdgcn_s_memtime(); dg.cyc_trace += t_b1 - t_b0;)
        if constexpr (BATCH < 64 && tier_full(TIER)) {
            RT_DIAG_ONLY(const unsigned long long t_mb = __builtin_amdgcn_s_memtime();)
            if (!walking && !(DEFER && deferred)) media_phase<TIER>(S, ray, T, stk, rng, med);
            RT_DIAG_ONLY(dg.cyc_media += __builtin_amdgcn_s_memtime() - t_mb;)
        }
        if constexpr (DEFER) {
            // wave-uniform: defer this round's candidates while few are ready,
            // other lanes still walk, and the wave has not waited too long
            const bool others = __ballot(walking) != 0ull;
            const unsigned long long cm = __ballot(!walking && T.found && shade_deferrable(S, T.hit.ref));
            if (cm != 0ull && others && __popcll(cm) < RT_SHADE_DEFER_K && defer_rounds < RT_SHADE_DEFER_WAIT) {
                ++defer_rounds;
                if ((cm >> __lane_id()) & 1ull) deferred = true;
            } else {
                defer_rounds = 0;
                deferred = false;
            }
        }
        if (BATCH < 64 && (walking || (DEFER && deferred))) {
            if constexpr (PARK) trace_park(T, pk);
            continue;
        }
        bool panic = false;
        Draws Dr{};
        if constexpr (!tier_full(TIER)) {  // (the mesh tier: the shading draws made here)
            if (T.found) {
                uint32_t ovf = 0;
                Dr.xi0 = rng.next(ovf);
                Dr.xi1 = rng.next(ovf);
                k_sincos_2pi(Dr.xi0, &Dr.sn, &Dr.cs);
            }
        }
#ifdef RT_DIAG
        {  // the round's shading classes (diagnostic build): one dependent load for the material
            uint32_t cls = 0;  // miss
            if (T.found) {
                const uint32_t k = ref_kind(T.hit.ref), i = ref_index(T.hit.ref);
                const int32_t m = k == K_SPHERE ? S.sphere_mat[i] : k == K_MSPHERE ? S.msph_mat[i]
                                : (k == K_QUAD || k == K_TRI) ? S.planar_mat[i] : k == K_MEDIUM ? S.media[i].phase_mat : -1;
                const int32_t mt = m >= 0 ? S.materials[m].type : -1;
                cls = mt == M_LAMBERTIAN ? 1u + (uint32_t)min(S.textures[S.materials[m].tex].type, 4)
                    : mt == M_METAL ? 6u : mt == M_DIELECTRIC ? 7u : mt == M_DIFFUSE_LIGHT ? 8u : mt == M_ISOTROPIC ? 9u : 10u;
            }
            const unsigned long long act = __ballot(true);
            uint32_t kinds = 0;
            const bool first = __lane_id() == (uint32_t)(__ffsll((long long)act) - 1);
            for (uint32_t c = 0; c <= 10u; ++c) {
                const unsigned long long bc = __ballot(cls == c);
                kinds += bc != 0ull ? 1u : 0u;
                if (first && bc) {
                    ++dg.cls_rounds[c];
                    dg.cls_lanes[c] += (unsigned long long)__popcll(bc);
                }
            }
            if (first) {
                ++dg.sh_rounds;
                dg.sh_lanes += (unsigned long long)__popcll(act);
                dg.sh_classes += kinds;
            }
        }
#endif
        bool end_path = shade<TIER>(S, ray, beta, L, rng, T.found, T.hit, panic, Dr);
        RT_DIAG_ONLY(dg.cyc_shade += __builtin_amdgcn_s_memtime() - t_b1;)
        if (panic) {
            ++n_panics;
            end_path = true;
        }
        if (!end_path) {
            ++vertex;
            if (vertex > F.max_depth) end_path = true;  // depth == 0 -> BLACK (camera.rs:282-284)
        }
        if (end_path) {
            if (isnan(L.x) || isnan(L.y) || isnan(L.z)) {  // camera.rs:323
                ++n_panics;
                L = d3(0, 0, 0);
            }
            in_path = false;
            ++s_j;
            if constexpr (ACC_LDS) {
                const D3 a = d3(pst[6 * RT_BLOCK], pst[7 * RT_BLOCK], pst[8 * RT_BLOCK]) + L;
                if (s_j == (sie >> 16)) {
                    double* dst = P->partial + (uint64_t)pit[BLK].y * 3;
                    dst[0] = a.x;
                    dst[1] = a.y;
                    dst[2] = a.z;
                    need = true;
                } else {
                    pst[6 * RT_BLOCK] = a.x, pst[7 * RT_BLOCK] = a.y, pst[8 * RT_BLOCK] = a.z;
                }
            } else {
                acc = acc + L;
                if (s_j == (sie >> 16)) {
                    double* dst = P->partial + (uint64_t)slot * 3;
                    dst[0] = acc.x;
                    dst[1] = acc.y;
                    dst[2] = acc.z;
                    need = true;
                }
            }
        }
    }
    }  // full tiers
    const uint32_t lane = __lane_id();
#ifdef RT_DIAG
    // wave-uniform cycle counts: lane 0 of each wave; lane counters: every lane
    if (lane == 0) {
        atomicAdd(&g_diag[0], dg.cyc_refill);
        atomicAdd(&g_diag[1], dg.cyc_trace);
        atomicAdd(&g_diag[2], dg.cyc_shade);
        atomicAdd(&g_diag[4], dg.main_iters);
        atomicAdd(&g_diag[13], dg.cyc_media);
        atomicAdd(&g_diag[21], dg.cyc_miss);
        atomicAdd(&g_diag[22], dg.cyc_queue);
        atomicAdd(&g_diag[23], dg.cyc_draws);
    }
    atomicAdd(&g_diag[3], dg.wave_trace_iters);  // counted by the first active lane of each wave iteration
    atomicAdd(&g_diag[5], dg.lane_trace_iters);
    atomicAdd(&g_diag[6], dg.node_visits);
    atomicAdd(&g_diag[7], dg.sphere_tests);
    atomicAdd(&g_diag[8], (unsigned long long)n_rays);
    atomicAdd(&g_diag[9], dg.load_cyc);
    atomicAdd(&g_diag[10], dg.loads);
    atomicAdd(&g_diag[11], dg.pops);
    atomicAdd(&g_diag[12], dg.pop_reads);
    atomicAdd(&g_diag[14], dg.big_tests);
    atomicAdd(&g_diag[15], dg.big_hits);
    atomicAdd(&g_diag[16], dg.u_steps);
    atomicAdd(&g_diag[17], dg.u_uniform);
    atomicAdd(&g_diag[18], dg.u_uniform_node);
    atomicAdd(&g_diag[19], dg.u_active);
    atomicAdd(&g_diag[20], dg.u_same);
    for (int k = 0; k < 4; ++k) {
        atomicAdd(&g_diag[24 + k], dg.u_top[k]);
        atomicAdd(&g_diag[28 + k], dg.l_top[k]);
    }
    atomicAdd(&g_diag[32], dg.l_node);
    // counted by the first active lane of a round, which need not be lane 0
    // (lanes whose walk has ended are masked off): flushed from every lane,
    // as g_diag[3]
    atomicAdd(&g_diag[33], dg.sh_rounds);
    atomicAdd(&g_diag[34], dg.sh_lanes);
    atomicAdd(&g_diag[35], dg.sh_classes);
    atomicAdd(&g_diag[36], dg.pure_rounds);
    atomicAdd(&g_diag[37], dg.pure_lanes);
    atomicAdd(&g_diag[38], dg.pure_max_pn);
    for (int k = 0; k < 11; ++k) {
        atomicAdd(&g_diag[39 + k], dg.cls_rounds[k]);
        atomicAdd(&g_diag[50 + k], dg.cls_lanes[k]);
    }
#endif
#ifdef RT_WAVE_TRACE
    hist.flush();
    if (trace_lane < RT_TRACE_LANES) {
        unsigned long long* t = g_lane_trace + (uint64_t)trace_lane * RT_TRACE_W;
        t[0] = trace_t0;
        t[1] = __builtin_amdgcn_s_memrealtime();
        t[2] = trace_items;
        t[3] = n_rays;
        t[4] = trace_tq;
        t[5] = trace_q;
        t[6] = trace_rays;
        t[7] = __builtin_amdgcn_s_memtime() - trace_c0;  // shader clocks over the lane's life
        t[8] = trace_steps;  // walk steps (wave iterations the lane walked in)
        t[9] = trace_steps_q;  // ... at its last refill
        t[10] = trace_atomic_ticks | ((unsigned long long)trace_atomics << 40);  // wave's atomic wait, count
        t[11] = trace_atomic_first;  // when the wave's first atomic returned (ticks after its start)
    }
#endif
    // one atomic per wave, not per lane: 262 144 adds to one address at the
    // end of every launch
    uint32_t rays_w = n_rays, panics_w = n_panics;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        rays_w += __shfl_xor(rays_w, o);
        panics_w += __shfl_xor(panics_w, o);
    }
    if (lane == 0) {
        atomicAdd(&P->stats[0], (unsigned long long)rays_w);
        if (panics_w) atomicAdd(&P->stats[1], (unsigned long long)panics_w);
    }
}


}  // namespace rtk

// ------------------------------------------------------------------ host launchers
// The product library compiles this file once per kernel tier (-DRT_TIER_ONLY=N,
// each with its own code-generation flags, raytracer-2025_amd/Makefile) plus
// once for the common part (-DRT_COMMON_ONLY); diagnostic / A-B builds compile
// it whole.
#define RT_TIER_ENTRY(N)                                                                                        \
    extern "C" hipError_t rtk_launch_path_##N(int grid, hipStream_t stream, const rtk::KParams* P) {          \
        hipLaunchKernelGGL(rtk::rt_path_kernel<N>, dim3(grid), dim3(N == 0 ? RT_BLOCK_BASIC : RT_BLOCK), 0, stream, P); \
        return hipGetLastError();                                                                            \
    }                                                                                                        \
    extern "C" int rtk_occupancy_##N(int* blocks_per_cu) {                                                   \
        return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rtk::rt_path_kernel<N>,            \
                                                                 N == 0 ? RT_BLOCK_BASIC : RT_BLOCK, 0);         \
    }
#if !defined(RT_COMMON_ONLY)
#if !defined(RT_TIER_ONLY) || RT_TIER_ONLY == 0
RT_TIER_ENTRY(0)
// the basic tier's wide variant (trees past NODE_LDS_CAP_BATCH nodes)
extern "C" hipError_t rtk_launch_path_0w(int grid, hipStream_t stream, const rtk::KParams* P) {
    hipLaunchKernelGGL((rtk::rt_path_kernel<0, true>), dim3(grid), dim3(RT_BLOCK_BASIC), 0, stream, P);
    return hipGetLastError();
}
#endif
#if !defined(RT_TIER_ONLY) || RT_TIER_ONLY == 1
RT_TIER_ENTRY(1)
#endif
#if !defined(RT_TIER_ONLY) || RT_TIER_ONLY == 2
RT_TIER_ENTRY(2)
#endif
#if !defined(RT_TIER_ONLY) || RT_TIER_ONLY == 3
RT_TIER_ENTRY(3)
#endif
#if !defined(RT_TIER_ONLY) || RT_TIER_ONLY == 4
RT_TIER_ENTRY(4)
#endif
#if defined(RT_WAVE_TRACE)
extern "C" int rt_lane_trace(unsigned long long* out, uint64_t n_lanes) {
    if (n_lanes > rtk::RT_TRACE_LANES) n_lanes = rtk::RT_TRACE_LANES;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rtk::g_lane_trace),
                                    n_lanes * rtk::RT_TRACE_W * sizeof(unsigned long long));
}
// the rays-begun histogram (RT_HIST_N buckets of 0.25 ms); out == NULL: zero it
extern "C" int rt_ray_hist(unsigned long long* out, uint64_t n) {
    static const unsigned long long zero[rtk::RT_HIST_N] = {};
    if (!out) return (int)hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_ray_hist), zero, sizeof zero);
    if (n > rtk::RT_HIST_N) n = rtk::RT_HIST_N;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rtk::g_ray_hist), n * sizeof(unsigned long long));
}
#endif
#if defined(RT_CHECK)
// check build: {refs past their arrays, 1 << 32 | the first bad ref} on the
// current device (rt_render.cpp wait())
extern "C" int rtk_check_read(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(rtk::g_check), sizeof(unsigned long long) * 2);
    if (reset) {
        unsigned long long z[2] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_check), z, sizeof z);
    }
    return (int)e;
}
#endif
#if defined(RT_DIAG)
// diagnostic build: the counters live with the (DIAG_TIER) kernel that adds to them
extern "C" int rt_diag_counters(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(rtk::g_diag), sizeof(unsigned long long) * rtk::RT_DIAG_N);
    if (reset) {
        unsigned long long z[rtk::RT_DIAG_N] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_diag), z, sizeof z);
    }
    return (int)e;
}
#endif
#endif

#if !defined(RT_TIER_ONLY)
extern "C" hipError_t rtk_launch_path_0(int, hipStream_t, const rtk::KParams*);
extern "C" hipError_t rtk_launch_path_0w(int, hipStream_t, const rtk::KParams*);
extern "C" hipError_t rtk_launch_path_1(int, hipStream_t, const rtk::KParams*);
extern "C" hipError_t rtk_launch_path_2(int, hipStream_t, const rtk::KParams*);
extern "C" hipError_t rtk_launch_path_3(int, hipStream_t, const rtk::KParams*);
extern "C" hipError_t rtk_launch_path_4(int, hipStream_t, const rtk::KParams*);
extern "C" int rtk_occupancy_0(int*);
extern "C" int rtk_occupancy_1(int*);
extern "C" int rtk_occupancy_2(int*);
extern "C" int rtk_occupancy_3(int*);
extern "C" int rtk_occupancy_4(int*);

namespace rtk {
// Color::to_rgb (utils/color.rs:14-36): optional ACES fit, clamp, then the sRGB
// OETF and f64 -> u8 (palette restated as in oracle/rt_oracle.cpp to_rgb;
// parity unpinned).  No contraction, so the arithmetic is the host's.
__device__ __forceinline__ uint8_t srgb_u8(double x, int toon) {
#pragma clang fp contract(off)
    if (toon == 1) {
        const double m = (x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14);
        x = m < 0.0 ? 0.0 : (m > 1.0 ? 1.0 : m);
    }
    const double sv = x <= 0.0031308 ? 12.92 * x : 1.055 * pow(x, 1.0 / 2.4) - 0.055;
    const double q = round(sv * 255.0);
    return (uint8_t)(q < 0.0 ? 0.0 : (q > 255.0 ? 255.0 : q));
}

// Sums the S stratum rows of each pixel in s_i order -- a row = its one
// whole-row sum (pixels below whole_px), or its `parts` part sums added in
// part order (the tail rows); the slots in queue order (Frame) -- *
// pixel_sample_scale, to linear f32 (camera.rs:193), and -- when srgb is
// given -- the pixel's to_rgb bytes from the f64 sum, as the reference
// converts its f64 color.  One lane per (pixel, channel), 21 pixels a wave:
// a pixel's sums are contiguous in the slot order, so a wave's load reads 21
// runs of 24 B and its next loads the same lines (one lane per pixel read 64
// lines per load, three times: 1.8 ms for C2's 3.8 GB against 0.8 at HBM rate).
constexpr uint32_t REDUCE_PX_PER_WAVE = 21;
__global__ void __launch_bounds__(256) rt_reduce_kernel(const double* __restrict__ partial, uint32_t p_lo, uint32_t npix,
                                                       uint32_t S, uint32_t parts, uint32_t whole_px, uint32_t parts2,
                                                       uint32_t fine_px, double scale, float* __restrict__ out,
                                                       uint8_t* __restrict__ srgb, int toon) {
    const uint32_t lane = threadIdx.x & 63u, wave = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
    if (lane >= 3u * REDUCE_PX_PER_WAVE) return;
    const uint32_t p = p_lo + wave * REDUCE_PX_PER_WAVE + lane / 3u, c = lane % 3u;  // pixels [p_lo, npix)
    if (p >= npix) return;
    // pixels [0, whole_px): one sum per stratum row; [whole_px, fine_px):
    // `parts`; [fine_px, npix): `parts2` (the fine rows)
    const bool whole = p < whole_px, fine = p >= fine_px;
    const uint32_t np = whole ? 1u : (fine ? parts2 : parts);
    const uint64_t part_first = (uint64_t)whole_px * S + (uint64_t)(fine_px - whole_px) * S * parts;
    const uint64_t first = whole ? (uint64_t)p * S
                         : fine  ? part_first + (uint64_t)(p - fine_px) * S * parts2
                                 : (uint64_t)whole_px * S + (uint64_t)(p - whole_px) * S * parts;
    const double* src = partial + first * 3 + c;
    double acc = 0.0;
    for (uint32_t k = 0; k < S; ++k) {
        const double* row = src + (uint64_t)k * np * 3;
        double rr = row[0];
        for (uint32_t j = 1; j < np; ++j) rr += row[j * 3];
        acc += rr;
    }
    const double v = acc * scale;
    out[(uint64_t)p * 3 + c] = (float)v;
    if (srgb) srgb[(uint64_t)p * 3 + c] = srgb_u8(v, toon);
}

// The same sums, staged through LDS: one wave per group of
// `pw` consecutive pixels of one region (whole rows: np = 1; tail rows: np =
// parts; fine rows: np = parts2), whose part sums are contiguous in slot
// order.  The wave copies the group's doubles into LDS with whole-line loads
// (each lane 8 B, 64 lanes 512 B a step), adds each (pixel, s_i, channel)'s
// parts in part order into the slot of part 0, then each (pixel, channel)'s
// S row sums in s_i order -- rt_reduce_kernel's additions in its order, so
// the same bits -- where that kernel's lanes read 21 pixels' 24-B runs per
// load and re-read each line from the cache several times.
constexpr uint32_t REDUCE_LDS_DOUBLES = 2048;  // 16 KiB per wave
__global__ void __launch_bounds__(64) rt_reduce_lds_kernel(const double* __restrict__ partial, uint32_t p_begin,
                                                          uint32_t p_end, uint64_t slot0, uint32_t S, uint32_t np,
                                                          uint32_t pw, double scale, float* __restrict__ out,
                                                          uint8_t* __restrict__ srgb, int toon) {
    __shared__ double buf[REDUCE_LDS_DOUBLES];
    const uint32_t lane = threadIdx.x;
    const uint32_t p0 = p_begin + blockIdx.x * pw;
    if (p0 >= p_end) return;
    const uint32_t n = min(pw, p_end - p0);
    const uint32_t row = np * 3u;          // doubles per stratum row
    const uint32_t per_px = S * row;       // doubles per pixel
    const uint32_t total = n * per_px;     // <= REDUCE_LDS_DOUBLES (host)
    const double* src = partial + (slot0 + (uint64_t)(p0 - p_begin) * S * np) * 3u;
    // (8 loads in flight per lane before their LDS stores)
    uint32_t i0 = lane;
    for (; i0 + 7u * 64u < total; i0 += 8u * 64u) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[i0 + u * 64u];
#pragma unroll
        for (int u = 0; u < 8; ++u) buf[i0 + u * 64u] = v[u];
    }
    for (; i0 < total; i0 += 64u) buf[i0] = src[i0];
    __syncthreads();
    if (np > 1u) {
        // (pixel, s_i, channel): its parts in order, into part 0's slot
        for (uint32_t i = lane; i < n * S * 3u; i += 64u) {
            const uint32_t c = i % 3u, ps = i / 3u;  // ps = pixel * S + s_i
            double* r = buf + ps * row + c;
            double rr = r[0];
            for (uint32_t j = 1; j < np; ++j) rr += r[j * 3u];
            r[0] = rr;
        }
        __syncthreads();
    }
    for (uint32_t i = lane; i < n * 3u; i += 64u) {
        const uint32_t c = i % 3u, px = i / 3u;
        const double* r = buf + px * per_px + c;
        double acc = 0.0;
        for (uint32_t k = 0; k < S; ++k) acc += r[k * row];
        const double v = acc * scale;
        const uint64_t o = (uint64_t)(p0 + px) * 3u + c;
        out[o] = (float)v;
        if (srgb) srgb[o] = srgb_u8(v, toon);
    }
}

// Math self-test (rt_math_selftest): the kernel's f64 functions (impl 0,
// rt_crmath.h) or ROCm's device libm (impl 1, ocml) on n arguments.
__global__ void __launch_bounds__(256) rt_math_kernel(int fn, int impl, const double* __restrict__ a,
                                                     const double* __restrict__ b, double* __restrict__ out,
                                                     uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i], y = b ? b[i] : 0.0;
    double r = 0.0, s = 0.0, c = 0.0;
    if (impl == 0) {
        switch (fn) {
            case 0: r = rtcr::sin(x); break;
            case 1: r = rtcr::cos(x); break;
            case 2: rtcr::sincos(x, &s, &c), r = s; break;
            case 3: rtcr::sincos(x, &s, &c), r = c; break;
            case 4: r = rtcr::log(x); break;
            case 5: r = rtcr::acos(x); break;
            case 6: r = rtcr::atan2(x, y); break;
            case 8: rtcr::sincos_2pi(x, &s, &c), r = s; break;
            case 9: rtcr::sincos_2pi(x, &s, &c), r = c; break;
            default: r = k_sqrt(x); break;  // the path's square root (RT_FAST_SQRT)
        }
    } else {
        switch (fn) {
            case 0: r = ::sin(x); break;
            case 1: r = ::cos(x); break;
            case 2: ::sincos(x, &s, &c), r = s; break;
            case 3: ::sincos(x, &s, &c), r = c; break;
            case 4: r = ::log(x); break;
            case 5: r = ::acos(x); break;
            case 6: r = ::atan2(x, y); break;
            case 8: ::sincos(2.0 * PI * x, &s, &c), r = s; break;
            case 9: ::sincos(2.0 * PI * x, &s, &c), r = c; break;
            default: r = ::sqrt(x); break;
        }
    }
    out[i] = r;
}

// to_rgb of a linear f32 framebuffer already on the device (e.g. the gathered
// multi-GPU frame).
__global__ void __launch_bounds__(256) rt_to_rgb_kernel(const float* __restrict__ lin, uint8_t* __restrict__ srgb,
                                                       uint64_t n, int toon) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) srgb[i] = srgb_u8((double)lin[i], toon);
}
// Frame row j of a gathered shard came from part j % parts, as that part's
// compact row j / parts.  One thread per float of the frame.
__global__ void __launch_bounds__(256) rt_deinterleave_kernel(const float* __restrict__ staging, uint64_t slice,
                                                              float* __restrict__ out, uint32_t rows, uint32_t W,
                                                              uint32_t parts) {
    const uint64_t row_floats = (uint64_t)W * 3;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)rows * row_floats) return;
    const uint32_t j = (uint32_t)(i / row_floats);
    const uint64_t x = i - (uint64_t)j * row_floats;
    out[i] = staging[(uint64_t)(j % parts) * slice + (uint64_t)(j / parts) * row_floats + x];
}
// The same for a gathered shard's to_rgb bytes.
__global__ void __launch_bounds__(256) rt_deinterleave_u8_kernel(const uint8_t* __restrict__ staging, uint64_t slice,
                                                                 uint8_t* __restrict__ out, uint32_t rows, uint32_t W,
                                                                 uint32_t parts) {
    const uint64_t row_bytes = (uint64_t)W * 3;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)rows * row_bytes) return;
    const uint32_t j = (uint32_t)(i / row_bytes);
    const uint64_t x = i - (uint64_t)j * row_bytes;
    out[i] = staging[(uint64_t)(j % parts) * slice + (uint64_t)(j / parts) * row_bytes + x];
}
}  // namespace rtk

extern "C" int rtk_tier_for(uint32_t features, uint32_t stack_need) {
    return rtk::plan::tier_for(features, stack_need, RT_BVH4 != 0, RT_STACK_BASIC);
}

extern "C" int rtk_basic_bvh4(void) { return RT_BVH4; }
extern "C" int rtk_planar_filter(void) { return RT_PLANAR_FILTER; }
extern "C" int rtk_block_threads(int tier) { return tier == rtk::TIER_BASIC ? RT_BLOCK_BASIC : RT_BLOCK; }
extern "C" int rtk_mesh_bvh4(void) { return RT_MESH_BVH4; }
extern "C" int rtk_full_bvh4(void) { return RT_FULL_BVH4; }

extern "C" uint32_t rtk_stack_entries(int tier) {
    return tier == rtk::TIER_BASIC ? RT_STACK_BASIC : RT_STACK_MAX;
}

static void fill_kparams(rtk::KParams& K, const rtk::SceneView* view, const rtk_frame_desc* fd, uint32_t* queue,
                         double* partial, unsigned long long* stats, int tier, int grid, void* stack_ovf,
                         uint32_t static_entries) {
    K.S = *view;
    rtk::Frame& F = K.F;
    F.W = fd->W;
    F.rows = fd->rows;
    F.row_offset = fd->row_offset;
    F.row_stride = fd->row_stride;
    F.S = fd->S;
    F.max_depth = fd->max_depth;
    F.key0 = (uint32_t)fd->seed;
    F.key1 = (uint32_t)(fd->seed >> 32);
    F.total_items = fd->W * fd->rows * fd->S;
    F.parts = fd->parts > 1 ? fd->parts : 1u;  // the host's rtk_row_parts: no part empty
    F.part_len = (fd->S + F.parts - 1) / F.parts;
    F.parts2 = fd->parts2 > 1 ? fd->parts2 : F.parts;
    F.part_len2 = (fd->S + F.parts2 - 1) / F.parts2;
    const uint32_t whole_rows = F.parts > 1 ? (fd->whole_rows < fd->rows ? fd->whole_rows : fd->rows) : fd->rows;
    // the shard's rows from fine_row on are the fine rows (none: rows)
    const uint32_t fine_row = fd->fine_row < whole_rows ? whole_rows : (fd->fine_row < fd->rows ? fd->fine_row : fd->rows);
    F.whole_items = fd->W * whole_rows * fd->S;
    F.fine_item0 = fd->W * fine_row * fd->S;
    F.fine_q0 = F.whole_items + (F.fine_item0 - F.whole_items) * F.parts;
    F.queue_total = F.fine_q0 + (F.total_items - F.fine_item0) * F.parts2;
    F.static_entries = static_entries;
    F.chunk_min = fd->chunk_min;
    F.chunk_min_whole = fd->chunk_min_whole;
    auto inv_up = [](uint32_t d) { return std::nextafter(1.0 / (double)d, 2.0); };
    F.inv_parts = inv_up(F.parts);
    F.inv_parts2 = inv_up(F.parts2);
    F.S_f = (float)F.S;
    F.part_len_f = (float)F.part_len;
    F.part_len2_f = (float)F.part_len2;
    F.inv_S_f = 1.0f / F.S_f;
    F.inv_part_len_f = 1.0f / F.part_len_f;
    F.inv_part_len2_f = 1.0f / F.part_len2_f;
    F.inv_S = inv_up(F.S);
    F.inv_W = inv_up(F.W);
    F.chunk_cap = fd->chunk_cap ? fd->chunk_cap : (tier == rtk::TIER_MESH ? RT_QUEUE_CHUNK_MESH : RT_QUEUE_CHUNK);
    F.inv_guide = 1.0f / (float)((uint64_t)grid * (rtk_block_threads(tier) / 64) * (fd->guide ? fd->guide : RT_QUEUE_GUIDE));
    F.defocus = fd->defocus;
    F.recip_sqrt_spp = fd->recip_sqrt_spp;
    F.pixel_sample_scale = fd->pixel_sample_scale;
    F.center = rtk::D3{fd->center[0], fd->center[1], fd->center[2]};
    F.pixel00 = rtk::D3{fd->pixel00[0], fd->pixel00[1], fd->pixel00[2]};
    F.du = rtk::D3{fd->du[0], fd->du[1], fd->du[2]};
    F.dv = rtk::D3{fd->dv[0], fd->dv[1], fd->dv[2]};
    F.disk_u = rtk::D3{fd->disk_u[0], fd->disk_u[1], fd->disk_u[2]};
    F.disk_v = rtk::D3{fd->disk_v[0], fd->disk_v[1], fd->disk_v[2]};
    K.queue = queue;
    K.partial = partial;
    K.stats = stats;
    K.stack_ovf = (RT_GLOBAL uint2*)stack_ovf;
}

static hipError_t launch_reduce(const rtk_frame_desc* fd, const rtk::Frame& F, double* partial, float* out,
                                uint8_t* srgb, int toon, hipStream_t stream) {
    const uint32_t npix = fd->W * fd->rows;
    // the three regions of the slot order (rtk::Frame): whole rows, tail
    // parts, fine parts; a region whose pixel does not fit the wave's LDS
    // (S x np x 24 B > 16 KiB, e.g. C5's 64 x 16 tail parts) takes the
    // direct kernel for that region
    const uint32_t whole_px = F.whole_items / fd->S, fine_px = F.fine_item0 / fd->S;
    const struct { uint32_t b, e, np; } reg[3] = {
        {0u, whole_px, 1u}, {whole_px, fine_px, F.parts}, {fine_px, npix, F.parts2}};
    uint64_t slot = 0;
    for (const auto& r : reg) {
        if (r.e > r.b) {
            const uint64_t dpp = (uint64_t)fd->S * r.np * 3u;  // doubles per pixel
            if (dpp <= rtk::REDUCE_LDS_DOUBLES) {
                const uint32_t pw = (uint32_t)std::min<uint64_t>(64u, rtk::REDUCE_LDS_DOUBLES / dpp);
                const uint32_t groups = (r.e - r.b + pw - 1u) / pw;
                hipLaunchKernelGGL(rtk::rt_reduce_lds_kernel, dim3(groups), dim3(64), 0, stream, partial, r.b,
                                   r.e, slot, fd->S, r.np, pw, fd->pixel_sample_scale, out, srgb, toon);
            } else {
                const uint32_t waves = (r.e - r.b + rtk::REDUCE_PX_PER_WAVE - 1) / rtk::REDUCE_PX_PER_WAVE;
                hipLaunchKernelGGL(rtk::rt_reduce_kernel, dim3((waves + 3) / 4), dim3(256), 0, stream, partial,
                                   r.b, r.e, fd->S, F.parts, whole_px, F.parts2, fine_px,
                                   fd->pixel_sample_scale, out, srgb, toon);
            }
        }
        slot += (uint64_t)(r.e - r.b) * fd->S * r.np;
    }
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_frame(const rtk::SceneView* view, const rtk_frame_desc* fd, uint32_t* queue,
                                       double* partial, unsigned long long* stats, float* out, uint8_t* srgb,
                                       int toon, hipStream_t stream, int tier, int grid, void* params_dev,
                                       void* stack_ovf) {
    rtk::KParams K;
    fill_kparams(K, view, fd, queue, partial, stats, tier, grid, stack_ovf,
                 (uint32_t)grid * (uint32_t)rtk_block_threads(tier));
    rtk::KParams* Pd = (rtk::KParams*)params_dev;
    hipError_t e = hipMemcpyAsync(Pd, &K, sizeof K, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(queue, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    if (fd->ev_start) (void)hipEventRecord((hipEvent_t)fd->ev_start, stream);
    // the basic tier: shading batches over trees that leave room for the
    // park area, whole-wave shading over the rest (rt_path_kernel WIDE)
    e = tier == rtk::TIER_BASIC  ? (view->n_nodes4 > rtk::NODE_LDS_CAP_BATCH ? rtk_launch_path_0w(grid, stream, Pd)
                                                                            : rtk_launch_path_0(grid, stream, Pd))
        : tier == rtk::TIER_MESH ? rtk_launch_path_1(grid, stream, Pd)
        : tier == rtk::TIER_FULL ? rtk_launch_path_2(grid, stream, Pd)
        : tier == rtk::TIER_FULL_FLAT ? rtk_launch_path_3(grid, stream, Pd)
                                      : rtk_launch_path_4(grid, stream, Pd);
    if (e != hipSuccess) return e;
    if (fd->ev_stop) (void)hipEventRecord((hipEvent_t)fd->ev_stop, stream);
    return launch_reduce(fd, K.F, partial, out, srgb, toon, stream);
}

extern "C" hipError_t rtk_launch_deinterleave(const float* staging, size_t slice, float* out, uint32_t rows, uint32_t W,
                                              uint32_t parts, hipStream_t stream) {
    const uint64_t n = (uint64_t)rows * W * 3;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rtk::rt_deinterleave_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, staging,
                       (uint64_t)slice, out, rows, W, parts);
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_deinterleave_u8(const uint8_t* staging, size_t slice, uint8_t* out, uint32_t rows,
                                                 uint32_t W, uint32_t parts, hipStream_t stream) {
    const uint64_t n = (uint64_t)rows * W * 3;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rtk::rt_deinterleave_u8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, staging,
                       (uint64_t)slice, out, rows, W, parts);
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_math(int fn, int impl, const double* a, const double* b, double* out, uint64_t n,
                                      hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rtk::rt_math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, fn, impl, a, b, out,
                       n);
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_to_rgb(const float* lin, uint8_t* srgb, uint64_t n, int toon, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rtk::rt_to_rgb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, lin, srgb, n, toon);
    return hipGetLastError();
}

// the frame plan (rt_plan.h), for rt_render.cpp
extern "C" uint32_t rtk_row_parts(uint32_t S, uint32_t part_samples) { return rtk::plan::row_parts(S, part_samples); }

extern "C" uint32_t rtk_tail_rows(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint64_t budget_bytes,
                                  uint32_t permille) {
    return rtk::plan::tail_rows(W, H, S, parts, budget_bytes, permille);
}

extern "C" void rtk_tail_split(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint32_t parts2,
                               uint64_t budget_bytes, uint32_t permille, uint32_t fine_permille, uint32_t* tail,
                               uint32_t* fine) {
    rtk::plan::tail_split(W, H, S, parts, parts2, budget_bytes, permille, fine_permille, tail, fine);
}

extern "C" uint32_t rtk_shard_whole_rows(uint32_t H, uint32_t tail, uint32_t row_offset, uint32_t row_stride,
                                         uint32_t rows) {
    return rtk::plan::shard_whole_rows(H, tail, row_offset, row_stride, rows);
}

extern "C" size_t rtk_params_bytes(void) { return sizeof(rtk::KParams); }


extern "C" int rtk_path_kernel_occupancy(int tier, int* blocks_per_cu) {
    return tier == rtk::TIER_BASIC  ? rtk_occupancy_0(blocks_per_cu)
         : tier == rtk::TIER_MESH ? rtk_occupancy_1(blocks_per_cu)
         : tier == rtk::TIER_FULL ? rtk_occupancy_2(blocks_per_cu)
         : tier == rtk::TIER_FULL_FLAT ? rtk_occupancy_3(blocks_per_cu)
                                       : rtk_occupancy_4(blocks_per_cu);
}
#endif  // !RT_TIER_ONLY
