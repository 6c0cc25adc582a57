// rt_kernel.h -- interface between the host render driver (rt_render.cpp) and
// the gfx950 kernels (rt_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.h"

#define RT_BLOCK 256        // 4 waves of 64 (mesh and full tiers)
// Basic tier: one 1024-thread block per CU (16 waves, 4 per SIMD: the same
// 128-VGPR budget) so that one LDS copy of the world's 4-wide nodes serves
// the whole CU.  LDS: stack entries * 1024 * 4 B + the sphere
// queue (RT_PEND_CAP * 1024 * 2 B) + RT_NODE_LDS_BYTES of nodes <= 160 KiB.
#ifndef RT_BLOCK_BASIC
#define RT_BLOCK_BASIC 1024
#endif
// traversal-stack entries per lane; LDS = entries * block * 4 B
#ifndef RT_STACK_BASIC
#define RT_STACK_BASIC 18   // 72 KiB of the basic tier's 1024-lane block
#endif
#ifndef RT_NODE_LDS_BYTES
// basic tier: the world's 4-wide nodes in LDS, 658 of them: 160 KiB - 72 KiB
// of stack - 16 KiB of sphere queue, in 112-B nodes.  With the 18-entry stack
// sphere BVHs of up to about 1 200 spheres stay in the basic tier
// (sphere-count scaling)
#define RT_NODE_LDS_BYTES 73696
#endif
#ifndef RT_NODE_LDS_BATCH_BYTES
// basic tier with shading batches (trees of at most 365 nodes, C1 / C2: 241):
// the node copy shrinks by the 32-KiB park area (8 words per lane)
#define RT_NODE_LDS_BATCH_BYTES 40880
#endif
#ifndef RT_STACK_MESH
// mesh tier: 16 entries = 32 KiB in LDS beside the 8-KiB park area (the walk
// state of lanes whose walk carries over a shading batch: 8 words), 40 KiB
// per block, 4 blocks: the whole 160 KiB; deeper entries in a global
// overflow column
#define RT_STACK_MESH 16
#endif
#ifndef RT_STACK_FULL
#define RT_STACK_FULL 16    // full tiers, likewise
#endif
#ifndef RT_STACK_FLAT
#define RT_STACK_FLAT 4     // full-flat tier (lists only: C3 needs 4); deeper ones overflow
#endif
#define RT_STACK_MAX 96     // LDS + overflow entries (mesh and full tiers)
#ifndef RT_MEDIA_CAP
#define RT_MEDIA_CAP 2      // full tier: media a walk queues (in LDS, 16 B each) before testing them inline
#endif

namespace rtk {
// Kernel tiers: the launcher picks the smallest that covers the flattened world.
//  BASIC: spheres / lists / BVH, Lambertian / Metal / Dielectric / Empty,
//         solid / sky / checker textures, no lights (C1, C2);
//  MESH:  BASIC + quads / triangles + OBJ RemappedMaterial (C4);
//  FULL:  everything (transforms, media, moving spheres, lights, all materials
//         and textures: C3, C5).
//  FULL_FLAT: FULL for worlds without any BVH node (C3): the walk carries no
//         BVH code, which leaves the registers to the rest (fewer spills).
//  FULL_GL: FULL with general lights (Transforms, nested lists, moving
//         spheres in the lights tree); kept apart so that the light-tree
//         code does not weigh on the C3 / C5 tiers.
enum Tier : int { TIER_BASIC = 0, TIER_MESH = 1, TIER_FULL = 2, TIER_FULL_FLAT = 3, TIER_FULL_GL = 4 };
constexpr int N_TIERS = 5;
__host__ __device__ constexpr bool tier_full(int t) { return t >= TIER_FULL; }
// full tiers that walk BVH nodes
__host__ __device__ constexpr bool tier_full_bvh(int t) { return t == TIER_FULL || t == TIER_FULL_GL; }
// traversal-stack entries a lane keeps in LDS (deeper ones: global overflow column)
__host__ __device__ constexpr uint32_t lds_stack_entries(int t) {
    return t == TIER_BASIC ? RT_STACK_BASIC : t == TIER_MESH ? RT_STACK_MESH : tier_full_bvh(t) ? RT_STACK_FULL : RT_STACK_FLAT;
}
}  // namespace rtk

// Camera::initilize results (camera.rs:204-245) for one shard.
struct rtk_frame_desc {
    uint32_t W, rows, row_offset, row_stride;
    uint32_t S, max_depth;
    uint64_t seed;
    uint32_t defocus, pad;
    // the stratum rows of the shard's first whole_rows rows are one queue
    // entry each; every later row is `parts` entries of consecutive samples
    // (rtk::Frame; rtk_row_parts, rtk_tail_rows), summed in part order
    uint32_t parts;
    uint32_t chunk_min;  // smallest guided chunk of queue entries (0: what the wave needs)
    uint32_t whole_rows;
    uint32_t chunk_cap;  // most entries per queue atomic (0: the tier's RT_QUEUE_CHUNK[_MESH])
    uint32_t guide;      // guided chunks: work left / (waves x guide) (0: RT_QUEUE_GUIDE)
    uint32_t chunk_min_whole;  // smallest guided chunk while whole-row entries are left
    // the shard's rows from fine_row on (the frame's last rtk_tail_split
    // `fine` rows) go out in parts2 entries per stratum row
    uint32_t parts2, fine_row;

    double recip_sqrt_spp, pixel_sample_scale;
    double center[3], pixel00[3], du[3], dv[3], disk_u[3], disk_v[3];
    void* ev_start;  // hipEvent_t recorded around the path kernel (or NULL)
    void* ev_stop;
};

extern "C" int rtk_tier_for(uint32_t features, uint32_t stack_need);
extern "C" uint32_t rtk_stack_entries(int tier);
// 1 if the basic tier's kernel walks 4-wide BVH nodes (rth::bvh4_basic)
extern "C" int rtk_basic_bvh4(void);
// 1 if the mesh tier's kernel walks 4-wide BVH nodes with every child boxed
extern "C" int rtk_mesh_bvh4(void);
// 1 if the kernel runs the f32 quad / triangle pre-test (rt_planar_filter.h)
extern "C" int rtk_planar_filter(void);
extern "C" int rtk_full_bvh4(void);
extern "C" hipError_t rtk_launch_frame(const rtk::SceneView* view, const rtk_frame_desc* fd, uint32_t* queue,
                                       double* partial, unsigned long long* stats, float* out, uint8_t* srgb,
                                       int toon, hipStream_t stream, int tier, int grid, void* params_dev,
                                       void* stack_ovf);
// Queue entries per tail stratum row at S x S samples: parts of about
// part_samples samples (0: whole rows), none empty.
extern "C" uint32_t rtk_row_parts(uint32_t S, uint32_t part_samples);
// The tail of a W x H frame: its last image rows whose stratum rows go out in
// `parts` entries -- about permille / 1000 of H, fewer when the tail's extra
// part sums (parts - 1 per stratum row, 24 B each) would pass budget_bytes or
// the frame's queue 2^32 entries.  A function of the frame only, not of a
// shard, so every row shard and device count sums a row the same way; each
// shard's tail rows are its last rows, so every shard ends on short entries.
extern "C" uint32_t rtk_tail_rows(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint64_t budget_bytes,
                                  uint32_t permille);
// The rows of a shard (image rows row_offset + r * row_stride, r < rows) above
// The frame's tail and, within it, its fine rows: the last `fine` image rows
// (about fine_permille / 1000 of H, within half the budget and half the
// queue's room) go out in parts2 entries per stratum row, the `tail` - `fine`
// rows above them in `parts`; tail >= fine.  Like rtk_tail_rows a function
// of the frame only.
extern "C" void rtk_tail_split(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint32_t parts2,
                               uint64_t budget_bytes, uint32_t permille, uint32_t fine_permille, uint32_t* tail,
                               uint32_t* fine);
// a frame's tail of `tail` rows: its first rtk_shard_whole_rows rows; the rest
// are tail rows, each shard's last.
extern "C" uint32_t rtk_shard_whole_rows(uint32_t H, uint32_t tail, uint32_t row_offset, uint32_t row_stride,
                                         uint32_t rows);
// Re-interleaves a gathered frame: staging holds `parts` slices of `slice`
// floats, slice k = the compact rows k, k + parts, ... of the frame; out gets
// the frame's `rows` compact rows (rows x W x 3 f32).
extern "C" hipError_t rtk_launch_deinterleave(const float* staging, size_t slice, float* out, uint32_t rows, uint32_t W,
                                              uint32_t parts, hipStream_t stream);
extern "C" hipError_t rtk_launch_deinterleave_u8(const uint8_t* staging, size_t slice, uint8_t* out, uint32_t rows,
                                                 uint32_t W, uint32_t parts, hipStream_t stream);
extern "C" hipError_t rtk_launch_to_rgb(const float* lin, uint8_t* srgb, uint64_t n, int toon, hipStream_t stream);
extern "C" hipError_t rtk_launch_math(int fn, int impl, const double* a, const double* b, double* out, uint64_t n,
                                      hipStream_t stream);
// device bytes rtk_launch_frame needs at params_dev
extern "C" size_t rtk_params_bytes(void);
extern "C" int rtk_path_kernel_occupancy(int tier, int* blocks_per_cu);
// threads per block of a tier's path kernel
extern "C" int rtk_block_threads(int tier);
