// rt_kernel.h -- interface between the host render driver (rt_render.cpp) and
// the gfx950 kernels (rt_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.h"

#define RT_BLOCK 256  // 4 waves of 64
#define RT_STACK 32   // traversal-stack entries per lane (LDS: RT_STACK * RT_BLOCK * 4 B = 32 KiB per block)

// Camera::initilize results (camera.rs:204-245) for one shard.
struct rtk_frame_desc {
    uint32_t W, rows, row_offset, row_stride;
    uint32_t S, max_depth;
    uint64_t seed;
    uint32_t defocus, pad;
    double recip_sqrt_spp, pixel_sample_scale;
    double center[3], pixel00[3], du[3], dv[3], disk_u[3], disk_v[3];
    void* ev_start;  // hipEvent_t recorded around the path kernel (or NULL)
    void* ev_stop;
};

extern "C" hipError_t rtk_launch_frame(const rtk::SceneView* view, const rtk_frame_desc* fd, uint32_t* queue,
                                       double* partial, unsigned long long* stats, float* out, hipStream_t stream,
                                       int grid);
extern "C" int rtk_path_kernel_occupancy(int* blocks_per_cu);
