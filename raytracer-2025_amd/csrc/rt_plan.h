// rt_plan.h -- the host-side frame plan of a launch: which kernel tier a
// flattened world takes, how a shard's stratum rows split into queue entries
// (whole rows, tail parts, fine parts).  Pure host arithmetic, shared by the
// product (the extern "C" rtk_* entry points in rt_kernel.hip, which
// rt_render.cpp calls) and the launcher's CPU test build
// (tests/cpp/hip_stub.cpp: the same plan under TSan, against a stub device
// layer).  No HIP calls here.
#pragma once
#include <stdint.h>

#include <algorithm>

#include "rt_layout.h"

namespace rtk {
namespace plan {

// The smallest kernel tier covering a flattened world's features (rt_kernel.h
// Tier).  bvh4: the basic tier walks 4-wide nodes, whose stack need the
// launcher checks itself (rt_render.cpp prepare_tier).
inline int tier_for(uint32_t features, uint32_t stack_need, bool bvh4, uint32_t stack_basic) {
    const uint32_t full = F_XFORM | F_MEDIUM | F_MSPHERE | F_LIGHTS | F_TEXFULL | F_MATFULL | F_NORMALMAP;
    if (features & F_GENERAL) return 4;          // TIER_FULL_GL
    if (features & full) return 2;               // TIER_FULL
    if (features & (F_PLANAR | F_REMAP)) return 1;  // TIER_MESH
    // the two-box tree's stack need; with 4-wide nodes the launcher decides on
    // the 4-wide tree's (shallower: a 1 500-sphere world needs 22 entries as
    // two-box nodes and fits the basic tier's 14 as 4-wide ones)
    if (!bvh4 && stack_need > stack_basic) return 1;
    return 0;  // TIER_BASIC
}

// Parts of about part_samples samples a stratum row of S samples splits into
// (none empty).
inline uint32_t row_parts(uint32_t S, uint32_t part_samples) {
    if (part_samples == 0 || S <= part_samples) return 1;
    const uint32_t parts = (S + part_samples - 1) / part_samples;
    const uint32_t len = (S + parts - 1) / parts;
    return (S + len - 1) / len;  // as many parts of that length as S takes: none empty
}

// The frame's last rows rendered in `parts` entries per stratum row: permille
// of H, within the part-sum budget and the queue's 2^32 entries.
inline uint32_t tail_rows(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint64_t budget_bytes,
                          uint32_t permille) {
    if (parts <= 1 || W == 0 || S == 0) return 0;
    uint64_t t = ((uint64_t)H * permille + 999) / 1000;
    if (t > H) t = H;
    // the tail's part sums beyond one sum per row within the budget
    const uint64_t extra_row = (uint64_t)W * S * (parts - 1);
    const uint64_t by_budget = budget_bytes / (extra_row * 3 * sizeof(double));
    if (t > by_budget) t = by_budget;
    // the queue of the whole frame below 2^32 entries
    const uint64_t whole = (uint64_t)W * H * S;
    if (whole >= 0xFFF00000ull) return 0;
    const uint64_t by_queue = (0xFFF00000ull - 1 - whole) / extra_row;
    if (t > by_queue) t = by_queue;
    return (uint32_t)t;
}

// The tail (rows in `parts` or `parts2` entries) and, inside it, the fine rows
// (the frame's last fine_permille rows, in parts2 entries), both counted from
// the frame's end; tail >= fine.
inline void tail_split(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint32_t parts2, uint64_t budget_bytes,
                       uint32_t permille, uint32_t fine_permille, uint32_t* tail, uint32_t* fine) {
    *tail = *fine = 0;
    if (parts <= 1 || W == 0 || S == 0) return;
    const uint64_t whole = (uint64_t)W * H * S;
    if (whole >= 0xFFF00000ull) return;
    uint64_t room = 0xFFF00000ull - 1 - whole;  // queue entries beyond one per stratum row
    uint64_t f = 0;
    if (parts2 > parts) {
        f = ((uint64_t)H * fine_permille + 999) / 1000;
        if (f > H) f = H;
        const uint64_t extra_f = (uint64_t)W * S * (parts2 - 1);
        f = std::min<uint64_t>(f, (budget_bytes / 2) / (extra_f * 3 * sizeof(double)));
        f = std::min<uint64_t>(f, (room / 2) / extra_f);
        budget_bytes -= f * extra_f * 3 * sizeof(double);
        room -= f * extra_f;
    }
    uint64_t tp = ((uint64_t)H * permille + 999) / 1000;  // the whole tail, fine rows included
    if (tp > H) tp = H;
    tp = tp > f ? tp - f : 0;  // its rows in `parts`
    const uint64_t extra_row = (uint64_t)W * S * (parts - 1);
    tp = std::min<uint64_t>(tp, budget_bytes / (extra_row * 3 * sizeof(double)));
    tp = std::min<uint64_t>(tp, room / extra_row);
    *fine = (uint32_t)f;
    *tail = (uint32_t)(f + tp);
}

// A shard's rows (row_offset + k * row_stride, `rows` of them) above a frame
// tail of `tail` rows: its first shard_whole_rows rows.
inline uint32_t shard_whole_rows(uint32_t H, uint32_t tail, uint32_t row_offset, uint32_t row_stride, uint32_t rows) {
    const uint32_t whole_img = tail < H ? H - tail : 0u;
    const uint32_t stride = row_stride ? row_stride : 1u;
    if (whole_img <= row_offset) return 0u;
    const uint32_t n = (whole_img - row_offset + stride - 1) / stride;
    return n < rows ? n : rows;
}

}  // namespace plan
}  // namespace rtk
