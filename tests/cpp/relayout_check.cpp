// tests/cpp/relayout_check.cpp -- rth::bvh4_relayout keeps a world's meaning:
// the re-laid-out tree (mode 1: sibling groups; mode 2: + triangle records in
// leaf order) is walked beside the build-order tree (mode 0) from the roots,
// and every slot must name the same kind, carry the same f32 box and reach a
// bit-identical primitive record (planar record, material, remap, area).
// Linked against librt_mi355x.so (host code only: no device needed).
//   relayout_check <terrain.obj>  ->  "<mode> <slots> <mismatches>" per mode
#include <cstdio>
#include <cstring>
#include <utility>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_scene.hpp"

using namespace rth;

static size_t compare(const HostWorld& A, const HostWorld& B, size_t& slots) {
    size_t bad = 0;
    std::vector<std::pair<uint32_t, uint32_t>> todo{{A.world_root, B.world_root}};
    while (!todo.empty()) {
        const auto [ra, rb] = todo.back();
        todo.pop_back();
        const uint32_t ka = rtk::ref_kind(ra), kb = rtk::ref_kind(rb);
        ++slots;
        if (ka != kb) {
            ++bad;
            continue;
        }
        const uint32_t ia = rtk::ref_index(ra), ib = rtk::ref_index(rb);
        if (ka == rtk::K_BVH) {
            if (ia >= A.nodes4.size() || ib >= B.nodes4.size()) {
                ++bad;
                continue;
            }
            const rtk::DNode4 &na = A.nodes4[ia], &nb = B.nodes4[ib];
            if (std::memcmp(na.lo, nb.lo, sizeof na.lo) || std::memcmp(na.hi, nb.hi, sizeof na.hi)) ++bad;
            for (int s = 0; s < 4; ++s)
                if (na.ref[s] != rtk::REF_NONE || nb.ref[s] != rtk::REF_NONE) todo.push_back({na.ref[s], nb.ref[s]});
        } else if (ka == rtk::K_TRI || ka == rtk::K_QUAD) {
            if (ia >= A.planars.size() || ib >= B.planars.size() ||
                std::memcmp(&A.planars[ia], &B.planars[ib], sizeof(rtk::DPlanar)) ||
                A.planar_mat[ia] != B.planar_mat[ib] || A.planar_remap[ia] != B.planar_remap[ib] ||
                A.planar_area[ia] != B.planar_area[ib])
                ++bad;
        } else if (ra != rb) {
            ++bad;
        }
    }
    return bad;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    rt_scene* s = rt_scene_create();
    const int32_t world = rt_hittables_new(s);
    const int32_t mesh = rt_wavefront_load(s, argv[1], 1);
    if (mesh < 0) {
        std::printf("load failed: %s\n", rt_last_error());
        return 1;
    }
    rt_hittables_add(s, world, mesh);
    const double c1[3] = {-0.9, 1.0, 0.6}, c2[3] = {1.1, 0.95, -0.3}, white[3] = {1, 1, 1};
    const int32_t m = rt_mat_lambertian(s, rt_tex_solid(s, white));
    rt_hittables_add(s, world, rt_sphere(s, c1, 0.45, m));
    rt_hittables_add(s, world, rt_sphere(s, c2, 0.4, m));
    HostWorld base;
    if (flatten(s, world, -1, -1, false, base) != RT_OK) return 1;
    bvh4_convert(base, 96, false);
    int rc = 0;
    for (int mode = 1; mode <= 2; ++mode) {
        HostWorld w;
        flatten(s, world, -1, -1, false, w);
        bvh4_convert(w, 96, false);
        bvh4_relayout(w, mode);
        size_t moved = 0;
        for (size_t k = 0; k < w.nodes4.size() && k < base.nodes4.size(); ++k)
            moved += std::memcmp(&w.nodes4[k], &base.nodes4[k], sizeof(rtk::DNode4)) != 0;
        size_t slots = 0;
        const size_t bad = compare(base, w, slots);
        std::printf("%d %zu %zu %zu\n", mode, slots, bad, moved);
        if (bad) rc = 1;
    }
    rt_scene_destroy(s);
    return rc;
}
