// rt_scene.cpp -- builder half of the C ABI (include/rt_mi355x.h) and the
// world flattener.  Host code only; the device half is rt_render.hip.
#include "rt_kernel.h"
#include "rt_image.hpp"
#include "rt_scene.hpp"

#include <algorithm>
#include <cstring>
#include <exception>
#include <functional>
#include <limits>
#include <system_error>
#include <thread>
#include <unordered_map>

#include "../../include/rt_mi355x.h"

#ifndef RT_EXPAND_LEAF_LISTS
#define RT_EXPAND_LEAF_LISTS 1  // lists of primitives under a BVH become BVH leaves (Flattener::collect_leaves)
#endif

namespace rth {

static thread_local std::string g_error;
int32_t set_error(int32_t code, const std::string& msg) {
    g_error = msg;
    return code;
}

static const double INF = std::numeric_limits<double>::infinity();
// rt_world_selftest: this thread's flattens build their BVHs serially
static thread_local bool g_serial_build = false;

// aabb.rs:43-51 pad_to_minimums, interval.rs:28-34 expand, 44-46 size
static Iv pad(Iv t) {
    const double DELTA = 0.0001;
    double size = std::fmax(t.hi - t.lo, 0.0);
    if (size < DELTA) {
        double p = DELTA / 2.0;
        return Iv{t.lo - p, t.hi + p};
    }
    return t;
}
Box3 Box3::empty() {
    Box3 b;
    for (auto& i : b.a) i = Iv{INF, -INF};
    return b;
}
Box3 Box3::from_points(V3 p, V3 q) {
    Box3 b;
    for (int k = 0; k < 3; ++k) b.a[k] = pad(Iv{std::fmin(p[k], q[k]), std::fmax(p[k], q[k])});
    return b;
}
Box3 Box3::unite(const Box3& o) const {
    Box3 b;
    for (int k = 0; k < 3; ++k) b.a[k] = Iv{std::fmin(a[k].lo, o.a[k].lo), std::fmax(a[k].hi, o.a[k].hi)};
    return b;
}
int Box3::longest_axis() const {
    double lx = std::fmax(a[0].hi - a[0].lo, 0.0), ly = std::fmax(a[1].hi - a[1].lo, 0.0),
           lz = std::fmax(a[2].hi - a[2].lo, 0.0);
    if (lx > ly) return lx > lz ? 0 : 2;
    return ly > lz ? 1 : 2;
}
Quat Quat::operator*(const Quat& r) const {
    return Quat{w * r.w - x * r.x - y * r.y - z * r.z, w * r.x + x * r.w + y * r.z - z * r.y,
                w * r.y - x * r.z + y * r.w + z * r.x, w * r.z + x * r.y - y * r.x + z * r.w};
}
V3 Quat::rotate(V3 v) const {
    Quat p{0.0, v.x, v.y, v.z};
    Quat res = (*this * p) * conj();
    return V3(res.x, res.y, res.z);
}

// total_cmp (f64::total_cmp) used by box_compare, bvh.rs:48-54
static bool total_less(double a, double b) {
    int64_t ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    ia ^= (int64_t)(((uint64_t)(ia >> 63)) >> 1);
    ib ^= (int64_t)(((uint64_t)(ib >> 63)) >> 1);
    return ia < ib;
}

// bvh.rs:16-46, restated over a compact (box, id) array and built in
// parallel, node for node the tree and the object ids of bvh_from_vec_serial
// below (kept as the statement of the recursion): a call makes one node, its
// left subtree's nodes first, then its right subtree's, then itself (post
// order), so the ids of a subtree of n objects are a block of
// bvh_node_count(n) ids fixed by n alone and both halves can be filled at
// once.  1M-triangle OBJ models: ~3 s per model serial, mostly cache misses
// of the comparator reading each object's box.
namespace {
struct BvhItem {
    Box3 box;
    int id;
};
size_t bvh_node_count(size_t n) {
    // nodes for n objects: one per call, a call on <= 2 objects is a leaf
    // node; sizes at one depth are floor / ceil of one quotient, so few
    // distinct n come up
    static thread_local std::unordered_map<size_t, size_t> memo;
    if (n <= 2) return 1;
    auto it = memo.find(n);
    if (it != memo.end()) return it->second;
    const size_t c = 1 + bvh_node_count(n / 2) + bvh_node_count(n - n / 2);
    memo.emplace(n, c);
    return c;
}
void bvh_build(rt_scene* s, BvhItem* it, size_t len, size_t base, int par) {
    Box3 bbox = Box3::empty();
    for (size_t i = 0; i < len; ++i) bbox = bbox.unite(it[i].box);  // the same order as the serial loop
    const int axis = bbox.longest_axis();
    Obj node;
    node.kind = O_BVH;
    node.hidden = true;
    node.bbox = bbox;
    size_t self = base;
    if (len == 1) {
        node.left = it[0].id;
    } else if (len == 2) {
        node.left = it[0].id;
        node.right = it[1].id;
    } else {
        // the stable sort on (key, position) pairs, then one gather: a third
        // of the bytes a sort of the 56-B items moves
        {
            std::vector<std::pair<int64_t, uint32_t>> kp(len);
            for (size_t i = 0; i < len; ++i) {
                int64_t k;
                std::memcpy(&k, &it[i].box.a[axis].lo, 8);
                k ^= (int64_t)(((uint64_t)(k >> 63)) >> 1);  // total_less's order as integers
                kp[i] = {k, (uint32_t)i};
            }
            std::stable_sort(kp.begin(), kp.end(),
                             [](const std::pair<int64_t, uint32_t>& a, const std::pair<int64_t, uint32_t>& b) {
                                 return a.first < b.first;
                             });
            std::vector<BvhItem> tmp(it, it + len);
            for (size_t i = 0; i < len; ++i) it[i] = tmp[kp[i].second];
        }
        const size_t mid = len / 2, nl = bvh_node_count(mid), nr = bvh_node_count(len - mid);
        node.left = (int)(base + nl - 1);  // a subtree's root is its last node
        node.right = (int)(base + nl + nr - 1);
        std::thread t;
        std::exception_ptr err;
        if (par > 0 && len >= 16384) {
            try {
                t = std::thread([&] {
                    try {
                        bvh_build(s, it, mid, base, par - 1);
                    } catch (...) {
                        err = std::current_exception();
                    }
                });
            } catch (const std::system_error&) {  // no thread to be had: this one builds both
            }
        }
        if (t.joinable()) {
            std::exception_ptr err_r;
            try {
                bvh_build(s, it + mid, len - mid, base + nl, par - 1);
            } catch (...) {
                err_r = std::current_exception();
            }
            t.join();  // before anything leaves this frame
            if (err || err_r) std::rethrow_exception(err ? err : err_r);
        } else {
            bvh_build(s, it, mid, base, 0);
            bvh_build(s, it + mid, len - mid, base + nl, 0);
        }
        self = base + nl + nr;
    }
    s->objs[self] = std::move(node);
}
}  // namespace
static int bvh_from_vec(rt_scene* s, const std::vector<int>& objects) {
    std::vector<BvhItem> items(objects.size());
    for (size_t i = 0; i < objects.size(); ++i) items[i] = BvhItem{s->objs[objects[i]].bbox, objects[i]};
    const size_t base = s->objs.size(), n = bvh_node_count(objects.size());
    s->objs.resize(base + n);
    try {
        bvh_build(s, items.data(), items.size(), base, 4);  // up to 16 threads
    } catch (...) {
        s->objs.resize(base);  // no half-built nodes left behind
        throw;
    }
    return (int)(base + n - 1);
}

// bvh.rs:16-46 -- returns the object id of the new BVH node (the serial
// recursion; tests/test_tiers_cpu.py checks bvh_from_vec against it)
int bvh_from_vec_serial(rt_scene* s, std::vector<int> objects) {
    Box3 bbox = Box3::empty();
    for (int o : objects) bbox = bbox.unite(s->objs[o].bbox);
    int axis = bbox.longest_axis();
    Obj node;
    node.kind = O_BVH;
    node.hidden = true;
    node.bbox = bbox;
    size_t len = objects.size();
    if (len == 1) {
        node.left = objects[0];
    } else if (len == 2) {
        node.left = objects[0];
        node.right = objects[1];
    } else {
        std::stable_sort(objects.begin(), objects.end(), [&](int a, int b) {
            return total_less(s->objs[a].bbox.a[axis].lo, s->objs[b].bbox.a[axis].lo);
        });
        size_t mid = len / 2;
        std::vector<int> lv(objects.begin(), objects.begin() + mid), rv(objects.begin() + mid, objects.end());
        node.left = bvh_from_vec_serial(s, std::move(lv));
        node.right = bvh_from_vec_serial(s, std::move(rv));
    }
    s->objs.push_back(node);
    return (int)s->objs.size() - 1;
}

// ------------------------------------------------------------------ flatten
namespace {

float round_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}
float round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
}
// The f32 pre-test record of a quad / triangle (rt_planar_filter.h): n, D,
// Q rounded to nearest, a = v x w and b = w x u from the f64 vectors, and
// the error-bound magnitudes rounded up.
rtk::PlanarF planar_f(const Obj& o) {
    rtk::PlanarF F{};
    const V3 a = cross(o.v, o.w), b = cross(o.w, o.u);
    auto l1 = [](V3 x) { return std::fabs(x.x) + std::fabs(x.y) + std::fabs(x.z); };
    F.n[0] = (float)o.normal.x, F.n[1] = (float)o.normal.y, F.n[2] = (float)o.normal.z, F.D = (float)o.D;
    F.q[0] = (float)o.anchor.x, F.q[1] = (float)o.anchor.y, F.q[2] = (float)o.anchor.z;
    F.g = round_up(8.0 * l1(o.anchor) + 2.0 * std::fabs(o.D));
    F.a[0] = (float)a.x, F.a[1] = (float)a.y, F.a[2] = (float)a.z, F.sa = round_up(l1(a));
    F.b[0] = (float)b.x, F.b[1] = (float)b.y, F.b[2] = (float)b.z, F.sb = round_up(l1(b));
    return F;
}

double half_area(const Box3& b) {
    double dx = std::fmax(b.a[0].hi - b.a[0].lo, 0.0), dy = std::fmax(b.a[1].hi - b.a[1].lo, 0.0),
           dz = std::fmax(b.a[2].hi - b.a[2].lo, 0.0);
    return dx * dy + dy * dz + dz * dx;
}

constexpr int MAX_XF_NESTING = 2;  // rt_kernel.hip MAX_XF

struct Flattener {
    const rt_scene* s;
    HostWorld& out;
    bool reference_bvh;
    std::unordered_map<int, std::pair<uint32_t, uint32_t>> memo;  // obj -> (ref, stack need)
    // The lights list keeps its run even with one object: Hittables::random
    // spends a draw on `choose` regardless (hits.rs:69-75).
    bool no_collapse = false;
    std::unordered_map<int, Box3> tight_memo;
    std::string err;
    int32_t code = RT_OK;
    static constexpr uint32_t REF_NONE_ = rtk::REF_NONE;

    uint32_t fail(int32_t c, const std::string& m) {
        if (code == RT_OK) {
            code = c;
            err = m;
        }
        return REF_NONE_;
    }

    // Tight box of everything an object can report a hit in.  The reference
    // boxes (kept in Obj::bbox for the reference topology) include the origin
    // for Hittables built from Hittables::default() (hits.rs:9, aabb.rs:9); the
    // SAH build uses these tight ones instead.
    Box3 tight(int id) {
        const Obj& o = s->objs[id];
        // primitives: their own box; a BVH's inner nodes are reached only
        // through their parent (objects are moved, never shared): neither is
        // worth a memo entry (1M-triangle meshes: two million of them)
        if (o.kind != O_LIST && o.kind != O_BVH && o.kind != O_XFORM && o.kind != O_MEDIUM) return o.bbox;
        if (o.kind == O_BVH && o.hidden) {
            Box3 b = Box3::empty();
            if (o.left >= 0) b = b.unite(tight(o.left));
            if (o.right >= 0) b = b.unite(tight(o.right));
            return b;
        }
        auto it = tight_memo.find(id);
        if (it != tight_memo.end()) return it->second;
        Box3 b = o.bbox;
        switch (o.kind) {
            case O_LIST:
                b = Box3::empty();
                for (int c : o.children) b = b.unite(tight(c));
                break;
            case O_BVH:
                b = Box3::empty();
                if (o.left >= 0) b = b.unite(tight(o.left));
                if (o.right >= 0) b = b.unite(tight(o.right));
                break;
            case O_XFORM: {
                Box3 cb = tight(o.child);
                const double INFD = std::numeric_limits<double>::infinity();
                V3 mn(INFD, INFD, INFD), mx(-INFD, -INFD, -INFD);
                for (int i = 0; i < 8; ++i) {
                    V3 p(cb.a[0].lo, cb.a[1].lo, cb.a[2].lo);
                    if (i & 4) p.x = cb.a[0].hi;
                    if (i & 2) p.y = cb.a[1].hi;
                    if (i & 1) p.z = cb.a[2].hi;
                    V3 t = o.q.rotate(p * o.scale) + o.offset;
                    mn = V3(std::fmin(mn.x, t.x), std::fmin(mn.y, t.y), std::fmin(mn.z, t.z));
                    mx = V3(std::fmax(mx.x, t.x), std::fmax(mx.y, t.y), std::fmax(mx.z, t.z));
                }
                b = Box3::from_points(mn, mx);
                break;
            }
            case O_MEDIUM: b = tight(o.child); break;
            default: break;
        }
        tight_memo[id] = b;
        return b;
    }

    static rtk::DBoxF boxf(const Box3& b) {
        rtk::DBoxF r{};
        for (int k = 0; k < 3; ++k) {
            r.lo[k] = round_down(b.a[k].lo);
            r.hi[k] = round_up(b.a[k].hi);
        }
        return r;
    }
    void set_box(rtk::DNode& n, int which, const Box3& b) {
        auto& bx = n.slot[which].box;
        for (int k = 0; k < 3; ++k) {
            bx.lo[k] = round_down(b.a[k].lo);
            bx.hi[k] = round_up(b.a[k].hi);
        }
        bx.pad[0] = bx.pad[1] = 0;
    }
    // child slot: the sphere itself for a sphere child, else its box
    void set_child(rtk::DNode& n, int which, uint32_t ref, const Box3& b) {
        if (rtk::ref_kind(ref) == rtk::K_SPHERE)
        {
            const double4 sp = out.spheres[rtk::ref_index(ref)];
            n.slot[which].sphere[0] = sp.x;
            n.slot[which].sphere[1] = sp.y;
            n.slot[which].sphere[2] = sp.z;
            n.slot[which].sphere[3] = sp.w;
        }
        else
            set_box(n, which, b);
    }

    struct Item {
        uint32_t ref, need;
        Box3 box;
        double c[3];
    };

    // Nodes of a subtree under construction: refs to nodes made by the same
    // build are relative to `n` (flag `local`), every other ref (the items'
    // own: primitives, nested BVHs already in out.nodes) is final.
    struct NodeBuf {
        std::vector<rtk::DNode> n;
        std::vector<uint8_t> local;  // bit 0: c0 is a node of this build, bit 1: c1
        // appends `sub` (its local refs rebased by where it lands); returns that offset
        uint32_t splice(const NodeBuf& sub) {
            const uint32_t off = (uint32_t)n.size();
            n.insert(n.end(), sub.n.begin(), sub.n.end());
            local.insert(local.end(), sub.local.begin(), sub.local.end());
            for (size_t k = off; k < n.size(); ++k) {
                if (local[k] & 1u) n[k].c0 += off;  // (index field only: no carry into the kind)
                if (local[k] & 2u) n[k].c1 += off;
            }
            return off;
        }
    };
    struct Built {
        uint32_t ref, need;
        bool local;
    };
    // Binned SAH (32 bins x 3 axes) over items[b, e); leaves hold one object,
    // the parent carries each child's box.  Returns (ref, need).  Nodes are
    // numbered in preorder (a node, its left subtree, its right subtree); the
    // two halves of a large node are built at once into their own buffers and
    // spliced in that order, so the tree and its numbering do not depend on
    // the threads (1M-triangle OBJ models: ~1.3 s per model serial).
    std::pair<uint32_t, uint32_t> sah(std::vector<Item>& it, size_t b, size_t e) {
        NodeBuf nb;
        const Built r = sah_build(it, b, e, nb, g_serial_build ? 0 : 4);  // up to 16 threads
        const uint32_t off = (uint32_t)out.nodes.size();
        out.nodes.insert(out.nodes.end(), nb.n.begin(), nb.n.end());
        for (size_t k = 0; k < nb.n.size(); ++k) {
            if (nb.local[k] & 1u) out.nodes[off + k].c0 += off;
            if (nb.local[k] & 2u) out.nodes[off + k].c1 += off;
        }
        return {r.local ? r.ref + off : r.ref, r.need};
    }
    Built sah_build(std::vector<Item>& it, size_t b, size_t e, NodeBuf& nb, int par) {
        if (e - b == 1) return {it[b].ref, it[b].need, false};
        size_t mid = b + (e - b) / 2;
        double cmin[3], cmax[3];
        for (int k = 0; k < 3; ++k) {
            cmin[k] = std::numeric_limits<double>::infinity();
            cmax[k] = -cmin[k];
        }
        for (size_t i = b; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                cmin[k] = std::fmin(cmin[k], it[i].c[k]);
                cmax[k] = std::fmax(cmax[k], it[i].c[k]);
            }
        constexpr int NB = 32;
        double best = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_bin = 0;
        for (int k = 0; k < 3; ++k) {
            double ext = cmax[k] - cmin[k];
            if (!(ext > 0)) continue;
            Box3 bb[NB];
            size_t cnt[NB] = {};
            for (auto& x : bb) x = Box3::empty();
            for (size_t i = b; i < e; ++i) {
                int bin = (int)((it[i].c[k] - cmin[k]) / ext * NB);
                bin = bin < 0 ? 0 : (bin >= NB ? NB - 1 : bin);
                bb[bin] = bb[bin].unite(it[i].box);
                ++cnt[bin];
            }
            double right_area[NB];
            size_t right_cnt[NB];
            Box3 acc = Box3::empty();
            size_t n = 0;
            for (int i = NB - 1; i > 0; --i) {
                acc = acc.unite(bb[i]);
                n += cnt[i];
                right_area[i] = half_area(acc);
                right_cnt[i] = n;
            }
            acc = Box3::empty();
            n = 0;
            for (int i = 0; i < NB - 1; ++i) {
                acc = acc.unite(bb[i]);
                n += cnt[i];
                if (n == 0 || right_cnt[i + 1] == 0) continue;
                double cost = half_area(acc) * (double)n + right_area[i + 1] * (double)right_cnt[i + 1];
                if (cost < best) {
                    best = cost;
                    best_axis = k;
                    best_bin = i;
                }
            }
        }
        if (best_axis >= 0) {
            const int k = best_axis;
            const double ext = cmax[k] - cmin[k];
            auto pivot = std::stable_partition(it.begin() + b, it.begin() + e, [&](const Item& x) {
                int bin = (int)((x.c[k] - cmin[k]) / ext * NB);
                bin = bin < 0 ? 0 : (bin >= NB ? NB - 1 : bin);
                return bin <= best_bin;
            });
            mid = (size_t)(pivot - it.begin());
            if (mid == b || mid == e) mid = b + (e - b) / 2;
        }
        const uint32_t idx = (uint32_t)nb.n.size();
        nb.n.emplace_back();
        nb.local.push_back(0);
        Built L, R;
        NodeBuf lb, rb;
        std::thread t;
        std::exception_ptr err;
        if (par > 0 && e - b >= 32768) {
            try {
                t = std::thread([&] {
                    try {
                        L = sah_build(it, b, mid, lb, par - 1);
                    } catch (...) {
                        err = std::current_exception();
                    }
                });
            } catch (const std::system_error&) {  // no thread to be had: this one builds both
            }
        }
        if (t.joinable()) {
            std::exception_ptr err_r;
            try {
                R = sah_build(it, mid, e, rb, par - 1);
            } catch (...) {
                err_r = std::current_exception();
            }
            t.join();  // before anything leaves this frame
            if (err || err_r) std::rethrow_exception(err ? err : err_r);
            const uint32_t offl = nb.splice(lb);
            if (L.local) L.ref += offl;
            const uint32_t offr = nb.splice(rb);
            if (R.local) R.ref += offr;
        } else {
            L = sah_build(it, b, mid, nb, 0);
            R = sah_build(it, mid, e, nb, 0);
        }
        Box3 bl = Box3::empty(), br = Box3::empty();
        for (size_t i = b; i < mid; ++i) bl = bl.unite(it[i].box);
        for (size_t i = mid; i < e; ++i) br = br.unite(it[i].box);
        rtk::DNode& n = nb.n[idx];
        set_child(n, 0, L.ref, bl);
        set_child(n, 1, R.ref, br);
        n.c0 = L.ref;
        n.c1 = R.ref;
        nb.local[idx] = (L.local ? 1u : 0u) | (R.local ? 2u : 0u);
        // near-first: the far child waits on the stack while the near one is walked
        return {rtk::make_ref(rtk::K_BVH, idx), 1 + std::max(L.need, R.need), true};
    }

    // Reference topology (bvh.rs:16-46) in the two-box node format.
    std::pair<uint32_t, uint32_t> ref_bvh(int id, bool in_boundary, int xf_depth, bool root) {
        const Obj& o = s->objs[id];
        if (!root && (o.kind != O_BVH || !o.hidden)) return emit(id, in_boundary, xf_depth);
        uint32_t idx = (uint32_t)out.nodes.size();
        out.nodes.emplace_back();
        auto L = ref_bvh(o.left, in_boundary, xf_depth, false);
        std::pair<uint32_t, uint32_t> R{REF_NONE_, 0};
        if (o.right >= 0) R = ref_bvh(o.right, in_boundary, xf_depth, false);
        rtk::DNode& n = out.nodes[idx];
        set_child(n, 0, L.first, s->objs[o.left].bbox);
        if (o.right >= 0) set_child(n, 1, R.first, s->objs[o.right].bbox);
        else set_box(n, 1, Box3::empty());
        n.c0 = L.first;
        n.c1 = R.first;
        return {rtk::make_ref(rtk::K_BVH, idx), 1 + std::max(L.second, R.second)};
    }

    // an object that is a BVH or a list holding one (through nested lists)
    bool holds_bvh(int id, int depth) const {
        const Obj& o = s->objs[id];
        if (o.kind == O_BVH) return true;
        if (o.kind != O_LIST || depth >= 8) return false;
        return std::any_of(o.children.begin(), o.children.end(), [&](int c) { return holds_bvh(c, depth + 1); });
    }
    // the elements of a list with nested lists opened, in order (the min of
    // hits.rs:34-46 over nested lists is the min over their elements)
    void list_elements(int id, std::vector<int>& out_ids, int depth) const {
        const Obj& o = s->objs[id];
        if (o.kind == O_LIST && depth < 8) {  // an empty list adds nothing (nothing to hit)
            for (int c : o.children) list_elements(c, out_ids, depth + 1);
        } else {
            out_ids.push_back(id);
        }
    }
    // A list of plain primitives under a BVH (C5's ground boxes: six quads
    // each) becomes leaves of that BVH too: the min over its children
    // (hits.rs:34-46) is the BVH's closest hit over them (up to exact t ties,
    // as for every rebuilt BVH), and the walk culls faces by their boxes
    // instead of testing all of them.
    static bool primitive(int kind) { return kind == O_SPHERE || kind == O_QUAD || kind == O_TRI || kind == O_MSPHERE; }
    void collect_leaves(int id, std::vector<int>& leaves) {
        const Obj& o = s->objs[id];
        if (o.kind == O_BVH && (o.hidden || leaves.empty())) {
            collect_leaves(o.left, leaves);
            if (o.right >= 0) collect_leaves(o.right, leaves);
        } else if (RT_EXPAND_LEAF_LISTS && o.kind == O_LIST && !o.children.empty() &&
                   std::all_of(o.children.begin(), o.children.end(),
                               [&](int c) { return primitive(s->objs[c].kind); })) {
            for (int c : o.children) leaves.push_back(c);
        } else {
            leaves.push_back(id);
        }
    }

    // A medium boundary that is one sphere, one quad / triangle or a flat list
    // of at most RT_MED_PLANAR_MAX of them stored consecutively (build_box),
    // inside at most two Transforms, is marked for the kernel's one-pass
    // boundary test; anything else keeps planar_n = bsphere = 0.
    void planar_boundary(uint32_t ref, rtk::DMedium& m) const {
        auto planar = [](uint32_t r) { return rtk::ref_kind(r) == rtk::K_QUAD || rtk::ref_kind(r) == rtk::K_TRI; };
        m.planar_n = m.planar_first = m.tri_mask = m.bxf_n = m.bsphere = 0;
        m.bxf[0] = m.bxf[1] = 0;
        uint32_t nxf = 0;
        while (rtk::ref_kind(ref) == rtk::K_XFORM) {
            if (nxf == 2) return;
            m.bxf[nxf++] = rtk::ref_index(ref);
            ref = out.xforms[rtk::ref_index(ref)].child;
        }
        if (rtk::ref_kind(ref) == rtk::K_SPHERE) {
            m.bsphere = rtk::ref_index(ref) + 1;
            m.bxf_n = nxf;
            return;
        }
        std::vector<uint32_t> el;
        if (planar(ref)) {
            el.push_back(ref);
        } else if (rtk::ref_kind(ref) == rtk::K_LIST) {
            for (uint32_t li = rtk::ref_index(ref); out.list_children[li] != REF_NONE_; ++li) {
                if (!planar(out.list_children[li]) || el.size() >= rtk::RT_MED_PLANAR_MAX) return;
                el.push_back(out.list_children[li]);
            }
        }
        if (el.empty()) return;
        for (size_t k = 0; k < el.size(); ++k) {
            if (rtk::ref_index(el[k]) != rtk::ref_index(el[0]) + k) return;
            if (rtk::ref_kind(el[k]) == rtk::K_TRI) m.tri_mask |= 1u << k;
        }
        m.planar_first = rtk::ref_index(el[0]);
        m.planar_n = (uint32_t)el.size();
        m.bxf_n = nxf;
    }

    // Returns (ref, need): need = traversal-stack entries used below the entry
    // that held this ref (rt_kernel.hip trace()).
    std::pair<uint32_t, uint32_t> emit(int id, bool in_boundary, int xf_depth) {
        auto it = memo.find(id);
        if (it != memo.end()) return it->second;
        const Obj& o = s->objs[id];
        std::pair<uint32_t, uint32_t> r{REF_NONE_, 0};
        switch (o.kind) {
            case O_SPHERE: {
                uint32_t idx = (uint32_t)out.spheres.size();
                out.spheres.push_back(make_double4(o.c1.x, o.c1.y, o.c1.z, o.radius));
                out.sphere_mat.push_back(o.mat);
                out.sphere_rinv.push_back(1.0 / o.radius);  // vec3.rs:225-227: v / r = (1.0 / r) * v
                r = {rtk::make_ref(rtk::K_SPHERE, idx), 0};
                ++out.n_prims;
                break;
            }
            case O_MSPHERE: {
                uint32_t idx = (uint32_t)out.msph_center.size();
                out.msph_center.push_back(make_double4(o.c1.x, o.c1.y, o.c1.z, o.radius));
                out.msph_dir.push_back(make_double4(o.cdir.x, o.cdir.y, o.cdir.z, 0.0));
                out.msph_mat.push_back(o.mat);
                r = {rtk::make_ref(rtk::K_MSPHERE, idx), 0};
                out.features |= rtk::F_MSPHERE;
                ++out.n_prims;
                break;
            }
            case O_QUAD:
            case O_TRI: {
                uint32_t idx = (uint32_t)out.planars.size();
                rtk::DPlanar p;
                double f[16] = {o.normal.x, o.normal.y, o.normal.z, o.D,  o.anchor.x, o.anchor.y, o.anchor.z, o.u.x,
                                o.u.y,      o.u.z,      o.v.x,      o.v.y, o.v.z,      o.w.x,      o.w.y,      o.w.z};
                std::memcpy(p.f, f, sizeof f);
                out.planars.push_back(p);
                if (rtk_planar_filter()) out.planars_f.push_back(planar_f(o));
                out.planar_area.push_back(o.area);
                out.planar_mat.push_back(o.mat);
                if (o.remap) {
                    rtk::DRemap rm{};
                    for (int j = 0; j < 3; ++j) {
                        rm.n[3 * j] = o.rn[j].x;
                        rm.n[3 * j + 1] = o.rn[j].y;
                        rm.n[3 * j + 2] = o.rn[j].z;
                    }
                    for (int j = 0; j < 2; ++j) {
                        rm.tex_ori[j] = o.tex_ori[j];
                        rm.tex_u[j] = o.tex_u[j];
                        rm.tex_v[j] = o.tex_v[j];
                    }
                    rm.normal_tex = o.normal_tex;
                    rm.uv_ok = o.uv_ok ? 1 : 0;
                    rtk::DRemapNM nm{};
                    if (o.normal_tex >= 0) {
                        nm.u_vec[0] = o.u_vec.x; nm.u_vec[1] = o.u_vec.y; nm.u_vec[2] = o.u_vec.z;
                        nm.v_vec[0] = o.v_vec.x; nm.v_vec[1] = o.v_vec.y; nm.v_vec[2] = o.v_vec.z;
                        out.features |= rtk::F_NORMALMAP;
                    }
                    out.planar_remap.push_back((int32_t)out.remaps.size());
                    out.remaps.push_back(rm);
                    out.remap_nm.push_back(nm);
                    out.features |= rtk::F_REMAP;
                } else {
                    out.planar_remap.push_back(-1);
                }
                r = {rtk::make_ref(o.kind == O_QUAD ? rtk::K_QUAD : rtk::K_TRI, idx), 0};
                out.features |= rtk::F_PLANAR;
                ++out.n_prims;
                break;
            }
            case O_LIST: {
                if (o.children.size() == 1 && !no_collapse) {  // world: min_by over one element is the element
                    r = emit(o.children[0], in_boundary, xf_depth);
                    break;
                }
                // A list holding BVHs (the C4 / C5 worlds: meshes or sphere
                // clouds beside a few loose objects) is walked as a BVH over
                // its elements: Hittables::hit keeps the closest of all its
                // children (hits.rs:34-46), which any BVH over them finds too
                // (up to exact t ties, as for every rebuilt BVH) -- without
                // one walk iteration per element.  Lists of plain primitives
                // (C3's Cornell box) stay lists: they keep the BVH-free tier.
                // Nested lists (an OBJ's per-model BVHs beside C4's two
                // spheres) join the rebuilt BVH element by element.
                if (!reference_bvh && !no_collapse && o.children.size() >= 2 &&
                    std::any_of(o.children.begin(), o.children.end(), [&](int c) { return holds_bvh(c, 0); })) {
                    std::vector<int> elems;
                    for (int c : o.children) list_elements(c, elems, 0);
                    std::vector<Item> items;
                    for (int c : elems) {
                        auto e = emit(c, in_boundary, xf_depth);
                        Item x;
                        x.ref = e.first;
                        x.need = e.second;
                        x.box = tight(c);
                        for (int k = 0; k < 3; ++k) x.c[k] = 0.5 * (x.box.a[k].lo + x.box.a[k].hi);
                        items.push_back(x);
                    }
                    out.n_bvh_leaves += items.size();
                    r = sah(items, 0, items.size());
                    break;
                }
                std::vector<std::pair<uint32_t, uint32_t>> kids;
                for (int c : o.children) kids.push_back(emit(c, in_boundary, xf_depth));
                uint32_t start = (uint32_t)out.list_children.size();
                for (size_t i = 0; i < kids.size(); ++i) {
                    out.list_children.push_back(kids[i].first);
                    out.list_boxes.push_back(boxf(tight(o.children[i])));
                }
                out.list_children.push_back(REF_NONE_);
                out.list_boxes.push_back(boxf(Box3::empty()));
                // iterator form: popping (LIST,p) pushes (LIST,p+1) then walks child p
                uint32_t need = 0;
                for (size_t i = 0; i < kids.size(); ++i) {
                    bool last = i + 1 == kids.size();
                    need = std::max(need, last ? kids[i].second : 1 + kids[i].second);
                }
                r = {rtk::make_ref(rtk::K_LIST, start), need};
                break;
            }
            case O_BVH: {
                if (reference_bvh) {
                    r = ref_bvh(id, in_boundary, xf_depth, true);
                    break;
                }
                std::vector<int> leaves;
                collect_leaves(id, leaves);
                std::vector<Item> items;
                items.reserve(leaves.size());
                for (int l : leaves) {
                    auto e = emit(l, in_boundary, xf_depth);
                    Item x;
                    x.ref = e.first;
                    x.need = e.second;
                    x.box = tight(l);
                    for (int k = 0; k < 3; ++k) x.c[k] = 0.5 * (x.box.a[k].lo + x.box.a[k].hi);
                    items.push_back(x);
                }
                out.n_bvh_leaves += items.size();
                if (items.size() == 1) {
                    // BVH over one object: a node with one child keeps the box test
                    uint32_t idx = (uint32_t)out.nodes.size();
                    out.nodes.emplace_back();
                    rtk::DNode& n = out.nodes[idx];
                    set_child(n, 0, items[0].ref, items[0].box);
                    set_box(n, 1, Box3::empty());
                    n.c0 = items[0].ref;
                    n.c1 = REF_NONE_;
                    r = {rtk::make_ref(rtk::K_BVH, idx), std::max<uint32_t>(1, items[0].need)};
                } else {
                    r = sah(items, 0, items.size());
                }
                break;
            }
            case O_XFORM: {
                if (xf_depth >= MAX_XF_NESTING)
                    return {fail(RT_EUNSUPPORTED, "Transform nested deeper than 2 levels"), 0};
                auto C = emit(o.child, in_boundary, xf_depth + 1);
                uint32_t idx = (uint32_t)out.xforms.size();
                rtk::DXform x{};
                x.off[0] = o.offset.x; x.off[1] = o.offset.y; x.off[2] = o.offset.z;
                x.scale[0] = o.scale.x; x.scale[1] = o.scale.y; x.scale[2] = o.scale.z;
                x.q[0] = o.q.w;
                x.q[1] = o.q.x;
                x.q[2] = o.q.y;
                x.q[3] = o.q.z;
                x.child = C.first;
                x.flags = (o.scale.x == 1.0 && o.scale.y == 1.0 && o.scale.z == 1.0) ? rtk::XF_UNIT_SCALE : 0u;
                out.xforms.push_back(x);
                out.features |= rtk::F_XFORM;
                r = {rtk::make_ref(rtk::K_XFORM, idx), 1 + C.second};
                break;
            }
            case O_MEDIUM: {
                if (in_boundary) return {fail(RT_EUNSUPPORTED, "ConstantMedium inside a medium boundary"), 0};
                auto B = emit(o.child, true, xf_depth);
                uint32_t idx = (uint32_t)out.media.size();
                rtk::DMedium m{};
                m.neg_inv_density = o.neg_inv_density;
                m.boundary = B.first;
                m.phase_mat = o.phase_mat;
                m.medium_id = o.medium_id;
                planar_boundary(B.first, m);
                out.media.push_back(m);
                out.features |= rtk::F_MEDIUM;
                r = {rtk::make_ref(rtk::K_MEDIUM, idx), B.second};
                break;
            }
        }
        memo[id] = r;
        return r;
    }
};

// The lights tree of HittablePDF (camera.rs:298-304): 1 = a primitive or one
// flat list of static spheres / quads / triangles (the FULL tiers' light
// code), 2 = any other tree of lists and Transforms over spheres (static or
// moving), quads and triangles (tier FULL_GL: hits.rs:52-75, shapes.rs:117-132),
// or an RT_E* code: a BVH or a ConstantMedium has no pdf_value / random
// (hit.rs:52-60 unimplemented!(): the reference panics at the first light
// sample), an empty list panics in Hittables::random (hits.rs:71-73).
constexpr int LIGHT_TREE_DEPTH = 4;  // rt_kernel.hip RT_LIGHT_DEPTH
int light_tree(const rt_scene* s, int id, int depth, std::string& err) {
    const Obj& o = s->objs[id];
    switch (o.kind) {
        case O_SPHERE:
        case O_QUAD:
        case O_TRI: return 1;
        case O_MSPHERE: return 2;
        case O_LIST: {
            if (o.children.empty()) {
                err = "The collection of objects is empty! (Hittables::random of the lights, hits.rs:71-73)";
                return RT_EPANIC;
            }
            if (depth >= LIGHT_TREE_DEPTH) {
                err = "lights tree deeper than " + std::to_string(LIGHT_TREE_DEPTH) + " list / Transform levels";
                return RT_EUNSUPPORTED;
            }
            int kind = depth == 0 ? 1 : 2;
            for (int c : o.children) {
                const ObjKind ck = s->objs[c].kind;
                int k = light_tree(s, c, depth + 1, err);
                if (k < 0) return k;
                if (k == 2 || !(ck == O_SPHERE || ck == O_QUAD || ck == O_TRI)) kind = 2;
            }
            return kind;
        }
        case O_XFORM: {
            if (depth >= LIGHT_TREE_DEPTH) {
                err = "lights tree deeper than " + std::to_string(LIGHT_TREE_DEPTH) + " list / Transform levels";
                return RT_EUNSUPPORTED;
            }
            int k = light_tree(s, o.child, depth + 1, err);
            return k < 0 ? k : 2;
        }
        case O_BVH:
            err = "pdf_value: unimplemented!() -- BVH has no Hittable::pdf_value / random (bvh.rs, hit.rs:52-60)";
            return RT_EPANIC;
        case O_MEDIUM:
            err = "pdf_value: unimplemented!() -- ConstantMedium has no Hittable::pdf_value / random (volume.rs, hit.rs:52-60)";
            return RT_EPANIC;
    }
    return RT_EUNSUPPORTED;
}
}  // namespace

static int tex_needs_uv(const rt_scene* s, int t, int depth = 0) {
    if (t < 0 || depth > 16) return 0;
    const TexRec& r = s->texs[t];
    if (r.type == rtk::T_IMAGE) return r.h != 0;
    if (r.type == rtk::T_CHECKER) return tex_needs_uv(s, r.even, depth + 1) | tex_needs_uv(s, r.odd, depth + 1);
    return 0;
}

int32_t flatten(const rt_scene* s, int32_t world, int32_t lights, int32_t background_tex, bool reference_bvh,
                HostWorld& out) {
    out = HostWorld();
    // textures (texture.rs) and materials (material.rs) keep their handle ids
    for (size_t i = 0; i < s->texs.size(); ++i) {
        const TexRec& r = s->texs[i];
        rtk::DTexture t{};
        t.type = r.type;
        for (int k = 0; k < 3; ++k) {
            t.color[k] = r.color[k];
            t.color2[k] = r.color2[k];
        }
        t.scale = r.scale;
        t.a = r.type == rtk::T_CHECKER ? r.even : (int32_t)r.w;
        t.b = r.type == rtk::T_CHECKER ? r.odd : (int32_t)r.h;
        t.c = r.linear;
        t.data = r.type == rtk::T_IMAGE ? r.texel_offset : (uint64_t)(r.perlin < 0 ? 0 : r.perlin);
        t.needs_uv = tex_needs_uv(s, (int)i);
        out.textures.push_back(t);
    }
    out.texels = s->texels;
    out.perlin = s->perlins;
    for (size_t i = 0; i < s->mats.size(); ++i) {
        const MatRec& r = s->mats[i];
        rtk::DMaterial m{};
        m.type = r.type;
        m.tex = r.tex;
        m.inner = r.inner;
        m.inner2 = r.inner2;
        for (int k = 0; k < 3; ++k) m.albedo[k] = r.albedo[k];
        m.fuzz = r.param;
        out.materials.push_back(m);
    }
    // flags: uv need and emission, resolved through DiffuseLight/Mix nesting
    for (size_t i = 0; i < out.materials.size(); ++i) {
        rtk::DMaterial& m = out.materials[i];
        uint32_t f = 0;
        if (m.tex >= 0 && tex_needs_uv(s, m.tex)) f |= rtk::MF_NEEDS_UV;
        if (m.type == rtk::M_DIFFUSE_LIGHT) f |= rtk::MF_EMISSIVE;
        // a solid-colour texture on a material that does not use albedo
        // itself: the colour in albedo, read with the material record
        if (m.type != rtk::M_METAL && m.tex >= 0 && s->texs[m.tex].type == rtk::T_SOLID) {
            f |= rtk::MF_SOLID;
            for (int k = 0; k < 3; ++k) m.albedo[k] = s->texs[m.tex].color[k];
        }
        m.flags = f;
    }
    for (int pass = 0; pass < 4; ++pass)
        for (size_t i = 0; i < out.materials.size(); ++i) {
            rtk::DMaterial& m = out.materials[i];
            if (m.type == rtk::M_DIFFUSE_LIGHT || m.type == rtk::M_MIX) {
                for (int sub : {m.inner, m.inner2})
                    if (sub >= 0) m.flags |= out.materials[sub].flags & (rtk::MF_NEEDS_UV | rtk::MF_EMISSIVE);
            }
        }
    if (background_tex >= (int32_t)s->texs.size()) return set_error(RT_EHANDLE, "unknown background texture");

    Flattener F{s, out, reference_bvh, {}, false, {}, {}, RT_OK};
    auto W = F.emit(world, false, 0);
    if (F.code != RT_OK) return set_error(F.code, F.err);
    out.world_root = W.first;
    out.stack_need = 1 + W.second;
    out.lights_root = rtk::REF_NONE;
    if (lights >= 0) {
        std::string lerr;
        const int lk = light_tree(s, lights, 0, lerr);
        if (lk < 0) return set_error(lk, lerr);
        if (lk == 2) out.features |= rtk::F_GENERAL;
        F.no_collapse = true;
        F.memo.erase(lights);
        auto Lr = F.emit(lights, false, 0);
        F.no_collapse = false;
        if (F.code != RT_OK) return set_error(F.code, F.err);
        out.lights_root = Lr.first;
        out.features |= rtk::F_LIGHTS;
    }
    // Materials and textures reachable from the emitted primitives and the
    // background decide the kernel tier (an unused DiffuseLight in the scene
    // must not force the full tier) and are the ones checked for support.
    std::vector<char> mat_used(out.materials.size(), 0), tex_used(out.textures.size(), 0);
    std::vector<int> work;
    auto use_mat = [&](int m) {
        if (m >= 0 && !mat_used[m]) {
            mat_used[m] = 1;
            work.push_back(m);
        }
    };
    for (int32_t m : out.sphere_mat) use_mat(m);
    for (int32_t m : out.msph_mat) use_mat(m);
    for (int32_t m : out.planar_mat) use_mat(m);
    for (const auto& md : out.media) use_mat(md.phase_mat);
    while (!work.empty()) {
        const int m = work.back();
        work.pop_back();
        use_mat(out.materials[m].inner);
        use_mat(out.materials[m].inner2);
    }
    std::vector<int> twork;
    auto use_tex = [&](int t) {
        if (t >= 0 && !tex_used[t]) {
            tex_used[t] = 1;
            twork.push_back(t);
        }
    };
    use_tex(background_tex);
    for (const auto& rm : out.remaps) use_tex(rm.normal_tex);
    for (size_t i = 0; i < out.materials.size(); ++i)
        if (mat_used[i]) use_tex(out.materials[i].tex);
    while (!twork.empty()) {
        const int t = twork.back();
        twork.pop_back();
        if (out.textures[t].type == rtk::T_CHECKER) {
            use_tex(out.textures[t].a);
            use_tex(out.textures[t].b);
        }
    }
    for (size_t i = 0; i < out.textures.size(); ++i)
        if (tex_used[i] && (out.textures[i].type == rtk::T_IMAGE || out.textures[i].type == rtk::T_NOISE))
            out.features |= rtk::F_TEXFULL;
    for (size_t i = 0; i < out.materials.size(); ++i) {
        if (!mat_used[i]) continue;
        const rtk::DMaterial& m = out.materials[i];
        if (m.type == rtk::M_DIFFUSE_LIGHT || m.type == rtk::M_ISOTROPIC || m.type == rtk::M_TRANSPARENT ||
            m.type == rtk::M_MIX)
            out.features |= rtk::F_MATFULL;
    }
    // Wrapper materials (DiffuseLight with a material, Mix): the C3 / C5 tiers
    // take one level whose Mix ratio is a constant; deeper trees and
    // Mix::from_image ratios run the FULL_GL tier (rt_kernel.hip emitted_tree),
    // up to RT_MAT_DEPTH (4) wrapper levels.
    std::function<int(int)> wrap_depth = [&](int mid) -> int {
        const rtk::DMaterial& m = out.materials[mid];
        if (m.type == rtk::M_MIX) return 1 + std::max(wrap_depth(m.inner), wrap_depth(m.inner2));
        if (m.type == rtk::M_DIFFUSE_LIGHT && m.inner >= 0) return 1 + wrap_depth(m.inner);
        return 0;
    };
    for (size_t i = 0; i < out.materials.size(); ++i) {
        if (!mat_used[i]) continue;
        const rtk::DMaterial& m = out.materials[i];
        const int depth = wrap_depth((int)i);
        if (depth > 4) return set_error(RT_EUNSUPPORTED, "DiffuseLight / Mix wrappers nested deeper than 4 levels");
        bool general = m.type == rtk::M_MIX && m.tex >= 0;
        if (m.type == rtk::M_MIX)
            for (int sub : {m.inner, m.inner2}) {
                const int st = out.materials[sub].type;
                if (st == rtk::M_MIX || (st == rtk::M_DIFFUSE_LIGHT && out.materials[sub].inner >= 0)) general = true;
            }
        if (m.type == rtk::M_DIFFUSE_LIGHT && m.inner >= 0) {
            const int st = out.materials[m.inner].type;
            if (st == rtk::M_MIX || st == rtk::M_DIFFUSE_LIGHT) general = true;
        }
        if (general) out.features |= rtk::F_GENERAL;
    }
    if (out.list_children.empty()) {
        out.list_children.push_back(rtk::REF_NONE);
        out.list_boxes.push_back(rtk::DBoxF{});
    }
    // planar runs of the lists (DBoxF::run): the flat tier tests a run in one
    // walk step
    auto planar = [](uint32_t r) { return rtk::ref_kind(r) == rtk::K_QUAD || rtk::ref_kind(r) == rtk::K_TRI; };
    for (size_t i = 0; i < out.list_children.size(); ++i) {
        const uint32_t c = out.list_children[i];
        uint32_t run = 0;
        if (planar(c)) {
            uint32_t n = 0;
            while (n < rtk::RT_PLANAR_RUN_MAX && i + n < out.list_children.size() && planar(out.list_children[i + n]) &&
                   rtk::ref_index(out.list_children[i + n]) == rtk::ref_index(c) + n) {
                if (rtk::ref_kind(out.list_children[i + n]) == rtk::K_TRI) run |= 1u << (8 + n);
                ++n;
            }
            run |= n;
        }
        out.list_boxes[i].run = run;
    }
    return RT_OK;
}

}  // namespace rth

using namespace rth;

// ------------------------------------------------------------------ C ABI (builders)
namespace {
bool bad(const double* p) { return p == nullptr; }
int32_t check_obj(const rt_scene* s, int32_t o) {
    if (o < 0 || (size_t)o >= s->objs.size() || s->objs[o].hidden) return set_error(RT_EHANDLE, "unknown object handle");
    if (s->objs[o].moved) return set_error(RT_EMOVED, "object handle already moved (Box<dyn Hittable> is owned)");
    return RT_OK;
}
bool tex_ok(const rt_scene* s, int32_t t) { return t >= 0 && (size_t)t < s->texs.size(); }
bool mat_ok(const rt_scene* s, int32_t m) { return m >= 0 && (size_t)m < s->mats.size(); }
int32_t push_obj(rt_scene* s, Obj o) {
    s->objs.push_back(std::move(o));
    ++s->generation;
    return (int32_t)s->objs.size() - 1;
}
int32_t push_tex(rt_scene* s, TexRec t) {
    s->texs.push_back(t);
    ++s->generation;
    return (int32_t)s->texs.size() - 1;
}
int32_t push_mat(rt_scene* s, MatRec m) {
    s->mats.push_back(m);
    ++s->generation;
    return (int32_t)s->mats.size() - 1;
}
Obj make_planar(ObjKind k, V3 q, V3 u, V3 v, int mat) {
    Obj o;
    o.kind = k;
    V3 n = cross(u, v);
    o.normal = div(n, length(n));
    o.D = dot(o.normal, q);
    o.w = div(n, dot(n, n));
    o.area = k == O_QUAD ? length(n) : length(n) / 2.0;
    o.anchor = q;
    o.u = u;
    o.v = v;
    o.mat = mat;
    if (k == O_QUAD)  // quad.rs:50-55
        o.bbox = Box3::from_points(q, q + u + v).unite(Box3::from_points(q + u, q + v));
    else  // triangle.rs:49-54
        o.bbox = Box3::from_points(q, q + u).unite(Box3::from_points(q, q + v));
    return o;
}
}  // namespace

extern "C" {

int32_t rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return rth::g_error.c_str(); }
rt_scene* rt_scene_create(void) {
    try {
        return new rt_scene();
    } catch (...) {
        set_error(RT_ENOMEM, "out of memory");
        return nullptr;
    }
}

// ---- textures
int32_t rt_tex_solid(rt_scene* s, const double rgb[3]) {
    if (!s || bad(rgb)) return set_error(RT_EINVAL, "null argument");
    TexRec t{};
    t.type = rtk::T_SOLID;
    std::memcpy(t.color, rgb, 24);
    return push_tex(s, t);
}
int32_t rt_tex_checker(rt_scene* s, double scale, int32_t even, int32_t odd) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if (!tex_ok(s, even) || !tex_ok(s, odd)) return set_error(RT_EHANDLE, "unknown texture");
    TexRec t{};
    t.type = rtk::T_CHECKER;
    t.scale = 1.0 / scale;  // inv_scale (texture.rs:52)
    t.even = even;
    t.odd = odd;
    return push_tex(s, t);
}
int32_t rt_tex_image(rt_scene* s, uint32_t w, uint32_t h, const float* rgba, int32_t linear) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if ((w == 0) != (h == 0)) return set_error(RT_EINVAL, "image must have both dimensions or none");
    if (w && !rgba) return set_error(RT_EINVAL, "null pixels");
    TexRec t{};
    t.type = rtk::T_IMAGE;
    t.w = w;
    t.h = h;
    t.linear = linear != 0;
    t.texel_offset = s->texels.size();
    if (w) s->texels.insert(s->texels.end(), rgba, rgba + (size_t)w * h * 4);
    return push_tex(s, t);
}
int32_t rt_tex_image_file(rt_scene* s, const char* path, int32_t raw, int32_t linear) {
    if (!s || !path) return set_error(RT_EINVAL, "null argument");
    uint32_t w = 0, h = 0;
    std::vector<float> px;
    std::string err;
    const rtimg::Status st = rtimg::load(path, raw != 0, w, h, px, err);
    if (st == rtimg::UNSUPPORTED) return set_error(RT_EUNSUPPORTED, err);
    return rt_tex_image(s, w, h, px.empty() ? nullptr : px.data(), linear);  // MISSING: 0 x 0, cyan
}
int32_t rt_tex_noise(rt_scene* s, double scale, uint64_t seed) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    // perlin.rs:16-36 drawn from SplitMix64(seed) (the RNG contract)
    rtk::DPerlin p{};
    uint64_t st = seed;
    auto next = [&st]() {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        return (double)(z >> 11) * (1.0 / 9007199254740992.0);
    };
    const double PI = 3.14159265358979323846;
    for (int i = 0; i < 256; ++i) {
        double r1 = next(), r2 = next();
        p.randvec[i][0] = std::cos(2.0 * PI * r1) * 2.0 * std::sqrt(r2 * (1.0 - r2));
        p.randvec[i][1] = std::sin(2.0 * PI * r1) * 2.0 * std::sqrt(r2 * (1.0 - r2));
        p.randvec[i][2] = 1.0 - 2.0 * r2;
    }
    for (int a = 0; a < 3; ++a) {
        for (int i = 0; i < 256; ++i) p.perm[a][i] = i;
        for (int i = 255; i >= 1; --i) {
            int target = (int)(next() * (double)(i + 1));
            if (target > i) target = i;
            std::swap(p.perm[a][i], p.perm[a][target]);
        }
    }
    s->perlins.push_back(p);
    TexRec t{};
    t.type = rtk::T_NOISE;
    t.scale = scale;
    t.perlin = (int)s->perlins.size() - 1;
    return push_tex(s, t);
}
int32_t rt_tex_sky_gradient(rt_scene* s, const double horizon[3], const double zenith[3]) {
    if (!s || bad(horizon) || bad(zenith)) return set_error(RT_EINVAL, "null argument");
    TexRec t{};
    t.type = rtk::T_SKY;
    std::memcpy(t.color, horizon, 24);
    std::memcpy(t.color2, zenith, 24);
    return push_tex(s, t);
}

// ---- materials
int32_t rt_mat_empty(rt_scene* s) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    MatRec m{};
    m.type = rtk::M_EMPTY;
    return push_mat(s, m);
}
int32_t rt_mat_lambertian(rt_scene* s, int32_t tex) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if (!tex_ok(s, tex)) return set_error(RT_EHANDLE, "unknown texture");
    MatRec m{};
    m.type = rtk::M_LAMBERTIAN;
    m.tex = tex;
    return push_mat(s, m);
}
int32_t rt_mat_metal(rt_scene* s, const double albedo[3], double fuzz) {
    if (!s || bad(albedo)) return set_error(RT_EINVAL, "null argument");
    MatRec m{};
    m.type = rtk::M_METAL;
    std::memcpy(m.albedo, albedo, 24);
    m.param = std::clamp(fuzz, 0.0, 1.0);  // material.rs:77
    return push_mat(s, m);
}
int32_t rt_mat_dielectric(rt_scene* s, int32_t tex, double ior) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if (!tex_ok(s, tex)) return set_error(RT_EHANDLE, "unknown texture");
    MatRec m{};
    m.type = rtk::M_DIELECTRIC;
    m.tex = tex;
    m.param = ior;
    return push_mat(s, m);
}
int32_t rt_mat_diffuse_light(rt_scene* s, int32_t tex, int32_t inner) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if (!tex_ok(s, tex)) return set_error(RT_EHANDLE, "unknown texture");
    if (inner != -1 && !mat_ok(s, inner)) return set_error(RT_EHANDLE, "unknown material");
    MatRec m{};
    m.type = rtk::M_DIFFUSE_LIGHT;
    m.tex = tex;
    m.inner = inner;
    return push_mat(s, m);
}
int32_t rt_mat_isotropic(rt_scene* s, int32_t tex) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if (!tex_ok(s, tex)) return set_error(RT_EHANDLE, "unknown texture");
    MatRec m{};
    m.type = rtk::M_ISOTROPIC;
    m.tex = tex;
    return push_mat(s, m);
}
int32_t rt_mat_transparent(rt_scene* s) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    MatRec m{};
    m.type = rtk::M_TRANSPARENT;
    return push_mat(s, m);
}
int32_t rt_mat_mix(rt_scene* s, int32_t m1, int32_t m2, double ratio) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if (!mat_ok(s, m1) || !mat_ok(s, m2)) return set_error(RT_EHANDLE, "unknown material");
    MatRec m{};
    m.type = rtk::M_MIX;
    m.inner = m1;
    m.inner2 = m2;
    m.param = ratio;
    return push_mat(s, m);
}

int32_t rt_mat_mix_image(rt_scene* s, int32_t m1, int32_t m2, int32_t tex) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    if (!mat_ok(s, m1) || !mat_ok(s, m2)) return set_error(RT_EHANDLE, "unknown material");
    if (!tex_ok(s, tex) || s->texs[tex].type != rtk::T_IMAGE)
        return set_error(RT_EHANDLE, "Mix::from_image takes an ImageTexture");
    MatRec m{};
    m.type = rtk::M_MIX;
    m.inner = m1;
    m.inner2 = m2;
    m.tex = tex;  // ratio = tex.alpha(u, v, p) (material.rs:237-247, texture.rs:99-106)
    return push_mat(s, m);
}

// ---- hittables
int32_t rt_sphere(rt_scene* s, const double c[3], double r, int32_t mat) {
    if (!s || bad(c)) return set_error(RT_EINVAL, "null argument");
    if (!mat_ok(s, mat)) return set_error(RT_EHANDLE, "unknown material");
    Obj o;
    o.kind = O_SPHERE;
    o.c1 = V3(c);
    o.radius = std::fmax(0.0, r);
    o.mat = mat;
    V3 rv(r, r, r);
    o.bbox = Box3::from_points(o.c1 - rv, o.c1 + rv);  // sphere.rs:31
    return push_obj(s, o);
}
int32_t rt_sphere_moving(rt_scene* s, const double c1[3], const double c2[3], double r, int32_t mat) {
    if (!s || bad(c1) || bad(c2)) return set_error(RT_EINVAL, "null argument");
    if (!mat_ok(s, mat)) return set_error(RT_EHANDLE, "unknown material");
    Obj o;
    o.kind = O_MSPHERE;
    o.c1 = V3(c1);
    o.cdir = V3(c2) - V3(c1);
    o.radius = std::fmax(0.0, r);
    o.mat = mat;
    V3 rv(r, r, r);
    V3 at0 = o.c1 + 0.0 * o.cdir, at1 = o.c1 + 1.0 * o.cdir;  // sphere.rs:44-47
    o.bbox = Box3::from_points(at0 - rv, at0 + rv).unite(Box3::from_points(at1 - rv, at1 + rv));
    return push_obj(s, o);
}
int32_t rt_quad(rt_scene* s, const double q[3], const double u[3], const double v[3], int32_t mat) {
    if (!s || bad(q) || bad(u) || bad(v)) return set_error(RT_EINVAL, "null argument");
    if (!mat_ok(s, mat)) return set_error(RT_EHANDLE, "unknown material");
    V3 n = cross(V3(u), V3(v));
    if (!finite(div(n, length(n)))) return set_error(RT_EPANIC, "The length of normal should be normalizable!");
    return push_obj(s, make_planar(O_QUAD, V3(q), V3(u), V3(v), mat));
}
int32_t rt_triangle(rt_scene* s, const double a[3], const double u[3], const double v[3], int32_t mat) {
    if (!s || bad(a) || bad(u) || bad(v)) return set_error(RT_EINVAL, "null argument");
    if (!mat_ok(s, mat)) return set_error(RT_EHANDLE, "unknown material");
    V3 n = cross(V3(u), V3(v));
    if (!finite(div(n, length(n)))) return set_error(RT_EDEGENERATE, "degenerate triangle (Triangle::new -> None)");
    return push_obj(s, make_planar(O_TRI, V3(a), V3(u), V3(v), mat));
}
int32_t rt_hittables_new(rt_scene* s) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    Obj o;
    o.kind = O_LIST;  // bbox = AABB::default() (hits.rs:9)
    return push_obj(s, o);
}
int32_t rt_hittables_add(rt_scene* s, int32_t list, int32_t object) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    int32_t rc;
    if ((rc = check_obj(s, list)) != RT_OK) return rc;
    if ((rc = check_obj(s, object)) != RT_OK) return rc;
    if (s->objs[list].kind != O_LIST) return set_error(RT_EHANDLE, "not a Hittables object");
    if (list == object) return set_error(RT_EINVAL, "cannot add a list to itself");
    s->objs[list].bbox = s->objs[list].bbox.unite(s->objs[object].bbox);  // hits.rs:28
    s->objs[list].children.push_back(object);
    s->objs[object].moved = true;
    ++s->generation;
    return RT_OK;
}
int32_t rt_bvh_new(rt_scene* s, int32_t list) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    int32_t rc;
    if ((rc = check_obj(s, list)) != RT_OK) return rc;
    if (s->objs[list].kind != O_LIST) return set_error(RT_EHANDLE, "not a Hittables object");
    if (s->objs[list].children.empty()) return set_error(RT_EPANIC, "BVH node must contain at least one object");
    int root;
    try {
        root = bvh_from_vec(s, s->objs[list].children);
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
    s->objs[list].moved = true;
    s->objs[root].hidden = false;
    ++s->generation;
    return root;
}
int32_t rt_bvh_selftest(rt_scene* s, int32_t list) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    int32_t rc;
    if ((rc = check_obj(s, list)) != RT_OK) return rc;
    if (s->objs[list].kind != O_LIST || s->objs[list].children.empty())
        return set_error(RT_EHANDLE, "not a non-empty Hittables object");
    try {
        rt_scene a, b;
        a.objs = s->objs;
        b.objs = s->objs;
        const int ra = bvh_from_vec(&a, s->objs[list].children);
        const int rb = bvh_from_vec_serial(&b, s->objs[list].children);
        if (ra != rb || a.objs.size() != b.objs.size()) return 0;
        for (size_t i = s->objs.size(); i < a.objs.size(); ++i) {
            const Obj &x = a.objs[i], &y = b.objs[i];
            if (x.kind != y.kind || x.left != y.left || x.right != y.right || x.hidden != y.hidden ||
                std::memcmp(&x.bbox, &y.bbox, sizeof(Box3)) != 0)
                return 0;
        }
        return 1;
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
}
int32_t rt_world_selftest(rt_scene* s, int32_t world, int32_t lights, int32_t background_tex) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    try {
        HostWorld p, q;
        int32_t rc = flatten(s, world, lights, background_tex, false, p);
        if (rc != RT_OK) return rc;
        g_serial_build = true;
        rc = flatten(s, world, lights, background_tex, false, q);
        g_serial_build = false;
        if (rc != RT_OK) return rc;
        auto same = [](const auto& x, const auto& y) {
            return x.size() == y.size() && (x.empty() || std::memcmp(x.data(), y.data(), x.size() * sizeof(x[0])) == 0);
        };
        return (same(p.nodes, q.nodes) && same(p.list_children, q.list_children) && same(p.planars, q.planars) &&
                same(p.spheres, q.spheres) && p.world_root == q.world_root && p.lights_root == q.lights_root &&
                p.stack_need == q.stack_need)
                   ? 1
                   : 0;
    } catch (const std::bad_alloc&) {
        g_serial_build = false;
        return set_error(RT_ENOMEM, "out of host memory");
    }
}
int32_t rt_build_box(rt_scene* s, const double a[3], const double b[3], int32_t mat) {
    if (!s || bad(a) || bad(b)) return set_error(RT_EINVAL, "null argument");
    if (!mat_ok(s, mat)) return set_error(RT_EHANDLE, "unknown material");
    // quad.rs:128-189
    V3 mn(std::fmin(a[0], b[0]), std::fmin(a[1], b[1]), std::fmin(a[2], b[2]));
    V3 mx(std::fmax(a[0], b[0]), std::fmax(a[1], b[1]), std::fmax(a[2], b[2]));
    V3 dx(mx.x - mn.x, 0, 0), dy(0, mx.y - mn.y, 0), dz(0, 0, mx.z - mn.z);
    int32_t list = rt_hittables_new(s);
    const V3 anchors[6] = {V3(mn.x, mn.y, mx.z), V3(mx.x, mn.y, mx.z), V3(mx.x, mn.y, mn.z),
                           V3(mn.x, mn.y, mn.z), V3(mn.x, mx.y, mx.z), V3(mn.x, mn.y, mn.z)};
    const V3 us[6] = {dx, -dz, -dx, dz, dx, dx};
    const V3 vs[6] = {dy, dy, dy, dy, -dz, dz};
    for (int k = 0; k < 6; ++k) {
        double q[3] = {anchors[k].x, anchors[k].y, anchors[k].z}, u[3] = {us[k].x, us[k].y, us[k].z},
               v[3] = {vs[k].x, vs[k].y, vs[k].z};
        int32_t side = rt_quad(s, q, u, v, mat);
        if (side < 0) return side;
        rt_hittables_add(s, list, side);
    }
    return list;
}
int32_t rt_transform_new(rt_scene* s, int32_t object, const double* off, const double* q, const double* sc) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    int32_t rc;
    if ((rc = check_obj(s, object)) != RT_OK) return rc;
    Obj o;
    o.kind = O_XFORM;
    o.child = object;
    o.offset = off ? V3(off) : V3(0, 0, 0);
    o.q = q ? Quat{q[0], q[1], q[2], q[3]} : Quat{};
    o.scale = sc ? V3(sc) : V3(1, 1, 1);
    // shapes.rs:49-72: AABB of the 8 transformed corners
    const Box3& cb = s->objs[object].bbox;
    V3 mn(INF, INF, INF), mx(-INF, -INF, -INF);
    for (int i = 0; i < 8; ++i) {
        V3 p(cb.a[0].lo, cb.a[1].lo, cb.a[2].lo);
        if (i & 4) p.x = cb.a[0].hi;
        if (i & 2) p.y = cb.a[1].hi;
        if (i & 1) p.z = cb.a[2].hi;
        V3 t = o.q.rotate(p * o.scale) + o.offset;
        mn = V3(std::fmin(mn.x, t.x), std::fmin(mn.y, t.y), std::fmin(mn.z, t.z));
        mx = V3(std::fmax(mx.x, t.x), std::fmax(mx.y, t.y), std::fmax(mx.z, t.z));
    }
    o.bbox = Box3::from_points(mn, mx);
    s->objs[object].moved = true;
    return push_obj(s, o);
}
int32_t rt_constant_medium_new(rt_scene* s, int32_t boundary, double density, int32_t tex) {
    if (!s) return set_error(RT_EINVAL, "null argument");
    int32_t rc;
    if ((rc = check_obj(s, boundary)) != RT_OK) return rc;
    if (!tex_ok(s, tex)) return set_error(RT_EHANDLE, "unknown texture");
    Obj o;
    o.kind = O_MEDIUM;
    o.child = boundary;
    o.bbox = s->objs[boundary].bbox;  // volume.rs:75-77
    o.neg_inv_density = -1.0 / density;
    o.phase_mat = rt_mat_isotropic(s, tex);  // Box<Isotropic> (volume.rs:31)
    o.medium_id = s->next_medium_id++;
    s->objs[boundary].moved = true;
    return push_obj(s, o);
}

int32_t rt_quat_from_axis_angle(const double axis[3], double deg, double out[4]) {
    if (bad(axis) || !out) return set_error(RT_EINVAL, "null argument");
    // quaternion.rs:40-53
    const double PI = 3.14159265358979323846;
    double half = deg * (PI / 180.0) * 0.5;
    double sn = std::sin(half), c = std::cos(half);
    V3 a(axis);
    V3 u = div(a, length(a));
    if (!finite(u)) return set_error(RT_EPANIC, "Quaternion::from_axis_angle: axis not normalizable");
    out[0] = c;
    out[1] = u.x * sn;
    out[2] = u.y * sn;
    out[3] = u.z * sn;
    return RT_OK;
}
void rt_quat_from_euler(double yaw, double pitch, double roll, double out[4]) {
    // quaternion.rs:23-38
    double cy = std::cos(0.5 * yaw), sy = std::sin(0.5 * yaw);
    double cp = std::cos(0.5 * pitch), sp = std::sin(0.5 * pitch);
    double cr = std::cos(0.5 * roll), sr = std::sin(0.5 * roll);
    out[0] = cr * cp * cy + sr * sp * sy;
    out[1] = sr * cp * cy - cr * sp * sy;
    out[2] = cr * sp * cy + sr * cp * sy;
    out[3] = cr * cp * sy - sr * sp * cy;
}

void rt_camera_default(rt_camera* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->aspect_ratio = 1.0;  // camera.rs:76-104
    c->image_width = 100;
    c->samples_per_pixel = 10;
    c->max_depth = 10;
    c->background_tex = -1;
    c->vertical_fov_in_degrees = 90.0;
    c->look_at[2] = -1.0;
    c->vec_up[1] = 1.0;
    c->focus_distance = 10.0;
}
uint32_t rt_camera_image_height(const rt_camera* c) {
    if (!c || !(c->aspect_ratio > 0)) return 1;
    uint32_t h = (uint32_t)((double)c->image_width / c->aspect_ratio);  // camera.rs:205-210
    return h < 1 ? 1 : h;
}
void rt_render_opts_default(rt_render_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->struct_size = sizeof(*o);
    o->seed = 1;
    o->row_stride = 1;
}
uint32_t rt_shard_rows(const rt_camera* c, const rt_render_opts* o) {
    uint32_t H = rt_camera_image_height(c);
    uint32_t stride = (o && o->row_stride > 1) ? o->row_stride : 1;
    uint32_t off = o ? o->row_offset : 0;
    if (off >= H) return 0;
    return (H - off + stride - 1) / stride;
}

void rt_scene_destroy(rt_scene* s) {
    if (!s) return;
    if (s->rs) destroy_render_state(s->rs);
    delete s;
}

}  // extern "C"

namespace rth {
}  // namespace rth

#ifndef RT_BVH4_SPHERES_FIRST
#define RT_BVH4_SPHERES_FIRST 1
#endif

namespace rth {
constexpr uint32_t BVH4_TOP = 341;  // 1 + 4 + 16 + 64 + 256
// Collapses the two-box BVHs of a world into 4-wide nodes: starting from a
// node's two children, the inner child with the largest box (surface area) is
// replaced by its own children until there are four or no inner child is left
// (the usual top-down BVH2 -> BVH4 collapse).  Child boxes are the parents' f32
// boxes, already rounded outward.  filter_spheres (basic tier): sphere children
// become filter records and are queued, not stacked, so need(node) = (inner
// children - 1) + max need(inner child); otherwise (mesh tier) a sphere child
// gets its box rounded outward and, like every child, is walked near-first
// through the stack: need(node) = (children - 1) + max need(child).
uint32_t bvh4_convert(HostWorld& hw, uint32_t max_need, bool filter_spheres, size_t max_nodes) {
    using rtk::REF_NONE;
    struct Child {
        uint32_t ref;
        float lo[3], hi[3];
        double area;
    };
    std::vector<rtk::DNode4> out;
    std::vector<uint32_t> map(hw.nodes.size(), REF_NONE);
    auto kids = [&](uint32_t idx, std::vector<Child>& v) {
        const rtk::DNode& n = hw.nodes[idx];
        const uint32_t refs[2] = {n.c0, n.c1};
        for (int k = 0; k < 2; ++k) {
            if (refs[k] == REF_NONE) continue;
            Child c{};
            c.ref = refs[k];
            if (rtk::ref_kind(refs[k]) == rtk::K_SPHERE) {
                c.area = -1.0;
                const double* sp = n.slot[k].sphere;
                for (int a = 0; a < 3; ++a) {
                    c.lo[a] = round_down(sp[a] - sp[3]);
                    c.hi[a] = round_up(sp[a] + sp[3]);
                }
            } else {
                for (int a = 0; a < 3; ++a) {
                    c.lo[a] = n.slot[k].box.lo[a];
                    c.hi[a] = n.slot[k].box.hi[a];
                }
                const double dx = std::fmax((double)c.hi[0] - c.lo[0], 0.0), dy = std::fmax((double)c.hi[1] - c.lo[1], 0.0),
                             dz = std::fmax((double)c.hi[2] - c.lo[2], 0.0);
                c.area = dx * dy + dy * dz + dz * dx;
            }
            v.push_back(c);
        }
    };
    std::function<uint32_t(uint32_t)> conv = [&](uint32_t idx) -> uint32_t {
        if (map[idx] != REF_NONE) return map[idx];
        std::vector<Child> ch;
        kids(idx, ch);
        for (;;) {
            if (ch.size() >= 4) break;
            int best = -1;
            for (size_t i = 0; i < ch.size(); ++i)
                if (rtk::ref_kind(ch[i].ref) == rtk::K_BVH && (best < 0 || ch[i].area > ch[best].area)) best = (int)i;
            if (best < 0) break;
            std::vector<Child> sub;
            kids(rtk::ref_index(ch[best].ref), sub);
            ch.erase(ch.begin() + best);
            ch.insert(ch.begin() + best, sub.begin(), sub.end());
        }
#if RT_BVH4_SPHERES_FIRST
        // basic tier: sphere children in the low slots, boxes after them, empty
        // slots last -- a wave tests a slot's filter / slab only when one of its
        // lanes has that kind there (rt_kernel.hip visit4_rows); most leaf-level
        // nodes hold 2 or 3 spheres
        if (filter_spheres)
            std::stable_partition(ch.begin(), ch.end(),
                                  [](const Child& c) { return rtk::ref_kind(c.ref) == rtk::K_SPHERE; });
#endif
        const uint32_t at = (uint32_t)out.size();
        out.emplace_back();
        map[idx] = rtk::make_ref(rtk::K_BVH, at);
        rtk::DNode4 n{};
        for (int i = 0; i < 4; ++i) {
            n.ref[i] = REF_NONE;
            for (int a = 0; a < 3; ++a) {
                n.lo[a][i] = 1.0f;  // empty slot: inverted box, and masked by its REF_NONE
                n.hi[a][i] = 0.0f;
            }
        }
        for (size_t i = 0; i < ch.size(); ++i) {
            uint32_t r = ch[i].ref;
            if (filter_spheres && rtk::ref_kind(r) == rtk::K_SPHERE) {
                const double4 sp = hw.spheres[rtk::ref_index(r)];
                const float c[3] = {(float)sp.x, (float)sp.y, (float)sp.z}, rad = (float)sp.w;
                for (int a = 0; a < 3; ++a) n.lo[a][i] = c[a];
                n.hi[0][i] = rad;
                n.hi[1][i] = round_up(std::fabs((double)c[0]) + std::fabs((double)c[1]) + std::fabs((double)c[2]) +
                                      std::fabs((double)rad));
                n.hi[2][i] = 0.0f;
            } else {
                if (rtk::ref_kind(r) == rtk::K_BVH) r = conv(rtk::ref_index(r));
                for (int a = 0; a < 3; ++a) {
                    n.lo[a][i] = ch[i].lo[a];
                    n.hi[a][i] = ch[i].hi[a];
                }
            }
            n.ref[i] = r;
        }
        out[at] = n;
        return map[idx];
    };
    std::vector<uint32_t> lists = hw.list_children;
    for (uint32_t& r : lists)
        if (rtk::ref_kind(r) == rtk::K_BVH) r = conv(rtk::ref_index(r));
    uint32_t root = hw.world_root;
    if (rtk::ref_kind(root) == rtk::K_BVH) root = conv(rtk::ref_index(root));
    std::vector<rtk::DXform> xforms = hw.xforms;
    for (rtk::DXform& x : xforms)
        if (rtk::ref_kind(x.child) == rtk::K_BVH) x.child = conv(rtk::ref_index(x.child));
    std::vector<rtk::DMedium> media = hw.media;
    for (rtk::DMedium& m : media)
        if (rtk::ref_kind(m.boundary) == rtk::K_BVH) m.boundary = conv(rtk::ref_index(m.boundary));
    // stack need of a ref in the converted world
    std::unordered_map<uint32_t, uint32_t> memo;
    std::function<uint32_t(uint32_t)> need = [&](uint32_t r) -> uint32_t {
        const uint32_t kind = rtk::ref_kind(r), idx = rtk::ref_index(r);
        if (kind == rtk::K_XFORM) return 1 + need(xforms[idx].child);  // + its POPXF marker
        if (kind == rtk::K_MEDIUM) return need(media[idx].boundary);    // boundary walks from the same sp
        if (kind != rtk::K_BVH && kind != rtk::K_LIST) return 0;
        auto it = memo.find(r);
        if (it != memo.end()) return it->second;
        uint32_t v = 0;
        if (kind == rtk::K_BVH) {
            uint32_t inner = 0, deepest = 0;
            for (int i = 0; i < 4; ++i) {
                const uint32_t c = out[idx].ref[i];
                if (c == REF_NONE || (filter_spheres && rtk::ref_kind(c) == rtk::K_SPHERE)) continue;
                ++inner;
                deepest = std::max(deepest, need(c));
            }
            v = inner ? (inner - 1) + deepest : 0;
        } else {  // iterator form: popping (LIST,p) pushes (LIST,p+1) then walks child p
            for (uint32_t p = idx; lists[p] != REF_NONE; ++p) {
                const bool last = lists[p + 1] == REF_NONE;
                v = std::max(v, (last ? 0u : 1u) + need(lists[p]));
            }
        }
        memo[r] = v;
        return v;
    };
    const uint32_t sn = 1 + need(root);
    if (sn > max_need) return sn;
    if (out.size() > max_nodes) return UINT32_MAX;
    // (RT_BVH4_TOP_BFS=0: the build's depth-first order throughout -- an A/B
    // knob of the layout, read from the environment like rt_render.cpp's)
    const char* bfs_env = std::getenv("RT_BVH4_TOP_BFS");
    if (!filter_spheres && !(bfs_env && bfs_env[0] == '0')) {
        // the mesh / full tiers: the first BVH4_TOP nodes breadth-first from the
        // world's root BVH (levels 0-4 of a full 4-wide tree) take indices
        // 0 .. BVH4_TOP - 1, the rest keep the build's depth-first order after
        // them -- so that "index < K" names the top levels (the diagnostic
        // build's top-level step counts).  A layout only: the walk
        // visits the same nodes in the same order.
        std::vector<uint32_t> seeds;
        if (rtk::ref_kind(root) == rtk::K_BVH) seeds.push_back(rtk::ref_index(root));
        if (rtk::ref_kind(root) == rtk::K_LIST)
            for (uint32_t p = rtk::ref_index(root); lists[p] != REF_NONE; ++p)
                if (rtk::ref_kind(lists[p]) == rtk::K_BVH) seeds.push_back(rtk::ref_index(lists[p]));
        constexpr uint32_t UNPLACED = UINT32_MAX;  // (REF_NONE is 0: a valid index)
        std::vector<uint32_t> order, newidx(out.size(), UNPLACED);
        order.reserve(out.size());
        for (size_t head = 0; head < seeds.size() && order.size() < BVH4_TOP; ++head) {
            const uint32_t n = seeds[head];
            if (newidx[n] != UNPLACED) continue;
            newidx[n] = (uint32_t)order.size();
            order.push_back(n);
            for (int i = 0; i < 4; ++i)
                if (rtk::ref_kind(out[n].ref[i]) == rtk::K_BVH) seeds.push_back(rtk::ref_index(out[n].ref[i]));
        }
        for (uint32_t n = 0; n < (uint32_t)out.size(); ++n)
            if (newidx[n] == UNPLACED) newidx[n] = (uint32_t)order.size(), order.push_back(n);
        auto remap = [&](uint32_t& r) {
            if (rtk::ref_kind(r) == rtk::K_BVH) r = rtk::make_ref(rtk::K_BVH, newidx[rtk::ref_index(r)]);
        };
        std::vector<rtk::DNode4> perm(out.size());
        for (uint32_t k = 0; k < (uint32_t)order.size(); ++k) {
            perm[k] = out[order[k]];
            for (int i = 0; i < 4; ++i) remap(perm[k].ref[i]);
        }
        out.swap(perm);
        for (uint32_t& r : lists) remap(r);
        for (rtk::DXform& x : xforms) remap(x.child);
        for (rtk::DMedium& m : media) remap(m.boundary);
        remap(root);
    }
    hw.nodes4 = std::move(out);
    hw.nodes.clear();  // the two-box nodes are not walked any more
    hw.list_children = std::move(lists);
    hw.xforms = std::move(xforms);
    hw.media = std::move(media);
    hw.world_root = root;
    hw.stack_need = sn;
    return sn;
}

}  // namespace rth
