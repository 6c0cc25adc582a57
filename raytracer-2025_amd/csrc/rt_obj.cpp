// rt_obj.cpp -- Wavefont::new (src/shapes/obj.rs:117-134) for the C ABI:
// rt_wavefront_load.
//
// OBJ/MTL parsing restates what the reference gets from tobj 4.0.3 with
// GPU_LOAD_OPTIONS (obj.rs:93, 104): single_index (one vertex per distinct
// v/vt/vn triple, so positions/texcoords/normals share one index), triangulate
// (fan 0,i,i+1), a new model at every `o`/`g` and at every `usemtl` that
// changes the material of a model that already has faces.  tobj itself is not
// in this image (parity unpinned for the parser).  Reference
// behaviour kept on purpose:
//  - models are zipped with the MTL materials (obj.rs:129): only the first
//    min(#models, #materials) models are loaded;
//  - every face vertex must carry vt and vn (obj.rs:148-158 index them
//    unconditionally -> panic otherwise);
//  - degenerate triangles are skipped (obj.rs:185-187), an empty model adds
//    nothing (obj.rs:189-193);
//  - each triangle's material is a RemappedMaterial (obj.rs:20-81): the
//    shading normal is the normalised barycentric mix of the vertex normals and
//    (u, v) become texture coordinates.
#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <iterator>
#include <fstream>
#include <map>
#include <sstream>
#include <tuple>
#include <unordered_map>

#include "../../include/rt_mi355x.h"
#include "rt_scene.hpp"

using namespace rth;

namespace {

struct MtlRec {
    std::string name;
    bool has_diffuse = false;
    double diffuse[3] = {0, 0, 0};
    std::string diffuse_texture, normal_texture, dissolve_texture;
    bool has_ior = false, has_dissolve = false;
    double ior = 1.45, dissolve = 1.0;
    std::map<std::string, std::string> unknown;
};

std::string trim(const std::string& s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

bool parse_mtl(const std::string& path, std::vector<MtlRec>& out, std::string& err) {
    std::ifstream f(path);
    if (!f) {
        err = "cannot open MTL " + path;
        return false;
    }
    std::string line;
    while (std::getline(f, line)) {
        line = trim(line);
        if (line.empty() || line[0] == '#') continue;
        std::istringstream is(line);
        std::string key;
        is >> key;
        std::string rest;
        std::getline(is, rest);
        rest = trim(rest);
        if (key == "newmtl") {
            out.emplace_back();
            out.back().name = rest;
            continue;
        }
        if (out.empty()) continue;
        MtlRec& m = out.back();
        std::istringstream vs(rest);
        if (key == "Kd") {
            vs >> m.diffuse[0] >> m.diffuse[1] >> m.diffuse[2];
            m.has_diffuse = true;
        } else if (key == "Ni") {
            vs >> m.ior;
            m.has_ior = true;
        } else if (key == "d") {
            vs >> m.dissolve;
            m.has_dissolve = true;
        } else if (key == "map_Kd") {
            m.diffuse_texture = rest;
        } else if (key == "map_Bump" || key == "map_bump" || key == "bump" || key == "norm") {
            m.normal_texture = rest;
        } else if (key == "map_d") {
            m.dissolve_texture = rest;
        } else if (key == "Ka" || key == "Ks" || key == "Ns" || key == "illum" || key == "map_Ka" || key == "map_Ks" ||
                   key == "map_Ns") {
            // known to tobj, unused by obj.rs
        } else {
            m.unknown[key] = rest;
        }
    }
    return true;
}

// unknown_param.get(key).and_then(|s| s.parse::<f64>().ok()): the whole value must parse
double param_or(const MtlRec& m, const char* key, double def) {
    auto it = m.unknown.find(key);
    if (it == m.unknown.end() || it->second.empty()) return def;
    char* end = nullptr;
    double v = std::strtod(it->second.c_str(), &end);
    return *end == 0 ? v : def;
}
// split_whitespace().filter_map(|s| s.parse::<f64>().ok())
std::vector<double> params(const MtlRec& m, const char* key) {
    std::vector<double> v;
    auto it = m.unknown.find(key);
    if (it == m.unknown.end()) return v;
    std::istringstream is(it->second);
    std::string tok;
    while (is >> tok) {
        char* end = nullptr;
        double x = std::strtod(tok.c_str(), &end);
        if (*end == 0) v.push_back(x);
    }
    return v;
}
struct Corner {
    int64_t v, t, n;
    bool operator==(const Corner& o) const { return v == o.v && t == o.t && n == o.n; }
};
struct CornerHash {
    size_t operator()(const Corner& c) const {
        uint64_t h = (uint64_t)c.v * 0x9E3779B97F4A7C15ull;
        h ^= (uint64_t)c.t + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
        h ^= (uint64_t)c.n + 0x85EBCA77C2B2AE63ull + (h << 6) + (h >> 2);
        return (size_t)h;
    }
};
struct Model {
    std::string name;
    int material_id = -1;
    std::vector<int64_t> pos, tex, nrm;  // per single-index vertex: source indices
    std::vector<uint32_t> indices;       // triangles
    std::unordered_map<Corner, uint32_t, CornerHash> vmap;  // (v, vt, vn) -> vertex, first use numbers it
};

// The whitespace-separated words of one line, in place: each word is
// NUL-terminated in the (mutable) line buffer.
struct Words {
    char* p;
    char* end;
    char* next() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\f' || *p == '\v')) ++p;
        if (p >= end) return nullptr;
        char* w = p;
        while (p < end && !(*p == ' ' || *p == '\t' || *p == '\r' || *p == '\f' || *p == '\v')) ++p;
        if (p < end) *p++ = 0;
        else *p = 0;  // the buffer keeps one byte past every line
        return w;
    }
    // the rest of the line, trimmed
    std::string rest() {
        while (p < end && (*p == ' ' || *p == '\t')) ++p;
        char* e = end;
        while (e > p && (e[-1] == ' ' || e[-1] == '\t' || e[-1] == '\r' || e[-1] == '\f' || e[-1] == '\v')) --e;
        return std::string(p, (size_t)(e - p));
    }
};
// f64::from_str on one word: the whole word must parse
bool parse_f64(const char* w, double& x) {
    if (!w) return false;
    char* e = nullptr;
    x = std::strtod(w, &e);
    return e != w && *e == 0;
}
// a face index (std::stoll semantics: leading digits, error when there are none)
int64_t parse_index(const char* b, const char* e) {
    char buf[32];
    const size_t n = std::min<size_t>((size_t)(e - b), sizeof buf - 1);
    std::memcpy(buf, b, n);
    buf[n] = 0;
    char* end = nullptr;
    errno = 0;
    const long long v = std::strtoll(buf, &end, 10);
    if (end == buf) throw std::invalid_argument("face index '" + std::string(buf) + "'");
    if (errno == ERANGE) throw std::out_of_range("face index '" + std::string(buf) + "'");
    return v;
}

}  // namespace

extern "C" int32_t rt_wavefront_load(rt_scene* s, const char* obj_path, int32_t vanilla) {
    if (!s || !obj_path) return set_error(RT_EINVAL, "null argument");
    try {
        std::ifstream f(obj_path, std::ios::binary);
        if (!f) return set_error(RT_EINVAL, std::string("cannot open OBJ ") + obj_path);
        // the whole file, parsed in place line by line (1M-triangle OBJs: a
        // stream extraction per word took ~3 s)
        std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        text.push_back('\n');
        text.push_back(0);
        std::string path(obj_path);
        std::string dir = path.find('/') == std::string::npos ? "." : path.substr(0, path.rfind('/'));
        std::vector<double> P, T, N;  // v / vt / vn
        std::vector<Model> models(1);
        std::vector<MtlRec> mtls;
        std::unordered_map<std::string, int> mtl_index;
        bool mtl_failed = false;  // materials: Err(..) -> `if let Ok` skips them (obj.rs:124-126)
        auto finish_model = [&](const std::string& next_name) {
            Model& cur = models.back();
            if (!cur.indices.empty()) {
                Model nm;
                nm.name = next_name;
                nm.material_id = cur.material_id;
                models.push_back(std::move(nm));
            } else {
                cur.name = next_name;
            }
        };
        auto resolve = [](int64_t i, size_t n) -> int64_t { return i < 0 ? (int64_t)n + i : i - 1; };
        std::vector<uint32_t> face;
        char* const text_end = &text[text.size() - 1];  // the final NUL
        for (char* line = &text[0]; line < text_end;) {
            char* eol = (char*)std::memchr(line, '\n', (size_t)(text_end - line));
            if (!eol) eol = text_end;
            char* next_line = eol + 1;
            char* hash = (char*)std::memchr(line, '#', (size_t)(eol - line));
            Words is{line, hash ? hash : eol};
            line = next_line;
            const char* key = is.next();
            if (!key) continue;
            if (key[0] == 'v' && (key[1] == 0 || (key[2] == 0 && (key[1] == 't' || key[1] == 'n')))) {
                double x[3] = {0, 0, 0};
                if (key[1] == 't') {  // vt u [v]: missing values read as 0
                    double u;
                    if (parse_f64(is.next(), u)) {
                        x[0] = u;
                        if (parse_f64(is.next(), u)) x[1] = u;
                    }
                    T.insert(T.end(), {x[0], x[1]});
                    continue;
                }
                for (int k = 0; k < 3; ++k)
                    if (!parse_f64(is.next(), x[k]))  // tobj: PositionParseError / NormalParseError
                        return set_error(RT_EPANIC, std::string("OBJ ") + (key[1] ? "normal" : "position") +
                                                        " parse error (Wavefont::new expects the load to succeed)");
                (key[1] ? N : P).insert((key[1] ? N : P).end(), {x[0], x[1], x[2]});
            } else if (!std::strcmp(key, "o") || !std::strcmp(key, "g")) {
                finish_model(is.rest());
            } else if (!std::strcmp(key, "mtllib")) {
                std::string err;
                if (!parse_mtl(dir + "/" + is.rest(), mtls, err)) mtl_failed = true;
                mtl_index.clear();
                for (size_t i = 0; i < mtls.size(); ++i) mtl_index[mtls[i].name] = (int)i;
            } else if (!std::strcmp(key, "usemtl")) {
                auto it = mtl_index.find(is.rest());
                int id = it == mtl_index.end() ? -1 : it->second;
                Model& cur = models.back();
                if (!cur.indices.empty() && cur.material_id != id) {
                    Model nm;
                    nm.name = cur.name;
                    models.push_back(std::move(nm));
                }
                models.back().material_id = id;
            } else if (!std::strcmp(key, "f")) {
                face.clear();
                Model& m = models.back();
                while (const char* tok = is.next()) {
                    int64_t ti = INT64_MIN, ni = INT64_MIN;
                    const char* tend = tok + std::strlen(tok);
                    const char* a = std::strchr(tok, '/');
                    const int64_t vi = resolve(parse_index(tok, a ? a : tend), P.size() / 3);
                    if (a) {
                        const char* b = std::strchr(a + 1, '/');
                        const char* te = b ? b : tend;
                        if (te > a + 1) ti = resolve(parse_index(a + 1, te), T.size() / 2);
                        if (b && b + 1 < tend) ni = resolve(parse_index(b + 1, tend), N.size() / 3);
                    }
                    const Corner key3{vi, ti, ni};
                    auto ins = m.vmap.emplace(key3, (uint32_t)m.pos.size());
                    if (ins.second) {
                        m.pos.push_back(vi);
                        m.tex.push_back(ti);
                        m.nrm.push_back(ni);
                    }
                    face.push_back(ins.first->second);
                }
                for (size_t i = 1; i + 1 < face.size(); ++i) m.indices.insert(m.indices.end(), {face[0], face[i], face[i + 1]});
            }
        }
        if (models.back().indices.empty() && models.size() > 1) models.pop_back();

        if (mtl_failed) mtls.clear();
        // load_materials (obj.rs:212-345)
        std::vector<int32_t> mats, normal_maps;
        // ImageTexture::new(prefix/file) / new_raw_image: decoded once per
        // (file, raw, interpolation) and shared (a missing file reads as cyan)
        std::map<std::tuple<std::string, int, int>, int32_t> images;
        auto image_tex = [&](const std::string& file, bool raw, bool linear) -> int32_t {
            auto key = std::make_tuple(file, (int)raw, (int)linear);
            auto it = images.find(key);
            if (it != images.end()) return it->second;
            const int32_t h = rt_tex_image_file(s, (dir + "/" + file).c_str(), raw, linear);
            if (h >= 0) images[key] = h;
            return h;
        };
        for (const MtlRec& m : mtls) {
            int32_t base_tex;
            if (!m.diffuse_texture.empty()) {
                base_tex = image_tex(m.diffuse_texture, false, false);
                if (base_tex < 0) return base_tex;
            } else if (m.has_diffuse) {
                base_tex = rt_tex_solid(s, m.diffuse);
            } else {
                return set_error(RT_EPANIC, "The material should at least have one diffuse!");
            }
            const double roughness = param_or(m, "Pr", 0.5), metallic = param_or(m, "Pm", 0.0);
            const double ior = m.has_ior ? m.ior : 1.45;
            std::vector<double> tf = params(m, "Tf");
            double spec_trans = 0.0;
            if (m.unknown.count("Tf")) {  // empty -> 0/0 = NaN, as the reference
                double sum = 0;
                for (double x : tf) sum += x;
                spec_trans = sum / (double)tf.size();
            }
            int32_t mat;
            if (vanilla && metallic == 1.0) {
                // Metal::new(base_color.value(0, 0, ZERO), Pr): an image's pixel
                // at u = 0, v = 0 -> (0, height) clamped to the last row
                // (texture.rs:109-118, image.rs:63-82); a missing one is cyan
                const TexRec& t = s->texs[base_tex];
                double albedo[3] = {0.0, 1.0, 1.0};
                if (t.type == rtk::T_SOLID) {
                    for (int k = 0; k < 3; ++k) albedo[k] = t.color[k];
                } else if (t.h != 0) {
                    const float* px = &s->texels[t.texel_offset + (size_t)(t.h - 1) * t.w * 4];
                    for (int k = 0; k < 3; ++k) albedo[k] = (double)px[k];
                }
                mat = rt_mat_metal(s, albedo, roughness);
            } else if (vanilla && spec_trans == 1.0) {
                mat = rt_mat_dielectric(s, base_tex, ior);
            } else {
                return set_error(RT_EUNSUPPORTED, "Disney BSDF materials (obj.rs:299-311) are not on the kernel path");
            }
            std::vector<double> ke = params(m, "Ke");
            if (ke.size() == 3) mat = rt_mat_diffuse_light(s, rt_tex_solid(s, ke.data()), mat);
            if (m.unknown.count("map_Ke")) {  // obj.rs:319-323
                const int32_t et = image_tex(m.unknown.at("map_Ke"), false, false);
                if (et < 0) return et;
                mat = rt_mat_diffuse_light(s, et, mat);
            }
            if (!m.dissolve_texture.empty()) {  // obj.rs:325-332: Mix::from_image(Transparent, mat, tex)
                const int32_t dt = image_tex(m.dissolve_texture, false, false);
                if (dt < 0) return dt;
                mat = rt_mat_mix_image(s, rt_mat_transparent(s), mat, dt);
            }
            if (m.has_dissolve && m.dissolve < 1.0) mat = rt_mat_mix(s, rt_mat_transparent(s), mat, m.dissolve);
            if (mat < 0) return mat;
            mats.push_back(mat);
            // normal map (obj.rs:324-343): "file" or "-bm <scale> file" -> prefix/file,
            // ImageTexture::new_raw_image; a missing file reads as cyan
            int32_t ntex = -1;
            if (!m.normal_texture.empty()) {
                std::string name = m.normal_texture;
                if (name.compare(0, 3, "-bm") == 0) {
                    std::istringstream is(name.substr(3));
                    std::string part, last;
                    while (is >> part) last = part;
                    if (!last.empty()) name = last;
                }
                ntex = image_tex(name, true, true);
                if (ntex < 0) return ntex;
            }
            normal_maps.push_back(ntex);
        }

        int32_t objs = rt_hittables_new(s);
        const int32_t empty = mats.empty() ? -1 : rt_mat_empty(s);
        const size_t nload = std::min(models.size(), mtls.size());  // zip (obj.rs:129)
        {  // room for every triangle and its model's BVH nodes (about one per triangle) up front
            size_t ntri = 0;
            for (size_t mi = 0; mi < nload; ++mi) ntri += models[mi].indices.size() / 3;
            s->objs.reserve(s->objs.size() + 2 * ntri + 2 * nload + 1);
        }
        for (size_t mi = 0; mi < nload; ++mi) {
            const Model& m = models[mi];
            int32_t list = rt_hittables_new(s);
            size_t added = 0;
            const int32_t base = m.material_id >= 0 ? mats[m.material_id] : empty;
            for (size_t k = 0; k + 2 < m.indices.size(); k += 3) {
                uint32_t id[3] = {m.indices[k], m.indices[k + 1], m.indices[k + 2]};
                V3 p[3], n[3];
                double tc[3][2];
                for (int j = 0; j < 3; ++j) {
                    if (m.tex[id[j]] == INT64_MIN || m.nrm[id[j]] == INT64_MIN)
                        return set_error(RT_EPANIC, "index out of bounds: face vertex without vt/vn (obj.rs:148-158)");
                    const int64_t pi = m.pos[id[j]], ti = m.tex[id[j]], ni = m.nrm[id[j]];
                    if (pi < 0 || (size_t)pi * 3 + 2 >= P.size() || ti < 0 || (size_t)ti * 2 + 1 >= T.size() || ni < 0 ||
                        (size_t)ni * 3 + 2 >= N.size())
                        return set_error(RT_EPANIC, "index out of bounds in OBJ face");
                    p[j] = V3(&P[pi * 3]);
                    n[j] = V3(&N[ni * 3]);
                    tc[j][0] = T[ti * 2];
                    tc[j][1] = T[ti * 2 + 1];
                }
                V3 wu = p[1] - p[0], wv = p[2] - p[0];
                double a[3] = {p[0].x, p[0].y, p[0].z}, u[3] = {wu.x, wu.y, wu.z}, v[3] = {wv.x, wv.y, wv.z};
                int32_t tri = rt_triangle(s, a, u, v, base);
                if (tri == RT_EDEGENERATE) continue;
                if (tri < 0) return tri;
                Obj& o = s->objs[tri];
                o.remap = true;
                for (int j = 0; j < 3; ++j) o.rn[j] = n[j];
                o.tex_ori[0] = tc[0][0];
                o.tex_ori[1] = tc[0][1];
                o.tex_u[0] = tc[1][0] - tc[0][0];
                o.tex_u[1] = tc[1][1] - tc[0][1];
                o.tex_v[0] = tc[2][0] - tc[0][0];
                o.tex_v[1] = tc[2][1] - tc[0][1];
                o.normal_tex = normal_maps[mi];
                if (o.normal_tex >= 0) {
                    // uv_local_to_world (obj.rs:196-210)
                    const double tux = o.tex_u[0], tuy = o.tex_u[1], tvx = o.tex_v[0], tvy = o.tex_v[1];
                    const double ua = tvy / (-tuy * tvx + tux * tvy);
                    const double ub = tuy / (tuy * tvx - tux * tvy);
                    const double va = tvx / (tuy * tvx - tux * tvy);
                    const double vb = tux / (-tuy * tvx + tux * tvy);
                    const V3 uw = ua * wu + ub * wv, vw = va * wu + vb * wv;
                    const V3 un = div(uw, length(uw)), vn = div(vw, length(vw));
                    o.uv_ok = finite(un) && finite(vn);  // else .unwrap() panics when shaded
                    o.u_vec = un;
                    o.v_vec = vn;
                }
                rt_hittables_add(s, list, tri);
                ++added;
            }
            if (added) {
                int32_t bvh = rt_bvh_new(s, list);  // BVH::from_vec (obj.rs:190)
                if (bvh < 0) return bvh;
                rt_hittables_add(s, objs, bvh);
            }
        }
        return objs;
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    } catch (const std::exception& e) {
        return set_error(RT_EINVAL, std::string("OBJ parse error: ") + e.what());
    }
}
