// oracle/rt_oracle_obj.cpp -- TEST INFRASTRUCTURE ONLY.
//
// What the reference gets from `tobj::load_obj(path, &tobj::GPU_LOAD_OPTIONS)`
// (shapes/obj.rs:86-104; tobj 4.0.3 with features = ["use_f64"], Cargo.toml:13),
// restated from tobj's published behaviour because tobj is not in this image
// (parity of the parser itself is unpinned):
//  - `v`/`vt`/`vn` append to global f64 lists; `f` corners are `v`, `v/vt`,
//    `v//vn` or `v/vt/vn`, 1-based or negative (relative to the list so far);
//  - single_index: within one model every distinct (v, vt, vn) corner becomes
//    one vertex, numbered in first-use order, positions/texcoords/normals
//    copied per vertex;
//  - triangulate: a polygon (c0..cn-1) becomes the fan (c0, ci, ci+1);
//  - `o`/`g` close the current model when it has faces and rename;
//    `usemtl` closes it when it has faces and the material changes, the new
//    model keeping the name; the material id carries over `o`/`g`;
//  - `mtllib` loads the MTL next to the OBJ; any MTL failure makes the whole
//    material list Err (which obj.rs:124 then ignores).
// The MTL keys obj.rs reads: Kd, Ni, d, map_Kd, map_Bump/map_bump/bump (normal
// texture), map_d; everything tobj does not know goes to unknown_param
// (Pr, Pm, Tf, Ke, map_Ke, ...), value = rest of the line, trimmed.
#include <climits>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#include "rt_oracle.hpp"

namespace orc {

namespace {

std::string strip(const std::string& s) {
    const char* ws = " \t\r\n";
    const size_t b = s.find_first_not_of(ws);
    if (b == std::string::npos) return "";
    return s.substr(b, s.find_last_not_of(ws) - b + 1);
}

// key = first whitespace-delimited word, rest = remainder trimmed
void split_key(const std::string& line, std::string& key, std::string& rest) {
    const size_t e = line.find_first_of(" \t");
    key = line.substr(0, e);
    rest = e == std::string::npos ? "" : strip(line.substr(e));
}

std::vector<double> numbers(const std::string& rest) {
    std::vector<double> out;
    std::istringstream is(rest);
    std::string w;
    while (is >> w) out.push_back(std::stod(w));
    return out;
}

bool load_mtl(const std::string& path, std::vector<ObjMaterial>& mats) {
    std::ifstream in(path);
    if (!in) return false;
    std::string line, key, rest;
    ObjMaterial* cur = nullptr;
    while (std::getline(in, line)) {
        line = strip(line);
        if (line.empty() || line[0] == '#') continue;
        split_key(line, key, rest);
        if (key == "newmtl") {
            mats.push_back(ObjMaterial{});
            cur = &mats.back();
            cur->name = rest;
            continue;
        }
        if (!cur) continue;
        if (key == "Kd") {
            std::vector<double> v = numbers(rest);
            if (v.size() < 3) return false;
            cur->diffuse = Vec3(v[0], v[1], v[2]);
            cur->has_diffuse = true;
        } else if (key == "Ni") {
            cur->optical_density = std::stod(rest);
            cur->has_optical_density = true;
        } else if (key == "d") {
            cur->dissolve = std::stod(rest);
            cur->has_dissolve = true;
        } else if (key == "map_Kd") {
            cur->diffuse_texture = rest;
        } else if (key == "map_Bump" || key == "map_bump" || key == "bump" || key == "norm") {
            cur->normal_texture = rest;
        } else if (key == "map_d") {
            cur->dissolve_texture = rest;
        } else if (key == "Ka" || key == "Ks" || key == "Ns" || key == "illum" || key == "map_Ka" ||
                   key == "map_Ks" || key == "map_Ns") {
            // parsed by tobj, not read by obj.rs
        } else {
            cur->unknown_param[key] = rest;
        }
    }
    return true;
}

struct Corner {
    long long v, vt, vn;
    bool operator<(const Corner& o) const {
        return v != o.v ? v < o.v : (vt != o.vt ? vt < o.vt : vn < o.vn);
    }
};

long long to_index(const std::string& s, size_t count) {
    const long long i = std::stoll(s);
    return i < 0 ? (long long)count + i : i - 1;
}

}  // namespace

ObjFile load_obj_file(const std::string& path) {
    std::ifstream in(path);
    if (!in) throw std::invalid_argument("OpenFileFailed: " + path);  // Wavefont::new -> None
    const size_t slash = path.rfind('/');
    const std::string dir = slash == std::string::npos ? "." : path.substr(0, slash);

    std::vector<double> pos, tex, nrm;
    ObjFile out;
    bool mtl_ok = true;
    std::map<std::string, int> mat_by_name;

    // the model being read
    std::string name = "unnamed";
    int mat_id = -1;
    std::vector<std::vector<Corner>> faces;

    auto export_model = [&]() {
        ObjModel m;
        m.name = name;
        m.material_id = mat_id;
        std::map<Corner, uint32_t> seen;
        for (const auto& face : faces) {
            std::vector<uint32_t> ids;
            for (const Corner& c : face) {
                auto it = seen.find(c);
                if (it != seen.end()) {
                    ids.push_back(it->second);
                    continue;
                }
                const uint32_t id = (uint32_t)seen.size();
                seen.emplace(c, id);
                ids.push_back(id);
                if (c.v < 0 || (size_t)(c.v * 3 + 2) >= pos.size()) throw Panic("FaceVertexOutOfBounds");
                for (int k = 0; k < 3; ++k) m.positions.push_back(pos[c.v * 3 + k]);
                if (c.vt != LLONG_MIN) {
                    if (c.vt < 0 || (size_t)(c.vt * 2 + 1) >= tex.size()) throw Panic("FaceTexCoordOutOfBounds");
                    for (int k = 0; k < 2; ++k) m.texcoords.push_back(tex[c.vt * 2 + k]);
                }
                if (c.vn != LLONG_MIN) {
                    if (c.vn < 0 || (size_t)(c.vn * 3 + 2) >= nrm.size()) throw Panic("FaceNormalOutOfBounds");
                    for (int k = 0; k < 3; ++k) m.normals.push_back(nrm[c.vn * 3 + k]);
                }
            }
            for (size_t i = 1; i + 1 < ids.size(); ++i) {
                m.indices.push_back(ids[0]);
                m.indices.push_back(ids[i]);
                m.indices.push_back(ids[i + 1]);
            }
        }
        out.models.push_back(std::move(m));
        faces.clear();
    };

    std::string line, key, rest;
    while (std::getline(in, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line.erase(hash);
        line = strip(line);
        if (line.empty()) continue;
        split_key(line, key, rest);
        if (key == "v") {
            std::vector<double> v = numbers(rest);
            for (int k = 0; k < 3; ++k) pos.push_back(v.at(k));
        } else if (key == "vt") {
            std::vector<double> v = numbers(rest);
            tex.push_back(v.size() > 0 ? v[0] : 0.0);
            tex.push_back(v.size() > 1 ? v[1] : 0.0);
        } else if (key == "vn") {
            std::vector<double> v = numbers(rest);
            for (int k = 0; k < 3; ++k) nrm.push_back(v.at(k));
        } else if (key == "f") {
            std::istringstream is(rest);
            std::string w;
            std::vector<Corner> face;
            while (is >> w) {
                Corner c{0, LLONG_MIN, LLONG_MIN};
                const size_t s1 = w.find('/');
                c.v = to_index(w.substr(0, s1), pos.size() / 3);
                if (s1 != std::string::npos) {
                    const size_t s2 = w.find('/', s1 + 1);
                    const std::string a = w.substr(s1 + 1, s2 == std::string::npos ? std::string::npos : s2 - s1 - 1);
                    if (!a.empty()) c.vt = to_index(a, tex.size() / 2);
                    if (s2 != std::string::npos && s2 + 1 < w.size()) c.vn = to_index(w.substr(s2 + 1), nrm.size() / 3);
                }
                face.push_back(c);
            }
            faces.push_back(std::move(face));
        } else if (key == "o" || key == "g") {
            if (!faces.empty()) export_model();
            name = rest.empty() ? "unnamed" : rest;
        } else if (key == "mtllib") {
            if (!load_mtl(dir + "/" + rest, out.materials)) mtl_ok = false;
            for (size_t i = 0; i < out.materials.size(); ++i) mat_by_name[out.materials[i].name] = (int)i;
        } else if (key == "usemtl") {
            auto it = mat_by_name.find(rest);
            const int id = it == mat_by_name.end() ? -1 : it->second;
            if (id != mat_id && !faces.empty()) export_model();
            mat_id = id;
        }
    }
    if (!faces.empty()) export_model();
    out.materials_ok = mtl_ok;
    if (!mtl_ok) out.materials.clear();
    return out;
}

}  // namespace orc
