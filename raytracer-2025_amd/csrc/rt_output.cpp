// rt_output.cpp -- the output side of the path behind the C ABI:
//   rt_write_png        img.save("output/<dir>/<name>.png") with its
//                       create_dir_all (main.rs:39-47; image 0.25 PNG encoder)
//   rt_camera_from_json Camera::from_json / load_from_path (camera.rs:33-43,
//                       119-159; serde_json)
// PNG: 8-bit RGB, filter 0, zlib "stored" deflate blocks with Adler-32, CRC-32
// per chunk -- a valid PNG any decoder reads back to the same bytes (the
// reference's compressed byte stream is not reproduced; pixels are).
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_scene.hpp"

using namespace rth;

namespace {

uint32_t crc_table[256];
bool crc_ready = false;
uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    if (!crc_ready) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t v = i;
            for (int k = 0; k < 8; ++k) v = (v & 1u) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
            crc_table[i] = v;
        }
        crc_ready = true;
    }
    for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    return c;
}

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t>& png, const char type[4], const std::vector<uint8_t>& data) {
    put_be32(png, (uint32_t)data.size());
    const size_t start = png.size();
    png.insert(png.end(), type, type + 4);
    png.insert(png.end(), data.begin(), data.end());
    put_be32(png, crc32(png.data() + start, png.size() - start) ^ 0xFFFFFFFFu);
}

int mkdirs(const std::string& dir) {  // std::fs::create_dir_all
    if (dir.empty()) return 0;
    std::string cur;
    std::stringstream ss(dir);
    std::string part;
    if (dir[0] == '/') cur = "/";
    while (std::getline(ss, part, '/')) {
        if (part.empty()) continue;
        cur += part;
        if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
        cur += "/";
    }
    return 0;
}

// ---- a small JSON reader for the CameraParams schema (serde_json semantics:
// unknown keys ignored, every field required, numbers typed)
struct Json {
    const char* p;
    const char* end;
    std::string err;
    void ws() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool lit(const char* s) {
        size_t n = std::strlen(s);
        if ((size_t)(end - p) >= n && std::strncmp(p, s, n) == 0) {
            p += n;
            return true;
        }
        return false;
    }
    bool string(std::string& out) {
        ws();
        if (p >= end || *p != '"') return fail("expected string");
        ++p;
        out.clear();
        while (p < end && *p != '"') {
            if (*p == '\\') {
                ++p;
                if (p >= end) return fail("bad escape");
                const char c = *p;
                out.push_back(c == 'n' ? '\n' : c == 't' ? '\t' : c);
                if (c == 'u') p += 4;  // key names are ASCII in this schema
            } else {
                out.push_back(*p);
            }
            ++p;
        }
        if (p >= end) return fail("unterminated string");
        ++p;
        return true;
    }
    bool number(double& out, bool& integral) {
        ws();
        const char* s = p;
        if (p < end && (*p == '-' || *p == '+')) ++p;
        integral = true;
        while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '-' || *p == '+')) {
            if (*p == '.' || *p == 'e' || *p == 'E') integral = false;
            ++p;
        }
        if (p == s) return fail("expected number");
        out = std::strtod(std::string(s, p).c_str(), nullptr);
        return true;
    }
    bool skip() {  // any value
        ws();
        if (p >= end) return fail("unexpected end");
        if (*p == '"') {
            std::string t;
            return string(t);
        }
        if (*p == '{' || *p == '[') {
            const char close = *p == '{' ? '}' : ']';
            const bool obj = *p == '{';
            ++p;
            ws();
            if (p < end && *p == close) {
                ++p;
                return true;
            }
            for (;;) {
                if (obj) {
                    std::string k;
                    if (!string(k)) return false;
                    ws();
                    if (p >= end || *p != ':') return fail("expected ':'");
                    ++p;
                }
                if (!skip()) return false;
                ws();
                if (p < end && *p == ',') {
                    ++p;
                    continue;
                }
                if (p < end && *p == close) {
                    ++p;
                    return true;
                }
                return fail("expected ',' or close");
            }
        }
        if (lit("true") || lit("false") || lit("null")) return true;
        double d;
        bool i;
        return number(d, i);
    }
    bool vec3(double out[3]) {  // Vec3 deserializes from [f64; 3] (vec3.rs:26-34)
        ws();
        if (p >= end || *p != '[') return fail("expected [x, y, z]");
        ++p;
        for (int k = 0; k < 3; ++k) {
            bool i;
            if (!number(out[k], i)) return false;
            ws();
            if (k < 2) {
                if (p >= end || *p != ',') return fail("expected 3 numbers");
                ++p;
            }
        }
        ws();
        if (p >= end || *p != ']') return fail("expected 3 numbers");
        ++p;
        return true;
    }
    bool fail(const char* m) {
        if (err.empty()) err = m;
        return false;
    }
};

}  // namespace

extern "C" int32_t rt_write_png(const char* path, uint32_t width, uint32_t height, const uint8_t* rgb) {
    if (!path || (!rgb && width && height)) return set_error(RT_EINVAL, "null argument");
    if (width == 0 || height == 0) return set_error(RT_EINVAL, "zero-sized image");
    try {
        std::string ps(path);
        const size_t slash = ps.rfind('/');
        if (slash != std::string::npos && mkdirs(ps.substr(0, slash)) != 0)
            return set_error(RT_EINVAL, "Cannot create all the parents");  // main.rs:43 expect
        std::vector<uint8_t> raw;
        raw.reserve((size_t)height * (1 + (size_t)width * 3));
        for (uint32_t y = 0; y < height; ++y) {
            raw.push_back(0);  // filter: none
            raw.insert(raw.end(), rgb + (size_t)y * width * 3, rgb + (size_t)(y + 1) * width * 3);
        }
        std::vector<uint8_t> z = {0x78, 0x01};
        uint32_t a = 1, b = 0;
        for (uint8_t c : raw) {
            a = (a + c) % 65521u;
            b = (b + a) % 65521u;
        }
        for (size_t off = 0; off < raw.size() || off == 0;) {
            const size_t n = std::min<size_t>(65535, raw.size() - off);
            const bool last = off + n == raw.size();
            z.push_back(last ? 1 : 0);
            z.push_back((uint8_t)(n & 0xFF));
            z.push_back((uint8_t)(n >> 8));
            z.push_back((uint8_t)(~n & 0xFF));
            z.push_back((uint8_t)((~n >> 8) & 0xFF));
            z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
            off += n;
            if (last) break;
        }
        put_be32(z, (b << 16) | a);
        std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
        std::vector<uint8_t> ihdr;
        put_be32(ihdr, width);
        put_be32(ihdr, height);
        ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, RGB, deflate, filter 0, no interlace
        chunk(png, "IHDR", ihdr);
        chunk(png, "IDAT", z);
        chunk(png, "IEND", {});
        std::ofstream f(ps, std::ios::binary);
        if (!f) return set_error(RT_EINVAL, "Cannot save the image to the file");  // main.rs:47 expect
        f.write((const char*)png.data(), (std::streamsize)png.size());
        return f ? RT_OK : set_error(RT_EINVAL, "Cannot save the image to the file");
    } catch (const std::bad_alloc&) {
        return set_error(RT_ENOMEM, "out of host memory");
    }
}

extern "C" int32_t rt_camera_from_json(const char* path, rt_camera* cam) {
    if (!path || !cam) return set_error(RT_EINVAL, "null argument");
    std::ifstream f(path, std::ios::binary);
    if (!f) return set_error(RT_EINVAL, std::string("cannot open ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    Json J{text.data(), text.data() + text.size(), {}};
    rt_camera c;
    rt_camera_default(&c);  // ..Default::default() (camera.rs:156)
    enum { AR = 1, IW = 2, FOV = 4, LF = 8, LA = 16, UP = 32, DEF = 64, FD = 128, ALL = 255 };
    int seen = 0;
    J.ws();
    if (J.p >= J.end || *J.p != '{') return set_error(RT_EINVAL, "camera JSON: expected an object");
    ++J.p;
    J.ws();
    bool ok = true;
    if (J.p < J.end && *J.p == '}') {
        ++J.p;
    } else {
        for (;;) {
            std::string key;
            if (!(ok = J.string(key))) break;
            J.ws();
            if (J.p >= J.end || *J.p != ':') {
                ok = J.fail("expected ':'");
                break;
            }
            ++J.p;
            double v;
            bool integral;
            if (key == "aspect_ratio") {
                ok = J.number(c.aspect_ratio, integral), seen |= AR;
            } else if (key == "image_width") {
                ok = J.number(v, integral) && (integral && v >= 0 && v <= 4294967295.0 ? true : J.fail("image_width: u32"));
                c.image_width = (uint32_t)v;
                seen |= IW;
            } else if (key == "vertical_fov_in_degrees") {
                ok = J.number(c.vertical_fov_in_degrees, integral), seen |= FOV;
            } else if (key == "look_from") {
                ok = J.vec3(c.look_from), seen |= LF;
            } else if (key == "look_at") {
                ok = J.vec3(c.look_at), seen |= LA;
            } else if (key == "vec_up") {
                ok = J.vec3(c.vec_up), seen |= UP;
            } else if (key == "defocus_angle_in_degrees") {
                ok = J.number(c.defocus_angle_in_degrees, integral), seen |= DEF;
            } else if (key == "focus_distance") {
                ok = J.number(c.focus_distance, integral), seen |= FD;
            } else {
                ok = J.skip();  // serde ignores unknown fields
            }
            if (!ok) break;
            J.ws();
            if (J.p < J.end && *J.p == ',') {
                ++J.p;
                continue;
            }
            if (J.p < J.end && *J.p == '}') {
                ++J.p;
                break;
            }
            ok = J.fail("expected ',' or '}'");
            break;
        }
    }
    if (!ok) return set_error(RT_EINVAL, "camera JSON: " + J.err);
    if (seen != ALL) return set_error(RT_EINVAL, "camera JSON: missing field");
    J.ws();
    if (J.p != J.end) return set_error(RT_EINVAL, "camera JSON: trailing characters");
    *cam = c;
    return RT_OK;
}
