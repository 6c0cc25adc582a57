// rt_hdr.hpp -- Radiance RGBE (.hdr) decoding for ImageTexture (host only).
//
// The reference's Image keeps HDR pixels linear -- pixel_data returns them
// raw whatever the texture's `raw` flag (utils/image.rs:76-80) -- after the
// `image` crate 0.25.6 decoded them (codecs/hdr): a "#?RADIANCE" signature,
// header lines up to an empty one (FORMAT must be 32-bit_rle_rgbe), the
// "-Y h +X w" resolution line, then scanlines flat, old-style RLE or
// new-style (2, 2, w) per-channel RLE; an RGBE pixel becomes
// c * 2^(e - 136) per channel (0 when e = 0), alpha 1.  The crate's source is
// not in the reference mount, so this restatement is parity unpinned;
// tests/test_jpeg_cpu.py checks it on files it writes in every scanline
// encoding.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace rthdr {

enum Status { OK = 0, CORRUPT = 2, UNSUPPORTED = 3 };  // UNSUPPORTED: a library limit

inline float rgbe_channel(uint8_t c, uint8_t e) { return e ? std::ldexp((float)c, (int)e - 136) : 0.0f; }

inline Status decode(const std::vector<uint8_t>& f, uint32_t& W, uint32_t& H, std::vector<float>& rgba, std::string& err) {
    W = H = 0;
    rgba.clear();
    size_t pos = 0;
    auto line = [&](std::string& s) -> bool {
        s.clear();
        while (pos < f.size() && f[pos] != '\n') s.push_back((char)f[pos++]);
        if (pos >= f.size()) return false;
        ++pos;
        return true;
    };
    std::string s;
    if (!line(s) || s.compare(0, 10, "#?RADIANCE") != 0) {
        err = "not a Radiance HDR file";
        return CORRUPT;
    }
    for (;;) {
        if (!line(s)) {
            err = "truncated HDR header";
            return CORRUPT;
        }
        if (s.empty()) break;
        if (s.compare(0, 7, "FORMAT=") == 0 && s.substr(7) != "32-bit_rle_rgbe") {
            err = "HDR format other than 32-bit_rle_rgbe";
            return CORRUPT;
        }
    }
    if (!line(s)) {
        err = "missing HDR resolution";
        return CORRUPT;
    }
    long h = 0, w = 0;
    char ya[3] = {}, xa[3] = {};
    if (std::sscanf(s.c_str(), "%2s %ld %2s %ld", ya, &h, xa, &w) != 4 || std::strcmp(ya, "-Y") || std::strcmp(xa, "+X") ||
        h <= 0 || w <= 0) {
        err = "HDR orientation other than -Y h +X w";
        return CORRUPT;
    }
    // the crate's HDR decoder yields Rgb32F (12 B/px), reserved against its
    // default 512 MiB limit before decoding: larger fails (-> Image::EMPTY)
    if ((uint64_t)h * (uint64_t)w * 12 > (512ull << 20)) {
        err = "HDR's decoded buffer exceeds the image crate's default 512 MiB allocation limit";
        return CORRUPT;
    }
    if ((uint64_t)h * (uint64_t)w > (1ull << 28)) {
        err = "HDR larger than this library's 2^28-pixel limit";
        return UNSUPPORTED;
    }
    W = (uint32_t)w;
    H = (uint32_t)h;
    std::vector<uint8_t> row((size_t)W * 4);
    rgba.assign((size_t)W * H * 4, 1.0f);
    auto byte = [&](uint8_t& b) -> bool {
        if (pos >= f.size()) return false;
        b = f[pos++];
        return true;
    };
    for (uint32_t y = 0; y < H; ++y) {
        bool ok = true;
        const bool new_rle = W >= 8 && W < 0x8000 && pos + 4 <= f.size() && f[pos] == 2 && f[pos + 1] == 2 &&
                             !(f[pos + 2] & 0x80) && ((uint32_t)f[pos + 2] << 8 | f[pos + 3]) == W;
        if (new_rle) {
            pos += 4;
            for (int c = 0; c < 4 && ok; ++c) {
                uint32_t x = 0;
                while (x < W && ok) {
                    uint8_t code, v;
                    if (!(ok = byte(code))) break;
                    if (code > 128) {
                        const uint32_t cnt = code - 128u;
                        if (!(ok = byte(v) && x + cnt <= W)) break;
                        for (uint32_t k = 0; k < cnt; ++k) row[(size_t)(x++) * 4 + c] = v;
                    } else {
                        if (!(ok = code > 0 && x + code <= W)) break;
                        for (uint32_t k = 0; k < code && ok; ++k) ok = byte(row[(size_t)(x++) * 4 + c]);
                    }
                }
            }
        } else {  // flat pixels, (1, 1, 1, n) repeating the previous one n << shift times
            uint32_t x = 0;
            int shift = 0;
            while (x < W && ok) {
                if (!(ok = pos + 4 <= f.size())) break;
                const uint8_t* p = &f[pos];
                pos += 4;
                if (p[0] == 1 && p[1] == 1 && p[2] == 1) {
                    // the shift grows by 8 per consecutive repeat marker (Radiance's
                    // oldreadcolrs); past 24 bits any nonzero count exceeds the
                    // 2^28-pixel limit, so such a chain is corrupt (and a shift of
                    // 64 would be undefined)
                    if (!(ok = shift <= 24 || p[3] == 0)) break;
                    const uint64_t cnt = shift <= 24 ? (uint64_t)p[3] << shift : 0u;
                    if (!(ok = x > 0 && cnt <= W - x)) break;
                    for (uint64_t k = 0; k < cnt; ++k, ++x) std::memcpy(&row[(size_t)x * 4], &row[(size_t)(x - 1) * 4], 4);
                    shift = shift < 32 ? shift + 8 : 32;
                } else {
                    std::memcpy(&row[(size_t)(x++) * 4], p, 4);
                    shift = 0;
                }
            }
        }
        if (!ok) {
            err = "truncated or corrupt HDR scanline";
            W = H = 0;
            rgba.clear();
            return CORRUPT;
        }
        float* o = &rgba[(size_t)y * W * 4];
        for (uint32_t x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) o[x * 4 + c] = rgbe_channel(row[(size_t)x * 4 + c], row[(size_t)x * 4 + 3]);
    }
    return OK;
}

}  // namespace rthdr
