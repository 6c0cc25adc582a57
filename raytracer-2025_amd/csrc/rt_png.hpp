// rt_png.hpp -- PNG decoding for ImageTexture (host only, header-only).
//
// The reference decodes images with the `image` crate (0.25.6) into
// Rgba32FImage (`into_rgba32f`: an 8-bit sample v becomes v / 255, a 16-bit
// one v / 65535; gray expands to (g, g, g), palette to its RGB, a missing
// alpha is 1, tRNS keys become alpha 0) and then, unless the texture is raw or
// the format is HDR / EXR / AVIF, converts RGB with palette's sRGB EOTF
// (utils/image.rs:21-82).  This restates that pipeline's PNG decode over
// zlib's inflate, interlaced (Adam7) or not; rt_image.hpp picks the decoder
// by extension and applies the EOTF.
// tests/test_png_cpu.py pins the decoder against PIL on the reference's own
// PNG assets (8-bit RGB / RGBA / gray, 4-bit palette) and on synthetic files
// covering every color type, bit depth and filter.
#pragma once
#include <zlib.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace rtpng {

enum Status { OK = 0, MISSING = 1, CORRUPT = 2, UNSUPPORTED = 3 };

// image 0.25 Limits::default().max_alloc (512 MiB): ImageReader::decode fails
// on an image whose decoded buffer is larger (limits.reserve(total_bytes))
constexpr uint64_t CRATE_MAX_ALLOC = 512ull << 20;

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// palette 0.7 Srgb -> LinSrgb for f32 components (the IEC 61966-2-1 EOTF)
inline float srgb_to_linear(float x) {
    return x <= 0.04045f ? x / 12.92f : std::pow((x + 0.055f) / 1.055f, 2.4f);
}

inline uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (uint8_t)((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
}

// Decodes a PNG file image into RGBA f32 in [0, 1] (into_rgba32f), row 0 = top.
inline Status decode(const std::vector<uint8_t>& f, uint32_t& W, uint32_t& H, std::vector<float>& rgba, std::string& err) {
    static const uint8_t SIG[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || std::memcmp(f.data(), SIG, 8) != 0) {
        err = "not a PNG file";
        return CORRUPT;
    }
    size_t pos = 8;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    bool ihdr = false;
    while (pos + 8 <= f.size()) {
        const uint32_t len = be32(&f[pos]);
        const char* type = (const char*)&f[pos + 4];
        if (pos + 12 + (size_t)len > f.size()) break;
        const uint8_t* d = &f[pos + 8];
        if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
            W = be32(d);
            H = be32(d + 4);
            depth = d[8];
            ctype = d[9];
            interlace = d[12];
            ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(d, d + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(d, d + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + (size_t)len;
    }
    if (!ihdr || W == 0 || H == 0 || idat.empty()) {
        err = "PNG without IHDR / IDAT";
        return CORRUPT;
    }
    if (interlace > 1) {
        err = "bad PNG interlace method";
        return CORRUPT;
    }
    int channels;
    switch (ctype) {
        case 0: channels = 1; break;
        case 2: channels = 3; break;
        case 3: channels = 1; break;
        case 4: channels = 2; break;
        case 6: channels = 4; break;
        default: err = "bad PNG color type"; return CORRUPT;
    }
    const bool depth_ok = (ctype == 0 && (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) ||
                          (ctype == 3 && (depth == 1 || depth == 2 || depth == 4 || depth == 8)) ||
                          ((ctype == 2 || ctype == 4 || ctype == 6) && (depth == 8 || depth == 16));
    if (!depth_ok || (ctype == 3 && plte.empty())) {
        err = "bad PNG bit depth / palette";
        return CORRUPT;
    }
    // image 0.25's ImageReader::decode reserves the decoded buffer against
    // its default Limits (max_alloc 512 MiB) before decoding: a larger image
    // fails to decode there (-> Image::EMPTY, utils/image.rs:50-52).  Its PNG
    // decoder expands palettes to RGB, low bit depths to 8 and tRNS to an
    // alpha channel, and keeps 16-bit samples 16-bit.
    {
        const uint64_t out_ch = (ctype == 3 ? 3 : channels) + ((!trns.empty() && (ctype == 0 || ctype == 2 || ctype == 3)) ? 1 : 0);
        if ((uint64_t)W * H * out_ch * (depth == 16 ? 2 : 1) > CRATE_MAX_ALLOC) {
            err = "PNG's decoded buffer exceeds the image crate's default 512 MiB allocation limit";
            return CORRUPT;
        }
    }
    if ((uint64_t)W * H > (1ull << 28)) {
        err = "PNG larger than this library's 2^28-pixel limit";
        return UNSUPPORTED;  // a library limit, not a bad file
    }
    const size_t bpp_bits = (size_t)channels * depth;
    const size_t bpp = std::max<size_t>(1, bpp_bits / 8);  // filter byte distance
    // the passes: the whole image, or Adam7's seven (x0, y0, dx, dy) sub-images,
    // each its own run of filtered scanlines
    static const uint32_t ADAM7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                         {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    static const uint32_t WHOLE[1][4] = {{0, 0, 1, 1}};
    const uint32_t (*passes)[4] = interlace ? ADAM7 : WHOLE;
    const int n_pass = interlace ? 7 : 1;
    size_t raw_size = 0;
    for (int k = 0; k < n_pass; ++k) {
        const uint32_t pw = (W - passes[k][0] + passes[k][2] - 1) / passes[k][2];
        const uint32_t ph = (H - passes[k][1] + passes[k][3] - 1) / passes[k][3];
        if (W > passes[k][0] && H > passes[k][1] && pw && ph) raw_size += ((pw * bpp_bits + 7) / 8 + 1) * (size_t)ph;
    }
    std::vector<uint8_t> raw(raw_size);
    uLongf out_len = (uLongf)raw.size();
    if (uncompress(raw.data(), &out_len, idat.data(), (uLong)idat.size()) != Z_OK || out_len != raw.size()) {
        err = "PNG zlib stream does not inflate to the image size";
        return CORRUPT;
    }
    rgba.assign((size_t)W * H * 4, 1.0f);
    const float max_v = depth == 16 ? 65535.0f : 255.0f;
    auto sample = [&](const uint8_t* row, size_t idx) -> uint32_t {  // idx-th sample of the row
        if (depth == 8) return row[idx];
        if (depth == 16) return (uint32_t)row[2 * idx] << 8 | row[2 * idx + 1];
        const size_t bit = idx * depth;
        return (row[bit / 8] >> (8 - depth - bit % 8)) & ((1u << depth) - 1);
    };
    size_t at = 0;
    for (int k = 0; k < n_pass; ++k) {
        const uint32_t x0 = passes[k][0], y0 = passes[k][1], dx = passes[k][2], dy = passes[k][3];
        if (W <= x0 || H <= y0) continue;
        const uint32_t pw = (W - x0 + dx - 1) / dx, ph = (H - y0 + dy - 1) / dy;
        const size_t stride = ((size_t)pw * bpp_bits + 7) / 8;
        // unfilter the pass (filter types 0-4), each row against the pass's previous row
        std::vector<uint8_t> img(stride * ph);
        for (uint32_t y = 0; y < ph; ++y) {
            const uint8_t ft = raw[at + y * (stride + 1)];
            const uint8_t* src = &raw[at + y * (stride + 1) + 1];
            uint8_t* cur = &img[y * stride];
            const uint8_t* prev = y ? &img[(y - 1) * stride] : nullptr;
            for (size_t i = 0; i < stride; ++i) {
                const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0,
                          c = (prev && i >= bpp) ? prev[i - bpp] : 0;
                int v = src[i];
                switch (ft) {
                    case 0: break;
                    case 1: v += a; break;
                    case 2: v += b; break;
                    case 3: v += (a + b) >> 1; break;
                    case 4: v += paeth(a, b, c); break;
                    default: err = "bad PNG filter type"; return CORRUPT;
                }
                cur[i] = (uint8_t)v;
            }
        }
        at += (stride + 1) * ph;
        for (uint32_t y = 0; y < ph; ++y) {
            const uint8_t* row = &img[y * stride];
            for (uint32_t x = 0; x < pw; ++x) {
                float* o = &rgba[((size_t)(y0 + y * dy) * W + (x0 + x * dx)) * 4];
                if (ctype == 3) {
                    const uint32_t kk = sample(row, x);
                    if (3 * kk + 2 >= plte.size()) {
                        err = "PNG palette index out of range";
                        return CORRUPT;
                    }
                    for (int c = 0; c < 3; ++c) o[c] = (float)plte[3 * kk + c] / 255.0f;
                    o[3] = kk < trns.size() ? (float)trns[kk] / 255.0f : 1.0f;
                } else if (ctype == 0 || ctype == 4) {
                    const uint32_t g = sample(row, (size_t)x * channels);
                    // sub-8-bit gray is scaled to 8 bits first (the png crate's EXPAND)
                    const float gv = depth < 8 ? (float)(g * 255u / ((1u << depth) - 1)) / 255.0f : (float)g / max_v;
                    o[0] = o[1] = o[2] = gv;
                    if (ctype == 4) o[3] = (float)sample(row, (size_t)x * 2 + 1) / max_v;
                    else if (trns.size() >= 2 && g == ((uint32_t)trns[0] << 8 | trns[1])) o[3] = 0.0f;
                } else {
                    uint32_t v[4];
                    for (int c = 0; c < channels; ++c) v[c] = sample(row, (size_t)x * channels + c);
                    for (int c = 0; c < 3; ++c) o[c] = (float)v[c] / max_v;
                    if (ctype == 6) o[3] = (float)v[3] / max_v;
                    else if (trns.size() >= 6 && v[0] == ((uint32_t)trns[0] << 8 | trns[1]) &&
                             v[1] == ((uint32_t)trns[2] << 8 | trns[3]) && v[2] == ((uint32_t)trns[4] << 8 | trns[5]))
                        o[3] = 0.0f;
                }
            }
        }
    }
    return OK;
}

}  // namespace rtpng
