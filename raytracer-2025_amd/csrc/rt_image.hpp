// rt_image.hpp -- Image::new(path, raw) + pixel_data's colour handling
// (utils/image.rs:21-82) for a path given directly (host only).
//
// The reference opens a texture with ImageReader::open, which takes the
// format from the file's extension (image 0.25.6 ImageFormat::from_path),
// and returns Image::EMPTY (cyan) when the extension names no format or the
// file cannot be opened or decoded in that format.  Decoded pixels are RGBA
// f32 (into_rgba32f); RGB goes through palette's sRGB EOTF unless the texture
// is raw or the format is HDR / EXR / AVIF, whose pixels stay linear.
// Decoded here: PNG (rt_png.hpp), JPEG (rt_jpeg.hpp), Radiance HDR
// (rt_hdr.hpp).  Formats the crate reads and this library does not (GIF,
// WebP, TIFF, BMP, EXR, AVIF, ...) are UNSUPPORTED -- never a wrong image.
#pragma once
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <string>
#include <vector>

#include "rt_hdr.hpp"
#include "rt_jpeg.hpp"
#include "rt_png.hpp"

namespace rtimg {

enum Status { OK = 0, MISSING = 1, UNSUPPORTED = 3 };
enum Format { F_NONE, F_PNG, F_JPEG, F_HDR, F_OTHER };

// ImageFormat::from_extension (case-insensitive)
inline Format format_of(const std::string& path) {
    const size_t dot = path.find_last_of('.'), slash = path.find_last_of('/');
    if (dot == std::string::npos || (slash != std::string::npos && dot < slash)) return F_NONE;
    std::string e = path.substr(dot + 1);
    std::transform(e.begin(), e.end(), e.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    if (e == "png" || e == "apng") return F_PNG;
    if (e == "jpg" || e == "jpeg" || e == "jfif") return F_JPEG;
    if (e == "hdr") return F_HDR;
    static const char* other[] = {"avif", "gif", "webp", "tif", "tiff", "tga", "dds", "bmp", "ico", "exr",
                                  "pbm", "pam", "ppm", "pgm", "pnm", "ff", "qoi", "pcx"};
    for (const char* o : other)
        if (e == o) return F_OTHER;
    return F_NONE;
}

inline Status load(const std::string& path, bool raw, uint32_t& W, uint32_t& H, std::vector<float>& rgba,
                   std::string& err) {
    W = H = 0;
    rgba.clear();
    const Format fmt = format_of(path);
    if (fmt == F_NONE) return MISSING;  // ir.format()? -> None
    if (fmt == F_OTHER) {
        err = path + ": image format not decoded by this library (PNG, JPEG and Radiance HDR are)";
        return UNSUPPORTED;
    }
    std::FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) return MISSING;
    std::vector<uint8_t> f;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) f.insert(f.end(), buf, buf + n);
    std::fclose(fp);
    // Each decoder returns 3 (UNSUPPORTED) for what this library does not
    // decode -- a library limit (more than 2^28 pixels within the crate's
    // 512 MiB allocation limit) or a coding process it leaves out -- which
    // the crate might decode: RT_EUNSUPPORTED, never a cyan image; anything
    // else that fails (a bad signature, a corrupt stream, a decoded buffer
    // past the crate's 512 MiB default limit) is the crate's decode error ->
    // Image::EMPTY.
    int st;
    if (fmt == F_PNG)
        st = (int)rtpng::decode(f, W, H, rgba, err);
    else if (fmt == F_JPEG)
        st = (int)rtjpeg::decode(f, W, H, rgba, err);
    else
        st = (int)rthdr::decode(f, W, H, rgba, err);
    static_assert((int)rtpng::UNSUPPORTED == 3 && (int)rtjpeg::UNSUPPORTED == 3 && (int)rthdr::UNSUPPORTED == 3, "");
    if (st == 3) {
        err = path + ": " + err;
        W = H = 0;
        rgba.clear();
        return UNSUPPORTED;
    }
    if (st != 0) {  // ImageReader::decode().ok()? -> None -> Image::EMPTY
        W = H = 0;
        rgba.clear();
        return MISSING;
    }
    if (!raw && fmt != F_HDR)
        for (size_t i = 0; i < rgba.size(); i += 4)
            for (int c = 0; c < 3; ++c) rgba[i + c] = rtpng::srgb_to_linear(rgba[i + c]);
    return OK;
}

}  // namespace rtimg
