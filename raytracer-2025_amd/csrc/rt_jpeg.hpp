// rt_jpeg.hpp -- JPEG decoding for ImageTexture (host only, header-only).
//
// The reference decodes a .jpg / .jpeg texture with the `image` crate 0.25.6
// (zune-jpeg underneath) into Rgba32FImage and applies the sRGB EOTF unless
// the texture is raw (utils/image.rs:21-82); the crate's Rust sources are not
// in the reference mount, so its exact upsampling and IDCT roundings are
// parity unpinned.  This decoder restates ITU-T T.81 for the files a scene
// uses -- baseline and extended sequential Huffman (SOF0 / SOF1) and
// progressive Huffman (SOF2), 8-bit samples, 1 (gray) or 3 (YCbCr or RGB)
// components, any sampling factors 1..4, restart intervals -- with the
// reconstruction libjpeg(-turbo) does by default (the integer "islow" IDCT,
// "fancy" triangle-filter chroma upsampling, its fixed-point YCbCr -> RGB),
// so that tests/test_jpeg_cpu.py can hold it bit-exact against PIL on the
// reference's own JPEG asset (assets/Final/normal.jpg, 4:2:0) and on
// synthetic files of every subsampling, progressive or not, with restarts.
// Arithmetic coding, lossless, hierarchical, 12-bit and 4-component (CMYK /
// YCCK) files are UNSUPPORTED, never decoded into something else.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace rtjpeg {

enum Status { OK = 0, CORRUPT = 2, UNSUPPORTED = 3 };

// zigzag index -> natural (row-major) index of the 8x8 block
static const uint8_t ZZ[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                               41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                               30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// A Huffman table (T.81 Annex C): canonical codes from the 16 length counts;
// symbols of codes up to 9 bits straight from a lookahead table.
struct Huff {
    bool present = false;
    uint8_t look_len[512] = {}, look_val[512] = {};
    int32_t maxcode[18] = {}, valptr[17] = {}, mincode[17] = {};
    uint8_t vals[256] = {};
    // dc: a DC table, whose symbols are bit counts of a difference -- above 15
    // they are rejected, as libjpeg's jpeg_make_d_derived_tbl does (a count
    // above 32 would also be an undefined shift in Bits::get / extend)
    bool build(const uint8_t counts[16], const uint8_t* v, int nv, bool dc) {
        int total = 0;
        for (int l = 0; l < 16; ++l) total += counts[l];
        if (total > 256 || total > nv) return false;
        std::memcpy(vals, v, (size_t)total);
        if (dc)
            for (int i = 0; i < total; ++i)
                if (vals[i] > 15) return false;
        std::memset(look_len, 0, sizeof look_len);
        int32_t code = 0;
        int k = 0;
        for (int l = 1; l <= 16; ++l) {
            valptr[l] = k;
            mincode[l] = code;
            const int n = counts[l - 1];
            for (int i = 0; i < n; ++i, ++code, ++k) {
                // over-subscribed: checked per code, before the code's
                // lookahead entries are written (code < 2^l keeps them
                // inside the 512-entry tables)
                if (code >= (1 << l)) return false;
                if (l <= 9) {
                    const int lo = code << (9 - l), hi = (code + 1) << (9 - l);
                    for (int c = lo; c < hi; ++c) look_len[c] = (uint8_t)l, look_val[c] = vals[k];
                }
            }
            maxcode[l] = n ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        present = true;
        return true;
    }
};

// Entropy-coded data: 0xFF00 is a stuffed 0xFF; any other marker ends the
// segment's bits, after which zeros are read (as libjpeg does).
struct Bits {
    const uint8_t* d = nullptr;
    size_t n = 0, pos = 0;
    uint32_t acc = 0;
    int cnt = 0;
    bool marker = false;
    void fill() {
        while (cnt <= 24) {
            uint32_t b = 0;
            if (!marker && pos < n) {
                b = d[pos];
                if (b == 0xFF) {
                    const uint8_t nx = pos + 1 < n ? d[pos + 1] : 0xD9;
                    if (nx == 0x00) {
                        pos += 2;
                    } else {
                        marker = true;
                        b = 0;
                    }
                } else {
                    ++pos;
                }
            }
            acc |= b << (24 - cnt);
            cnt += 8;
        }
    }
    uint32_t peek(int k) {
        fill();
        return acc >> (32 - k);
    }
    void skip(int k) {
        acc <<= k;
        cnt -= k;
    }
    int32_t get(int k) {
        if (k == 0) return 0;
        const int32_t v = (int32_t)peek(k);
        skip(k);
        return v;
    }
    // a restart: drop the bits left of the interval and the RSTn marker
    void restart() {
        acc = 0;
        cnt = 0;
        while (pos + 1 < n && !(d[pos] == 0xFF && d[pos + 1] != 0x00 && d[pos + 1] != 0xFF)) ++pos;
        if (pos + 1 < n && d[pos + 1] >= 0xD0 && d[pos + 1] <= 0xD7) pos += 2;
        marker = false;
    }
};

inline int decode_sym(Bits& b, const Huff& h) {
    const uint32_t look = b.peek(9);
    const int l = h.look_len[look];
    if (l) {
        b.skip(l);
        return h.look_val[look];
    }
    const uint32_t code16 = b.peek(16);
    for (int len = 10; len <= 16; ++len) {
        const int32_t c = (int32_t)(code16 >> (16 - len));
        if (c <= h.maxcode[len]) {
            b.skip(len);
            return h.vals[(h.valptr[len] + c - h.mincode[len]) & 0xff];
        }
    }
    b.skip(16);  // bad code: libjpeg warns and takes symbol 0
    return 0;
}
inline int32_t extend(int32_t v, int s) { return s && v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int bw = 0, bh = 0;           // allocated blocks (MCU-padded)
    int bw_real = 0, bh_real = 0;  // blocks covering the component's samples
    int dw = 0, dh = 0;            // downsampled width / height (samples)
    int32_t pred = 0;
    bool latched = false;
    uint16_t q[64] = {};  // natural order
    std::vector<int16_t> coef;
    std::vector<uint8_t> plane;  // bw * 8 x bh * 8 samples
};

// jidctint.c (islow): 13-bit constants, 2 extra bits between the passes
namespace idct {
constexpr int CB = 13, P1 = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
                  F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
inline int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }
}  // namespace idct

// libjpeg's post-IDCT range limit: x + 128 clamped to [0, 255], indexed by
// (x & 1023) so that garbage coefficients wrap as they do there.
inline uint8_t idct_limit(int32_t x) {
    const int y = x & 1023;
    if (y < 128) return (uint8_t)(y + 128);
    if (y < 512) return 255;
    if (y < 896) return 0;
    return (uint8_t)(y - 896);
}

inline void idct_block(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
    using namespace idct;
    int32_t ws[64];
    for (int c = 0; c < 8; ++c) {  // columns
        auto D = [&](int r) { return (int32_t)in[r * 8 + c] * (int32_t)q[r * 8 + c]; };
        int64_t z2 = D(2), z3 = D(6);
        int64_t z1 = (z2 + z3) * F0541;
        const int64_t t2 = z1 + z3 * -F1847, t3 = z1 + z2 * F0765;
        z2 = D(0), z3 = D(4);
        const int64_t t0 = (z2 + z3) * (1 << CB), t1 = (z2 - z3) * (1 << CB);
        const int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        int64_t o0 = D(7), o1 = D(5), o2 = D(3), o3 = D(1);
        z1 = o0 + o3;
        z2 = o1 + o2;
        z3 = o0 + o2;
        int64_t z4 = o1 + o3;
        const int64_t z5 = (z3 + z4) * F1175;
        o0 *= F0298, o1 *= F2053, o2 *= F3072, o3 *= F1501;
        z1 *= -F0899, z2 *= -F2562, z3 *= -F1961, z4 *= -F0390;
        z3 += z5, z4 += z5;
        o0 += z1 + z3, o1 += z2 + z4, o2 += z2 + z3, o3 += z1 + z4;
        ws[0 * 8 + c] = descale(t10 + o3, CB - P1);
        ws[7 * 8 + c] = descale(t10 - o3, CB - P1);
        ws[1 * 8 + c] = descale(t11 + o2, CB - P1);
        ws[6 * 8 + c] = descale(t11 - o2, CB - P1);
        ws[2 * 8 + c] = descale(t12 + o1, CB - P1);
        ws[5 * 8 + c] = descale(t12 - o1, CB - P1);
        ws[3 * 8 + c] = descale(t13 + o0, CB - P1);
        ws[4 * 8 + c] = descale(t13 - o0, CB - P1);
    }
    for (int r = 0; r < 8; ++r) {  // rows
        const int32_t* w = ws + r * 8;
        int64_t z2 = w[2], z3 = w[6];
        int64_t z1 = (z2 + z3) * F0541;
        const int64_t t2 = z1 + z3 * -F1847, t3 = z1 + z2 * F0765;
        const int64_t t0 = ((int64_t)w[0] + w[4]) * (1 << CB), t1 = ((int64_t)w[0] - w[4]) * (1 << CB);
        const int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        int64_t o0 = w[7], o1 = w[5], o2 = w[3], o3 = w[1];
        z1 = o0 + o3;
        z2 = o1 + o2;
        z3 = o0 + o2;
        int64_t z4 = o1 + o3;
        const int64_t z5 = (z3 + z4) * F1175;
        o0 *= F0298, o1 *= F2053, o2 *= F3072, o3 *= F1501;
        z1 *= -F0899, z2 *= -F2562, z3 *= -F1961, z4 *= -F0390;
        z3 += z5, z4 += z5;
        o0 += z1 + z3, o1 += z2 + z4, o2 += z2 + z3, o3 += z1 + z4;
        uint8_t* o = out + (size_t)r * stride;
        constexpr int S = CB + P1 + 3;
        o[0] = idct_limit(descale(t10 + o3, S));
        o[7] = idct_limit(descale(t10 - o3, S));
        o[1] = idct_limit(descale(t11 + o2, S));
        o[6] = idct_limit(descale(t11 - o2, S));
        o[2] = idct_limit(descale(t12 + o1, S));
        o[5] = idct_limit(descale(t12 - o1, S));
        o[3] = idct_limit(descale(t13 + o0, S));
        o[4] = idct_limit(descale(t13 - o0, S));
    }
}

struct Decoder {
    const uint8_t* d;
    size_t n;
    Decoder(const uint8_t* data, size_t size) : d(data), n(size) {}
    uint16_t qt[4][64] = {};
    bool qt_ok[4] = {};
    Huff dc[4], ac[4];
    std::vector<Comp> comps;
    int W = 0, H = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool progressive = false, frame = false, jfif = false, adobe = false;
    int adobe_transform = -1;
    uint32_t restart_interval = 0;
    int32_t eobrun = 0;
    std::string err;

    Status fail(Status s, const char* what) {
        err = what;
        return s;
    }
    static uint16_t be16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

    Status sof(const uint8_t* p, size_t len) {
        if (frame) return fail(CORRUPT, "two frames");
        if (len < 6) return fail(CORRUPT, "short SOF");
        if (p[0] != 8) return fail(UNSUPPORTED, "JPEG sample precision other than 8 bits");
        H = be16(p + 1);
        W = be16(p + 3);
        const int nc = p[5];
        if (W == 0 || H == 0) return fail(UNSUPPORTED, "JPEG without its height in the frame header (DNL)");
        // the crate decodes to L8 (gray) or Rgb8, reserved against its
        // default 512 MiB limit before decoding: larger fails (-> Image::EMPTY)
        if ((uint64_t)W * H * (nc == 1 ? 1 : 3) > (512ull << 20))
            return fail(CORRUPT, "JPEG's decoded buffer exceeds the image crate's default 512 MiB allocation limit");
        if ((uint64_t)W * H > (1ull << 28)) return fail(UNSUPPORTED, "JPEG larger than 2^28 pixels");
        if (nc != 1 && nc != 3) return fail(UNSUPPORTED, "JPEG with other than 1 or 3 components (CMYK / YCCK)");
        if (len < 6 + 3 * (size_t)nc) return fail(CORRUPT, "short SOF");
        comps.resize(nc);
        for (int i = 0; i < nc; ++i) {
            Comp& c = comps[i];
            c.id = p[6 + 3 * i];
            c.h = p[7 + 3 * i] >> 4;
            c.v = p[7 + 3 * i] & 15;
            c.tq = p[8 + 3 * i];
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return fail(CORRUPT, "bad component");
            hmax = std::max(hmax, c.h);
            vmax = std::max(vmax, c.v);
        }
        mcux = (W + 8 * hmax - 1) / (8 * hmax);
        mcuy = (H + 8 * vmax - 1) / (8 * vmax);
        for (Comp& c : comps) {
            if (hmax % c.h || vmax % c.v) return fail(UNSUPPORTED, "JPEG sampling factors that do not divide the maximum");
            c.bw = mcux * c.h;
            c.bh = mcuy * c.v;
            c.dw = (int)(((int64_t)W * c.h + hmax - 1) / hmax);
            c.dh = (int)(((int64_t)H * c.v + vmax - 1) / vmax);
            c.bw_real = (c.dw + 7) / 8;
            c.bh_real = (c.dh + 7) / 8;
            c.coef.assign((size_t)c.bw * c.bh * 64, 0);
        }
        frame = true;
        return OK;
    }

    Status dht(const uint8_t* p, size_t len) {
        size_t i = 0;
        while (i + 17 <= len) {
            const int tc = p[i] >> 4, th = p[i] & 15;
            if (tc > 1 || th > 3) return fail(CORRUPT, "bad DHT");
            int total = 0;
            for (int l = 0; l < 16; ++l) total += p[i + 1 + l];
            if (i + 17 + (size_t)total > len) return fail(CORRUPT, "short DHT");
            Huff& h = tc == 0 ? dc[th] : ac[th];
            if (!h.build(p + i + 1, p + i + 17, total, tc == 0)) return fail(CORRUPT, "bad Huffman table");
            i += 17 + (size_t)total;
        }
        return OK;
    }

    Status dqt(const uint8_t* p, size_t len) {
        size_t i = 0;
        while (i < len) {
            const int pq = p[i] >> 4, tq = p[i] & 15;
            if (pq > 1 || tq > 3) return fail(CORRUPT, "bad DQT");
            const size_t need = 1 + 64 * (pq ? 2 : 1);
            if (i + need > len) return fail(CORRUPT, "short DQT");
            for (int k = 0; k < 64; ++k) qt[tq][ZZ[k]] = pq ? be16(p + i + 1 + 2 * k) : p[i + 1 + k];
            qt_ok[tq] = true;
            i += need;
        }
        return OK;
    }

    int16_t* block(Comp& c, int bx, int by) { return c.coef.data() + ((size_t)by * c.bw + bx) * 64; }

    // one block of a scan (T.81 F.2.2 sequential; G.1.2 progressive)
    void decode_block(Bits& b, Comp& c, int16_t* blk, int ss, int se, int ah, int al) {
        if (!progressive) {
            const int s = decode_sym(b, dc[c.td]);
            c.pred += s ? extend(b.get(s), s) : 0;
            blk[0] = (int16_t)c.pred;
            for (int k = 1; k < 64; ++k) {
                const int rs = decode_sym(b, ac[c.ta]), r = rs >> 4, s2 = rs & 15;
                if (s2) {
                    k += r;
                    if (k > 63) break;
                    blk[ZZ[k]] = (int16_t)extend(b.get(s2), s2);
                } else {
                    if (r != 15) break;
                    k += 15;
                }
            }
            return;
        }
        if (ss == 0) {  // DC scans
            if (ah == 0) {
                const int s = decode_sym(b, dc[c.td]);
                c.pred += s ? extend(b.get(s), s) : 0;
                blk[0] = (int16_t)(int32_t)((uint32_t)c.pred << al);
            } else if (b.get(1)) {
                blk[0] = (int16_t)(blk[0] | (1 << al));
            }
            return;
        }
        if (ah == 0) {  // AC first scan
            if (eobrun > 0) {
                --eobrun;
                return;
            }
            for (int k = ss; k <= se; ++k) {
                const int rs = decode_sym(b, ac[c.ta]), r = rs >> 4, s = rs & 15;
                if (s) {
                    k += r;
                    if (k > 63) break;
                    blk[ZZ[k]] = (int16_t)(int32_t)((uint32_t)extend(b.get(s), s) << al);
                } else {
                    if (r != 15) {
                        eobrun = (1 << r) - 1;
                        if (r) eobrun += b.get(r);
                        break;
                    }
                    k += 15;
                }
            }
            return;
        }
        // AC refinement (libjpeg's decode_mcu_AC_refine)
        const int p1 = 1 << al, m1 = -(1 << al);
        int k = ss;
        auto refine = [&](int16_t& co) {
            if (b.get(1) && (co & p1) == 0) co = (int16_t)(co >= 0 ? co + p1 : co + m1);
        };
        if (eobrun == 0) {
            for (; k <= se; ++k) {
                const int rs = decode_sym(b, ac[c.ta]);
                int r = rs >> 4, s = rs & 15;
                if (s) {
                    s = b.get(1) ? p1 : m1;  // a new coefficient is +-1 at this bit
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) eobrun += b.get(r);
                    break;
                }
                do {
                    int16_t& co = blk[ZZ[k]];
                    if (co != 0) {
                        refine(co);
                    } else {
                        if (--r < 0) break;
                    }
                    ++k;
                } while (k <= se);
                if (s && k <= 63) blk[ZZ[k]] = (int16_t)s;
            }
        }
        if (eobrun > 0) {
            for (; k <= se; ++k) {
                int16_t& co = blk[ZZ[k]];
                if (co != 0) refine(co);
            }
            --eobrun;
        }
    }

    Status sos(const uint8_t* p, size_t len, size_t& pos) {
        if (!frame) return fail(CORRUPT, "scan before frame");
        if (len < 1) return fail(CORRUPT, "short SOS");
        const int ns = p[0];
        if (ns < 1 || ns > 4 || len < 4 + 2 * (size_t)ns) return fail(CORRUPT, "bad SOS");
        std::vector<Comp*> sc;
        for (int i = 0; i < ns; ++i) {
            Comp* c = nullptr;
            for (Comp& k : comps)
                if (k.id == p[1 + 2 * i]) c = &k;
            if (!c) return fail(CORRUPT, "scan names an unknown component");
            c->td = p[2 + 2 * i] >> 4;
            c->ta = p[2 + 2 * i] & 15;
            if (c->td > 3 || c->ta > 3) return fail(CORRUPT, "bad table index");
            if (!c->latched) {  // libjpeg latches a component's table at its first scan
                if (!qt_ok[c->tq]) return fail(CORRUPT, "missing quantization table");
                std::memcpy(c->q, qt[c->tq], sizeof c->q);
                c->latched = true;
            }
            sc.push_back(c);
        }
        const int ss = p[1 + 2 * ns], se = p[2 + 2 * ns], ah = p[3 + 2 * ns] >> 4, al = p[3 + 2 * ns] & 15;
        if (progressive) {
            if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13)
                return fail(CORRUPT, "bad progressive scan");
        }
        for (Comp* c : sc) {
            const bool need_dc = !progressive || ss == 0, need_ac = !progressive || ss > 0;
            if ((need_dc && !(progressive && ah) && !dc[c->td].present) || (need_ac && !ac[c->ta].present))
                return fail(CORRUPT, "missing Huffman table");
        }
        Bits b;
        b.d = d;
        b.n = n;
        b.pos = pos;
        for (Comp* c : sc) c->pred = 0;
        eobrun = 0;
        uint32_t todo = restart_interval;
        auto maybe_restart = [&]() {
            if (!restart_interval) return;
            if (todo == 0) {
                b.restart();
                for (Comp* c : sc) c->pred = 0;
                eobrun = 0;
                todo = restart_interval;
            }
            --todo;
        };
        if (ns == 1) {  // non-interleaved: the component's own blocks, one per MCU
            Comp& c = *sc[0];
            for (int by = 0; by < c.bh_real; ++by)
                for (int bx = 0; bx < c.bw_real; ++bx) {
                    maybe_restart();
                    decode_block(b, c, block(c, bx, by), ss, se, ah, al);
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    maybe_restart();
                    for (Comp* c : sc)
                        for (int v = 0; v < c->v; ++v)
                            for (int h = 0; h < c->h; ++h)
                                decode_block(b, *c, block(*c, mx * c->h + h, my * c->v + v), ss, se, ah, al);
                }
        }
        // resume marker parsing at the next marker after the entropy data
        size_t q = b.pos;
        while (q + 1 < n && !(d[q] == 0xFF && d[q + 1] != 0x00 && !(d[q + 1] >= 0xD0 && d[q + 1] <= 0xD7) && d[q + 1] != 0xFF))
            ++q;
        pos = q;
        return OK;
    }

    Status parse() {
        if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return fail(CORRUPT, "not a JPEG file");
        size_t pos = 2;
        bool eoi = false, any_scan = false;
        while (pos + 4 <= n && !eoi) {
            if (d[pos] != 0xFF) {
                ++pos;  // garbage between markers (libjpeg warns and skips)
                continue;
            }
            const uint8_t m = d[pos + 1];
            if (m == 0xFF) {
                ++pos;
                continue;
            }
            if (m == 0xD9) break;
            if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) {
                pos += 2;
                continue;
            }
            const size_t len = be16(d + pos + 2);
            if (len < 2 || pos + 2 + len > n) return fail(CORRUPT, "truncated marker segment");
            const uint8_t* p = d + pos + 4;
            const size_t pl = len - 2;
            pos += 2 + len;
            Status st = OK;
            switch (m) {
                case 0xC0:
                case 0xC1:
                    st = sof(p, pl);
                    break;
                case 0xC2:
                    progressive = true;
                    st = sof(p, pl);
                    break;
                case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE:
                case 0xCF:
                    return fail(UNSUPPORTED, "JPEG coding process other than Huffman sequential / progressive");
                case 0xC4:
                    st = dht(p, pl);
                    break;
                case 0xDB:
                    st = dqt(p, pl);
                    break;
                case 0xDD:
                    if (pl < 2) return fail(CORRUPT, "short DRI");
                    restart_interval = be16(p);
                    break;
                case 0xE0:
                    if (pl >= 5 && !std::memcmp(p, "JFIF\0", 5)) jfif = true;
                    break;
                case 0xEE:
                    if (pl >= 12 && !std::memcmp(p, "Adobe", 5)) adobe = true, adobe_transform = p[11];
                    break;
                case 0xDA:
                    st = sos(p, pl, pos);
                    any_scan = true;
                    break;
                default:
                    break;  // APPn, COM, DNL, ...
            }
            if (st != OK) return st;
        }
        if (!frame || !any_scan) return fail(CORRUPT, "JPEG without a frame or scan");
        return OK;
    }

    // jdcolor.c: is the 3-component frame RGB rather than YCbCr?
    bool rgb_frame() const {
        if (jfif) return false;
        if (adobe) return adobe_transform == 0;
        return comps[0].id == 'R' && comps[1].id == 'G' && comps[2].id == 'B';
    }

    // The component's samples upsampled to hmax x vmax per sample, W x H
    // (jdsample.c with do_fancy_upsampling: fancy h2v1 / h1v2 / h2v2 where
    // libjpeg-turbo uses them, box replication otherwise).
    std::vector<uint8_t> upsample(const Comp& c) const {
        std::vector<uint8_t> out((size_t)W * H);
        const int stride = c.bw * 8;
        const uint8_t* pl = c.plane.data();
        auto S = [&](int x, int y) -> int { return pl[(size_t)y * stride + x]; };
        const int fx = hmax / c.h, fy = vmax / c.v;
        const int dw = c.dw, dh = c.dh;
        if (fx == 1 && fy == 1) {
            for (int y = 0; y < H; ++y) std::memcpy(&out[(size_t)y * W], pl + (size_t)y * stride, (size_t)W);
            return out;
        }
        std::vector<uint8_t> row((size_t)dw * 2 + 16);
        if (fx == 2 && fy == 1 && dw > 2) {  // h2v1_fancy_upsample
            for (int y = 0; y < H; ++y) {
                uint8_t* o = row.data();
                int inv = S(0, y);
                *o++ = (uint8_t)inv;
                *o++ = (uint8_t)((inv * 3 + S(1, y) + 2) >> 2);
                for (int x = 1; x < dw - 1; ++x) {
                    inv = S(x, y) * 3;
                    *o++ = (uint8_t)((inv + S(x - 1, y) + 1) >> 2);
                    *o++ = (uint8_t)((inv + S(x + 1, y) + 2) >> 2);
                }
                inv = S(dw - 1, y);
                *o++ = (uint8_t)((inv * 3 + S(dw - 2, y) + 1) >> 2);
                *o++ = (uint8_t)inv;
                std::memcpy(&out[(size_t)y * W], row.data(), (size_t)W);
            }
            return out;
        }
        if (fx == 1 && fy == 2) {  // h1v2_fancy_upsample
            for (int y = 0; y < H; ++y) {
                const int r = y >> 1, far = (y & 1) ? std::min(r + 1, dh - 1) : std::max(r - 1, 0);
                const int bias = (y & 1) ? 2 : 1;
                for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = (uint8_t)((S(x, r) * 3 + S(x, far) + bias) >> 2);
            }
            return out;
        }
        if (fx == 2 && fy == 2 && dw > 2) {  // h2v2_fancy_upsample
            for (int y = 0; y < H; ++y) {
                const int r = y >> 1, far = (y & 1) ? std::min(r + 1, dh - 1) : std::max(r - 1, 0);
                auto col = [&](int x) { return S(x, r) * 3 + S(x, far); };
                uint8_t* o = row.data();
                int this_s = col(0), next_s = col(1), last_s;
                *o++ = (uint8_t)((this_s * 4 + 8) >> 4);
                *o++ = (uint8_t)((this_s * 3 + next_s + 7) >> 4);
                last_s = this_s;
                this_s = next_s;
                for (int x = 2; x < dw; ++x) {
                    next_s = col(x);
                    *o++ = (uint8_t)((this_s * 3 + last_s + 8) >> 4);
                    *o++ = (uint8_t)((this_s * 3 + next_s + 7) >> 4);
                    last_s = this_s;
                    this_s = next_s;
                }
                *o++ = (uint8_t)((this_s * 3 + last_s + 8) >> 4);
                *o++ = (uint8_t)((this_s * 4 + 7) >> 4);
                std::memcpy(&out[(size_t)y * W], row.data(), (size_t)W);
            }
            return out;
        }
        for (int y = 0; y < H; ++y)  // int_upsample / h2v1 / h2v2 (box)
            for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = (uint8_t)S(x / fx, y / fy);
        return out;
    }

    // RGBA f32 in [0, 1] (into_rgba32f of the RGB / L image), row 0 = top
    Status decode(uint32_t& w, uint32_t& h, std::vector<float>& rgba) {
        Status st = parse();
        if (st != OK) return st;
        for (Comp& c : comps) {
            if (!c.latched) {  // a component no scan named: libjpeg leaves its coefficients zero
                if (!qt_ok[c.tq]) return fail(CORRUPT, "missing quantization table");
                std::memcpy(c.q, qt[c.tq], sizeof c.q);
            }
            const int stride = c.bw * 8;
            c.plane.assign((size_t)stride * c.bh * 8, 0);
            for (int by = 0; by < c.bh; ++by)
                for (int bx = 0; bx < c.bw; ++bx)
                    idct_block(block(c, bx, by), c.q, c.plane.data() + (size_t)by * 8 * stride + bx * 8, stride);
        }
        w = (uint32_t)W;
        h = (uint32_t)H;
        rgba.assign((size_t)W * H * 4, 1.0f);
        if (comps.size() == 1) {
            const std::vector<uint8_t> g = upsample(comps[0]);
            for (size_t i = 0; i < g.size(); ++i) rgba[i * 4] = rgba[i * 4 + 1] = rgba[i * 4 + 2] = (float)g[i] / 255.0f;
            return OK;
        }
        const std::vector<uint8_t> a = upsample(comps[0]), b = upsample(comps[1]), c = upsample(comps[2]);
        if (rgb_frame()) {
            for (size_t i = 0; i < a.size(); ++i) {
                rgba[i * 4] = (float)a[i] / 255.0f;
                rgba[i * 4 + 1] = (float)b[i] / 255.0f;
                rgba[i * 4 + 2] = (float)c[i] / 255.0f;
            }
            return OK;
        }
        // jdcolor.c ycc_rgb_convert: 16-bit fixed point tables
        int32_t cr_r[256], cb_b[256], cr_g[256], cb_g[256];
        auto FIX = [](double x) { return (int32_t)(x * 65536.0 + 0.5); };
        for (int i = 0; i < 256; ++i) {
            const int32_t x = i - 128;
            cr_r[i] = (int32_t)(((int64_t)FIX(1.40200) * x + 32768) >> 16);
            cb_b[i] = (int32_t)(((int64_t)FIX(1.77200) * x + 32768) >> 16);
            cr_g[i] = -FIX(0.71414) * x;
            cb_g[i] = -FIX(0.34414) * x + 32768;
        }
        auto lim = [](int32_t v) { return (float)(v < 0 ? 0 : v > 255 ? 255 : v) / 255.0f; };
        for (size_t i = 0; i < a.size(); ++i) {
            const int y = a[i], cb = b[i], cr = c[i];
            rgba[i * 4] = lim(y + cr_r[cr]);
            rgba[i * 4 + 1] = lim(y + (int32_t)(((int64_t)cb_g[cb] + cr_g[cr]) >> 16));
            rgba[i * 4 + 2] = lim(y + cb_b[cb]);
        }
        return OK;
    }
};

// Decodes a JPEG file image into RGBA f32 in [0, 1], row 0 = top.
inline Status decode(const std::vector<uint8_t>& f, uint32_t& w, uint32_t& h, std::vector<float>& rgba,
                     std::string& err) {
    Decoder dec{f.data(), f.size()};
    const Status st = dec.decode(w, h, rgba);
    if (st != OK) {
        err = dec.err;
        w = h = 0;
        rgba.clear();
    }
    return st;
}

}  // namespace rtjpeg
