// png_decode.cpp -- PNG -> 8-bit RGB with the semantics of stbi_load(path, &w, &h, &n, STBI_rgb),
// the texture loader of Image::Image (reference src/image.cpp:37-73; stb_image.h pinned at
// b42009b by framework/cmake/download_framework_packages.cmake).  Restated from the PNG
// specification and stb_image's documented conversions, on top of the system zlib:
//   * colour types 0 (grey), 2 (RGB), 3 (palette), 4 (grey+alpha), 6 (RGBA); bit depths 1-16;
//   * grey below 8 bits is scaled by 0xff / 0x55 / 0x11 (1 / 2 / 4 bits); palette indices are not;
//   * 16-bit samples keep their high byte (stbi__convert_16_to_8);
//   * to RGB: grey g -> (g, g, g), alpha dropped;
//   * the reported channel count is the file's: 1, 2, 3, 4, and 3 or 4 (tRNS) for palettes.
// Interlaced (Adam7) files are rejected.
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "rt_internal.h"

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

struct Png {
    int w = 0, h = 0, depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
};

bool parse(const uint8_t* d, long n, Png& p, std::string& err) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(d, sig, 8) != 0) {
        err = "not a PNG file";
        return false;
    }
    long o = 8;
    bool have_ihdr = false;
    while (o + 12 <= n) {
        const uint32_t len = be32(d + o);
        const uint8_t* type = d + o + 4;
        const uint8_t* body = d + o + 8;
        if ((long)len > n - o - 12) {
            err = "truncated chunk";
            return false;
        }
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) {
                err = "bad IHDR";
                return false;
            }
            p.w = (int)be32(body);
            p.h = (int)be32(body + 4);
            p.depth = body[8];
            p.ctype = body[9];
            p.interlace = body[12];
            have_ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            p.plte.assign(body, body + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            p.trns.assign(body, body + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            p.idat.insert(p.idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        o += 12 + (long)len;
    }
    if (!have_ihdr || p.w <= 0 || p.h <= 0) {
        err = "missing IHDR";
        return false;
    }
    if (p.interlace != 0) {
        err = "interlaced PNG is not supported";
        return false;
    }
    const int c = p.ctype;
    const int dp = p.depth;
    const bool ok = (c == 0 && (dp == 1 || dp == 2 || dp == 4 || dp == 8 || dp == 16)) ||
                    (c == 3 && (dp == 1 || dp == 2 || dp == 4 || dp == 8)) ||
                    ((c == 2 || c == 4 || c == 6) && (dp == 8 || dp == 16));
    if (!ok) {
        err = "unsupported PNG colour type / bit depth";
        return false;
    }
    if (c == 3 && p.plte.empty()) {
        err = "palette PNG without PLTE";
        return false;
    }
    return true;
}

int samples_per_pixel(int ctype) { return ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 1; }

}  // namespace

extern "C" int rt_decode_png(const uint8_t* data, long size, int* width, int* height, int* channels, uint8_t* rgb,
                             long rgb_size) {
    if (!data || size <= 0 || !width || !height || !channels) {
        rt::set_error("rt_decode_png: null argument");
        return RT_ERR_INVALID;
    }
    Png p;
    std::string err;
    if (!parse(data, size, p, err)) {
        rt::set_error("rt_decode_png: " + err);
        return RT_ERR_INVALID;
    }
    *width = p.w;
    *height = p.h;
    const int spp = samples_per_pixel(p.ctype);
    *channels = p.ctype == 3 ? (p.trns.empty() ? 3 : 4) : spp;
    if (!rgb) return RT_OK;
    if (rgb_size < (long)p.w * p.h * 3) {
        rt::set_error("rt_decode_png: output buffer too small");
        return RT_ERR_INVALID;
    }
    // inflate: one filter byte + packed samples per row
    const size_t bits_pp = (size_t)spp * p.depth;
    const size_t stride = ((size_t)p.w * bits_pp + 7) / 8;
    const size_t raw_size = (stride + 1) * (size_t)p.h;
    std::vector<uint8_t> raw(raw_size);
    uLongf out_len = (uLongf)raw_size;
    const int zr = uncompress(raw.data(), &out_len, p.idat.data(), (uLong)p.idat.size());
    if ((zr != Z_OK && zr != Z_BUF_ERROR) || out_len < raw_size) {
        rt::set_error("rt_decode_png: corrupt image data");
        return RT_ERR_INVALID;
    }
    // unfilter (bytes per complete pixel, at least 1)
    const size_t bpp = bits_pp >= 8 ? bits_pp / 8 : 1;
    std::vector<uint8_t> img(stride * (size_t)p.h);
    for (int y = 0; y < p.h; ++y) {
        const uint8_t ft = raw[(size_t)y * (stride + 1)];
        const uint8_t* src = raw.data() + (size_t)y * (stride + 1) + 1;
        uint8_t* cur = img.data() + (size_t)y * stride;
        const uint8_t* prev = y ? cur - stride : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= bpp ? cur[i - bpp] : 0;
            const int b = prev ? prev[i] : 0;
            const int c = (prev && i >= bpp) ? prev[i - bpp] : 0;
            int v = src[i];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default:
                    rt::set_error("rt_decode_png: bad filter type");
                    return RT_ERR_INVALID;
            }
            cur[i] = (uint8_t)v;
        }
    }
    // samples -> 8-bit RGB
    auto sample = [&](const uint8_t* row, int x, int s) -> int {
        const size_t idx = (size_t)x * spp + s;
        if (p.depth == 8) return row[idx];
        if (p.depth == 16) return row[2 * idx];  // high byte
        const size_t bit = idx * p.depth;
        const int v = (row[bit >> 3] >> (8 - p.depth - (int)(bit & 7))) & ((1 << p.depth) - 1);
        return v;
    };
    const int scale = p.depth == 1 ? 0xff : p.depth == 2 ? 0x55 : p.depth == 4 ? 0x11 : 1;
    for (int y = 0; y < p.h; ++y) {
        const uint8_t* row = img.data() + (size_t)y * stride;
        uint8_t* out = rgb + (size_t)y * p.w * 3;
        for (int x = 0; x < p.w; ++x) {
            int r, g, b;
            if (p.ctype == 3) {
                const int i = sample(row, x, 0);
                if ((size_t)(3 * i + 2) < p.plte.size()) {
                    r = p.plte[3 * i];
                    g = p.plte[3 * i + 1];
                    b = p.plte[3 * i + 2];
                } else {
                    r = g = b = 0;
                }
            } else if (p.ctype == 0 || p.ctype == 4) {
                const int v = sample(row, x, 0) * (p.depth < 8 ? scale : 1);
                r = g = b = v;
            } else {
                r = sample(row, x, 0);
                g = sample(row, x, 1);
                b = sample(row, x, 2);
            }
            out[3 * x] = (uint8_t)r;
            out[3 * x + 1] = (uint8_t)g;
            out[3 * x + 2] = (uint8_t)b;
        }
    }
    return RT_OK;
}
