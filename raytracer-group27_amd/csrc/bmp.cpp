// bmp.cpp -- the file step of Screen::writeBitmapToFile (src/screen.cpp:52-53): stbi_write_bmp
// with comp = 4 as the reference's pinned stb (framework/cmake/download_optional_packages.cmake)
// emits it -- a 24-bit BITMAPINFOHEADER file, rows bottom-up, BGR, alpha dropped, each row padded
// to 4 bytes, image-size and resolution fields 0.  The reference's own render.bmp has exactly this
// header (tests/test_post.py round-trips it byte for byte).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "rt_internal.h"

namespace {
void put16(uint8_t*& p, uint32_t v) {
    p[0] = (uint8_t)(v & 0xFF);
    p[1] = (uint8_t)((v >> 8) & 0xFF);
    p += 2;
}
void put32(uint8_t*& p, uint32_t v) {
    for (int k = 0; k < 4; ++k) p[k] = (uint8_t)((v >> (8 * k)) & 0xFF);
    p += 4;
}
}  // namespace

extern "C" long rt_encode_bmp(int width, int height, const uint8_t* rgba8, uint8_t* out, long out_size) {
    if (width <= 0 || height <= 0 || !rgba8 || !out) {
        rt::set_error("rt_encode_bmp: invalid argument");
        return RT_ERR_INVALID;
    }
    const long pad = (long)((-width * 3) & 3);
    const long need = 54 + ((long)width * 3 + pad) * height;
    if (out_size < need) {
        rt::set_error("rt_encode_bmp: output buffer too small");
        return RT_ERR_INVALID;
    }
    uint8_t* p = out;
    *p++ = 'B';
    *p++ = 'M';
    put32(p, (uint32_t)need);  // file size
    put16(p, 0);
    put16(p, 0);
    put32(p, 54);  // pixel data offset
    put32(p, 40);  // BITMAPINFOHEADER
    put32(p, (uint32_t)width);
    put32(p, (uint32_t)height);
    put16(p, 1);   // planes
    put16(p, 24);  // bits per pixel
    for (int k = 0; k < 6; ++k) put32(p, 0);  // compression, image size, ppm x/y, colours
    for (int y = height - 1; y >= 0; --y) {   // bottom-up: the last (bottom) row first
        const uint8_t* row = rgba8 + (size_t)y * width * 4;
        for (int x = 0; x < width; ++x) {
            *p++ = row[4 * x + 2];
            *p++ = row[4 * x + 1];
            *p++ = row[4 * x + 0];
        }
        for (long k = 0; k < pad; ++k) *p++ = 0;
    }
    return need;
}

extern "C" int rt_write_bmp(const char* path, int width, int height, const uint8_t* rgba8) {
    if (!path || width <= 0 || height <= 0 || !rgba8) {
        rt::set_error("rt_write_bmp: invalid argument");
        return RT_ERR_INVALID;
    }
    const long pad = (long)((-width * 3) & 3);
    std::vector<uint8_t> buf((size_t)(54 + ((long)width * 3 + pad) * height));
    const long n = rt_encode_bmp(width, height, rgba8, buf.data(), (long)buf.size());
    if (n < 0) return (int)n;
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        rt::set_error(std::string("rt_write_bmp: cannot open ") + path);
        return RT_ERR_IO;
    }
    const size_t w = std::fwrite(buf.data(), 1, (size_t)n, f);
    std::fclose(f);
    if (w != (size_t)n) {
        rt::set_error(std::string("rt_write_bmp: short write to ") + path);
        return RT_ERR_IO;
    }
    return RT_OK;
}
