// ref_post.cpp -- ORACLE (test infrastructure only): CPU restatement of the reference's Screen
// post-processing, src/screen.cpp (catalinlup/RayTracer-Group27).  Loaded only by tests/ as the
// checker of the HIP post-processing kernels (raytracer-group27_amd/csrc/rt_post.hip).
//
// Follows, line by line:
//   writeBitmapToFile            src/screen.cpp:40-54   (bloom in place, clamp, *255, truncate)
//   postprocessImage             src/screen.cpp:56-69   (bloom if live, then gamma)
//   applyBloomEffect             src/screen.cpp:226-275
//   filterLightPixels            src/screen.cpp:279-292 (grayscale >= 1 keeps the pixel)
//   applyKernel / boxKernel / gaussianKernel / gaussianFunction   src/screen.cpp:296-345
//   addImages, clamp, reinhardToneMap, exposureToneMap, gammaCorrection, convertToGrayscale,
//   getPixel (black border)      src/screen.cpp:348-393
// glm semantics: vec3 ops are per-component float ops; glm::dot = (x*x' + y*y') + z*z';
// glm::exp/pow on float call expf/powf; vec3 /= int divides by float(int); glm::clamp = min(max).
// Parity status: the Bloom option with the default box kernel is pinned by the reference's render.bmp
// (tests/test_render_bmp_pin.py); the other options only by this restatement (glm 0.9.9.8 is not in the image).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../include/rt_amd.h"

namespace {

struct P3 {
    float x, y, z;
};

constexpr double kRefPi = 3.1415926535893238;  // #define M_PI in src/screen.cpp:13 (sic)

inline float gmaxf(float a, float b) { return (a < b) ? b : a; }
inline float gminf(float a, float b) { return (b < a) ? b : a; }

struct Screen {
    int W, H;
    std::vector<P3> px;
    rt_post_params s;

    P3 get(int x, int y, const std::vector<P3>& img) const {
        if (x < 0 || y < 0 || x >= W || y >= H) return P3{0.0f, 0.0f, 0.0f};
        return img[(size_t)y * W + x];
    }
    static float gray(const P3& p) {
        const float wx = (float)0.2126, wy = (float)0.7152, wz = (float)0.0722;
        return (p.x * wx + p.y * wy) + p.z * wz;
    }
    float gauss(float x, float y) const {
        const float sg = s.sigma;
        const double a = 1.0 / ((double)(sg * sg * 2.0f) * kRefPi);
        const float e = std::exp(-(x * x + y * y) / (2.0f * sg * sg));
        return (float)(a * (double)e);
    }
    void light_pixels(std::vector<P3>& out) const {
        out.clear();
        for (const P3& p : px) out.push_back(gray(p) >= 1.0f ? p : P3{0.0f, 0.0f, 0.0f});
    }
    void kernel(std::vector<P3>& image) const {
        const std::vector<P3> src(image);
        const int fs = s.filter_size;
        for (int x = 0; x < W; ++x)
            for (int y = 0; y < H; ++y) {
                P3 sum{0.0f, 0.0f, 0.0f};
                for (int i = -fs; i < fs + 1; ++i)
                    for (int j = -fs; j < fs + 1; ++j) {
                        const P3 p = get(x + i, y + j, src);
                        if (s.kernel == RT_KERNEL_GAUSSIAN) {
                            const float w = gauss((float)i, (float)j);
                            sum.x += w * p.x;
                            sum.y += w * p.y;
                            sum.z += w * p.z;
                        } else {
                            sum.x += p.x;
                            sum.y += p.y;
                            sum.z += p.z;
                        }
                    }
                if (s.kernel != RT_KERNEL_GAUSSIAN) {
                    const float n = (float)((2 * fs + 1) * (2 * fs + 1));
                    sum.x /= n;
                    sum.y /= n;
                    sum.z /= n;
                }
                image[(size_t)y * W + x] = sum;
            }
    }
    void bloom() {
        const int opt = s.filtering_option;
        if (opt == RT_BLOOM_NONE) return;
        std::vector<P3> light;
        light_pixels(light);
        if (opt == RT_BLOOM_ONLY_LIGHT) {
            px = light;
            return;
        }
        if (opt == RT_BLOOM_ONLY_LIGHT_KERNEL) {
            kernel(light);
            px = light;
            return;
        }
        for (int i = 1; i <= s.repetitions; ++i) kernel(light);
        for (size_t k = 0; k < px.size(); ++k) {
            P3 v{px[k].x + light[k].x, px[k].y + light[k].y, px[k].z + light[k].z};
            if (opt == RT_BLOOM) {
                v = P3{gminf(gmaxf(v.x, 0.0f), 1.0f), gminf(gmaxf(v.y, 0.0f), 1.0f), gminf(gmaxf(v.z, 0.0f), 1.0f)};
            } else if (opt == RT_BLOOM_REINHARD) {
                v = P3{v.x / (v.x + 1.0f), v.y / (v.y + 1.0f), v.z / (v.z + 1.0f)};
            } else if (opt == RT_BLOOM_EXPOSURE) {
                const float e = s.exposure;
                v = P3{1.0f - std::exp(-v.x * e), 1.0f - std::exp(-v.y * e), 1.0f - std::exp(-v.z * e)};
            }
            px[k] = v;
        }
    }
    void gamma() {
        const float g = 1.0f / s.gamma;
        for (P3& p : px) p = P3{std::pow(p.x, g), std::pow(p.y, g), std::pow(p.z, g)};
    }
};

Screen make(const rt_post_params* p, int W, int H, const float* rgb) {
    Screen sc;
    sc.W = W;
    sc.H = H;
    sc.s = *p;
    sc.s.repetitions = std::max(1, p->repetitions);  // setKernelNumRepetitions
    sc.s.sigma = std::max(0.001f, p->sigma);          // setSigma (glm::max(0.001f, x))
    sc.px.resize((size_t)W * H);
    for (size_t k = 0; k < sc.px.size(); ++k) sc.px[k] = P3{rgb[3 * k], rgb[3 * k + 1], rgb[3 * k + 2]};
    return sc;
}

void store(const Screen& sc, float* rgb) {
    for (size_t k = 0; k < sc.px.size(); ++k) {
        rgb[3 * k] = sc.px[k].x;
        rgb[3 * k + 1] = sc.px[k].y;
        rgb[3 * k + 2] = sc.px[k].z;
    }
}

}  // namespace

extern "C" {

int oracle_postprocess(const rt_post_params* p, int W, int H, float* rgb) {
    Screen sc = make(p, W, H, rgb);
    if (p->bloom_live) sc.bloom();
    if (p->gamma_correction) sc.gamma();
    store(sc, rgb);
    return 0;
}

int oracle_bitmap(const rt_post_params* p, int W, int H, float* rgb, uint8_t* rgba8) {
    Screen sc = make(p, W, H, rgb);
    sc.bloom();
    store(sc, rgb);
    for (size_t k = 0; k < sc.px.size(); ++k) {
        const float c[3] = {sc.px[k].x, sc.px[k].y, sc.px[k].z};
        for (int a = 0; a < 3; ++a) rgba8[4 * k + a] = (uint8_t)(gminf(gmaxf(c[a], 0.0f), 1.0f) * 255.0f);
        rgba8[4 * k + 3] = (uint8_t)(1.0f * 255.0f);
    }
    return 0;
}

}  // extern "C"
