// rt_post.hip -- Screen post-processing on the GPU (src/screen.cpp:40-69, 226-393): bright-pass,
// box / Gaussian bloom kernels, image add + tone mapping, gamma, 8-bit quantisation.
//
// All of it is HBM/LDS-bound stencil and elementwise work on W*H*3 floats.  The blur keeps the
// reference's summation order exactly (column offset i outer, row offset j inner, one float add
// per tap, src/screen.cpp:318-343) so box blur is bit-identical to the CPU; a separable filter
// would round differently.  A 16x16 output tile stages its (16+2r)^2 input halo in LDS as three
// colour planes when r <= 16 (27.6 KB), otherwise every tap reads the (L1/L2-resident) source.
// Gaussian weights are computed on the host with the reference's own float/double expression
// (gaussianFunction, src/screen.cpp:347-349), so the device multiplies by the same bits.
// expf / powf (exposure tone map, gamma) are the device math library: within 2 ulp of glibc.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "rt_internal.h"

namespace {

constexpr int kTile = 16;
constexpr int kLdsRadius = 16;
constexpr double kRefPi = 3.1415926535893238;  // src/screen.cpp:13

__device__ __forceinline__ float gmaxf(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float gminf(float a, float b) { return (b < a) ? b : a; }

// filterLightPixels: keep the pixel iff dot(p, (0.2126, 0.7152, 0.0722)) >= 1
__global__ void post_bright_kernel(const float* __restrict__ in, float* __restrict__ light, int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float r = in[3 * k], g = in[3 * k + 1], b = in[3 * k + 2];
    const float gray = (r * 0.2126f + g * 0.7152f) + b * 0.0722f;
    const bool keep = gray >= 1.0f;
    light[3 * k] = keep ? r : 0.0f;
    light[3 * k + 1] = keep ? g : 0.0f;
    light[3 * k + 2] = keep ? b : 0.0f;
}

// boxKernel / gaussianKernel over the whole image (applyKernel), halo staged in LDS
template <bool GAUSS, bool LDS>
__global__ __launch_bounds__(256) void post_blur_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                        int W, int H, int fs, const float* __restrict__ wtab) {
    extern __shared__ float halo[];  // 3 planes of R*R
    const int tx = threadIdx.x, ty = threadIdx.y;
    const int x0 = blockIdx.x * kTile, y0 = blockIdx.y * kTile;
    const int x = x0 + tx, y = y0 + ty;
    const int R = kTile + 2 * fs;
    if (LDS) {
        const int RR = R * R;
        for (int k = ty * kTile + tx; k < RR; k += kTile * kTile) {
            const int hx = x0 - fs + k % R, hy = y0 - fs + k / R;
            float r = 0.0f, g = 0.0f, b = 0.0f;
            if (hx >= 0 && hy >= 0 && hx < W && hy < H) {
                const size_t o = ((size_t)hy * W + hx) * 3;
                r = src[o];
                g = src[o + 1];
                b = src[o + 2];
            }
            halo[k] = r;
            halo[RR + k] = g;
            halo[2 * RR + k] = b;
        }
        __syncthreads();
    }
    if (x >= W || y >= H) return;
    float sr = 0.0f, sg = 0.0f, sb = 0.0f;
    const int n1 = 2 * fs + 1;
    for (int i = -fs; i < fs + 1; ++i) {
        for (int j = -fs; j < fs + 1; ++j) {
            float r, g, b;
            if (LDS) {
                const int RR = R * R;
                const int k = (ty + fs + j) * R + (tx + fs + i);
                r = halo[k];
                g = halo[RR + k];
                b = halo[2 * RR + k];
            } else {
                const int px = x + i, py = y + j;
                if (px < 0 || py < 0 || px >= W || py >= H) {
                    r = g = b = 0.0f;
                } else {
                    const size_t o = ((size_t)py * W + px) * 3;
                    r = src[o];
                    g = src[o + 1];
                    b = src[o + 2];
                }
            }
            if (GAUSS) {
                const float w = wtab[(i + fs) * n1 + (j + fs)];
                sr += w * r;
                sg += w * g;
                sb += w * b;
            } else {
                sr += r;
                sg += g;
                sb += b;
            }
        }
    }
    if (!GAUSS) {
        const float n = (float)(n1 * n1);
        sr /= n;
        sg /= n;
        sb /= n;
    }
    const size_t o = ((size_t)y * W + x) * 3;
    dst[o] = sr;
    dst[o + 1] = sg;
    dst[o + 2] = sb;
}

// addImages + the tone map of applyBloomEffect (src/screen.cpp:264-273)
__global__ void post_tone_kernel(float* __restrict__ img, const float* __restrict__ light, int n3, int mode,
                                 float exposure) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n3) return;
    float v = img[k] + light[k];
    if (mode == RT_BLOOM)
        v = gminf(gmaxf(v, 0.0f), 1.0f);
    else if (mode == RT_BLOOM_REINHARD)
        v = v / (v + 1.0f);
    else if (mode == RT_BLOOM_EXPOSURE)
        v = 1.0f - expf(-v * exposure);
    img[k] = v;
}

// gammaCorrection: pow(p, 1/gamma) per component
__global__ void post_gamma_kernel(float* __restrict__ img, int n3, float inv_gamma) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n3) return;
    img[k] = powf(img[k], inv_gamma);
}

// writeBitmapToFile: clamp to [0,1], *255, truncate to u8; alpha 255 (vec4(c, 1) * 255)
__global__ void post_quantize_kernel(const float* __restrict__ img, uint8_t* __restrict__ rgba8, int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uchar4 o;
    o.x = (uint8_t)(gminf(gmaxf(img[3 * k], 0.0f), 1.0f) * 255.0f);
    o.y = (uint8_t)(gminf(gmaxf(img[3 * k + 1], 0.0f), 1.0f) * 255.0f);
    o.z = (uint8_t)(gminf(gmaxf(img[3 * k + 2], 0.0f), 1.0f) * 255.0f);
    o.w = (uint8_t)255;
    reinterpret_cast<uchar4*>(rgba8)[k] = o;
}

// gaussianFunction(i, j) exactly as the reference evaluates it (float/double mix)
float gauss_weight(float sigma, float x, float y) {
    const double a = 1.0 / ((double)(sigma * sigma * 2.0f) * kRefPi);
    const float e = std::exp(-(x * x + y * y) / (2.0f * sigma * sigma));
    return (float)(a * (double)e);
}

struct Settings {  // the setters' effect on the raw GUI values
    rt_post_params p;
    explicit Settings(const rt_post_params& raw) : p(raw) {
        p.repetitions = std::max(1, raw.repetitions);
        p.sigma = std::max(0.001f, raw.sigma);
    }
};

#define POST_TRY(expr)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            rt::set_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #expr); \
            return RT_ERR_HIP;                                                             \
        }                                                                                  \
    } while (0)

int blur(const Settings& S, int W, int H, const float* src, float* dst, const float* d_w, hipStream_t st) {
    const int fs = S.p.filter_size;
    if (fs < 0) {  // the loops of boxKernel/gaussianKernel run zero times: sum = 0 (then / (2fs+1)^2)
        // 0 / n stays 0 (n >= 1 for any int fs); write zeros
        POST_TRY(hipMemsetAsync(dst, 0, (size_t)W * H * 3 * sizeof(float), st));
        return RT_OK;
    }
    const dim3 block(kTile, kTile), grid((W + kTile - 1) / kTile, (H + kTile - 1) / kTile);
    const bool gauss = S.p.kernel == RT_KERNEL_GAUSSIAN;
    if (fs <= kLdsRadius) {
        const int R = kTile + 2 * fs;
        const size_t lds = (size_t)3 * R * R * sizeof(float);
        if (gauss)
            hipLaunchKernelGGL((post_blur_kernel<true, true>), grid, block, lds, st, src, dst, W, H, fs, d_w);
        else
            hipLaunchKernelGGL((post_blur_kernel<false, true>), grid, block, lds, st, src, dst, W, H, fs, d_w);
    } else {
        if (gauss)
            hipLaunchKernelGGL((post_blur_kernel<true, false>), grid, block, 0, st, src, dst, W, H, fs, d_w);
        else
            hipLaunchKernelGGL((post_blur_kernel<false, false>), grid, block, 0, st, src, dst, W, H, fs, d_w);
    }
    POST_TRY(hipGetLastError());
    return RT_OK;
}

// applyBloomEffect (src/screen.cpp:226-275) on d_rgb in place; scratch = light | tmp
int bloom(const Settings& S, int W, int H, float* d_rgb, float* d_scratch, hipStream_t st) {
    const int opt = S.p.filtering_option;
    if (opt == RT_BLOOM_NONE) return RT_OK;
    if (opt < RT_BLOOM_NONE || opt > RT_BLOOM_ONLY_LIGHT_KERNEL) {
        rt::set_error("bloom: unknown filtering option");
        return RT_ERR_INVALID;
    }
    const int n = W * H;
    const size_t n3 = (size_t)n * 3;
    float* light = d_scratch;
    float* tmp = d_scratch + n3;
    hipLaunchKernelGGL(post_bright_kernel, dim3((n + 255) / 256), dim3(256), 0, st, d_rgb, light, n);
    POST_TRY(hipGetLastError());
    if (opt == RT_BLOOM_ONLY_LIGHT)
        return hipMemcpyAsync(d_rgb, light, n3 * sizeof(float), hipMemcpyDeviceToDevice, st) == hipSuccess ? RT_OK
                                                                                                           : RT_ERR_HIP;
    // Gaussian weight table (2fs+1)^2, host-evaluated like gaussianFunction
    float* d_w = nullptr;
    const int fs = S.p.filter_size;
    if (S.p.kernel == RT_KERNEL_GAUSSIAN && fs >= 0) {
        const int n1 = 2 * fs + 1;
        std::vector<float> w((size_t)n1 * n1);
        for (int i = -fs; i < fs + 1; ++i)
            for (int j = -fs; j < fs + 1; ++j) w[(size_t)(i + fs) * n1 + (j + fs)] = gauss_weight(S.p.sigma, (float)i, (float)j);
        POST_TRY(hipMallocAsync((void**)&d_w, w.size() * sizeof(float), st));
        POST_TRY(hipMemcpyAsync(d_w, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice, st));
        // the host vector must outlive the copy
        POST_TRY(hipStreamSynchronize(st));
    }
    int rc = RT_OK;
    const int reps = (opt == RT_BLOOM_ONLY_LIGHT_KERNEL) ? 1 : S.p.repetitions;
    for (int r = 0; r < reps && rc == RT_OK; ++r) {
        rc = blur(S, W, H, light, tmp, d_w, st);
        std::swap(light, tmp);
    }
    if (rc == RT_OK) {
        if (opt == RT_BLOOM_ONLY_LIGHT_KERNEL) {
            if (hipMemcpyAsync(d_rgb, light, n3 * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess) rc = RT_ERR_HIP;
        } else {
            hipLaunchKernelGGL(post_tone_kernel, dim3((unsigned)((n3 + 255) / 256)), dim3(256), 0, st, d_rgb, light,
                               (int)n3, opt, S.p.exposure);
            if (hipGetLastError() != hipSuccess) rc = RT_ERR_HIP;
        }
    }
    if (d_w) hipFreeAsync(d_w, st);
    return rc;
}

bool valid(const rt_post_params* p, int W, int H) {
    return p && W > 0 && H > 0 && (long long)W * H * 3 < (1ll << 31);
}

}  // namespace

extern "C" int rt_postprocess_device(const rt_post_params* p, int width, int height, float* d_rgb, float* d_scratch,
                                     void* stream) {
    if (!valid(p, width, height) || !d_rgb || (p->bloom_live && !d_scratch)) {
        rt::set_error("rt_postprocess_device: invalid argument");
        return RT_ERR_INVALID;
    }
    const Settings S(*p);
    hipStream_t st = (hipStream_t)stream;
    if (S.p.bloom_live) {
        const int rc = bloom(S, width, height, d_rgb, d_scratch, st);
        if (rc != RT_OK) return rc;
    }
    if (S.p.gamma_correction) {
        const int n3 = width * height * 3;
        hipLaunchKernelGGL(post_gamma_kernel, dim3((n3 + 255) / 256), dim3(256), 0, st, d_rgb, n3, 1.0f / S.p.gamma);
        POST_TRY(hipGetLastError());
    }
    return RT_OK;
}

extern "C" int rt_bitmap_device(const rt_post_params* p, int width, int height, float* d_rgb, float* d_scratch,
                                uint8_t* d_rgba8, void* stream) {
    if (!valid(p, width, height) || !d_rgb || !d_rgba8 || (p->filtering_option != RT_BLOOM_NONE && !d_scratch)) {
        rt::set_error("rt_bitmap_device: invalid argument");
        return RT_ERR_INVALID;
    }
    const Settings S(*p);
    hipStream_t st = (hipStream_t)stream;
    const int rc = bloom(S, width, height, d_rgb, d_scratch, st);
    if (rc != RT_OK) return rc;
    const int n = width * height;
    hipLaunchKernelGGL(post_quantize_kernel, dim3((n + 255) / 256), dim3(256), 0, st, d_rgb, d_rgba8, n);
    POST_TRY(hipGetLastError());
    return RT_OK;
}

namespace {
struct DevBufs {
    float* rgb = nullptr;
    float* scratch = nullptr;
    uint8_t* rgba = nullptr;
    ~DevBufs() {
        if (rgb) hipFree(rgb);
        if (scratch) hipFree(scratch);
        if (rgba) hipFree(rgba);
    }
};
}  // namespace

extern "C" int rt_postprocess(const rt_post_params* p, int width, int height, float* rgb) {
    if (!valid(p, width, height) || !rgb) {
        rt::set_error("rt_postprocess: invalid argument");
        return RT_ERR_INVALID;
    }
    const size_t n3 = (size_t)width * height * 3;
    DevBufs B;
    POST_TRY(hipMalloc((void**)&B.rgb, n3 * sizeof(float)));
    POST_TRY(hipMalloc((void**)&B.scratch, 2 * n3 * sizeof(float)));
    POST_TRY(hipMemcpy(B.rgb, rgb, n3 * sizeof(float), hipMemcpyHostToDevice));
    const int rc = rt_postprocess_device(p, width, height, B.rgb, B.scratch, nullptr);
    if (rc != RT_OK) return rc;
    POST_TRY(hipMemcpy(rgb, B.rgb, n3 * sizeof(float), hipMemcpyDeviceToHost));
    return RT_OK;
}

extern "C" int rt_bitmap(const rt_post_params* p, int width, int height, float* rgb, uint8_t* rgba8) {
    if (!valid(p, width, height) || !rgb || !rgba8) {
        rt::set_error("rt_bitmap: invalid argument");
        return RT_ERR_INVALID;
    }
    const size_t n = (size_t)width * height, n3 = n * 3;
    DevBufs B;
    POST_TRY(hipMalloc((void**)&B.rgb, n3 * sizeof(float)));
    POST_TRY(hipMalloc((void**)&B.scratch, 2 * n3 * sizeof(float)));
    POST_TRY(hipMalloc((void**)&B.rgba, n * 4));
    POST_TRY(hipMemcpy(B.rgb, rgb, n3 * sizeof(float), hipMemcpyHostToDevice));
    const int rc = rt_bitmap_device(p, width, height, B.rgb, B.scratch, B.rgba, nullptr);
    if (rc != RT_OK) return rc;
    POST_TRY(hipMemcpy(rgb, B.rgb, n3 * sizeof(float), hipMemcpyDeviceToHost));
    POST_TRY(hipMemcpy(rgba8, B.rgba, n * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}
