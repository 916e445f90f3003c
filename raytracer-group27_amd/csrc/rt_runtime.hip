// rt_runtime.hip -- device context behind the C-ABI: scene upload (once), launches, stats.
// Replaces BoundingVolumeHierarchy's constructor + renderRayTracing's pixel loop
// (reference src/bounding_volume_hierarchy.cpp:5-9, src/main.cpp:340-400).
//
// One shipped render path per scene-size class: the whole-traversal persistent
// kernel below 65 536 triangles, the dynamic-fetch persistent kernel above.  Nothing here reads the
// environment; the developer / test hooks are explicit context options (rt_ctx_set_option).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_amd.h"
#include "bvh_build.h"
#include "rt_build.h"
#include "rt_internal.h"
#include "rt_kernels.hip"
#include "rt_megakernel.hip"
#include "rt_wavefront.hip"

using namespace rt;

// dynamic-fetch kernel below this many triangles only when forced (RT_OPT_KERNEL): a query on a small
// scene is a handful of node visits and the per-step refill bookkeeping does not pay (measured on
// MI355X, DESIGN.md section 6: C1/C2/C5 vs C3/C4)
#define RT_DF_MIN_TRIANGLES 65536
// scenes from this many triangles build their structures on the GPU (rt_build.hip); smaller ones, and
// any scene the GPU path declines, on the host (bvh_build.cpp)
#define RT_GPU_BUILD_MIN 65536
static int g_build_mode = 0;  // rt_set_build_mode: 0 by size, 1 host, 2 GPU

// One host thread per extra device of a multi-device context: it creates that device's
// scene replica and enqueues that device's part of every split render, so the devices' host work
// (argument setup, launches, the stats read-back) runs side by side.  post() hands over one task,
// wait() returns once it has run.
class DeviceWorker {
public:
    DeviceWorker() : th_([this] { loop(); }) {}
    ~DeviceWorker() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void post(std::function<void()> f) {
        std::lock_guard<std::mutex> lk(m_);
        task_ = std::move(f);
        has_ = true;
        done_ = false;
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return done_; });
    }

private:
    void loop() {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || has_; });
            if (!has_) return;  // stop
            std::function<void()> f = std::move(task_);
            has_ = false;
            lk.unlock();
            f();
            lk.lock();
            done_ = true;
            cv_.notify_all();
        }
    }
    std::mutex m_;
    std::condition_variable cv_;
    std::function<void()> task_;
    bool has_ = false, done_ = true, stop_ = false;
    std::thread th_;  // last: starts once the members above exist
};

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevScene S{};  // quantised BVH8 nodes + triangle records in its leaf order, shading data, lights
    std::vector<void*> allocs;
    unsigned long long* d_stats = nullptr;
    unsigned long long* h_stats = nullptr;  // pinned host copy of the launch's first 13 counters (stats readback)
    float* d_img = nullptr;
    size_t img_bytes = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int nnodes = 0, nrec = 0, ntri = 0, nmesh = 0;
    int ref_nodes = 0, ref_levels = 0;
    int bvh8_depth = 0;
    bool df_ok = true;  // the BVH8 fits the dynamic-fetch kernel's LDS stack
    bool glossy_material = false;  // opaque, ks > 0, shininess != 0 (glossy_ray_count > 1 draws lobes)
    int persistent_blocks[1024] = {0};  // resident 64-lane blocks per (kernel class, variant)
    int opaque_blocks[6] = {0, 0, 0, 0, 0, 0};  // ... of the opaque-scene kernel (4 / 3 waves per SIMD; SPLIT; A/Bs)
    int tree_blocks[4] = {0, 0, 0, 0};  // ... of the recursion-tree kernel (3-wave, re-visit, checked 4-wave, 4-wave)
    // recursion-tree kernel: the lanes' pending refracted rays (KParams::frames)
    float* d_frames = nullptr;
    float4* d_plane_tab = nullptr;  // plane lights: their sample grids and normals (KParams::plane_tab)
    size_t frames_bytes = 0;
    // lights (re-uploadable: rt_update_lights)
    void* d_lights[4] = {nullptr, nullptr, nullptr, nullptr};
    // developer wave trace (RT_OPT_WAVE_TRACE)
    float* d_wave_trace = nullptr;
    size_t wave_trace_bytes = 0;
    int wave_trace_n = 0;
    int phase_trace_n = 0;  // waves with a phase trace (RT_OPT_WAVE_TRACE 2)
    int job_trace_n = 0;
    double create_ms[8] = {0};  // rt_create phases (rt_debug_create_ms)
    int built_on_gpu = 0, bvh2_nodes = 0, bvh2_depth = 0;
    // view batch (rt_render_views_device): per-view cameras, 12 floats each
    float* d_views = nullptr;
    size_t views_bytes = 0;
    // rt_ctx_set_option: test / developer hooks (defaults = the shipped path)
    int opt_kernel = RT_KERNEL_AUTO;
    int opt_coop = -1;      // -1: per render shape; 0 off; 1 drain only; 2 drain + full-wave stragglers
    int opt_coop_max = 0;   // 0: the largest count the LDS pool allows
    int opt_refill = 0;     // 0: per render shape
    int opt_wave_trace = 0;
    int opt_fan = 1;        // dynamic-fetch kernel: spherical-light samples as wave-shared fans
    int opt_interleave = -1;  // job -> pixel interleave: -1 by render shape, 0 off, 1 over 64 tiles, 2..6 over 2^k
    int opt_il_tail = 0;      // opaque batches: their last views interleaved over 16 tiles (RT_OPT_INTERLEAVE_TAIL)
    int opt_centre_first = -1;  // job -> tile: upper ranges bottom-up: -1 by render shape, 0 off, 1 on
    int opt_fan_cap = 0;      // pixels a wave may have waiting on fans before it stops taking new ones (0: default)
    int opt_dual = -1;        // dynamic-fetch steps: record and node visit in one iteration (-1 default, 0 off, 1 on)
    int opt_variant = -1;   // -1: the shipped variant for the render shape (RT_DF_BATCH / _FRAME, RT_WT_DEFAULT)
    int opt_opaque = -1;    // opaque-scene kernel: -1 where eligible (4-wave build), 0 never, 1 4-wave, 2 3-wave, 3 re-visit A/B
    int opt_tree = -1;      // recursion-tree kernel: -1 / 2 where eligible, 0 never, 1 its re-visit group stack build (A/B)
    char last_kernel[64] = {0};
    // view batches: the camera table's pinned host staging and the event of its last copy (the buffer
    // is refilled only once that copy has read it)
    float* h_views = nullptr;
    size_t h_views_bytes = 0;
    hipEvent_t ev_views = nullptr;
    // multi-device context (rt_create over a device list): replicas[0] is this context on devices[0],
    // replicas[i] a whole scene replica on devices[i] driven by workers[i]; a split render gives
    // replica i every band b with b % n == i (of the caller's bands) and lands its pixels straight in
    // the caller's images on devices[0] (peer access)
    std::vector<int> devices;
    std::vector<rt_ctx*> replicas;
    std::vector<std::unique_ptr<DeviceWorker>> workers;
    hipEvent_t ev_ready = nullptr;  // devices[0]: the caller stream's work before a split render
    hipEvent_t ev_done = nullptr;   // this replica's part of the last split render
    // the exchange of a split render: a replica with peer access to devices[0] stores its pixels straight
    // into the caller's images; one without it (no xGMI peer path, RT_OPT_PEER_STORES 0, or images the
    // library opened from another process) renders band-dense into d_bands on its own device, copies them
    // into stage[i] on devices[0] (hipMemcpyPeerAsync) and one scatter launch there puts them in place
    bool peer_ok = true;   // rt_create: peer access to devices[0] is enabled (or the same device)
    int opt_peer = -1;     // RT_OPT_PEER_STORES: -1 where peer access works, 0 never
    float* d_bands = nullptr;
    size_t bands_bytes = 0;
    std::vector<float*> stage;        // devices[0] (primary context only): replica i's band copy
    std::vector<size_t> stage_bytes;
    // wavefront path (rt_wavefront.hip): its counters, path-ray results, queues and shading points
    int opt_wavefront = -1;
    float* d_wf = nullptr;   // one allocation, carved by wf_layout
    size_t wf_bytes = 0;
    int wf_trace_blocks[12] = {0};  // resident blocks of the trace kernel's builds (plain, counting)
    int opt_wf_build = 0;          // RT_OPT_WF_BUILD
    int opt_wf_streams = 0;        // RT_OPT_WF_STREAMS (0: RT_WF_STREAMS)
    int opt_prio = -1;             // RT_OPT_PRIO (-1: by render shape)
    int opt_wf_chunk = 0;          // RT_OPT_WF_CHUNK: camera jobs per wavefront chunk at most (0: the memory budget's)
    const void* wf_last_cnt = nullptr;  // the WfCnt of the stream set that ran the last render's last wavefront chunk
                                        // (nullptr: the last render took a megakernel; rt_debug_counters)
    hipStream_t wf_streams[4] = {nullptr, nullptr, nullptr, nullptr};  // the chunks' extra streams ([0] unused)
    hipEvent_t wf_done[4] = {nullptr, nullptr, nullptr, nullptr};
};

// device ranges this library opened from other processes (rt_ipc_open): mapped for the opening device only
static std::mutex g_ipc_mu;
static std::vector<std::pair<uintptr_t, size_t>> g_ipc_ranges;
static bool ipc_mapped(const void* p) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    const uintptr_t a = (uintptr_t)p;
    for (const auto& r : g_ipc_ranges)
        if (a >= r.first && a < r.first + r.second) return true;
    return false;
}

// Image::Image + initMipmap (src/image.cpp:37-73,408-452): texel k = rgb[k*channels + 0..2] / 255.0f
// (the reference strides by the file's channel count over the 3-channel stb buffer; bytes past
// its end read as 0 here), then for square power-of-two images the chain down to 1x1, each texel
// 0.25f * (((upper-left + lower-left) + upper-right) + lower-right).  Appends every level to
// `out` (3 floats per texel); `levels` = mip levels including level 0, or 0 without a chain.
static void build_texels(const rt_texture& t, std::vector<float>& out, int& levels) {
    const size_t n = (size_t)t.width * t.height, nbytes = n * 3;
    const size_t base = out.size();
    out.resize(base + n * 3);
    for (size_t k = 0; k < n; ++k)
        for (int ch = 0; ch < 3; ++ch) {
            const size_t i = k * (size_t)t.channels + ch;
            out[base + 3 * k + ch] = (i < nbytes ? (float)t.rgb[i] : 0.0f) / 255.0f;
        }
    const int w = t.width, h = t.height;
    const bool mip = ((h & (h - 1)) == 0) && ((w & (w - 1)) == 0) && (w == h);
    levels = 0;
    if (!mip) return;
    levels = 1;
    size_t prev = base;
    for (int k = w; k > 1; k /= 2) {
        const int rw = k / 2;
        const size_t cur = out.size();
        out.resize(cur + (size_t)rw * rw * 3);
        for (int x = 0, rx = 0; x + 1 < k && rx < rw; x += 2, rx++)
            for (int y = 0, ry = 0; y + 1 < k && ry < rw; y += 2, ry++)
                for (int ch = 0; ch < 3; ++ch) {
                    const float lu = out[prev + 3 * ((size_t)y * k + x) + ch];
                    const float ll = out[prev + 3 * ((size_t)(y + 1) * k + x) + ch];
                    const float ru = out[prev + 3 * ((size_t)y * k + x + 1) + ch];
                    const float rl = out[prev + 3 * ((size_t)(y + 1) * k + x + 1) + ch];
                    out[cur + 3 * ((size_t)ry * rw + rx) + ch] = 0.25f * (((lu + ll) + ru) + rl);
                }
        prev = cur;
        ++levels;
    }
}

// d_stats: 16 counters, then the 8 per-XCD job heads (128-B apart) of the dynamic-fetch kernel
#define RT_STATS_BYTES ((RT_STATS_EXTRA + 24) * sizeof(unsigned long long))

#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) {                                                                 \
            set_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #expr);       \
            return RT_ERR_HIP;                                                                  \
        }                                                                                       \
    } while (0)

static int upload_bytes(rt_ctx* c, const void* host, size_t bytes, void** dev_out) {
    *dev_out = nullptr;
    if (bytes == 0) return RT_OK;
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, bytes));
    c->allocs.push_back(p);
    HIP_TRY(hipMemcpy(p, host, bytes, hipMemcpyHostToDevice));
    *dev_out = p;
    return RT_OK;
}

#define UP(host, count, dst)                                                          \
    do {                                                                               \
        void* p_ = nullptr;                                                            \
        int rc_ = upload_bytes(c, host, (size_t)(count) * sizeof(*(host)), &p_);       \
        if (rc_ != RT_OK) {                                                            \
            rt_destroy(c);                                                             \
            return rc_;                                                                \
        }                                                                              \
        dst = reinterpret_cast<decltype(dst)>(p_);                                     \
    } while (0)


static int ensure(rt_ctx* c, float** buf, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return RT_OK;
    if (*buf) hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc((void**)buf, bytes));
    *cap = bytes;
    return RT_OK;
}

extern "C" int rt_destroy(rt_ctx* c) {
    if (!c) return RT_OK;
    c->workers.clear();  // joins the device threads
    for (size_t i = 1; i < c->replicas.size(); ++i) rt_destroy(c->replicas[i]);
    c->replicas.clear();
    hipSetDevice(c->device);
    for (float* p : c->stage)
        if (p) hipFree(p);
    if (c->d_bands) hipFree(c->d_bands);
    if (c->ev_ready) hipEventDestroy(c->ev_ready);
    if (c->ev_done) hipEventDestroy(c->ev_done);
    if (c->ev_views) hipEventDestroy(c->ev_views);
    if (c->h_views) hipHostFree(c->h_views);
    for (void* p : c->allocs) hipFree(p);
    for (void* p : c->d_lights)
        if (p) hipFree(p);
    if (c->d_stats) hipFree(c->d_stats);
    if (c->h_stats) hipHostFree(c->h_stats);
    if (c->d_img) hipFree(c->d_img);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->d_wave_trace) hipFree(c->d_wave_trace);
    if (c->d_views) hipFree(c->d_views);
    if (c->d_frames) hipFree(c->d_frames);
    if (c->d_plane_tab) hipFree(c->d_plane_tab);
    if (c->d_wf) hipFree(c->d_wf);
    for (int k = 1; k < 4; ++k) {
        if (c->wf_streams[k]) hipStreamDestroy(c->wf_streams[k]);
        if (c->wf_done[k]) hipEventDestroy(c->wf_done[k]);
    }
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return RT_OK;
}

// glossy lobe half-width of getFinalColor (src/main.cpp:224), evaluated on the host with the
// reference's float/double mix so every device (and the oracle) uses the same bits
static float glossy_width(float shininess) {
    if (shininess == 0.0f) return 0.0f;
    return (float)((double)std::pow(0.5f, -1 / shininess) * std::sqrt(1 - std::pow(0.5, (double)(2 / shininess))));
}

// Visible devices (initialises this library's HIP runtime).
extern "C" int rt_device_count(int* n) {
    if (!n) {
        set_error("rt_device_count: null argument");
        return RT_ERR_INVALID;
    }
    *n = 0;
    const hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) {
        *n = 0;
        set_error(std::string("rt_device_count: no HIP device available (the MI355X path has no CPU fallback): ") +
                  hipGetErrorString(e));
        return RT_ERR_NO_DEVICE;
    }
    return RT_OK;
}

// Materials of the meshes and spheres as the kernels read them (+ the glossy lobe width), and the
// scene-wide flags they imply.
static void device_materials(const rt_material* mm, int nmesh, std::vector<DMat>& mats, bool& all_opaque,
                             bool& glossy) {
    mats.assign(nmesh, DMat{});
    for (int m = 0; m < nmesh; ++m) {
        const rt_material& sm = mm[m];
        for (int k = 0; k < 3; ++k) {
            mats[m].kd[k] = sm.kd[k];
            mats[m].ks[k] = sm.ks[k];
        }
        mats[m].shin = sm.shininess;
        mats[m].transp = sm.transparency;
        mats[m].gd = glossy_width(sm.shininess);
        if (sm.transparency != 1.0f) all_opaque = false;
        if (sm.transparency == 1.0f && (sm.ks[0] > 0 || sm.ks[1] > 0 || sm.ks[2] > 0) && sm.shininess != 0.0f)
            glossy = true;
    }
}

static DMat device_material(const rt_material& sm, bool& all_opaque, bool& glossy) {
    std::vector<DMat> one;
    device_materials(&sm, 1, one, all_opaque, glossy);
    return one[0];
}

// (Re-)upload the four light arrays (getPointLights & co. read them, src/shadow.cpp:106-321).
static int upload_lights(rt_ctx* c, const rt_scene_desc* d) {
    std::vector<DSpot> spots(d->num_spot_lights);
    for (int i = 0; i < d->num_spot_lights; ++i) {
        const rt_spot_light& L = d->spot_lights[i];
        for (int k = 0; k < 3; ++k) {
            spots[i].pos[k] = L.position[k];
            spots[i].dir[k] = L.direction[k];
            spots[i].color[k] = L.color[k];
        }
        // std::cos(glm::radians(light.angle)) (src/shadow.cpp:235)
        spots[i].cos_angle = std::cos(L.angle * static_cast<float>(0.01745329251994329576923690768489));
    }
    const void* src[4] = {d->point_lights, d->spherical_lights, spots.data(), d->plane_lights};
    const size_t bytes[4] = {(size_t)d->num_point_lights * sizeof(rt_point_light),
                             (size_t)d->num_spherical_lights * sizeof(rt_spherical_light),
                             spots.size() * sizeof(DSpot), (size_t)d->num_plane_lights * sizeof(rt_plane_light)};
    for (int k = 0; k < 4; ++k) {
        if (c->d_lights[k]) hipFree(c->d_lights[k]);
        c->d_lights[k] = nullptr;
        if (bytes[k] == 0) continue;
        if (!src[k]) {
            set_error("light array is null but its count is not 0");
            return RT_ERR_INVALID;
        }
        HIP_TRY(hipMalloc(&c->d_lights[k], bytes[k]));
        HIP_TRY(hipMemcpy(c->d_lights[k], src[k], bytes[k], hipMemcpyHostToDevice));
    }
    DevScene& S = c->S;
    S.pl = static_cast<const rt_point_light*>(c->d_lights[0]);
    S.sl = static_cast<const rt_spherical_light*>(c->d_lights[1]);
    S.spot = static_cast<const DSpot*>(c->d_lights[2]);
    S.plane = static_cast<const rt_plane_light*>(c->d_lights[3]);
    S.npl = d->num_point_lights;
    S.nsl = d->num_spherical_lights;
    S.nspot = d->num_spot_lights;
    S.nplane = d->num_plane_lights;
    // getPlaneLights' sample points (src/shadow.cpp:259-299) for every grid size a fan takes (k = 2..8): px of row i,
    // column j reached by the loop's own additions (py += dy per row, px += dx per column, dx = (1 / (k - 1)) * w),
    // and the light's normalize(cross(w, h)) -- float arithmetic the kernels would repeat per sample
    if (c->d_plane_tab) hipFree(c->d_plane_tab);
    c->d_plane_tab = nullptr;
    if (d->num_plane_lights > 0) {
        std::vector<float4> tab((size_t)d->num_plane_lights * RT_PLANE_TAB);
        for (int l = 0; l < d->num_plane_lights; ++l) {
            const rt_plane_light& pl = d->plane_lights[l];
            const v3 w{pl.width[0], pl.width[1], pl.width[2]}, h{pl.height[0], pl.height[1], pl.height[2]};
            float4* t = tab.data() + (size_t)l * RT_PLANE_TAB;
            for (int k = 2; k <= RT_PLANE_TAB_KMAX; ++k) {
                const v3 dx = (1.0f / (float)(k - 1)) * w, dy = (1.0f / (float)(k - 1)) * h;
                v3 py{pl.position[0], pl.position[1], pl.position[2]};
                for (int i = 0; i < k; ++i) {
                    v3 px = py;
                    for (int j = 0; j < k; ++j) {
                        t[plane_tab_at(k, i * k + j)] = make_float4(px.x, px.y, px.z, 0.0f);
                        px = px + dx;
                    }
                    py = py + dy;
                }
            }
            const v3 n = normalize(cross(w, h));
            t[RT_PLANE_TAB - 1] = make_float4(n.x, n.y, n.z, 0.0f);
        }
        HIP_TRY(hipMalloc(&c->d_plane_tab, tab.size() * sizeof(float4)));
        HIP_TRY(hipMemcpy(c->d_plane_tab, tab.data(), tab.size() * sizeof(float4), hipMemcpyHostToDevice));
    }
    return RT_OK;
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// One scene replica on one device: the acceleration structures (GPU or host build), the uploads, the
// per-render scratch.  rt_create makes one per entry of its device list.
static int create_one(const rt_scene_desc* desc, int device, rt_ctx** out) {
    const auto t_start = std::chrono::steady_clock::now();
    *out = nullptr;
    const int ntri = desc->num_triangles;
    if (ntri < 0 || (ntri > 0 && (!desc->positions || !desc->normals || !desc->mesh_index)) ||
        desc->num_meshes < 0 || (ntri > 0 && !desc->materials) || desc->num_spheres < 0 ||
        (desc->num_spheres > 0 && !desc->spheres) || desc->num_point_lights < 0 || desc->num_spherical_lights < 0 ||
        desc->num_spot_lights < 0 || desc->num_plane_lights < 0 || desc->num_textures < 0) {
        set_error("rt_create: invalid scene description");
        return RT_ERR_INVALID;
    }
    for (int t = 0; t < ntri; ++t)
        if (desc->mesh_index[t] < 0 || desc->mesh_index[t] >= desc->num_meshes) {
            set_error("rt_create: mesh_index out of range");
            return RT_ERR_INVALID;
        }
    rt_ctx* c = new rt_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        set_error("rt_create: hipSetDevice failed");
        return RT_ERR_HIP;
    }
    c->ntri = ntri;
    c->nmesh = desc->num_meshes;
    c->create_ms[0] = ms_since(t_start);  // validation + device

    // --- reference BVH (object order: triangles, then spheres) ---
    std::vector<float> sph4(desc->num_spheres * 4);
    for (int s = 0; s < desc->num_spheres; ++s) {
        for (int k = 0; k < 3; ++k) sph4[s * 4 + k] = desc->spheres[s].center[k];
        sph4[s * 4 + 3] = desc->spheres[s].radius;
    }
    // the GPU build (rt_build.hip) for large scenes; the host builders otherwise
    GpuBuild gbuild;
    bool gpu_built = false;
    double t_gpu = 0.0;
    if (g_build_mode == 2 || (g_build_mode == 0 && ntri >= RT_GPU_BUILD_MIN)) {
        std::string gerr;
        t_gpu = ms_since(t_start);
        gpu_built = gpu_build(desc->positions, ntri, sph4.data(), desc->num_spheres, gbuild, gerr);
        if (gpu_built) {  // the context owns the built records and nodes from here on (every exit frees them)
            c->allocs.push_back(gbuild.tri);
            c->allocs.push_back(gbuild.nodes);
        }
        if (!gpu_built && g_build_mode == 2) {
            set_error("rt_create: " + gerr);
            rt_destroy(c);
            return RT_ERR_INVALID;
        }
    }
    RefBvh ref;
    try {
        if (gpu_built) ref = std::move(gbuild.ref);
        else ref = build_ref_bvh(desc->positions, ntri, sph4.data(), desc->num_spheres, 4);
    } catch (const std::exception& ex) {
        set_error(std::string("rt_create: ") + ex.what());
        rt_destroy(c);
        return RT_ERR_INVALID;
    }
    c->create_ms[1] = gpu_built ? t_gpu + gbuild.ms[0] : ms_since(t_start);  // + reference BVH
    c->ref_nodes = (int)ref.nodes.size();
    c->ref_levels = ref.max_level_achieved + 1;
    if (c->ref_nodes > RT_MAX_REF_NODES) {
        set_error("rt_create: reference BVH larger than 31 nodes");
        rt_destroy(c);
        return RT_ERR_INVALID;
    }
    std::vector<DRefNode> refn(ref.nodes.size());
    for (size_t i = 0; i < ref.nodes.size(); ++i) {
        refn[i].lo[0] = ref.nodes[i].lower.x;
        refn[i].lo[1] = ref.nodes[i].lower.y;
        refn[i].lo[2] = ref.nodes[i].lower.z;
        refn[i].hi[0] = ref.nodes[i].upper.x;
        refn[i].hi[1] = ref.nodes[i].upper.y;
        refn[i].hi[2] = ref.nodes[i].upper.z;
    }
    std::vector<int> leaf_path(32 * 8, 0);
    for (size_t l = 0; l < ref.leaf_path.size(); ++l) {
        leaf_path[l * 8] = (int)ref.leaf_path[l].size();
        for (size_t k = 0; k < ref.leaf_path[l].size(); ++k) leaf_path[l * 8 + 1 + k] = ref.leaf_path[l][k];
    }

    // --- binned-SAH BVH2 (boxes inflated by eps, DESIGN.md "conservative traversal") collapsed into
    // the quantised BVH8 the kernels walk ---
    std::vector<float> chunk_max((ntri + (1 << 15) - 1) / (1 << 15) + 1, 8.0f);
    if (!gpu_built) parallel_chunks(ntri, 1 << 15, [&](int b, int e) {
        float m = 8.0f;
        for (size_t i = (size_t)b * 9; i < (size_t)e * 9; ++i) m = std::max(m, std::fabs(desc->positions[i]));
        chunk_max[b >> 15] = m;
    });
    float max_abs = 8.0f;
    for (float m : chunk_max) max_abs = std::max(max_abs, m);
    const float eps = std::ldexp(max_abs, -16);
    Bvh8 bvh8;
    if (gpu_built) {
        c->S.tri = static_cast<const float4*>(gbuild.tri);
        c->S.nodes = static_cast<const float4*>(gbuild.nodes);
        bvh8.max_depth = gbuild.max_depth;
        c->built_on_gpu = 1;
        c->bvh2_nodes = gbuild.bvh2_nodes;
        c->bvh2_depth = gbuild.bvh2_depth;
    } else {
        try {
            const Bvh2 bvh = build_bvh2(desc->positions, ntri, eps, RT_MAX_LEAF);
            bvh8 = build_bvh8(bvh, 8);
            c->bvh2_nodes = (int)bvh.nodes.size();
            c->bvh2_depth = bvh.max_depth;
        } catch (const std::exception& ex) {
            set_error(std::string("rt_create: ") + ex.what());
            rt_destroy(c);
            return RT_ERR_INVALID;
        }
    }
    c->create_ms[2] = gpu_built ? t_gpu + gbuild.ms[2] : ms_since(t_start);  // + BVH2 / BVH8
    c->bvh8_depth = bvh8.max_depth;
    c->df_ok = bvh8.max_depth + 2 < RT_STACK8;  // else the whole-traversal kernel's deeper stack
    if (bvh8.max_depth + 2 >= RT_STACK_SIZE || (!gpu_built && (int)bvh8.order.size() != ntri)) {
        set_error("rt_create: BVH8 deeper than the traversal stack");
        rt_destroy(c);
        return RT_ERR_INVALID;
    }
    c->nnodes = gpu_built ? gbuild.nnodes : (int)(bvh8.nodes.size() / RT_NODE_SDW);
    if (c->nnodes >= (1 << 23)) c->df_ok = false;  // the DIRECT group stack's entries hold child_base << 9
    c->nrec = ntri;

    // --- triangle records (64 B) in BVH8 leaf order: v0|n.x, v1|n.y, v2|n.z, D|key_brute|key_bvh|ref_leaf ---
    std::vector<float> rec(gpu_built ? 0 : (size_t)ntri * 16);
    if (!gpu_built) parallel_chunks(ntri, 1 << 15, [&](int rb, int re) {
    for (int r = rb; r < re; ++r) {
        const int t = bvh8.order[r];
        const float* p = desc->positions + (size_t)t * 9;
        const v3 v0{p[0], p[1], p[2]}, v1{p[3], p[4], p[5]}, v2{p[6], p[7], p[8]};
        // trianglePlane (src/ray_tracing.cpp:91-100)
        const v3 n = normalize(cross(v0 - v2, v1 - v2));
        const float D = dot(n, v0);
        float* o = rec.data() + (size_t)r * 16;
        o[0] = v0.x; o[1] = v0.y; o[2] = v0.z; o[3] = n.x;
        o[4] = v1.x; o[5] = v1.y; o[6] = v1.z; o[7] = n.y;
        o[8] = v2.x; o[9] = v2.y; o[10] = v2.z; o[11] = n.z;
        int ib[3] = {t, ref.tri_key[t], ref.tri_leaf[t]};
        std::memcpy(&o[12], &D, 4);
        std::memcpy(&o[13], ib, 12);
    }
    });

    c->create_ms[3] = ms_since(t_start);  // + records (the GPU build's are made with its BVH8)
    bool all_opaque = true, glossy = false;
    std::vector<DMat> mats;
    device_materials(desc->materials, desc->num_meshes, mats, all_opaque, glossy);
    std::vector<DSph> sph(desc->num_spheres);
    for (int s = 0; s < desc->num_spheres; ++s) {
        const rt_sphere& ss = desc->spheres[s];
        for (int k = 0; k < 3; ++k) sph[s].c[k] = ss.center[k];
        sph[s].r = ss.radius;
        sph[s].m = device_material(ss.material, all_opaque, glossy);
        sph[s].key_bvh = ref.sph_key[s];
        sph[s].leaf = ref.sph_leaf[s];
    }
    c->glossy_material = glossy;

    // kd textures: texels and mip chains (built here, once), per-mesh texture index
    std::vector<float> texels;
    std::vector<int4> tex_info;
    std::vector<int> mat_tex(desc->num_meshes, -1);
    for (int t = 0; t < desc->num_textures; ++t) {
        const rt_texture& tx = desc->textures[t];
        if (tx.width <= 0 || tx.height <= 0 || !tx.rgb || tx.channels < 3) {
            set_error("rt_create: texture " + std::to_string(t) + " is invalid (needs >= 3 channels)");
            rt_destroy(c);
            return RT_ERR_INVALID;
        }
        int levels = 0;
        const size_t off = texels.size() / 3;
        build_texels(tx, texels, levels);
        tex_info.push_back(make_int4((int)off, tx.width, tx.height, levels));
    }
    for (int m = 0; m < desc->num_meshes; ++m) {
        const rt_material& sm = desc->materials[m];
        if (!sm.has_texture) continue;
        if (sm.texture >= 0 && sm.texture < desc->num_textures) mat_tex[m] = sm.texture;
        else if (desc->num_textures > 0) {
            set_error("rt_create: material " + std::to_string(m) + " names texture " + std::to_string(sm.texture) +
                      " of " + std::to_string(desc->num_textures));
            rt_destroy(c);
            return RT_ERR_INVALID;
        }
    }

    c->create_ms[4] = ms_since(t_start);  // + materials, textures
    DevScene& S = c->S;
    if (!gpu_built) {
        UP(reinterpret_cast<const float4*>(rec.data()), (size_t)ntri * 4, S.tri);
        UP(reinterpret_cast<const float4*>(bvh8.nodes.data()), bvh8.nodes.size() / 4, S.nodes);
    }
    std::vector<float> uvz;
    const float* uvp = desc->texcoords;
    if (!uvp) {
        uvz.assign((size_t)ntri * 6, 0.0f);
        uvp = uvz.data();
    }
    UP(desc->normals, (size_t)ntri * 9, S.nrm);
    UP(uvp, (size_t)ntri * 6, S.uv);
    UP(desc->mesh_index, (size_t)ntri, S.mesh);
    UP(mats.data(), mats.size(), S.mats);
    UP(sph.data(), sph.size(), S.sph);
    UP(refn.data(), refn.size(), S.refn);
    UP(leaf_path.data(), leaf_path.size(), S.leaf_path);
    UP(texels.data(), texels.size(), S.tex);
    UP(tex_info.data(), tex_info.size(), S.tex_info);
    UP(mat_tex.data(), mat_tex.size(), S.mat_tex);
    S.ntex = desc->num_textures;
    S.ntri = ntri;
    S.nnodes = c->nnodes;
    S.nsph = desc->num_spheres;
    S.nref = (int)refn.size();
    S.all_opaque = all_opaque ? 1 : 0;
    c->create_ms[5] = ms_since(t_start);  // + uploads
    int rc = upload_lights(c, desc);
    if (rc != RT_OK) {
        rt_destroy(c);
        return rc;
    }
    if (hipMalloc(&c->d_stats, RT_STATS_BYTES) != hipSuccess ||
        hipHostMalloc((void**)&c->h_stats, 16 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        set_error("rt_create: HIP allocation failed");
        rt_destroy(c);
        return RT_ERR_HIP;
    }
    c->create_ms[6] = ms_since(t_start);  // total
    *out = c;
    return RT_OK;
}

static std::string last_error_text() {
    char buf[1024] = {0};
    rt_last_error(buf, sizeof(buf));
    return buf;
}

// BoundingVolumeHierarchy(Scene*) (src/bounding_volume_hierarchy.h:24) over a device list:
// a whole scene replica per device (the OpenMP threads of renderRayTracing share one read-only BVH,
// src/main.cpp:344-347; here each GPU reads its own copy), built side by side by the device threads.
extern "C" int rt_create(const rt_scene_desc* desc, const int* devices, int ndev, rt_ctx** out) {
    if (!desc || !out || !devices || ndev <= 0) {
        set_error("rt_create: null argument or empty device list");
        return RT_ERR_INVALID;
    }
    *out = nullptr;
    int nvis = 0;
    const hipError_t de = hipGetDeviceCount(&nvis);
    if (de != hipSuccess || nvis == 0) {
        set_error(std::string("rt_create: no HIP device available (the MI355X path has no CPU fallback): ") +
                  (de != hipSuccess ? hipGetErrorString(de) : "0 devices"));
        return RT_ERR_NO_DEVICE;
    }
    for (int i = 0; i < ndev; ++i)
        if (devices[i] < 0 || devices[i] >= nvis) {
            set_error("rt_create: device index out of range");
            return RT_ERR_INVALID;
        }
    std::vector<rt_ctx*> reps(ndev, nullptr);
    std::vector<int> rcs(ndev, RT_OK);
    std::vector<std::string> errs(ndev);
    std::vector<std::unique_ptr<DeviceWorker>> workers(ndev);
    for (int i = 1; i < ndev; ++i) {
        workers[i].reset(new DeviceWorker());
        workers[i]->post([&, i] {
            rcs[i] = create_one(desc, devices[i], &reps[i]);
            if (rcs[i] != RT_OK) errs[i] = last_error_text();
        });
    }
    rcs[0] = create_one(desc, devices[0], &reps[0]);
    if (rcs[0] != RT_OK) errs[0] = last_error_text();
    for (int i = 1; i < ndev; ++i) workers[i]->wait();
    int rc = RT_OK;
    std::string err;
    for (int i = 0; i < ndev && rc == RT_OK; ++i)
        if (rcs[i] != RT_OK) {
            rc = rcs[i];
            err = errs[i];
        }
    // the other devices write their pixels straight into devices[0]'s images where they have peer access
    // to it; a device without (no peer path, or enabling it fails) renders band-dense and copies (rt_ctx)
    for (int i = 1; i < ndev && rc == RT_OK; ++i) {
        if (devices[i] == devices[0]) continue;
        int can = 0;
        hipSetDevice(devices[i]);
        if (hipDeviceCanAccessPeer(&can, devices[i], devices[0]) != hipSuccess || !can) {
            reps[i]->peer_ok = false;
        } else {
            const hipError_t e = hipDeviceEnablePeerAccess(devices[0], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) reps[i]->peer_ok = false;
        }
        (void)hipGetLastError();  // (an already-enabled or refused peer leaves a sticky status)
    }
    for (int i = 0; i < ndev && rc == RT_OK; ++i) {
        hipSetDevice(devices[i]);
        if (hipEventCreateWithFlags(&reps[i]->ev_done, hipEventDisableTiming) != hipSuccess ||
            (i == 0 && hipEventCreateWithFlags(&reps[0]->ev_ready, hipEventDisableTiming) != hipSuccess)) {
            rc = RT_ERR_HIP;
            err = "rt_create: hipEventCreate failed";
        }
    }
    if (rc != RT_OK) {
        workers.clear();
        for (rt_ctx* r : reps) rt_destroy(r);
        set_error(err);
        return rc;
    }
    rt_ctx* c = reps[0];
    c->devices.assign(devices, devices + ndev);
    c->replicas = reps;
    c->stage.assign(ndev, nullptr);
    c->stage_bytes.assign(ndev, 0);
    c->workers = std::move(workers);
    hipSetDevice(devices[0]);
    *out = c;
    return RT_OK;
}

extern "C" int rt_ctx_devices(rt_ctx* c, int* out, int n) {
    if (!c) {
        set_error("rt_ctx_devices: null ctx");
        return RT_ERR_INVALID;
    }
    const int nd = (int)c->devices.size();
    for (int i = 0; i < n && i < nd && out; ++i) out[i] = c->devices[i];
    return nd;
}

// 1 per replica that stores its pixels straight into devices[0] (peer access), 0 for one that copies
extern "C" int rt_ctx_peer_stores(rt_ctx* c, int* out, int n) {
    if (!c) {
        set_error("rt_ctx_peer_stores: null ctx");
        return RT_ERR_INVALID;
    }
    const int nd = (int)c->replicas.size();
    for (int i = 0; i < n && i < nd && out; ++i)
        out[i] = (i == 0 || (c->replicas[i]->peer_ok && c->replicas[i]->opt_peer != 0)) ? 1 : 0;
    return nd;
}

// developer / test hooks of the scene build (include/rt_amd.h)
extern "C" int rt_set_build_mode(int mode) {
    if (mode < 0 || mode > 2) {
        set_error("rt_set_build_mode: mode must be 0 (by size), 1 (host) or 2 (GPU)");
        return RT_ERR_INVALID;
    }
    g_build_mode = mode;
    return RT_OK;
}

extern "C" int rt_debug_build_info(rt_ctx* c, int* out, int n) {
    if (!c || !out) return RT_ERR_INVALID;
    const int v[4] = {c->built_on_gpu, c->bvh2_nodes, c->bvh2_depth, c->nnodes};
    for (int i = 0; i < n && i < 4; ++i) out[i] = v[i];
    return RT_OK;
}

extern "C" int rt_debug_records(rt_ctx* c, float* out, int first, int count) {
    if (!c || !out || first < 0 || count < 0 || first + count > c->nrec) {
        set_error("rt_debug_records: range out of bounds");
        return RT_ERR_INVALID;
    }
    if (count == 0) return RT_OK;
    HIP_TRY(hipMemcpy(out, c->S.tri + (size_t)first * 4, (size_t)count * 64, hipMemcpyDeviceToHost));
    return RT_OK;
}

// The reference depth-4 BVH (src/bounding_volume_hierarchy.cpp:108-217) as the context's kernels use it,
// read back from the device: node boxes [nref][6] (lo, hi; BFS creation order), per node its leaf id or -1,
// and per object (triangles in scene order, then spheres) its leaf id and depth-first visit key -- a leaf's
// stored object list is its objects ordered by key.  Any output may be null; returns nref.
extern "C" int rt_debug_ref_bvh(rt_ctx* c, float* boxes, int* node_leaf, int* obj_leaf, int* obj_key) {
    if (!c) {
        set_error("rt_debug_ref_bvh: null ctx");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    const int nref = c->S.nref;
    std::vector<DRefNode> refn(nref);
    std::vector<int> paths(32 * 8);
    if (nref > 0) HIP_TRY(hipMemcpy(refn.data(), c->S.refn, nref * sizeof(DRefNode), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(paths.data(), c->S.leaf_path, paths.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int i = 0; i < nref; ++i) {
        if (boxes)
            for (int k = 0; k < 3; ++k) {
                boxes[i * 6 + k] = refn[i].lo[k];
                boxes[i * 6 + 3 + k] = refn[i].hi[k];
            }
        if (node_leaf) node_leaf[i] = -1;
    }
    if (node_leaf)
        for (int l = 0; l < 32; ++l) {
            const int cnt = paths[l * 8];
            if (cnt > 0 && cnt < 8 && paths[l * 8 + cnt] >= 0 && paths[l * 8 + cnt] < nref) node_leaf[paths[l * 8 + cnt]] = l;
        }
    if (obj_leaf || obj_key) {
        std::vector<float> rec((size_t)c->nrec * 16);
        if (c->nrec > 0) HIP_TRY(hipMemcpy(rec.data(), c->S.tri, rec.size() * sizeof(float), hipMemcpyDeviceToHost));
        for (int r = 0; r < c->nrec; ++r) {
            int sidx, key, leaf;
            std::memcpy(&sidx, &rec[(size_t)r * 16 + 13], 4);
            std::memcpy(&key, &rec[(size_t)r * 16 + 14], 4);
            std::memcpy(&leaf, &rec[(size_t)r * 16 + 15], 4);
            if (sidx < 0 || sidx >= c->ntri) continue;
            if (obj_leaf) obj_leaf[sidx] = leaf;
            if (obj_key) obj_key[sidx] = key;
        }
        std::vector<DSph> sph(c->S.nsph);
        if (!sph.empty()) HIP_TRY(hipMemcpy(sph.data(), c->S.sph, sph.size() * sizeof(DSph), hipMemcpyDeviceToHost));
        for (int s2 = 0; s2 < (int)sph.size(); ++s2) {
            if (obj_leaf) obj_leaf[c->ntri + s2] = sph[s2].leaf;
            if (obj_key) obj_key[c->ntri + s2] = sph[s2].key_bvh;
        }
    }
    return nref;
}

// rt_create's phase clock (cumulative ms: device, reference BVH, BVH2/BVH8, records, materials and
// textures, uploads, total)
extern "C" int rt_debug_create_ms(rt_ctx* c, double* out, int n) {
    if (!c || !out) return RT_ERR_INVALID;
    for (int i = 0; i < n && i < 8; ++i) out[i] = c->create_ms[i];
    return RT_OK;
}

// ImGui light edits after the BVH exists (src/main.cpp:511-613): the light arrays of `desc` replace
// the context's; geometry, materials and textures are untouched, nothing is rebuilt.
extern "C" int rt_update_lights(rt_ctx* c, const rt_scene_desc* desc) {
    if (!c || !desc || desc->num_point_lights < 0 || desc->num_spherical_lights < 0 || desc->num_spot_lights < 0 ||
        desc->num_plane_lights < 0) {
        set_error("rt_update_lights: invalid argument");
        return RT_ERR_INVALID;
    }
    for (rt_ctx* r : c->replicas) {
        // renders run on the caller's streams: wait for every one in flight on the device, so none reads
        // a half-replaced array (the ordering contract in rt_amd.h)
        HIP_TRY(hipSetDevice(r->device));
        HIP_TRY(hipDeviceSynchronize());
        const int rc = upload_lights(r, desc);
        if (rc != RT_OK) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    return RT_OK;
}

// Material edits (kd, ks, shininess, transparency of a mesh or a sphere) after the BVH exists: the
// reference's BVH and shadow culling do not depend on materials, so nothing is rebuilt.
static int update_materials_one(rt_ctx* c, int num_meshes, const rt_material* materials, int num_spheres,
                                const rt_material* sphere_materials) {
    if (!c || num_meshes != c->nmesh || num_spheres != c->S.nsph || (num_meshes > 0 && !materials) ||
        (num_spheres > 0 && !sphere_materials)) {
        set_error("rt_update_materials: counts must match the context's meshes and spheres");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());  // every render in flight on the device (caller streams), see rt_amd.h
    bool all_opaque = true, glossy = false;
    std::vector<DMat> mats;
    device_materials(materials, num_meshes, mats, all_opaque, glossy);
    std::vector<DSph> sph(num_spheres);
    if (num_spheres > 0)
        HIP_TRY(hipMemcpy(sph.data(), c->S.sph, sph.size() * sizeof(DSph), hipMemcpyDeviceToHost));
    for (int s = 0; s < num_spheres; ++s) sph[s].m = device_material(sphere_materials[s], all_opaque, glossy);
    if (!mats.empty())
        HIP_TRY(hipMemcpy(const_cast<DMat*>(c->S.mats), mats.data(), mats.size() * sizeof(DMat), hipMemcpyHostToDevice));
    if (!sph.empty())
        HIP_TRY(hipMemcpy(const_cast<DSph*>(c->S.sph), sph.data(), sph.size() * sizeof(DSph), hipMemcpyHostToDevice));
    c->S.all_opaque = all_opaque ? 1 : 0;
    c->glossy_material = glossy;  // (texture bindings cannot change here: textures are uploaded once)
    return RT_OK;
}

extern "C" int rt_update_materials(rt_ctx* c, int num_meshes, const rt_material* materials, int num_spheres,
                                   const rt_material* sphere_materials) {
    if (!c) {
        set_error("rt_update_materials: null ctx");
        return RT_ERR_INVALID;
    }
    for (rt_ctx* r : c->replicas) {
        const int rc = update_materials_one(r, num_meshes, materials, num_spheres, sphere_materials);
        if (rc != RT_OK) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    return RT_OK;
}

static int set_option_one(rt_ctx* c, int option, int value) {
    switch (option) {
        case RT_OPT_KERNEL:
            if (value < RT_KERNEL_AUTO || value > RT_KERNEL_DYNAMIC_FETCH) break;
            if (value == RT_KERNEL_DYNAMIC_FETCH && !c->df_ok) {
                set_error("rt_ctx_set_option: BVH8 too deep for the dynamic-fetch kernel's stack");
                return RT_ERR_INVALID;
            }
            c->opt_kernel = value;
            return RT_OK;
        case RT_OPT_COOP:
            if (value < -1 || value > 2) break;
            c->opt_coop = value;
            return RT_OK;
        case RT_OPT_COOP_MAX:
            if (value < 0 || value > COOP_Q) break;
            c->opt_coop_max = value;
            return RT_OK;
        case RT_OPT_REFILL:
            if (value < 0 || value > 64) break;
            c->opt_refill = value;
            return RT_OK;
        case RT_OPT_WAVE_TRACE:
            c->opt_wave_trace = value == 2 ? 2 : value ? 1 : 0;
            return RT_OK;
        case RT_OPT_FAN_CAP:
            if (value < 0 || value > 64) break;
            c->opt_fan_cap = value;
            return RT_OK;
        case RT_OPT_INTERLEAVE:
            if (value < -1 || value > 6) break;
            c->opt_interleave = value;
            return RT_OK;
        case RT_OPT_CENTRE_FIRST:
            if (value < -1 || value > 1) break;
            c->opt_centre_first = value;
            return RT_OK;
        case RT_OPT_DUAL_STEP:
            if (value < -1 || value > 1) break;
            c->opt_dual = value;
            return RT_OK;
        case RT_OPT_FAN:
            if (value < 0 || value > 1) break;
            c->opt_fan = value;
            return RT_OK;
        case RT_OPT_VARIANT:
            if (value < -1 || value > 511) break;
            c->opt_variant = value;
            return RT_OK;
        case RT_OPT_OPAQUE:
            if (value < -1 || value > 7) break;
            c->opt_opaque = value;
            return RT_OK;
        case RT_OPT_TREE:
            if (value < -1 || value > 5) break;
            c->opt_tree = value;
            return RT_OK;
        case RT_OPT_PEER_STORES:
            if (value < -1 || value > 0) break;
            c->opt_peer = value;
            return RT_OK;
        case RT_OPT_INTERLEAVE_TAIL:
            if (value < 0 || value > 65535) break;
            c->opt_il_tail = value;
            return RT_OK;
        case RT_OPT_WAVEFRONT:
            if (value < -1 || value > 64) break;
            c->opt_wavefront = value;
            return RT_OK;
        case RT_OPT_WF_BUILD:
            if (value < 0 || value > 5) break;
            c->opt_wf_build = value;
            return RT_OK;
        case RT_OPT_WF_STREAMS:
            if (value < 0 || value > 4) break;
            c->opt_wf_streams = value;
            return RT_OK;
        case RT_OPT_PRIO:
            if (value < -1 || value > 100000) break;
            c->opt_prio = value;
            return RT_OK;
        case RT_OPT_WF_CHUNK:
            if (value < 0 || (value & 63)) break;
            c->opt_wf_chunk = value;
            return RT_OK;
        default:
            set_error("rt_ctx_set_option: unknown option");
            return RT_ERR_INVALID;
    }
    set_error("rt_ctx_set_option: value out of range");
    return RT_ERR_INVALID;
}

extern "C" int rt_ctx_set_option(rt_ctx* c, int option, int value) {
    if (!c) {
        set_error("rt_ctx_set_option: null ctx");
        return RT_ERR_INVALID;
    }
    for (rt_ctx* r : c->replicas) {
        const int rc = set_option_one(r, option, value);
        if (rc != RT_OK) return rc;
    }
    return RT_OK;
}


// lights whose samples the dynamic-fetch kernel traces as wave-shared fans pay for that kernel on a
// small scene too: at least 16 and at most 64 samples per spherical or plane light (C5, 3 plane lights of
// 8 x 8 with a glass sphere: single frame 813 -> 351 ms, 4-view batch 218 -> 204 ms/frame)
static bool fans_pay(const rt_ctx* c, const KParams& K) {
    if (!c->opt_fan) return false;
    const int ns = K.S.nsl > 0 ? 1 + K.sl_m * K.sl_n : 0, np = K.S.nplane > 0 ? K.plane_k * K.plane_k : 0;
    return (ns >= 16 && ns <= 64) || (np >= 16 && np <= 64);
}

// the scene's pixels can be drawn by the opaque-scene or the recursion-tree kernel (opaque_path / tree_path
// without the class test): no textures, no glossy lobes, sample fans within a wave
static bool lite_eligible(const rt_ctx* c, const KParams& K) {
    if (c->opt_variant >= 0 || K.S.tex_on || !(K.glossy_n == 1 || !c->glossy_material)) return false;
    const bool opaque = c->opt_opaque != 0 && K.S.all_opaque && K.S.nsl == 0 && K.S.nplane == 0;
    const bool tree = c->opt_tree != 0 && c->opt_fan && (K.S.nsl == 0 || 1 + K.sl_m * K.sl_n <= 64) &&
                      (K.S.nplane == 0 || K.plane_k * K.plane_k <= 64) &&
                      (long long)K.S.npl + K.S.nsl + K.S.nspot + K.S.nplane < 65536;
    return opaque || tree;
}

// the kernel class a render runs: dynamic fetch for large scenes, sample-heavy lights and every scene the opaque or
// recursion-tree kernel draws (round 6: C2 64-view batch 0.268 -> 0.109 ms/frame, frame 0.626 -> 0.38-0.50 ms;
// profiles/r06/ab_r06e.log); whole-traversal refill for the small scenes left (textures, glossy lobes)
static bool use_df(const rt_ctx* c, const KParams& K) {
    if (!c->df_ok || c->opt_kernel == RT_KERNEL_WHOLE_TRAVERSAL) return false;
    if (c->opt_kernel == RT_KERNEL_DYNAMIC_FETCH) return true;
    return c->ntri >= RT_DF_MIN_TRIANGLES || fans_pay(c, K) || lite_eligible(c, K);
}

// Kernel variants compiled (rt_megakernel.hip RT_V_*).  The dynamic-fetch class ships two, chosen by
// render shape: view batches run the lean 4-waves-per-SIMD variant (state machine
// out of line, no node prefetch, no drain lane groups: C3 16 views 0.785 ms/frame vs 0.907 at 3 waves,
// 0.99 at 5, 1.11 for the 2-wave frame variant; C4 14.96 vs 17.8 / 18.7 / 24.1 ms/frame), single
// frames the 2-wave variant with the drain lane groups (their tail dominates: C3 2.16-2.19 vs
// 2.29-2.67 ms).  The whole-traversal class (small scenes) keeps the inline 2-wave variant (C2 0.76 vs
// 0.81 ms, C5 742 vs 804 ms).  The alternates are kept for A/B measurement (RT_OPT_VARIANT); all
// render identical bits.
#define RT_DF_BATCH (RT_V_CALL | RT_V_NOPF | RT_V_NOCOOP | RT_V_W4)
#define RT_DF_FRAME 0
#define RT_WT_DEFAULT 0
// the one A/B alternate: the batch variant with the drain lane groups, called out of line
#define RT_DF_ALT (RT_V_CALL | RT_V_NOPF | RT_V_W4)
// the opaque-scene kernel (rt_megakernel.hip persistent_opaque_kernel): 4 waves per SIMD
// by render shape: view batches at 4 waves per SIMD (C3 64 views 0.558 vs 0.573 ms/frame at 3), single frames at
// 3 (their tail is a few waves' serial chains, which run faster with more registers: 1.40-1.45 vs 1.56-1.63 ms)
#define RT_OPAQUE_V (RT_V_W4 | RT_V_NOPF)
#define RT_OPAQUE_V3 (RT_V_W3 | RT_V_NOPF)

// Renders that the opaque-scene kernel draws: pixels (not rt_shade's explicit rays) of a large scene
// (the dynamic-fetch class) whose materials are all opaque, lit by point and spot lights only, without
// textures and without glossy lobes (glossy_ray_count 1, or no glossy material).  RT_OPT_OPAQUE 0 and any
// RT_OPT_VARIANT choice select the general kernels instead.
static bool use_df(const rt_ctx* c, const KParams& K);
static bool split_ok(const KParams& K);
static bool opaque_path(const rt_ctx* c, const KParams& K, bool pixels) {
    // (small scenes with more than one light: the recursion-tree kernel draws them faster -- C2 64-view batch 0.104
    // vs 0.100 ms/frame, frame 0.459 vs 0.376 ms, profiles/r06/ab_r06m.log -- unless RT_OPT_OPAQUE asks for it)
    if (c->opt_opaque < 0 && c->ntri < RT_DF_MIN_TRIANGLES && !split_ok(K)) return false;
    return pixels && c->opt_opaque != 0 && c->opt_variant < 0 && use_df(c, K) && K.S.all_opaque && K.S.nsl == 0 &&
           K.S.nplane == 0 && !K.S.tex_on && (K.glossy_n == 1 || !c->glossy_material);
}
// the opaque kernel's build: 4 waves per SIMD for batches and single frames (round 4, with the direct group stack
// and the leaf bound 2: C3 frame 1.237 vs 1.246 ms at 3 waves, profiles/r04/ab_r04g_refill.log), with SPLIT (a
// node's shadow segment traced beside its mirror child, rt_megakernel.hip split_node) where the scene has one
// light (point or spot) and at most 16 levels (the LDS result bits): its lane keeps 3 dwords between phases, so
// the 4-wave build has no spills (31 VGPRs before) -- C3 64-view batch 0.376-0.378 -> 0.373 ms/frame, frame
// 1.045-1.074 -> 0.95-0.97 ms (profiles/r05/ab_r05m.log, ab_r05n.log).  RT_OPT_OPAQUE 1 the 4-wave build without
// SPLIT, 2 the 3-wave build, 3 the 4-wave re-visit A/B, 4 / 5 SPLIT at 4 / 3 waves, 6 / 7 SPLIT without the
// drain lane groups at 5 / 4 waves (A/Bs: 0.388 / 0.377 ms/frame, frames 1.26 / 1.14 ms)
#define RT_OPAQUE_V5S (RT_V_W5 | RT_V_NOPF | RT_V_NOCOOP | RT_V_SPLIT)   // A/B: 5 waves, no drain lane groups
#define RT_OPAQUE_V4SN (RT_V_W4 | RT_V_NOPF | RT_V_NOCOOP | RT_V_SPLIT)  // A/B: 4 waves, no drain lane groups
static bool split_ok(const KParams& K) { return K.S.npl + K.S.nspot == 1 && K.max_level < 16; }
#define RT_V5_MIN_FRAMES 13.0
static int opaque_variant(const rt_ctx* c, const KParams& K) {
    // launches of at least RT_V5_MIN_FRAMES frames' worth of pixels with SPLIT: 5 waves per SIMD without the drain
    // lane groups (round 6, every automatic variable defined: 20 spilled VGPRs instead of 33; C3 64-view batch 0.372
    // -> 0.352 ms/frame, profiles/r06/ab_r06m.log).  Its per-launch drain is longer: the views fit is 0.334 + 1.128 /
    // frames ms/frame against the 4-wave build's 0.3625 + 0.766 / frames (views_r06.log, views_r05fb.log), so the
    // builds cross at ~13 frames' worth -- a band-split launch at N = 8 GPUs (64 views x 1/8 of each frame) keeps
    // the 4-wave build with the lane groups, and so do single frames (1.13 vs 0.92 ms without them)
    const double frames = (double)std::max(1, K.n_views) * K.n_local_bands * K.band_rows / std::max(1, K.H);
    if (c->opt_opaque == -1 && frames >= RT_V5_MIN_FRAMES && split_ok(K)) return RT_OPAQUE_V5S;
    if (c->opt_opaque == 2) return RT_OPAQUE_V3;
    if (c->opt_opaque == 3) return RT_OPAQUE_V | RT_V_REVISIT;
    if (c->opt_opaque == 1 || !split_ok(K)) return RT_OPAQUE_V;
    if (c->opt_opaque == 6) return RT_OPAQUE_V5S;
    if (c->opt_opaque == 7) return RT_OPAQUE_V4SN;
    return (c->opt_opaque == 5 ? RT_OPAQUE_V3 : RT_OPAQUE_V) | RT_V_SPLIT;
}

// the recursion-tree kernel (rt_megakernel.hip persistent_tree_kernel): 4 / 3 waves per SIMD
// View batches run the 4-wave build, single frames the 3-wave one (round 6: C4 16-view batch 6.77-6.82 -> 6.09-6.13
// ms/frame, C4 frame 6.92-6.95 vs 7.32-7.57 ms at 4 waves; profiles/r06/ab_r06k*.log).  The 4-wave build faulted
// in rounds 4-5 when compiled with undef values in its IR; with every automatic variable defined (build.py
// HIP_FLAGS) it runs every size bit-identically.
#define RT_TREE_V3 (RT_V_W3 | RT_V_NOPF)
#define RT_TREE_VR (RT_V_W3 | RT_V_NOPF | RT_V_REVISIT)  // A/B: the re-visit group stack (RT_OPT_TREE 1)
// developer diagnosis of the 4-wave build's fault (RT_OPT_TREE 3): that build with every index checked (RT_V_CHK)
#define RT_TREE_V4C (RT_V_W4 | RT_V_NOPF | RT_V_CHK)
#define RT_TREE_V4 (RT_V_W4 | RT_V_NOPF)  // launches of >= 6 frames (RT_OPT_TREE 4 forces it, 5 the 3-wave build)
#define RT_TREE_V4_MIN_FRAMES 6.0

// Renders that the recursion-tree kernel draws: pixels of a dynamic-fetch-class render the opaque kernel
// does not take, without textures or glossy lobes, whose spherical and plane lights fit one fan (<= 64
// samples; fans on).  RT_OPT_TREE 0 and any RT_OPT_VARIANT choice select the general kernels instead.
static bool tree_path(const rt_ctx* c, const KParams& K, bool pixels) {
    if (!pixels || c->opt_tree == 0 || c->opt_variant >= 0 || !c->opt_fan || !use_df(c, K) || opaque_path(c, K, pixels))
        return false;
    if (K.S.tex_on || !(K.glossy_n == 1 || !c->glossy_material)) return false;
    if (K.S.nsl > 0 && 1 + K.sl_m * K.sl_n > 64) return false;
    if (K.S.nplane > 0 && K.plane_k * K.plane_k > 64) return false;
    return (long long)K.S.npl + K.S.nsl + K.S.nspot + K.S.nplane < 65536;  // TreeLane::li
}
static int tree_variant(const rt_ctx* c, const KParams& K) {
    if (c->opt_tree == 1) return RT_TREE_VR;
    if (c->opt_tree == 3) return RT_TREE_V4C;
    if (c->opt_tree == 4) return RT_TREE_V4;
    if (c->opt_tree == 5) return RT_TREE_V3;
    // by frames' worth of pixels per launch, as the opaque kernel's builds: C4 16 views over 8 / 4 / 2 GPUs' band
    // shares (2 / 4 / 8 frames) 2.17 / 2.53 / 3.96 ms/frame at 3 waves vs 2.29 / 2.57 / 3.62 at 4; C2 64 views
    // over 8 GPUs (8 frames) 0.017 vs 0.016 (profiles/r06/ab_r06v_*.log)
    const double frames = (double)std::max(1, K.n_views) * K.n_local_bands * K.band_rows / std::max(1, K.H);
    return frames >= RT_TREE_V4_MIN_FRAMES ? RT_TREE_V4 : RT_TREE_V3;
}

// by render shape: view batches and sample-fan renders run the lean 4-wave variant (C4 single frame
// with fans: 27.1 vs 30.3 ms), other single frames the 2-wave variant with the drain lane groups
static int variant_of(const rt_ctx* c, bool df, const KParams& K) {
    if (!df) return c->opt_variant >= 0 ? c->opt_variant : RT_WT_DEFAULT;
    const int v = c->opt_variant >= 0 ? c->opt_variant : ((K.n_views > 1 || K.fan) ? RT_DF_BATCH : RT_DF_FRAME);
    return K.fan ? (v | RT_V_FAN) : v;  // shape_options keeps K.fan to variants compiled with fans
}

template <bool DF, bool COUNT, bool TEX, int V>
static void launch_v(int grid, hipStream_t st, const KParams& K, const JobSrc& J) {
    if constexpr (DF)
        hipLaunchKernelGGL((persistent_df_kernel<COUNT, TEX, V>), dim3(grid), dim3(64), 0, st, K, J);
    else
        hipLaunchKernelGGL((persistent_kernel<COUNT, TEX, V>), dim3(grid), dim3(64), 0, st, K, J);
}

// every (COUNT, TEX) instance of the shipped variants; the A/B alternates plain only
template <bool COUNT, bool TEX>
static bool launch_shipped(bool df, int v, int grid, hipStream_t st, const KParams& K, const JobSrc& J) {
    if (df && v == RT_DF_BATCH) launch_v<true, COUNT, TEX, RT_DF_BATCH>(grid, st, K, J);
    else if (df && v == (RT_DF_BATCH | RT_V_FAN)) launch_v<true, COUNT, TEX, RT_DF_BATCH | RT_V_FAN>(grid, st, K, J);
    else if (df && v == RT_DF_FRAME) launch_v<true, COUNT, TEX, RT_DF_FRAME>(grid, st, K, J);
    else if (!df && v == RT_WT_DEFAULT) launch_v<false, COUNT, TEX, RT_WT_DEFAULT>(grid, st, K, J);
    else return false;
    return true;
}

template <bool COUNT>
static int launch_persistent(int grid, hipStream_t st, const KParams& K, const JobSrc& J, rt_ctx* c) {
    if (opaque_path(c, K, J.mode == 0)) {
        const int v = opaque_variant(c, K);
        if (v == (RT_OPAQUE_V | RT_V_REVISIT)) {  // A/B: the 4-wave build with the re-visit group stack
            hipLaunchKernelGGL((persistent_opaque_kernel<COUNT, RT_OPAQUE_V | RT_V_REVISIT>), dim3(grid), dim3(64), 0, st,
                               K, J);
        } else if (v == RT_OPAQUE_V3) {
            hipLaunchKernelGGL((persistent_opaque_kernel<COUNT, RT_OPAQUE_V3>), dim3(grid), dim3(64), 0, st, K, J);
        } else if (v == (RT_OPAQUE_V | RT_V_SPLIT)) {
            hipLaunchKernelGGL((persistent_opaque_kernel<COUNT, RT_OPAQUE_V | RT_V_SPLIT>), dim3(grid), dim3(64), 0, st, K, J);
        } else if (v == (RT_OPAQUE_V3 | RT_V_SPLIT)) {
            hipLaunchKernelGGL((persistent_opaque_kernel<COUNT, RT_OPAQUE_V3 | RT_V_SPLIT>), dim3(grid), dim3(64), 0, st, K, J);
        } else if (v == RT_OPAQUE_V5S) {
            hipLaunchKernelGGL((persistent_opaque_kernel<COUNT, RT_OPAQUE_V5S>), dim3(grid), dim3(64), 0, st, K, J);
        } else if (v == RT_OPAQUE_V4SN) {
            hipLaunchKernelGGL((persistent_opaque_kernel<COUNT, RT_OPAQUE_V4SN>), dim3(grid), dim3(64), 0, st, K, J);

        } else {
            hipLaunchKernelGGL((persistent_opaque_kernel<COUNT, RT_OPAQUE_V>), dim3(grid), dim3(64), 0, st, K, J);
        }
        std::snprintf(c->last_kernel, sizeof(c->last_kernel), "rt::persistent_opaque_kernel<%s, %d>",
                      COUNT ? "true" : "false", v);
        return RT_OK;
    }
    if (tree_path(c, K, J.mode == 0)) {
        const int v = tree_variant(c, K);
        if (v == RT_TREE_VR) hipLaunchKernelGGL((persistent_tree_kernel<COUNT, RT_TREE_VR>), dim3(grid), dim3(64), 0, st, K, J);
        else if (v == RT_TREE_V4C) hipLaunchKernelGGL((persistent_tree_kernel<COUNT, RT_TREE_V4C>), dim3(grid), dim3(64), 0, st, K, J);
        else if (v == RT_TREE_V4) hipLaunchKernelGGL((persistent_tree_kernel<COUNT, RT_TREE_V4>), dim3(grid), dim3(64), 0, st, K, J);
        else hipLaunchKernelGGL((persistent_tree_kernel<COUNT, RT_TREE_V3>), dim3(grid), dim3(64), 0, st, K, J);
        std::snprintf(c->last_kernel, sizeof(c->last_kernel), "rt::persistent_tree_kernel<%s, %d>",
                      COUNT ? "true" : "false", v);
        return RT_OK;
    }
    const bool df = use_df(c, K);
    const bool tex = COUNT || K.S.tex_on;  // counting builds keep the texture code (one instance each)
    const int v = variant_of(c, df, K);
    bool ok = tex ? launch_shipped<COUNT, true>(df, v, grid, st, K, J) : launch_shipped<COUNT, false>(df, v, grid, st, K, J);
    if (!ok && !COUNT && !tex) {
        ok = true;
        if (df && v == RT_DF_ALT) launch_v<true, false, false, RT_DF_ALT>(grid, st, K, J);
        else ok = false;
    }
    if (!ok) {
        set_error("kernel variant not compiled for this render (counting and textured renders: shipped variants only)");
        return RT_ERR_INVALID;
    }
    // the name rocprofv3 lists for this launch (bench.py's roofline.kernel)
    std::snprintf(c->last_kernel, sizeof(c->last_kernel), "rt::%s<%s, %s, %d>",
                  df ? "persistent_df_kernel" : "persistent_kernel", COUNT ? "true" : "false", tex ? "true" : "false",
                  v);
    return RT_OK;
}

template <bool DF, int V>
static int occupancy_of(int* per_cu) {
    if constexpr (DF)
        return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, persistent_df_kernel<false, false, V>, 64, 0);
    else
        return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, persistent_kernel<false, false, V>, 64, 0);
}

// resident 64-lane blocks of the kernel (the persistent grid)
static int persistent_grid(rt_ctx* c, const KParams& K, bool pixels) {
    if (opaque_path(c, K, pixels)) {
        const int v = opaque_variant(c, K);
        const int key = v == RT_OPAQUE_V5S ? 4 : v == RT_OPAQUE_V4SN ? 5 : ((v & RT_V_W3) ? 1 : 0) + ((v & RT_V_SPLIT) ? 2 : 0);
        if (c->opaque_blocks[key] > 0) return c->opaque_blocks[key];
        int cus = 0, per_cu = 0;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
        const hipError_t e =
            key == 5   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_opaque_kernel<false, RT_OPAQUE_V4SN>, 64, 0)
            : key == 4 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_opaque_kernel<false, RT_OPAQUE_V5S>, 64, 0)
            : key == 3 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_opaque_kernel<false, RT_OPAQUE_V3 | RT_V_SPLIT>, 64, 0)
            : key == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_opaque_kernel<false, RT_OPAQUE_V | RT_V_SPLIT>, 64, 0)
            : key == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_opaque_kernel<false, RT_OPAQUE_V3>, 64, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_opaque_kernel<false, RT_OPAQUE_V>, 64, 0);
        if (e != hipSuccess || per_cu <= 0) per_cu = 8;
        c->opaque_blocks[key] = std::max(1, cus) * per_cu;
        return c->opaque_blocks[key];
    }
    if (tree_path(c, K, pixels)) {
        const int tv = tree_variant(c, K);
        const int key = tv == RT_TREE_VR ? 1 : tv == RT_TREE_V4C ? 2 : tv == RT_TREE_V4 ? 3 : 0;
        if (c->tree_blocks[key] > 0) return c->tree_blocks[key];
        int cus = 0, per_cu = 0;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
        const hipError_t e =
            key == 3   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_tree_kernel<false, RT_TREE_V4>, 64, 0)
            : key == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_tree_kernel<false, RT_TREE_VR>, 64, 0)
            : key == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_tree_kernel<false, RT_TREE_V4C>, 64, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_tree_kernel<false, RT_TREE_V3>, 64, 0);
        if (e != hipSuccess || per_cu <= 0) per_cu = 8;
        c->tree_blocks[key] = std::max(1, cus) * per_cu;
        return c->tree_blocks[key];
    }
    const bool df = use_df(c, K);
    const int v = variant_of(c, df, K);
    const int key = (df ? 512 : 0) + (v & 511);
    if (c->persistent_blocks[key] > 0) return c->persistent_blocks[key];
    int cus = 0, per_cu = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    int e = 1;
    if (df) {
        if (v == RT_DF_BATCH) e = occupancy_of<true, RT_DF_BATCH>(&per_cu);
        else if (v == (RT_DF_BATCH | RT_V_FAN)) e = occupancy_of<true, RT_DF_BATCH | RT_V_FAN>(&per_cu);
        else if (v == RT_DF_FRAME) e = occupancy_of<true, RT_DF_FRAME>(&per_cu);
        else e = occupancy_of<true, RT_DF_ALT>(&per_cu);
    } else {
        e = occupancy_of<false, RT_WT_DEFAULT>(&per_cu);
    }
    if (e != 0 || per_cu <= 0) per_cu = 8;
    c->persistent_blocks[key] = std::max(1, cus) * per_cu;
    return c->persistent_blocks[key];
}

static int fill_params(rt_ctx* c, const rt_camera* cam, const rt_params* p, int W, int H, KParams& K) {
    if (!c || !p) {
        set_error("null argument");
        return RT_ERR_INVALID;
    }
    if (p->max_reflection_level < 0 || p->max_reflection_level >= RT_MAX_DEPTH) {
        set_error("max_reflection_level must be in [0, 15]");
        return RT_ERR_INVALID;
    }
    if (p->glossy_ray_count < 1) {
        set_error("glossy_ray_count must be >= 1");
        return RT_ERR_INVALID;
    }
    if (p->multiple_rays && !(p->sample_size == 4 || p->sample_size == 16 || p->sample_size == 64)) {
        set_error("sample_size must be 4, 16 or 64");
        return RT_ERR_INVALID;
    }
    if (p->sphere_light_ray_count < 2 && c->S.nsl > 0) {
        set_error("sphere_light_ray_count must be >= 2 (getSpherelights divides by (count - 1) / m)");
        return RT_ERR_INVALID;
    }
    if (p->plane_light_1D_ray_count < 2 && c->S.nplane > 0) {
        set_error("plane_light_1D_ray_count must be >= 2 (getPlaneLights divides by k - 1)");
        return RT_ERR_INVALID;
    }
    if (p->texture_filtering < RT_TEX_NEAREST || p->texture_filtering > RT_TEX_TRILINEAR ||
        p->out_of_bounds_x < RT_OOB_BORDER || p->out_of_bounds_x > RT_OOB_REPEAT ||
        p->out_of_bounds_y < RT_OOB_BORDER || p->out_of_bounds_y > RT_OOB_REPEAT) {
        set_error("texture_filtering / out_of_bounds rule out of range");
        return RT_ERR_INVALID;
    }
    if (p->shade_level < 0 || p->shade_level >= RT_MAX_DEPTH) {
        set_error("shade_level must be in [0, 15]");
        return RT_ERR_INVALID;
    }
    // the state machine's light cursor holds light index and sample in 16-bit fields
    // (rt_megakernel.hip Lane::li / ls)
    const int nl_max = std::max(std::max(c->S.npl, c->S.nsl), std::max(c->S.nspot, c->S.nplane));
    if (nl_max >= 32767 || (long long)p->sphere_light_ray_count >= 32767 ||
        (long long)p->plane_light_1D_ray_count * p->plane_light_1D_ray_count >= 32767) {
        set_error("more than 32766 lights of one kind or light samples per light");
        return RT_ERR_INVALID;
    }
    if ((size_t)W * (size_t)H >= (size_t)1 << 32) {
        set_error("image too large (pixel ids are 32-bit)");
        return RT_ERR_INVALID;
    }
    std::memset(&K, 0, sizeof(K));
    K.S = c->S;
    // per-render texture state (useTextures, textureFiltering, out-of-bounds rules, border colour)
    K.S.tex_on = (p->use_textures && c->S.ntex > 0) ? 1 : 0;
    K.S.tex_filter = p->texture_filtering;
    K.S.tex_oob_x = p->out_of_bounds_x;
    K.S.tex_oob_y = p->out_of_bounds_y;
    for (int k = 0; k < 3; ++k) K.S.tex_border[k] = p->border_color[k];
    K.max_level = p->max_reflection_level;
    K.shade_level = p->shade_level;
    K.glossy_n = p->glossy_ray_count;
    K.seed_lo = (uint32_t)(p->rng_seed & 0xFFFFFFFFull);
    K.seed_hi = (uint32_t)(p->rng_seed >> 32);
    K.plane_k = p->plane_light_1D_ray_count;
    K.plane_tab = c->d_plane_tab;
    K.use_bvh = p->use_bvh ? 1 : 0;
    K.refr = p->refraction_factor;
    // getSpherelights ring/spoke counts (src/shadow.cpp:190-195), host float math as the reference
    const int rc = std::max(2, p->sphere_light_ray_count);
    const int m = std::max(1, (int)(rc / std::round(std::sqrt(2 * 3.14159365358979f * rc))));
    const int n = std::max(1, (rc - 1) / m);
    K.sl_m = m;
    K.sl_n = n;
    K.sl_count = m * n + 1;
    const float angle = 2 * 3.14159365358979f / n;
    K.sl_sin = std::sin(angle);
    K.sl_1mcos = 1 - std::cos(angle);
    if (cam) {
        for (int k = 0; k < 3; ++k) K.cam[k] = cam->position[k];
        for (int k = 0; k < 4; ++k) K.q[k] = cam->quat[k];
        K.hh = cam->half_height;
        K.hw = cam->half_width;
    }
    K.W = W;
    K.H = H;
    K.n_views = 1;
    K.aa = p->anti_aliasing ? 1 : 0;
    K.multi = (!p->anti_aliasing && p->multiple_rays) ? 1 : 0;
    K.sample_size = p->sample_size;
    // getPixelRays (src/main.cpp:309-335): offsets partly in double via glm::sqrt(int)
    if (K.multi) {
        const double sq = std::sqrt((double)p->sample_size);
        K.ms_offx = (float)((double)(1.0f / (float)W) * (double)(1.0f / (sq * 2)));
        K.ms_offy = (float)((double)(1.0f / (float)H) * (double)(1.0f / (sq * 2)));
        K.ms_moves = (int)(sq - 1);
    }
    // anti-aliasing offsets (src/main.cpp:360-361)
    K.aa_offx = 1.0f / (float)W * 0.25f;
    K.aa_offy = 1.0f / (float)H * 0.25f;
    K.stats = c->d_stats;
    // dynamic-fetch refill and drain lane groups, by render shape: a single
    // frame with sample-heavy lights (spherical / plane) advances at 24 waiting lanes; frames with few
    // shadow samples per shading point and view batches advance whole waves (64), and hand the last
    // queries a full-wave refill waits for to lane groups (coop 2)
    const bool few_samples = K.S.nsl * K.sl_count + K.S.nplane * K.plane_k * K.plane_k <= 4;
    K.refill = few_samples ? 64 : 24;
    K.coop = few_samples ? 2 : 1;
    // a group of G lanes owns COOP_POOL * G / 64 pool slots: the depth-first reserve plus a breadth
    // step of min(G, 4) nodes must fit (coop_group_trace narrows its steps to the free slots above the
    // reserve); coop_max = the largest query count whose groups still do
    K.coop_reserve = 7 * (c->bvh8_depth + 1) + 8;
    K.coop_max = 0;
    for (int k = 1; k <= COOP_Q; ++k) {
        int G = 64;
        while (G > 1 && k * G > 64) G >>= 1;
        if (COOP_POOL * G / 64 >= K.coop_reserve + 8 * std::min(G, 4)) K.coop_max = k;
    }
    return RT_OK;
}

// batches (n_views > 1) advance whole waves (C3, 8 views: refill 24 -> 64 = 1.59 -> 1.37 ms/frame)
// with lane groups for the stragglers (16 views 1.29 -> 1.17 ms/frame); then the context's options
static void shape_options(const rt_ctx* c, KParams& K) {
    if (K.n_views > 1) {
        K.refill = 64;
        K.coop = 2;
    }
    if (c->opt_refill > 0) K.refill = c->opt_refill;
    // single frames: the waves whose phase is still tracing after 16 iterations issue first, so the frame's longest
    // query chains run ahead of fresh work (C3 frame 0.951-0.968 -> 0.904-0.937 ms; batches neutral, 0.374-0.377 vs
    // 0.376 ms/frame: profiles/r05/ab_r05z6_prio.log, ab_r05z7_prio.log, ab_r05z8_prio.log)
    K.prio_iters = c->opt_prio >= 0 ? c->opt_prio : (K.n_views <= 1 ? 16 : 0);
    if (c->opt_coop >= 0) K.coop = c->opt_coop;
    if (c->opt_coop_max > 0) K.coop_max = std::min(K.coop_max, c->opt_coop_max);
    if (K.coop_max <= 0) K.coop = 0;
    // spherical lights as wave-shared fans (rt_megakernel.hip FanTable): dynamic-fetch kernel, opaque
    // scenes (every sample a plain any-hit query), at most 64 samples per light (one mask)
    // spherical lights (bit 0) and plane lights (bit 1) as wave-shared fans (rt_megakernel.hip FanTable):
    // dynamic-fetch kernel, at most 64 samples per light (one mask); scenes with transparent materials
    // carry each sample's intensity
    const bool sph_fans = K.S.nsl > 0 && 1 + K.sl_m * K.sl_n <= 64;
    const bool plane_fans = K.S.nplane > 0 && K.plane_k * K.plane_k <= 64;
    K.fan = (c->opt_fan && use_df(c, K)) ? ((sph_fans ? 1 : 0) | (plane_fans ? 2 : 0)) : 0;
    if (c->opt_variant >= 0 && c->opt_variant != RT_DF_BATCH) K.fan = 0;  // fans are compiled into that variant only
    K.fan_cap = c->opt_fan_cap > 0 ? c->opt_fan_cap : 16;
    // single frames with fans: a wave's jobs spread over 64 tiles (C4 52.9 -> 31.4 ms; the tile order
    // keeps its coherence elsewhere: C3 2.18 vs 2.41 ms, C2 0.77 vs 0.98 ms)
    // ... and single frames of the opaque-scene kernel over 16 tiles (4 pixels of each per wave; round 4, with the
    // direct group stack: C3 frame 1.06 ms vs 1.20 untouched, 1.14 over 64 tiles, profiles/r04/ab_r04n_interleave.log;
    // over 64 tiles it had lost in round 3, 1.41 vs 1.33)
    const bool opq = opaque_path(c, K, true), opq_frame = K.n_views <= 1 && opq;
    const int il = c->opt_interleave >= 0 ? c->opt_interleave : (opq_frame ? 4 : (K.fan && K.n_views <= 1 ? 1 : 0));
    K.interleave = il == 1 ? 6 : il;  // log2 of the tiles a wave's jobs spread over (option 1: 64 tiles)
    K.interleave_view = 0;
    // opaque-kernel batches: the last RT_OPT_INTERLEAVE_TAIL views (the launch's drain) over 16 tiles, the rest
    // in tile order (a whole batch interleaved loses its coherence: 64 views 0.625 vs 0.407 ms/frame)
    if (opq && K.n_views > 1 && c->opt_interleave < 0 && c->opt_il_tail > 0) {
        K.interleave = 4;
        K.interleave_view = std::max(0, K.n_views - c->opt_il_tail);
    }
    // single frames of the opaque-scene kernel start every XCD range at its rows nearest the image centre: the
    // frame's longest query chains (reflections inside the object) start first (C3 frame 1.40 -> 1.33 ms; the
    // 64-view batch and the fan renders, C4 / C5, gain nothing or lose: DESIGN.md section 6c)
    K.centre_first = c->opt_centre_first >= 0 ? c->opt_centre_first : (K.n_views <= 1 && opaque_path(c, K, true) ? 1 : 0);
    // fan renders advance whole waves: the fans keep a wave's free lanes busy, so waiting for all 64
    // costs little and each pass takes many new pixels (C4 single frame, refill 24 -> 64: 27.0 -> 13.2 ms)
    if (K.fan && c->opt_refill == 0) K.refill = 64;
    // (C3 16-view batch 0.81 -> 0.71 ms/frame, C4 single frame 13.1 -> 11.1 ms; a second record per
    // step for lanes without a node visit measured slower: 0.72 / 11.4)
    K.dual = c->opt_dual >= 0 ? c->opt_dual : 1;
}

// ---- the wavefront path (rt_wavefront.hip) ----
// its scope: the opaque kernel's renders with one camera sample per pixel and at most 32 lights (one bit each)
#define RT_WF_REFILL 16             // trace kernel: waiting lanes that take new queries together (RT_OPT_WAVEFRONT 2..64)
#ifndef RT_WF_MAX_CHUNK
#define RT_WF_MAX_CHUNK ((1ll << 27) - 64)  // camera jobs per chunk at most (the segment tag's 27-bit shading point)
#endif
#define RT_WF_STREAMS 2       // streams the chunks of a large render are spread over (RT_OPT_WF_STREAMS)
#define RT_WF_MAX_STREAMS 4
#define RT_WF_BUDGET (64ull << 30)  // bytes of queues and shading points per chunk of camera jobs (at most; and
                                    // at most a third of the free HBM)
// -1 (the default) is the megakernel: no render shape measured faster on the wavefront path
static bool wf_path(const rt_ctx* c, const KParams& K) {
    if (c->opt_wavefront == 0 || !opaque_path(c, K, true) || K.aa || K.multi) return false;
    if (K.S.npl + K.S.nspot > 32) return false;
    return c->opt_wavefront > 0;
}

// the trace kernel's builds (RT_OPT_WF_BUILD): 5 waves per SIMD (default), 6, 4 with the node prefetch, 8
template <bool COUNT, int WV>
static int wf_occupancy(int* per_cu) {
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, wf_trace_kernel<COUNT, false, WV>, 64, 0);
}
static int wf_trace_grid(rt_ctx* c, bool count, int build) {
    int& g = c->wf_trace_blocks[count ? 6 + build : build];
    if (g > 0) return g;
    int cus = 0, per_cu = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    int e = 1;
    if (count) e = wf_occupancy<true, RT_WF_W5>(&per_cu);
    else if (build == 1) e = wf_occupancy<false, 6>(&per_cu);
    else if (build == 2) e = wf_occupancy<false, 4 | RT_WF_PF>(&per_cu);
    else if (build == 3) e = wf_occupancy<false, 8>(&per_cu);
    else if (build == 4) e = wf_occupancy<false, RT_WF_W5 | RT_WF_OVL>(&per_cu);
    else if (build == 5) e = wf_occupancy<false, 4 | RT_WF_OVL>(&per_cu);
    else e = wf_occupancy<false, RT_WF_W5>(&per_cu);
    if (e != 0 || per_cu <= 0) per_cu = 8;
    g = std::max(1, cus) * per_cu;
    return g;
}
template <bool COUNT, bool PRIMARY>
static void wf_launch_trace(int build, int grid, hipStream_t st, const KParams& K, const WfBufs& B) {
    if (COUNT || build == 0) hipLaunchKernelGGL((wf_trace_kernel<COUNT, PRIMARY, RT_WF_W5>), dim3(grid), dim3(64), 0, st, K, B);
    else if (build == 1) hipLaunchKernelGGL((wf_trace_kernel<false, PRIMARY, 6>), dim3(grid), dim3(64), 0, st, K, B);
    else if (build == 2) hipLaunchKernelGGL((wf_trace_kernel<false, PRIMARY, 4 | RT_WF_PF>), dim3(grid), dim3(64), 0, st, K, B);
    else if (build == 3) hipLaunchKernelGGL((wf_trace_kernel<false, PRIMARY, 8>), dim3(grid), dim3(64), 0, st, K, B);
    else if (build == 4)
        hipLaunchKernelGGL((wf_trace_kernel<false, PRIMARY, RT_WF_W5 | RT_WF_OVL>), dim3(grid), dim3(64), 0, st, K, B);
    else hipLaunchKernelGGL((wf_trace_kernel<false, PRIMARY, 4 | RT_WF_OVL>), dim3(grid), dim3(64), 0, st, K, B);
}

// A render as the wavefront of rt_wavefront.hip: the camera jobs in chunks whose worst-case queues fit
// RT_WF_BUDGET (every path ray may hit, every shading point may need a segment per light), per chunk
// T_0 S_0 T_1 S_1 ... T_{L+1} S_{L+1} (L = max_reflection_level) on the caller's stream.
template <bool COUNT>
static int launch_wavefront(rt_ctx* c, KParams& K, hipStream_t st, rt_stats* stats) {
    const long long tiles_x = (K.W + 7) / 8, tiles_y = (K.band_rows + 7) / 8;
    const long long view_jobs = tiles_x * tiles_y * K.n_local_bands * 64;
    const long long njobs = view_jobs * std::max(1, K.n_views);
    const long long pix_max = (long long)std::max(1, K.n_views) * (K.out_image ? K.H : K.view_rows) * K.W;
    if (njobs > 0x7FFFFFFFll || pix_max >= (1ll << 32)) {
        set_error("wavefront render: batch too large (job or pixel index overflows)");
        return RT_ERR_INVALID;
    }
    K.view_jobs = (int)view_jobs;
    K.interleave = 0;
    K.interleave_view = 0;
    K.centre_first = 0;
    K.refill = c->opt_wavefront >= 2 ? c->opt_wavefront : RT_WF_REFILL;
    HIP_TRY(hipMemsetAsync(c->d_stats, 0, RT_STATS_BYTES, st));
    const int nl = std::max(1, K.S.npl + K.S.nspot);
    // the camera jobs in chunks spread over up to RT_WF_STREAMS streams, so one chunk's small levels (whose
    // waves mostly wait on a few long queries) overlap another chunk's busy ones: per stream one set of
    // buffers, per camera job of a chunk two hit lists (16 B), two path-ray queues (80 B), the segment queue
    // (64 B per light) and two shading-point arrays (64 B) -- every path ray may hit
    const size_t per_job = 2 * sizeof(int4) + 2 * 80 + 64 * (size_t)nl + 2 * 64;
    size_t budget = RT_WF_BUDGET, free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) budget = std::min(budget, (size_t)(free_b / 3) + c->wf_bytes);
    const int want_streams = c->opt_wf_streams > 0 ? c->opt_wf_streams : RT_WF_STREAMS;
    const long long tiles = njobs / 64;
    // (by default only renders of at least 1 024 tiles per stream split; an explicit RT_OPT_WF_STREAMS always does)
    const int nstreams = (int)std::max<long long>(
        1, std::min<long long>(want_streams, c->opt_wf_streams > 0 ? tiles : tiles / 1024));
    long long J = std::max<long long>(64, (long long)(budget / nstreams / per_job));  // jobs per chunk (at most)
    // a segment's tag packs its shading point as h << 5 | light (rt_wavefront.hip): h < J must stay below 2^27, and
    // below the EMPTY marker's (2^27 - 1, light 31)
    J = std::min<long long>(J, RT_WF_MAX_CHUNK);
    if (c->opt_wf_chunk > 0) J = std::min<long long>(J, c->opt_wf_chunk);
    long long nchunks = std::max<long long>(nstreams, (njobs + J - 1) / J);
    nchunks = (nchunks + nstreams - 1) / nstreams * nstreams;  // whole rounds of the streams
    J = ((njobs + nchunks - 1) / nchunks + 63) / 64 * 64;
    nchunks = (njobs + J - 1) / J;
    const size_t cnt_bytes = (sizeof(WfCnt) + 255) & ~(size_t)255;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t b_hit = al(J * sizeof(int4)), b_qp = al(J * 80), b_qs = al(J * 64 * (size_t)nl), b_nd = al(J * 64);
    const size_t per_set = cnt_bytes + 2 * b_hit + 2 * b_qp + b_qs + 2 * b_nd;
    int rc = ensure(c, &c->d_wf, &c->wf_bytes, per_set * nstreams);
    if (rc != RT_OK) return rc;
    WfBufs Bs[RT_WF_MAX_STREAMS];
    for (int k = 0; k < nstreams; ++k) {
        char* base = reinterpret_cast<char*>(c->d_wf) + per_set * k;
        WfBufs& B = Bs[k];
        B = WfBufs{};
        B.cnt = reinterpret_cast<WfCnt*>(base);
        base += cnt_bytes;
        for (int q = 0; q < 2; ++q) {
            B.hit[q] = reinterpret_cast<int4*>(base);
            base += b_hit;
        }
        for (int q = 0; q < 2; ++q) {
            B.qp[q] = reinterpret_cast<float4*>(base);
            base += b_qp;
        }
        B.qs = reinterpret_cast<float4*>(base);
        base += b_qs;
        for (int q = 0; q < 2; ++q) {
            B.nodes[q] = reinterpret_cast<float4*>(base);
            base += b_nd;
        }
        B.nl = K.S.npl + K.S.nspot;
    }
    const int build = COUNT ? 0 : c->opt_wf_build;
    const int tgrid = wf_trace_grid(c, COUNT, build);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    const int sgrid = std::max(1, cus) * 8;
    // stream 0 is the caller's; the others start after the caller's earlier work and end before its later work
    hipStream_t sts[RT_WF_MAX_STREAMS] = {st};
    HIP_TRY(hipEventRecord(c->ev0, st));
    for (int k = 1; k < nstreams; ++k) {
        if (!c->wf_streams[k]) {
            HIP_TRY(hipStreamCreateWithFlags(&c->wf_streams[k], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&c->wf_done[k], hipEventDisableTiming));
        }
        sts[k] = c->wf_streams[k];
        HIP_TRY(hipStreamWaitEvent(sts[k], c->ev0, 0));
    }
    for (long long ch = 0; ch < nchunks; ++ch) {
        const int k = (int)(ch % nstreams);
        WfBufs& B = Bs[k];
        const long long g0 = ch * J;
        B.job0 = (int)g0;
        B.njobs = (int)std::min<long long>(J, njobs - g0);
        HIP_TRY(hipMemsetAsync(B.cnt, 0, sizeof(WfCnt), sts[k]));
        for (int l = 0; l <= K.max_level + 1; ++l) {
            B.level = l;
            if (l == 0)
                wf_launch_trace<COUNT, true>(build, tgrid, sts[k], K, B);
            else
                wf_launch_trace<COUNT, false>(build, tgrid, sts[k], K, B);
            hipLaunchKernelGGL((wf_shade_kernel<COUNT>), dim3(sgrid), dim3(256), 0, sts[k], K, B);
        }
    }
    HIP_TRY(hipGetLastError());
    c->wf_last_cnt = Bs[(int)((nchunks - 1) % nstreams)].cnt;
    for (int k = 1; k < nstreams; ++k) {
        HIP_TRY(hipEventRecord(c->wf_done[k], sts[k]));
        HIP_TRY(hipStreamWaitEvent(st, c->wf_done[k], 0));
    }
    HIP_TRY(hipEventRecord(c->ev1, st));
    std::snprintf(c->last_kernel, sizeof(c->last_kernel), "rt::wf_trace_kernel<%s", COUNT ? "true" : "false");
    if (stats) {
        // (into pinned memory: a pageable destination stages the copy, ~10 us more per frame)
        unsigned long long* h = c->h_stats;
        HIP_TRY(hipMemcpyAsync(h, c->d_stats, 13 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        std::memset(stats, 0, sizeof(*stats));
        stats->rays = h[0];
        stats->node_visits = h[1];
        stats->tri_tests = h[2];
        stats->hits = h[3];
        stats->ub_hits = h[12];
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
        stats->kernel_ms = ms;
        stats->node_bytes = RT_NODE_DW * 4u;
        std::memcpy(stats->kernel, c->last_kernel, sizeof(stats->kernel));
        stats->kernel[sizeof(stats->kernel) - 1] = 0;
    }
    return RT_OK;
}

static int launch_render(rt_ctx* c, KParams& K, hipStream_t st, int count_mode, rt_stats* stats) {
    const int tiles_x = (K.W + 7) / 8;
    const int tiles_y = (K.band_rows + 7) / 8;
    const long long blocks = (long long)tiles_x * tiles_y * K.n_local_bands;
    shape_options(c, K);
    if (blocks > 0 && wf_path(c, K))
        return count_mode ? launch_wavefront<true>(c, K, st, stats) : launch_wavefront<false>(c, K, st, stats);
    c->wf_last_cnt = nullptr;
    HIP_TRY(hipMemsetAsync(c->d_stats, 0, RT_STATS_BYTES, st));
    if (blocks > 0) {
        JobSrc J{};
        J.mode = 0;
        J.n_views = std::max(1, K.n_views);
        J.view_jobs = (int)(blocks * 64);
        J.njobs = J.n_views * J.view_jobs;
        K.view_jobs = J.view_jobs;
        J.counter = reinterpret_cast<int*>(c->d_stats + 7);
        J.xq = use_df(c, K) ? reinterpret_cast<int*>(c->d_stats + 16) : nullptr;
        const int grid = (int)std::min<long long>(blocks * J.n_views, persistent_grid(c, K, true));
        if (tree_path(c, K, true)) {
            // the tree kernel's frame stacks: max_level frames of 48 B per resident lane
            const size_t slots = (size_t)grid * 64;
            const int rc = ensure(c, &c->d_frames, &c->frames_bytes, slots * std::max(1, K.max_level) * 48);
            if (rc != RT_OK) return rc;
            K.frames = reinterpret_cast<float4*>(c->d_frames);
            K.frame_slots = (int)slots;
        } else if (opaque_path(c, K, true) && (opaque_variant(c, K) & RT_V_SPLIT)) {
            // SPLIT: max_level + 1 node frames of 32 B per resident lane
            const size_t slots = (size_t)grid * 64;
            const int rc = ensure(c, &c->d_frames, &c->frames_bytes, slots * (K.max_level + 1) * 32);
            if (rc != RT_OK) return rc;
            K.frames = reinterpret_cast<float4*>(c->d_frames);
            K.frame_slots = (int)slots;
        }
        if (c->opt_wave_trace) {
            const size_t ph = c->opt_wave_trace == 2 ? (size_t)grid * RT_PHASE_EV * 2 : 0;  // phase trace words
            const int rc = ensure(c, &c->d_wave_trace, &c->wave_trace_bytes,
                                  (size_t)grid * 8 * 8 + (size_t)J.njobs * 3 * 8 + ph * 8);
            if (rc != RT_OK) return rc;
            K.wave_trace = reinterpret_cast<unsigned long long*>(c->d_wave_trace);
            K.job_trace = K.wave_trace + (size_t)grid * 8;
            K.phase_trace = ph ? K.job_trace + (size_t)J.njobs * 3 : nullptr;
            HIP_TRY(hipMemsetAsync(K.job_trace, 0, ((size_t)J.njobs * 3 + ph) * 8, st));
            c->wave_trace_n = grid;
            c->job_trace_n = J.njobs;
            c->phase_trace_n = ph ? grid : 0;
        }
        HIP_TRY(hipEventRecord(c->ev0, st));
        const int lrc = count_mode ? launch_persistent<true>(grid, st, K, J, c) : launch_persistent<false>(grid, st, K, J, c);
        if (lrc != RT_OK) return lrc;
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev1, st));
    }
    if (stats) {
        // (into pinned memory: a pageable destination stages the copy, ~10 us more per frame)
        unsigned long long* h = c->h_stats;
        HIP_TRY(hipMemcpyAsync(h, c->d_stats, 13 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        std::memset(stats, 0, sizeof(*stats));
        stats->rays = h[0];
        stats->node_visits = h[1];
        stats->tri_tests = h[2];
        stats->hits = h[3];
        stats->ub_hits = h[12];
        float ms = 0.0f;
        if (blocks > 0) HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
        stats->kernel_ms = ms;
        stats->node_bytes = RT_NODE_DW * 4u;  // quantised BVH8 node
        std::memcpy(stats->kernel, c->last_kernel, sizeof(stats->kernel));
        stats->kernel[sizeof(stats->kernel) - 1] = 0;
    }
    return RT_OK;
}

static int g_count_mode = 0;  // set by rt_set_counting (counting build of the same kernel)

extern "C" int rt_set_counting(int on) {
    g_count_mode = on ? 1 : 0;
    return RT_OK;
}

// A view batch's camera table (12 floats per view: position, quat, hh, hw) into the context's device
// array, copied on the render's stream from pinned staging that outlives the call (the staging is
// refilled only after the previous batch's copy has read it).
static int upload_views(rt_ctx* c, const rt_camera* cams, int n_views, hipStream_t st, KParams& K) {
    const size_t bytes = (size_t)n_views * 12 * sizeof(float);
    int rc = ensure(c, &c->d_views, &c->views_bytes, bytes);
    if (rc != RT_OK) return rc;
    if (c->ev_views) HIP_TRY(hipEventSynchronize(c->ev_views));
    else HIP_TRY(hipEventCreateWithFlags(&c->ev_views, hipEventDisableTiming));
    if (c->h_views_bytes < bytes) {
        if (c->h_views) HIP_TRY(hipHostFree(c->h_views));
        c->h_views = nullptr;
        c->h_views_bytes = 0;
        HIP_TRY(hipHostMalloc((void**)&c->h_views, bytes, hipHostMallocDefault));
        c->h_views_bytes = bytes;
    }
    for (int i = 0; i < n_views; ++i) {
        float* o = c->h_views + 12 * i;
        for (int k = 0; k < 3; ++k) o[k] = cams[i].position[k];
        for (int k = 0; k < 4; ++k) o[3 + k] = cams[i].quat[k];
        o[7] = cams[i].half_height;
        o[8] = cams[i].half_width;
        o[9] = o[10] = o[11] = 0.0f;
    }
    HIP_TRY(hipMemcpyAsync(c->d_views, c->h_views, bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(c->ev_views, st));
    K.views = reinterpret_cast<const float*>(c->d_views);
    return RT_OK;
}

extern "C" int rt_render_device(rt_ctx* c, const rt_camera* cam, const rt_params* p, int W, int H, int band_rows,
                                int band_rank, int band_count, float* d_out, void* stream, rt_stats* stats) {
    if (!c || !cam || !p || !d_out || W <= 0 || H <= 0 || band_rows <= 0 || band_count <= 0 || band_rank < 0 ||
        band_rank >= band_count) {
        set_error("rt_render_device: invalid argument");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    KParams K;
    int rc = fill_params(c, cam, p, W, H, K);
    if (rc != RT_OK) return rc;
    const int nbands = (H + band_rows - 1) / band_rows;
    K.band_rows = band_rows;
    K.band_rank = band_rank;
    K.band_count = band_count;
    K.n_local_bands = nbands > band_rank ? (nbands - band_rank + band_count - 1) / band_count : 0;
    K.view_rows = K.n_local_bands * band_rows;
    K.out = d_out;
    hipStream_t st = (hipStream_t)stream;  // NULL: the null stream, ordered with the caller's default-stream work
    return launch_render(c, K, st, g_count_mode, stats);
}

extern "C" int rt_render_views_device(rt_ctx* c, const rt_camera* cams, int n_views, const rt_params* p, int W, int H,
                                      int band_rows, int band_rank, int band_count, float* d_out, void* stream,
                                      rt_stats* stats) {
    if (!c || !cams || n_views <= 0 || !p || !d_out || W <= 0 || H <= 0 || band_rows <= 0 || band_count <= 0 ||
        band_rank < 0 || band_rank >= band_count) {
        set_error("rt_render_views_device: invalid argument");
        return RT_ERR_INVALID;
    }
    if (n_views == 1)
        return rt_render_device(c, cams, p, W, H, band_rows, band_rank, band_count, d_out, stream, stats);
    HIP_TRY(hipSetDevice(c->device));
    KParams K;
    int rc = fill_params(c, cams, p, W, H, K);
    if (rc != RT_OK) return rc;
    const int nbands = (H + band_rows - 1) / band_rows;
    K.band_rows = band_rows;
    K.band_rank = band_rank;
    K.band_count = band_count;
    K.n_local_bands = nbands > band_rank ? (nbands - band_rank + band_count - 1) / band_count : 0;
    const long long view_jobs = (long long)((W + 7) / 8) * ((band_rows + 7) / 8) * K.n_local_bands * 64;
    if (view_jobs * n_views > 0x7FFFFFFFll) {
        set_error("rt_render_views_device: batch too large (job index overflows int)");
        return RT_ERR_INVALID;
    }
    K.out = d_out;
    K.n_views = n_views;
    // views are spaced by the padded band count every rank has (ceil(nbands / band_count)), so the
    // band_count ranks' buffers gather into one [rank][view][band][row] array whatever rank renders
    // fewer bands (rt_unpermute_views_device)
    K.view_rows = ((nbands + band_count - 1) / band_count) * band_rows;
    hipStream_t st = (hipStream_t)stream;  // NULL: the null stream, ordered with the caller's default-stream work
    rc = upload_views(c, cams, n_views, st, K);
    if (rc != RT_OK) return rc;
    return launch_render(c, K, st, g_count_mode, stats);
}

// One replica's part of an image-layout render: the bands b with b % band_count == band_rank of every
// view, each pixel written to its setPixel place in d_images (on this device or a peer's).
static int launch_image(rt_ctx* c, const rt_camera* cams, int n_views, const rt_params* p, int W, int H,
                        int band_rows, int band_rank, int band_count, float* d_images, hipStream_t st, rt_stats* stats) {
    HIP_TRY(hipSetDevice(c->device));
    KParams K;
    int rc = fill_params(c, cams, p, W, H, K);
    if (rc != RT_OK) return rc;
    const int nbands = (H + band_rows - 1) / band_rows;
    K.band_rows = band_rows;
    K.band_rank = band_rank;
    K.band_count = band_count;
    K.n_local_bands = nbands > band_rank ? (nbands - band_rank + band_count - 1) / band_count : 0;
    const long long view_jobs = (long long)((W + 7) / 8) * ((band_rows + 7) / 8) * K.n_local_bands * 64;
    if (view_jobs * n_views > 0x7FFFFFFFll || (long long)W * H * n_views * 3 >= (1ll << 40)) {
        set_error("image-layout render: batch too large (job index overflows int)");
        return RT_ERR_INVALID;
    }
    K.out = d_images;
    K.out_image = 1;
    K.view_rows = H;
    K.n_views = n_views;
    if (n_views > 1) {
        rc = upload_views(c, cams, n_views, st, K);
        if (rc != RT_OK) return rc;
    }
    return launch_render(c, K, st, g_count_mode, stats);
}

// One replica's part of a split render without peer stores: the bands b % band_count == band_rank of every
// view rendered band-dense into the replica's own d_bands ([view][local band][row][W][3]); returns the
// buffer's size in *bytes.
static int launch_bands(rt_ctx* c, const rt_camera* cams, int n_views, const rt_params* p, int W, int H, int band_rows,
                        int band_rank, int band_count, hipStream_t st, size_t* bytes, rt_stats* stats) {
    HIP_TRY(hipSetDevice(c->device));
    KParams K;
    int rc = fill_params(c, cams, p, W, H, K);
    if (rc != RT_OK) return rc;
    const int nbands = (H + band_rows - 1) / band_rows;
    const int max_local = (nbands + band_count - 1) / band_count;
    K.band_rows = band_rows;
    K.band_rank = band_rank;
    K.band_count = band_count;
    K.n_local_bands = nbands > band_rank ? (nbands - band_rank + band_count - 1) / band_count : 0;
    const long long view_jobs = (long long)((W + 7) / 8) * ((band_rows + 7) / 8) * K.n_local_bands * 64;
    if (view_jobs * n_views > 0x7FFFFFFFll) {
        set_error("split render: batch too large (job index overflows int)");
        return RT_ERR_INVALID;
    }
    *bytes = (size_t)n_views * max_local * band_rows * W * 3 * sizeof(float);
    rc = ensure(c, &c->d_bands, &c->bands_bytes, std::max<size_t>(*bytes, 4));
    if (rc != RT_OK) return rc;
    K.out = c->d_bands;
    K.n_views = n_views;
    K.view_rows = max_local * band_rows;
    if (n_views > 1) {
        rc = upload_views(c, cams, n_views, st, K);
        if (rc != RT_OK) return rc;
    }
    return launch_render(c, K, st, g_count_mode, stats);
}

static void add_stats(rt_stats& a, const rt_stats& b) {
    a.rays += b.rays;
    a.node_visits += b.node_visits;
    a.tri_tests += b.tri_tests;
    a.hits += b.hits;
    a.ub_hits += b.ub_hits;
    a.kernel_ms = std::max(a.kernel_ms, b.kernel_ms);
}

// renderRayTracing's pixel loop split over the context's devices (the OpenMP row split of
// src/main.cpp:344-347, here interleaved 8-row bands): replica i renders the caller's bands
// b % band_count == band_rank that also have (b / band_count) % n == i, on its own stream, ordered
// after the caller stream's earlier work (ev_ready) and before its later work (ev_done), every pixel
// stored straight into d_images on devices[0].  No gather and no un-permute: the pixels land where
// setPixel puts them while the frame renders.
static int render_split(rt_ctx* c, const rt_camera* cams, int n_views, const rt_params* p, int W, int H,
                        int band_rows, int band_rank, int band_count, float* d_images, hipStream_t st,
                        rt_stats* stats) {
    const int n = std::max<int>(1, (int)c->replicas.size());
    if (n == 1) return launch_image(c, cams, n_views, p, W, H, band_rows, band_rank, band_count, d_images, st, stats);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipEventRecord(c->ev_ready, st));
    std::vector<rt_stats> rs(n);
    std::vector<int> rcs(n, RT_OK);
    std::vector<std::string> errs(n);
    const int count = band_count * n;
    // peer stores, or band-dense + copy: images opened from another process are mapped for devices[0] only
    const bool foreign = ipc_mapped(d_images);
    std::vector<char> copy(n, 0);
    for (int i = 1; i < n; ++i) {
        const rt_ctx* r = c->replicas[i];
        copy[i] = (foreign && r->device != c->device) || !r->peer_ok || r->opt_peer == 0;
    }
    // the staging buffers on devices[0] (the host thread's device) before the workers copy into them
    const int nbands = (H + band_rows - 1) / band_rows;
    const size_t stage_need = (size_t)n_views * ((nbands + count - 1) / count) * band_rows * W * 3 * sizeof(float);
    for (int i = 1; i < n; ++i)
        if (copy[i]) {
            const int rc = ensure(c, &c->stage[i], &c->stage_bytes[i], std::max<size_t>(stage_need, 4));
            if (rc != RT_OK) return rc;
        }
    for (int i = 1; i < n; ++i) {
        c->workers[i]->post([&, i] {
            rt_ctx* r = c->replicas[i];
            rcs[i] = hipSetDevice(r->device) == hipSuccess && hipStreamWaitEvent(r->stream, c->ev_ready, 0) == hipSuccess
                         ? RT_OK : RT_ERR_HIP;
            if (rcs[i] == RT_OK && !copy[i]) {
                rcs[i] = launch_image(r, cams, n_views, p, W, H, band_rows, band_rank + band_count * i, count, d_images,
                                      r->stream, stats ? &rs[i] : nullptr);
            } else if (rcs[i] == RT_OK) {
                size_t bytes = 0;
                rcs[i] = launch_bands(r, cams, n_views, p, W, H, band_rows, band_rank + band_count * i, count, r->stream,
                                      &bytes, stats ? &rs[i] : nullptr);
                if (rcs[i] == RT_OK && bytes > 0 &&
                    hipMemcpyPeerAsync(c->stage[i], c->device, r->d_bands, r->device, bytes, r->stream) != hipSuccess) {
                    set_error("split render: hipMemcpyPeerAsync of the band copy failed");
                    rcs[i] = RT_ERR_HIP;
                }
            }
            if (rcs[i] == RT_OK && hipEventRecord(r->ev_done, r->stream) != hipSuccess) rcs[i] = RT_ERR_HIP;
            if (rcs[i] != RT_OK) errs[i] = last_error_text();
        });
    }
    rcs[0] = launch_image(c, cams, n_views, p, W, H, band_rows, band_rank, count, d_images, st, stats ? &rs[0] : nullptr);
    if (rcs[0] != RT_OK) errs[0] = last_error_text();
    for (int i = 1; i < n; ++i) c->workers[i]->wait();
    HIP_TRY(hipSetDevice(c->device));
    for (int i = 1; i < n; ++i)
        if (rcs[i] == RT_OK) {
            HIP_TRY(hipStreamWaitEvent(st, c->replicas[i]->ev_done, 0));
            if (copy[i]) {
                // the replica's bands from the staging copy to their setPixel places (on devices[0])
                const int rank = band_rank + band_count * i, max_local = (nbands + count - 1) / count;
                const size_t total = (size_t)n_views * max_local * band_rows * W;
                if (total > 0) {
                    hipLaunchKernelGGL(scatter_bands_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W,
                                       H, band_rows, rank, count, max_local, n_views, c->stage[i], d_images);
                    HIP_TRY(hipGetLastError());
                }
            }
        }
    for (int i = 0; i < n; ++i)
        if (rcs[i] != RT_OK) {
            set_error(errs[i].empty() ? "split render failed on device " + std::to_string(c->devices[i]) : errs[i]);
            return rcs[i];
        }
    if (stats) {
        *stats = rs[0];
        for (int i = 1; i < n; ++i) add_stats(*stats, rs[i]);
    }
    return RT_OK;
}

extern "C" int rt_render_views_image_device(rt_ctx* c, const rt_camera* cams, int n_views, const rt_params* p, int W,
                                            int H, int band_rows, int band_rank, int band_count, float* d_images,
                                            void* stream, rt_stats* stats) {
    if (!c || !cams || n_views <= 0 || !p || !d_images || W <= 0 || H <= 0 || band_rows <= 0 || band_count <= 0 ||
        band_rank < 0 || band_rank >= band_count) {
        set_error("rt_render_views_image_device: invalid argument");
        return RT_ERR_INVALID;
    }
    return render_split(c, cams, n_views, p, W, H, band_rows, band_rank, band_count, d_images, (hipStream_t)stream,
                        stats);
}

extern "C" int rt_unpermute_bands_device(int W, int H, int band_rows, int band_count, const float* d_gathered,
                                         float* d_image, void* stream) {
    if (W <= 0 || H <= 0 || band_rows <= 0 || band_count <= 0 || !d_gathered || !d_image) {
        set_error("rt_unpermute_bands_device: invalid argument");
        return RT_ERR_INVALID;
    }
    const int nbands = (H + band_rows - 1) / band_rows;
    const int max_local = (nbands + band_count - 1) / band_count;
    const size_t total = (size_t)W * H;
    hipLaunchKernelGGL(unpermute_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, W,
                       H, band_rows, band_count, max_local, d_gathered, d_image);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

extern "C" int rt_unpermute_views_device(int W, int H, int band_rows, int band_count, int n_views,
                                         const float* d_gathered, float* d_images, void* stream) {
    if (W <= 0 || H <= 0 || band_rows <= 0 || band_count <= 0 || n_views <= 0 || !d_gathered || !d_images) {
        set_error("rt_unpermute_views_device: invalid argument");
        return RT_ERR_INVALID;
    }
    const int nbands = (H + band_rows - 1) / band_rows;
    const int max_local = (nbands + band_count - 1) / band_count;
    const size_t total = (size_t)W * H * n_views;
    hipLaunchKernelGGL(unpermute_views_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       W, H, band_rows, band_count, max_local, n_views, d_gathered, d_images);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

extern "C" int rt_render(rt_ctx* c, const rt_camera* cam, const rt_params* p, int W, int H, float* rgb_out,
                         rt_stats* stats) {
    if (!c || !cam || !p || !rgb_out || W <= 0 || H <= 0) {
        set_error("rt_render: invalid argument");
        return RT_ERR_INVALID;
    }
    return rt_render_views(c, cam, 1, p, W, H, rgb_out, stats);
}

// renderRayTracing for a batch of cameras to host memory: every device of the context renders its
// bands straight into the images on devices[0], which are then copied out.
extern "C" int rt_render_views(rt_ctx* c, const rt_camera* cams, int n_views, const rt_params* p, int W, int H,
                               float* rgb_out, rt_stats* stats) {
    if (!c || !cams || n_views <= 0 || !p || !rgb_out || W <= 0 || H <= 0) {
        set_error("rt_render_views: invalid argument");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    const size_t view_img = (size_t)W * H * 3;
    int rc = ensure(c, &c->d_img, &c->img_bytes, view_img * n_views * sizeof(float));
    if (rc != RT_OK) return rc;
    rt_stats local{};
    rc = render_split(c, cams, n_views, p, W, H, 8, 0, 1, c->d_img, c->stream, &local);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(rgb_out, c->d_img, view_img * n_views * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (stats) *stats = local;
    return RT_OK;
}

// the slab test's quotient bounds against its IEEE quotients, per (box, ray) pair (rt_debug_slab_check)
__global__ void slab_check_kernel(const float* boxes, const float* rays, int n, int* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    DRefNode b;
    for (int k = 0; k < 3; ++k) {
        b.lo[k] = boxes[6 * i + k];
        b.hi[k] = boxes[6 * i + 3 + k];
    }
    const v3 o{rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]}, nd{rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]};
    out[i] = (ref_slab_div(b, o, nd) ? 1 : 0) | (ref_slab_bounds(b, o, nd) << 1);
}

extern "C" int rt_debug_slab_check(const float* boxes, const float* rays, int n, int* out) {
    if (n < 0 || (n > 0 && (!boxes || !rays || !out))) {
        set_error("rt_debug_slab_check: invalid argument");
        return RT_ERR_INVALID;
    }
    if (n == 0) return RT_OK;
    float* d_b = nullptr;
    int* d_o = nullptr;
    HIP_TRY(hipMalloc(&d_b, sizeof(float) * 12 * (size_t)n));
    hipError_t e = hipMalloc(&d_o, sizeof(int) * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(d_b, boxes, sizeof(float) * 6 * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_b + 6 * (size_t)n, rays, sizeof(float) * 6 * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(slab_check_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, d_b, d_b + 6 * (size_t)n, n, d_o);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, d_o, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost);
    hipFree(d_b);
    if (d_o) hipFree(d_o);
    if (e != hipSuccess) {
        set_error(std::string("rt_debug_slab_check: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    return RT_OK;
}

extern "C" int rt_intersect(rt_ctx* c, const rt_ray* rays, int n, int use_bvh, rt_hit* hits) {
    if (!c || n < 0 || (n > 0 && (!rays || !hits))) {
        set_error("rt_intersect: invalid argument");
        return RT_ERR_INVALID;
    }
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(c->device));
    rt_ray* d_r = nullptr;
    rt_hit* d_h = nullptr;
    HIP_TRY(hipMalloc(&d_r, sizeof(rt_ray) * n));
    if (hipMalloc(&d_h, sizeof(rt_hit) * n) != hipSuccess) {
        hipFree(d_r);
        set_error("rt_intersect: hipMalloc failed");
        return RT_ERR_HIP;
    }
    hipError_t e = hipMemcpy(d_r, rays, sizeof(rt_ray) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(intersect_kernel, dim3((n + 63) / 64), dim3(64), 0, c->stream, c->S, d_r, n, use_bvh ? 1 : 0,
                           d_h);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(hits, d_h, sizeof(rt_hit) * n, hipMemcpyDeviceToHost);
    hipFree(d_r);
    hipFree(d_h);
    if (e != hipSuccess) {
        set_error(std::string("rt_intersect: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    return RT_OK;
}

extern "C" int rt_shade(rt_ctx* c, const rt_ray* rays, int n, const rt_params* p, float* rgb, uint64_t* ray_counts) {
    if (!c || !p || n < 0 || (n > 0 && (!rays || !rgb))) {
        set_error("rt_shade: invalid argument");
        return RT_ERR_INVALID;
    }
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(c->device));
    KParams K;
    int rc = fill_params(c, nullptr, p, 1, 1, K);
    if (rc != RT_OK) return rc;
    shape_options(c, K);
    rt_ray* d_r = nullptr;
    float* d_c = nullptr;
    unsigned long long* d_n = nullptr;
    hipError_t e = hipMalloc(&d_r, sizeof(rt_ray) * n);
    if (e == hipSuccess) e = hipMalloc(&d_c, sizeof(float) * 3 * n);
    if (e == hipSuccess) e = hipMalloc(&d_n, sizeof(unsigned long long) * n);
    if (e == hipSuccess) e = hipMemcpy(d_r, rays, sizeof(rt_ray) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_stats, 0, RT_STATS_BYTES, c->stream);
    if (e == hipSuccess) {
        JobSrc J{};
        J.mode = 1;
        J.njobs = n;
        J.rays = d_r;
        J.rgb = d_c;
        J.ray_counts = d_n;
        J.n_views = 1;
        J.view_jobs = n;
        J.counter = reinterpret_cast<int*>(c->d_stats + 7);
        J.xq = use_df(c, K) ? reinterpret_cast<int*>(c->d_stats + 16) : nullptr;
        const int grid = std::min((n + 63) / 64, persistent_grid(c, K, false));
        const int lrc = g_count_mode ? launch_persistent<true>(grid, c->stream, K, J, c)
                                     : launch_persistent<false>(grid, c->stream, K, J, c);
        if (lrc != RT_OK) e = hipErrorInvalidValue;
        else e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(rgb, d_c, sizeof(float) * 3 * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && ray_counts) e = hipMemcpy(ray_counts, d_n, sizeof(uint64_t) * n, hipMemcpyDeviceToHost);
    if (d_r) hipFree(d_r);
    if (d_c) hipFree(d_c);
    if (d_n) hipFree(d_n);
    if (e != hipSuccess) {
        set_error(std::string("rt_shade: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    return RT_OK;
}

// Image::getPixel(uv, lod) of texture `texture` under the params' filtering / out-of-bounds rules
// for n (u, v, lod) triples (host buffers): the device sampler the renderer calls, for parity tests.
extern "C" int rt_texture_sample(rt_ctx* c, int texture, int n, const float* uv_lod, const rt_params* p, float* rgb) {
    if (!c || !p || n < 0 || (n > 0 && (!uv_lod || !rgb)) || texture < 0 || texture >= c->S.ntex) {
        set_error("rt_texture_sample: invalid argument");
        return RT_ERR_INVALID;
    }
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(c->device));
    KParams K;
    int rc = fill_params(c, nullptr, p, 1, 1, K);
    if (rc != RT_OK) return rc;
    float *d_in = nullptr, *d_out = nullptr;
    hipError_t e = hipMalloc(&d_in, sizeof(float) * 3 * n);
    if (e == hipSuccess) e = hipMalloc(&d_out, sizeof(float) * 3 * n);
    if (e == hipSuccess) e = hipMemcpy(d_in, uv_lod, sizeof(float) * 3 * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(tex_sample_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, K.S, texture, d_in, n,
                           d_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(rgb, d_out, sizeof(float) * 3 * n, hipMemcpyDeviceToHost);
    if (d_in) hipFree(d_in);
    if (d_out) hipFree(d_out);
    if (e != hipSuccess) {
        set_error(std::string("rt_texture_sample: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    return RT_OK;
}

// Developer counters of the last counting launch ([8..11] state-machine / traversal clocks).
extern "C" int rt_debug_counters(rt_ctx* c, uint64_t* out, int n) {
    if (!c || !out || n <= 0) return RT_ERR_INVALID;
    unsigned long long h[RT_STATS_EXTRA + 24] = {0};
    HIP_TRY(hipMemcpy(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < n && i < 32; ++i) out[i] = h[i < 16 ? i : RT_STATS_EXTRA + i - 16];
    // [50 .. 57]: the tree kernel's phase-A clocks (counting builds): finished samples and segments, owners resuming,
    // fan hand-out; [53], [54]: the opaque kernel's camera misses' node visits and records
    for (int i = 50; i < n && i < 58; ++i) out[i] = h[RT_STATS_EXTRA + 16 + (i - 50)];
    // [32 ..]: the last wavefront chunk's hits per level (WfCnt::hits of the stream set that ran it); zero when
    // the last render took a megakernel
    for (int i = 32; i < n && i < 32 + RT_MAX_DEPTH + 2; ++i) out[i] = 0;
    if (n > 32 && c->wf_last_cnt) {
        int wh[RT_MAX_DEPTH + 2] = {0};
        HIP_TRY(hipDeviceSynchronize());  // the chunk's stream set is not ordered with the null stream's copy
        HIP_TRY(hipMemcpy(wh, c->wf_last_cnt, sizeof(wh), hipMemcpyDeviceToHost));
        for (int i = 32; i < n && i < 32 + RT_MAX_DEPTH + 2; ++i) out[i] = (uint64_t)wh[i - 32];
    }
    return RT_OK;
}

extern "C" int rt_ctx_info(rt_ctx* c, int* num_nodes, int* num_tri_records, int* ref_bvh_nodes, int* ref_bvh_levels) {
    if (!c) {
        set_error("rt_ctx_info: null ctx");
        return RT_ERR_INVALID;
    }
    if (num_nodes) *num_nodes = c->nnodes;
    if (num_tri_records) *num_tri_records = c->nrec;
    if (ref_bvh_nodes) *ref_bvh_nodes = c->ref_nodes;
    if (ref_bvh_levels) *ref_bvh_levels = c->ref_levels;
    return RT_OK;
}

extern "C" int rt_debug_job_trace(rt_ctx* c, uint64_t* out, int max_jobs) {
    if (!c || !out || max_jobs <= 0) return RT_ERR_INVALID;
    const int n = std::min(max_jobs, c->job_trace_n);
    if (n > 0)
        HIP_TRY(hipMemcpy(out, reinterpret_cast<unsigned long long*>(c->d_wave_trace) + (size_t)c->wave_trace_n * 8,
                          (size_t)n * 3 * 8, hipMemcpyDeviceToHost));
    return n;
}

extern "C" int rt_debug_phase_trace(rt_ctx* c, uint64_t* out, int max_waves) {
    if (!c || !out || max_waves <= 0) return RT_ERR_INVALID;
    const int n = std::min(max_waves, c->phase_trace_n);
    if (n > 0)
        HIP_TRY(hipMemcpy(out,
                          reinterpret_cast<unsigned long long*>(c->d_wave_trace) + (size_t)c->wave_trace_n * 8 +
                              (size_t)c->job_trace_n * 3,
                          (size_t)n * RT_PHASE_EV * 2 * 8, hipMemcpyDeviceToHost));
    return n;
}

extern "C" int rt_debug_wave_trace(rt_ctx* c, uint64_t* out, int max_waves) {
    if (!c || !out || max_waves <= 0) return RT_ERR_INVALID;
    const int n = std::min(max_waves, c->wave_trace_n);
    if (n > 0) HIP_TRY(hipMemcpy(out, c->d_wave_trace, (size_t)n * 8 * 8, hipMemcpyDeviceToHost));
    return n;
}

extern "C" int rt_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    if (!ctr || !key || !out) {
        set_error("rt_philox4x32_10: null argument");
        return RT_ERR_INVALID;
    }
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    philox4x32_10(c, key[0], key[1]);
    for (int k = 0; k < 4; ++k) out[k] = c[k];
    return RT_OK;
}

extern "C" int rt_selftest_math(rt_ctx* c, const float* x, const float* y, int n, float* out) {
    if (!c || n <= 0 || !x || !y || !out) {
        set_error("rt_selftest_math: invalid argument");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc(&dx, n * 4));
    HIP_TRY(hipMalloc(&dy, n * 4));
    HIP_TRY(hipMalloc(&dout, n * 16));
    hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dy, y, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, dx, dy, n, dout);
    hipStreamSynchronize(c->stream);
    hipMemcpy(out, dout, n * 16, hipMemcpyDeviceToHost);
    hipFree(dx);
    hipFree(dy);
    hipFree(dout);
    return RT_OK;
}

// ---- device buffers shared across processes (the one-process-per-GPU split, bench.py N > 1) ----
// Rank 0 allocates the images and exports them; every rank opens them and renders its bands straight
// into them (rt_render_views_image_device), so the framebuffer exchange is the kernels' own pixel
// stores over xGMI while they render -- no gather step after the frame.
// Measured on the MI355X image (ROCm 7.2, dmabuf IPC: HSA_ENABLE_IPC_MODE_LEGACY=0): hipIpcOpenMemHandle of an
// exported buffer of 2^31 bytes or more never returns in the importing process (2 145 386 496 B maps in
// milliseconds, 2 147 483 648 B does not return within 60 s: tools/ipc_probe.py --bytes),
// so such a buffer is refused here, where the exporter can fall back, instead of hanging its importers.
#define RT_IPC_MAX_BYTES ((size_t)1 << 31)
extern "C" int rt_ipc_alloc(int device, size_t bytes, void** d_ptr, uint8_t handle[RT_IPC_HANDLE_BYTES]) {
    if (!d_ptr || !handle || bytes == 0) {
        set_error("rt_ipc_alloc: invalid argument");
        return RT_ERR_INVALID;
    }
    if (bytes >= RT_IPC_MAX_BYTES) {
        *d_ptr = nullptr;
        set_error("rt_ipc_alloc: " + std::to_string(bytes) + " bytes: buffers of 2 GiB or more are not exported "
                  "(this runtime's hipIpcOpenMemHandle never returns for them in the importing process)");
        return RT_ERR_INVALID;
    }
    *d_ptr = nullptr;
    HIP_TRY(hipSetDevice(device));
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, bytes));
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, p);
    if (e != hipSuccess) {
        hipFree(p);
        set_error(std::string("rt_ipc_alloc: hipIpcGetMemHandle: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    static_assert(sizeof(h) == RT_IPC_HANDLE_BYTES, "IPC handle size");
    std::memcpy(handle, &h, RT_IPC_HANDLE_BYTES);
    *d_ptr = p;
    return RT_OK;
}

extern "C" int rt_ipc_open(int device, const uint8_t handle[RT_IPC_HANDLE_BYTES], void** d_ptr) {
    if (!d_ptr || !handle) {
        set_error("rt_ipc_open: invalid argument");
        return RT_ERR_INVALID;
    }
    *d_ptr = nullptr;
    HIP_TRY(hipSetDevice(device));
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, RT_IPC_HANDLE_BYTES);
    HIP_TRY(hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess));
    // remembered: a multi-device context's other replicas cannot store into this mapping (render_split)
    void* base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, *d_ptr) != hipSuccess || !base) {
        base = *d_ptr;
        size = 1;
    }
    (void)hipGetLastError();
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    g_ipc_ranges.emplace_back((uintptr_t)base, size);
    return RT_OK;
}

extern "C" int rt_ipc_close(void* d_ptr) {
    if (!d_ptr) return RT_OK;
    {
        std::lock_guard<std::mutex> lk(g_ipc_mu);
        for (size_t i = 0; i < g_ipc_ranges.size(); ++i)
            if ((uintptr_t)d_ptr >= g_ipc_ranges[i].first &&
                (uintptr_t)d_ptr < g_ipc_ranges[i].first + g_ipc_ranges[i].second) {
                g_ipc_ranges.erase(g_ipc_ranges.begin() + i);
                break;
            }
    }
    HIP_TRY(hipIpcCloseMemHandle(d_ptr));
    return RT_OK;
}

extern "C" int rt_device_free(int device, void* d_ptr) {
    if (!d_ptr) return RT_OK;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipFree(d_ptr));
    return RT_OK;
}

// Wait for every stream of the device (the split render's device threads enqueue on their own streams).
extern "C" int rt_device_synchronize(int device) {
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipDeviceSynchronize());
    return RT_OK;
}

// Synchronous device-to-host copy (a buffer this library allocated or opened, e.g. rt_ipc_alloc's).
extern "C" int rt_memcpy_dtoh(void* host, const void* d_ptr, size_t bytes) {
    if ((!host || !d_ptr) && bytes) {
        set_error("rt_memcpy_dtoh: null pointer");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipMemcpy(host, d_ptr, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}
