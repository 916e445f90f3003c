// rt_runtime.hip -- device context behind the C-ABI: scene upload (once), launches, stats.
// Replaces BoundingVolumeHierarchy's constructor + renderRayTracing's pixel loop
// (reference src/bounding_volume_hierarchy.cpp:5-9, src/main.cpp:340-400).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "bvh_build.h"
#include "rt_internal.h"
#include "rt_kernels.hip"
#include "rt_megakernel.hip"
#include "rt_wavefront.hip"
#include "rt_packet.hip"
#include "rt_schedule.hip"

using namespace rt;

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevScene S{};
    DevScene S8{};  // same scene, nodes/records of the quantised wide BVH (bw > 2)
    int bw = 8;     // BVH width the persistent kernel walks (fixed at rt_create)
    std::vector<void*> allocs;
    unsigned long long* d_stats = nullptr;
    float* d_fb = nullptr;
    size_t fb_bytes = 0;
    float* d_img = nullptr;
    size_t img_bytes = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int nnodes = 0, nrec = 0, ntri = 0;
    int ref_nodes = 0, ref_levels = 0;
    int bvh_depth = 0;
    bool glossy_material = false;  // opaque, ks > 0, shininess != 0 (glossy_ray_count > 1 would call rand())
    int persistent_blocks[5] = {0, 0, 0, 0, 0};  // resident 64-lane blocks per WPE variant
    // wavefront path (rt_wavefront.hip): queues, path state, frames, counters
    float* d_wf_st = nullptr;  // 2 x WF_NFIELDS x cap
    size_t wf_st_bytes = 0;
    float* d_wf_res = nullptr;  // res_t[cap] | res_rec[cap]
    size_t wf_res_bytes = 0;
    float* d_wf_frames = nullptr;
    size_t wf_frames_bytes = 0;
    int* d_wf_cnt = nullptr;  // n[0], n[1], head, pad
    int* h_wf_cnt = nullptr;  // pinned readback
    int wf_trace_blocks[5] = {0, 0, 0, 0, 0};
    std::vector<hipEvent_t> wf_ev;  // trace-launch event pairs
    // primary packet pass (rt_packet.hip): per-job primary hit
    float* d_pre = nullptr;  // pre_t[njobs] | pre_rec[njobs]
    size_t pre_bytes = 0;
    int bvh8_depth = 0;
    bool df_ok = true;
    // longest-first schedule (rt_schedule.hip): tile hits | tile offsets | job order
    float* d_sched = nullptr;
    size_t sched_bytes = 0;
    // cost-ordered schedule (RT_SCHED=2): per-job query counts of the previous frame + partition
    float* d_cost = nullptr;  // cost[njobs] | block hist [16][nblk] | order[njobs]
    size_t cost_bytes = 0;
    long long cost_key = -1;  // launch geometry the stored costs belong to
    // developer wave trace (RT_WAVE_TRACE=1)
    float* d_wave_trace = nullptr;
    size_t wave_trace_bytes = 0;
    int wave_trace_n = 0;
    // view batch (rt_render_views_device): per-view cameras, 12 floats each
    float* d_views = nullptr;
    size_t views_bytes = 0;
};

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

// waves per SIMD the persistent kernel is compiled for (register cap); RT_WPE overrides for A/B runs
static int wpe() {
    const char* w = std::getenv("RT_WPE");
    const int v = w ? std::atoi(w) : 2;
    return (v == 1 || v == 3 || v == 4) ? v : 2;
}

// BVH the persistent kernel walks, read once at rt_create: 8 (quantised 8-wide, default),
// 4 (same node format, 4 slots) or 2 (binary, full-precision boxes); RT_BVH selects for A/B runs
static int bvh_width_env() {
    const char* b = std::getenv("RT_BVH");
    const int v = b ? std::atoi(b) : 8;
    return (v == 2 || v == 4) ? v : 8;
}

// RT_KERNEL: "tile" (rt_kernels.hip render_kernel), "persistent" (whole-traversal refill),
// default: the dynamic-fetch persistent kernel (per-node-visit refill)
// Default (no RT_KERNEL): whole-traversal refill for small scenes, where a query is a handful of
// node visits and the per-step refill bookkeeping does not pay; dynamic fetch for large ones
// (measured on MI355X, DESIGN.md section 6: C1/C2/C5 vs C3/C4).
static bool use_whole_traversal_kernel(int ntri) {
    const char* k = std::getenv("RT_KERNEL");
    if (k && std::strcmp(k, "persistent") == 0) return true;
    if (k && std::strcmp(k, "df") == 0) return false;
    return ntri < 65536;
}

// waiting lanes that end a traversal phase of the dynamic-fetch kernel; RT_REFILL overrides
// (measured on MI355X, 10 rotated rounds: C3 2.46 / 2.38 / 2.34 ms at 16 / 20 / 24, C4 43.0 ms at all three)
static int refill_threshold() {
    const char* r = std::getenv("RT_REFILL");
    const int v = r ? std::atoi(r) : 24;
    return std::min(64, std::max(1, v));
}

// lanes with postponed leaf records that start a leaf phase (64: only when no lane can visit a
// node); RT_LEAFBATCH overrides
static int leaf_batch_threshold() {
    const char* r = std::getenv("RT_LEAFBATCH");
    const int v = r ? std::atoi(r) : 0;
    return std::min(64, std::max(0, v));  // 0: if-if (one leaf record or node visit per iteration)
}

template <bool COUNT, int BW>
static void launch_wide(int grid, hipStream_t st, const KParams& K, const JobSrc& J, bool df_ok) {
    if (df_ok && !use_whole_traversal_kernel(K.S.ntri)) {
        if (wpe() == 1)
            hipLaunchKernelGGL((persistent_df_kernel<COUNT, 1, BW>), dim3(grid), dim3(64), 0, st, K, J);
        else if (wpe() == 4)
            hipLaunchKernelGGL((persistent_df_kernel<COUNT, 4, BW>), dim3(grid), dim3(64), 0, st, K, J);
        else if (wpe() == 3)
            hipLaunchKernelGGL((persistent_df_kernel<COUNT, 3, BW>), dim3(grid), dim3(64), 0, st, K, J);
        else if (!COUNT && !K.S.tex_on)  // production variant: no texture code at all
            hipLaunchKernelGGL((persistent_df_kernel<false, 2, BW, false>), dim3(grid), dim3(64), 0, st, K, J);
        else
            hipLaunchKernelGGL((persistent_df_kernel<COUNT, 2, BW>), dim3(grid), dim3(64), 0, st, K, J);
        return;
    }
    if (wpe() == 1)
        hipLaunchKernelGGL((persistent_kernel<COUNT, 1, BW>), dim3(grid), dim3(64), 0, st, K, J);
    else if (!COUNT && !K.S.tex_on && BW == 8)
        hipLaunchKernelGGL((persistent_kernel<false, 2, 8, false>), dim3(grid), dim3(64), 0, st, K, J);
    else
        hipLaunchKernelGGL((persistent_kernel<COUNT, 2, BW>), dim3(grid), dim3(64), 0, st, K, J);
}

template <bool COUNT>
static void launch_persistent(int grid, hipStream_t st, KParams K, const JobSrc& J, const rt_ctx* c) {
    if (c->bw > 2) {
        K.S = c->S8;
        if (c->bw == 4)
            launch_wide<COUNT, 4>(grid, st, K, J, c->df_ok);
        else
            launch_wide<COUNT, 8>(grid, st, K, J, c->df_ok);
    } else {
        if (wpe() == 1)
            hipLaunchKernelGGL((persistent_kernel<COUNT, 1, 2>), dim3(grid), dim3(64), 0, st, K, J);
        else
            hipLaunchKernelGGL((persistent_kernel<COUNT, 2, 2>), dim3(grid), dim3(64), 0, st, K, J);
    }
}

static int persistent_grid(rt_ctx* c) {
    if (const char* g = std::getenv("RT_GRID")) {  // A/B override: blocks per CU
        int cus = 0;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
        return std::max(1, cus) * std::max(1, std::atoi(g));
    }
    if (c->persistent_blocks[wpe()] > 0) return c->persistent_blocks[wpe()];
    int cus = 0, per_cu = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    hipError_t e = hipErrorInvalidValue;
    // every BVH width compiles to the same LDS footprint and register cap per WPE
    if (wpe() == 1)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_df_kernel<false, 1, 8>, 64, 0);
    else if (wpe() == 3)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_df_kernel<false, 3, 8>, 64, 0);
    else if (wpe() == 4)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_df_kernel<false, 4, 8>, 64, 0);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_df_kernel<false, 2, 8>, 64, 0);
    if (e != hipSuccess || per_cu <= 0) per_cu = 8;
    c->persistent_blocks[wpe()] = std::max(1, cus) * per_cu;
    return c->persistent_blocks[wpe()];
}

// d_stats: 16 counters, then the 8 per-XCD job heads (128-B apart) of the dynamic-fetch kernel
#define RT_STATS_BYTES ((16 + 8 * 16) * sizeof(unsigned long long))

// per-XCD job ranges for the dynamic-fetch kernel (RT_XCD=0: one global job counter)
static bool use_xcd_queues() {
    const char* x = std::getenv("RT_XCD");
    return !(x && x[0] == '0');
}

static bool use_tile_kernel() {
    const char* k = std::getenv("RT_KERNEL");
    return k && std::strcmp(k, "tile") == 0;
}

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

extern "C" int rt_destroy(rt_ctx* c) {
    if (!c) return RT_OK;
    hipSetDevice(c->device);
    for (void* p : c->allocs) hipFree(p);
    if (c->d_stats) hipFree(c->d_stats);
    if (c->d_fb) hipFree(c->d_fb);
    if (c->d_img) hipFree(c->d_img);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->d_wf_st) hipFree(c->d_wf_st);
    if (c->d_wf_res) hipFree(c->d_wf_res);
    if (c->d_wf_frames) hipFree(c->d_wf_frames);
    if (c->d_wf_cnt) hipFree(c->d_wf_cnt);
    if (c->d_pre) hipFree(c->d_pre);
    if (c->d_wave_trace) hipFree(c->d_wave_trace);
    if (c->d_views) hipFree(c->d_views);
    if (c->d_sched) hipFree(c->d_sched);
    if (c->d_cost) hipFree(c->d_cost);
    if (c->h_wf_cnt) hipHostFree(c->h_wf_cnt);
    for (hipEvent_t e : c->wf_ev) hipEventDestroy(e);
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
        set_error(std::string("rt_device_count: ") + hipGetErrorString(e));
        return RT_ERR_NO_DEVICE;
    }
    return RT_OK;
}

extern "C" int rt_create(const rt_scene_desc* desc, int device, rt_ctx** out) {
    if (!desc || !out) {
        set_error("rt_create: null argument");
        return RT_ERR_INVALID;
    }
    *out = nullptr;
    int ndev = 0;
    const hipError_t de = hipGetDeviceCount(&ndev);
    if (de != hipSuccess || ndev == 0) {
        set_error(std::string("rt_create: no HIP device available (the MI355X path has no CPU fallback): ") +
                  (de != hipSuccess ? hipGetErrorString(de) : "0 devices"));
        return RT_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= ndev) {
        set_error("rt_create: device index out of range");
        return RT_ERR_INVALID;
    }
    const int ntri = desc->num_triangles;
    if (ntri < 0 || (ntri > 0 && (!desc->positions || !desc->normals || !desc->mesh_index)) ||
        desc->num_meshes < 0 || (ntri > 0 && !desc->materials) || desc->num_spheres < 0 ||
        (desc->num_spheres > 0 && !desc->spheres)) {
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

    // --- reference BVH (object order: triangles, then spheres) ---
    std::vector<float> sph4(desc->num_spheres * 4);
    for (int s = 0; s < desc->num_spheres; ++s) {
        for (int k = 0; k < 3; ++k) sph4[s * 4 + k] = desc->spheres[s].center[k];
        sph4[s * 4 + 3] = desc->spheres[s].radius;
    }
    RefBvh ref = build_ref_bvh(desc->positions, ntri, sph4.data(), desc->num_spheres, 4);
    c->ref_nodes = (int)ref.nodes.size();
    c->ref_levels = ref.max_level_achieved + 1;
    if (c->ref_nodes > RT_MAX_REF_NODES) {
        set_error("rt_create: reference BVH larger than 31 nodes");
        delete c;
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

    // --- BVH2 over triangles, boxes inflated by eps (see DESIGN.md "conservative traversal") ---
    float max_abs = 8.0f;
    for (size_t i = 0; i < (size_t)ntri * 9; ++i) max_abs = std::max(max_abs, std::fabs(desc->positions[i]));
    const float eps = std::ldexp(max_abs, -16);
    Bvh2 bvh = build_bvh2(desc->positions, ntri, eps, 4);
    c->bvh_depth = bvh.max_depth;
    if (bvh.max_depth + 2 >= RT_STACK_SIZE) {
        set_error("rt_create: BVH deeper than the traversal stack");
        delete c;
        return RT_ERR_INVALID;
    }
    c->nnodes = (int)bvh.nodes.size();
    c->nrec = ntri;

    // --- triangle records (64 B): v0|n.x, v1|n.y, v2|n.z, D|key_brute|key_bvh|ref_leaf ---
    auto make_records = [&](const std::vector<int>& order) {
        std::vector<float> rec((size_t)ntri * 16);
        for (int r = 0; r < ntri; ++r) {
            const int t = order[r];
            const float* p = desc->positions + (size_t)t * 9;
            const v3 v0{p[0], p[1], p[2]}, v1{p[3], p[4], p[5]}, v2{p[6], p[7], p[8]};
            // trianglePlane (src/ray_tracing.cpp:91-100)
            const v3 n = normalize(cross(v0 - v2, v1 - v2));
            const float D = dot(n, v0);
            float* o = rec.data() + (size_t)r * 16;
            o[0] = v0.x; o[1] = v0.y; o[2] = v0.z; o[3] = n.x;
            o[4] = v1.x; o[5] = v1.y; o[6] = v1.z; o[7] = n.y;
            o[8] = v2.x; o[9] = v2.y; o[10] = v2.z; o[11] = n.z;
            int ib[4] = {0, t, ref.tri_key[t], ref.tri_leaf[t]};
            std::memcpy(&o[12], &D, 4);
            std::memcpy(&o[13], &ib[1], 12);
        }
        return rec;
    };
    const std::vector<float> rec = make_records(bvh.order);
    c->bw = bvh_width_env();
    Bvh8 bvh8;
    try {
        if (c->bw > 2) bvh8 = build_bvh8(bvh, c->bw);
    } catch (const std::exception& ex) {
        set_error(std::string("rt_create: ") + ex.what());
        delete c;
        return RT_ERR_INVALID;
    }
    c->bvh8_depth = bvh8.max_depth;
    c->df_ok = bvh8.max_depth + 2 < RT_STACK8;  // the dynamic-fetch kernel's smaller LDS stack
    if (c->bw > 2 && (bvh8.max_depth + 2 >= RT_STACK_SIZE || (int)bvh8.order.size() != ntri)) {
        set_error("rt_create: BVH8 deeper than the traversal stack");
        delete c;
        return RT_ERR_INVALID;
    }
    const std::vector<float> rec8 = c->bw > 2 ? make_records(bvh8.order) : std::vector<float>();
    std::vector<float> nodes((size_t)bvh.nodes.size() * 16);
    for (size_t i = 0; i < bvh.nodes.size(); ++i) {
        const Bvh2Node& nd = bvh.nodes[i];
        float* o = nodes.data() + i * 16;
        o[0] = nd.lo0[0]; o[1] = nd.lo0[1]; o[2] = nd.lo0[2]; o[3] = nd.hi0[0];
        o[4] = nd.hi0[1]; o[5] = nd.hi0[2]; o[6] = nd.lo1[0]; o[7] = nd.lo1[1];
        o[8] = nd.lo1[2]; o[9] = nd.hi1[0]; o[10] = nd.hi1[1]; o[11] = nd.hi1[2];
        std::memcpy(&o[12], &nd.child[0], 4);
        std::memcpy(&o[13], &nd.child[1], 4);
        std::memcpy(&o[14], &nd.count[0], 4);
        std::memcpy(&o[15], &nd.count[1], 4);
    }

    std::vector<DMat> mats(desc->num_meshes);
    bool all_opaque = true;
    for (int m = 0; m < desc->num_meshes; ++m) {
        const rt_material& sm = desc->materials[m];
        for (int k = 0; k < 3; ++k) {
            mats[m].kd[k] = sm.kd[k];
            mats[m].ks[k] = sm.ks[k];
        }
        mats[m].shin = sm.shininess;
        mats[m].transp = sm.transparency;
        mats[m].gd = glossy_width(sm.shininess);
        if (sm.transparency != 1.0f) all_opaque = false;
        if (sm.transparency == 1.0f && (sm.ks[0] > 0 || sm.ks[1] > 0 || sm.ks[2] > 0) && sm.shininess != 0.0f)
            c->glossy_material = true;
    }
    std::vector<DSph> sph(desc->num_spheres);
    for (int s = 0; s < desc->num_spheres; ++s) {
        const rt_sphere& ss = desc->spheres[s];
        for (int k = 0; k < 3; ++k) {
            sph[s].c[k] = ss.center[k];
            sph[s].m.kd[k] = ss.material.kd[k];
            sph[s].m.ks[k] = ss.material.ks[k];
        }
        sph[s].r = ss.radius;
        sph[s].m.shin = ss.material.shininess;
        sph[s].m.transp = ss.material.transparency;
        sph[s].m.gd = glossy_width(ss.material.shininess);
        sph[s].key_bvh = ref.sph_key[s];
        sph[s].leaf = ref.sph_leaf[s];
        if (ss.material.transparency != 1.0f) all_opaque = false;
        const rt_material& sm = ss.material;
        if (sm.transparency == 1.0f && (sm.ks[0] > 0 || sm.ks[1] > 0 || sm.ks[2] > 0) && sm.shininess != 0.0f)
            c->glossy_material = true;
    }
    std::vector<DSpot> spots(desc->num_spot_lights);
    for (int i = 0; i < desc->num_spot_lights; ++i) {
        const rt_spot_light& L = desc->spot_lights[i];
        for (int k = 0; k < 3; ++k) {
            spots[i].pos[k] = L.position[k];
            spots[i].dir[k] = L.direction[k];
            spots[i].color[k] = L.color[k];
        }
        // std::cos(glm::radians(light.angle)) (src/shadow.cpp:235)
        spots[i].cos_angle = std::cos(L.angle * static_cast<float>(0.01745329251994329576923690768489));
    }

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

    DevScene& S = c->S;
    const float4* d_rec = nullptr;
    const float4* d_nodes = nullptr;
    UP(reinterpret_cast<const float4*>(rec.data()), (size_t)ntri * 4, d_rec);
    UP(reinterpret_cast<const float4*>(nodes.data()), bvh.nodes.size() * 4, d_nodes);
    S.tri = d_rec;
    S.nodes = d_nodes;
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
    UP(desc->point_lights, (size_t)desc->num_point_lights, S.pl);
    UP(desc->spherical_lights, (size_t)desc->num_spherical_lights, S.sl);
    UP(spots.data(), spots.size(), S.spot);
    UP(desc->plane_lights, (size_t)desc->num_plane_lights, S.plane);
    UP(texels.data(), texels.size(), S.tex);
    UP(tex_info.data(), tex_info.size(), S.tex_info);
    UP(mat_tex.data(), mat_tex.size(), S.mat_tex);
    S.ntex = desc->num_textures;
    S.ntri = ntri;
    S.nsph = desc->num_spheres;
    S.nref = (int)refn.size();
    S.npl = desc->num_point_lights;
    S.nsl = desc->num_spherical_lights;
    S.nspot = desc->num_spot_lights;
    S.nplane = desc->num_plane_lights;
    S.all_opaque = all_opaque ? 1 : 0;

    // 8-wide variant: same scene, records permuted into the BVH8 leaf order
    c->S8 = S;
    const float4* d_rec8 = nullptr;
    const float4* d_nodes8 = nullptr;
    UP(reinterpret_cast<const float4*>(rec8.data()), rec8.size() / 4, d_rec8);
    UP(reinterpret_cast<const float4*>(bvh8.nodes.data()), bvh8.nodes.size() / 4, d_nodes8);
    c->S8.tri = d_rec8;
    c->S8.nodes = d_nodes8;

    if (hipMalloc(&c->d_stats, RT_STATS_BYTES) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        set_error("rt_create: HIP allocation failed");
        rt_destroy(c);
        return RT_ERR_HIP;
    }
    *out = c;
    return RT_OK;
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
    if (p->glossy_ray_count != 1 && c->glossy_material && p->max_reflection_level > 0 && use_tile_kernel()) {
        set_error("glossy_ray_count > 1: the tile kernel has no glossy lobes (use the persistent kernels)");
        return RT_ERR_INVALID;
    }
    if (p->multiple_rays && !(p->sample_size == 4 || p->sample_size == 16 || p->sample_size == 64)) {
        set_error("sample_size must be 4, 16 or 64");
        return RT_ERR_INVALID;
    }
    if (p->texture_filtering < RT_TEX_NEAREST || p->texture_filtering > RT_TEX_TRILINEAR ||
        p->out_of_bounds_x < RT_OOB_BORDER || p->out_of_bounds_x > RT_OOB_REPEAT ||
        p->out_of_bounds_y < RT_OOB_BORDER || p->out_of_bounds_y > RT_OOB_REPEAT) {
        set_error("texture_filtering / out_of_bounds rule out of range");
        return RT_ERR_INVALID;
    }
    std::memset(&K, 0, sizeof(K));
    // per-render texture state (useTextures, textureFiltering, out-of-bounds rules, border colour)
    for (DevScene* sc : {&c->S, &c->S8}) {
        sc->tex_on = (p->use_textures && c->S.ntex > 0) ? 1 : 0;
        sc->tex_filter = p->texture_filtering;
        sc->tex_oob_x = p->out_of_bounds_x;
        sc->tex_oob_y = p->out_of_bounds_y;
        for (int k = 0; k < 3; ++k) sc->tex_border[k] = p->border_color[k];
    }
    K.S = c->S;
    K.max_level = p->max_reflection_level;
    K.glossy_n = p->glossy_ray_count;
    K.seed_lo = (uint32_t)(p->rng_seed & 0xFFFFFFFFull);
    K.seed_hi = (uint32_t)(p->rng_seed >> 32);
    K.plane_k = p->plane_light_1D_ray_count;
    K.use_bvh = p->use_bvh ? 1 : 0;
    K.refr = p->refraction_factor;
    // getSpherelights ring/spoke counts (src/shadow.cpp:190-195), host float math as the reference
    const int rc = p->sphere_light_ray_count;
    const int m = std::max(1, (int)(rc / std::round(std::sqrt(2 * 3.14159365358979f * rc))));
    const int n = (rc - 1) / m;
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
    K.refill = refill_threshold();
    {
        const char* cp = std::getenv("RT_COOP");  // drain-phase cooperative traversal (default on)
        K.coop = (cp && cp[0] == '0') ? 0 : ((cp && cp[0] == '2') ? 2 : 1);
        // a group of G lanes owns COOP_POOL * G / 64 pool slots: the depth-first reserve plus one
        // breadth step must fit; coop_max = the largest query count whose groups still do
        K.coop_reserve = 7 * (c->bvh8_depth + 1) + 8;
        K.coop_max = 0;
        for (int k = 1; k <= COOP_Q; ++k) {
            int G = 64;
            while (G > 1 && k * G > 64) G >>= 1;
            if (COOP_POOL * G / 64 >= K.coop_reserve + 8 * G) K.coop_max = k;
        }
        if (const char* cm = std::getenv("RT_COOP_MAX")) K.coop_max = std::min(K.coop_max, std::atoi(cm));
        if (K.coop_max <= 0) K.coop = 0;
    }
    K.leaf_batch = leaf_batch_threshold();
    return RT_OK;
}

static int ensure(rt_ctx* c, float** buf, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return RT_OK;
    if (*buf) hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc((void**)buf, bytes));
    *cap = bytes;
    return RT_OK;
}

// ---- wavefront path -------------------------------------------------------------------------
static bool use_wavefront() {
    const char* k = std::getenv("RT_KERNEL");
    return k && std::strcmp(k, "wavefront") == 0;
}

static int wf_env(const char* name, int dflt, int lo, int hi) {
    const char* v = std::getenv(name);
    const int x = v ? std::atoi(v) : dflt;
    return std::min(hi, std::max(lo, x));
}

static bool wf_debug() {
    const char* v = std::getenv("RT_WF_DEBUG");
    return v && v[0] == '1';
}

// trace-kernel waves per SIMD (register cap); RT_WF_WPE overrides for A/B runs
static int wf_wpe() {
    return wf_env("RT_WF_WPE", 4, 2, 4) >= 4 ? 4 : 2;  // 6 and 8 do not fit: the kernel needs ~105 VGPRs
}

template <bool COUNT, int BW>
static void wf_launch_trace(int grid, hipStream_t st, const KParams& K, const WfBufs& W) {
    switch (wf_wpe()) {
        case 4: hipLaunchKernelGGL((wf_trace_kernel<COUNT, 4, BW>), dim3(grid), dim3(64), 0, st, K, W); break;
        default: hipLaunchKernelGGL((wf_trace_kernel<COUNT, 2, BW>), dim3(grid), dim3(64), 0, st, K, W); break;
    }
}

template <bool COUNT>
static void wf_trace(const rt_ctx* c, int grid, hipStream_t st, KParams K, const WfBufs& W) {
    K.S = c->S8;
    if (c->bw == 4)
        wf_launch_trace<COUNT, 4>(grid, st, K, W);
    else
        wf_launch_trace<COUNT, 8>(grid, st, K, W);
}

static int wf_trace_grid(rt_ctx* c) {
    const int w = wf_wpe();
    const int slot = (w == 8) ? 4 : (w == 6) ? 3 : (w == 4) ? 2 : 1;
    if (c->wf_trace_blocks[slot] > 0) return c->wf_trace_blocks[slot];
    int cus = 0, per_cu = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    hipError_t e;
    switch (w) {
        case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wf_trace_kernel<false, 4, 8>, 64, 0); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wf_trace_kernel<false, 2, 8>, 64, 0); break;
    }
    if (e != hipSuccess || per_cu <= 0) per_cu = 4 * w;
    c->wf_trace_blocks[slot] = std::max(1, cus) * per_cu;
    return c->wf_trace_blocks[slot];
}

// One frame (or one rt_shade batch) as seed -> (trace -> shade)* iterations until every
// sub-queue is empty.  The lengths live on the device; the host checks their sum every `batch`
// iterations (kernels of an empty queue return at once).  trace_ms sums the trace launches.
static int launch_wavefront(rt_ctx* c, const KParams& K0, const JobSrc& J, hipStream_t st, int count_mode,
                            float* trace_ms, int* trace_launches) {
    KParams K = K0;
    K.S = c->S8;  // records are addressed in the wide BVH's leaf order by trace and shade alike
    const int njobs = J.njobs;
    if (njobs <= 0) return RT_OK;
    if (c->bw <= 2) {
        set_error("wavefront path needs the wide BVH (RT_BVH=4 or 8)");
        return RT_ERR_INVALID;
    }
    const int nchunks = (njobs + 63) / 64;
    const int seg = ((nchunks + WF_NQ - 1) / WF_NQ) * 64;
    const int cap = seg * WF_NQ;
    const int fpj = K.max_level + 1;  // frames 0..max_level (the deepest keeps its shading kd)
    int rc = ensure(c, &c->d_wf_st, &c->wf_st_bytes, (size_t)2 * WF_NFIELDS * cap * sizeof(float));
    if (rc != RT_OK) return rc;
    rc = ensure(c, &c->d_wf_res, &c->wf_res_bytes, (size_t)2 * cap * sizeof(float));
    if (rc != RT_OK) return rc;
    rc = ensure(c, &c->d_wf_frames, &c->wf_frames_bytes, (size_t)njobs * fpj * sizeof(Frame));
    if (rc != RT_OK) return rc;
    const size_t cnt_ints = (size_t)WF_C_KINDS * WF_NQ * WF_CSTRIDE + 64;
    if (!c->d_wf_cnt) HIP_TRY(hipMalloc((void**)&c->d_wf_cnt, cnt_ints * sizeof(int)));
    if (!c->h_wf_cnt) HIP_TRY(hipHostMalloc((void**)&c->h_wf_cnt, WF_NQ * sizeof(int)));
    int* cn[2] = {c->d_wf_cnt + (size_t)WF_C_N0 * WF_NQ * WF_CSTRIDE, c->d_wf_cnt + (size_t)WF_C_N1 * WF_NQ * WF_CSTRIDE};
    int* chead = c->d_wf_cnt + (size_t)WF_C_HEAD * WF_NQ * WF_CSTRIDE;
    int* crays = c->d_wf_cnt + (size_t)WF_C_RAYS * WF_NQ * WF_CSTRIDE;
    int* ctotal = c->d_wf_cnt + (size_t)WF_C_KINDS * WF_NQ * WF_CSTRIDE;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    // both grids are multiples of WF_NQ (block b serves sub-queue b % WF_NQ)
    int tgrid = std::max(WF_NQ, (wf_trace_grid(c) / WF_NQ) * WF_NQ);
    if (const char* g = std::getenv("RT_WF_TGRID")) tgrid = std::max(WF_NQ, (std::atoi(g) / WF_NQ) * WF_NQ);
    const int sgrid = std::max(WF_NQ, (std::max(1, cus) * 8 / WF_NQ) * WF_NQ);
    float* st0 = c->d_wf_st;
    float* st1 = c->d_wf_st + (size_t)WF_NFIELDS * cap;
    WfBufs W{};
    W.cap = cap;
    W.seg = seg;
    W.res_t = c->d_wf_res;
    W.res_rec = reinterpret_cast<int*>(c->d_wf_res + cap);
    W.frames = reinterpret_cast<Frame*>(c->d_wf_frames);
    W.fpj = fpj;
    W.refill = wf_env("RT_WF_REFILL", 8, 1, 64);
    W.leaf_batch = wf_env("RT_WF_LEAFBATCH", 0, 0, 64);
    W.head = chead;
    W.rays = crays;
    // seed -> queue 0; sub-queue q holds the jobs of chunks q, q + WF_NQ, ...
    HIP_TRY(hipMemsetAsync(c->d_wf_cnt, 0, cnt_ints * sizeof(int), st));
    hipLaunchKernelGGL(wf_seed_counts_kernel, dim3(1), dim3(WF_NQ), 0, st, cn[0], njobs);
    W.st_out = st0;
    const int seed_grid = (int)std::min<long long>(((long long)njobs + 63) / 64, (long long)std::max(1, cus) * 16);
    hipLaunchKernelGGL(wf_seed_kernel, dim3(seed_grid), dim3(64), 0, st, K, J, W);
    HIP_TRY(hipGetLastError());
    const int batch = wf_env("RT_WF_BATCH", 4, 1, 64);
    const bool timed = (trace_ms != nullptr);
    int cur = 0, launches = 0;
    std::vector<std::pair<int, int>> evs;  // event indices per trace launch
    for (int iter = 0;;) {
        for (int b = 0; b < batch; ++b, ++iter) {
            const int out = 1 - cur;
            W.st_in = cur ? st1 : st0;
            W.n_in = cn[cur];
            W.st_out = out ? st1 : st0;
            W.n_out = cn[out];
            hipLaunchKernelGGL(wf_reset_kernel, dim3(1), dim3(WF_NQ), 0, st, W.n_out, W.head);
            if (timed) {
                const size_t need = 2 * (evs.size() + 1);
                while (c->wf_ev.size() < need) {
                    hipEvent_t e;
                    HIP_TRY(hipEventCreate(&e));
                    c->wf_ev.push_back(e);
                }
                const int e0 = (int)(2 * evs.size());
                evs.push_back({e0, e0 + 1});
                HIP_TRY(hipEventRecord(c->wf_ev[e0], st));
            }
            if (count_mode)
                wf_trace<true>(c, tgrid, st, K, W);
            else
                wf_trace<false>(c, tgrid, st, K, W);
            if (timed) HIP_TRY(hipEventRecord(c->wf_ev[evs.back().second], st));
            ++launches;
            if (count_mode)
                hipLaunchKernelGGL(wf_shade_kernel<true>, dim3(sgrid), dim3(64), 0, st, K, J, W);
            else
                hipLaunchKernelGGL(wf_shade_kernel<false>, dim3(sgrid), dim3(64), 0, st, K, J, W);
            HIP_TRY(hipGetLastError());
            cur = out;
            if (wf_debug()) {  // RT_WF_DEBUG=1: per-iteration queue length and trace time (synchronous)
                hipLaunchKernelGGL(wf_total_kernel, dim3(1), dim3(WF_NQ), 0, st, W.n_in, ctotal);
                HIP_TRY(hipMemcpyAsync(c->h_wf_cnt, ctotal, sizeof(int), hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                float ms = 0.0f;
                if (timed) hipEventElapsedTime(&ms, c->wf_ev[evs.back().first], c->wf_ev[evs.back().second]);
                std::fprintf(stderr, "wf iter %d: queries %d trace %.3f ms\n", iter, c->h_wf_cnt[0], ms);
            }
        }
        hipLaunchKernelGGL(wf_total_kernel, dim3(1), dim3(WF_NQ), 0, st, cn[cur], ctotal);
        HIP_TRY(hipMemcpyAsync(c->h_wf_cnt, ctotal, sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (c->h_wf_cnt[0] == 0) break;
        if (iter > 1000000) {
            set_error("wavefront: queue did not drain");
            return RT_ERR_INVALID;
        }
    }
    hipLaunchKernelGGL(wf_finish_kernel, dim3(1), dim3(WF_NQ), 0, st, crays, c->d_stats);
    HIP_TRY(hipGetLastError());
    if (timed) {
        float tot = 0.0f;
        for (auto& e : evs) {
            float ms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, c->wf_ev[e.first], c->wf_ev[e.second]));
            tot += ms;
        }
        *trace_ms = tot;
    }
    if (trace_launches) *trace_launches = launches;
    return RT_OK;
}

// primary packet pass (rt_packet.hip) ahead of the megakernels; RT_PACKET=0 disables it
static bool use_packets(const rt_ctx* c, const KParams& K) {
    const char* v = std::getenv("RT_PACKET");
    if (!v || v[0] != '1') return false;  // opt-in: measured slower than the megakernels' own primaries
    // one camera ray per pixel; the shared stack holds at most (width-1) entries per level
    return c->bw > 2 && !K.aa && !K.multi && c->bvh8_depth * (c->bw - 1) + 2 <= PK_STACK;
}

static int launch_packets(rt_ctx* c, KParams& K, hipStream_t st, int count_mode, int njobs) {
    int rc = ensure(c, &c->d_pre, &c->pre_bytes, (size_t)2 * njobs * sizeof(float));
    if (rc != RT_OK) return rc;
    K.pre_t = c->d_pre;
    K.pre_rec = reinterpret_cast<const int*>(c->d_pre + njobs);
    KParams Kp = K;
    Kp.S = c->S8;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    const int ntiles = (njobs + 63) / 64;
    const int grid = std::min(ntiles, std::max(1, cus) * 16);
    float* pt = c->d_pre;
    int* pr = reinterpret_cast<int*>(c->d_pre + njobs);
    if (c->bw == 4) {
        if (count_mode)
            hipLaunchKernelGGL((primary_packet_kernel<true, 4>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, ntiles);
        else
            hipLaunchKernelGGL((primary_packet_kernel<false, 4>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, ntiles);
    } else {
        if (count_mode)
            hipLaunchKernelGGL((primary_packet_kernel<true, 8>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, ntiles);
        else
            hipLaunchKernelGGL((primary_packet_kernel<false, 8>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, ntiles);
    }
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

// Longest-first schedule: primary pass + hit-first job order (rt_schedule.hip).  RT_SCHED=0
// disables it; it needs one camera ray per pixel and the wide BVH.
static bool use_schedule(const rt_ctx* c, const KParams& K) {
    const char* v = std::getenv("RT_SCHED");
    if (!v || v[0] != '1') return false;  // opt-in: measured no gain
    return c->bw > 2 && !K.aa && !K.multi;
}

static int launch_schedule(rt_ctx* c, KParams& K, hipStream_t st, int count_mode, int njobs) {
    const int ntiles = (njobs + 63) / 64;
    int rc = ensure(c, &c->d_pre, &c->pre_bytes, (size_t)2 * njobs * sizeof(float));
    if (rc != RT_OK) return rc;
    rc = ensure(c, &c->d_sched, &c->sched_bytes, ((size_t)2 * (ntiles + 1) + njobs) * sizeof(int));
    if (rc != RT_OK) return rc;
    float* pt = c->d_pre;
    int* pr = reinterpret_cast<int*>(c->d_pre + njobs);
    int* hits = reinterpret_cast<int*>(c->d_sched);
    int* off = hits + (ntiles + 1);
    int* order = off + (ntiles + 1);
    KParams Kp = K;
    Kp.S = c->S8;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    const int grid = std::min(ntiles, std::max(1, cus) * 16);
    if (c->bw == 4) {
        if (count_mode)
            hipLaunchKernelGGL((primary_kernel<true, 4>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, hits, ntiles);
        else
            hipLaunchKernelGGL((primary_kernel<false, 4>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, hits, ntiles);
    } else {
        if (count_mode)
            hipLaunchKernelGGL((primary_kernel<true, 8>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, hits, ntiles);
        else
            hipLaunchKernelGGL((primary_kernel<false, 8>), dim3(grid), dim3(64), 0, st, Kp, pt, pr, hits, ntiles);
    }
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, st, hits, off, ntiles);
    hipLaunchKernelGGL(job_order_kernel, dim3(grid), dim3(64), 0, st, pr, off, order, Kp, ntiles);
    HIP_TRY(hipGetLastError());
    K.pre_t = pt;
    K.pre_rec = pr;
    K.job_order = order;
    return RT_OK;
}

// RT_SCHED=2: jobs ordered by the previous frame's per-pixel query counts (most expensive first).
static int launch_cost_schedule(rt_ctx* c, KParams& K, hipStream_t st, int njobs) {
    const int nblk = (njobs + CS_BLOCK - 1) / CS_BLOCK;
    const size_t bytes = ((size_t)2 * njobs + (size_t)CS_BUCKETS * nblk) * sizeof(int);
    const long long key = ((long long)K.W * 65536 + K.H) * 4096 + (long long)K.band_rank * 64 + K.band_count +
                          ((long long)K.band_rows << 40);
    const bool fresh = (c->cost_bytes < bytes) || (c->cost_key != key);
    int rc = ensure(c, &c->d_cost, &c->cost_bytes, bytes);
    if (rc != RT_OK) return rc;
    int* cost = reinterpret_cast<int*>(c->d_cost);
    int* hist = cost + njobs;
    int* order = hist + (size_t)CS_BUCKETS * nblk;
    if (fresh) {
        HIP_TRY(hipMemsetAsync(cost, 0, (size_t)njobs * sizeof(int), st));
        c->cost_key = key;
    } else {
        hipLaunchKernelGGL(cost_hist_kernel, dim3(nblk), dim3(CS_BLOCK), 0, st, cost, njobs, hist);
        hipLaunchKernelGGL(cost_scan_kernel, dim3(1), dim3(1024), 0, st, hist, CS_BUCKETS * nblk);
        hipLaunchKernelGGL(cost_scatter_kernel, dim3(nblk), dim3(CS_BLOCK), 0, st, cost, njobs, hist, order);
        HIP_TRY(hipGetLastError());
        K.job_order = order;
    }
    K.job_cost = cost;
    return RT_OK;
}

static int launch_render(rt_ctx* c, KParams& K, hipStream_t st, int count_mode, rt_stats* stats) {
    const int tiles_x = (K.W + 7) / 8;
    const int tiles_y = (K.band_rows + 7) / 8;
    const long long blocks = (long long)tiles_x * tiles_y * K.n_local_bands;
    float trace_ms = 0.0f;
    int trace_launches = 0;
    HIP_TRY(hipMemsetAsync(c->d_stats, 0, RT_STATS_BYTES, st));
    if (blocks > 0) {
        HIP_TRY(hipEventRecord(c->ev0, st));
        if (use_wavefront() && c->bw > 2) {
            JobSrc J{};
            J.mode = 0;
            J.njobs = (int)(blocks * 64);
            J.n_views = 1;
            J.view_jobs = J.njobs;
            int rc = launch_wavefront(c, K, J, st, count_mode, stats ? &trace_ms : nullptr,
                                      stats ? &trace_launches : nullptr);
            if (rc != RT_OK) return rc;
        } else if (use_tile_kernel()) {
            if (count_mode)
                hipLaunchKernelGGL(render_kernel<true>, dim3((unsigned)blocks), dim3(64), 0, st, K);
            else
                hipLaunchKernelGGL(render_kernel<false>, dim3((unsigned)blocks), dim3(64), 0, st, K);
        } else {
            JobSrc J{};
            J.mode = 0;
            J.n_views = std::max(1, K.n_views);
            J.view_jobs = (int)(blocks * 64);
            J.njobs = J.n_views * J.view_jobs;
            K.view_jobs = J.view_jobs;
            J.counter = reinterpret_cast<int*>(c->d_stats + 7);
            J.xq = use_xcd_queues() ? reinterpret_cast<int*>(c->d_stats + 16) : nullptr;
            if (use_packets(c, K)) {
                const int rc = launch_packets(c, K, st, count_mode, J.njobs);
                if (rc != RT_OK) return rc;
            } else if (use_schedule(c, K)) {
                const int rc = launch_schedule(c, K, st, count_mode, J.njobs);
                if (rc != RT_OK) return rc;
            }
            const char* cs = std::getenv("RT_SCHED");
            if (cs && cs[0] == '2' && !K.job_order) {
                const int rc = launch_cost_schedule(c, K, st, J.njobs);
                if (rc != RT_OK) return rc;
            }
            const int grid = (int)std::min<long long>(blocks, persistent_grid(c));
            const char* wt = std::getenv("RT_WAVE_TRACE");
            if (wt && wt[0] == '1') {
                const int rc = ensure(c, &c->d_wave_trace, &c->wave_trace_bytes, (size_t)grid * 8 * 8);
                if (rc != RT_OK) return rc;
                K.wave_trace = reinterpret_cast<unsigned long long*>(c->d_wave_trace);
                c->wave_trace_n = grid;
            }
            if (count_mode)
                launch_persistent<true>(grid, st, K, J, c);
            else
                launch_persistent<false>(grid, st, K, J, c);
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev1, st));
    }
    if (stats) {
        unsigned long long h[8] = {0};
        HIP_TRY(hipMemcpyAsync(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        stats->rays = h[0];
        stats->node_visits = h[1];
        stats->tri_tests = h[2];
        stats->hits = h[3];
        float ms = 0.0f;
        if (blocks > 0) HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
        stats->kernel_ms = ms;
        stats->node_bytes = (use_tile_kernel() || c->bw == 2) ? 64u : 128u;
        stats->trace_ms = trace_ms;
        stats->trace_launches = (uint32_t)trace_launches;
    }
    return RT_OK;
}

static int g_count_mode = 0;  // set by rt_set_counting (counting build of the same kernel)

extern "C" int rt_set_counting(int on) {
    g_count_mode = on ? 1 : 0;
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
    K.out = d_out;
    // Few shadow samples per shading point (point/spot lights: long mirror and camera queries):
    // full-wave refill + lane groups for the stragglers (C3 2.37 -> 2.18 ms).  Sample-heavy
    // lights (sphere/plane lights, many short shadow queries) keep the 24-lane refill (C4 43.6 ms
    // against 48.5 ms with it).
    if (!std::getenv("RT_REFILL") && !std::getenv("RT_COOP") && K.coop == 1 &&
        K.S.nsl * K.sl_count + K.S.nplane * K.plane_k * K.plane_k <= 4) {
        K.refill = 64;
        K.coop = 2;
    }
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
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
    if (use_wavefront() || use_tile_kernel() || (std::getenv("RT_PACKET") && std::getenv("RT_PACKET")[0] == '1') || std::getenv("RT_SCHED")) {
        set_error("rt_render_views_device: view batches run on the persistent kernels only");
        return RT_ERR_INVALID;
    }
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
    // dynamic-fetch refill threshold: in a batch only the last frame drains, and advancing all 64
    // lanes at once amortises the state machine's spills best (C3, 8 views: 24 -> 64 lanes = 1.59 ->
    // 1.37 ms/frame); the last queries a full-wave refill waits for go to lane groups (coop 2:
    // C3, 16 views, 1.29 -> 1.17 ms/frame; C4 neutral)
    if (!std::getenv("RT_REFILL")) K.refill = 64;
    if (!std::getenv("RT_COOP") && K.coop == 1) K.coop = 2;
    K.n_views = n_views;
    K.view_rows = K.n_local_bands * band_rows;
    std::vector<float> v((size_t)n_views * 12, 0.0f);
    for (int i = 0; i < n_views; ++i) {
        float* o = v.data() + 12 * i;
        for (int k = 0; k < 3; ++k) o[k] = cams[i].position[k];
        for (int k = 0; k < 4; ++k) o[3 + k] = cams[i].quat[k];
        o[7] = cams[i].half_height;
        o[8] = cams[i].half_width;
    }
    rc = ensure(c, &c->d_views, &c->views_bytes, v.size() * sizeof(float));
    if (rc != RT_OK) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIP_TRY(hipMemcpyAsync(c->d_views, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice, st));
    K.views = reinterpret_cast<const float*>(c->d_views);
    return launch_render(c, K, st, g_count_mode, stats);
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

extern "C" int rt_render(rt_ctx* c, const rt_camera* cam, const rt_params* p, int W, int H, float* rgb_out,
                         rt_stats* stats) {
    if (!c || !cam || !p || !rgb_out || W <= 0 || H <= 0) {
        set_error("rt_render: invalid argument");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    const int band_rows = 8;
    const int nbands = (H + band_rows - 1) / band_rows;
    const size_t fb = (size_t)nbands * band_rows * W * 3 * sizeof(float);
    int rc = ensure(c, &c->d_fb, &c->fb_bytes, fb);
    if (rc != RT_OK) return rc;
    rc = ensure(c, &c->d_img, &c->img_bytes, (size_t)W * H * 3 * sizeof(float));
    if (rc != RT_OK) return rc;
    rt_stats local{};
    rc = rt_render_device(c, cam, p, W, H, band_rows, 0, 1, c->d_fb, c->stream, &local);
    if (rc != RT_OK) return rc;
    rc = rt_unpermute_bands_device(W, H, band_rows, 1, c->d_fb, c->d_img, c->stream);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(rgb_out, c->d_img, (size_t)W * H * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (stats) *stats = local;
    return RT_OK;
}

extern "C" int rt_render_views(rt_ctx* c, const rt_camera* cams, int n_views, const rt_params* p, int W, int H,
                               float* rgb_out, rt_stats* stats) {
    if (!c || !cams || n_views <= 0 || !p || !rgb_out || W <= 0 || H <= 0) {
        set_error("rt_render_views: invalid argument");
        return RT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    const int band_rows = 8;
    const int nbands = (H + band_rows - 1) / band_rows;
    const size_t view_fb = (size_t)nbands * band_rows * W * 3;
    const size_t view_img = (size_t)W * H * 3;
    int rc = ensure(c, &c->d_fb, &c->fb_bytes, view_fb * n_views * sizeof(float));
    if (rc != RT_OK) return rc;
    rc = ensure(c, &c->d_img, &c->img_bytes, view_img * n_views * sizeof(float));
    if (rc != RT_OK) return rc;
    rt_stats local{};
    rc = rt_render_views_device(c, cams, n_views, p, W, H, band_rows, 0, 1, c->d_fb, c->stream, &local);
    if (rc != RT_OK) return rc;
    for (int v = 0; v < n_views; ++v) {
        rc = rt_unpermute_bands_device(W, H, band_rows, 1, c->d_fb + v * view_fb, c->d_img + v * view_img, c->stream);
        if (rc != RT_OK) return rc;
    }
    HIP_TRY(hipMemcpyAsync(rgb_out, c->d_img, view_img * n_views * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (stats) *stats = local;
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
    KParams K;
    std::memset(&K, 0, sizeof(K));
    K.S = c->S;
    hipMemcpy(d_r, rays, sizeof(rt_ray) * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(intersect_kernel, dim3((n + 63) / 64), dim3(64), 0, c->stream, K, d_r, n, use_bvh ? 1 : 0, d_h);
    hipError_t e = hipGetLastError();
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
    rt_ray* d_r = nullptr;
    float* d_c = nullptr;
    unsigned long long* d_n = nullptr;
    HIP_TRY(hipMalloc(&d_r, sizeof(rt_ray) * n));
    HIP_TRY(hipMalloc(&d_c, sizeof(float) * 3 * n));
    HIP_TRY(hipMalloc(&d_n, sizeof(unsigned long long) * n));
    hipMemcpy(d_r, rays, sizeof(rt_ray) * n, hipMemcpyHostToDevice);
    if (use_wavefront() && c->bw > 2) {
        JobSrc J{};
        J.mode = 1;
        J.njobs = n;
        J.n_views = 1;
        J.view_jobs = n;
        J.rays = d_r;
        J.rgb = d_c;
        J.ray_counts = d_n;
        hipMemsetAsync(c->d_stats, 0, RT_STATS_BYTES, c->stream);
        const int rc = launch_wavefront(c, K, J, c->stream, 0, nullptr, nullptr);
        if (rc != RT_OK) {
            hipFree(d_r);
            hipFree(d_c);
            hipFree(d_n);
            return rc;
        }
    } else if (use_tile_kernel()) {
        hipLaunchKernelGGL(shade_kernel, dim3((n + 63) / 64), dim3(64), 0, c->stream, K, d_r, n, d_c, d_n);
    } else {
        JobSrc J{};
        J.mode = 1;
        J.njobs = n;
        J.rays = d_r;
        J.rgb = d_c;
        J.ray_counts = d_n;
        J.n_views = 1;
        J.view_jobs = n;
        J.counter = reinterpret_cast<int*>(c->d_stats + 7);
        J.xq = use_xcd_queues() ? reinterpret_cast<int*>(c->d_stats + 16) : nullptr;
        hipMemsetAsync(c->d_stats, 0, RT_STATS_BYTES, c->stream);
        const int grid = std::min((n + 63) / 64, persistent_grid(c));
        launch_persistent<false>(grid, c->stream, K, J, c);
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(rgb, d_c, sizeof(float) * 3 * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && ray_counts) e = hipMemcpy(ray_counts, d_n, sizeof(uint64_t) * n, hipMemcpyDeviceToHost);
    hipFree(d_r);
    hipFree(d_c);
    hipFree(d_n);
    if (e != hipSuccess) {
        set_error(std::string("rt_shade: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    return RT_OK;
}

// Debug counters of the last counting launch: [8..13] per-query node-visit histogram
// (<16, <64, <256, <1024, <4096, >=4096), [14] max node visits, [15] max triangle records.
extern "C" int rt_debug_counters(rt_ctx* c, uint64_t* out, int n) {
    if (!c || !out || n <= 0) return RT_ERR_INVALID;
    unsigned long long h[16] = {0};
    HIP_TRY(hipMemcpy(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < n && i < 16; ++i) out[i] = h[i];
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
