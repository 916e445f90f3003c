// rt_runtime.hip -- device context behind the C-ABI: scene upload (once), launches, stats.
// Replaces BoundingVolumeHierarchy's constructor + renderRayTracing's pixel loop
// (reference src/bounding_volume_hierarchy.cpp:5-9, src/main.cpp:340-400).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "bvh_build.h"
#include "rt_internal.h"
#include "rt_kernels.hip"
#include "rt_megakernel.hip"

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
};

// waves per SIMD the persistent kernel is compiled for (register cap); RT_WPE overrides for A/B runs
static int wpe() {
    const char* w = std::getenv("RT_WPE");
    const int v = w ? std::atoi(w) : 2;
    return (v == 1) ? 1 : 2;
}

// BVH the persistent kernel walks, read once at rt_create: 8 (quantised 8-wide, default),
// 4 (same node format, 4 slots) or 2 (binary, full-precision boxes); RT_BVH selects for A/B runs
static int bvh_width_env() {
    const char* b = std::getenv("RT_BVH");
    const int v = b ? std::atoi(b) : 8;
    return (v == 2 || v == 4) ? v : 8;
}

template <bool COUNT, int BW>
static void launch_wide(int grid, hipStream_t st, const KParams& K, const JobSrc& J) {
    if (wpe() == 1)
        hipLaunchKernelGGL((persistent_kernel<COUNT, 1, BW>), dim3(grid), dim3(64), 0, st, K, J);
    else
        hipLaunchKernelGGL((persistent_kernel<COUNT, 2, BW>), dim3(grid), dim3(64), 0, st, K, J);
}

template <bool COUNT>
static void launch_persistent(int grid, hipStream_t st, KParams K, const JobSrc& J, const rt_ctx* c) {
    if (c->bw > 2) {
        K.S = c->S8;
        if (c->bw == 4)
            launch_wide<COUNT, 4>(grid, st, K, J);
        else
            launch_wide<COUNT, 8>(grid, st, K, J);
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
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_kernel<false, 1, 8>, 64, 0);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_kernel<false, 2, 8>, 64, 0);
    if (e != hipSuccess || per_cu <= 0) per_cu = 8;
    c->persistent_blocks[wpe()] = std::max(1, cus) * per_cu;
    return c->persistent_blocks[wpe()];
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
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return RT_OK;
}

extern "C" int rt_create(const rt_scene_desc* desc, int device, rt_ctx** out) {
    if (!desc || !out) {
        set_error("rt_create: null argument");
        return RT_ERR_INVALID;
    }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("rt_create: no HIP device available (the MI355X path has no CPU fallback)");
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

    if (hipMalloc(&c->d_stats, 16 * sizeof(unsigned long long)) != hipSuccess ||
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
    if (p->glossy_ray_count != 1 && c->glossy_material && p->max_reflection_level > 0) {
        set_error("glossy_ray_count > 1 with a glossy material is not supported yet (the reference uses rand())");
        return RT_ERR_INVALID;
    }
    if (p->multiple_rays && !(p->sample_size == 4 || p->sample_size == 16 || p->sample_size == 64)) {
        set_error("sample_size must be 4, 16 or 64");
        return RT_ERR_INVALID;
    }
    std::memset(&K, 0, sizeof(K));
    K.S = c->S;
    K.max_level = p->max_reflection_level;
    K.glossy_n = p->glossy_ray_count;
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

static int launch_render(rt_ctx* c, KParams& K, hipStream_t st, int count_mode, rt_stats* stats) {
    const int tiles_x = (K.W + 7) / 8;
    const int tiles_y = (K.band_rows + 7) / 8;
    const long long blocks = (long long)tiles_x * tiles_y * K.n_local_bands;
    HIP_TRY(hipMemsetAsync(c->d_stats, 0, 16 * sizeof(unsigned long long), st));
    if (blocks > 0) {
        HIP_TRY(hipEventRecord(c->ev0, st));
        if (use_tile_kernel()) {
            if (count_mode)
                hipLaunchKernelGGL(render_kernel<true>, dim3((unsigned)blocks), dim3(64), 0, st, K);
            else
                hipLaunchKernelGGL(render_kernel<false>, dim3((unsigned)blocks), dim3(64), 0, st, K);
        } else {
            JobSrc J{};
            J.mode = 0;
            J.njobs = (int)(blocks * 64);
            J.counter = reinterpret_cast<int*>(c->d_stats + 7);
            const int grid = (int)std::min<long long>(blocks, persistent_grid(c));
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
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
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
    if (use_tile_kernel()) {
        hipLaunchKernelGGL(shade_kernel, dim3((n + 63) / 64), dim3(64), 0, c->stream, K, d_r, n, d_c, d_n);
    } else {
        JobSrc J{};
        J.mode = 1;
        J.njobs = n;
        J.rays = d_r;
        J.rgb = d_c;
        J.ray_counts = d_n;
        J.counter = reinterpret_cast<int*>(c->d_stats + 7);
        hipMemsetAsync(c->d_stats, 0, 16 * sizeof(unsigned long long), c->stream);
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
