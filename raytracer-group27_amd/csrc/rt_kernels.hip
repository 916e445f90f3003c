// rt_kernels.hip -- device arithmetic shared by the MI355X (gfx950) render kernels.
//
// The reference's per-pixel hot path, restated exactly where it decides geometry:
//   renderRayTracing (src/main.cpp:340-400) -> Trackball::generateRay (framework/src/trackball.cpp:87-98)
//   -> getFinalColor (src/main.cpp:129-301) -> BoundingVolumeHierarchy::intersect (src/bounding_volume_hierarchy.cpp:49-78)
//   -> light gathering + cansee (src/shadow.cpp:32-321) -> calcColor (src/main.cpp:112-121)
// Every candidate is accepted or rejected with the reference's own arithmetic (plane/edge test,
// src/ray_tracing.cpp:42-128; sphere quadratic in double, :182-209), and ties in t go to the first
// object in the reference's visit order, so the hit is the one the reference's brute-force loop
// (useBVH=false) or its depth-4 BVH walk (useBVH=true, every shadow ray) returns.  useBVH=true
// additionally requires every box on the candidate's reference leaf path to pass the reference slab
// test (src/ray_tracing.cpp:213-264), evaluated lazily and cached per ray.  The schedule (persistent
// ray-state-machine kernels, quantised BVH8) lives in rt_megakernel.hip.
//
// Compiled with -ffp-contract=off (no FMA contraction), IEEE div/sqrt, f32 denormals kept.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

#include "rt_math.h"
#include "rt_internal.h"

namespace rt {

struct DMat {
    float kd[3];
    float ks[3];
    float shin;
    float transp;
    float gd;  // glossy lobe half-width d = pow(0.5f, -1/s) * sqrt(1 - pow(0.5, 2/s)) (src/main.cpp:224), host-evaluated
};
struct DSph {
    float c[3];
    float r;
    DMat m;
    int key_bvh;
    int leaf;
    int pad_[1];
};
struct DRefNode {
    float lo[3];
    float hi[3];
};
struct DSpot {
    float pos[3];
    float dir[3];
    float cos_angle;  // std::cos(glm::radians(angle)), host constant
    float color[3];
};

struct DevScene {
    const float4* __restrict__ tri;      // [nrec][4] triangle records, BVH8 leaf order
    const float4* __restrict__ nodes;    // [nnodes][8] quantised BVH8 nodes (bvh_build.h)
    const float* __restrict__ nrm;       // [ntri][9] scene order (shading normals)
    const float* __restrict__ uv;        // [ntri][6] scene order
    const int* __restrict__ mesh;        // [ntri] scene order
    const DMat* __restrict__ mats;       // [nmesh]
    const DSph* __restrict__ sph;        // [nsph]
    const DRefNode* __restrict__ refn;   // [nref]
    const int* __restrict__ leaf_path;   // [32][8]: count, node ids root..leaf
    const rt_point_light* __restrict__ pl;
    const rt_spherical_light* __restrict__ sl;
    const DSpot* __restrict__ spot;
    const rt_plane_light* __restrict__ plane;
    int ntri, nsph, nref;
    int nnodes;      // BVH8 nodes (the checked builds' bounds)
    int npl, nsl, nspot, nplane;
    int all_opaque;  // every mesh and sphere material has transparency == 1.0f
    // kd textures (Image, src/image.cpp): texels (r, g, b) of every level of every texture;
    // per texture (level-0 texel offset, width, height, mip levels or 0); per mesh texture or -1
    const float* __restrict__ tex;
    const int4* __restrict__ tex_info;
    const int* __restrict__ mat_tex;
    int ntex;
    // per render (rt_params): useTextures, textureFiltering, outOfBoundsRuleX/Y, textureBorderColor
    int tex_on, tex_filter, tex_oob_x, tex_oob_y;
    float tex_border[3];
};

struct KParams {
    DevScene S;
    int max_level;
    int glossy_n;
    int plane_k;
    int use_bvh;
    float refr;
    int sl_m, sl_n, sl_count;
    float sl_sin, sl_1mcos;
    // camera
    float cam[3];
    float q[4];
    float hh, hw;
    int W, H;
    int aa, multi, sample_size, ms_moves;
    float ms_offx, ms_offy;
    float aa_offx, aa_offy;
    // bands
    int band_rows, band_rank, band_count, n_local_bands;
    float* out;
    int out_image;              // 0: band-dense rows (rt_render_device); 1: Screen::m_textureData order, view v's
                                // image at out + v * W * H * 3 (setPixel's row H-1-y, src/screen.cpp:32-38)
    unsigned long long* stats;  // rays, node visits, tri tests, hits, ..., UB-regime hits
    int refill;                 // dynamic-fetch kernel: waiting lanes that end a traversal phase
    int shade_level;            // rt_shade: recursion level of the explicit rays (getFinalColor's `level`)
    int fan;                    // dynamic-fetch kernel: bit 0 spherical-, bit 1 plane-light samples as wave-shared fans
    int interleave;             // job -> pixel: 0 a wave's 64 jobs are one 8x8 tile; k > 0 they spread over 2^k tiles
    int interleave_view;        // ... in the views from this one on (a batch's last views: its drain)
    int centre_first;           // job -> tile: the upper half's per-XCD tile ranges walked bottom-up (single frames)
    int prio_iters;             // opaque kernel: a traversal phase raises its wave's issue priority after this many
                                // iterations (0: never)
    int fan_cap;                // ... a wave with this many pixels waiting on fans takes no new pixels
    int dual;                   // dynamic-fetch kernel: a lane testing a leaf's records also visits its next node
    uint32_t seed_lo, seed_hi;  // glossy sampling: Philox-4x32-10 key (rt_params.rng_seed)
    unsigned long long* wave_trace;  // developer wave trace (rt_ctx_set_option RT_OPT_WAVE_TRACE), or null
    unsigned long long* job_trace;   // ... and per job: start, end (100 MHz clock), queries
    unsigned long long* phase_trace; // ... and per wave RT_PHASE_EV traversal phases (RT_OPT_WAVE_TRACE 2), or null
    int coop;                        // dynamic-fetch kernel: lane-group traversal of the drain's queries
    int coop_max;                    // ... when at most this many queries are left in the wave
    int coop_reserve;                // ... free pool slots kept for depth-first steps
    // view batch (rt_render_views_device): n_views frames of the same scene in one launch, view v's
    // camera at views[12 v] (cam xyz, quat wxyz, hh, hw), its rows at out + v * view_rows * W * 3
    int n_views, view_jobs, view_rows;
    const float* views;
    // recursion-tree kernel: the lanes' pending refracted rays, frame f of lane slot s (= block * 64 + lane)
    // at frames + (f * frame_slots + s) * 3 (3 float4: origin + child level, direction, weight)
    float4* frames;
    int frame_slots;
    // plane lights (fan renders): per light RT_PLANE_TAB float4 -- getPlaneLights' grid points px for k = 2..8
    // (plane_tab_at), then normalize(cross(width, height)); built on the host with the loop's own additions
    const float4* plane_tab;
};

// the plane-light table: grid points of every k in 2..8 (sum of k^2 = 203), then the light's normal
#define RT_PLANE_TAB 204
#define RT_PLANE_TAB_KMAX 8
__host__ __device__ __forceinline__ int plane_tab_at(int k, int s) { return (k - 1) * k * (2 * k - 1) / 6 - 1 + s; }

// Philox-4x32-10 (Salmon et al., SC'11; the Random123 constants): the counter-based stream that
// replaces the reference's rand() for glossy lobes.  Counter = (draw, pixel, sample, 0).
__host__ __device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
    }
}

// uniform float in [0, 1) from the top 24 bits (stands in for the reference's rand() / (float)RAND_MAX)
__host__ __device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-8f; }

struct Cnt {
    uint32_t rays, nodes, tris, hits;
    uint32_t ub;                   // shaded hits where barycentricCoordinates returns false (counting builds)
    uint32_t wnodes, wtris, wadv;  // wave-level steps (counted by the first active lane): SIMD efficiency
    unsigned long long cyc_a, cyc_b;  // shader clocks per wave in the state machine / in traversal (df kernel)
    unsigned long long cyc_c, cyc_d;  // ... of cyc_a: advancing finished queries / fetching jobs
    uint32_t hist[3];  // df kernel traversal iterations by tracing lanes 1-16 / 17-32 / 33-64 (leader)
    // node visits that re-test a node popped from the stack (slot mask < 0xFF), the popped groups' slot
    // counts and how many of those slots still hit (counting builds: the cost of the re-visit scheme)
    uint32_t rv, rvk, rvj;
    // the ray mix (counting builds): cansee segments and light samples, camera queries that hit nothing
    uint32_t shad, cmiss;
    // the tree kernel's phase A in parts (counting builds, wave leader): finished samples and segments, owners
    // resuming and advancing, the fan hand-out
    unsigned long long cyc_e, cyc_f, cyc_g;
    // node visits and records of the camera queries that hit nothing (the opaque kernel's counting build)
    uint32_t cmn, cmr;
};

// reference-box tests of candidate culling (ref_slab): lane evaluations, the wave's executions (the most any lane
// did per record step) and the last record step's count on this lane (the opaque kernel's counting build)
// ... and the traversal loop's lane iterations: tracing lanes, lanes with a node visit and a record test, lanes held
// to a record test with a node to visit (their last visit's leaf hits still pending)
struct SlabCnt {
    uint32_t slab, wslab, step;
    uint32_t iters, both, blocked;
};

// true on the lowest active lane of the wave (counting builds: one count per wave instruction stream)
__device__ __forceinline__ bool wave_leader() {
    return (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1;
}

// ------------------------------------------------------------------------------------------
// Reference slab test (src/ray_tracing.cpp:213-264), dir = normalize(ray.direction).
// ------------------------------------------------------------------------------------------
// RT_SLAB_FILTER (A/B build option, default 0): the six IEEE divisions are first bounded by reciprocal products,
// and the exact quotients are formed only for a ray whose answer the bounds leave open (ref_slab_bounds), in the
// opaque and tree kernels' record tests (template FILTER).  Measured neutral (C3 16-view batch 0.445 / 0.443 vs
// 0.447 / 0.444 ms/frame, C5 frame 152.4 vs 152.7 ms, profiles/r04/ab_r04s_slab.log: the culling's box tests are
// 0.10 wave executions per ray, and the filter's code adds 10 spilled VGPRs to the 4-wave opaque build), so the
// shipped kernels keep the plain test; rt_debug_slab_check checks the bounds either way.
#ifndef RT_SLAB_FILTER
#define RT_SLAB_FILTER 0
#endif

// The slab test's answer from bounds on its quotients: 0 miss, 1 hit, 2 open (the exact test decides).
// In range (every |d| in [2^-40, 2^40], every |a| zero or in [2^-40, 2^40]; checked on the magnitude bits, so
// NaN and infinity fall outside) every quotient is a normal float or an exact zero.  q' = a * rcp(d)
// (v_rcp_f32: 1 ulp; the product: 1/2 ulp) lies within 2^-21 |q'| of the correctly rounded a / d, so
// [q' - 2^-18 |q'|, q' + 2^-18 |q'|] holds the reference's quotient (zero numerators give exact zeros).
// Per axis the reference's min / max of the two quotients is the min / max of the two products (both
// roundings are monotonic, and the products share the reciprocal; equal products bound both quotients).
// tin > tout is decided when the bounds of max(tin_k) and min(tout_k) do not overlap, and tout < 0 by the
// signs of the tout products (no quotient underflows to zero in range).
__device__ __forceinline__ int ref_slab_bounds(const DRefNode& b, v3 o, v3 nd) {
    const float a0x = b.lo[0] - o.x, a1x = b.hi[0] - o.x, a0y = b.lo[1] - o.y, a1y = b.hi[1] - o.y,
                a0z = b.lo[2] - o.z, a1z = b.hi[2] - o.z;
    auto mag = [](float x) { return __float_as_uint(x) & 0x7FFFFFFFu; };
    constexpr uint32_t LO = 0x2B800000u, HI = 0x53800000u;  // 2^-40, 2^40
    const uint32_t dmax = max(max(mag(nd.x), mag(nd.y)), mag(nd.z)), dmin = min(min(mag(nd.x), mag(nd.y)), mag(nd.z));
    const uint32_t amax = max(max(max(mag(a0x), mag(a1x)), max(mag(a0y), mag(a1y))), max(mag(a0z), mag(a1z)));
    // smallest nonzero magnitude: a zero maps to 0xFFFFFFFF
    const uint32_t anz = min(min(min(mag(a0x) - 1u, mag(a1x) - 1u), min(mag(a0y) - 1u, mag(a1y) - 1u)),
                             min(mag(a0z) - 1u, mag(a1z) - 1u));
    if (!(dmax <= HI && dmin >= LO && amax <= HI && anz >= LO - 1u)) return 2;
    const float rx = __builtin_amdgcn_rcpf(nd.x), ry = __builtin_amdgcn_rcpf(nd.y), rz = __builtin_amdgcn_rcpf(nd.z);
    const float p0x = a0x * rx, p1x = a1x * rx, p0y = a0y * ry, p1y = a1y * ry, p0z = a0z * rz, p1z = a1z * rz;
    const float ix = fminf(p0x, p1x), iy = fminf(p0y, p1y), iz = fminf(p0z, p1z);
    const float ox = fmaxf(p0x, p1x), oy = fmaxf(p0y, p1y), oz = fmaxf(p0z, p1z);
    constexpr float E = 0x1p-18f;
    const float eix = fabsf(ix) * E, eiy = fabsf(iy) * E, eiz = fabsf(iz) * E;
    const float eox = fabsf(ox) * E, eoy = fabsf(oy) * E, eoz = fabsf(oz) * E;
    const float in_lo = fmaxf(fmaxf(ix - eix, iy - eiy), iz - eiz), in_hi = fmaxf(fmaxf(ix + eix, iy + eiy), iz + eiz);
    const float out_lo = fminf(fminf(ox - eox, oy - eoy), oz - eoz), out_hi = fminf(fminf(ox + eox, oy + eoy), oz + eoz);
    if (in_lo > out_hi) return 0;      // tin > tout
    if (!(in_hi <= out_lo)) return 2;  // open
    return fminf(fminf(ox, oy), oz) < 0.0f ? 0 : 1;  // tin <= tout: a hit unless tout < 0
}

// the slab test's quotient part (src/ray_tracing.cpp:220-260) with the reference's IEEE divisions
__device__ __forceinline__ bool ref_slab_div(const DRefNode& b, v3 o, v3 nd) {
    const float txmin = (b.lo[0] - o.x) / nd.x;
    const float txmax = (b.hi[0] - o.x) / nd.x;
    const float tymin = (b.lo[1] - o.y) / nd.y;
    const float tymax = (b.hi[1] - o.y) / nd.y;
    const float tzmin = (b.lo[2] - o.z) / nd.z;
    const float tzmax = (b.hi[2] - o.z) / nd.z;
    const float tinx = (txmax < txmin) ? txmax : txmin;  // std::min
    const float tiny = (tymax < tymin) ? tymax : tymin;
    const float tinz = (tzmax < tzmin) ? tzmax : tzmin;
    const float toutx = (txmin < txmax) ? txmax : txmin;  // std::max
    const float touty = (tymin < tymax) ? tymax : tymin;
    const float toutz = (tzmin < tzmax) ? tzmax : tzmin;
    const float tin = gmax(gmax(tinx, tiny), tinz);
    const float tout = gmin(gmin(toutx, touty), toutz);
    return !(tin > tout || tout < 0.0f);
}

template <bool FILTER = false>
__device__ __forceinline__ bool ref_slab(const DRefNode& b, v3 o, v3 nd) {
    if (b.lo[0] == FLT_MAX && b.lo[1] == FLT_MAX && b.lo[2] == FLT_MAX && b.hi[0] == -FLT_MAX &&
        b.hi[1] == -FLT_MAX && b.hi[2] == -FLT_MAX)
        return false;
    if (o.x > b.lo[0] && o.y > b.lo[1] && o.z > b.lo[2] && o.x < b.hi[0] && o.y < b.hi[1] && o.z < b.hi[2])
        return true;  // origin strictly inside: hit (t is restored by intersectNode)
    if (FILTER && RT_SLAB_FILTER) {
        const int f = ref_slab_bounds(b, o, nd);
        if (f != 2) return f != 0;
    }
    return ref_slab_div(b, o, nd);
}

struct RefMask {
    uint32_t known, pass;
};

template <bool FILTER = false>
__device__ __forceinline__ bool leaf_reachable_p(const int* leaf_path, const DRefNode* refn, int leaf, v3 o, v3 nd,
                                                 RefMask& m) {
    const int* p = leaf_path + leaf * 8;
    const int cnt = p[0];
    for (int k = 1; k <= cnt; ++k) {
        const int node = p[k];
        const uint32_t bit = 1u << node;
        if (!(m.known & bit)) {
            m.known |= bit;
            if (ref_slab<FILTER>(refn[node], o, nd)) m.pass |= bit;
        }
        if (!(m.pass & bit)) return false;
    }
    return true;
}

// The reference BVH in LDS (opaque and tree kernels, RT_REF_LDS): its <= 31 node boxes and every leaf's root path
// packed in one word (count in bits 0-2, node ids in 5-bit fields; all ones: a path of more than 5 nodes, read from
// device memory) -- the culling's loads without a device-memory round trip per path level
struct RefLds {
    DRefNode box[32];
    uint32_t path[32];
};
__device__ __forceinline__ void ref_lds_load(const DevScene& S, RefLds& r, int lane) {
    const float* src = reinterpret_cast<const float*>(S.refn);
    float* dst = &r.box[0].lo[0];
    for (int i = lane; i < S.nref * 6; i += 64) dst[i] = src[i];
    if (lane < 32) {
        const int* p = S.leaf_path + lane * 8;
        const int cnt = p[0];
        uint32_t w = 0xFFFFFFFFu;
        if (cnt <= 5) {
            w = (uint32_t)cnt;
            for (int k = 0; k < cnt; ++k) w |= (uint32_t)p[1 + k] << (3 + 5 * k);
        }
        r.path[lane] = w;
    }
}
template <bool FILTER = false>
__device__ __forceinline__ bool leaf_reachable_lds(const DevScene& S, const RefLds& r, int leaf, v3 o, v3 nd,
                                                   RefMask& m) {
    const uint32_t w = r.path[leaf];
    if (w == 0xFFFFFFFFu) return leaf_reachable_p<FILTER>(S.leaf_path, S.refn, leaf, o, nd, m);
    const int cnt = (int)(w & 7u);
    for (int k = 0; k < cnt; ++k) {
        const int node = (int)((w >> (3 + 5 * k)) & 31u);
        const uint32_t bit = 1u << node;
        if (!(m.known & bit)) {
            m.known |= bit;
            if (ref_slab<FILTER>(r.box[node], o, nd)) m.pass |= bit;
        }
        if (!(m.pass & bit)) return false;
    }
    return true;
}

template <bool FILTER = false>
__device__ __forceinline__ bool leaf_reachable(const DevScene& S, int leaf, v3 o, v3 nd, RefMask& m) {
    return leaf_reachable_p<FILTER>(S.leaf_path, S.refn, leaf, o, nd, m);
}

// ------------------------------------------------------------------------------------------
// Closest / any hit.
// ------------------------------------------------------------------------------------------
struct Best {
    float t;
    int key;
    int rec;  // >= 0: triangle record index; < 0: -(sphere index) - 1; INT_MIN: none
};

#define RT_NO_HIT (-0x7fffffff - 1)

// Reference triangle test for one record.  Returns true and the reference t when the
// reference would accept the triangle with ray.t = +inf (order-free part).
__device__ __forceinline__ bool tri_test(const float4 r0, const float4 r1, const float4 r2, const float4 r3,
                                         v3 o, v3 d, v3 nd, float& t_out) {
    const v3 v0{r0.x, r0.y, r0.z};
    const v3 v1{r1.x, r1.y, r1.z};
    const v3 v2{r2.x, r2.y, r2.z};
    const v3 n{r0.w, r1.w, r2.w};
    const float D = r3.x;
    // intersectRayWithPlane (src/ray_tracing.cpp:63-89)
    const float nDotd = dot(nd, n);
    if (nDotd == 0.0f) return false;
    const float t = (D - dot(o, n)) / nDotd;
    if (!(t >= 0.0f)) return false;
    if (!(t < FLT_MAX)) return false;  // t < ray.t with the initial FLT_MAX
    // pointInTriangle on p = o + dir * t (raw direction; src/ray_tracing.cpp:42-61,104-128)
    const v3 p = o + d * t;
    const bool s0 = dot(cross(p - v0, v2 - v0), n) >= 0.0f;
    const bool s1 = dot(cross(p - v2, v1 - v2), n) >= 0.0f;
    const bool s2 = dot(cross(p - v1, v0 - v1), n) >= 0.0f;
    if (!((s0 && s1 && s2) || (!s0 && !s1 && !s2))) return false;
    t_out = t;
    return true;
}

// Sphere quadratic with the double promotions of glm::pow(float,int) (src/ray_tracing.cpp:182-209).
__device__ __forceinline__ bool sphere_test(const DSph& s, v3 o, v3 d, float& t_out) {
    const v3 m = o - v3{s.c[0], s.c[1], s.c[2]};
    const float A = (float)(((double)d.x * (double)d.x + (double)d.y * (double)d.y) + (double)d.z * (double)d.z);
    const float B = 2.0f * ((d.x * m.x + d.y * m.y) + d.z * m.z);
    const float C = (float)((((double)m.x * (double)m.x + (double)m.y * (double)m.y) + (double)m.z * (double)m.z) -
                            (double)s.r * (double)s.r);
    const float disc = (float)((double)B * (double)B - (double)((4.0f * A) * C));
    if (disc >= 0.0f) {
        float t0 = (-B + sqrtf(disc)) / (2.0f * A);
        float t1 = (-B - sqrtf(disc)) / (2.0f * A);
        if (t0 < 0.0f) t0 = t1;
        if (t1 < 0.0f) t1 = t0;
        const float tm = gmin(t0, t1);
        if (tm > 0.0f && tm < FLT_MAX) {
            t_out = tm;
            return true;
        }
    }
    return false;
}

// The direction's reciprocals for the BVH8 slab tests, which only cull: every box is inflated by eps =
// max(8, max |coordinate|) * 2^-16 (bvh_build.cpp, rt_build.hip), so a point the reference's triangle test
// accepts lies >= eps * |inv| inside every slab interval in t, while a reciprocal off by 1 ulp moves each slab
// t by <= 2^-23 |t| <= 2^-23 * (scene extent + origin distance) * |inv|: ~100x inside the margin, and the signs
// (near / far plane choice) are exact.  So v_rcp_f32 (1 ulp) replaces the IEEE division's ~10-instruction
// sequence per axis with the same culling outcome for every accepted candidate.
__device__ __forceinline__ v3 safe_inv(v3 d) {
    const float e = 1e-20f;
    const float x = fabsf(d.x) < e ? copysignf(e, d.x) : d.x;
    const float y = fabsf(d.y) < e ? copysignf(e, d.y) : d.y;
    const float z = fabsf(d.z) < e ? copysignf(e, d.z) : d.z;
    return v3{__builtin_amdgcn_rcpf(x), __builtin_amdgcn_rcpf(y), __builtin_amdgcn_rcpf(z)};
}

// HitInfo for the winner: hitPoint, normal (interpolated + flipped), material, uv.
struct Surf {
    v3 p;
    v3 n;
    v2 uv;
    DMat m;
    int mesh;
    int prim;
    bool is_tri;
    bool ub;  // triangle hit where barycentricCoordinates returns false (src/ray_tracing.cpp:281-295)
};

// ------------------------------------------------------------------------------------------
// kd textures: Image::getPixel (src/image.cpp:77-110) and its filters (:200-360), with the level
// of detail of computeLevelOfDetails (src/ray_differentials.cpp:112-139).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ v3 tex_texel(const DevScene& S, int4 ti, int level, uint32_t x, uint32_t y) {
    size_t off = (size_t)ti.x;
    for (int l = 0; l < level; ++l) off += (size_t)(ti.y >> l) * (size_t)(ti.z >> l);
    const float* p = S.tex + 3 * (off + (size_t)y * (uint32_t)(ti.y >> level) + x);
    return v3{p[0], p[1], p[2]};
}

// toImageCoordinates (:114-130)
__device__ __forceinline__ v2 tex_image_coords(int4 ti, v2 tc, int level) {
    const uint32_t w = (uint32_t)(ti.y >> level), h = (uint32_t)(ti.z >> level);
    return v2{tc.x * (float)(w - 1u), (1.0f - tc.y) * (float)(h - 1u)};
}

// nearestNeighbor (:201-229): round, clamp to the last row / column
__device__ __forceinline__ v3 tex_nearest(const DevScene& S, int4 ti, v2 ic, int level) {
    const uint32_t w = (uint32_t)(ti.y >> level), h = (uint32_t)(ti.z >> level);
    uint32_t x = (uint32_t)roundf(ic.x), y = (uint32_t)roundf(ic.y);
    if (x >= w) x = w - 1u;
    if (y >= h) y = h - 1u;
    return tex_texel(S, ti, level, x, y);
}

// linearInterpolation (:329-339)
__device__ __forceinline__ v3 tex_lerp(float lo, float hi, v3 cl, v3 ch, float p) {
    if ((double)fabsf(hi - lo) < 1e-6) return cl;
    const float c = (p - lo) / (hi - lo);
    return (1.0f - c) * cl + c * ch;
}

// bilinearInterpolation (:232-252)
__device__ __forceinline__ v3 tex_bilinear(const DevScene& S, int4 ti, v2 ic, int level) {
    const float xl = floorf(ic.x), xh = ceilf(ic.x), yl = floorf(ic.y), yh = ceilf(ic.y);
    const v3 c_ll = tex_texel(S, ti, level, (uint32_t)xl, (uint32_t)yl);
    const v3 c_lr = tex_texel(S, ti, level, (uint32_t)xh, (uint32_t)yl);
    const v3 c_hl = tex_texel(S, ti, level, (uint32_t)xl, (uint32_t)yh);
    const v3 c_hr = tex_texel(S, ti, level, (uint32_t)xh, (uint32_t)yh);
    const v3 lo = tex_lerp(xl, xh, c_ll, c_lr, ic.x);
    const v3 hi = tex_lerp(xl, xh, c_hl, c_hr, ic.x);
    return tex_lerp(yl, yh, lo, hi, ic.y);
}

// clampRepeatTextureCoordinate (:133-191)
__device__ __forceinline__ float tex_wrap(float c, int rule) {
    if (rule == RT_OOB_CLAMP) return c > 1.0f ? 1.0f : (c < 0.0f ? 0.0f : c);
    if (rule == RT_OOB_REPEAT && (c < 0.0f || c > 1.0f)) return c - floorf(c);
    return c;
}

// getPixel (:77-110); levels per getBestLevelMipmap (:500-540)
__device__ v3 tex_get_pixel(const DevScene& S, int t, v2 tc, float lod) {
    if (S.tex_oob_x == RT_OOB_BORDER && (tc.x < 0.0f || tc.x > 1.0f))
        return v3{S.tex_border[0], S.tex_border[1], S.tex_border[2]};
    if (S.tex_oob_y == RT_OOB_BORDER && (tc.y < 0.0f || tc.y > 1.0f))
        return v3{S.tex_border[0], S.tex_border[1], S.tex_border[2]};
    const v2 in{tex_wrap(tc.x, S.tex_oob_x), tex_wrap(tc.y, S.tex_oob_y)};
    const int4 ti = S.tex_info[t];
    const int f = S.tex_filter;
    if (f == RT_TEX_NEAREST) return tex_nearest(S, ti, tex_image_coords(ti, in, 0), 0);
    if (f == RT_TEX_BILINEAR) return tex_bilinear(S, ti, tex_image_coords(ti, in, 0), 0);
    const int nlev = ti.w;
    // getBestLevelMipmap (:495-529): mode 1 = min(levels - 1, ceil(lod)), mode 2 = max(0, floor(lod)),
    // mode 0 = the nearer of the two.  The floor level is not clamped from above: at lod >= levels
    // (+inf included) getWidthHeightForLevel fails (:478-486) and the filter returns its error colour
    // -- black for trilinear (:334-337), white for the nearest-level modes (:270-274, :294-298).
    // The level is compared as a float before any int conversion, so a huge lod is never converted.
    if (f == RT_TEX_TRILINEAR) {
        if (nlev == 0) return v3{0.0f, 0.0f, 0.0f};
        const float flo = gmax(0.0f, floorf(lod));
        if (!(flo < (float)nlev)) return v3{0.0f, 0.0f, 0.0f};
        const int hi = (int)gmin((float)nlev - 1.0f, ceilf(lod));
        const int lo = (int)flo;
        const v3 cl = tex_bilinear(S, ti, tex_image_coords(ti, in, lo), lo);
        const v3 ch = tex_bilinear(S, ti, tex_image_coords(ti, in, hi), hi);
        return tex_lerp((float)lo, (float)hi, cl, ch, lod);
    }
    if (nlev == 0) return v3{1.0f, 1.0f, 1.0f};
    const float fbest = (lod - floorf(lod) < ceilf(lod) - lod) ? gmax(0.0f, floorf(lod))
                                                              : gmin((float)nlev - 1.0f, ceilf(lod));
    if (!(fbest < (float)nlev)) return v3{1.0f, 1.0f, 1.0f};
    const int best = (int)fbest;
    const v2 ic = tex_image_coords(ti, in, best);
    return f == RT_TEX_MIP_NEAREST ? tex_nearest(S, ti, ic, best) : tex_bilinear(S, ti, ic, best);
}

// computeDerivativeOfBarycentricCoordinate (src/ray_differentials.cpp:36-45)
__device__ __forceinline__ float tex_dbary(v3 a, v3 b, v3 p, v3 pd, float area) {
    const v3 term1 = cross(pd, p - b) + cross(p - a, pd);
    const v3 term2 = cross(a - p, b - p);
    const float nom = dot(term1, term2) + dot(term2, term1);
    const float den = 2.0f * area * sqrtf(dot(term2, term2));
    return nom / den;
}

// computeTexturePartialDerivativeInInterpolatedTrianglePoint (:66-80)
__device__ __forceinline__ v2 tex_dT(v3 v0, v3 v1, v3 v2p, v2 t0, v2 t1, v2 t2, v3 p, v3 pd) {
    const float area = length(cross(v2p - v0, v1 - v0));
    const float a = tex_dbary(v2p, v1, p, pd, area);
    const float b = tex_dbary(v0, v2p, p, pd, area);
    const float g = tex_dbary(v1, v0, p, pd, area);
    return v2{(a * t0.x + b * t1.x) + g * t2.x, (a * t0.y + b * t1.y) + g * t2.y};
}

// Level of detail of a triangle hit: the ray's differentials as Ray's member initialisers give
// them (right = (1,0,0), up = (0,-1,0); a camera ray is default-constructed with direction
// (0,0,-1) and set afterwards, a secondary ray is built with its direction), transferred to the
// hit (transfer_ray_differentials, :5-15), then computeLevelOfDetails (:112-139).  The reference
// reads `right`/`up` before their initialisers run (ray.h:19-20 vs :25-28); this is the value
// the initialisers intend.
__device__ float tex_lod(v3 d, float t, v3 normal, bool primary, v3 v0, v3 v1, v3 v2p, v2 t0, v2 t1, v2 t2,
                         v3 p) {
    const v3 right{1.0f, 0.0f, 0.0f}, up{0.0f, -1.0f, 0.0f};
    const v3 dc = primary ? v3{0.0f, 0.0f, -1.0f} : d;
    const float dd = dot(dc, dc);
    const float pw = powf(dd, 1.5f);
    const v3 dDx = (dd * right - dot(dc, right) * dc) / pw;
    const v3 dDy = (dd * up - dot(dc, up) * dc) / pw;
    const v3 N = normalize(normal), D = normalize(d);
    const v3 zero{0.0f, 0.0f, 0.0f};
    const v3 ax = zero + t * dDx, ay = zero + t * dDy;
    const float dtx = -dot(ax, N) / dot(D, N);
    const float dty = -dot(ay, N) / dot(D, N);
    const v3 dPx = ax + dtx * D, dPy = ay + dty * D;
    const v2 dTx = tex_dT(v0, v1, v2p, t0, t1, t2, p, 1.0f * dPx);
    const v2 dTy = tex_dT(v0, v1, v2p, t0, t1, t2, p, 1.0f * dPy);
    const float lx = sqrtf(dTx.x * dTx.x + dTx.y * dTx.y), ly = sqrtf(dTy.x * dTy.x + dTy.y * dTy.y);
    const float m = (lx < ly) ? ly : lx;  // glm::max
    const float l2 = log2f(m);
    return (0.0f < l2) ? l2 : 0.0f;
}

// shade = the hit is shaded (getFinalColor): a textured triangle's kd comes from its texture
// (src/main.cpp:155-171); primary = the ray is a camera ray (level 0)
__device__ __forceinline__ Surf surface(const DevScene& S, v3 o, v3 d, const Best& b, bool shade = false,
                                        bool primary = false) {
    Surf s;
    if (b.rec >= 0) {
        const float4* tp = S.tri + b.rec * 4;
        const float4 r0 = tp[0], r1 = tp[1], r2 = tp[2], r3 = tp[3];
        const v3 v0{r0.x, r0.y, r0.z}, v1{r1.x, r1.y, r1.z}, v2{r2.x, r2.y, r2.z};
        const v3 fn{r0.w, r1.w, r2.w};
        const int sidx = __float_as_int(r3.y);
        s.p = o + d * b.t;
        // barycentricCoordinates (src/ray_tracing.cpp:276-308), "unthresholded" semantics
        const float A = length(cross(v1 - v0, v2 - v0));
        v3 bc{0.0f, 0.0f, 0.0f};
        if (A > 0.0f) {
            bc.x = length(cross(v1 - s.p, v2 - s.p)) / A;
            bc.y = length(cross(s.p - v0, v2 - v0)) / A;
            bc.z = length(cross(v1 - v0, s.p - v0)) / A;
        }
        // the reference's own checks (isZero = |x| < 1e-4 compared in double, :15-24): off the
        // triangle's plane, or a parallelogram area below 1e-4 -- the pointInTriangle check passes,
        // it is the test that accepted the hit.  Where they fail the reference interpolates from
        // uninitialised coordinates (:147-157); the unthresholded ones above are used instead.
        s.ub = !((double)fabsf(dot(fn, s.p - v0)) < 1e-4) || ((double)A < 1e-4);
        const float* nn = S.nrm + (size_t)sidx * 9;
        const v3 n0{nn[0], nn[1], nn[2]}, n1{nn[3], nn[4], nn[5]}, n2{nn[6], nn[7], nn[8]};
        v3 n = (n0 * bc.x + n1 * bc.y) + n2 * bc.z;
        if (dot(n, fn) < 0.0f) n = -n;
        s.n = n;
        const float* uu = S.uv + (size_t)sidx * 6;
        s.uv = rt::v2{(uu[0] * bc.x + uu[2] * bc.y) + uu[4] * bc.z, (uu[1] * bc.x + uu[3] * bc.y) + uu[5] * bc.z};
        s.mesh = S.mesh[sidx];
        s.m = S.mats[s.mesh];
        s.prim = sidx;
        s.is_tri = true;
        if (shade && S.tex_on) {
            const int tx = S.mat_tex[s.mesh];
            if (tx >= 0) {
                float lod = 0.0f;
                if (S.tex_filter >= RT_TEX_MIP_NEAREST)
                    lod = tex_lod(d, b.t, s.n, primary, v0, v1, v2, rt::v2{uu[0], uu[1]}, rt::v2{uu[2], uu[3]},
                                  rt::v2{uu[4], uu[5]}, s.p);
                const v3 kd = tex_get_pixel(S, tx, s.uv, lod);
                s.m.kd[0] = kd.x;
                s.m.kd[1] = kd.y;
                s.m.kd[2] = kd.z;
            }
        }
    } else {
        const int si = -b.rec - 1;
        const DSph sp = S.sph[si];
        s.p = o + b.t * d;
        s.n = normalize(s.p - v3{sp.c[0], sp.c[1], sp.c[2]});
        s.uv = rt::v2{0.0f, 0.0f};
        s.m = sp.m;
        s.mesh = -1;
        s.prim = S.ntri + si;
        s.is_tri = false;
        s.ub = false;
    }
    return s;
}

// calcColor (src/main.cpp:112-121)
__device__ __forceinline__ v3 calc_color(v3 lcolor, float intensity, float cosL, float cosS, const DMat& m) {
    const v3 kd{m.kd[0], m.kd[1], m.kd[2]};
    const v3 ks{m.ks[0], m.ks[1], m.ks[2]};
    const v3 diffuse = ((kd * lcolor) * intensity) * cosL;
    v3 spec{0.0f, 0.0f, 0.0f};
    if (m.shin > 0.0f) spec = (lcolor * ks) * powf(cosS, m.shin);
    return diffuse + spec;
}

__device__ __forceinline__ v3 ld3(const float* p) { return v3{p[0], p[1], p[2]}; }

// ------------------------------------------------------------------------------------------
// getFinalColor's recursion tree (src/main.cpp:187-290), walked depth first with the colours
// accumulated forward: a node at weight w adds w * (its direct light) to the sample's colour and
// hands w * (edge weight) to its children -- ks*ks for a mirror child (ks*ks/N with shininess),
// R and 1-R for the reflected and refracted rays of a transparent node, ks*max(pow(.)..)/N for a
// glossy lobe sample.  This is the reference's nested sum reassociated (relative drift ~1e-7,
// inside the 1e-5 tolerance; the geometry and the ray tree are unchanged).  Only branching nodes
// leave work behind, so only they push a frame: the pending refracted ray of a transparent node,
// the lobe of a glossy one (glossy_ray_count > 1).  Pure mirror chains keep no stack.
// ------------------------------------------------------------------------------------------
enum { FR_REFRACT = 0, FR_GLOSSY = 1 };
struct Frame {
    v3 o, d;     // REFRACT: the refracted ray | GLOSSY: hit point, reflect direction
    v3 w;        // REFRACT: the child's weight | GLOSSY: the node's weight * ks / glossy_ray_count
    v3 nraw;     // GLOSSY: hitInfo.normal (unnormalised, the lobe's side test)
    float shin, gd;  // GLOSSY: shininess and the lobe half-width d (host-evaluated per material)
    int mode;
    int level;   // recursion level of the child rays
    int sample;  // GLOSSY: lobe samples drawn so far (1 .. glossy_ray_count - 1)
};

__device__ __forceinline__ void gen_ray(const KParams& P, float px, float py, v3& o, v3& d) {
    const v3 csd = normalize(v3{-px * P.hw, py * P.hh, 1.0f});
    o = v3{P.cam[0], P.cam[1], P.cam[2]};
    d = quat_rotate(P.q[0], P.q[1], P.q[2], P.q[3], csd);
}

// camera ray of view v of a view batch (the same Trackball::generateRay arithmetic, per-view camera)
__device__ __forceinline__ void gen_ray_view(const KParams& P, int v, float px, float py, v3& o, v3& d) {
    const float* c = P.views + 12 * v;
    const v3 csd = normalize(v3{-px * c[8], py * c[7], 1.0f});
    o = v3{c[0], c[1], c[2]};
    d = quat_rotate(c[3], c[4], c[5], c[6], csd);
}

template <bool COUNT>
__device__ void flush_counters(const KParams& P, const Cnt& c) {
    // wave-level reduction, one atomic per wave and counter
    unsigned long long r = c.rays, nv = c.nodes, tt = c.tris, h = c.hits;
    for (int off = 32; off > 0; off >>= 1) {
        r += __shfl_xor(r, off);
        if (COUNT) {
            nv += __shfl_xor(nv, off);
            tt += __shfl_xor(tt, off);
            h += __shfl_xor(h, off);
        }
    }
    unsigned long long wn = c.wnodes, wt = c.wtris, wa = c.wadv;
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            wn += __shfl_xor(wn, off);
            wt += __shfl_xor(wt, off);
            wa += __shfl_xor(wa, off);
        }
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(P.stats + 0, r);
        if (COUNT) {
            atomicAdd(P.stats + 1, nv);
            atomicAdd(P.stats + 2, tt);
            atomicAdd(P.stats + 3, h);
            atomicAdd(P.stats + 4, wn);
            atomicAdd(P.stats + 5, wt);
            atomicAdd(P.stats + 6, wa);
            atomicAdd(P.stats + 8, c.cyc_a);
            atomicAdd(P.stats + 9, c.cyc_b);
            atomicAdd(P.stats + 10, c.cyc_c);
            atomicAdd(P.stats + 11, c.cyc_d);
        }
    }
    if (COUNT) {
        unsigned long long u = c.ub;
        for (int off = 32; off > 0; off >>= 1) u += __shfl_xor(u, off);
        if ((threadIdx.x & 63) == 0) atomicAdd(P.stats + 12, u);
        for (int k = 0; k < 3; ++k) {
            unsigned long long v = c.hist[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if ((threadIdx.x & 63) == 0) atomicAdd(P.stats + 13 + k, v);
        }
        const uint32_t xs[3] = {c.rv, c.rvk, c.rvj};
        for (int k = 0; k < 3; ++k) {
            unsigned long long v = xs[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if ((threadIdx.x & 63) == 0) atomicAdd(P.stats + RT_STATS_EXTRA + k, v);
        }
        if ((threadIdx.x & 63) == 0) {  // rt_debug_counters [50], [51], [52]
            atomicAdd(P.stats + RT_STATS_EXTRA + 16, c.cyc_e);
            atomicAdd(P.stats + RT_STATS_EXTRA + 17, c.cyc_f);
            atomicAdd(P.stats + RT_STATS_EXTRA + 18, c.cyc_g);
        }
        const uint32_t cm[2] = {c.cmn, c.cmr};  // rt_debug_counters [53], [54]
        for (int k = 0; k < 2; ++k) {
            unsigned long long v = cm[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if ((threadIdx.x & 63) == 0) atomicAdd(P.stats + RT_STATS_EXTRA + 19 + k, v);
        }
        const uint32_t mix[2] = {c.shad, c.cmiss};  // rt_debug_counters [26], [27]
        for (int k = 0; k < 2; ++k) {
            unsigned long long v = mix[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if ((threadIdx.x & 63) == 0) atomicAdd(P.stats + RT_STATS_EXTRA + 10 + k, v);
        }
    }
}

// the opaque kernel's ref_slab and lane-iteration counters (rt_debug_counters [19..23])
template <bool COUNT>
__device__ void flush_slab_counters(const KParams& P, const SlabCnt& c) {
    if (!COUNT) return;
    const uint32_t xs[5] = {c.slab, c.wslab, c.blocked, c.both, c.iters};
    for (int k = 0; k < 5; ++k) {
        unsigned long long v = xs[k];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0) atomicAdd(P.stats + RT_STATS_EXTRA + 3 + k, v);
    }
}

// Gathered band buffers [band_count][max_local][band_rows][W][3] -> setPixel layout
// (src/screen.cpp:32-38: index (H-1-y)*W + x).
__global__ void unpermute_kernel(int W, int H, int band_rows, int band_count, int max_local, const float* src,
                                 float* dst) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)W * H;
    if (idx >= total) return;
    const int x = (int)(idx % W);
    const int y = (int)(idx / W);
    const int gb = y / band_rows;
    const int r = y % band_rows;
    const int rank = gb % band_count;
    const int lb = gb / band_count;
    const float* s = src + ((((size_t)rank * max_local + lb) * band_rows + r) * W + x) * 3;
    float* d = dst + ((size_t)(H - 1 - y) * W + x) * 3;
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
}

// Image::getPixel(uv, lod) on texture `t` for n (u, v, lod) triples (rt_texture_sample).
// A view batch gathered from band_count ranks, [band_count][n_views][max_local][band_rows][W][3] (each
// rank's rt_render_views_device buffer back to back), -> n_views images in the setPixel layout.
__global__ void unpermute_views_kernel(int W, int H, int band_rows, int band_count, int max_local, int n_views,
                                       const float* src, float* dst) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t per_view = (size_t)W * H;
    if (idx >= per_view * n_views) return;
    const int v = (int)(idx / per_view);
    const size_t pix = idx - (size_t)v * per_view;
    const int x = (int)(pix % W);
    const int y = (int)(pix / W);
    const int gb = y / band_rows;
    const int r = y % band_rows;
    const int rank = gb % band_count;
    const int lb = gb / band_count;
    const float* s = src + (((((size_t)rank * n_views + v) * max_local + lb) * band_rows + r) * W + x) * 3;
    float* d = dst + ((size_t)v * per_view + (size_t)(H - 1 - y) * W + x) * 3;
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
}

// One rank's band-dense buffer [n_views][max_local][band_rows][W][3] (rank of count: its local band lb is
// the frame's band lb * count + rank) -> its rows of the n_views images in the setPixel layout.
__global__ void scatter_bands_kernel(int W, int H, int band_rows, int rank, int count, int max_local, int n_views,
                                     const float* src, float* dst) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t per_view = (size_t)max_local * band_rows * W;
    if (idx >= per_view * n_views) return;
    const int v = (int)(idx / per_view);
    const size_t k = idx - (size_t)v * per_view;
    const int x = (int)(k % W);
    const int r = (int)(k / W);  // row of the rank's band-dense view
    const int lb = r / band_rows, row = r % band_rows;
    const int y = (lb * count + rank) * band_rows + row;
    if (y >= H) return;
    const float* s = src + idx * 3;
    float* d = dst + ((size_t)v * H * W + (size_t)(H - 1 - y) * W + x) * 3;
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
}

__global__ void tex_sample_kernel(DevScene S, int t, const float* uvl, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const v3 c = tex_get_pixel(S, t, v2{uvl[3 * i], uvl[3 * i + 1]}, uvl[3 * i + 2]);
    out[3 * i] = c.x;
    out[3 * i + 1] = c.y;
    out[3 * i + 2] = c.z;
}

__global__ void selftest_kernel(const float* x, const float* y, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i * 4 + 0] = sqrtf(x[i]);
    out[i * 4 + 1] = 1.0f / x[i];
    out[i * 4 + 2] = x[i] / y[i];
    out[i * 4 + 3] = powf(x[i], y[i]);
}

}  // namespace rt
