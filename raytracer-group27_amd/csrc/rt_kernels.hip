// rt_kernels.hip -- MI355X (gfx950) megakernel for the reference's per-pixel hot path.
//
// One lane = one pixel (one 8x8 pixel tile per 64-lane wave).  Per lane the kernel runs the
// reference's recursion tree iteratively:
//   renderRayTracing (src/main.cpp:340-400) -> Trackball::generateRay (framework/src/trackball.cpp:87-98)
//   -> getFinalColor (src/main.cpp:129-301) -> BoundingVolumeHierarchy::intersect (src/bounding_volume_hierarchy.cpp:49-78)
//   -> light gathering + cansee (src/shadow.cpp:32-321) -> calcColor (src/main.cpp:112-121)
// Closest-hit queries walk a binned-SAH BVH2 (64-B nodes, both child boxes per node, near-first,
// short stack in LDS) but every candidate is accepted or rejected with the reference's own
// arithmetic (plane/edge test, src/ray_tracing.cpp:42-128; sphere quadratic in double,
// :182-209), and ties in t go to the first object in the reference's visit order, so the hit is
// the one the reference's brute-force loop (useBVH=false) or its depth-4 BVH walk (useBVH=true,
// every shadow ray) returns.  useBVH=true additionally requires every box on the candidate's
// reference leaf path to pass the reference slab test (src/ray_tracing.cpp:213-264), evaluated
// lazily and cached per ray.
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
    const float4* __restrict__ tri;      // [nrec][4] BVH2 leaf order
    const float4* __restrict__ nodes;    // [nnodes][4]
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
    unsigned long long* stats;  // rays, node visits, tri tests, hits
    int refill;                 // dynamic-fetch kernel: waiting lanes that end a traversal phase
    int leaf_batch;             // dynamic-fetch kernel: lanes with postponed leaves that start a leaf phase
    const float* pre_t;         // precomputed primary hits per job (rt_packet.hip), or null
    const int* pre_rec;
    uint32_t seed_lo, seed_hi;  // glossy sampling: Philox-4x32-10 key (rt_params.rng_seed)
    unsigned long long* wave_trace;  // developer trace (RT_WAVE_TRACE=1): per wave (start, end, jobs), or null
    const int* job_order;            // persistent kernels: k-th job handed out is job_order[k] (rt_schedule.hip), or null
    int* job_cost;                   // persistent kernels (pixels): queries each job took, or null
    int coop;                        // dynamic-fetch kernel: lane-group traversal of the drain's queries
    int coop_max;                    // ... when at most this many queries are left in the wave
    int coop_reserve;                // ... free pool slots kept for depth-first steps
    // view batch (rt_render_views_device): n_views frames of the same scene in one launch, view v's
    // camera at views[12 v] (cam xyz, quat wxyz, hh, hw), its rows at out + v * view_rows * W * 3
    int n_views, view_jobs, view_rows;
    const float* views;
};

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
    uint32_t wnodes, wtris, wadv;  // wave-level steps (counted by the first active lane): SIMD efficiency
    unsigned long long cyc_a, cyc_b;  // shader clocks per wave in the state machine / in traversal (df kernel)
    unsigned long long cyc_c, cyc_d;  // ... of cyc_a: advancing finished queries / fetching jobs
};

// true on the lowest active lane of the wave (counting builds: one count per wave instruction stream)
__device__ __forceinline__ bool wave_leader() {
    return (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1;
}

// ------------------------------------------------------------------------------------------
// Reference slab test (src/ray_tracing.cpp:213-264), dir = normalize(ray.direction).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool ref_slab(const DRefNode& b, v3 o, v3 nd) {
    if (b.lo[0] == FLT_MAX && b.lo[1] == FLT_MAX && b.lo[2] == FLT_MAX && b.hi[0] == -FLT_MAX &&
        b.hi[1] == -FLT_MAX && b.hi[2] == -FLT_MAX)
        return false;
    if (o.x > b.lo[0] && o.y > b.lo[1] && o.z > b.lo[2] && o.x < b.hi[0] && o.y < b.hi[1] && o.z < b.hi[2])
        return true;  // origin strictly inside: hit (t is restored by intersectNode)
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

struct RefMask {
    uint32_t known, pass;
};

__device__ __forceinline__ bool leaf_reachable_p(const int* leaf_path, const DRefNode* refn, int leaf, v3 o, v3 nd,
                                                 RefMask& m) {
    const int* p = leaf_path + leaf * 8;
    const int cnt = p[0];
    for (int k = 1; k <= cnt; ++k) {
        const int node = p[k];
        const uint32_t bit = 1u << node;
        if (!(m.known & bit)) {
            m.known |= bit;
            if (ref_slab(refn[node], o, nd)) m.pass |= bit;
        }
        if (!(m.pass & bit)) return false;
    }
    return true;
}

__device__ __forceinline__ bool leaf_reachable(const DevScene& S, int leaf, v3 o, v3 nd, RefMask& m) {
    return leaf_reachable_p(S.leaf_path, S.refn, leaf, o, nd, m);
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
#define RT_PRE_NONE (-0x7fffffff)  // INT_MIN + 1: no precomputed primary hit (rt_packet.hip); trace it

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

__device__ __forceinline__ v3 safe_inv(v3 d) {
    const float e = 1e-20f;
    const float x = fabsf(d.x) < e ? copysignf(e, d.x) : d.x;
    const float y = fabsf(d.y) < e ? copysignf(e, d.y) : d.y;
    const float z = fabsf(d.z) < e ? copysignf(e, d.z) : d.z;
    return v3{1.0f / x, 1.0f / y, 1.0f / z};
}

// Conservative slab test against an inflated BVH2 child box; returns the entry distance.
__device__ __forceinline__ bool box_hit(float lx, float ly, float lz, float hx, float hy, float hz, v3 o, v3 inv,
                                        float tmax, float& tnear) {
    const float ax = (lx - o.x) * inv.x, bx = (hx - o.x) * inv.x;
    const float ay = (ly - o.y) * inv.y, by = (hy - o.y) * inv.y;
    const float az = (lz - o.z) * inv.z, bz = (hz - o.z) * inv.z;
    const float t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    tnear = t0;
    return t0 <= t1 && t1 >= 0.0f && t0 <= tmax;
}

// mode REF: useBVH=true semantics (leaf-path mask + DFS-rank tie-break)
// ANY: any-hit with threshold `thr` (occluded iff some valid candidate has t <= thr)
template <bool REF, bool ANY, bool COUNT>
__device__ bool traverse(const DevScene& S, v3 o, v3 d, v3 nd, float t_init, float thr, Best& best, int* stk,
                         Cnt& cnt) {
    best.t = t_init;
    best.key = -1;  // a candidate tying the caller's initial ray.t is rejected (strict t < ray.t)
    best.rec = RT_NO_HIT;
    RefMask mask{0u, 0u};
    const v3 inv = safe_inv(d);
    float tcull = ANY ? thr : t_init;
    int sp = 0;
    int node = 0;
    bool found = false;
    // The reference measures t along normalize(dir) but places the test point at o + dir*t
    // (src/ray_tracing.cpp:71,111), so for a non-unit direction the accepted point lies off the
    // triangle and no bounding volume can find it: such rays (only reachable through
    // rt_intersect / rt_shade; every ray the renderer makes is unit length) test every record.
    const float dd = dot(d, d);
    if (!(fabsf(dd - 1.0f) <= 4e-6f)) {
        for (int r = 0; r < S.ntri; ++r) {
            const float4* tp = S.tri + r * 4;
            const float4 r0 = tp[0], r1 = tp[1], r2 = tp[2], r3 = tp[3];
            if (COUNT) cnt.tris++;
            float t;
            if (!tri_test(r0, r1, r2, r3, o, d, nd, t)) continue;
            const int key = REF ? __float_as_int(r3.z) : __float_as_int(r3.y);
            if (ANY) {
                if (!(t <= thr)) continue;
            } else {
                if (!(t < best.t || (t == best.t && key < best.key))) continue;
            }
            if (REF && !leaf_reachable(S, __float_as_int(r3.w), o, nd, mask)) continue;
            best.t = t;
            best.key = key;
            best.rec = r;
            found = true;
            if (ANY) return true;
        }
    } else if (S.ntri > 0) {
        for (;;) {
            const float4* np = S.nodes + node * 4;
            const float4 a = np[0];
            const float4 b = np[1];
            const float4 c = np[2];
            const float4 e = np[3];
            const int c0 = __float_as_int(e.x), c1 = __float_as_int(e.y);
            const int n0 = __float_as_int(e.z), n1 = __float_as_int(e.w);
            if (COUNT) cnt.nodes++;
            float tn0 = 0.0f, tn1 = 0.0f;
            bool h0 = (c0 >= 0) && box_hit(a.x, a.y, a.z, a.w, b.x, b.y, o, inv, tcull, tn0);
            bool h1 = (c1 >= 0) && box_hit(b.z, b.w, c.x, c.y, c.z, c.w, o, inv, tcull, tn1);
            // leaves are tested in place
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                const bool hs = side == 0 ? h0 : h1;
                const int cnum = side == 0 ? n0 : n1;
                const int first = side == 0 ? c0 : c1;
                if (hs && cnum > 0) {
                    for (int r = first; r < first + cnum; ++r) {
                        const float4* tp = S.tri + r * 4;
                        const float4 r0 = tp[0], r1 = tp[1], r2 = tp[2], r3 = tp[3];
                        if (COUNT) cnt.tris++;
                        float t;
                        if (!tri_test(r0, r1, r2, r3, o, d, nd, t)) continue;
                        const int key = REF ? __float_as_int(r3.z) : __float_as_int(r3.y);
                        if (ANY) {
                            if (!(t <= thr)) continue;
                        } else {
                            if (!(t < best.t || (t == best.t && key < best.key))) continue;
                        }
                        if (REF && !leaf_reachable(S, __float_as_int(r3.w), o, nd, mask)) continue;
                        best.t = t;
                        best.key = key;
                        best.rec = r;
                        found = true;
                        if (ANY) return true;
                        tcull = t;
                    }
                    if (side == 0) h0 = false;
                    else h1 = false;
                }
            }
            h0 = h0 && tn0 <= tcull;
            h1 = h1 && tn1 <= tcull;
            if (h0 && h1) {
                const bool first0 = tn0 <= tn1;
                stk[sp * RT_WAVE] = first0 ? c1 : c0;
                ++sp;
                node = first0 ? c0 : c1;
            } else if (h0) {
                node = c0;
            } else if (h1) {
                node = c1;
            } else {
                if (sp == 0) break;
                --sp;
                node = stk[sp * RT_WAVE];
            }
        }
    }
    // spheres: all tested (few); order handled by key
    for (int s = 0; s < S.nsph; ++s) {
        const DSph sp_ = S.sph[s];
        float t;
        if (!sphere_test(sp_, o, d, t)) continue;
        const int key = REF ? sp_.key_bvh : S.ntri + s;
        if (ANY) {
            if (!(t <= thr)) continue;
        } else {
            if (!(t < best.t || (t == best.t && key < best.key))) continue;
        }
        if (REF && !leaf_reachable(S, sp_.leaf, o, nd, mask)) continue;
        best.t = t;
        best.key = key;
        best.rec = -s - 1;
        found = true;
        if (ANY) return true;
    }
    return found;
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
    if (f == RT_TEX_TRILINEAR) {
        if (nlev == 0) return v3{0.0f, 0.0f, 0.0f};
        const int hi = (int)gmin((float)nlev - 1.0f, ceilf(lod));
        const int lo = (int)gmax(0.0f, floorf(lod));
        const v3 cl = tex_bilinear(S, ti, tex_image_coords(ti, in, lo), lo);
        const v3 ch = tex_bilinear(S, ti, tex_image_coords(ti, in, hi), hi);
        return tex_lerp((float)lo, (float)hi, cl, ch, lod);
    }
    if (nlev == 0) return v3{1.0f, 1.0f, 1.0f};
    const int best = (lod - floorf(lod) < ceilf(lod) - lod) ? (int)gmax(0.0f, floorf(lod))
                                                           : (int)gmin((float)nlev - 1.0f, ceilf(lod));
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
    }
    return s;
}

// ------------------------------------------------------------------------------------------
// cansee (src/shadow.cpp:32-69): loop over transparent occluders with Fresnel attenuation.
// ------------------------------------------------------------------------------------------
template <bool COUNT>
__device__ bool cansee(const DevScene& S, v3 p1, v3 p2, float& intensity, int* stk, Cnt& cnt) {
    v3 o = p1;
    v3 d = p2 - p1;
    float distance = length(d);
    d = normalize(d);
    o = o + 0.0005f * d;
    // d is already normalized; normalize(d) inside the triangle test is recomputed as the
    // reference does (normalize of a unit vector is not always the identity in float).
    const v3 nd = normalize(d);
    while (distance > 0.0005f) {
        cnt.rays++;
        const float thr = distance - 2.0f * 0.0005f;
        Best b;
        if (S.all_opaque) {
            // no transparent candidate can exist: occluded iff any valid candidate has t <= thr
            return !traverse<true, true, COUNT>(S, o, d, nd, FLT_MAX, thr, b, stk, cnt);
        }
        const bool hit = traverse<true, false, COUNT>(S, o, d, nd, FLT_MAX, 0.0f, b, stk, cnt);
        if (!hit || (b.t > thr)) return true;
        const Surf s = surface(S, o, d, b);
        if (s.m.transp != 1.0f) {
            distance -= b.t;
            o = s.p + 0.0005f * d;
            const float c = fabsf(dot(d, s.n));
            const float R0 = s.m.transp;
            intensity = (float)((double)intensity *
                                (1.0 - ((double)R0 + (double)(1.0f - R0) * pow((double)(1.0f - c), 5.0))));
        } else {
            return false;
        }
    }
    return true;
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

// Direct light: getPointLights, getSpherelights, getSpotLichts, getPlaneLights (src/shadow.cpp:106-321),
// summed in that order as getFinalColor does (src/main.cpp:174-185).
template <bool COUNT>
__device__ v3 direct_light(const KParams& P, const Surf& s, v3 refl, int* stk, Cnt& cnt) {
    const DevScene& S = P.S;
    v3 color{0.0f, 0.0f, 0.0f};
    const v3 nN = normalize(s.n);
    const v3 nR = normalize(refl);
    for (int i = 0; i < S.npl; ++i) {
        const rt_point_light L = S.pl[i];
        const v3 lp = ld3(L.position);
        float intensity = 1.0f;
        if (cansee<COUNT>(S, s.p, lp, intensity, stk, cnt)) {
            const v3 ldir = normalize(lp - s.p);
            const float cosL = fabsf(dot(nN, ldir));
            const float dd = dot(nR, ldir);
            const float cosS = (0.0f < dd) ? dd : 0.0f;  // std::max(0.0f, x)
            color += calc_color(ld3(L.color), intensity, cosL, cosS, s.m);
        }
    }
    for (int i = 0; i < S.nsl; ++i) {
        const rt_spherical_light L = S.sl[i];
        const v3 lp = ld3(L.position);
        float intensity = 1.0f;
        float intensitySum = 1.0f;
        int hits = 0;
        if (cansee<COUNT>(S, s.p, lp, intensitySum, stk, cnt)) hits++;
        v3 dd = lp - s.p;
        dd = normalize(dd);
        v3 notd = dd;
        if (dd.x != 0.0f) {
            notd.y = -dd.x;
            notd.x = dd.y;
        } else {
            notd.y = -dd.z;
            notd.z = dd.y;
        }
        v3 perp = normalize(cross(dd, notd)) * L.radius;
        const m3 rot = rodrigues(P.sl_sin, P.sl_1mcos, dd);
        const int m = P.sl_m, n = P.sl_n;
        for (int i2 = 0; i2 < n; ++i2) {
            for (int j = 0; j < m; ++j) {
                intensity = 1.0f;
                if (cansee<COUNT>(S, s.p, lp + ((float)(m - j) / (float)m) * perp, intensity, stk, cnt)) {
                    hits++;
                    intensitySum += intensity;
                }
            }
            perp = mul(rot, perp);
        }
        if (hits > 0) {
            const float li = intensitySum / (float)P.sl_count;
            const v3 ldir = normalize(lp - s.p);
            const float cosL = fabsf(dot(nN, ldir));
            const float d2 = dot(nR, ldir);
            const float cosS = (0.0f < d2) ? d2 : 0.0f;
            color += calc_color(ld3(L.color), li, cosL, cosS, s.m);
        }
    }
    for (int i = 0; i < S.nspot; ++i) {
        const DSpot L = S.spot[i];
        const v3 lp = ld3(L.pos);
        if (dot(normalize(ld3(L.dir)), normalize(s.p - lp)) > L.cos_angle) {
            float intensity = 1.0f;
            if (cansee<COUNT>(S, s.p, lp, intensity, stk, cnt)) {
                const v3 ldir = normalize(lp - s.p);
                const float cosL = fabsf(dot(nN, ldir));
                const float d2 = dot(nR, ldir);
                const float cosS = (0.0f < d2) ? d2 : 0.0f;
                color += calc_color(ld3(L.color), intensity, cosL, cosS, s.m);
            }
        }
    }
    for (int i = 0; i < S.nplane; ++i) {
        const rt_plane_light L = S.plane[i];
        const int k = P.plane_k;
        float hit = 0.0f;
        int hitCount = 0;
        float maxCos = 0.0f;
        float intensitySum = 0.0f;
        float intensity = 1.0f;
        const v3 w = ld3(L.width), h = ld3(L.height), lpos = ld3(L.position);
        const v3 dx = (1.0f / (float)(k - 1)) * w;
        const v3 dy = (1.0f / (float)(k - 1)) * h;
        v3 py = lpos;
        const v3 normal = normalize(cross(w, h));
        if (dot(normalize(s.p - (lpos + 0.5f * (w + h))), normal) > 0.0f) {
            for (int i2 = 0; i2 < k; ++i2) {
                v3 px = py;
                for (int j = 0; j < k; ++j) {
                    intensity = 1.0f;
                    if (cansee<COUNT>(S, s.p, px, intensity, stk, cnt)) {
                        intensitySum += intensity;
                        const float dn = dot(normalize(s.p - px), normal);
                        hit += ((dn < 0.0f) ? 0.0f : dn) / length(s.p - px);
                        hitCount++;
                        const float c2 = dot(nR, normalize(px - s.p));
                        maxCos = (maxCos < c2) ? c2 : maxCos;
                    }
                    px = px + dx;
                }
                py = py + dy;
            }
        }
        if (hit > 0.0f) {
            const float li = (intensitySum / (float)hitCount) * hit / (float)(k * k);
            color += calc_color(ld3(L.color), li, 1.0f, maxCos, s.m);
        }
    }
    return color;
}

// ------------------------------------------------------------------------------------------
// getFinalColor as an iterative depth-first walk of its recursion tree.  Each frame keeps the
// parent's partial colour so children are folded in with the reference's exact nesting:
//   mirror:      color += (ks * (0 + ks * child)) / glossy_ray_count   (or ks * (...) if shininess == 0)
//   transparent: color += R * reflectChild;  color += (1-R) * refractChild   (src/main.cpp:191-290)
// ------------------------------------------------------------------------------------------
enum { FR_MIRROR = 0, FR_TRANS_A = 1, FR_TRANS_B = 2, FR_GLOSSY = 3 };
struct Frame {
    v3 color;
    v3 w;      // ks (mirror, glossy) | (reflectionChance, refractionChance, -) (transparent)
    v3 o2, d2; // pending refracted ray | glossy: reflectColor accumulator, reflect
    int mode;
    int flag;  // mirror: shininess != 0 ; transparent: refracted ray traced ; glossy: sample index
    // glossy lobe (src/main.cpp:204-250): hit point, hitInfo.normal (unnormalised), current sample
    // direction, shininess and the lobe half-width d (host-evaluated per material)
    v3 hp, nraw, sdir;
    float shin, gd;
    v3 kd;  // persistent kernels: kd of the shading point at this level (texture or material)
};

template <bool COUNT>
__device__ v3 get_final_color(const KParams& P, v3 o, v3 d, float t_init, int* stk, Cnt& cnt) {
    const DevScene& S = P.S;
    Frame fr[RT_MAX_DEPTH];
    int level = 0;
    for (;;) {
        v3 col{0.0f, 0.0f, 0.0f};
        bool descend = false;
        cnt.rays++;
        Best b;
        const v3 nd = normalize(d);
        bool hit = P.use_bvh ? traverse<true, false, COUNT>(S, o, d, nd, t_init, 0.0f, b, stk, cnt)
                             : traverse<false, false, COUNT>(S, o, d, nd, t_init, 0.0f, b, stk, cnt);
        t_init = FLT_MAX;
        if (hit) {
            if (COUNT) cnt.hits++;
            const Surf s = surface(S, o, d, b, true, level == 0);
            const v3 refl = reflect(normalize(d), normalize(s.n));
            col = direct_light<COUNT>(P, s, refl, stk, cnt);
            if (level < P.max_level) {
                if (s.m.transp == 1.0f) {
                    if (s.m.ks[0] > 0.0f || s.m.ks[1] > 0.0f || s.m.ks[2] > 0.0f) {
                        Frame& f = fr[level];
                        f.color = col;
                        f.w = v3{s.m.ks[0], s.m.ks[1], s.m.ks[2]};
                        f.mode = FR_MIRROR;
                        f.flag = (s.m.shin != 0.0f);
                        o = s.p + 0.01f * refl;
                        d = refl;
                        descend = true;
                    }
                } else {
                    const v3 l = normalize(d);
                    const v3 n = normalize(s.n);
                    const float r = P.refr;
                    const float c = fabsf(dot(l, n));
                    v3 refr = r * l + (r * c - sqrtf(1.0f - r * r * (1.0f - c * c))) * n;
                    refr = normalize(refr);
                    const float R0 = s.m.transp;
                    const float reflC = (float)((double)R0 + (double)(1.0f - R0) * pow((double)(1.0f - c), 5.0));
                    const float refrC = 1.0f - reflC;
                    Frame& f = fr[level];
                    f.color = col;
                    f.w = v3{reflC, refrC, 0.0f};
                    f.o2 = s.p + 0.01f * refr;
                    f.d2 = refr;
                    f.mode = FR_TRANS_A;
                    f.flag = (r * r * (1.0f - c * c) <= 1.0f);
                    o = s.p + 0.01f * refl;
                    d = refl;
                    descend = true;
                }
            }
        }
        if (descend) {
            ++level;
            continue;
        }
        v3 child = col;
        bool resumed = false;
        while (level > 0) {
            --level;
            Frame& f = fr[level];
            if (f.mode == FR_MIRROR) {
                const v3 rc = v3{0.0f, 0.0f, 0.0f} + f.w * child;
                const v3 add = f.flag ? (f.w * rc) / (float)P.glossy_n : f.w * rc;
                child = f.color + add;
            } else if (f.mode == FR_TRANS_A) {
                f.color = f.color + f.w.x * child;
                if (f.flag) {
                    f.mode = FR_TRANS_B;
                    o = f.o2;
                    d = f.d2;
                    ++level;
                    resumed = true;
                    break;
                }
                child = f.color;
            } else {
                child = f.color + f.w.y * child;
            }
        }
        if (!resumed) return child;
    }
}

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
}

// One 64-lane block renders one 8x8 pixel tile of one band.
template <bool COUNT>
__global__ __launch_bounds__(64) void render_kernel(KParams P) {
    __shared__ int stack_lds[RT_STACK_SIZE * RT_WAVE];
    const int lane = threadIdx.x;
    int* stk = stack_lds + lane;
    const int tiles_x = (P.W + 7) / 8;
    const int tiles_y_band = (P.band_rows + 7) / 8;
    const int tile = blockIdx.x;
    const int tx = tile % tiles_x;
    const int rest = tile / tiles_x;
    const int ty = rest % tiles_y_band;
    const int lb = rest / tiles_y_band;  // local band
    const int gb = lb * P.band_count + P.band_rank;
    const int row_in_band = ty * 8 + (lane >> 3);
    const int x = tx * 8 + (lane & 7);
    const int y = gb * P.band_rows + row_in_band;
    Cnt cnt{0u, 0u, 0u, 0u};
    const bool active = (x < P.W) && (row_in_band < P.band_rows) && (y < P.H) && (lb < P.n_local_bands);
    if (active) {
        const float ndx = (float)x / (float)P.W * 2.0f - 1.0f;
        const float ndy = (float)y / (float)P.H * 2.0f - 1.0f;
        v3 col;
        v3 o, d;
        if (P.aa) {
            const float sx[4] = {ndx - P.aa_offx, ndx + P.aa_offx, ndx - P.aa_offx, ndx + P.aa_offx};
            const float sy[4] = {ndy + P.aa_offy, ndy + P.aa_offy, ndy - P.aa_offy, ndy - P.aa_offy};
            v3 acc{0.0f, 0.0f, 0.0f};
            for (int i = 0; i < 4; ++i) {
                gen_ray(P, sx[i], sy[i], o, d);
                acc += get_final_color<COUNT>(P, o, d, FLT_MAX, stk, cnt);
            }
            col = acc * 0.25f;
        } else if (P.multi) {
            const float qs[4][2] = {{-1.0f, 1.0f}, {1.0f, 1.0f}, {-1.0f, -1.0f}, {1.0f, -1.0f}};
            v3 acc{0.0f, 0.0f, 0.0f};
            for (int i = 0; i < 4; ++i)
                for (int xx = 1; xx <= P.ms_moves; xx += 2)
                    for (int yy = 1; yy <= P.ms_moves; yy += 2) {
                        const float rx = ndx + (P.ms_offx * qs[i][0] * (float)xx);
                        const float ry = ndy + (P.ms_offy * qs[i][1] * (float)yy);
                        gen_ray(P, rx, ry, o, d);
                        acc += get_final_color<COUNT>(P, o, d, FLT_MAX, stk, cnt);
                    }
            col = acc * (float)(1.0f / (float)P.sample_size);
        } else {
            gen_ray(P, ndx, ndy, o, d);
            col = get_final_color<COUNT>(P, o, d, FLT_MAX, stk, cnt);
        }
        float* dst = P.out + (((size_t)lb * P.band_rows + row_in_band) * P.W + x) * 3;
        dst[0] = col.x;
        dst[1] = col.y;
        dst[2] = col.z;
    }
    flush_counters<COUNT>(P, cnt);
}

// Per-ray kernels for rt_intersect / rt_shade.
__global__ __launch_bounds__(64) void intersect_kernel(KParams P, const rt_ray* rays, int n, int use_bvh, rt_hit* hits) {
    __shared__ int stack_lds[RT_STACK_SIZE * RT_WAVE];
    const int i = blockIdx.x * 64 + threadIdx.x;
    int* stk = stack_lds + threadIdx.x;
    if (i >= n) return;
    const rt_ray r = rays[i];
    const v3 o{r.origin[0], r.origin[1], r.origin[2]};
    const v3 d{r.direction[0], r.direction[1], r.direction[2]};
    const v3 nd = normalize(d);
    Best b;
    Cnt cnt{0u, 0u, 0u, 0u};
    const bool hit = use_bvh ? traverse<true, false, false>(P.S, o, d, nd, r.t, 0.0f, b, stk, cnt)
                             : traverse<false, false, false>(P.S, o, d, nd, r.t, 0.0f, b, stk, cnt);
    rt_hit h;
    h.hit = hit ? 1 : 0;
    h.t = hit ? b.t : r.t;
    if (hit) {
        const Surf s = surface(P.S, o, d, b);
        h.normal[0] = s.n.x;
        h.normal[1] = s.n.y;
        h.normal[2] = s.n.z;
        h.hit_point[0] = s.p.x;
        h.hit_point[1] = s.p.y;
        h.hit_point[2] = s.p.z;
        h.uv[0] = s.uv.x;
        h.uv[1] = s.uv.y;
        h.material_index = s.mesh;
        h.prim_id = s.prim;
        h.is_triangle = s.is_tri ? 1 : 0;
    } else {
        for (int k = 0; k < 3; ++k) h.normal[k] = h.hit_point[k] = 0.0f;
        h.uv[0] = h.uv[1] = 0.0f;
        h.material_index = -1;
        h.prim_id = -1;
        h.is_triangle = 0;
    }
    hits[i] = h;
}

__global__ __launch_bounds__(64) void shade_kernel(KParams P, const rt_ray* rays, int n, float* rgb,
                                                   unsigned long long* ray_counts) {
    __shared__ int stack_lds[RT_STACK_SIZE * RT_WAVE];
    const int i = blockIdx.x * 64 + threadIdx.x;
    int* stk = stack_lds + threadIdx.x;
    if (i >= n) return;
    const rt_ray r = rays[i];
    Cnt cnt{0u, 0u, 0u, 0u};
    const v3 c = get_final_color<false>(P, v3{r.origin[0], r.origin[1], r.origin[2]},
                                        v3{r.direction[0], r.direction[1], r.direction[2]}, r.t, stk, cnt);
    rgb[i * 3 + 0] = c.x;
    rgb[i * 3 + 1] = c.y;
    rgb[i * 3 + 2] = c.z;
    ray_counts[i] = cnt.rays;
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

__global__ void selftest_kernel(const float* x, const float* y, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i * 4 + 0] = sqrtf(x[i]);
    out[i * 4 + 1] = 1.0f / x[i];
    out[i * 4 + 2] = x[i] / y[i];
    out[i * 4 + 3] = powf(x[i], y[i]);
}

}  // namespace rt
