// rt_build.hip -- rt_create's acceleration structures built on the GPU (scenes of >= 65536
// triangles; smaller scenes and every fallback use the host builders of bvh_build.cpp):
//
//   1. the reference's depth-4 median BVH (src/bounding_volume_hierarchy.cpp:108-366): four stable
//      radix sorts of (segment, attribute) over all objects give its leaf order, from which each
//      triangle's tie-break key (depth-first visit rank) and leaf id follow;
//   2. the binned-SAH BVH2 of bvh_build.cpp (same 32-bin single-axis SAH, leaf size and depth
//      guard): ranges above kSmall triangles level by level across the whole GPU, smaller ranges as
//      whole subtrees, one wavefront each;
//   3. the greedy BVH8 collapse with conservative 16-bit quantisation, breadth first, one level per
//      pass (the layout build_bvh8 produces);
//   4. the 64-B triangle records in BVH8 leaf order (plane normal and D with the host's float ops).
//
// Everything the renderer's results depend on is identical to the host build: the reference BVH
// boxes, keys and leaf ids, and the records' plane data.  The BVH2 / BVH8 shapes may differ from the
// host's (a different partition order), which only moves work: every box is conservative and the
// winning candidate is the lexicographic minimum of (t, key) in any visit order.
#include <cstring>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cfloat>
#include <cmath>
#include <string>
#include <vector>

#include "bvh_build.h"
#include "rt_build.h"
#include "rt_math.h"

namespace rt {
namespace gb {

constexpr int NB = 32;          // SAH bins (bvh_build.cpp Bvh2Builder)
constexpr int kMaxLeaf = RT_MAX_LEAF;  // build_bvh2(..., max_leaf = RT_MAX_LEAF)
constexpr int kMaxDepth = 36;   // bvh_build.cpp kMaxDepth (median splits past the guard)
#ifndef RT_KSMALL
#define RT_KSMALL 512
#endif
constexpr int kSmall = RT_KSMALL;  // ranges up to this size are built as whole subtrees by one wave
constexpr int kChunk = 4096;    // level-synchronous phase: triangles per workgroup
constexpr int kBinW = 13;       // bin: count, box lo/hi, centroid lo/hi (ordered-uint min/max)
constexpr int kAxes = RT_SAH_AXES;         // binned axes per range (bvh_build.h)
constexpr int kTaskBins = kAxes * NB * kBinW;  // a range's bins: axis-major
constexpr int kStack = 48;      // subtree wave: pending ranges

// float <-> order-preserving uint (min/max by integer atomics)
__device__ __forceinline__ uint32_t f2o(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

struct Box6 {
    float lo[3], hi[3];
};

__device__ __forceinline__ float box_area(const float* lo, const float* hi) {
    // bvh_build.cpp Box::area (an empty box has area 0)
    if (hi[0] < lo[0]) return 0.0f;
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

// ---------------------------------------------------------------------------------------------
// per-triangle setup: eps-inflated boxes, centroids, the reference BVH's three sort attributes
// ---------------------------------------------------------------------------------------------
__global__ void k_max_abs(const float* __restrict__ pos, size_t n, uint32_t* out) {
    uint32_t m = 0u;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        m = max(m, __float_as_uint(fabsf(pos[i])));
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

__global__ void k_prim_setup(const float* __restrict__ pos, int ntri, const uint32_t* max_abs_bits, float4* bmin,
                             float4* bmax, float4* cent, float* attr) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntri) return;
    const float eps = ldexpf(fmaxf(8.0f, __uint_as_float(*max_abs_bits)), -16);
    const float* p = pos + (size_t)t * 9;
    const v3 a{p[0], p[1], p[2]}, b{p[3], p[4], p[5]}, c{p[6], p[7], p[8]};
    // Box::grow from (FLT_MAX, -FLT_MAX) over the three vertices, then -/+ eps
    v3 lo{FLT_MAX, FLT_MAX, FLT_MAX}, hi{-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (const v3& v : {a, b, c}) {
        lo = v3{fminf(lo.x, v.x), fminf(lo.y, v.y), fminf(lo.z, v.z)};
        hi = v3{fmaxf(hi.x, v.x), fmaxf(hi.y, v.y), fmaxf(hi.z, v.z)};
    }
    lo = lo - splat(eps);
    hi = hi + splat(eps);
    const v3 ce = (lo + hi) * 0.5f;
    bmin[t] = make_float4(lo.x, lo.y, lo.z, 0.0f);
    bmax[t] = make_float4(hi.x, hi.y, hi.z, 0.0f);
    cent[t] = make_float4(ce.x, ce.y, ce.z, 0.0f);
    // RefBuild::build's tkey (same float ops)
    attr[t] = (a.x + b.x + c.x) / 3;
    attr[(size_t)ntri + t] = (a.y + b.y + c.y) / 3;
    attr[2 * (size_t)ntri + t] = (a.z + b.z + c.z) / 3;
}

// ---------------------------------------------------------------------------------------------
// exclusive prefix sums (1024 per block, block totals scanned recursively, added back) and a stable
// LSD radix sort of 64-bit keys with int values, 8 bits per pass (no library primitives: rocPRIM's
// read the environment, and the library reads none)
// ---------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const T u = __shfl_up(v, o);
        if (lane >= o) v += u;
    }
    return v;
}

template <typename T>
__global__ __launch_bounds__(1024) void k_scan_blocks(const T* __restrict__ in, int n, T* out, T* block_sum) {
    __shared__ T ws[16];
    const int i = blockIdx.x * 1024 + threadIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const T v = i < n ? in[i] : T(0);
    const T inc = wave_incl_scan(v);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    if (w == 0) {
        const T s = lane < 16 ? ws[lane] : T(0);
        const T si = wave_incl_scan(s);
        if (lane < 16) ws[lane] = si - s;  // exclusive wave offsets
        if (lane == 15) block_sum[blockIdx.x] = si;
    }
    __syncthreads();
    if (i < n) out[i] = ws[w] + inc - v;
}

template <typename T>
__global__ void k_scan_add(T* out, int n, const T* __restrict__ block_sum) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] += block_sum[i / 1024];
}

constexpr int kRadixTile = 4096;  // keys per workgroup and pass (256 threads x 16)

__global__ __launch_bounds__(256) void k_radix_hist(const unsigned long long* __restrict__ key, int n, int shift,
                                                    int nblk, uint32_t* hist) {
    __shared__ uint32_t c[256];
    c[threadIdx.x] = 0u;
    __syncthreads();
    const int b0 = blockIdx.x * kRadixTile;
    for (int i = b0 + threadIdx.x; i < min(n, b0 + kRadixTile); i += 256)
        atomicAdd(&c[(uint32_t)(key[i] >> shift) & 255u], 1u);
    __syncthreads();
    hist[threadIdx.x * nblk + blockIdx.x] = c[threadIdx.x];  // digit-major: the scan gives stable offsets
}

__global__ __launch_bounds__(256) void k_radix_scatter(const unsigned long long* __restrict__ key,
                                                       const int* __restrict__ val, int n, int shift, int nblk,
                                                       const uint32_t* __restrict__ offs, unsigned long long* key_out,
                                                       int* val_out) {
    __shared__ uint32_t base[256], wcnt[4][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    base[threadIdx.x] = offs[threadIdx.x * nblk + blockIdx.x];
    const int b0 = blockIdx.x * kRadixTile;
    for (int s0 = b0; s0 < min(n, b0 + kRadixTile); s0 += 256) {
        for (int k = 0; k < 4; ++k) wcnt[k][threadIdx.x] = 0u;
        __syncthreads();
        const int i = s0 + threadIdx.x;
        const bool valid = i < n;
        const unsigned long long k = valid ? key[i] : 0ull;
        const uint32_t d = (uint32_t)(k >> shift) & 255u;
        // lanes of this wave with the same digit (one ballot per digit bit)
        unsigned long long m = __ballot(valid);
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bl = __ballot(valid && ((d >> b) & 1u));
            m &= ((d >> b) & 1u) ? bl : ~bl;
        }
        const unsigned long long below = (1ull << lane) - 1ull;
        const uint32_t rank = (uint32_t)__popcll(m & below);
        if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(m);
        __syncthreads();
        if (valid) {
            uint32_t pos = base[d] + rank;
            for (int k2 = 0; k2 < w; ++k2) pos += wcnt[k2][d];
            key_out[pos] = k;
            val_out[pos] = val[i];
        }
        __syncthreads();
        base[threadIdx.x] += wcnt[0][threadIdx.x] + wcnt[1][threadIdx.x] + wcnt[2][threadIdx.x] + wcnt[3][threadIdx.x];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// 1. reference BVH: the objects (triangles, then spheres) of every level-L node are a contiguous
//    segment of `perm`; sortObjects' std::sort of (attribute, position) pairs within each node is a
//    stable sort by (segment, attribute); a node's children are the halves of its sorted segment
// ---------------------------------------------------------------------------------------------
struct SegBounds {
    int b[17];  // segment s of the level = [b[s], b[s + 1])
    int n;      // segments
};

__device__ __forceinline__ int seg_of(const SegBounds& sb, int i) {
    int s = 0;
    while (s + 1 < sb.n && i >= sb.b[s + 1]) ++s;
    return s;
}

__global__ void k_ref_keys(const int* __restrict__ perm, int nobj, int ntri, const float* __restrict__ attr,
                           const float* __restrict__ sph4, int a, SegBounds sb, unsigned long long* key, int* val) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nobj) return;
    const int o = perm[i];
    float f = o < ntri ? attr[(size_t)a * ntri + o] : sph4[(o - ntri) * 4 + a];
    if (f == 0.0f) f = 0.0f;  // -0 and +0 compare equal in the pair sort
    const uint32_t u = __float_as_uint(f);
    const uint32_t k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    key[i] = ((unsigned long long)seg_of(sb, i) << 32) | k;
    val[i] = o;
}

// leaf boxes (createAabbFromObjects: min / max, order-free) and the keys / leaf ids of the final order
__global__ void k_ref_leaves(const int* __restrict__ perm, int nobj, int ntri, const float* __restrict__ pos,
                             const float* __restrict__ sph4, SegBounds sb, int* tri_key, int* tri_leaf, int* sph_kl,
                             uint32_t* leaf_box) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nobj) return;
    const int o = perm[i];
    const int l = seg_of(sb, i);
    v3 lo, hi;
    if (o < ntri) {
        tri_key[o] = i;
        tri_leaf[o] = l;
        const float* p = pos + (size_t)o * 9;
        const v3 a{p[0], p[1], p[2]}, b{p[3], p[4], p[5]}, c{p[6], p[7], p[8]};
        lo = gmin(gmin(a, b), c);
        hi = gmax(gmax(a, b), c);
    } else {
        const int s = o - ntri;
        sph_kl[2 * s] = i;
        sph_kl[2 * s + 1] = l;
        const v3 cen{sph4[s * 4], sph4[s * 4 + 1], sph4[s * 4 + 2]};
        const v3 smin = cen - splat(sph4[s * 4 + 3]), smax = cen + splat(sph4[s * 4 + 3]);
        lo = gmin(smin, smax);
        hi = gmax(smin, smax);
    }
    // a wave within one leaf (all but the <= 15 at leaf boundaries) reduces first: 16 boxes take the
    // atomics of every object otherwise
    uint32_t v[6] = {f2o(lo.x), f2o(lo.y), f2o(lo.z), f2o(hi.x), f2o(hi.y), f2o(hi.z)};
    uint32_t* lb = leaf_box + l * 6;
    const int l0 = __shfl(l, 0);
    if (__ballot(true) == ~0ull && __all(l == l0)) {  // (a full wave: the shuffles read every lane)
        for (int o = 32; o > 0; o >>= 1)
            for (int k = 0; k < 6; ++k) {
                const uint32_t u = (uint32_t)__shfl_xor((int)v[k], o);
                v[k] = k < 3 ? min(v[k], u) : max(v[k], u);
            }
        if ((threadIdx.x & 63) != 0) return;
    }
    for (int k = 0; k < 6; ++k) {
        if (k < 3) atomicMin(lb + k, v[k]);
        else atomicMax(lb + k, v[k]);
    }
}

// ---------------------------------------------------------------------------------------------
// 2. BVH2, level-synchronous phase (ranges above kSmall)
// ---------------------------------------------------------------------------------------------
struct LTask {
    int begin, end, depth, node;
    float lo[3], hi[3], clo[3], chi[3];
};
struct STask {  // a range built as a whole subtree by one wave; parent: node * 2 + side to patch
    int begin, end, depth, node, parent;
    float lo[3], hi[3], clo[3], chi[3];
};
struct Split {  // per level task: the bin rule and where its left half ends
    int axis, best_b, mid, median;
    float cmin, scale;
};
struct Chunk {
    int task, begin, end, pad;
};

__device__ __forceinline__ void bin_rule(const float* clo, const float* chi, int& axis, float& cmin, float& cext,
                                         float& scale) {
    // Bvh2Builder::build: the axis of the largest centroid extent, 32 bins over it
    const float ex = chi[0] - clo[0], ey = chi[1] - clo[1], ez = chi[2] - clo[2];
    axis = 0;
    if (ey > ex) axis = 1;
    if (ez > (axis == 0 ? ex : ey)) axis = 2;
    cmin = clo[axis];
    cext = axis == 0 ? ex : (axis == 1 ? ey : ez);
    scale = cext > 0.0f ? (float)NB / cext : 0.0f;
}

// the bins of axis slot s (0 .. kAxes-1): every axis (kAxes 3), or the largest centroid extent's (kAxes 1)
__device__ __forceinline__ void axis_rule(const float* clo, const float* chi, int s, int& axis, float& cmin,
                                          float& cext, float& scale) {
    if (kAxes == 1) {
        bin_rule(clo, chi, axis, cmin, cext, scale);
        return;
    }
    axis = s;
    cmin = clo[s];
    cext = chi[s] - clo[s];
    scale = cext > 0.0f ? (float)NB / cext : 0.0f;
}

__device__ __forceinline__ int bin_of(float c, float cmin, float scale) {
    const int b = (int)((c - cmin) * scale);
    return b < 0 ? 0 : (b >= NB ? NB - 1 : b);
}

__device__ __forceinline__ float comp(const float4& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

__global__ void k_init_bins(uint32_t* bins, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * kTaskBins) return;
    const int w = i % kBinW;
    bins[i] = w == 0 ? 0u : ((w == 1 || w == 2 || w == 3 || w == 7 || w == 8 || w == 9) ? 0xFFFFFFFFu : 0u);
}

// bin layout: 0 count, 1-3 box lo, 4-6 box hi, 7-9 centroid lo, 10-12 centroid hi
__global__ __launch_bounds__(256) void k_bin(const Chunk* __restrict__ chunks, const LTask* __restrict__ tasks,
                                             const int* __restrict__ idx, const float4* __restrict__ bmin,
                                             const float4* __restrict__ bmax, const float4* __restrict__ cent,
                                             uint32_t* bins) {
    __shared__ uint32_t lb[kTaskBins];
    const Chunk ch = chunks[blockIdx.x];
    const LTask T = tasks[ch.task];
    for (int i = threadIdx.x; i < kTaskBins; i += blockDim.x) {
        const int w = i % kBinW;
        lb[i] = w == 0 ? 0u : ((w >= 1 && w <= 3) || (w >= 7 && w <= 9) ? 0xFFFFFFFFu : 0u);
    }
    __syncthreads();
    for (int s = 0; s < kAxes; ++s) {
        int axis;
        float cmin, cext, scale;
        axis_rule(T.clo, T.chi, s, axis, cmin, cext, scale);
        for (int i = ch.begin + threadIdx.x; i < ch.end; i += blockDim.x) {
            const int p = idx[i];
            const float4 c = cent[p], lo = bmin[p], hi = bmax[p];
            uint32_t* b = lb + (s * NB + bin_of(comp(c, axis), cmin, scale)) * kBinW;
            atomicAdd(b, 1u);
            atomicMin(b + 1, f2o(lo.x));
            atomicMin(b + 2, f2o(lo.y));
            atomicMin(b + 3, f2o(lo.z));
            atomicMax(b + 4, f2o(hi.x));
            atomicMax(b + 5, f2o(hi.y));
            atomicMax(b + 6, f2o(hi.z));
            atomicMin(b + 7, f2o(c.x));
            atomicMin(b + 8, f2o(c.y));
            atomicMin(b + 9, f2o(c.z));
            atomicMax(b + 10, f2o(c.x));
            atomicMax(b + 11, f2o(c.y));
            atomicMax(b + 12, f2o(c.z));
        }
    }
    __syncthreads();
    uint32_t* g = bins + (size_t)ch.task * kTaskBins;
    for (int i = threadIdx.x; i < kTaskBins; i += blockDim.x) {
        const int w = i % kBinW;
        if (w == 0) {
            if (lb[i]) atomicAdd(g + i, lb[i]);
        } else if ((w >= 1 && w <= 3) || (w >= 7 && w <= 9)) {
            atomicMin(g + i, lb[i]);
        } else {
            atomicMax(g + i, lb[i]);
        }
    }
}

// the union of bins [b0, b1): count, box, centroid box
__device__ __forceinline__ int bins_union(const uint32_t* bins, int b0, int b1, float* lo, float* hi, float* clo,
                                          float* chi) {
    uint32_t m[12];
    for (int k = 0; k < 12; ++k) m[k] = (k < 3 || (k >= 6 && k < 9)) ? 0xFFFFFFFFu : 0u;
    int n = 0;
    for (int b = b0; b < b1; ++b) {
        const uint32_t* x = bins + b * kBinW;
        if (x[0] == 0u) continue;
        n += (int)x[0];
        for (int k = 0; k < 12; ++k)
            m[k] = (k < 3 || (k >= 6 && k < 9)) ? min(m[k], x[1 + k]) : max(m[k], x[1 + k]);
    }
    for (int a = 0; a < 3; ++a) {
        lo[a] = n ? o2f(m[a]) : FLT_MAX;
        hi[a] = n ? o2f(m[3 + a]) : -FLT_MAX;
        clo[a] = n ? o2f(m[6 + a]) : FLT_MAX;
        chi[a] = n ? o2f(m[9 + a]) : -FLT_MAX;
    }
    return n;
}

__device__ __forceinline__ void write_child(Bvh2Node& nd, int k, const float* lo, const float* hi, int child, int count) {
    float* l = k == 0 ? nd.lo0 : nd.lo1;
    float* h = k == 0 ? nd.hi0 : nd.hi1;
    for (int a = 0; a < 3; ++a) {
        l[a] = lo[a];
        h[a] = hi[a];
    }
    nd.child[k] = child;
    nd.count[k] = count;
}

struct Ctrs {
    int nodes;      // BVH2 nodes allocated
    int nlarge;     // next level's large tasks
    int nsmall;     // subtree tasks
    int max_depth;
    int error;      // 1: a degenerate large range (host fallback)
};

// the SAH decision of Bvh2Builder::build for bins that hold the whole range (n > kSmall > 2 * max_leaf:
// a split is always taken); children: leaf descriptors, subtree tasks or next-level tasks
__global__ void k_split(const LTask* __restrict__ tasks, int ntask, const uint32_t* __restrict__ bins, Split* splits,
                        Bvh2Node* nodes, LTask* next, int cap_next, STask* small, int cap_small, Ctrs* ctr) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntask) return;
    const LTask T = tasks[t];
    const int n = T.end - T.begin;
    int need = 0;
    while ((kMaxLeaf << need) < n) ++need;
    // the cheapest split over the binned axes (the first axis slot, then the first bin, on equal costs)
    int axis = 0, best_b = -1, best_s = 0;
    float cmin = 0.0f, scale = 0.0f, best = FLT_MAX;
    bool any_ext = false;
    for (int s = 0; s < kAxes; ++s) {
        int ax;
        float cm, ce, sc;
        axis_rule(T.clo, T.chi, s, ax, cm, ce, sc);
        if (!(ce > 0.0f)) continue;
        any_ext = true;
        const uint32_t* bs = bins + (size_t)t * kTaskBins + s * NB * kBinW;
        float rarea[NB];
        int rcnt[NB];
        {
            float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
            int cnt = 0;
            for (int b = NB - 1; b > 0; --b) {
                const uint32_t* x = bs + b * kBinW;
                if (x[0]) {
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = fminf(lo[a], o2f(x[1 + a]));
                        hi[a] = fmaxf(hi[a], o2f(x[4 + a]));
                    }
                }
                cnt += (int)x[0];
                rarea[b] = box_area(lo, hi);
                rcnt[b] = cnt;
            }
        }
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        int lcnt = 0;
        for (int b = 1; b < NB; ++b) {
            const uint32_t* x = bs + (b - 1) * kBinW;
            if (x[0]) {
                for (int a = 0; a < 3; ++a) {
                    lo[a] = fminf(lo[a], o2f(x[1 + a]));
                    hi[a] = fmaxf(hi[a], o2f(x[4 + a]));
                }
            }
            lcnt += (int)x[0];
            if (lcnt == 0 || rcnt[b] == 0) continue;
            const float cost = box_area(lo, hi) * lcnt + rarea[b] * rcnt[b];
            if (cost < best) {
                best = cost;
                best_b = b;
                best_s = s;
                axis = ax;
                cmin = cm;
                scale = sc;
            }
        }
    }
    Split sp{axis, -1, 0, 0, cmin, scale};
    if (!any_ext || T.depth + need >= kMaxDepth) {
        ctr->error = 1;  // degenerate centroids / depth guard on a large range: the host builds it
        splits[t] = sp;
        return;
    }
    const uint32_t* bn = bins + (size_t)t * kTaskBins + best_s * NB * kBinW;  // the chosen axis's bins
    if (best_b <= 0) {
        ctr->error = 1;
        splits[t] = sp;
        return;
    }
    float Llo[3], Lhi[3], Lclo[3], Lchi[3], Rlo[3], Rhi[3], Rclo[3], Rchi[3];
    const int nl = bins_union(bn, 0, best_b, Llo, Lhi, Lclo, Lchi);
    const int nr = bins_union(bn, best_b, NB, Rlo, Rhi, Rclo, Rchi);
    sp.best_b = best_b;
    sp.mid = T.begin + nl;
    splits[t] = sp;
    atomicMax(&ctr->max_depth, T.depth + 1);
    Bvh2Node nd;
    const int cb[2] = {T.begin, sp.mid}, cn[2] = {nl, nr};
    for (int k = 0; k < 2; ++k) {
        const float* clo = k == 0 ? Llo : Rlo;
        const float* chi = k == 0 ? Lhi : Rhi;
        const float* cclo = k == 0 ? Lclo : Rclo;
        const float* cchi = k == 0 ? Lchi : Rchi;
        if (cn[k] <= kMaxLeaf) {
            write_child(nd, k, clo, chi, cb[k], cn[k]);
            continue;
        }
        const int id = atomicAdd(&ctr->nodes, 1);
        write_child(nd, k, clo, chi, id, 0);
        if (cn[k] > kSmall) {
            LTask c;
            c.begin = cb[k];
            c.end = cb[k] + cn[k];
            c.depth = T.depth + 1;
            c.node = id;
            for (int a = 0; a < 3; ++a) {
                c.lo[a] = clo[a];
                c.hi[a] = chi[a];
                c.clo[a] = cclo[a];
                c.chi[a] = cchi[a];
            }
            // capacities hold by construction (disjoint ranges of > kSmall / > kMaxLeaf triangles); an
            // overflow is reported (host fallback) instead of written past the buffer
            const int slot = atomicAdd(&ctr->nlarge, 1);
            if (slot < cap_next) next[slot] = c;
            else ctr->error = 1;
        } else {
            STask c;
            c.begin = cb[k];
            c.end = cb[k] + cn[k];
            c.depth = T.depth + 1;
            c.node = id;
            c.parent = T.node * 2 + k;
            for (int a = 0; a < 3; ++a) {
                c.lo[a] = clo[a];
                c.hi[a] = chi[a];
                c.clo[a] = cclo[a];
                c.chi[a] = cchi[a];
            }
            const int slot = atomicAdd(&ctr->nsmall, 1);
            if (slot < cap_small) small[slot] = c;
            else ctr->error = 1;
        }
    }
    nodes[T.node] = nd;
}

__global__ __launch_bounds__(256) void k_part_count(const Chunk* __restrict__ chunks, const Split* __restrict__ splits,
                                                    const int* __restrict__ idx, const float4* __restrict__ cent,
                                                    int* nleft) {
    __shared__ int s;
    const Chunk ch = chunks[blockIdx.x];
    const Split sp = splits[ch.task];
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    int k = 0;
    for (int i = ch.begin + threadIdx.x; i < ch.end; i += blockDim.x)
        k += bin_of(comp(cent[idx[i]], sp.axis), sp.cmin, sp.scale) < sp.best_b;
    for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s, k);
    __syncthreads();
    if (threadIdx.x == 0) nleft[blockIdx.x] = s;
}

// per task, in chunk order: the left elements before each chunk (chunks of a task are consecutive)
__global__ void k_part_scan(const Chunk* __restrict__ chunks, int nchunks, int* nleft) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int run = 0, task = -1;
    for (int c = 0; c < nchunks; ++c) {
        if (chunks[c].task != task) {
            task = chunks[c].task;
            run = 0;
        }
        const int v = nleft[c];
        nleft[c] = run;
        run += v;
    }
}

// stable partition: each chunk's left elements go after the task's earlier chunks' left elements,
// its right elements after mid in the same order
__global__ __launch_bounds__(256) void k_part_scatter(const Chunk* __restrict__ chunks, const LTask* __restrict__ tasks,
                                                      const Split* __restrict__ splits, const int* __restrict__ nleft,
                                                      const int* __restrict__ idx, const float4* __restrict__ cent,
                                                      int* idx2) {
    __shared__ int wl[4], base_l, base_r;
    const Chunk ch = chunks[blockIdx.x];
    const Split sp = splits[ch.task];
    const LTask T = tasks[ch.task];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        base_l = T.begin + nleft[blockIdx.x];
        base_r = sp.mid + (ch.begin - T.begin - nleft[blockIdx.x]);
    }
    __syncthreads();
    for (int i0 = ch.begin; i0 < ch.end; i0 += 256) {
        const int i = i0 + threadIdx.x;
        const bool valid = i < ch.end;
        const int p = valid ? idx[i] : 0;
        const bool left = valid && bin_of(comp(cent[p], sp.axis), sp.cmin, sp.scale) < sp.best_b;
        const unsigned long long bl = __ballot(left), bv = __ballot(valid);
        if (lane == 0) wl[w] = __popcll(bl) | (__popcll(bv) << 16);
        __syncthreads();
        int pl = 0, pv = 0;
        for (int k = 0; k < w; ++k) {
            pl += wl[k] & 0xFFFF;
            pv += wl[k] >> 16;
        }
        int tl = 0, tv = 0;
        for (int k = 0; k < 4; ++k) {
            tl += wl[k] & 0xFFFF;
            tv += wl[k] >> 16;
        }
        const unsigned long long below = (1ull << lane) - 1ull;
        if (valid) {
            const int rl = pl + __popcll(bl & below);
            const int rv = pv + __popcll(bv & below);
            if (left) idx2[base_l + rl] = p;
            else idx2[base_r + (rv - rl)] = p;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            base_l += tl;
            base_r += tv - tl;
        }
        __syncthreads();
    }
}

__global__ void k_copy_chunks(const Chunk* __restrict__ chunks, const int* __restrict__ src, int* dst) {
    const Chunk ch = chunks[blockIdx.x];
    for (int i = ch.begin + threadIdx.x; i < ch.end; i += blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------------------------------------
// 2b. BVH2 subtrees: one wave per range (<= kSmall triangles), depth first with a stack in LDS;
//     each node: 32 bins in LDS, the SAH over them in 31 lanes, a stable in-wave partition
// ---------------------------------------------------------------------------------------------
// orders a wave's LDS accesses across lanes (the subtree waves of a block run independently, so no
// block barrier): a wavefront-scope fence for the compiler and the hardware, then the wave barrier
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

struct SEntry {
    int begin, end, depth, node, parent;
    float lo[3], hi[3], clo[3], chi[3];
};

__device__ __forceinline__ void wave_box(const int* idx, int b, int e, const float4* bmin, const float4* bmax,
                                         const float4* cent, float* lo, float* hi, float* clo, float* chi) {
    const int lane = threadIdx.x & 63;
    float l[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, h[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    float cl[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, chh[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = b + lane; i < e; i += 64) {
        const int p = idx[i];
        const float4 x = bmin[p], y = bmax[p], c = cent[p];
        l[0] = fminf(l[0], x.x), l[1] = fminf(l[1], x.y), l[2] = fminf(l[2], x.z);
        h[0] = fmaxf(h[0], y.x), h[1] = fmaxf(h[1], y.y), h[2] = fmaxf(h[2], y.z);
        cl[0] = fminf(cl[0], c.x), cl[1] = fminf(cl[1], c.y), cl[2] = fminf(cl[2], c.z);
        chh[0] = fmaxf(chh[0], c.x), chh[1] = fmaxf(chh[1], c.y), chh[2] = fmaxf(chh[2], c.z);
    }
    for (int o = 32; o > 0; o >>= 1)
        for (int a = 0; a < 3; ++a) {
            l[a] = fminf(l[a], __shfl_xor(l[a], o));
            h[a] = fmaxf(h[a], __shfl_xor(h[a], o));
            cl[a] = fminf(cl[a], __shfl_xor(cl[a], o));
            chh[a] = fmaxf(chh[a], __shfl_xor(chh[a], o));
        }
    for (int a = 0; a < 3; ++a) {
        lo[a] = l[a];
        hi[a] = h[a];
        clo[a] = cl[a];
        chi[a] = chh[a];
    }
}

__global__ __launch_bounds__(256) void k_subtrees(const STask* __restrict__ tasks, int ntask, int* idx, int* idx2,
                                                  const float4* __restrict__ bmin, const float4* __restrict__ bmax,
                                                  const float4* __restrict__ cent, Bvh2Node* nodes, Ctrs* ctr) {
    __shared__ uint32_t bins_s[4][kTaskBins];
    __shared__ SEntry stack_s[4][kStack];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + w;
    if (t >= ntask) return;
    uint32_t* bins = bins_s[w];
    SEntry* stk = stack_s[w];
    int sp = 0;
    if (lane == 0) {
        const STask T = tasks[t];
        SEntry e;
        e.begin = T.begin;
        e.end = T.end;
        e.depth = T.depth;
        e.node = T.node;
        e.parent = T.parent;
        for (int a = 0; a < 3; ++a) {
            e.lo[a] = T.lo[a];
            e.hi[a] = T.hi[a];
            e.clo[a] = T.clo[a];
            e.chi[a] = T.chi[a];
        }
        stk[0] = e;
    }
    sp = 1;
    int maxd = 0;
    wave_sync();
    while (sp > 0) {
        --sp;
        wave_sync();
        const SEntry E = stk[sp];
        wave_sync();
        const int n = E.end - E.begin;
        maxd = max(maxd, E.depth);
        int axis = 0;
        float cmin = 0.0f, scale = 0.0f;
        bool any_ext = false;
        for (int s = 0; s < kAxes; ++s) {
            int ax;
            float cm, ce, sc;
            axis_rule(E.clo, E.chi, s, ax, cm, ce, sc);
            any_ext = any_ext || ce > 0.0f;
        }
        int need = 0;
        while ((kMaxLeaf << need) < n) ++need;
        const bool sah_ok = E.depth + need < kMaxDepth;
        int mid = -1, best_b = -1;
        bool make_leaf = false;
        if (any_ext && sah_ok) {
            for (int i = lane; i < kTaskBins; i += 64) {
                const int k = i % kBinW;
                bins[i] = k == 0 ? 0u : ((k >= 1 && k <= 3) || (k >= 7 && k <= 9) ? 0xFFFFFFFFu : 0u);
            }
            wave_sync();
            for (int s = 0; s < kAxes; ++s) {
                int ax;
                float cm, ce, sc;
                axis_rule(E.clo, E.chi, s, ax, cm, ce, sc);
                for (int i = E.begin + lane; i < E.end; i += 64) {
                    const int p = idx[i];
                    const float4 c = cent[p], lo = bmin[p], hi = bmax[p];
                    uint32_t* b = bins + (s * NB + bin_of(comp(c, ax), cm, sc)) * kBinW;
                    atomicAdd(b, 1u);
                    atomicMin(b + 1, f2o(lo.x));
                    atomicMin(b + 2, f2o(lo.y));
                    atomicMin(b + 3, f2o(lo.z));
                    atomicMax(b + 4, f2o(hi.x));
                    atomicMax(b + 5, f2o(hi.y));
                    atomicMax(b + 6, f2o(hi.z));
                    atomicMin(b + 7, f2o(c.x));
                    atomicMin(b + 8, f2o(c.y));
                    atomicMin(b + 9, f2o(c.z));
                    atomicMax(b + 10, f2o(c.x));
                    atomicMax(b + 11, f2o(c.y));
                    atomicMax(b + 12, f2o(c.z));
                }
            }
            wave_sync();
            // lane b (1..31), per axis slot: the cost of splitting before bin b (Bvh2Builder's sweeps, per
            // lane); the key orders (cost, axis slot, bin): the first axis, then the first bin, on equal costs
            unsigned long long key = ~0ull;
            for (int s = 0; s < kAxes; ++s) {
                int ax;
                float cm, ce, sc;
                axis_rule(E.clo, E.chi, s, ax, cm, ce, sc);
                float cost = FLT_MAX;
                if (ce > 0.0f && lane >= 1 && lane < NB) {
                    const uint32_t* bs = bins + s * NB * kBinW;
                    float llo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, lhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                    float rlo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, rhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                    int nl = 0, nr = 0;
                    for (int b = 0; b < NB; ++b) {
                        const uint32_t* x = bs + b * kBinW;
                        if (!x[0]) continue;
                        float* lo = b < lane ? llo : rlo;
                        float* hi = b < lane ? lhi : rhi;
                        for (int a = 0; a < 3; ++a) {
                            lo[a] = fminf(lo[a], o2f(x[1 + a]));
                            hi[a] = fmaxf(hi[a], o2f(x[4 + a]));
                        }
                        (b < lane ? nl : nr) += (int)x[0];
                    }
                    if (nl > 0 && nr > 0) cost = box_area(llo, lhi) * nl + box_area(rlo, rhi) * nr;
                }
                const unsigned long long k = ((unsigned long long)__float_as_uint(cost) << 32) | (unsigned)(s * 64 + lane);
                key = k < key ? k : key;
            }
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long k2 = __shfl_xor(key, o);
                key = k2 < key ? k2 : key;
            }
            const float best = __uint_as_float((uint32_t)(key >> 32));
            best_b = best < FLT_MAX ? (int)(key & 63ull) : -1;
            const int best_s = best < FLT_MAX ? (int)((key >> 6) & 3ull) : 0;
            {
                float ce;
                axis_rule(E.clo, E.chi, best_s, axis, cmin, ce, scale);
            }
            const uint32_t* bs = bins + best_s * NB * kBinW;
            const float leaf_cost = box_area(E.lo, E.hi) * n;
            const float split_cost = RT_SAH_TRAVERSAL * box_area(E.lo, E.hi) + best;
            if (best_b > 0 && (split_cost < leaf_cost || n > 2 * kMaxLeaf)) {
                // stable partition into idx2, then back
                int nl = 0;
                for (int b = 0; b < best_b; ++b) nl += (int)bs[b * kBinW];
                int bl = E.begin, br = E.begin + nl;
                for (int i0 = E.begin; i0 < E.end; i0 += 64) {
                    const int i = i0 + lane;
                    const bool valid = i < E.end;
                    const int p = valid ? idx[i] : 0;
                    const bool left = valid && bin_of(comp(cent[p], axis), cmin, scale) < best_b;
                    const unsigned long long ml = __ballot(left), mv = __ballot(valid);
                    const unsigned long long below = (1ull << lane) - 1ull;
                    if (valid) {
                        if (left) idx2[bl + __popcll(ml & below)] = p;
                        else idx2[br + __popcll((mv & ~ml) & below)] = p;
                    }
                    bl += __popcll(ml);
                    br += __popcll(mv & ~ml);
                }
                wave_sync();
                for (int i = E.begin + lane; i < E.end; i += 64) idx[i] = idx2[i];
                mid = E.begin + nl;
                if (mid == E.begin || mid == E.end) mid = -1;
            } else if (best_b > 0) {
                make_leaf = true;  // SAH prefers a leaf (n <= 2 * max_leaf)
            }
        }
        wave_sync();
        if (make_leaf) {
            // this range becomes a leaf of its parent (its own node slot stays unreferenced)
            if (lane == 0) {
                Bvh2Node& pn = nodes[E.parent >> 1];
                const int k = E.parent & 1;
                pn.child[k] = E.begin;
                pn.count[k] = n;
            }
            continue;
        }
        if (mid < 0) mid = E.begin + n / 2;  // degenerate centroids / depth guard: halves in order
        // the two halves' boxes (exact unions of their triangles' boxes)
        float b2[2][12];
        wave_box(idx, E.begin, mid, bmin, bmax, cent, b2[0], b2[0] + 3, b2[0] + 6, b2[0] + 9);
        wave_box(idx, mid, E.end, bmin, bmax, cent, b2[1], b2[1] + 3, b2[1] + 6, b2[1] + 9);
        const int cb[2] = {E.begin, mid}, cn[2] = {mid - E.begin, E.end - mid};
        int ids[2] = {-1, -1};
        if (lane == 0) {
            for (int k = 0; k < 2; ++k)
                if (cn[k] > kMaxLeaf) ids[k] = atomicAdd(&ctr->nodes, 1);
        }
        ids[0] = __shfl(ids[0], 0);
        ids[1] = __shfl(ids[1], 0);
        if (lane == 0) {
            Bvh2Node nd;
            for (int k = 0; k < 2; ++k)
                write_child(nd, k, b2[k], b2[k] + 3, cn[k] > kMaxLeaf ? ids[k] : cb[k], cn[k] > kMaxLeaf ? 0 : cn[k]);
            nodes[E.node] = nd;
            for (int k = 1; k >= 0; --k) {
                if (cn[k] <= kMaxLeaf) continue;
                SEntry c;
                c.begin = cb[k];
                c.end = cb[k] + cn[k];
                c.depth = E.depth + 1;
                c.node = ids[k];
                c.parent = E.node * 2 + k;
                for (int a = 0; a < 3; ++a) {
                    c.lo[a] = b2[k][a];
                    c.hi[a] = b2[k][3 + a];
                    c.clo[a] = b2[k][6 + a];
                    c.chi[a] = b2[k][9 + a];
                }
                if (sp < kStack) stk[sp] = c;
                else atomicOr(&ctr->error, 2);
                ++sp;
            }
        }
        sp = __shfl(sp, 0);
        if (sp > kStack) sp = kStack;
        maxd = max(maxd, E.depth + 1);
        wave_sync();
    }
    if (lane == 0) atomicMax(&ctr->max_depth, maxd);
}

// ---------------------------------------------------------------------------------------------
// 3. BVH8 collapse (build_bvh8, one thread per node of a level)
// ---------------------------------------------------------------------------------------------
struct Child2 {
    float lo[3], hi[3];
    int child, count;
};
struct Item8 {
    int node2, slot, depth, pad;
};

__device__ __forceinline__ float area_of(const Child2& c) {
    const float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

__device__ __forceinline__ int children_of(const Bvh2Node* nodes, int node, Child2* out, int n) {
    const Bvh2Node nd = nodes[node];
    for (int k = 0; k < 2; ++k) {
        if (nd.child[k] < 0 && nd.count[k] == 0) continue;
        Child2 c;
        const float* lo = k == 0 ? nd.lo0 : nd.lo1;
        const float* hi = k == 0 ? nd.hi0 : nd.hi1;
        for (int a = 0; a < 3; ++a) {
            c.lo[a] = lo[a];
            c.hi[a] = hi[a];
        }
        c.child = nd.child[k];
        c.count = nd.count[k];
        out[n++] = c;
    }
    return n;
}

__device__ __forceinline__ float decode_q(float origin, int e, uint32_t q) {
    const float scale = ldexpf(1.0f, e);
    return origin + plane_q(q) * scale;
}

__global__ void k_collapse(const Item8* __restrict__ items, int m, const Bvh2Node* __restrict__ nodes2,
                           uint32_t* words, Child2* chl, unsigned long long* counts, int* err) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    Child2 ch[9];
    int nch = children_of(nodes2, items[j].node2, ch, 0);
    for (;;) {  // open the inner child with the largest area until 8 children
        if (nch >= 8) break;
        int best = -1;
        float best_a = -1.0f;
        for (int i = 0; i < nch; ++i)
            if (ch[i].count == 0 && area_of(ch[i]) > best_a) {
                best_a = area_of(ch[i]);
                best = i;
            }
        if (best < 0) break;
        Child2 sub[2];
        const int ns = children_of(nodes2, ch[best].child, sub, 0);
        if (nch - 1 + ns > 8) break;
        for (int i = best; i + 1 < nch; ++i) ch[i] = ch[i + 1];  // erase, then append in order
        --nch;
        for (int i = 0; i < ns; ++i) ch[nch++] = sub[i];
    }
    uint32_t* w = words + (size_t)j * RT_NODE_SDW;
    uint32_t wl[RT_NODE_SDW];
    for (int k = 0; k < RT_NODE_SDW; ++k) wl[k] = 0u;
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = 0; i < nch; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], ch[i].lo[a]);
            hi[a] = fmaxf(hi[a], ch[i].hi[a]);
        }
    const int axis = slot_order(ch, nch, lo, hi);
    int e[3];
    for (int a = 0; a < 3; ++a) {
        wl[a] = __float_as_uint(lo[a]);
        const double ext = (double)hi[a] - (double)lo[a];
        int ex = -126;
        if (ext > 0.0) {
            int fe = 0;
            frexp(ext / RT_PLANE_STEPS, &fe);
            ex = max(-126, fe - 2);
        }
        while (ex < 127 && ldexp(RT_PLANE_STEPS, ex) < ext) ++ex;
        if (ex > 40) atomicOr(err, 4);
        e[a] = ex;
    }
    wl[3] = (uint32_t)(e[0] + 127) | ((uint32_t)(e[1] + 127) << 8) | ((uint32_t)(e[2] + 127) << 16) |
            ((uint32_t)axis << 24);
    uint32_t imask = 0, lmask = 0, cnts = 0;
    uint32_t q[6][8];
    for (int sl = 0; sl < 8; ++sl)
        for (int k = 0; k < 6; ++k) q[k][sl] = (k < 3) ? plane_max() : 0u;
    int n_inner = 0, n_rec = 0;
    for (int sl = 0; sl < nch; ++sl) {
        const Child2& c = ch[sl];
        for (int a = 0; a < 3; ++a) {
            const float scale = ldexpf(1.0f, e[a]);
            long long ql = (long long)plane_down(((double)c.lo[a] - (double)lo[a]) / scale);
            long long qh = (long long)plane_up(((double)c.hi[a] - (double)lo[a]) / scale);
            const long long qmax = (long long)plane_max();
            while (ql > 0 && decode_q(lo[a], e[a], (uint32_t)ql) > c.lo[a]) --ql;
            while (qh < qmax && decode_q(lo[a], e[a], (uint32_t)qh) < c.hi[a]) ++qh;
            if (decode_q(lo[a], e[a], (uint32_t)ql) > c.lo[a] || decode_q(lo[a], e[a], (uint32_t)qh) < c.hi[a])
                atomicOr(err, 8);
            q[a][sl] = (uint32_t)ql;
            q[3 + a][sl] = (uint32_t)qh;
        }
        if (c.count > 0) {
            lmask |= 1u << sl;
            cnts |= (uint32_t)c.count << (4 * sl);
            n_rec += c.count;
        } else {
            imask |= 1u << sl;
            n_inner++;
        }
        chl[(size_t)j * 8 + sl] = c;
    }
    wl[6] = imask | (lmask << 8);
    wl[7] = cnts;
    pack_planes(wl, q);
    for (int k = 0; k < RT_NODE_SDW; ++k) w[k] = wl[k];
    counts[j] = ((unsigned long long)n_inner << 32) | (unsigned)n_rec;
}

// child / record numbering of a level (scan = exclusive prefix of counts): node words into place,
// the next level's items, the records' scene triangles
__global__ void k_emit(const Item8* __restrict__ items, int m, const uint32_t* __restrict__ words,
                       const Child2* __restrict__ chl, const unsigned long long* __restrict__ counts,
                       const unsigned long long* __restrict__ scan, int nodes_total, int rec_total, uint32_t* nodes8,
                       Item8* next, const int* __restrict__ idx, int* order8) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const Item8 it = items[j];
    const int child_base = nodes_total + (int)(scan[j] >> 32);
    const int tri_base = rec_total + (int)(scan[j] & 0xFFFFFFFFull);
    const uint32_t* w = words + (size_t)j * RT_NODE_SDW;
    uint32_t* o = nodes8 + (size_t)it.slot * RT_NODE_SDW;
    for (int k = 0; k < RT_NODE_SDW; ++k) o[k] = w[k];
    o[4] = (uint32_t)child_base;
    o[5] = (uint32_t)tri_base;
    const uint32_t masks = w[6];
    int ni = 0, nr = 0;
    for (int sl = 0; sl < 8; ++sl) {
        const uint32_t bit = 1u << sl;
        if (masks & bit) {
            const Child2 c = chl[(size_t)j * 8 + sl];
            next[(int)(scan[j] >> 32) + ni] = Item8{c.child, child_base + ni, it.depth + 1, 0};
            ++ni;
        } else if ((masks >> 8) & bit) {
            const Child2 c = chl[(size_t)j * 8 + sl];
            for (int r = 0; r < c.count; ++r) order8[tri_base + nr + r] = idx[c.child + r];
            nr += c.count;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// 4. triangle records (rt_create's record loop): v0|n.x, v1|n.y, v2|n.z, D|scene idx|ref key|ref leaf
// ---------------------------------------------------------------------------------------------
__global__ void k_records(const int* __restrict__ order8, int ntri, const float* __restrict__ pos,
                          const int* __restrict__ tri_key, const int* __restrict__ tri_leaf, float4* rec) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= ntri) return;
    const int t = order8[r];
    const float* p = pos + (size_t)t * 9;
    const v3 v0{p[0], p[1], p[2]}, v1{p[3], p[4], p[5]}, v2{p[6], p[7], p[8]};
    const v3 n = normalize(cross(v0 - v2, v1 - v2));  // trianglePlane (src/ray_tracing.cpp:91-100)
    const float D = dot(n, v0);
    float4* o = rec + (size_t)r * 4;
    o[0] = make_float4(v0.x, v0.y, v0.z, n.x);
    o[1] = make_float4(v1.x, v1.y, v1.z, n.y);
    o[2] = make_float4(v2.x, v2.y, v2.z, n.z);
    o[3] = make_float4(D, __int_as_float(t), __int_as_float(tri_key[t]), __int_as_float(tri_leaf[t]));
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
struct Bufs {
    std::vector<void*> all;
    template <typename T>
    T* get(size_t n) {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
        all.push_back(p);
        return static_cast<T*>(p);
    }
    ~Bufs() {
        for (void* p : all) hipFree(p);
    }
};

#define GB_CHECK(expr)                                                                        \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            err = std::string("GPU build: ") + hipGetErrorString(e_) + " at " #expr;           \
            return false;                                                                     \
        }                                                                                     \
    } while (0)
#define GB_ALLOC(ptr)                                      \
    do {                                                   \
        if (!(ptr)) {                                      \
            err = "GPU build: out of device memory";        \
            return false;                                  \
        }                                                  \
    } while (0)

static int grid(long long n, int b) { return (int)((n + b - 1) / b); }

// block totals of every recursion level of exclusive_scan
static size_t scan_tmp_size(long long n) {
    size_t t = 0;
    while (n > 1) {
        n = (n + 1023) / 1024;
        t += (size_t)n + 1;
    }
    return t + 1;
}

template <typename T>
static void exclusive_scan(const T* in, T* out, int n, T* tmp, hipStream_t st) {
    if (n <= 0) return;
    const int nb = grid(n, 1024);
    k_scan_blocks<T><<<nb, 1024, 0, st>>>(in, n, out, tmp);
    if (nb > 1) {
        exclusive_scan<T>(tmp, tmp, nb, tmp + nb + 1, st);  // (in place: each block reads before it writes)
        k_scan_add<T><<<grid(n, 256), 256, 0, st>>>(out, n, tmp);
    }
}

// stable sort of (key, val) by key bits [0, bits): LSD passes of 8 bits, ping-pong; the result ends in
// (k_out, v_out)
static void radix_sort(unsigned long long* k_in, int* v_in, unsigned long long* k_out, int* v_out,
                       unsigned long long* k_tmp, int* v_tmp, int n, int bits, uint32_t* hist, uint32_t* scan_tmp,
                       hipStream_t st) {
    const int nblk = grid(n, kRadixTile);
    const int passes = (bits + 7) / 8;
    unsigned long long* ks = k_in;
    int* vs = v_in;
    for (int p = 0; p < passes; ++p) {
        // the last pass lands in the output; earlier ones alternate so that it does
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        unsigned long long* kd = to_out ? k_out : k_tmp;
        int* vd = to_out ? v_out : v_tmp;
        k_radix_hist<<<nblk, 256, 0, st>>>(ks, n, 8 * p, nblk, hist);
        exclusive_scan<uint32_t>(hist, hist, 256 * nblk, scan_tmp, st);
        k_radix_scatter<<<nblk, 256, 0, st>>>(ks, vs, n, 8 * p, nblk, hist, kd, vd);
        ks = kd;
        vs = vd;
    }
}

static void seg_bounds(int n, int level, SegBounds& sb) {
    std::vector<std::pair<int, int>> segs{{0, n}};
    for (int l = 0; l < level; ++l) {
        std::vector<std::pair<int, int>> nx;
        for (auto s : segs) {
            const int half = (s.second - s.first + 1) / 2;
            nx.push_back({s.first, s.first + half});
            nx.push_back({s.first + half, s.second});
        }
        segs.swap(nx);
    }
    sb.n = (int)segs.size();
    for (int s = 0; s < sb.n; ++s) sb.b[s] = segs[s].first;
    sb.b[sb.n] = n;
}

}  // namespace gb

bool gpu_build(const float* h_pos, int ntri, const float* sph4, int nsph, GpuBuild& out, std::string& err) {
    using namespace gb;
    const auto t0 = std::chrono::steady_clock::now();
    auto ms_now = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
#ifdef RT_BUILD_TRACE
#define TRACE(tag) do { hipDeviceSynchronize(); fprintf(stderr, "build %-12s %7.2f ms\n", tag, ms_now()); } while (0)
#else
#define TRACE(tag) do { } while (0)
#endif
    const int nobj = ntri + nsph;
    if (ntri < 16 || nobj < 16) {
        err = "GPU build: too few objects";
        return false;
    }
    Bufs B;
    hipStream_t st = 0;
    float* pos = B.get<float>((size_t)ntri * 9);
    GB_ALLOC(pos);
    GB_CHECK(hipMemcpy(pos, h_pos, (size_t)ntri * 9 * sizeof(float), hipMemcpyHostToDevice));
    float* d_sph = B.get<float>((size_t)std::max(1, nsph) * 4);
    GB_ALLOC(d_sph);
    if (nsph) GB_CHECK(hipMemcpy(d_sph, sph4, (size_t)nsph * 4 * sizeof(float), hipMemcpyHostToDevice));
    uint32_t* maxabs = B.get<uint32_t>(1);
    float4 *bmin = B.get<float4>(ntri), *bmax = B.get<float4>(ntri), *cent = B.get<float4>(ntri);
    float* attr = B.get<float>((size_t)ntri * 3);
    GB_ALLOC(maxabs);
    GB_ALLOC(bmin);
    GB_ALLOC(bmax);
    GB_ALLOC(cent);
    GB_ALLOC(attr);
    GB_CHECK(hipMemsetAsync(maxabs, 0, 4, st));
    k_max_abs<<<1024, 256, 0, st>>>(pos, (size_t)ntri * 9, maxabs);
    TRACE("upload");
    k_prim_setup<<<grid(ntri, 256), 256, 0, st>>>(pos, ntri, maxabs, bmin, bmax, cent, attr);
    GB_CHECK(hipGetLastError());
    TRACE("setup");

    // ---- 1. reference BVH ----
    unsigned long long *k0 = B.get<unsigned long long>(nobj), *k1 = B.get<unsigned long long>(nobj);
    int *perm = B.get<int>(nobj), *v0 = B.get<int>(nobj);
    int *tri_key = B.get<int>(ntri), *tri_leaf = B.get<int>(ntri), *sph_kl = B.get<int>(2 * std::max(1, nsph));
    uint32_t* leaf_box = B.get<uint32_t>(16 * 6);
    GB_ALLOC(k0);
    GB_ALLOC(k1);
    GB_ALLOC(perm);
    GB_ALLOC(v0);
    GB_ALLOC(tri_key);
    GB_ALLOC(tri_leaf);
    GB_ALLOC(sph_kl);
    GB_ALLOC(leaf_box);
    {
        std::vector<int> iota(nobj);
        for (int i = 0; i < nobj; ++i) iota[i] = i;
        GB_CHECK(hipMemcpy(perm, iota.data(), (size_t)nobj * 4, hipMemcpyHostToDevice));
    }
    unsigned long long* k2 = B.get<unsigned long long>(nobj);
    int* v1 = B.get<int>(nobj);
    const int nblk = grid(nobj, kRadixTile);
    uint32_t* hist = B.get<uint32_t>((size_t)256 * nblk);
    uint32_t* hscan = B.get<uint32_t>(scan_tmp_size(256LL * nblk));
    GB_ALLOC(k2);
    GB_ALLOC(v1);
    GB_ALLOC(hist);
    GB_ALLOC(hscan);
    TRACE("ref alloc");
    for (int level = 0; level < 4; ++level) {  // the split levels 0..3; attribute (level + 1) % 3
        SegBounds sb;
        seg_bounds(nobj, level, sb);
        k_ref_keys<<<grid(nobj, 256), 256, 0, st>>>(perm, nobj, ntri, attr, d_sph, (level + 1) % 3, sb, k0, v0);
        // 32 attribute bits, then the segment (level <= 3: < 8 segments)
        radix_sort(k0, v0, k1, perm, k2, v1, nobj, level == 0 ? 32 : 40, hist, hscan, st);
    }
    TRACE("ref sorts");
    {
        std::vector<uint32_t> init(16 * 6);
        for (int l = 0; l < 16; ++l)
            for (int k = 0; k < 6; ++k) init[l * 6 + k] = k < 3 ? 0xFFFFFFFFu : 0u;
        GB_CHECK(hipMemcpy(leaf_box, init.data(), init.size() * 4, hipMemcpyHostToDevice));
        SegBounds sb;
        seg_bounds(nobj, 4, sb);
        k_ref_leaves<<<grid(nobj, 256), 256, 0, st>>>(perm, nobj, ntri, pos, d_sph, sb, tri_key, tri_leaf, sph_kl,
                                                     leaf_box);
        GB_CHECK(hipGetLastError());
        std::vector<uint32_t> lb(16 * 6);
        std::vector<int> skl(2 * std::max(1, nsph));
        GB_CHECK(hipMemcpyAsync(lb.data(), leaf_box, lb.size() * 4, hipMemcpyDeviceToHost, st));
        GB_CHECK(hipMemcpyAsync(skl.data(), sph_kl, skl.size() * 4, hipMemcpyDeviceToHost, st));
        GB_CHECK(hipStreamSynchronize(st));
        auto dec = [](uint32_t o) {
            const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
            float f;
            std::memcpy(&f, &u, 4);
            return f;
        };
        // 31 nodes in BFS order (level k: nodes 2^k - 1 .. 2^(k+1) - 2, left to right); the leaves'
        // boxes from the device, the inner boxes as unions of their children
        RefBvh& R = out.ref;
        R.nodes.assign(31, RefNode{});
        for (int l = 0; l < 16; ++l) {
            RefNode& nd = R.nodes[15 + l];
            nd.is_leaf = true;
            nd.lower = v3{dec(lb[l * 6]), dec(lb[l * 6 + 1]), dec(lb[l * 6 + 2])};
            nd.upper = v3{dec(lb[l * 6 + 3]), dec(lb[l * 6 + 4]), dec(lb[l * 6 + 5])};
        }
        for (int i = 14; i >= 0; --i) {
            RefNode& nd = R.nodes[i];
            nd.children = {2 * i + 1, 2 * i + 2};
            nd.lower = gmin(R.nodes[2 * i + 1].lower, R.nodes[2 * i + 2].lower);
            nd.upper = gmax(R.nodes[2 * i + 1].upper, R.nodes[2 * i + 2].upper);
        }
        R.max_level_achieved = 4;
        R.leaf_id_of_node.assign(31, -1);
        R.leaf_nodes.clear();
        R.leaf_path.clear();
        for (int l = 0; l < 16; ++l) {
            R.leaf_id_of_node[15 + l] = l;
            R.leaf_nodes.push_back(15 + l);
            std::vector<int> path;
            for (int k = 0; k <= 4; ++k) path.push_back((1 << k) - 1 + (l >> (4 - k)));
            R.leaf_path.push_back(path);
        }
        R.sph_key.resize(nsph);
        R.sph_leaf.resize(nsph);
        for (int s = 0; s < nsph; ++s) {
            R.sph_key[s] = skl[2 * s];
            R.sph_leaf[s] = skl[2 * s + 1];
        }
    }
    out.ms[0] = ms_now();  // + positions upload, triangle setup, reference BVH

    // ---- 2. BVH2 ----
    int *idx = B.get<int>(ntri), *idx2 = B.get<int>(ntri);
    const int cap_nodes = 2 * ntri + 16;
    Bvh2Node* nodes2 = B.get<Bvh2Node>(cap_nodes);
    Ctrs* ctr = B.get<Ctrs>(1);
    GB_ALLOC(idx);
    GB_ALLOC(idx2);
    GB_ALLOC(nodes2);
    GB_ALLOC(ctr);
    {
        std::vector<int> iota(ntri);
        for (int i = 0; i < ntri; ++i) iota[i] = i;
        GB_CHECK(hipMemcpy(idx, iota.data(), (size_t)ntri * 4, hipMemcpyHostToDevice));
        GB_CHECK(hipMemsetAsync(nodes2, 0xFF, sizeof(Bvh2Node) * (size_t)cap_nodes, st));
        Ctrs c0{1, 0, 0, 1, 0};
        GB_CHECK(hipMemcpy(ctr, &c0, sizeof(Ctrs), hipMemcpyHostToDevice));
    }
    // root: its box and centroid box (one range, a level of its own)
    const int max_tasks = ntri / kSmall + 16, max_small = ntri / kMaxLeaf + 16;
    LTask *lt = B.get<LTask>(max_tasks), *lt_next = B.get<LTask>(max_tasks);
    STask* small = B.get<STask>(max_small);
    Split* splits = B.get<Split>(max_tasks);
    uint32_t* bins = B.get<uint32_t>((size_t)max_tasks * kTaskBins);
    const int max_chunks = ntri / kChunk + max_tasks + 16;
    Chunk* d_chunks = B.get<Chunk>(max_chunks);
    int* nleft = B.get<int>(max_chunks);
    GB_ALLOC(lt);
    GB_ALLOC(lt_next);
    GB_ALLOC(small);
    GB_ALLOC(splits);
    GB_ALLOC(bins);
    GB_ALLOC(d_chunks);
    GB_ALLOC(nleft);
    {
        // the root's boxes: a one-task "level" whose bins are the whole range (any axis works for the
        // union), then the real root task with its centroid box
        LTask r{};
        r.begin = 0;
        r.end = ntri;
        r.depth = 1;
        r.node = 0;
        for (int a = 0; a < 3; ++a) {
            r.lo[a] = r.clo[a] = 0.0f;
            r.hi[a] = r.chi[a] = 0.0f;  // zero extent: every triangle in bin 0
        }
        std::vector<Chunk> chunks;
        for (int b = 0; b < ntri; b += kChunk) chunks.push_back(Chunk{0, b, std::min(ntri, b + kChunk), 0});
        GB_CHECK(hipMemcpy(lt, &r, sizeof(LTask), hipMemcpyHostToDevice));
        GB_CHECK(hipMemcpy(d_chunks, chunks.data(), chunks.size() * sizeof(Chunk), hipMemcpyHostToDevice));
        k_init_bins<<<grid(kTaskBins, 256), 256, 0, st>>>(bins, 1);
        k_bin<<<(int)chunks.size(), 256, 0, st>>>(d_chunks, lt, idx, bmin, bmax, cent, bins);
        std::vector<uint32_t> hb(NB * kBinW);
        GB_CHECK(hipMemcpyAsync(hb.data(), bins, hb.size() * 4, hipMemcpyDeviceToHost, st));
        GB_CHECK(hipStreamSynchronize(st));
        auto dec = [](uint32_t o) {
            const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
            float f;
            std::memcpy(&f, &u, 4);
            return f;
        };
        const uint32_t* x = hb.data();  // bin 0 holds everything
        for (int a = 0; a < 3; ++a) {
            r.lo[a] = dec(x[1 + a]);
            r.hi[a] = dec(x[4 + a]);
            r.clo[a] = dec(x[7 + a]);
            r.chi[a] = dec(x[10 + a]);
        }
        GB_CHECK(hipMemcpy(lt, &r, sizeof(LTask), hipMemcpyHostToDevice));
    }
    TRACE("bvh2 root");
    int nlevel = 1;
    std::vector<LTask> htasks;
    while (nlevel > 0) {
        htasks.resize(nlevel);
        GB_CHECK(hipMemcpyAsync(htasks.data(), lt, nlevel * sizeof(LTask), hipMemcpyDeviceToHost, st));
        GB_CHECK(hipStreamSynchronize(st));
        std::vector<Chunk> chunks;
        for (int t = 0; t < nlevel; ++t)
            for (int b = htasks[t].begin; b < htasks[t].end; b += kChunk)
                chunks.push_back(Chunk{t, b, std::min(htasks[t].end, b + kChunk), 0});
        if ((int)chunks.size() > max_chunks) {
            err = "GPU build: chunk list overflow";
            return false;
        }
        const int nc = (int)chunks.size();
        GB_CHECK(hipMemcpy(d_chunks, chunks.data(), nc * sizeof(Chunk), hipMemcpyHostToDevice));
        GB_CHECK(hipMemsetAsync(&ctr->nlarge, 0, sizeof(int), st));
        k_init_bins<<<grid((long long)nlevel * kTaskBins, 256), 256, 0, st>>>(bins, nlevel);
        k_bin<<<nc, 256, 0, st>>>(d_chunks, lt, idx, bmin, bmax, cent, bins);
        k_split<<<grid(nlevel, 64), 64, 0, st>>>(lt, nlevel, bins, splits, nodes2, lt_next, max_tasks, small, max_small,
                                                 ctr);
        k_part_count<<<nc, 256, 0, st>>>(d_chunks, splits, idx, cent, nleft);
        k_part_scan<<<1, 1, 0, st>>>(d_chunks, nc, nleft);
        k_part_scatter<<<nc, 256, 0, st>>>(d_chunks, lt, splits, nleft, idx, cent, idx2);
        k_copy_chunks<<<nc, 256, 0, st>>>(d_chunks, idx2, idx);
        GB_CHECK(hipGetLastError());
        Ctrs hc;
        GB_CHECK(hipMemcpyAsync(&hc, ctr, sizeof(Ctrs), hipMemcpyDeviceToHost, st));
        GB_CHECK(hipStreamSynchronize(st));
        if (hc.error) {
            err = "GPU build: degenerate large range";
            return false;
        }
        nlevel = hc.nlarge;
        if (nlevel > max_tasks) {
            err = "GPU build: task list overflow";
            return false;
        }
        std::swap(lt, lt_next);
    }
    Ctrs hc;
    GB_CHECK(hipMemcpyAsync(&hc, ctr, sizeof(Ctrs), hipMemcpyDeviceToHost, st));
    GB_CHECK(hipStreamSynchronize(st));
    TRACE("bvh2 levels");
    if (hc.error || hc.nsmall > max_small) {
        err = "GPU build: subtree task list overflow";
        return false;
    }
    if (hc.nsmall > 0) k_subtrees<<<grid(hc.nsmall, 4), 256, 0, st>>>(small, hc.nsmall, idx, idx2, bmin, bmax, cent,
                                                                      nodes2, ctr);
    GB_CHECK(hipGetLastError());
    GB_CHECK(hipMemcpyAsync(&hc, ctr, sizeof(Ctrs), hipMemcpyDeviceToHost, st));
    GB_CHECK(hipStreamSynchronize(st));
    if (hc.error || hc.nodes > cap_nodes) {
        err = "GPU build: subtree stack or node overflow";
        return false;
    }

    out.ms[1] = ms_now();  // + BVH2
    // ---- 3. BVH8 collapse, breadth first ----
    const int cap8 = hc.nodes + 1;
    uint32_t* nodes8 = B.get<uint32_t>((size_t)cap8 * RT_NODE_SDW);
    int* order8 = B.get<int>(ntri);
    Item8 *items = B.get<Item8>(cap8), *items_next = B.get<Item8>(cap8);
    uint32_t* words = B.get<uint32_t>((size_t)cap8 * RT_NODE_SDW);
    Child2* chl = B.get<Child2>((size_t)cap8 * 8);
    unsigned long long *cnt = B.get<unsigned long long>(cap8), *scan = B.get<unsigned long long>(cap8);
    int* d_err = B.get<int>(1);
    GB_ALLOC(nodes8);
    GB_ALLOC(order8);
    GB_ALLOC(items);
    GB_ALLOC(items_next);
    GB_ALLOC(words);
    GB_ALLOC(chl);
    GB_ALLOC(cnt);
    GB_ALLOC(scan);
    GB_ALLOC(d_err);
    GB_CHECK(hipMemsetAsync(d_err, 0, 4, st));
    {
        Item8 root{0, 0, 1, 0};
        GB_CHECK(hipMemcpy(items, &root, sizeof(Item8), hipMemcpyHostToDevice));
    }
    unsigned long long* scan_tmp = B.get<unsigned long long>(scan_tmp_size(cap8));
    GB_ALLOC(scan_tmp);
    int m = 1, nodes_total = 1, rec_total = 0, depth8 = 1;
    while (m > 0) {
        k_collapse<<<grid(m, 64), 64, 0, st>>>(items, m, nodes2, words, chl, cnt, d_err);
        exclusive_scan(cnt, scan, m, scan_tmp, st);
        k_emit<<<grid(m, 64), 64, 0, st>>>(items, m, words, chl, cnt, scan, nodes_total, rec_total, nodes8, items_next,
                                           idx, order8);
        GB_CHECK(hipGetLastError());
        unsigned long long last[2];
        GB_CHECK(hipMemcpyAsync(&last[0], scan + (m - 1), 8, hipMemcpyDeviceToHost, st));
        GB_CHECK(hipMemcpyAsync(&last[1], cnt + (m - 1), 8, hipMemcpyDeviceToHost, st));
        GB_CHECK(hipStreamSynchronize(st));
        const unsigned long long tot = last[0] + last[1];
        const int n_inner = (int)(tot >> 32), n_rec = (int)(tot & 0xFFFFFFFFull);
        nodes_total += n_inner;
        rec_total += n_rec;
        if (nodes_total > cap8) {
            err = "GPU build: BVH8 node overflow";
            return false;
        }
        if (n_inner > 0) ++depth8;
        m = n_inner;
        std::swap(items, items_next);
    }
    int herr = 0;
    GB_CHECK(hipMemcpy(&herr, d_err, 4, hipMemcpyDeviceToHost));
    if (herr) {
        err = "GPU build: BVH8 quantisation failed";
        return false;
    }
    if (rec_total != ntri) {
        err = "GPU build: record count mismatch";
        return false;
    }

    out.ms[2] = ms_now();  // + BVH8
    // ---- 4. records; outputs in exact-size buffers the context owns (handed over only on success:
    // every failure path below frees them) ----
    float4* rec = nullptr;
    float4* n8 = nullptr;
    GB_CHECK(hipMalloc(&rec, (size_t)ntri * 64));
    if (hipMalloc(&n8, (size_t)nodes_total * RT_NODE_SDW * 4) != hipSuccess) {
        hipFree(rec);
        err = "GPU build: out of device memory";
        return false;
    }
    k_records<<<grid(ntri, 256), 256, 0, st>>>(order8, ntri, pos, tri_key, tri_leaf, rec);
    hipError_t e = hipMemcpyAsync(n8, nodes8, (size_t)nodes_total * RT_NODE_SDW * 4, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) {
        hipFree(rec);
        hipFree(n8);
        err = std::string("GPU build: ") + hipGetErrorString(e) + " (records)";
        return false;
    }
    out.tri = rec;
    out.nodes = n8;
    out.ms[3] = ms_now();  // + records
    out.nnodes = nodes_total;
    out.max_depth = depth8;
    out.bvh2_nodes = hc.nodes;
    out.bvh2_depth = hc.max_depth;
    return true;
}

}  // namespace rt
