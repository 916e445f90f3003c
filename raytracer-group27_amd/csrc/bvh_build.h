// bvh_build.h -- host-side acceleration structures.
//
// 1. RefBvh: the reference's own depth-capped median BVH (src/bounding_volume_hierarchy.cpp:108-366,
//    max_level = 4 at src/bounding_volume_hierarchy.h:67).  The renderer does not traverse it for
//    speed; it is kept because shadow rays call intersect(..., useBVH=true) (src/shadow.cpp:42) and
//    the reference's slab test (src/ray_tracing.cpp:213-264) can reject boxes an exact test would
//    keep.  A candidate triangle is valid for a useBVH=true query only if every box on its leaf's
//    root path passes that slab test, and ties in t are broken by the leaf-DFS order.
// 2. Bvh2: a binned-SAH binary BVH whose node stores both children's boxes (64 B), with leaf
//    boxes inflated by `eps` so every point the reference's triangle test can accept lies inside.
#pragma once
#include <cstdint>
#include <functional>
#include <vector>

#include "rt_math.h"

namespace rt {

struct RefNode {
    v3 lower, upper;
    bool is_leaf = false;
    std::vector<int> children;          // node indices (inner) or object indices (leaf)
    std::vector<uint8_t> is_triangle;   // leaf only
};

struct RefBvh {
    std::vector<RefNode> nodes;         // BFS creation order, root = 0
    int max_level_achieved = 0;
    // derived
    std::vector<int> leaf_id_of_node;   // -1 for inner nodes
    std::vector<int> leaf_nodes;        // leaf id -> node index (leaf ids in DFS order)
    std::vector<int> tri_key;           // triangle -> DFS visit rank (tie-break order)
    std::vector<int> tri_leaf;          // triangle -> leaf id
    std::vector<int> sph_key, sph_leaf;
    std::vector<std::vector<int>> leaf_path;  // leaf id -> node indices root..leaf
};

// objects = triangles (scene order) then spheres; positions [ntri][3][3]
RefBvh build_ref_bvh(const float* positions, int ntri, const float* sph_center_radius /*[nsph][4]*/,
                     int nsph, int max_level = 4);

struct Bvh2Node {  // 64 bytes, matches the device layout
    float lo0[3], hi0[3], lo1[3], hi1[3];
    int child[2];  // leaf: first triangle record; inner: node index; -1: empty
    int count[2];  // leaf: number of records (>0); inner: 0
};
static_assert(sizeof(Bvh2Node) == 64, "Bvh2Node must be 64 bytes");

struct Bvh2 {
    std::vector<Bvh2Node> nodes;
    std::vector<int> order;  // record i -> scene triangle index
    float eps = 0.0f;
    int max_depth = 0;
};

// SAH: the cost of visiting an inner node relative to testing one triangle (both builders, bit-identical trees)
#ifndef RT_MAX_LEAF
#define RT_MAX_LEAF 2  // BVH2 leaf size bound of both builders (leaves up to 2x this where the SAH prefers them);
                       // 4 until round 4: C3 16-view batch 0.509 vs 0.475 ms/frame, C4 8.56 vs 8.05
#endif
#ifndef RT_SAH_AXES
#define RT_SAH_AXES 3  // binned SAH over every axis (3) or the largest centroid extent only (1; until round 4)
#endif
#ifndef RT_SAH_TRAVERSAL
#define RT_SAH_TRAVERSAL 0.5f
#endif
Bvh2 build_bvh2(const float* positions, int ntri, float eps, int max_leaf = RT_MAX_LEAF);

// Wide BVH collapsed from a Bvh2 (greedy: open the child with the largest area until `width`
// children, width <= 8; slots past `width` stay empty),
// 128-B nodes with 16-bit child boxes (80-B nodes with 8-bit ones: RT_PLANES_U8, pack_planes) quantised
// conservatively against the node origin:
//   dword 0-2 origin xyz (f32) | 3: (ex+127) | (ey+127)<<8 | (ez+127)<<16 (scale = 2^e)
//   4: child_base (first internal child node; internal children are contiguous in slot order)
//   5: tri_base (first record of the node's leaf children, contiguous in slot order)
//   6: internal-child mask | leaf-child mask << 8
//   7: per-slot triangle count, 4 bits per slot (0 for internal / empty slots)
//   8-31: q_lo_x[8] q_lo_y[8] q_lo_z[8] q_hi_x[8] q_hi_y[8] q_hi_z[8] as uint16 (RT_PLANES_U8: 8-19, as uint8)
// decoded bound = origin + float(q) * 2^e, verified on the host to contain the child box.
struct Bvh8 {
    std::vector<uint32_t> nodes;  // RT_NODE_DW dwords per node
    std::vector<int> order;       // record i -> scene triangle index
    int max_depth = 0;
};

Bvh8 build_bvh8(const Bvh2& b2, int width = 8);

// f(begin, end) over [0, n) in chunks of `chunk`, on the host's threads (scene upload loops)
void parallel_chunks(int n, int chunk, const std::function<void(int, int)>& f);

#ifndef RT_PLANES_U8
#define RT_PLANES_U8 0  // BVH8 child planes: 8-bit integer steps in 80-B nodes (1) or 16-bit words in 128-B nodes (0)
#endif
#ifndef RT_PLANES_F16
#define RT_PLANES_F16 1  // 16-bit planes: IEEE half offsets (1) or 16-bit integers (0; until round 4)
#endif
// dwords per BVH8 node: the 8-dword header, then the six planes of the 8 slots (1 or 2 bytes each)
#define RT_NODE_DW (RT_PLANES_U8 ? 20 : 32)
#define RT_NODE_F4 (RT_NODE_DW / 4)
// the node stride in dwords: RT_NODE_PAD keeps 80-B nodes on 128-B lines (5 loads, one line per node)
#ifndef RT_NODE_PAD
#define RT_NODE_PAD 0
#endif
#define RT_NODE_SDW ((RT_PLANES_U8 && RT_NODE_PAD) ? 32 : RT_NODE_DW)
#define RT_NODE_SF4 (RT_NODE_SDW / 4)
// the exponent rule's step budget: the smallest e with RT_PLANE_STEPS * 2^e >= the node's extent on the axis
#define RT_PLANE_STEPS (RT_PLANES_U8 ? 255.0 : 65000.0)

// BVH8 child planes (both builders, every traversal): a plane of axis a is origin[a] + q * 2^e[a] with q an 8-bit
// integer (RT_PLANES_U8), or a 16-bit word -- an IEEE binary16 value (RT_PLANES_F16: the traversal's slab distance is
// one v_fma_mix_f32 per plane, the half widened inside the fma) or an unsigned integer.  plane_q is q's value;
// plane_max the largest word.
RT_HD float plane_q(uint32_t q) {
    if (RT_PLANES_U8 || !RT_PLANES_F16) return (float)q;
    const uint32_t m = q & 0x3FFu, ex = (q >> 10) & 0x1Fu;  // non-negative finite halves only (q <= 0x7BFF)
    return ex == 0 ? (float)m * 5.9604644775390625e-08f : ldexpf(1.0f + (float)m * 0.0009765625f, (int)ex - 15);
}
RT_HD uint32_t plane_max() { return RT_PLANES_U8 ? 255u : RT_PLANES_F16 ? 0x7BFFu : 65535u; }
// the plane words into node dwords 8.. : plane k (lo x, y, z, hi x, y, z) of slot sl at byte sl of the plane's
// 8 bytes (U8: dwords 8 + 2k, 9 + 2k) or at half-word sl of its 16 bytes (dwords 8 + 4k .. 11 + 4k)
RT_HD void pack_planes(uint32_t* w, const uint32_t (&q)[6][8]) {
    for (int k = 0; k < 6; ++k) {
        if (RT_PLANES_U8) {
            for (int h = 0; h < 2; ++h)
                w[8 + 2 * k + h] = q[k][4 * h] | (q[k][4 * h + 1] << 8) | (q[k][4 * h + 2] << 16) | (q[k][4 * h + 3] << 24);
        } else {
            for (int sl = 0; sl < 8; sl += 2) w[8 + k * 4 + sl / 2] = q[k][sl] | (q[k][sl + 1] << 16);
        }
    }
}
// the largest word whose value is <= x (x >= 0), and the smallest whose value is >= x: the conservative rounding
// of a child's lo / hi plane (values grow with the word, so a binary search over the words)
RT_HD uint32_t plane_down(double x) {
    uint32_t lo = 0, hi = plane_max();
    if (!(x > 0.0)) return 0;
    if ((double)plane_q(hi) <= x) return hi;
    while (lo < hi) {  // invariant: value(lo) <= x < value(hi + 1)
        const uint32_t mid = (lo + hi + 1) >> 1;
        if ((double)plane_q(mid) <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
RT_HD uint32_t plane_up(double x) {
    uint32_t lo = 0, hi = plane_max();
    if (!(x > 0.0)) return 0;
    if ((double)plane_q(hi) < x) return hi;
    while (lo < hi) {  // the first word with value >= x
        const uint32_t mid = (lo + hi) >> 1;
        if ((double)plane_q(mid) >= x) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// BVH8 slot order, one rule for both builders (bvh_build.cpp build_bvh8, rt_build.hip k_collapse): the
// inner children first, sorted by the centre of their boxes (lo + hi) along the node's longest axis
// (stable), then the leaves in collapse order.  With the inner children in the low slots a child's node
// index is child_base + slot, so a traversal can take the next child of a stacked group without reading
// the parent node again, and the axis (returned; node word 3, bits 24-25) lets it take a group's children
// front to back along the ray's direction.  Slot order never changes a result, only the work.
template <class C>
RT_HD int slot_order(C* ch, int n, const float lo[3], const float hi[3]) {
    int axis = 0;
    float ext = hi[0] - lo[0];
    for (int a = 1; a < 3; ++a)
        if (hi[a] - lo[a] > ext) {
            ext = hi[a] - lo[a];
            axis = a;
        }
    for (int i = 1; i < n; ++i) {  // insertion sort (n <= 8), stable
        const C x = ch[i];
        const bool xl = x.count > 0;
        const float xc = x.lo[axis] + x.hi[axis];
        int j = i - 1;
        while (j >= 0) {
            const bool yl = ch[j].count > 0;
            const float yc = ch[j].lo[axis] + ch[j].hi[axis];
            if (!((!xl && yl) || (!xl && !yl && xc < yc))) break;
            ch[j + 1] = ch[j];
            --j;
        }
        ch[j + 1] = x;
    }
    return axis;
}

}  // namespace rt
