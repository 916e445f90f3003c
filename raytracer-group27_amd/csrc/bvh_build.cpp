// bvh_build.cpp -- RefBvh (restatement of the reference builder) and Bvh2 (binned SAH).
#include "bvh_build.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <queue>
#include <stdexcept>
#include <utility>

namespace rt {

// ---------------------------------------------------------------------------------------------
// Reference BVH: constructBVH / createNodeAndUpdateStats / createNodeFromObjects /
// createAabbFromObjects / sortObjects (src/bounding_volume_hierarchy.cpp:108-366)
// ---------------------------------------------------------------------------------------------
namespace {
struct RefBuild {
    const float* pos;
    int ntri;
    const float* sph;
    int nsph;
    int max_level;
    RefBvh bvh;
    std::vector<std::vector<int>> node_objs;
    std::vector<std::vector<uint8_t>> node_is_tri;

    v3 vtx(int t, int c) const { return v3{pos[t * 9 + c * 3 + 0], pos[t * 9 + c * 3 + 1], pos[t * 9 + c * 3 + 2]}; }

    void aabb(const std::vector<int>& objs, const std::vector<uint8_t>& is_tri, v3& lo, v3& hi) const {
        lo = splat(FLT_MAX);
        hi = splat(-FLT_MAX);
        for (size_t i = 0; i < objs.size(); ++i) {
            if (is_tri[i]) {
                const v3 a = vtx(objs[i], 0), b = vtx(objs[i], 1), c = vtx(objs[i], 2);
                lo = gmin(gmin(lo, a), gmin(b, c));
                hi = gmax(gmax(hi, a), gmax(b, c));
            } else {
                const float* s = sph + objs[i] * 4;
                const v3 cen{s[0], s[1], s[2]};
                const v3 smin = cen - splat(s[3]);
                const v3 smax = cen + splat(s[3]);
                lo = gmin(lo, gmin(smin, smax));
                hi = gmax(hi, gmax(smin, smax));
            }
        }
    }

    float sort_attr(int obj, bool is_tri, int level) const {
        const int attr = level % 3;
        if (is_tri) {
            const v3 a = vtx(obj, 0), b = vtx(obj, 1), c = vtx(obj, 2);
            if (attr == 0) return (a.x + b.x + c.x) / 3;
            if (attr == 1) return (a.y + b.y + c.y) / 3;
            return (a.z + b.z + c.z) / 3;
        }
        const float* s = sph + obj * 4;
        return attr == 0 ? s[0] : (attr == 1 ? s[1] : s[2]);
    }

    int create_node(std::vector<int>&& objs, std::vector<uint8_t>&& is_tri, int level) {
        RefNode n;
        n.is_leaf = (objs.size() <= 1 || level >= max_level);
        aabb(objs, is_tri, n.lower, n.upper);
        bvh.nodes.push_back(std::move(n));
        node_objs.push_back(std::move(objs));
        node_is_tri.push_back(std::move(is_tri));
        return (int)bvh.nodes.size() - 1;
    }

    void build() {
        std::vector<int> objs;
        std::vector<uint8_t> is_tri;
        for (int i = 0; i < ntri; ++i) {
            objs.push_back(i);
            is_tri.push_back(1);
        }
        for (int i = 0; i < nsph; ++i) {
            objs.push_back(i);
            is_tri.push_back(0);
        }
        bvh.max_level_achieved = objs.empty() ? -1 : 0;
        if (!objs.empty()) bvh.max_level_achieved = 0;
        std::queue<std::pair<int, int>> q;
        create_node(std::move(objs), std::move(is_tri), 0);
        q.push({0, 0});
        while (!q.empty()) {
            const int ni = q.front().first;
            int level = q.front().second;
            q.pop();
            bvh.max_level_achieved = std::max(bvh.max_level_achieved, level);
            std::vector<int> o = node_objs[ni];
            std::vector<uint8_t> t = node_is_tri[ni];
            if (bvh.nodes[ni].is_leaf) {
                bvh.nodes[ni].children = o;
                bvh.nodes[ni].is_triangle = t;
                continue;
            }
            ++level;
            // sortObjects: std::sort of (attribute, position) pairs
            std::vector<std::pair<float, int>> ai;
            ai.reserve(o.size());
            for (size_t i = 0; i < o.size(); ++i) ai.push_back({sort_attr(o[i], t[i] != 0, level), (int)i});
            std::sort(ai.begin(), ai.end());
            std::vector<int> so(o.size());
            std::vector<uint8_t> st(o.size());
            for (size_t i = 0; i < o.size(); ++i) {
                so[i] = o[ai[i].second];
                st[i] = t[ai[i].second];
            }
            const size_t half = (so.size() + 1) / 2;
            std::vector<int> lo(so.begin(), so.begin() + half), ro(so.begin() + half, so.end());
            std::vector<uint8_t> lt(st.begin(), st.begin() + half), rt_(st.begin() + half, st.end());
            if (!lo.empty()) {
                const int c = create_node(std::move(lo), std::move(lt), level);
                q.push({c, level});
                bvh.nodes[ni].children.push_back(c);
            }
            if (!ro.empty()) {
                const int c = create_node(std::move(ro), std::move(rt_), level);
                q.push({c, level});
                bvh.nodes[ni].children.push_back(c);
            }
        }
    }

    // intersectBVH visit order (src/bounding_volume_hierarchy.cpp:414-448): depth first,
    // children in stored order, leaf objects in stored order.
    void derive() {
        bvh.leaf_id_of_node.assign(bvh.nodes.size(), -1);
        bvh.tri_key.assign(ntri, -1);
        bvh.tri_leaf.assign(ntri, -1);
        bvh.sph_key.assign(nsph, -1);
        bvh.sph_leaf.assign(nsph, -1);
        int key = 0;
        std::vector<int> path;
        std::vector<std::pair<int, int>> st;  // (node, state)
        dfs(0, key, path);
    }
    void dfs(int ni, int& key, std::vector<int>& path) {
        path.push_back(ni);
        const RefNode& n = bvh.nodes[ni];
        if (n.is_leaf) {
            const int lid = (int)bvh.leaf_nodes.size();
            bvh.leaf_nodes.push_back(ni);
            bvh.leaf_id_of_node[ni] = lid;
            bvh.leaf_path.push_back(path);
            for (size_t i = 0; i < n.children.size(); ++i) {
                if (n.is_triangle[i]) {
                    bvh.tri_key[n.children[i]] = key++;
                    bvh.tri_leaf[n.children[i]] = lid;
                } else {
                    bvh.sph_key[n.children[i]] = key++;
                    bvh.sph_leaf[n.children[i]] = lid;
                }
            }
        } else {
            for (int c : n.children) dfs(c, key, path);
        }
        path.pop_back();
    }
};
}  // namespace

RefBvh build_ref_bvh(const float* positions, int ntri, const float* sph, int nsph, int max_level) {
    RefBuild b{positions, ntri, sph, nsph, max_level, {}, {}, {}};
    b.build();
    b.derive();
    if ((int)b.bvh.leaf_nodes.size() > 32) throw std::runtime_error("reference BVH has more than 32 leaves");
    return std::move(b.bvh);
}

// ---------------------------------------------------------------------------------------------
// Binned SAH BVH2
// ---------------------------------------------------------------------------------------------
namespace {
struct Box {
    v3 lo{FLT_MAX, FLT_MAX, FLT_MAX}, hi{-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const Box& b) {
        lo = v3{std::min(lo.x, b.lo.x), std::min(lo.y, b.lo.y), std::min(lo.z, b.lo.z)};
        hi = v3{std::max(hi.x, b.hi.x), std::max(hi.y, b.hi.y), std::max(hi.z, b.hi.z)};
    }
    void grow(v3 p) {
        lo = v3{std::min(lo.x, p.x), std::min(lo.y, p.y), std::min(lo.z, p.z)};
        hi = v3{std::max(hi.x, p.x), std::max(hi.y, p.y), std::max(hi.z, p.z)};
    }
    float area() const {
        if (hi.x < lo.x) return 0.0f;
        const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

constexpr int kMaxDepth = 36;

struct Bvh2Builder {
    std::vector<Box> pbox;
    std::vector<v3> cent;
    std::vector<int> idx;
    std::vector<Bvh2Node> nodes;
    int max_leaf;
    int max_depth = 0;

    struct Desc {
        int child;
        int count;
        Box box;
    };

    Desc build(int begin, int end, int depth) {
        max_depth = std::max(max_depth, depth);
        Box box, cb;
        for (int i = begin; i < end; ++i) {
            box.grow(pbox[idx[i]]);
            cb.grow(cent[idx[i]]);
        }
        const int n = end - begin;
        if (n <= max_leaf) return Desc{begin, n, box};
        int axis = 0;
        const v3 ext = cb.hi - cb.lo;
        if (ext.y > ext.x) axis = 1;
        if (ext.z > (axis == 0 ? ext.x : ext.y)) axis = 2;
        const float cmin = axis == 0 ? cb.lo.x : (axis == 1 ? cb.lo.y : cb.lo.z);
        const float cext = axis == 0 ? ext.x : (axis == 1 ? ext.y : ext.z);
        auto cval = [&](int p) { return axis == 0 ? cent[p].x : (axis == 1 ? cent[p].y : cent[p].z); };
        int mid = -1;
        // depth guard: median splits halve the range, so switching to them once
        // depth + ceil(log2(n / max_leaf)) reaches kMaxDepth bounds the tree depth (and the
        // traversal stack, RT_STACK_SIZE) by kMaxDepth + 1.
        int need = 0;
        while ((max_leaf << need) < n) ++need;
        const bool sah_ok = depth + need < kMaxDepth;
        if (cext > 0.0f && sah_ok) {
            constexpr int NB = 32;
            Box bb[NB];
            int bc[NB] = {0};
            const float scale = NB / cext;
            auto bin_of = [&](int p) {
                int b = (int)((cval(p) - cmin) * scale);
                return b < 0 ? 0 : (b >= NB ? NB - 1 : b);
            };
            for (int i = begin; i < end; ++i) {
                const int b = bin_of(idx[i]);
                bb[b].grow(pbox[idx[i]]);
                bc[b]++;
            }
            float rarea[NB];
            int rcnt[NB];
            Box acc;
            int cnt = 0;
            for (int b = NB - 1; b > 0; --b) {
                acc.grow(bb[b]);
                cnt += bc[b];
                rarea[b] = acc.area();
                rcnt[b] = cnt;
            }
            Box lacc;
            int lcnt = 0;
            float best = FLT_MAX;
            int best_b = -1;
            for (int b = 1; b < NB; ++b) {
                lacc.grow(bb[b - 1]);
                lcnt += bc[b - 1];
                if (lcnt == 0 || rcnt[b] == 0) continue;
                const float cost = lacc.area() * lcnt + rarea[b] * rcnt[b];
                if (cost < best) {
                    best = cost;
                    best_b = b;
                }
            }
            const float leaf_cost = box.area() * n;
            const float split_cost = 0.5f * box.area() + best;  // traversal cost ~ half a triangle
            if (best_b > 0 && (split_cost < leaf_cost || n > 2 * max_leaf)) {
                int* p = std::partition(idx.data() + begin, idx.data() + end,
                                        [&](int q) { return bin_of(q) < best_b; });
                mid = (int)(p - idx.data());
                if (mid == begin || mid == end) mid = -1;
            } else if (best_b > 0) {
                return Desc{begin, n, box};  // SAH prefers a leaf (n <= 2*max_leaf)
            }
        }
        if (mid < 0) {  // median split (degenerate centroids or depth guard)
            mid = begin + n / 2;
            std::nth_element(idx.data() + begin, idx.data() + mid, idx.data() + end,
                             [&](int a, int b) { return cval(a) < cval(b); });
        }
        const int ni = (int)nodes.size();
        nodes.push_back(Bvh2Node{});
        const Desc l = build(begin, mid, depth + 1);
        const Desc r = build(mid, end, depth + 1);
        set_node(ni, l, r);
        return Desc{ni, 0, box};
    }

    void set_node(int ni, const Desc& l, const Desc& r) {
        Bvh2Node& nd = nodes[ni];
        const Desc* d[2] = {&l, &r};
        for (int k = 0; k < 2; ++k) {
            float* lo = k == 0 ? nd.lo0 : nd.lo1;
            float* hi = k == 0 ? nd.hi0 : nd.hi1;
            lo[0] = d[k]->box.lo.x;
            lo[1] = d[k]->box.lo.y;
            lo[2] = d[k]->box.lo.z;
            hi[0] = d[k]->box.hi.x;
            hi[1] = d[k]->box.hi.y;
            hi[2] = d[k]->box.hi.z;
            nd.child[k] = d[k]->child;
            nd.count[k] = d[k]->count;
        }
    }
};
}  // namespace

Bvh2 build_bvh2(const float* pos, int ntri, float eps, int max_leaf) {
    Bvh2 out;
    out.eps = eps;
    Bvh2Builder b;
    b.max_leaf = max_leaf;
    b.pbox.resize(ntri);
    b.cent.resize(ntri);
    b.idx.resize(ntri);
    for (int t = 0; t < ntri; ++t) {
        Box bx;
        for (int c = 0; c < 3; ++c) bx.grow(v3{pos[t * 9 + c * 3], pos[t * 9 + c * 3 + 1], pos[t * 9 + c * 3 + 2]});
        bx.lo = bx.lo - splat(eps);
        bx.hi = bx.hi + splat(eps);
        b.pbox[t] = bx;
        b.cent[t] = (bx.lo + bx.hi) * 0.5f;
        b.idx[t] = t;
    }
    Bvh2Node empty{};
    for (int k = 0; k < 3; ++k) {
        empty.lo0[k] = empty.lo1[k] = FLT_MAX;
        empty.hi0[k] = empty.hi1[k] = -FLT_MAX;
    }
    empty.child[0] = empty.child[1] = -1;
    empty.count[0] = empty.count[1] = 0;
    if (ntri == 0) {
        b.nodes.push_back(empty);
    } else {
        b.nodes.push_back(empty);  // root slot 0
        // build children of the root directly so the root is always an inner node
        Bvh2Builder::Desc d = b.build(0, ntri, 1);
        if (d.count > 0) {
            // the whole scene is one leaf: root = {leaf, empty}
            Bvh2Builder::Desc e{-1, 0, Box{}};
            b.set_node(0, d, e);
            b.nodes[0].child[1] = -1;
        } else {
            // d.child is the index of the first pushed inner node (1): move it into slot 0
            b.nodes[0] = b.nodes[d.child];
            b.nodes[d.child] = empty;  // dead slot (never referenced)
        }
    }
    out.nodes = std::move(b.nodes);
    out.order = std::move(b.idx);
    out.max_depth = b.max_depth;
    return out;
}

// ---------------------------------------------------------------------------------------------
// BVH8 collapse + conservative 16-bit quantisation
// ---------------------------------------------------------------------------------------------
namespace {
struct Child2 {
    float lo[3], hi[3];
    int child, count;  // Bvh2 descriptor: count > 0 leaf range in b2.order, else inner node index
};

static float area_of(const Child2& c) {
    const float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

static void children_of(const Bvh2& b2, int node, std::vector<Child2>& out) {
    const Bvh2Node& n = b2.nodes[node];
    for (int k = 0; k < 2; ++k) {
        if (n.child[k] < 0 && n.count[k] == 0) continue;  // empty slot
        Child2 c;
        const float* lo = k == 0 ? n.lo0 : n.lo1;
        const float* hi = k == 0 ? n.hi0 : n.hi1;
        for (int a = 0; a < 3; ++a) {
            c.lo[a] = lo[a];
            c.hi[a] = hi[a];
        }
        c.child = n.child[k];
        c.count = n.count[k];
        out.push_back(c);
    }
}

static float decode(float origin, int e, uint32_t q) {
    const float scale = std::ldexp(1.0f, e);
    return origin + (float)q * scale;  // same two IEEE ops as the device decode
}
}  // namespace

Bvh8 build_bvh8(const Bvh2& b2, int width) {
    Bvh8 out;
    if (width < 2 || width > 8) throw std::runtime_error("BVH8 width must be 2..8");
    if (b2.nodes.empty()) return out;
    struct Item {
        int node2;  // Bvh2 inner node whose subtree this BVH8 node covers
        int slot;   // BVH8 node index
        int depth;
    };
    std::vector<Item> queue;
    queue.push_back({0, 0, 1});
    out.nodes.assign(32, 0u);
    size_t head = 0;
    while (head < queue.size()) {
        const Item it = queue[head++];
        out.max_depth = std::max(out.max_depth, it.depth);
        std::vector<Child2> ch;
        children_of(b2, it.node2, ch);
        // greedy collapse: open the inner child with the largest surface area until `width` children
        for (;;) {
            if ((int)ch.size() >= width) break;
            int best = -1;
            float best_a = -1.0f;
            for (size_t i = 0; i < ch.size(); ++i)
                if (ch[i].count == 0 && area_of(ch[i]) > best_a) {
                    best_a = area_of(ch[i]);
                    best = (int)i;
                }
            if (best < 0) break;
            std::vector<Child2> sub;
            children_of(b2, ch[best].child, sub);
            if ((int)(ch.size() - 1 + sub.size()) > width) break;
            ch.erase(ch.begin() + best);
            ch.insert(ch.end(), sub.begin(), sub.end());
        }
        uint32_t* w = out.nodes.data() + (size_t)it.slot * 32;
        // node box = union of the children
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (const Child2& c : ch)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], c.lo[a]);
                hi[a] = std::max(hi[a], c.hi[a]);
            }
        int e[3];
        for (int a = 0; a < 3; ++a) {
            std::memcpy(&w[a], &lo[a], 4);
            const double ext = (double)hi[a] - (double)lo[a];
            int ex = -126;
            while (ex < 127 && std::ldexp(65000.0, ex) < ext) ++ex;
            // the device forms 2^e * (1/d) with |1/d| <= 1e20: keep it finite
            if (ex > 40) throw std::runtime_error("BVH8: scene extent too large to quantise");
            e[a] = ex;
        }
        w[3] = (uint32_t)(e[0] + 127) | ((uint32_t)(e[1] + 127) << 8) | ((uint32_t)(e[2] + 127) << 16);
        uint32_t imask = 0, lmask = 0, counts = 0;
        const int child_base = (int)(out.nodes.size() / 32);
        const int tri_base = (int)out.order.size();
        w[4] = (uint32_t)child_base;
        w[5] = (uint32_t)tri_base;
        int n_inner = 0;
        uint16_t q[6][8];
        for (int s = 0; s < 8; ++s)
            for (int k = 0; k < 6; ++k) q[k][s] = (k < 3) ? 65535 : 0;  // empty: inverted box
        for (size_t s = 0; s < ch.size(); ++s) {
            const Child2& c = ch[s];
            for (int a = 0; a < 3; ++a) {
                const float scale = std::ldexp(1.0f, e[a]);
                long ql = (long)std::floor(((double)c.lo[a] - (double)lo[a]) / scale);
                long qh = (long)std::ceil(((double)c.hi[a] - (double)lo[a]) / scale);
                ql = std::max(0L, std::min(65535L, ql));
                qh = std::max(0L, std::min(65535L, qh));
                while (ql > 0 && decode(lo[a], e[a], (uint32_t)ql) > c.lo[a]) --ql;
                while (qh < 65535 && decode(lo[a], e[a], (uint32_t)qh) < c.hi[a]) ++qh;
                if (decode(lo[a], e[a], (uint32_t)ql) > c.lo[a] || decode(lo[a], e[a], (uint32_t)qh) < c.hi[a])
                    throw std::runtime_error("BVH8 quantisation is not conservative");
                q[a][s] = (uint16_t)ql;
                q[3 + a][s] = (uint16_t)qh;
            }
            if (c.count > 0) {
                lmask |= 1u << s;
                counts |= (uint32_t)c.count << (4 * s);
                for (int r = c.child; r < c.child + c.count; ++r) out.order.push_back(b2.order[r]);
            } else {
                imask |= 1u << s;
                n_inner++;
            }
        }
        w[6] = imask | (lmask << 8);
        w[7] = counts;
        for (int k = 0; k < 6; ++k)
            for (int s = 0; s < 8; s += 2) w[8 + k * 4 + s / 2] = (uint32_t)q[k][s] | ((uint32_t)q[k][s + 1] << 16);
        // allocate the inner children contiguously, in slot order
        out.nodes.resize(out.nodes.size() + (size_t)n_inner * 32, 0u);
        int rank = 0;
        for (size_t s = 0; s < ch.size(); ++s)
            if (ch[s].count == 0) queue.push_back({ch[s].child, child_base + rank++, it.depth + 1});
    }
    return out;
}

}  // namespace rt
