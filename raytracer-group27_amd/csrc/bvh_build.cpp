// bvh_build.cpp -- RefBvh (restatement of the reference builder) and Bvh2 (binned SAH).
#include "bvh_build.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <queue>
#include <stdexcept>
#include <string>
#include <array>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>

#include <unistd.h>

namespace rt {

namespace {
// run f(i) for i in [0, n) on up to `threads` host threads: a process-wide pool of workers started
// once (scene uploads call this hundreds of times); a call made from inside a pool task runs inline
class Pool {
   public:
    static Pool& get() {
        // never destroyed (its workers may outlive static destructors); a forked child (no workers
        // of its own) starts a new one
        static Pool* p = nullptr;
        static pid_t owner = 0;
        static std::mutex m;
        std::lock_guard<std::mutex> lk(m);
        if (!p || owner != getpid()) {
            p = new Pool();
            owner = getpid();
        }
        return *p;
    }
    template <typename F>
    void run(int n, int threads, F&& f) {
        if (n <= 0) return;
        if (threads <= 1 || n == 1 || tl_in_pool) {
            for (int i = 0; i < n; ++i) f(i);
            return;
        }
        std::lock_guard<std::mutex> one(call_);  // one parallel loop at a time
        std::function<void(int)> fn = [&](int i) { f(i); };
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &fn;
            n_ = n;
            next_ = 0;
            active_ = std::min(threads, (int)workers_.size() + 1) - 1;
            done_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        tl_in_pool = true;
        for (int i = next_++; i < n; i = next_++) fn(i);  // the caller works too
        tl_in_pool = false;
        std::unique_lock<std::mutex> lk(m_);
        cv_done_.wait(lk, [&] { return done_ == active_; });
        job_ = nullptr;
    }

   private:
    Pool() {
        const unsigned hc = std::thread::hardware_concurrency();
        const int nw = (int)std::max(1u, std::min(hc == 0 ? 1u : hc, 16u)) - 1;
        for (int w = 0; w < nw; ++w) workers_.emplace_back([this, w] { loop(w); });
        for (std::thread& t : workers_) t.detach();
    }
    void loop(int w) {
        tl_in_pool = true;
        unsigned seen = 0;
        for (;;) {
            std::function<void(int)>* job;
            int n;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (w >= active_) continue;  // not needed for this loop
                job = job_;
                n = n_;
            }
            for (int i = next_++; i < n; i = next_++) (*job)(i);
            {
                std::lock_guard<std::mutex> lk(m_);
                ++done_;
            }
            cv_done_.notify_one();
        }
    }
    static thread_local bool tl_in_pool;
    std::vector<std::thread> workers_;
    std::mutex call_, m_;
    std::condition_variable cv_, cv_done_;
    std::function<void(int)>* job_ = nullptr;
    int n_ = 0, active_ = 0, done_ = 0;
    unsigned gen_ = 0;
    std::atomic<int> next_{0};
};
thread_local bool Pool::tl_in_pool = false;

template <typename F>
void parallel_for(int n, int threads, F&& f) {
    Pool::get().run(n, threads, std::forward<F>(f));
}

int host_threads() {
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc == 0 ? 1u : hc, 16u));
}

}  // namespace

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

    std::vector<float> tkey[3];  // the three triangle attributes, precomputed (same float ops)

    float sort_attr(int obj, bool is_tri, int level) const {
        const int attr = level % 3;
        if (is_tri && !tkey[attr].empty()) return tkey[attr][obj];
        if (is_tri) {
            const v3 a = vtx(obj, 0), b = vtx(obj, 1), c = vtx(obj, 2);
            if (attr == 0) return (a.x + b.x + c.x) / 3;
            if (attr == 1) return (a.y + b.y + c.y) / 3;
            return (a.z + b.z + c.z) / 3;
        }
        const float* s = sph + obj * 4;
        return attr == 0 ? s[0] : (attr == 1 ? s[1] : s[2]);
    }

    int create_node(std::vector<int>&& objs, std::vector<uint8_t>&& is_tri, int level, const v3& lo, const v3& hi) {
        RefNode n;
        n.is_leaf = (objs.size() <= 1 || level >= max_level);
        n.lower = lo;
        n.upper = hi;
        bvh.nodes.push_back(std::move(n));
        node_objs.push_back(std::move(objs));
        node_is_tri.push_back(std::move(is_tri));
        return (int)bvh.nodes.size() - 1;
    }

    // createAabbFromObjects over a node's objects (min / max: any split of the loop gives the same box)
    void aabb_par(const std::vector<int>& objs, const std::vector<uint8_t>& is_tri, v3& lo, v3& hi, int nth) const {
        const int n = (int)objs.size(), ch = 1 << 15, nch = (n + ch - 1) / ch;
        if (nch <= 1) {
            aabb(objs, is_tri, lo, hi);
            return;
        }
        std::vector<v3> clo(nch), chi(nch);
        parallel_for(nch, nth, [&](int c) {
            const int b = c * ch, e = std::min(n, b + ch);
            std::vector<int> o(objs.begin() + b, objs.begin() + e);
            std::vector<uint8_t> t(is_tri.begin() + b, is_tri.begin() + e);
            aabb(o, t, clo[c], chi[c]);
        });
        lo = splat(FLT_MAX);
        hi = splat(-FLT_MAX);
        for (int c = 0; c < nch; ++c) {
            lo = gmin(lo, clo[c]);
            hi = gmax(hi, chi[c]);
        }
    }

    // sortObjects' std::sort of (attribute, position) pairs as a stable LSD radix sort of the
    // attribute (positions start in order, so equal attributes keep it, as the pair order does;
    // -0 and +0 compare equal there and share a key here)
    static void sort_order(const std::vector<float>& key, std::vector<int>& order, int nth) {
        const int n = (int)key.size();
        std::vector<uint32_t> k(n), k2(n);
        std::vector<int> o2(n);
        order.resize(n);
        const int ch = 1 << 15, nch = std::max(1, (n + ch - 1) / ch);
        parallel_for(nch, nth, [&](int c) {
            for (int i = c * ch; i < std::min(n, (c + 1) * ch); ++i) {
                const float f = key[i] == 0.0f ? 0.0f : key[i];
                uint32_t u;
                std::memcpy(&u, &f, 4);
                k[i] = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
                order[i] = i;
            }
        });
        // stable passes: per-chunk digit counts, digit-major offsets, then each chunk scatters its
        // elements in order
        std::vector<std::array<int, 256>> cnt(nch);
        for (int shift = 0; shift < 32; shift += 8) {
            parallel_for(nch, nth, [&](int c) {
                cnt[c].fill(0);
                for (int i = c * ch; i < std::min(n, (c + 1) * ch); ++i) cnt[c][(k[i] >> shift) & 255u]++;
            });
            int run = 0;
            for (int d = 0; d < 256; ++d)
                for (int c = 0; c < nch; ++c) {
                    const int v = cnt[c][d];
                    cnt[c][d] = run;
                    run += v;
                }
            parallel_for(nch, nth, [&](int c) {
                for (int i = c * ch; i < std::min(n, (c + 1) * ch); ++i) {
                    const int d = cnt[c][(k[i] >> shift) & 255u]++;
                    k2[d] = k[i];
                    o2[d] = order[i];
                }
            });
            k.swap(k2);
            order.swap(o2);
        }
    }

    void build() {
        const int nth = host_threads();
        for (int a = 0; a < 3; ++a) tkey[a].resize(ntri);
        parallel_for((ntri + (1 << 15) - 1) >> 15, nth, [&](int c) {
            for (int t = c << 15; t < std::min(ntri, (c + 1) << 15); ++t) {
                const v3 a = vtx(t, 0), b = vtx(t, 1), cc = vtx(t, 2);
                tkey[0][t] = (a.x + b.x + cc.x) / 3;
                tkey[1][t] = (a.y + b.y + cc.y) / 3;
                tkey[2][t] = (a.z + b.z + cc.z) / 3;
            }
        });
        std::vector<int> objs;
        std::vector<uint8_t> is_tri;
        objs.reserve(ntri + nsph);
        is_tri.reserve(ntri + nsph);
        for (int i = 0; i < ntri; ++i) {
            objs.push_back(i);
            is_tri.push_back(1);
        }
        for (int i = 0; i < nsph; ++i) {
            objs.push_back(i);
            is_tri.push_back(0);
        }
        bvh.max_level_achieved = objs.empty() ? -1 : 0;
        v3 lo, hi;
        aabb_par(objs, is_tri, lo, hi, nth);
        create_node(std::move(objs), std::move(is_tri), 0, lo, hi);
        // the reference's FIFO queue, one level at a time: the nodes of a level are split in
        // parallel, then their children are created in queue order (same node numbering)
        std::vector<int> level_nodes{0};
        int level = 0;
        while (!level_nodes.empty()) {
            bvh.max_level_achieved = std::max(bvh.max_level_achieved, level);
            const int m = (int)level_nodes.size();
            struct Split {
                std::vector<int> lo_o, ro;
                std::vector<uint8_t> lo_t, rt_;
                v3 llo, lhi, rlo, rhi;
            };
            std::vector<Split> sp(m);
            const int inner_threads = std::max(1, nth / std::max(1, m));
            parallel_for(m, nth, [&](int j) {
                const int ni = level_nodes[j];
                if (bvh.nodes[ni].is_leaf) return;
                const std::vector<int>& o = node_objs[ni];
                const std::vector<uint8_t>& t = node_is_tri[ni];
                const int n = (int)o.size(), ch = 1 << 15, nch = (n + ch - 1) / ch;
                std::vector<float> key(n);
                parallel_for(nch, inner_threads, [&](int c) {
                    for (int i = c * ch; i < std::min(n, (c + 1) * ch); ++i) key[i] = sort_attr(o[i], t[i] != 0, level + 1);
                });
                std::vector<int> order;
                sort_order(key, order, inner_threads);
                const int half = (n + 1) / 2;
                Split& S = sp[j];
                S.lo_o.resize(half);
                S.lo_t.resize(half);
                S.ro.resize(n - half);
                S.rt_.resize(n - half);
                parallel_for(nch, inner_threads, [&](int c) {
                    for (int i = c * ch; i < std::min(n, (c + 1) * ch); ++i) {
                        if (i < half) {
                            S.lo_o[i] = o[order[i]];
                            S.lo_t[i] = t[order[i]];
                        } else {
                            S.ro[i - half] = o[order[i]];
                            S.rt_[i - half] = t[order[i]];
                        }
                    }
                });
                if (!S.lo_o.empty()) aabb_par(S.lo_o, S.lo_t, S.llo, S.lhi, inner_threads);
                if (!S.ro.empty()) aabb_par(S.ro, S.rt_, S.rlo, S.rhi, inner_threads);
            });
            std::vector<int> next;
            for (int j = 0; j < m; ++j) {
                const int ni = level_nodes[j];
                if (bvh.nodes[ni].is_leaf) {
                    bvh.nodes[ni].children = node_objs[ni];
                    bvh.nodes[ni].is_triangle = node_is_tri[ni];
                    continue;
                }
                Split& S = sp[j];
                if (!S.lo_o.empty()) {
                    const int c = create_node(std::move(S.lo_o), std::move(S.lo_t), level + 1, S.llo, S.lhi);
                    next.push_back(c);
                    bvh.nodes[ni].children.push_back(c);
                }
                if (!S.ro.empty()) {
                    const int c = create_node(std::move(S.ro), std::move(S.rt_), level + 1, S.rlo, S.rhi);
                    next.push_back(c);
                    bvh.nodes[ni].children.push_back(c);
                }
            }
            level_nodes.swap(next);
            ++level;
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
    std::vector<Box>* pbox;
    std::vector<v3>* cent;
    std::vector<int>* idx;
    std::vector<Bvh2Node> nodes;
    int max_leaf;
    int max_depth = 0;
    // the top of the tree is built sequentially; ranges reaching par_depth become tasks, built in
    // parallel afterwards (each range is a disjoint slice of idx, so the result does not depend on
    // the order the tasks run in)
    int par_depth = -1;
    struct Task {
        int begin, end, depth;
    };
    std::vector<Task> tasks;

    struct Desc {
        int child;
        int count;
        Box box;
    };
    static constexpr int kTaskMark = -1000000000;  // child = kTaskMark - task: filled in after the tasks
    static constexpr int kParN = 1 << 17, kParChunk = 1 << 14;

    Desc build(int begin, int end, int depth) {
        max_depth = std::max(max_depth, depth);
        const std::vector<Box>& pb = *pbox;
        const std::vector<v3>& ce = *cent;
        int* ix = idx->data();
        const int n = end - begin;
        // ranges above kParN (the top levels, before the subtree tasks) run their O(n) passes on
        // all host threads, in fixed chunks merged in order (deterministic)
        const bool par = n > kParN && par_depth > 0;
        const int nch = par ? (n + kParChunk - 1) / kParChunk : 1;
        Box box, cb;
        if (par) {
            std::vector<Box> cbox(nch), ccb(nch);
            parallel_for(nch, host_threads(), [&](int c) {
                for (int i = begin + c * kParChunk; i < std::min(end, begin + (c + 1) * kParChunk); ++i) {
                    cbox[c].grow(pb[ix[i]]);
                    ccb[c].grow(ce[ix[i]]);
                }
            });
            for (int c = 0; c < nch; ++c) {
                box.grow(cbox[c]);
                cb.grow(ccb[c]);
            }
        } else {
            for (int i = begin; i < end; ++i) {
                box.grow(pb[ix[i]]);
                cb.grow(ce[ix[i]]);
            }
        }
        if (n <= max_leaf) return Desc{begin, n, box};
        if (depth == par_depth) {
            tasks.push_back(Task{begin, end, depth});
            return Desc{kTaskMark - (int)(tasks.size() - 1), 0, box};
        }
        int axis = 0;
        const v3 ext = cb.hi - cb.lo;
        if (ext.y > ext.x) axis = 1;
        if (ext.z > (axis == 0 ? ext.x : ext.y)) axis = 2;
        float cmin = axis == 0 ? cb.lo.x : (axis == 1 ? cb.lo.y : cb.lo.z);
        float cext = axis == 0 ? ext.x : (axis == 1 ? ext.y : ext.z);
        auto cval = [&](int p) { return axis == 0 ? ce[p].x : (axis == 1 ? ce[p].y : ce[p].z); };
        int mid = -1;
        // depth guard: median splits halve the range, so switching to them once
        // depth + ceil(log2(n / max_leaf)) reaches kMaxDepth bounds the tree depth (and the
        // traversal stack, RT_STACK_SIZE) by kMaxDepth + 1.
        int need = 0;
        while ((max_leaf << need) < n) ++need;
        const bool sah_ok = depth + need < kMaxDepth;
        if (cext > 0.0f && sah_ok) {
            constexpr int NB = 32;
            // RT_SAH_AXES 3: the binned SAH over every axis with centroid extent, the cheapest split wins (ties:
            // the lower axis); 1: the axis of the largest centroid extent only (rt_build.hip does the same)
            if (RT_SAH_AXES == 3) {
                float best_all = FLT_MAX;
                int best_axis = axis;
                for (int a = 0; a < 3; ++a) {
                    const float lo_a = a == 0 ? cb.lo.x : (a == 1 ? cb.lo.y : cb.lo.z);
                    const float ext_a = a == 0 ? ext.x : (a == 1 ? ext.y : ext.z);
                    if (!(ext_a > 0.0f)) continue;
                    const float sc = NB / ext_a;
                    Box ab[NB];
                    int ac[NB] = {0};
                    auto grow_bins = [&](int i0, int i1, Box* bx, int* cn) {
                        for (int i = i0; i < i1; ++i) {
                            const int p = ix[i];
                            const float c = a == 0 ? ce[p].x : (a == 1 ? ce[p].y : ce[p].z);
                            int b = (int)((c - lo_a) * sc);
                            b = b < 0 ? 0 : (b >= NB ? NB - 1 : b);
                            bx[b].grow(pb[p]);
                            cn[b]++;
                        }
                    };
                    if (par) {
                        std::vector<std::array<Box, NB>> cbb(nch);
                        std::vector<std::array<int, NB>> cbc(nch);
                        parallel_for(nch, host_threads(), [&](int c) {
                            cbc[c].fill(0);
                            grow_bins(begin + c * kParChunk, std::min(end, begin + (c + 1) * kParChunk), cbb[c].data(),
                                      cbc[c].data());
                        });
                        for (int c = 0; c < nch; ++c)
                            for (int b = 0; b < NB; ++b) {
                                ab[b].grow(cbb[c][b]);
                                ac[b] += cbc[c][b];
                            }
                    } else {
                        grow_bins(begin, end, ab, ac);
                    }
                    Box racc, lacc;
                    float rar[NB];
                    int rcn[NB], cnt = 0, lcnt = 0;
                    for (int b = NB - 1; b > 0; --b) {
                        racc.grow(ab[b]);
                        cnt += ac[b];
                        rar[b] = racc.area();
                        rcn[b] = cnt;
                    }
                    for (int b = 1; b < NB; ++b) {
                        lacc.grow(ab[b - 1]);
                        lcnt += ac[b - 1];
                        if (lcnt == 0 || rcn[b] == 0) continue;
                        const float cost = lacc.area() * lcnt + rar[b] * rcn[b];
                        if (cost < best_all) {
                            best_all = cost;
                            best_axis = a;
                        }
                    }
                }
                axis = best_axis;
                cmin = axis == 0 ? cb.lo.x : (axis == 1 ? cb.lo.y : cb.lo.z);
                cext = axis == 0 ? ext.x : (axis == 1 ? ext.y : ext.z);
            }
            Box bb[NB];
            int bc[NB] = {0};
            const float scale = NB / cext;
            auto bin_of = [&](int p) {
                int b = (int)((cval(p) - cmin) * scale);
                return b < 0 ? 0 : (b >= NB ? NB - 1 : b);
            };
            if (par) {
                std::vector<std::array<Box, NB>> cbb(nch);
                std::vector<std::array<int, NB>> cbc(nch);
                parallel_for(nch, host_threads(), [&](int c) {
                    cbc[c].fill(0);
                    for (int i = begin + c * kParChunk; i < std::min(end, begin + (c + 1) * kParChunk); ++i) {
                        const int b = bin_of(ix[i]);
                        cbb[c][b].grow(pb[ix[i]]);
                        cbc[c][b]++;
                    }
                });
                for (int c = 0; c < nch; ++c)
                    for (int b = 0; b < NB; ++b) {
                        bb[b].grow(cbb[c][b]);
                        bc[b] += cbc[c][b];
                    }
            } else {
                for (int i = begin; i < end; ++i) {
                    const int b = bin_of(ix[i]);
                    bb[b].grow(pb[ix[i]]);
                    bc[b]++;
                }
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
            const float split_cost = RT_SAH_TRAVERSAL * box.area() + best;  // traversal cost ~ half a triangle
            if (best_b > 0 && (split_cost < leaf_cost || n > 2 * max_leaf)) {
                if (par) {  // stable two-pass partition: per-chunk counts, then scatter in chunk order
                    std::vector<int> nleft(nch + 1, 0), tmp(n);
                    parallel_for(nch, host_threads(), [&](int c) {
                        int k = 0;
                        for (int i = begin + c * kParChunk; i < std::min(end, begin + (c + 1) * kParChunk); ++i)
                            k += bin_of(ix[i]) < best_b;
                        nleft[c + 1] = k;
                    });
                    for (int c = 0; c < nch; ++c) nleft[c + 1] += nleft[c];
                    const int total_left = nleft[nch];
                    parallel_for(nch, host_threads(), [&](int c) {
                        int l = nleft[c], r = total_left + (c * kParChunk - nleft[c]);
                        for (int i = begin + c * kParChunk; i < std::min(end, begin + (c + 1) * kParChunk); ++i)
                            tmp[bin_of(ix[i]) < best_b ? l++ : r++] = ix[i];
                    });
                    std::copy(tmp.begin(), tmp.end(), ix + begin);
                    mid = begin + total_left;
                } else {
                    int* p = std::partition(ix + begin, ix + end, [&](int q) { return bin_of(q) < best_b; });
                    mid = (int)(p - ix);
                }
                if (mid == begin || mid == end) mid = -1;
            } else if (best_b > 0) {
                return Desc{begin, n, box};  // SAH prefers a leaf (n <= 2*max_leaf)
            }
        }
        if (mid < 0) {  // median split (degenerate centroids or depth guard)
            mid = begin + n / 2;
            std::nth_element(ix + begin, ix + mid, ix + end, [&](int a, int b) { return cval(a) < cval(b); });
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
    std::vector<Box> pbox(ntri);
    std::vector<v3> cent(ntri);
    std::vector<int> idx(ntri);
    const int nth = host_threads();
    const int chunk = 1 << 16;
    parallel_for((ntri + chunk - 1) / chunk, nth, [&](int c) {
        for (int t = c * chunk; t < std::min(ntri, (c + 1) * chunk); ++t) {
            Box bx;
            for (int k = 0; k < 3; ++k) bx.grow(v3{pos[t * 9 + k * 3], pos[t * 9 + k * 3 + 1], pos[t * 9 + k * 3 + 2]});
            bx.lo = bx.lo - splat(eps);
            bx.hi = bx.hi + splat(eps);
            pbox[t] = bx;
            cent[t] = (bx.lo + bx.hi) * 0.5f;
            idx[t] = t;
        }
    });
    Bvh2Node empty{};
    for (int k = 0; k < 3; ++k) {
        empty.lo0[k] = empty.lo1[k] = FLT_MAX;
        empty.hi0[k] = empty.hi1[k] = -FLT_MAX;
    }
    empty.child[0] = empty.child[1] = -1;
    empty.count[0] = empty.count[1] = 0;
    Bvh2Builder b;
    b.pbox = &pbox;
    b.cent = &cent;
    b.idx = &idx;
    b.max_leaf = max_leaf;
    if (ntri == 0) {
        b.nodes.push_back(empty);
    } else {
        // the top levels sequentially, their subtrees (about 4 per thread) in parallel
        b.par_depth = ntri >= (1 << 15) ? 1 + 8 : -1;
        b.nodes.push_back(empty);  // root slot 0
        // build children of the root directly so the root is always an inner node
        Bvh2Builder::Desc d = b.build(0, ntri, 1);
        std::vector<Bvh2Builder> sub(b.tasks.size());
        std::vector<Bvh2Builder::Desc> sub_root(b.tasks.size());
        parallel_for((int)b.tasks.size(), nth, [&](int t) {
            Bvh2Builder& s = sub[t];
            s.pbox = &pbox;
            s.cent = &cent;
            s.idx = &idx;
            s.max_leaf = max_leaf;
            sub_root[t] = s.build(b.tasks[t].begin, b.tasks[t].end, b.tasks[t].depth);
        });
        // splice: task t's nodes follow the top nodes (and the earlier tasks'), child indices shifted
        std::vector<int> base(b.tasks.size());
        int total = (int)b.nodes.size();
        for (size_t t = 0; t < sub.size(); ++t) {
            base[t] = total;
            total += (int)sub[t].nodes.size();
            b.max_depth = std::max(b.max_depth, sub[t].max_depth);
        }
        auto resolve = [&](int& child, int& count) {
            if (count == 0 && child <= Bvh2Builder::kTaskMark && child > Bvh2Builder::kTaskMark - (int)sub.size()) {
                const int t = Bvh2Builder::kTaskMark - child;
                child = sub_root[t].count > 0 ? sub_root[t].child : base[t] + sub_root[t].child;
                count = sub_root[t].count;
            }
        };
        for (Bvh2Node& nd : b.nodes)
            for (int k = 0; k < 2; ++k) resolve(nd.child[k], nd.count[k]);
        b.nodes.reserve(total);
        for (size_t t = 0; t < sub.size(); ++t)
            for (Bvh2Node nd : sub[t].nodes) {
                for (int k = 0; k < 2; ++k)
                    if (nd.count[k] == 0 && nd.child[k] >= 0) nd.child[k] += base[t];
                b.nodes.push_back(nd);
            }
        if (d.count == 0 && d.child <= Bvh2Builder::kTaskMark) resolve(d.child, d.count);
        if (d.count > 0) {
            // the whole scene is one leaf: root = {leaf, empty}
            Bvh2Builder::Desc e{-1, 0, Box{}};
            b.set_node(0, d, e);
            b.nodes[0].child[1] = -1;
        } else {
            // d.child is the index of the first pushed inner node: move it into slot 0
            b.nodes[0] = b.nodes[d.child];
            b.nodes[d.child] = empty;  // dead slot (never referenced)
        }
    }
    out.nodes = std::move(b.nodes);
    out.order = std::move(idx);
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
    return origin + plane_q(q) * scale;  // same two IEEE ops as the device decode
}
}  // namespace

void parallel_chunks(int n, int chunk, const std::function<void(int, int)>& f) {
    const int nch = (n + chunk - 1) / chunk;
    parallel_for(nch, host_threads(), [&](int c) { f(c * chunk, std::min(n, (c + 1) * chunk)); });
}

Bvh8 build_bvh8(const Bvh2& b2, int width) {
    Bvh8 out;
    if (width < 2 || width > 8) throw std::runtime_error("BVH8 width must be 2..8");
    if (b2.nodes.empty()) return out;
    struct Item {
        int node2;  // Bvh2 inner node whose subtree this BVH8 node covers
        int slot;   // BVH8 node index
        int depth;
    };
    // breadth first, one level at a time: the nodes of a level are collapsed and quantised in
    // parallel, then their inner children (contiguous, in slot order) and leaf records are numbered
    // in level order -- the layout of the sequential breadth-first walk
    struct Done {
        Child2 ch[8];
        int nch = 0, n_inner = 0, n_rec = 0;
        uint32_t w[RT_NODE_SDW];
    };
    const int nth = host_threads();
    std::vector<Item> level{{0, 0, 1}};
    out.nodes.assign(RT_NODE_SDW, 0u);
    while (!level.empty()) {
        const int m = (int)level.size();
        std::vector<Done> done(m);
        std::vector<std::string> err(m);
        parallel_for((m + 255) / 256, nth, [&](int blk) {
            for (int j = blk * 256; j < std::min(m, (blk + 1) * 256); ++j) {
                Done& D = done[j];
                std::vector<Child2> ch;
                children_of(b2, level[j].node2, ch);
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
                uint32_t* w = D.w;
                std::memset(w, 0, sizeof(D.w));
                // node box = union of the children
                float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                for (const Child2& c : ch)
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = std::min(lo[a], c.lo[a]);
                        hi[a] = std::max(hi[a], c.hi[a]);
                    }
                const int axis = slot_order(ch.data(), (int)ch.size(), lo, hi);
                int e[3];
                for (int a = 0; a < 3; ++a) {
                    std::memcpy(&w[a], &lo[a], 4);
                    const double ext = (double)hi[a] - (double)lo[a];
                    // the smallest ex >= -126 with RT_PLANE_STEPS * 2^ex >= ext (frexp's guess, then the exact test)
                    int ex = -126;
                    if (ext > 0.0) {
                        int fe = 0;
                        std::frexp(ext / RT_PLANE_STEPS, &fe);
                        ex = std::max(-126, fe - 2);
                    }
                    while (ex < 127 && std::ldexp(RT_PLANE_STEPS, ex) < ext) ++ex;
                    // the device forms 2^e * (1/d) with |1/d| <= 1e20: keep it finite
                    if (ex > 40) err[j] = "BVH8: scene extent too large to quantise";
                    e[a] = ex;
                }
                w[3] = (uint32_t)(e[0] + 127) | ((uint32_t)(e[1] + 127) << 8) | ((uint32_t)(e[2] + 127) << 16) |
                       ((uint32_t)axis << 24);
                uint32_t imask = 0, lmask = 0, counts = 0;
                uint32_t q[6][8];
                for (int sl = 0; sl < 8; ++sl)
                    for (int k = 0; k < 6; ++k) q[k][sl] = (k < 3) ? plane_max() : 0;  // empty: inverted box
                for (size_t sl = 0; sl < ch.size(); ++sl) {
                    const Child2& c = ch[sl];
                    for (int a = 0; a < 3; ++a) {
                        const float scale = std::ldexp(1.0f, e[a]);
                        long ql = (long)plane_down(((double)c.lo[a] - (double)lo[a]) / scale);
                        long qh = (long)plane_up(((double)c.hi[a] - (double)lo[a]) / scale);
                        const long qmax = (long)plane_max();
                        while (ql > 0 && decode(lo[a], e[a], (uint32_t)ql) > c.lo[a]) --ql;
                        while (qh < qmax && decode(lo[a], e[a], (uint32_t)qh) < c.hi[a]) ++qh;
                        if (decode(lo[a], e[a], (uint32_t)ql) > c.lo[a] || decode(lo[a], e[a], (uint32_t)qh) < c.hi[a])
                            err[j] = "BVH8 quantisation is not conservative";
                        q[a][sl] = (uint32_t)ql;
                        q[3 + a][sl] = (uint32_t)qh;
                    }
                    if (c.count > 0) {
                        lmask |= 1u << sl;
                        counts |= (uint32_t)c.count << (4 * sl);
                        D.n_rec += c.count;
                    } else {
                        imask |= 1u << sl;
                        D.n_inner++;
                    }
                    D.ch[sl] = c;
                }
                D.nch = (int)ch.size();
                w[6] = imask | (lmask << 8);
                w[7] = counts;
                pack_planes(w, q);
            }
        });
        for (const std::string& e : err)
            if (!e.empty()) throw std::runtime_error(e);
        // number the children and records in level order
        std::vector<int> child_base(m), tri_base(m);
        int nodes_total = (int)(out.nodes.size() / RT_NODE_SDW), rec_total = (int)out.order.size();
        for (int j = 0; j < m; ++j) {
            child_base[j] = nodes_total;
            tri_base[j] = rec_total;
            nodes_total += done[j].n_inner;
            rec_total += done[j].n_rec;
        }
        out.nodes.resize((size_t)nodes_total * RT_NODE_SDW, 0u);
        out.order.resize(rec_total);
        std::vector<Item> next;
        next.reserve(nodes_total - (int)(out.nodes.size() / RT_NODE_SDW) + m * 8);
        for (int j = 0; j < m; ++j) {
            Done& D = done[j];
            D.w[4] = (uint32_t)child_base[j];
            D.w[5] = (uint32_t)tri_base[j];
            std::memcpy(out.nodes.data() + (size_t)level[j].slot * RT_NODE_SDW, D.w, sizeof(D.w));
            out.max_depth = std::max(out.max_depth, level[j].depth);
            int rank = 0, r = tri_base[j];
            for (int sl = 0; sl < D.nch; ++sl) {
                const Child2& c = D.ch[sl];
                if (c.count > 0) {
                    for (int k = c.child; k < c.child + c.count; ++k) out.order[r++] = b2.order[k];
                } else {
                    next.push_back({c.child, child_base[j] + rank++, level[j].depth + 1});
                }
            }
        }
        level.swap(next);
    }
    return out;
}

}  // namespace rt
