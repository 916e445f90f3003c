// rt_wavefront.hip -- the opaque-scene render as a wavefront of lean kernels (included by rt_runtime.hip
// after rt_megakernel.hip, whose traversal steps it reuses).
//
// Why: the persistent megakernels keep a pixel's whole getFinalColor state machine in the same wave as its
// traversal.  The state machine only runs between queries, yet its ~24 lane dwords stay live across every
// traversal step (the 4-wave opaque build spills 31 VGPRs), and a lane can only take new work when the
// whole wave stops to advance its state machine (refill 64): on the C3 batch a node step keeps 0.52 of the
// lanes busy and a record step 0.28 (profiles/r04/simd_r04w_C3.log).  Here the traversal is a kernel of
// its own that holds nothing but the query (Trav), so it fits more waves per SIMD and a lane that finishes
// its query takes the next one from the queue at once; the shading between queries is a separate, fully
// coherent elementwise kernel.  Per recursion level l (getFinalColor's `level`, src/main.cpp:129-301):
//
//   trace  T_l   the level's path rays (camera rays at l = 0, mirror rays after) -- closest hit, result per
//                ray -- and the cansee segments of the level-(l-1) shading points (src/shadow.cpp:32-69,
//                any hit: a visible segment sets its light's bit in its shading point's record)
//   shade  S_l   (a) resolve every level-(l-1) shading point: its node colour, the lights in getFinalColor's
//                order (getPointLights then getSpotLichts, src/main.cpp:174-185) whose bits are set, folded
//                into the pixel as acc = acc + w * colour -- the megakernels' forward fold, same operations
//                in the same order, so the images are bit-identical;
//                (b) shade every level-l hit (surface(), reflect): a shading-point record, one cansee
//                segment per light that needs a query (lights within SHADOW_ERROR_OFFSET count at once, spot
//                lights outside their cone not at all) and the mirror ray (ks^2-weighted child) below
//                max_reflection_level -- the queues of T_{l+1}.
//
// The pixel's colour lives in its output slot from S_0 on (0, then + w * colour per level in level order).
// Scope: the opaque kernel's scenes (all materials opaque, point and spot lights, no textures, no glossy
// lobes) with one camera sample per pixel; everything else keeps the megakernels.
namespace rt {

// per launch-sequence counters (zeroed before T_0): queue lengths and shading-point counts per level
struct WfCnt {
    int qp[RT_MAX_DEPTH + 2];     // path rays of level l (qp[0] unused: camera jobs)
    int qs[RT_MAX_DEPTH + 2];     // cansee segments traced in T_l (of level-(l-1) shading points)
    int nodes[RT_MAX_DEPTH + 2];  // shading points of level l
    int head[RT_MAX_DEPTH + 2][8 * 32];  // T_l: per-XCD queue heads, 128 B apart
};

// the buffers of one launch sequence (device pointers; capacities checked on the host)
struct WfBufs {
    WfCnt* cnt;
    int2* res;          // T_l path-ray results: (t bits, record) -- RT_NO_HIT: miss
    float4* qp[2];      // path rays of level l in qp[l & 1]: (o, level), (d, pixel), (w, 0)
    float4* qs;         // cansee segments of T_l: (o, sdist), (d, node << 5 | light)
    float4* nodes[2];   // shading points of level l in nodes[l & 1]: (hp, mat), (nN, vis), (refl, pixel), (w, 0)
    int level;          // l of this launch
    int njobs;          // camera jobs of this chunk (T_0 / S_0): the render's jobs job0 .. job0 + njobs - 1
    int job0;
    int nl;             // lights in getFinalColor's order: point lights, then spot lights
};

// the second kernel argument of the wavefront kernels (after KParams), read through the kernarg pointer
__device__ __forceinline__ const WfBufs& wf_bufs(const void* ka) {
    constexpr size_t off = (sizeof(KParams) + alignof(WfBufs) - 1) / alignof(WfBufs) * alignof(WfBufs);
    return *(const WfBufs*)(uniform_kernarg(ka) + off);
}

// light li of getFinalColor's order: its position and colour (spot lights after the point lights)
__device__ __forceinline__ void wf_light(const DevScene& S, int li, v3& lp, v3& lc) {
    if (li < S.npl) {
        const rt_point_light pl = S.pl[li];
        lp = ld3(pl.position);
        lc = ld3(pl.color);
    } else {
        const DSpot sp = S.spot[li - S.npl];
        lp = ld3(sp.pos);
        lc = ld3(sp.color);
    }
}

// ---- trace ----------------------------------------------------------------------------------------------
// Persistent: every wave walks its per-XCD range of the level's queue (path rays first, then the cansee
// segments), then the other ranges.  A lane whose query ends writes its result and takes the next query
// at the next refill (once `refill` lanes wait, or none traces); the traversal step is the opaque kernel's
// (dual record + node visit, the direct group stack in LDS, the reference BVH in LDS for the culling).
#ifndef RT_WF_WAVES
#define RT_WF_WAVES 5
#endif
#define RT_WF_CHUNK 64  // queries a wave reserves per queue-head atomic
template <bool COUNT, bool PRIMARY>
__global__ __launch_bounds__(64, RT_WF_WAVES) void wf_trace_kernel(KParams, WfBufs) {
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ int stack_lds[RT_STACK8 * RT_WAVE];
    __shared__ RefLds ref_lds;
    const int lane_id = threadIdx.x;
    int* stk = stack_lds + lane_id;
    // the level's work: n_path path rays (camera jobs at l = 0), then n_seg cansee segments
    int n_path, n_seg, level;
    {
        const WfBufs& B = wf_bufs(ka);
        level = B.level;
        n_path = PRIMARY ? B.njobs : B.cnt->qp[level];
        n_seg = PRIMARY ? 0 : B.cnt->qs[level];
    }
    const int n_all = n_path + n_seg;
    // a level with few queries runs on as many waves as give each lane one (the others leave at once: no
    // atomics on the queue heads, no reference-BVH load)
    if ((int)blockIdx.x >= ((n_all + 63) >> 6) + 8) return;
    if (RT_REF_LDS) {
        ref_lds_load(kernel_params(ka).S, ref_lds, lane_id);
        __syncthreads();
    }
    Trav T;
    trav_idle(T);
    Cnt cnt{};
    int src = -1;                // the query this lane traces: < n_path a path ray, else a segment
    uint32_t tag = 0u;           // a segment's shading point << 5 | light
    bool tracing = false, done = false;
    int xr = (int)(blockIdx.x & 7), xtried = 0;
    // the wave's reserved block of queries [nxt, end) (wave-uniform): one queue-head atomic per RT_WF_CHUNK
    int nxt = 0, end = 0;
    for (;;) {
        const KParams& P = *(const KParams*)fresh_kernarg(ka);
        const DevScene& S = P.S;
        // ---- refill: the waiting lanes take the next queries, from the wave's block, then new blocks ----
        {
            const bool idle = !tracing && !done;
            const unsigned long long want = __ballot(idle);
            const int nwant = __popcll(want);
            if (want && (nwant >= P.refill || !__any(tracing))) {
                const WfBufs& B = wf_bufs(ka);
                const int rank = __popcll(want & ((1ull << lane_id) - 1ull)), leader = __ffsll((long long)want) - 1;
                int k = -1, served = 0;
                for (;;) {  // wave-uniform
                    const int take = min(nwant - served, end - nxt);
                    if (idle && rank >= served && rank < served + take) k = nxt + (rank - served);
                    nxt += take;
                    served += take;
                    if (served == nwant || xtried >= 8) break;
                    // the next block of range xr: [xr * n_all / 8, (xr + 1) * n_all / 8)
                    const int lo = (int)(((long long)xr * n_all) >> 3), hi = (int)(((long long)(xr + 1) * n_all) >> 3);
                    int b = 0;
                    if (lane_id == leader) b = lo + atomicAdd(&B.cnt->head[level][32 * xr], RT_WF_CHUNK);
                    b = __shfl(b, leader);
                    if (b + RT_WF_CHUNK >= hi) {  // the range is used up with this block: the next one after it
                        xr = (xr + 1) & 7;
                        ++xtried;
                    }
                    nxt = min(b, hi);
                    end = min(b + RT_WF_CHUNK, hi);
                }
                if (idle) {
                    if (k >= 0) {
                        v3 o, d;
                        float t0 = FLT_MAX, sdist = 0.0f;
                        bool seg = false;
                        if (PRIMARY) {
                            uint32_t rpix;
                            int out_row;
                            if (job_pixel(P, B.job0 + k, rpix, out_row)) {
                                Query q;
                                camera_query(P, B.job0 + k, rpix, 0, q);
                                o = q.o;
                                d = q.d;
                                src = k;
                            } else {
                                src = -1;  // a padding pixel (S_0 skips it)
                            }
                        } else if (k < n_path) {
                            const float4* e = B.qp[level & 1] + (size_t)k * 3;
                            const float4 e0 = e[0], e1 = e[1];
                            o = v3{e0.x, e0.y, e0.z};
                            d = v3{e1.x, e1.y, e1.z};
                            src = k;
                        } else {
                            const float4* e = B.qs + (size_t)(k - n_path) * 2;
                            const float4 e0 = e[0], e1 = e[1];
                            o = v3{e0.x, e0.y, e0.z};
                            sdist = e0.w;
                            d = v3{e1.x, e1.y, e1.z};
                            tag = __float_as_uint(e1.w);
                            seg = true;
                            src = k;
                        }
                        if (src >= 0) {
                            cnt.rays++;
                            trav_init_q(S, P.use_bvh != 0, o, d, t0, seg, sdist, T);
                            tracing = true;
                        }
                    } else if (xtried >= 8) {
                        done = true;
                    }
                }
            }
        }
        if (!__any(tracing)) {
            if (__all(done)) break;
            continue;
        }
        // ---- one record test and / or one node visit per tracing lane ----
        if (tracing) {
            const bool rec = leaf_pending(T);
            if (rec) trav_record<COUNT, true, false, false>(S, T, cnt, nullptr, nullptr, &ref_lds);
            const bool nv = T.cur != RT_TRAV_NONE && (!rec || (P.dual && T.lh == 0u));
            if (nv) {
                float4 g[8];
                trav_node<COUNT, 8, false, true>(S, T, stk, g, cnt);
            }
            if (!leaf_pending(T) && T.cur == RT_TRAV_NONE) {
                trav_finish(S, T);
                const WfBufs& B = wf_bufs(ka);
                if (src < n_path) {
                    B.res[src] = make_int2(__float_as_int(T.best.t), T.found ? T.best.rec : RT_NO_HIT);
                } else if (!T.found) {
                    // the segment reached its light: that light's bit in its shading point's record
                    atomicOr(reinterpret_cast<unsigned int*>(B.nodes[(level - 1) & 1] + (size_t)(tag >> 5) * 4 + 1) + 3,
                             1u << (tag & 31u));
                }
                tracing = false;
                src = -1;
            }
        }
    }
    flush_counters<COUNT>(kernel_params(ka), cnt);
}

// ---- shade -----------------------------------------------------------------------------------------------
// Elementwise over (a) the level-(l-1) shading points (resolve) and (b) the level's path rays (shade hits);
// a grid-stride loop over the counts the previous kernels left on the device.
template <bool COUNT>
__global__ __launch_bounds__(256) void wf_shade_kernel(KParams, WfBufs) {
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const KParams& P = kernel_params(ka);
    const WfBufs& B = wf_bufs(ka);
    const DevScene& S = P.S;
    const int level = B.level;
    const int n_res = level > 0 ? B.cnt->nodes[level - 1] : 0;
    const int n_path = level == 0 ? B.njobs : B.cnt->qp[level];
    const int n_all = n_res + n_path;
    Cnt cnt{};
    const int lane_id = threadIdx.x & 63;
    const int stride = gridDim.x * blockDim.x;
    // every thread runs the same trip count (the wave-wide allocations below need whole waves)
    const int trips = (n_all + stride - 1) / stride;
    for (int it = 0; it < trips; ++it) {
        const int i = it * stride + blockIdx.x * blockDim.x + threadIdx.x;
        if (i < n_res) {
            // (a) resolve shading point i of level l - 1: calcColor of every visible light in getFinalColor's
            // order (lite_light_visible / lite_next_light's expressions), then acc = acc + w * colour
            const float4* nd = B.nodes[(level - 1) & 1] + (size_t)i * 4;
            const float4 n0 = nd[0], n1 = nd[1], n2 = nd[2], n3 = nd[3];
            const v3 hp{n0.x, n0.y, n0.z}, nN{n1.x, n1.y, n1.z}, refl{n2.x, n2.y, n2.z}, w{n3.x, n3.y, n3.z};
            const int mat = __float_as_int(n0.w);
            const uint32_t vis = __float_as_uint(n1.w);
            const uint32_t pix = __float_as_uint(n2.w);
            v3 color{0.0f, 0.0f, 0.0f};
            for (int li = 0; li < B.nl; ++li) {
                if (!((vis >> li) & 1u)) continue;
                v3 lp, lc;
                wf_light(S, li, lp, lc);
                const v3 ldir = normalize(lp - hp);
                const float cosL = fabsf(dot(nN, ldir));
                const float d2 = dot(normalize(refl), ldir);
                color += calc_color(lc, 1.0f, cosL, (0.0f < d2) ? d2 : 0.0f, load_mat(S, mat));
            }
            float* dst = P.out + (size_t)pix * 3;
            const v3 acc{dst[0], dst[1], dst[2]};
            const v3 r = acc + w * color;
            dst[0] = r.x;
            dst[1] = r.y;
            dst[2] = r.z;
        }
        // (b) path ray j of level l: its hit becomes a shading point
        const int j = i - n_res;
        bool hit = false;
        v3 o{0.0f, 0.0f, 0.0f}, d{0.0f, 0.0f, 0.0f}, w{1.0f, 1.0f, 1.0f};
        uint32_t pix = 0u;
        Best b{0.0f, -1, RT_NO_HIT};
        if (j >= 0 && j < n_path) {
            const int2 r = B.res[j];
            b.t = __int_as_float(r.x);
            b.rec = r.y;
            if (level == 0) {
                uint32_t rpix;
                int out_row;
                if (job_pixel(P, B.job0 + j, rpix, out_row)) {
                    pix = (uint32_t)out_row * (uint32_t)P.W + rpix % (uint32_t)P.W;
                    // the pixel's colour starts at 0 (a miss stays black: getFinalColor returns vec3(0))
                    float* dst = P.out + (size_t)pix * 3;
                    dst[0] = 0.0f;
                    dst[1] = 0.0f;
                    dst[2] = 0.0f;
                    if (b.rec != RT_NO_HIT) {
                        Query q;
                        camera_query(P, B.job0 + j, rpix, 0, q);
                        o = q.o;
                        d = q.d;
                        hit = true;
                    }
                }
            } else if (b.rec != RT_NO_HIT) {
                const float4* e = B.qp[level & 1] + (size_t)j * 3;
                const float4 e0 = e[0], e1 = e[1], e2 = e[2];
                o = v3{e0.x, e0.y, e0.z};
                d = v3{e1.x, e1.y, e1.z};
                pix = __float_as_uint(e1.w);
                w = v3{e2.x, e2.y, e2.z};
                hit = true;
            }
        }
        // the shading point's slot (wave-aggregated)
        const unsigned long long hm = __ballot(hit);
        if (!hm) continue;
        int nbase = 0;
        const int leader = __ffsll((long long)hm) - 1;
        if (lane_id == leader) nbase = atomicAdd(&B.cnt->nodes[level], __popcll(hm));
        nbase = __shfl(nbase, leader);
        const int n = nbase + __popcll(hm & ((1ull << lane_id) - 1ull));
        v3 hp{0.0f, 0.0f, 0.0f}, nN{0.0f, 0.0f, 0.0f}, refl{0.0f, 0.0f, 0.0f};
        int mat = 0;
        bool desc = false;
        if (hit) {
            // begin_node (src/main.cpp:131-256), the opaque branch: lite_advance's expressions
            const Surf s = surface(S, o, d, b, false, level == 0);
            if (COUNT) {
                cnt.hits++;
                if (s.ub) cnt.ub++;
            }
            hp = s.p;
            nN = normalize(s.n);
            refl = reflect(normalize(d), nN);
            mat = (b.rec >= 0) ? s.mesh : b.rec;
            if (level < P.max_level) {
                const v3 ks{s.m.ks[0], s.m.ks[1], s.m.ks[2]};
                if (ks.x > 0.0f || ks.y > 0.0f || ks.z > 0.0f) desc = true;
            }
        }
        // cansee segments (start_cansee) of the lights that need a query, light by light; lights within
        // SHADOW_ERROR_OFFSET are visible at once (src/shadow.cpp:38-40), spot lights outside their cone
        // contribute nothing (src/shadow.cpp:235-237)
        uint32_t vis = 0u;
        for (int li = 0; li < B.nl; ++li) {
            bool need = false;
            v3 sd{0.0f, 0.0f, 0.0f};
            float sdist = 0.0f;
            if (hit) {
                v3 lp, lc;
                wf_light(S, li, lp, lc);
                bool in = true;
                if (li >= S.npl) {
                    const DSpot sp = S.spot[li - S.npl];
                    in = dot(normalize(ld3(sp.dir)), normalize(hp - lp)) > sp.cos_angle;
                }
                if (in) {
                    sd = lp - hp;
                    sdist = length(sd);
                    sd = normalize(sd);
                    if (sdist > 0.0005f) need = true;
                    else vis |= 1u << li;
                }
            }
            const unsigned long long sm = __ballot(need);
            if (!sm) continue;
            int sbase = 0;
            const int sl = __ffsll((long long)sm) - 1;
            if (lane_id == sl) sbase = atomicAdd(&B.cnt->qs[level + 1], __popcll(sm));
            sbase = __shfl(sbase, sl);
            if (need) {
                const int k = sbase + __popcll(sm & ((1ull << lane_id) - 1ull));
                float4* e = B.qs + (size_t)k * 2;
                const v3 so = hp + 0.0005f * sd;
                e[0] = make_float4(so.x, so.y, so.z, sdist);
                e[1] = make_float4(sd.x, sd.y, sd.z, __uint_as_float(((uint32_t)n << 5) | (uint32_t)li));
            }
        }
        if (hit) {
            float4* nd = B.nodes[level & 1] + (size_t)n * 4;
            nd[0] = make_float4(hp.x, hp.y, hp.z, __int_as_float(mat));
            nd[1] = make_float4(nN.x, nN.y, nN.z, __uint_as_float(vis));
            nd[2] = make_float4(refl.x, refl.y, refl.z, __uint_as_float(pix));
            nd[3] = make_float4(w.x, w.y, w.z, 0.0f);
        }
        // the mirror child (lite_child_weight, then the child's query: origin hitPoint + 0.01 * reflect)
        const unsigned long long pm = __ballot(desc);
        if (!pm) continue;
        int pbase = 0;
        const int pl_ = __ffsll((long long)pm) - 1;
        if (lane_id == pl_) pbase = atomicAdd(&B.cnt->qp[level + 1], __popcll(pm));
        pbase = __shfl(pbase, pl_);
        if (desc) {
            const int k = pbase + __popcll(pm & ((1ull << lane_id) - 1ull));
            const DMat m = load_mat(S, mat);
            const v3 ks{m.ks[0], m.ks[1], m.ks[2]};
            const v3 wc = (m.shin != 0.0f) ? w * ((ks * ks) / (float)P.glossy_n) : w * (ks * ks);
            const v3 co = hp + 0.01f * refl;
            float4* e = B.qp[(level + 1) & 1] + (size_t)k * 3;
            e[0] = make_float4(co.x, co.y, co.z, __int_as_float(level + 1));
            e[1] = make_float4(refl.x, refl.y, refl.z, __uint_as_float(pix));
            e[2] = make_float4(wc.x, wc.y, wc.z, 0.0f);
        }
    }
    if (COUNT) {
        // hits and UB-regime hits of the shaded points (rt_stats.hits / ub_hits)
        unsigned long long h = cnt.hits, u = cnt.ub;
        for (int off = 32; off > 0; off >>= 1) {
            h += __shfl_xor(h, off);
            u += __shfl_xor(u, off);
        }
        if (lane_id == 0) {
            atomicAdd(P.stats + 3, h);
            atomicAdd(P.stats + 12, u);
        }
    }
}

}  // namespace rt
