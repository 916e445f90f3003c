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
// coherent elementwise kernel that also does the queries' set-up arithmetic.  Per recursion level l
// (getFinalColor's `level`, src/main.cpp:129-301):
//
//   trace  T_l   the level's path rays (camera rays at l = 0, mirror rays after) -- closest hit; the hits
//                are appended to the level's hit list -- and the cansee segments of the level-(l-1) shading
//                points (src/shadow.cpp:32-69, any hit: a visible segment sets its light's bit in its
//                shading point's record)
//   shade  S_l   (a) resolve every level-(l-1) shading point: its node colour, the lights in getFinalColor's
//                order (getPointLights then getSpotLichts, src/main.cpp:174-185) whose bits are set, folded
//                into the pixel as acc = acc + w * colour -- the megakernels' forward fold, same operations
//                in the same order, so the images are bit-identical;
//                (b) shade every level-l hit (surface(), reflect): shading-point record h, and in the slots
//                of h in T_{l+1}'s queues one cansee segment per light that needs a query (lights within
//                SHADOW_ERROR_OFFSET count at once, spot lights outside their cone not at all) and the
//                mirror ray (ks^2-weighted child) below max_reflection_level; an unused slot is marked
//                empty, so the shade kernel needs no atomics.
//
// The pixel's colour lives in its output slot: 0 once the camera ray is resolved (T_0 for a miss, S_0 for a
// hit), then + w * colour per level in level order.  Scope: the opaque kernel's scenes (all materials
// opaque, point and spot lights, no textures, no glossy lobes) with one camera sample per pixel;
// everything else keeps the megakernels.
namespace rt {

#define RT_WF_EMPTY 0xFFFFFFFFu  // a queue slot without a query

// per launch-sequence counters (zeroed before T_0)
struct WfCnt {
    int hits[RT_MAX_DEPTH + 2];          // path-ray hits of T_l (= shading points of level l)
    int head[RT_MAX_DEPTH + 2][8 * 32];  // T_l: per-XCD queue heads, 128 B apart
};

// the buffers of one launch sequence (device pointers; capacities checked on the host)
struct WfBufs {
    WfCnt* cnt;
    int4* hit[2];       // T_l's hits in hit[l & 1]: (path ray or camera job, t bits, record, 0)
    float4* qp[2];      // path rays of level l in qp[l & 1], slot = parent shading point (5 float4):
                        //   (o, pixel), (d, EMPTY or 0), (normalize(d), 0), (safe_inv(d), 0), (weight, 0)
    float4* qs;         // cansee segments of T_l, slot = shading point * nl + light (4 float4):
                        //   (o, sdist), (d, EMPTY or point << 5 | light), (normalize(d), 0), (safe_inv(d), 0)
    float4* nodes[2];   // shading points of level l in nodes[l & 1]: (hp, mat), (nN, vis), (refl, pixel), (w, 0)
    int level;          // l of this launch
    int njobs;          // camera jobs of this chunk (T_0 / S_0): the render's jobs job0 .. job0 + njobs - 1
    int job0;           // (a multiple of 64: chunks start at a tile)
    int nl;             // lights in getFinalColor's order: point lights, then spot lights (<= 32)
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

// the query set-up of trav_init_q with the direction's normalisation and reciprocals already formed (the
// same expressions, evaluated by the shade kernel)
__device__ __forceinline__ void wf_init(bool use_bvh, bool shadow, bool all_opaque, v3 o, v3 d, v3 nd, v3 inv,
                                        float sdist, int ntri, Trav& T) {
    T.o = o;
    T.d = d;
    T.nd = nd;
    T.inv = inv;
    T.ref = shadow || use_bvh;
    T.any = shadow && all_opaque;
    const float thr = sdist - 2.0f * 0.0005f;
    T.best.t = FLT_MAX;
    T.best.key = -1;
    T.best.rec = RT_NO_HIT;
    T.mask = RefMask{0u, 0u};
    T.tcull = T.any ? thr : FLT_MAX;
    T.found = false;
    T.sp = 0;
    T.lb = 0u;
    T.lc = 0u;
    T.lh = 0u;
    T.rr = 0;
    const float dd = dot(d, d);
    if (!(fabsf(dd - 1.0f) <= 4e-6f)) {  // non-unit direction: exhaustive (trav_init_q)
        T.rk = ntri;
        T.cur = RT_TRAV_NONE;
    } else {
        T.rk = 0;
        T.cur = (ntri > 0) ? 0xFFu : RT_TRAV_NONE;
    }
}

// ---- trace ----------------------------------------------------------------------------------------------
// Persistent: every wave reserves blocks of 64 queries of its per-XCD range of the level's queue (path rays
// first, then the cansee segments), then of the other ranges; a lane whose query ends takes the next one of
// the wave's block at the next refill (once `refill` lanes wait, or none traces).  The traversal step is the
// opaque kernel's (dual record + node visit, the direct group stack in LDS, the reference BVH in LDS for
// the culling).  Path hits go through a 64-entry LDS buffer to the level's hit list (one atomic per 64).
#define RT_WF_BLOCK 64  // queries a wave reserves per queue-head atomic (camera jobs: one 8x8 tile)
// builds (WV): waves per SIMD in the low 4 bits, RT_WF_PF: each lane's next node prefetched into registers
#define RT_WF_PF 16
#define RT_WF_OVL 32  // a dual step's node loads issued before its record test (one memory round trip, not two)
#define RT_WF_W5 5    // the default build
template <bool COUNT, bool PRIMARY, int WV = RT_WF_W5>
__global__ __launch_bounds__(64, WV & 15) void wf_trace_kernel(KParams, WfBufs) {
    constexpr bool PF = (WV & RT_WF_PF) != 0, OVL = (WV & RT_WF_OVL) != 0 && !PF;
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ int stack_lds[RT_STACK8 * RT_WAVE];
    __shared__ RefLds ref_lds;
    __shared__ int4 hst[RT_WAVE];  // path hits waiting for their hit-list slots
    const int lane_id = threadIdx.x;
    int* stk = stack_lds + lane_id;
    // the level's work: n_path path rays (camera jobs at l = 0), then n_seg cansee segments
    int n_path, n_seg, level;
    {
        const WfBufs& B = wf_bufs(ka);
        const KParams& P0 = kernel_params(ka);
        level = B.level;
        const int parents = PRIMARY ? 0 : B.cnt->hits[level - 1];
        n_path = PRIMARY ? B.njobs : (level - 1 < P0.max_level ? parents : 0);
        n_seg = PRIMARY ? 0 : parents * B.nl;
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
    float4 g[RT_NODE_F4];  // PF: the node the lane visits next
    Cnt cnt{};
    int src = -1;       // the query this lane traces: < n_path a path ray (camera job), else a segment
    uint32_t tag = 0u;  // a segment's shading point << 5 | light; a camera ray's output pixel
    bool tracing = false, done = false;
    int xr = (int)(blockIdx.x & 7), xtried = 0;
    // the wave's reserved block [nxt, end) (wave-uniform); camera jobs: the block is one tile, decoded once
    int nxt = 0, end = 0, bstart = 0;
    int t_view = 0, t_px0 = 0, t_py0 = 0, t_rib0 = 0, t_row0 = 0, t_lb = 0;
    int hpos = 0;                   // entries in hst (wave-uniform)
    const int ntiles = n_all >> 6;  // camera jobs: whole tiles (view_jobs and job0 are multiples of 64)
    for (;;) {
        const KParams& P = *(const KParams*)fresh_kernarg(ka);
        const DevScene& S = P.S;
        // ---- refill: the waiting lanes take the next queries of the wave's block (a new block when it is
        // used up; at most one block per refill) ----
        {
            const bool idle = !tracing && !done;
            const unsigned long long want = __ballot(idle);
            const int nwant = __popcll(want);
            if (want && (nwant >= P.refill || !__any(tracing))) {
                const WfBufs& B = wf_bufs(ka);
                const int leader = __ffsll((long long)want) - 1;
                while (nxt == end && xtried < 8) {  // wave-uniform: the next block of range xr
                    int lo, hi;
                    if (PRIMARY) {  // ranges of whole tiles
                        lo = ((xr * ntiles) >> 3) << 6;
                        hi = (((xr + 1) * ntiles) >> 3) << 6;
                    } else {
                        lo = (int)(((long long)xr * n_all) >> 3);
                        hi = (int)(((long long)(xr + 1) * n_all) >> 3);
                    }
                    int b = 0;
                    if (lane_id == leader) b = lo + atomicAdd(&B.cnt->head[level][32 * xr], RT_WF_BLOCK);
                    b = __shfl(b, leader);
                    if (b + RT_WF_BLOCK >= hi) {  // the range is used up with this block: the next one after it
                        xr = (xr + 1) & 7;
                        ++xtried;
                    }
                    nxt = min(b, hi);
                    end = min(b + RT_WF_BLOCK, hi);
                    bstart = nxt;
                    if (PRIMARY && nxt < end) {
                        // the tile's pixel 0 (job_pixel's decode, once per tile)
                        uint32_t rpix;
                        int out_row;
                        job_pixel(P, B.job0 + nxt, rpix, out_row);
                        int view;
                        const int tile = view_job(P, B.job0 + nxt, view) >> 6;
                        const int py = (int)(rpix / (uint32_t)P.W), px = (int)(rpix - (uint32_t)py * (uint32_t)P.W);
                        const int tiles_y_band = (P.band_rows + 7) / 8;
                        const int rest = tile / ((P.W + 7) / 8);
                        t_view = __builtin_amdgcn_readfirstlane(view);
                        t_px0 = __builtin_amdgcn_readfirstlane(px);
                        t_py0 = __builtin_amdgcn_readfirstlane(py);
                        t_rib0 = __builtin_amdgcn_readfirstlane((rest % tiles_y_band) * 8);
                        t_lb = __builtin_amdgcn_readfirstlane(rest / tiles_y_band);
                        t_row0 = __builtin_amdgcn_readfirstlane(out_row);
                    }
                }
                const int take = min(nwant, end - nxt);
                const int rank = __popcll(want & ((1ull << lane_id) - 1ull));
                const int k = (idle && rank < take) ? nxt + rank : -1;
                const int j = k - bstart;  // camera jobs: the pixel of the tile (a block is served over several refills)
                nxt += take;
                if (idle) {
                    if (k >= 0) {
                        if (PRIMARY) {
                            // job_pixel / camera_query for pixel j of the tile (no padding pixel is traced)
                            const int px = t_px0 + (j & 7), py = t_py0 + (j >> 3), rib = t_rib0 + (j >> 3);
                            if (px < P.W && rib < P.band_rows && py < P.H && t_lb < P.n_local_bands) {
                                const float ndx = (float)px / (float)P.W * 2.0f - 1.0f;
                                const float ndy = (float)py / (float)P.H * 2.0f - 1.0f;
                                v3 o, d;
                                if (P.n_views > 1)
                                    gen_ray_view(P, t_view, ndx, ndy, o, d);
                                else
                                    gen_ray(P, ndx, ndy, o, d);
                                src = k;
                                cnt.rays++;
                                wf_init(P.use_bvh != 0, false, S.all_opaque != 0, o, d, normalize(d), safe_inv(d),
                                        0.0f, S.ntri, T);
                                if (PF && T.cur != RT_TRAV_NONE) node_fetch(S.nodes, T.cur, g);
                                tracing = true;
                                // the pixel's output row (out_row of job_pixel: setPixel's H-1-y, or band rows)
                                tag = (uint32_t)(P.out_image ? t_row0 - (j >> 3) : t_row0 + (j >> 3)) * (uint32_t)P.W +
                                      (uint32_t)px;
                            }
                        } else {
                            const bool seg = k >= n_path;
                            const float4* e = seg ? B.qs + (size_t)(k - n_path) * 4 : B.qp[level & 1] + (size_t)k * 5;
                            const float4 e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
                            if (__float_as_uint(e1.w) != RT_WF_EMPTY) {
                                src = k;
                                tag = __float_as_uint(e1.w);
                                cnt.rays++;
                                wf_init(P.use_bvh != 0, seg, S.all_opaque != 0, v3{e0.x, e0.y, e0.z},
                                        v3{e1.x, e1.y, e1.z}, v3{e2.x, e2.y, e2.z}, v3{e3.x, e3.y, e3.z},
                                        seg ? e0.w : 0.0f, S.ntri, T);
                                if (PF && T.cur != RT_TRAV_NONE) node_fetch(S.nodes, T.cur, g);
                                tracing = true;
                            }
                        }
                    } else if (nxt == end && xtried >= 8) {
                        done = true;
                    }
                }
            }
        }
        const bool any_tracing = __any(tracing);
        // ---- one record test and / or one node visit per tracing lane ----
        bool fin = false;
        if (tracing) {
            const bool rec = leaf_pending(T);
            if (OVL) {
                // the node this step visits, decided before the record test: the test only pops the next hit leaf
                // (T.lh), or ends an any-hit query (then the node was loaded for nothing)
                const uint32_t lh_after = (rec && T.rk == 0) ? (T.lh & (T.lh - 1u)) : T.lh;
                if (T.cur != RT_TRAV_NONE && (!rec || (P.dual && lh_after == 0u))) node_fetch(S.nodes, T.cur, g);
            }
            if (rec) trav_record<COUNT, true, false, false>(S, T, cnt, nullptr, nullptr, &ref_lds);
            const bool nv = T.cur != RT_TRAV_NONE && (!rec || (P.dual && T.lh == 0u));
            if (nv) trav_node<COUNT, 8, PF, true, false, OVL>(S, T, stk, g, cnt);
            if (!leaf_pending(T) && T.cur == RT_TRAV_NONE) {
                trav_finish(S, T);
                fin = true;
                tracing = false;
            }
        }
        // ---- finished queries: misses and segments in place, path hits into the LDS buffer ----
        const bool phit = fin && src < n_path && T.found;
        if (fin && !phit) {
            const WfBufs& B = wf_bufs(ka);
            if (src < n_path) {
                if (PRIMARY) {  // a camera ray that hits nothing: getFinalColor returns black
                    float* dst = P.out + (size_t)tag * 3;
                    dst[0] = 0.0f;
                    dst[1] = 0.0f;
                    dst[2] = 0.0f;
                }
            } else if (!T.found) {
                // the segment reached its light: that light's bit in its shading point's record
                atomicOr(reinterpret_cast<unsigned int*>(B.nodes[(level - 1) & 1] + (size_t)(tag >> 5) * 4 + 1) + 3,
                         1u << (tag & 31u));
            }
        }
        const unsigned long long hm = __ballot(phit);
        const bool last = !any_tracing && __all(done);
        if (hm || (last && hpos > 0)) {
            const int nh = __popcll(hm);
            if (hpos + nh > RT_WAVE) {  // the buffer first: one hit-list atomic for its entries
                const WfBufs& B = wf_bufs(ka);
                int base = 0;
                if (lane_id == 0) base = atomicAdd(&B.cnt->hits[level], hpos);
                base = __shfl(base, 0);
                if (lane_id < hpos) B.hit[level & 1][base + lane_id] = hst[lane_id];
                hpos = 0;
            }
            if (phit)
                hst[hpos + __popcll(hm & ((1ull << lane_id) - 1ull))] = make_int4(src, __float_as_int(T.best.t),
                                                                                  T.best.rec, 0);
            hpos += nh;
            if (last) {  // the wave's last hits
                const WfBufs& B = wf_bufs(ka);
                int base = 0;
                if (lane_id == 0) base = atomicAdd(&B.cnt->hits[level], hpos);
                base = __shfl(base, 0);
                if (lane_id < hpos) B.hit[level & 1][base + lane_id] = hst[lane_id];
                hpos = 0;
            }
        }
        if (fin) src = -1;
        if (last) break;
    }
    flush_counters<COUNT>(kernel_params(ka), cnt);
}

// ---- shade -----------------------------------------------------------------------------------------------
// Elementwise over (a) the level-(l-1) shading points (resolve) and (b) the level's hits (shade); a
// grid-stride loop over the counts the previous kernels left on the device.
template <bool COUNT>
__global__ __launch_bounds__(256) void wf_shade_kernel(KParams, WfBufs) {
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const KParams& P = kernel_params(ka);
    const WfBufs& B = wf_bufs(ka);
    const DevScene& S = P.S;
    const int level = B.level, nl = B.nl;
    const int n_res = level > 0 ? B.cnt->hits[level - 1] : 0;
    const int n_hit = B.cnt->hits[level];
    const int n_all = n_res + n_hit;
    Cnt cnt{};
    const int stride = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_all; i += stride) {
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
            for (int li = 0; li < nl; ++li) {
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
            continue;
        }
        // (b) hit h of level l: a shading point (begin_node, src/main.cpp:131-256, the opaque branch:
        // lite_advance's expressions)
        const int h = i - n_res;
        const int4 hr = B.hit[level & 1][h];
        const Best b{__int_as_float(hr.y), -1, hr.z};
        v3 o, d, w{1.0f, 1.0f, 1.0f};
        uint32_t pix;
        if (level == 0) {
            uint32_t rpix;
            int out_row;
            job_pixel(P, B.job0 + hr.x, rpix, out_row);
            pix = (uint32_t)out_row * (uint32_t)P.W + rpix % (uint32_t)P.W;
            Query q;
            camera_query(P, B.job0 + hr.x, rpix, 0, q);
            o = q.o;
            d = q.d;
            float* dst = P.out + (size_t)pix * 3;  // the colour starts at 0
            dst[0] = 0.0f;
            dst[1] = 0.0f;
            dst[2] = 0.0f;
        } else {
            const float4* e = B.qp[level & 1] + (size_t)hr.x * 5;
            const float4 e0 = e[0], e1 = e[1], e4 = e[4];
            o = v3{e0.x, e0.y, e0.z};
            pix = __float_as_uint(e0.w);
            d = v3{e1.x, e1.y, e1.z};
            w = v3{e4.x, e4.y, e4.z};
        }
        const Surf s = surface(S, o, d, b, false, level == 0);
        if (COUNT) {
            cnt.hits++;
            if (s.ub) cnt.ub++;
        }
        const v3 hp = s.p, nN = normalize(s.n), refl = reflect(normalize(d), nN);
        const int mat = (b.rec >= 0) ? s.mesh : b.rec;
        // cansee segments (start_cansee) of the lights that need a query in slots h * nl + li; lights within
        // SHADOW_ERROR_OFFSET are visible at once (src/shadow.cpp:38-40), spot lights outside their cone
        // contribute nothing (src/shadow.cpp:235-237)
        uint32_t vis = 0u;
        for (int li = 0; li < nl; ++li) {
            float4* e = B.qs + ((size_t)h * nl + li) * 4;
            v3 lp, lc;
            wf_light(S, li, lp, lc);
            bool in = true;
            if (li >= S.npl) {
                const DSpot sp = S.spot[li - S.npl];
                in = dot(normalize(ld3(sp.dir)), normalize(hp - lp)) > sp.cos_angle;
            }
            bool need = false;
            if (in) {
                v3 sd = lp - hp;
                const float sdist = length(sd);
                sd = normalize(sd);
                if (sdist > 0.0005f) {
                    need = true;
                    const v3 so = hp + 0.0005f * sd, snd = normalize(sd), sinv = safe_inv(sd);
                    e[0] = make_float4(so.x, so.y, so.z, sdist);
                    e[1] = make_float4(sd.x, sd.y, sd.z, __uint_as_float(((uint32_t)h << 5) | (uint32_t)li));
                    e[2] = make_float4(snd.x, snd.y, snd.z, 0.0f);
                    e[3] = make_float4(sinv.x, sinv.y, sinv.z, 0.0f);
                } else {
                    vis |= 1u << li;
                }
            }
            if (!need) e[1] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(RT_WF_EMPTY));
        }
        float4* nd = B.nodes[level & 1] + (size_t)h * 4;
        nd[0] = make_float4(hp.x, hp.y, hp.z, __int_as_float(mat));
        nd[1] = make_float4(nN.x, nN.y, nN.z, __uint_as_float(vis));
        nd[2] = make_float4(refl.x, refl.y, refl.z, __uint_as_float(pix));
        nd[3] = make_float4(w.x, w.y, w.z, 0.0f);
        // the mirror child in slot h (lite_child_weight; its query from hitPoint + 0.01 * reflect)
        if (level < P.max_level) {
            float4* e = B.qp[(level + 1) & 1] + (size_t)h * 5;
            const v3 ks{s.m.ks[0], s.m.ks[1], s.m.ks[2]};
            if (ks.x > 0.0f || ks.y > 0.0f || ks.z > 0.0f) {
                const DMat m = load_mat(S, mat);
                const v3 mks{m.ks[0], m.ks[1], m.ks[2]};
                const v3 wc = (m.shin != 0.0f) ? w * ((mks * mks) / (float)P.glossy_n) : w * (mks * mks);
                const v3 co = hp + 0.01f * refl, cnd = normalize(refl), cinv = safe_inv(refl);
                e[0] = make_float4(co.x, co.y, co.z, __uint_as_float(pix));
                e[1] = make_float4(refl.x, refl.y, refl.z, 0.0f);
                e[2] = make_float4(cnd.x, cnd.y, cnd.z, 0.0f);
                e[3] = make_float4(cinv.x, cinv.y, cinv.z, 0.0f);
                e[4] = make_float4(wc.x, wc.y, wc.z, 0.0f);
            } else {
                e[1] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(RT_WF_EMPTY));
            }
        }
    }
    if (COUNT) {
        // hits and UB-regime hits of the shaded points (rt_stats.hits / ub_hits)
        unsigned long long hh = cnt.hits, u = cnt.ub;
        for (int off = 32; off > 0; off >>= 1) {
            hh += __shfl_xor(hh, off);
            u += __shfl_xor(u, off);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(P.stats + 3, hh);
            atomicAdd(P.stats + 12, u);
        }
    }
}

}  // namespace rt
