// rt_wavefront.hip -- wavefront (queue-driven) render path (included by rt_runtime.hip after
// rt_megakernel.hip, whose state machine and traversal steps it reuses).
//
// Why: the megakernels keep every lane's whole getFinalColor state (pixel, light loop, recursion,
// ~60 words) live in registers while the lane traverses, so they run at 2 waves per SIMD and
// every node fetch's latency is exposed (profiles/r01: TA 17 % busy, TD 41 %, VALU ~24 %).
// Here one frame is a sequence of iterations over a queue of pending queries:
//
//   seed   : every job (pixel or explicit ray) -> its first query         (queue 0)
//   trace  : every query of queue k -> closest/any hit (t, record)        lean kernel, 4+ waves/SIMD
//   shade  : every path of queue k  -> advance_lane() -> next query, appended (compacted) to
//            queue k+1, or the pixel written
//
// Path state lives in HBM as structure-of-arrays and is compacted with the queue, so every
// load/store of it is coalesced; the recursion frames stay put per job.  Queries are judged by
// the same trav_* steps and the state machine is the same advance_lane(), so the image and the
// ray count are bit-identical to the megakernels'.  Reference map: pixel loop src/main.cpp:340-400,
// getFinalColor :129-301, lights/cansee src/shadow.cpp:32-321, intersect
// src/bounding_volume_hierarchy.cpp:49-78.

namespace rt {

// path-state fields (32-bit words; ints stored by bit cast).  so/sd are not stored: whenever the
// state machine reads them they equal the shadow query's qo/qd (start_cansee, advance_lane).
enum WfField {
    WF_JOB = 0,
    WF_SAMPLE,
    WF_RAYS,
    WF_PACC,  // 3
    WF_QO = WF_PACC + 3,
    WF_QD = WF_QO + 3,
    WF_QT = WF_QD + 3,
    WF_QTYPE,
    WF_LEVEL,
    WF_CURD,  // 3
    WF_HP = WF_CURD + 3,
    WF_NN = WF_HP + 3,
    WF_NR = WF_NN + 3,
    WF_REFL = WF_NR + 3,
    WF_MAT = WF_REFL + 3,
    WF_COLOR,  // 3
    WF_LT = WF_COLOR + 3,
    WF_LI,
    WF_LS,
    WF_A,  // 4
    WF_U0 = WF_A + 4,
    WF_U1 = WF_U0 + 3,
    WF_SDIST = WF_U1 + 3,
    WF_SI,
    WF_NRAW,  // 3
    WF_DRAWS = WF_NRAW + 3,
    WF_NFIELDS
};

// The queue is split into WF_NQ independent sub-queues (interleaved 64-job chunks of the frame),
// each with its own length / work counters 4 KB apart, so the chunk grabs and appends of the
// waves serving different sub-queues never serialise on one address.
#define WF_NQ 64
#define WF_CSTRIDE 1024  // ints between two counters (4 KB)
enum WfCounter { WF_C_N0 = 0, WF_C_N1 = 1, WF_C_HEAD = 2, WF_C_RAYS = 3, WF_C_KINDS = 4 };

struct WfBufs {
    float* st_in;          // [WF_NFIELDS][cap] paths of the current queue
    float* st_out;         // [WF_NFIELDS][cap] paths of the next queue
    int cap;               // WF_NQ * seg
    int seg;               // capacity of one sub-queue
    const int* n_in;       // current lengths: n_in[q * WF_CSTRIDE]
    int* n_out;            // next lengths (appended to)
    int* head;             // trace chunk counters (zeroed per iteration)
    int* rays;             // per-sub-queue query counts (accumulated over the frame)
    float* res_t;          // [cap] trace result per current entry
    int* res_rec;          // [cap] RT_NO_HIT: miss
    Frame* frames;         // [njobs][fpj] recursion frames, by job
    int fpj;
    int refill;            // trace: idle lanes that trigger a refill
    int leaf_batch;        // trace: 0 = if-if steps, else while-while with this leaf batch
};

struct WfSt {
    float* p;
    int cap;
    __device__ __forceinline__ float f(int k, int i) const { return p[(size_t)k * cap + i]; }
    __device__ __forceinline__ int n(int k, int i) const { return __float_as_int(p[(size_t)k * cap + i]); }
    __device__ __forceinline__ v3 v(int k, int i) const { return v3{f(k, i), f(k + 1, i), f(k + 2, i)}; }
    __device__ __forceinline__ void sf(int k, int i, float x) const { p[(size_t)k * cap + i] = x; }
    __device__ __forceinline__ void sn(int k, int i, int x) const { p[(size_t)k * cap + i] = __int_as_float(x); }
    __device__ __forceinline__ void sv(int k, int i, v3 x) const {
        sf(k, i, x.x);
        sf(k + 1, i, x.y);
        sf(k + 2, i, x.z);
    }
};

__device__ __forceinline__ void wf_load(const WfSt& S, int i, Lane& L, uint32_t& rays) {
    L.job = S.n(WF_JOB, i);
    L.sample = S.n(WF_SAMPLE, i);
    rays = (uint32_t)S.n(WF_RAYS, i);
    L.pacc = S.v(WF_PACC, i);
    L.qo = S.v(WF_QO, i);
    L.qd = S.v(WF_QD, i);
    L.qt = S.f(WF_QT, i);
    L.qtype = S.n(WF_QTYPE, i);
    L.level = S.n(WF_LEVEL, i);
    L.cur_d = S.v(WF_CURD, i);
    L.hp = S.v(WF_HP, i);
    L.nN = S.v(WF_NN, i);
    L.nR = S.v(WF_NR, i);
    L.refl = S.v(WF_REFL, i);
    L.mat = S.n(WF_MAT, i);
    L.color = S.v(WF_COLOR, i);
    L.lt = S.n(WF_LT, i);
    L.li = S.n(WF_LI, i);
    L.ls = S.n(WF_LS, i);
    L.a0 = S.f(WF_A + 0, i);
    L.a1 = S.f(WF_A + 1, i);
    L.a2 = S.f(WF_A + 2, i);
    L.a3 = S.f(WF_A + 3, i);
    L.u0 = S.v(WF_U0, i);
    L.u1 = S.v(WF_U1, i);
    L.sdist = S.f(WF_SDIST, i);
    L.sI = S.f(WF_SI, i);
    L.nraw = S.v(WF_NRAW, i);
    L.draws = (uint32_t)S.n(WF_DRAWS, i);
    L.so = L.qo;
    L.sd = L.qd;
}

__device__ __forceinline__ void wf_store(const WfSt& S, int i, const Lane& L, uint32_t rays) {
    S.sn(WF_JOB, i, L.job);
    S.sn(WF_SAMPLE, i, L.sample);
    S.sn(WF_RAYS, i, (int)rays);
    S.sv(WF_PACC, i, L.pacc);
    S.sv(WF_QO, i, L.qo);
    S.sv(WF_QD, i, L.qd);
    S.sf(WF_QT, i, L.qt);
    S.sn(WF_QTYPE, i, L.qtype);
    S.sn(WF_LEVEL, i, L.level);
    S.sv(WF_CURD, i, L.cur_d);
    S.sv(WF_HP, i, L.hp);
    S.sv(WF_NN, i, L.nN);
    S.sv(WF_NR, i, L.nR);
    S.sv(WF_REFL, i, L.refl);
    S.sn(WF_MAT, i, L.mat);
    S.sv(WF_COLOR, i, L.color);
    S.sn(WF_LT, i, L.lt);
    S.sn(WF_LI, i, L.li);
    S.sn(WF_LS, i, L.ls);
    S.sf(WF_A + 0, i, L.a0);
    S.sf(WF_A + 1, i, L.a1);
    S.sf(WF_A + 2, i, L.a2);
    S.sf(WF_A + 3, i, L.a3);
    S.sv(WF_U0, i, L.u0);
    S.sv(WF_U1, i, L.u1);
    S.sf(WF_SDIST, i, L.sdist);
    S.sf(WF_SI, i, L.sI);
    S.sv(WF_NRAW, i, L.nraw);
    S.sn(WF_DRAWS, i, (int)L.draws);
}

// Wave-aggregated append: one atomic per wave; every lane of the wave must call it.
__device__ __forceinline__ int wave_append(int* counter, bool pred) {
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long m = __ballot(pred);
    if (!m) return -1;
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(m));
    base = __shfl(base, leader);
    return base + __popcll(m & ((1ull << lane) - 1ull));
}

// ---- seed: every job's first query -----------------------------------------------------------
// Job j goes to sub-queue q = (j / 64) % WF_NQ at position (j / 64 / WF_NQ) * 64 + j % 64, so the
// sub-queue lengths are known on the host.  A padding pixel (outside the image) becomes a dead
// entry: trace skips it, shade drops it.
#define Q_DEAD (-1)
__global__ __launch_bounds__(64) void wf_seed_kernel(KParams P, JobSrc J, WfBufs W) {
    const WfSt out{W.st_out, W.cap};
    for (int base = blockIdx.x * 64; base < J.njobs; base += gridDim.x * 64) {
        const int job = base + (int)threadIdx.x;
        if (job >= J.njobs) break;
        const int chunk = job >> 6;
        const int slot = (chunk % WF_NQ) * W.seg + (chunk / WF_NQ) * 64 + (job & 63);
        Lane L;
        L.job = job;
        L.sample = 0;
        L.pacc = v3{0.0f, 0.0f, 0.0f};
        L.level = 0;
        L.cur_d = L.hp = L.nN = L.nR = L.refl = L.color = L.u0 = L.u1 = v3{0.0f, 0.0f, 0.0f};
        L.mat = 0;
        L.lt = L_DONE;
        L.li = L.ls = 0;
        L.a0 = L.a1 = L.a2 = L.a3 = 0.0f;
        L.sdist = 0.0f;
        L.sI = 1.0f;
        L.nraw = v3{0.0f, 0.0f, 1.0f};
        L.draws = 0u;
        L.rpix = (uint32_t)job;
        L.qt = FLT_MAX;
        L.qtype = Q_PATH;
        L.qo = L.qd = v3{0.0f, 0.0f, 0.0f};
        if (J.mode == 0) {
            if (job_pixel(P, job, L))
                queue_camera(P, L);
            else
                L.qtype = Q_DEAD;
        } else {
            const rt_ray r = J.rays[job];
            L.qo = v3{r.origin[0], r.origin[1], r.origin[2]};
            L.qd = v3{r.direction[0], r.direction[1], r.direction[2]};
            L.qt = r.t;
        }
        wf_store(out, slot, L, 1u);
    }
}

// ---- trace: one query per lane, refilled from the queue as lanes finish ---------------------
#ifndef WF_PF
#define WF_PF false
#endif
template <bool COUNT, int WPE, int BW>
__global__ __launch_bounds__(64, WPE) void wf_trace_kernel(KParams P, WfBufs W) {
    __shared__ int stack_lds[RT_STACK_SIZE * RT_WAVE];
    const int lane = (int)threadIdx.x;
    int* stk = stack_lds + lane;
    const DevScene& S = P.S;
    const WfSt st{W.st_in, W.cap};
    const int q = (int)(blockIdx.x % WF_NQ);
    const int n = W.n_in[q * WF_CSTRIDE];
    const int qbase = q * W.seg;
    int* head = W.head + q * WF_CSTRIDE;
    Cnt cnt{};
    Trav T;
    float4 g[8];
    bool active = false, exhausted = false;
    int qi = 0;
    int c_next = 0, c_end = 0;  // wave-uniform: the chunk of the sub-queue being handed out
    bool q_empty = false;       // wave-uniform: the sub-queue has no chunk left
    unsigned int nrays = 0;
    uint32_t q_nodes0 = 0;  // counting builds: node visits before the current query
    for (;;) {
        // ---- refill idle lanes from 64-entry chunks (one atomic per chunk) ----
        unsigned long long wm = __ballot(!active && !exhausted);
        while (wm) {
            if (c_next >= c_end) {
                int v = n;
                if (!q_empty) {
                    if (lane == 0) v = atomicAdd(head, 64);
                    v = __shfl(v, 0);
                }
                if (v >= n) {
                    q_empty = true;
                    if ((wm >> lane) & 1ull) exhausted = true;
                    break;
                }
                c_next = v;
                c_end = min(v + 64, n);
            }
            // the first `take` wanting lanes (in lane order) get c_next, c_next + 1, ...
            const int take = min(__popcll(wm), c_end - c_next);
            const int rank = __popcll(wm & ((1ull << lane) - 1ull));
            if (((wm >> lane) & 1ull) && rank < take) {
                const int idx = qbase + c_next + rank;
                const int qt_ = st.n(WF_QTYPE, idx);
                if (qt_ == Q_DEAD) {  // padding pixel: a miss nobody reads; the lane asks again
                    W.res_t[idx] = FLT_MAX;
                    W.res_rec[idx] = RT_NO_HIT;
                } else {
                    qi = idx;
                    trav_init_q(S, P.use_bvh != 0, st.v(WF_QO, idx), st.v(WF_QD, idx), st.f(WF_QT, idx),
                                qt_ == Q_SHADOW, st.f(WF_SDIST, idx), T);
                    if (WF_PF && T.cur != RT_TRAV_NONE) node_fetch(S.nodes, T.cur, g);
                    active = true;
                    ++nrays;
                    q_nodes0 = cnt.nodes;
                }
            }
            c_next += take;
            wm = __ballot(((wm >> lane) & 1ull) && !active);
        }
        if (!__any(active)) break;
        // ---- traversal steps until `refill` lanes are idle ----
        for (;;) {
#ifdef WF_NO_WW
            if (true) {
#else
            if (W.leaf_batch == 0) {
#endif
                if (active) {
                    if (leaf_pending(T))
                        trav_record<COUNT>(S, T, cnt);
                    else if (T.cur != RT_TRAV_NONE)
                        trav_node<COUNT, BW, WF_PF>(S, T, stk, g, cnt);
                }
            } else {
                if (active && !leaf_pending(T) && T.cur != RT_TRAV_NONE) trav_node<COUNT, BW, WF_PF>(S, T, stk, g, cnt);
                const bool lp = active && leaf_pending(T);
                const bool more_nodes = __any(active && !leaf_pending(T) && T.cur != RT_TRAV_NONE);
                if (__any(lp) && (!more_nodes || __popcll(__ballot(lp)) >= W.leaf_batch)) {
                    bool work = lp;
                    while (__any(work)) {
                        if (work) {
                            trav_record<COUNT>(S, T, cnt);
                            work = leaf_pending(T);
                        }
                    }
                }
            }
            if (active && !leaf_pending(T) && T.cur == RT_TRAV_NONE) {
                trav_finish(S, T);
                W.res_t[qi] = T.best.t;
                W.res_rec[qi] = T.found ? T.best.rec : RT_NO_HIT;
                active = false;
                if (COUNT) {  // per-query work: max node visits [10], histogram [11..15]
                    const uint32_t nv = cnt.nodes - q_nodes0;
                    atomicMax(P.stats + 10, (unsigned long long)nv);
                    const int bkt = nv < 64 ? 11 : nv < 256 ? 12 : nv < 1024 ? 13 : nv < 4096 ? 14 : 15;
                    atomicAdd(P.stats + bkt, 1ull);
                }
            }
            if (!__any(active)) break;
            if (__popcll(__ballot(!active && !exhausted)) >= W.refill) break;
        }
    }
    // queries traced: one atomic per wave on the sub-queue's own counter
    for (int off = 32; off > 0; off >>= 1) nrays += __shfl_xor(nrays, off);
    if (lane == 0 && nrays) atomicAdd(W.rays + q * WF_CSTRIDE, (int)nrays);
    if (COUNT) flush_counters<COUNT>(P, cnt);
}

// ---- shade: advance every path of the queue to its next query -------------------------------
// Block b serves sub-queue b % WF_NQ; its continuing paths are appended to the same sub-queue
// of the next queue (one atomic per 64 entries on that sub-queue's counter).
template <bool COUNT>
__global__ __launch_bounds__(64) void wf_shade_kernel(KParams P, JobSrc J, WfBufs W) {
    const WfSt in{W.st_in, W.cap};
    const WfSt out{W.st_out, W.cap};
    const int q = (int)(blockIdx.x % WF_NQ);
    const int per_q = (int)(gridDim.x / WF_NQ);
    const int r = (int)(blockIdx.x / WF_NQ);
    const int n = W.n_in[q * WF_CSTRIDE];
    const int qbase = q * W.seg;
    int* n_out = W.n_out + q * WF_CSTRIDE;
    Cnt cnt{};
    for (int base = r * 64; base < n; base += per_q * 64) {
        const int i = base + (int)threadIdx.x;
        bool cont = false;
        Lane L;
        uint32_t rays = 0;
        if (i < n) {
            wf_load(in, qbase + i, L, rays);
            if (L.qtype != Q_DEAD) {
                if (J.mode == 0) {
                    job_pixel(P, L.job, L);
                    L.nsamples = P.aa ? 4 : (P.multi ? P.sample_size : 1);
                    L.rpix = (uint32_t)(L.py * P.W + L.px);
                } else {
                    L.nsamples = 1;
                    L.rpix = (uint32_t)L.job;
                }
                Best b;
                b.t = W.res_t[qbase + i];
                b.rec = W.res_rec[qbase + i];
                b.key = 0;
                const bool hit = (b.rec != RT_NO_HIT);
                Cnt jc{};
                jc.rays = rays;
                cont = advance_lane<COUNT>(P, J, L, W.frames + (size_t)L.job * W.fpj, hit, b, cnt, jc);
            }
        }
        const int j = wave_append(n_out, cont);
        if (cont) wf_store(out, qbase + j, L, rays + 1u);
    }
    if (COUNT) flush_counters<COUNT>(P, cnt);
}

// Lengths of queue 0 (seed layout: sub-queue q holds chunks q, q + WF_NQ, ... of 64 jobs).
__global__ void wf_seed_counts_kernel(int* n0, int njobs) {
    const int q = (int)threadIdx.x;
    if (q >= WF_NQ) return;
    const int nchunks = (njobs + 63) / 64;
    const int full = (q < nchunks) ? (nchunks - 1 - q) / WF_NQ + 1 : 0;
    int cnt = full * 64;
    if (full > 0 && ((nchunks - 1) % WF_NQ) == q) cnt -= nchunks * 64 - njobs;  // the last, partial chunk
    n0[q * WF_CSTRIDE] = cnt;
}

// Per-iteration reset (one block of WF_NQ lanes): next lengths and chunk counters to zero.
__global__ void wf_reset_kernel(int* n_out, int* head) {
    const int q = (int)threadIdx.x;
    if (q < WF_NQ) {
        n_out[q * WF_CSTRIDE] = 0;
        head[q * WF_CSTRIDE] = 0;
    }
}

// End of frame: the per-sub-queue query counts into stats[0] (rays), and total of n for checks.
__global__ void wf_finish_kernel(int* rays, unsigned long long* stats) {
    __shared__ unsigned long long acc;
    if (threadIdx.x == 0) acc = 0;
    __syncthreads();
    const int q = (int)threadIdx.x;
    if (q < WF_NQ) atomicAdd(&acc, (unsigned long long)rays[q * WF_CSTRIDE]);
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(stats, acc);
}

// Sum of the sub-queue lengths (host check of an empty queue).
__global__ void wf_total_kernel(const int* n, int* total) {
    __shared__ int acc;
    if (threadIdx.x == 0) acc = 0;
    __syncthreads();
    const int q = (int)threadIdx.x;
    if (q < WF_NQ) atomicAdd(&acc, n[q * WF_CSTRIDE]);
    __syncthreads();
    if (threadIdx.x == 0) *total = acc;
}

}  // namespace rt
