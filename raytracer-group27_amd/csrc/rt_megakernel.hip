// rt_megakernel.hip -- persistent ray-state-machine render kernels (included by rt_runtime.hip after
// rt_kernels.hip, whose device helpers they use).
//
// Why: the recursive reference (getFinalColor -> lights -> cansee -> intersect) compiled as nested
// inlined calls holds several traversal instances live at once and a wave is held by its slowest
// pixel.  Here every lane is a small state machine whose only expensive step is ONE shared
// traversal: each lane traces whatever query its state needs (camera ray, mirror / reflected /
// refracted / glossy ray, or one cansee segment), then advances its state until it needs the next
// query.  A lane that finishes its pixel takes the next one from a job counter (wave-aggregated
// atomic), so no lane idles while work remains.
//
// The arithmetic of every step is the reference's (rt_kernels.hip helpers); only the schedule
// differs.  Reference map: pixel/sample loop src/main.cpp:344-395, getFinalColor :129-301, lights
// src/shadow.cpp:106-321, cansee src/shadow.cpp:32-69.  Two kernels share the state machine:
//   persistent_kernel     whole-traversal refill (scenes < 65 536 triangles: a query is a handful of
//                         node visits and per-step bookkeeping does not pay)
//   persistent_df_kernel  dynamic fetch: the traversal is resumable and advanced one node visit or
//                         one triangle record per iteration; lanes whose query completes park until
//                         enough of the wave waits, then the wave advances them together.

namespace rt {

enum LType { L_POINT = 0, L_SPHERE = 1, L_SPOT = 2, L_PLANE = 3, L_DONE = 4 };

// The query a lane traces next: a getFinalColor ray or one cansee segment (Lane::shadow).
struct Query {
    v3 o, d;
    float t;  // initial ray.t: FLT_MAX, or the caller's ray.t for rt_shade's explicit rays
};

struct JobSrc;

// The render kernels' own arguments (KParams, then JobSrc), read through the kernarg segment pointer
// `ka` the kernel passes down.  The out-of-line parts of the state machine use these instead of
// reference parameters: a reference to a kernel argument makes the compiler copy the 400-B KParams
// into every lane's private memory and read it back with vector loads; through the (uniform) segment
// pointer the reads are scalar loads.
__device__ __forceinline__ const char* uniform_kernarg(const void* ka) {
    typedef const __attribute__((address_space(4))) char* CB;
    const uint64_t a = (uint64_t)ka;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return (const char*)(CB)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ const KParams& kernel_params(const void* ka) {
    return *(const KParams*)uniform_kernarg(ka);
}

// The kernarg segment pointer made opaque to the optimiser: reads through it are scalar loads issued
// where they are used (the scalar cache serves them), instead of kernel arguments the compiler loads
// once and keeps in SGPRs across the whole persistent loop -- ~100 dwords of KParams that otherwise
// spill into VGPR lanes and cost a v_readlane per use.
__device__ __forceinline__ const char* fresh_kernarg(const void* ka) {
    uint32_t lo = (uint32_t)(uint64_t)ka, hi = (uint32_t)((uint64_t)ka >> 32);
    asm volatile("" : "+s"(lo), "+s"(hi));
    typedef const __attribute__((address_space(4))) char* CB;
    return (const char*)(CB)(((uint64_t)hi << 32) | lo);
}

// Per-lane state between queries: the pixel, the position in the recursion tree and in the light
// loop of the current shading point.  Kept small (39 dwords without textures): it is live across
// every traversal step.
struct Lane {
    int job;        // >= 0 job index; -1 idle (fetch another); -2 no more work
    uint32_t rpix;  // the reference's pixel id y * W + x (rt_shade: the ray index), glossy Philox counter
    uint32_t sample : 7;  // camera sample (AA / getPixelRays: < 64)
    uint32_t level : 5;   // recursion level of the current node (<= RT_MAX_DEPTH)
    uint32_t nfr : 5;     // pending frames (transparent / glossy branches, <= RT_MAX_DEPTH)
    uint32_t lt : 3;      // light loop: type (LType)
    uint32_t desc : 1;    // the current node descends to its mirror / reflected child after its lights
    uint32_t shadow : 1;  // the query in flight is a cansee segment
    int li : 16, ls : 16; // light loop: index, sample (-1: before the first; fill_params bounds both)
    v3 acc;         // current camera sample: forward-accumulated colour
    v3 w, wc;       // weight of the current node / of its mirror or reflected child
    v3 hp, nN, refl;  // shading point: hitPoint, normalize(normal), reflect (nR = normalize(refl))
    int mat;        // >= 0 mesh material, < 0: sphere -(s+1)
    v3 color;       // direct light of the current node
    float a0, a1, a2, a3;  // per-light accumulators
    v3 u0, u1;             // spherical light: perp | plane light: (px, py)
    float sdist, sI;       // cansee: remaining distance, intensity
    uint32_t draws;        // glossy: Philox draws of this camera sample
    v3 kd;                 // TEX kernels only: kd of the shading point (texture or material)
};

static_assert(sizeof(Lane) == 42 * 4, "Lane layout (39 dwords + the TEX kernels' kd)");

__device__ __forceinline__ v3 lane_nR(const Lane& L) { return normalize(L.refl); }

__device__ __forceinline__ DMat load_mat(const DevScene& S, int m) {
    if (m >= 0) return S.mats[m];
    return S.sph[-m - 1].m;
}

// matForRendering (src/main.cpp:146-171): the shading point's material with the kd surface() took
// from its texture, if any
template <bool TEX>
__device__ __forceinline__ DMat render_mat(const DevScene& S, const Lane& L) {
    DMat m = load_mat(S, L.mat);
    if (TEX) {
        m.kd[0] = L.kd.x;
        m.kd[1] = L.kd.y;
        m.kd[2] = L.kd.z;
    }
    return m;
}

// 8-wide traversal over the quantised BVH8 (bvh_build.h).  The stack holds node groups
// (node << 8 | mask of inner children not yet visited), one per tree level, so it is bounded by
// the tree depth; a popped group's boxes are re-tested against the current best t and the
// nearest survivor is visited next.  Every candidate is judged with the same reference
// arithmetic and (t, key) order as trace_query.
// A triangle record's 64 B in one memory round trip (PIN): without the pin the compiler sinks the
// loads of D and the keys (r3) below the branches that use them, so a record costs three dependent
// trips.  The 4-wave batch variant keeps the sunk loads (its waves hide the latency, and the pinned
// registers cost it: C3 batch 0.69 vs 0.71 ms/frame); the others pin (C2 0.75 -> 0.72 ms).
template <bool PIN = true>
__device__ __forceinline__ void load_record(const float4* tp, float4& r0, float4& r1, float4& r2, float4& r3) {
    r0 = tp[0];
    r1 = tp[1];
    r2 = tp[2];
    r3 = tp[3];
    if (PIN) asm volatile("" ::"v"(r3.x), "v"(r3.y), "v"(r3.z), "v"(r3.w));
}

template <bool COUNT>
__device__ __forceinline__ bool test_records(const DevScene& S, int first, int count, v3 o, v3 d, v3 nd, float thr,
                                             bool REF, bool ANY, Best& best, RefMask& mask, float& tcull,
                                             bool& found, Cnt& cnt) {
    for (int r = first; r < first + count; ++r) {
        float4 r0, r1, r2, r3;
        load_record(S.tri + r * 4, r0, r1, r2, r3);
        if (COUNT) {
            cnt.tris++;
            if (wave_leader()) cnt.wtris++;
        }
        float t;
        if (!tri_test(r0, r1, r2, r3, o, d, nd, t)) continue;
        const int key = REF ? __float_as_int(r3.z) : __float_as_int(r3.y);
        if (ANY ? !(t <= thr) : !(t < best.t || (t == best.t && key < best.key))) continue;
        if (REF && !leaf_reachable(S, __float_as_int(r3.w), o, nd, mask)) continue;
        best.t = t;
        best.key = key;
        best.rec = r;
        found = true;
        if (ANY) return true;
        tcull = t;
    }
    return false;
}

__device__ __forceinline__ float pow2f(uint32_t biased) { return __int_as_float((int)(biased << 23)); }

// the value of the 16-bit child plane word at bit sh of w (bvh_build.h plane_q): a binary16 widened exactly
// (RT_PLANES_F16; used as an fma operand the widening folds into v_fma_mix_f32) or an unsigned integer
__device__ __forceinline__ float plane_f(uint32_t w, int sh) {
    const unsigned short h = (unsigned short)((w >> sh) & 0xFFFFu);
    if constexpr (RT_PLANES_F16) return (float)__builtin_bit_cast(_Float16, h);
    else return (float)h;
}

// the value of plane k (0-5: lo x, y, z, hi x, y, z) of slot s of a node held in its float4s g (bvh_build.h
// pack_planes): RT_PLANES_U8 an 8-bit step count (one v_cvt_f32_ubyteN of its dword), else the 16-bit word
__device__ __forceinline__ float node_plane(const float4* g, int k, int s) {
    if constexpr (RT_PLANES_U8) {
        const int dw = 2 * k + (s >> 2);
        const float4 v = g[2 + (dw >> 2)];
        const uint32_t w = __float_as_uint((dw & 3) == 0 ? v.x : (dw & 3) == 1 ? v.y : (dw & 3) == 2 ? v.z : v.w);
        return (float)((w >> (8 * (s & 3))) & 0xFFu);
    } else {
        const float4 v = g[2 + k];
        const int wi = s >> 1;
        return plane_f(__float_as_uint(wi == 0 ? v.x : wi == 1 ? v.y : wi == 2 ? v.z : v.w), (s & 1) * 16);
    }
}

template <bool COUNT, int NW>
__device__ __forceinline__ bool trace_query8(const DevScene& S, v3 o, v3 d, float t_init, float thr, bool REF,
                                             bool ANY, Best& best, int* stk, Cnt& cnt) {
    const v3 nd = normalize(d);
    best.t = t_init;
    best.key = -1;
    best.rec = RT_NO_HIT;
    RefMask mask{0u, 0u};
    float tcull = ANY ? thr : t_init;
    bool found = false;
    const float dd = dot(d, d);
    if (!(fabsf(dd - 1.0f) <= 4e-6f)) {
        // non-unit direction: exhaustive (see traverse() in rt_kernels.hip)
        if (test_records<COUNT>(S, 0, S.ntri, o, d, nd, thr, REF, ANY, best, mask, tcull, found, cnt)) return true;
    } else if (S.ntri > 0) {
        const v3 inv = safe_inv(d);
        const float4* nodes = S.nodes;
        int sp = 0;
        uint32_t cur = 0xFFu;  // node 0, every slot
        // software pipeline: the next node's bytes are requested before this node's leaf
        // triangles are tested, so the two memory latencies overlap
        float4 g[RT_NODE_F4];
#pragma unroll
        for (int k = 0; k < RT_NODE_F4; ++k) g[k] = nodes[k];
        for (;;) {
            const uint32_t node = cur >> 8;
            float4 gn[RT_NODE_F4];
#pragma unroll
            for (int k = 0; k < RT_NODE_F4; ++k) gn[k] = g[k];
            const float4 f0 = gn[0], f1 = gn[1];
            if (COUNT) {
                cnt.nodes++;
                if (wave_leader()) cnt.wnodes++;
            }
            const uint32_t w3 = __float_as_uint(f0.w);
            const uint32_t imask = __float_as_uint(f1.z) & 0xFFu;
            const uint32_t lmask = (__float_as_uint(f1.z) >> 8) & 0xFFu;
            const uint32_t counts = __float_as_uint(f1.w);
            const uint32_t child_base = __float_as_uint(f1.x);
            const uint32_t tri_base = __float_as_uint(f1.y);
            // slab distances straight from the 16-bit offsets: t = q * (2^e * inv) + (origin - o) * inv.
            // The two rounded products differ from the decoded-box form by a few ulps of |t|, the
            // same order as the decoded form's own error, and far inside the eps inflation.
            const float bx = pow2f(w3 & 0xFFu) * inv.x, by = pow2f((w3 >> 8) & 0xFFu) * inv.y,
                        bz = pow2f((w3 >> 16) & 0xFFu) * inv.z;
            const float ax = (f0.x - o.x) * inv.x, ay = (f0.y - o.y) * inv.y, az = (f0.z - o.z) * inv.z;
            const uint32_t m = (cur & 0xFFu) & (imask | lmask);
            // box tests; the nearest inner child is chosen here so no per-slot distances stay live.
            uint32_t hits = 0;
            float tbest = FLT_MAX;
            int sbest = -1;
#pragma unroll
            for (int s = 0; s < NW; ++s) {
                if (m & (1u << s)) {
                    const float tlx = fmaf(node_plane(gn, 0, s), bx, ax), thx = fmaf(node_plane(gn, 3, s), bx, ax);
                    const float tly = fmaf(node_plane(gn, 1, s), by, ay), thy = fmaf(node_plane(gn, 4, s), by, ay);
                    const float tlz = fmaf(node_plane(gn, 2, s), bz, az), thz = fmaf(node_plane(gn, 5, s), bz, az);
                    const float t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fminf(tlz, thz));
                    const float t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fmaxf(tlz, thz));
                    if (t0 <= t1 && t1 >= 0.0f && t0 <= tcull) {
                        hits |= 1u << s;
                        if ((imask & (1u << s)) && (t0 < tbest || sbest < 0)) {
                            tbest = t0;
                            sbest = s;
                        }
                    }
                }
            }
            // next node (decided before the leaf tests; a child or group that the leaf hits put
            // out of reach is culled when it is tested): the nearest inner child, the rest kept as
            // a group (node << 8 | slots) on the stack, else the top group
            const uint32_t ih = hits & imask;
            bool more = true;
            if (ih) {
                const uint32_t rest = ih & ~(1u << sbest);
                if (rest) {
                    stk[sp * RT_WAVE] = (int)((node << 8) | rest);
                    ++sp;
                }
                const uint32_t rank = __popc(imask & ((1u << sbest) - 1u));
                cur = ((child_base + rank) << 8) | 0xFFu;
            } else if (sp > 0) {
                --sp;
                cur = (uint32_t)stk[sp * RT_WAVE];
            } else {
                more = false;
            }
            if (more) {
                const float4* np = nodes + (size_t)(cur >> 8) * RT_NODE_SF4;
#pragma unroll
                for (int k = 0; k < RT_NODE_F4; ++k) g[k] = np[k];
            }
            // leaf children: records tri_base + (counts of lower leaf slots), in slot order
            uint32_t lh = hits & lmask;
            while (lh) {
                const int s = __ffs(lh) - 1;
                lh &= lh - 1u;
                const uint32_t below = s ? (counts & ((1u << (4 * s)) - 1u)) : 0u;
                uint32_t nib = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
                nib = (nib * 0x01010101u) >> 24;
                const int cnt_s = (int)((counts >> (4 * s)) & 15u);
                if (test_records<COUNT>(S, (int)(tri_base + nib), cnt_s, o, d, nd, thr, REF, ANY, best, mask, tcull,
                                        found, cnt))
                    return true;
            }
            if (!more) break;
        }
    }
    if (!(ANY && found)) {
        for (int s = 0; s < S.nsph; ++s) {
            const DSph sp_ = S.sph[s];
            float t;
            if (!sphere_test(sp_, o, d, t)) continue;
            const int key = REF ? sp_.key_bvh : S.ntri + s;
            if (ANY ? !(t <= thr) : !(t < best.t || (t == best.t && key < best.key))) continue;
            if (REF && !leaf_reachable(S, sp_.leaf, o, nd, mask)) continue;
            best.t = t;
            best.key = key;
            best.rec = -s - 1;
            found = true;
            if (ANY) break;
        }
    }
    return found;
}

// ---- light loop -----------------------------------------------------------------------------
// cansee(hp, target) (src/shadow.cpp:32-40): queues the first segment, or returns false when the
// loop condition distance > SHADOW_ERROR_OFFSET fails at once (cansee returns true, no intersect).
// a finished fan (the kernel's FanTable): visibility bit s of sample s, and (scenes with transparent
// materials) each sample's cansee intensity, both in sample order
struct FanResult {
    uint64_t vis;
    const float* inten;  // LDS; null for opaque scenes (every intensity is 1)
    bool done;           // the lane resumes from its fan (its own last query is not a cansee segment)
    const float* term;   // plane-light fans (LDS): each visible sample's hit term, computed by its sample lane
    float c2max;         // ... and the running maximum of the visible samples' specular cosines
};

__device__ __forceinline__ bool start_cansee(Lane& L, v3 target, Query& q) {
    v3 d = target - L.hp;
    L.sdist = length(d);
    d = normalize(d);
    L.sI = 1.0f;
    if (L.sdist > 0.0005f) {
        q.o = L.hp + 0.0005f * d;
        q.d = d;
        q.t = FLT_MAX;
        L.shadow = true;
        return true;
    }
    return false;
}

__device__ __forceinline__ void light_cos(const Lane& L, v3 lp, float& cosL, float& cosS) {
    const v3 ldir = normalize(lp - L.hp);
    cosL = fabsf(dot(L.nN, ldir));
    const float d2 = dot(lane_nR(L), ldir);
    cosS = (0.0f < d2) ? d2 : 0.0f;
}

// getSpherelights' first perp (src/shadow.cpp:160-175)
__device__ __forceinline__ v3 sphere_perp(v3 hp, v3 lp, float radius) {
    v3 dd = normalize(lp - hp);
    v3 notd = dd;
    if (dd.x != 0.0f) {
        notd.y = -dd.x;
        notd.x = dd.y;
    } else {
        notd.y = -dd.z;
        notd.z = dd.y;
    }
    return normalize(cross(dd, notd)) * radius;
}

// Advance the light loop (getPointLights, getSpherelights, getSpotLichts, getPlaneLights in the
// order getFinalColor sums them, src/main.cpp:174-185) until a shadow query is needed (true, query
// in q) or every light is done (false).  `vis` is the result of the cansee that just finished
// (valid when have_result).
template <bool TEX>
__device__ __forceinline__ bool advance_lights_body(const KParams& P, Lane& L, bool have_result, bool vis,
                                                    FanResult fan, Query& q) {
    const DevScene& S = P.S;
    for (;;) {
        if (L.lt == L_POINT) {
            if (have_result) {
                have_result = false;
                if (vis) {
                    const rt_point_light pl = S.pl[L.li];
                    float cosL, cosS;
                    light_cos(L, ld3(pl.position), cosL, cosS);
                    L.color += calc_color(ld3(pl.color), L.sI, cosL, cosS, render_mat<TEX>(S, L));
                }
                L.li++;
            }
            if (L.li >= S.npl) {
                L.lt = L_SPHERE;
                L.li = 0;
                L.ls = -1;
                continue;
            }
            if (start_cansee(L, ld3(S.pl[L.li].position), q)) return true;
            have_result = true;
            vis = true;
            continue;
        }
        if (L.lt == L_SPHERE) {
            if (L.li >= S.nsl) {
                L.lt = L_SPOT;
                L.li = 0;
                continue;
            }
            const rt_spherical_light sl = S.sl[L.li];
            const v3 lp = ld3(sl.position);
            if (have_result) {
                have_result = false;
                if (L.ls == -2) {
                    // the whole fan, traced by the wave (fan_sample_query): bit s of fan.vis = sample s
                    // visible, bit 0 the centre
                    if (!fan.inten) {
                        // opaque scene: every intensity is 1, so the loop's sums are these integer
                        // counts (exact in float)
                        const float nv = (float)__popcll(fan.vis >> 1);
                        L.a0 = 1.0f + nv;
                        L.a1 = (float)(fan.vis & 1ull) + nv;
                    } else {
                        // the loop's sums in its order: the centre's intensity (mutated even when
                        // blocked), then each visible sample's
                        L.a0 = fan.inten[0];
                        L.a1 = (fan.vis & 1ull) ? 1.0f : 0.0f;
                        for (int s = 1; s <= P.sl_m * P.sl_n; ++s)
                            if ((fan.vis >> s) & 1ull) {
                                L.a1 += 1.0f;
                                L.a0 += fan.inten[s];
                            }
                    }
                    L.ls = P.sl_m * P.sl_n;
                } else if (L.ls == -1) {
                    L.a0 = L.sI;  // intensitySum is the centre sample's intensity (mutated even if blocked)
                    L.a1 = vis ? 1.0f : 0.0f;
                    L.u0 = sphere_perp(L.hp, lp, sl.radius);
                    L.ls = 0;
                } else {
                    if (vis) {
                        L.a1 += 1.0f;
                        L.a0 += L.sI;
                    }
                    const int j = L.ls % P.sl_m;
                    if (j == P.sl_m - 1) {  // end of a spoke: perp = rotate * perp
                        const m3 rot = rodrigues(P.sl_sin, P.sl_1mcos, normalize(lp - L.hp));
                        L.u0 = mul(rot, L.u0);
                    }
                    L.ls++;
                }
            }
            if (L.ls >= P.sl_m * P.sl_n) {
                if (L.a1 > 0.0f) {
                    float cosL, cosS;
                    light_cos(L, lp, cosL, cosS);
                    L.color += calc_color(ld3(sl.color), L.a0 / (float)P.sl_count, cosL, cosS, render_mat<TEX>(S, L));
                }
                L.li++;
                L.ls = -1;
                continue;
            }
            if (L.ls == -1 && (P.fan & 1)) {
                // fan request: the kernel traces the centre and every sample of this light from hp
                // across the wave's lanes and resumes here with the visibility mask
                L.ls = -2;
                L.shadow = true;
                return true;
            }
            v3 target = lp;
            if (L.ls >= 0) {
                const int m = P.sl_m;
                const int j = L.ls % m;
                target = lp + ((float)(m - j) / (float)m) * L.u0;
            }
            if (start_cansee(L, target, q)) return true;
            have_result = true;
            vis = true;
            continue;
        }
        if (L.lt == L_SPOT) {
            if (have_result) {
                have_result = false;
                if (vis) {
                    const DSpot sp = S.spot[L.li];
                    float cosL, cosS;
                    light_cos(L, ld3(sp.pos), cosL, cosS);
                    L.color += calc_color(ld3(sp.color), L.sI, cosL, cosS, render_mat<TEX>(S, L));
                }
                L.li++;
            }
            if (L.li >= S.nspot) {
                L.lt = L_PLANE;
                L.li = 0;
                L.ls = -1;
                continue;
            }
            const DSpot sp = S.spot[L.li];
            const v3 lp = ld3(sp.pos);
            if (!(dot(normalize(ld3(sp.dir)), normalize(L.hp - lp)) > sp.cos_angle)) {
                L.li++;
                continue;
            }
            if (start_cansee(L, lp, q)) return true;
            have_result = true;
            vis = true;
            continue;
        }
        if (L.lt == L_PLANE) {
            if (L.li >= S.nplane) {
                L.lt = L_DONE;
                return false;
            }
            const rt_plane_light pl = S.plane[L.li];
            const int k = P.plane_k;
            const v3 w = ld3(pl.width), h = ld3(pl.height), lpos = ld3(pl.position);
            const v3 normal = normalize(cross(w, h));
            if (L.ls == -1) {
                // hit, hitCount, maxCos, intensitySum; px, py (src/shadow.cpp:259-270)
                L.a0 = 0.0f;
                L.a1 = 0.0f;
                L.a2 = 0.0f;
                L.a3 = 0.0f;
                L.u1 = lpos;
                L.u0 = lpos;
                if (dot(normalize(L.hp - (lpos + 0.5f * (w + h))), normal) > 0.0f) {
                    L.ls = 0;
                    if (P.fan & 2) {
                        // fan request: the kernel traces the light's k * k samples from hp across the
                        // wave's lanes and resumes here with their visibility and intensities
                        L.ls = -2;
                        L.shadow = true;
                        return true;
                    }
                } else {
                    L.ls = k * k;  // not in front of the light: no samples
                }
            } else if (have_result && L.ls == -2) {
                // the whole fan: the loop's accumulation replayed in sample order, each visible sample
                // with its traced intensity and the hit term its sample lane computed with the loop's
                // arithmetic (fan_plane_term); maxCos, a maximum, is order-free and came as one value
                have_result = false;
                for (int s = 0; s < k * k; ++s) {
                    if ((fan.vis >> s) & 1ull) {
                        L.a3 += fan.inten ? fan.inten[s] : 1.0f;
                        L.a0 += fan.term[s];
                        L.a1 += 1.0f;
                    }
                }
                L.a2 = fan.c2max;
                L.ls = k * k;
            } else if (have_result) {
                have_result = false;
                if (vis) {
                    const v3 px = L.u0;
                    L.a3 += L.sI;
                    const float dn = dot(normalize(L.hp - px), normal);
                    L.a0 += ((dn < 0.0f) ? 0.0f : dn) / length(L.hp - px);
                    L.a1 += 1.0f;
                    const float c2 = dot(lane_nR(L), normalize(px - L.hp));
                    L.a2 = (L.a2 < c2) ? c2 : L.a2;
                }
                const v3 dx = (1.0f / (float)(k - 1)) * w;
                L.u0 = L.u0 + dx;
                const int j = L.ls % k;
                if (j == k - 1) {
                    const v3 dy = (1.0f / (float)(k - 1)) * h;
                    L.u1 = L.u1 + dy;
                    L.u0 = L.u1;
                }
                L.ls++;
            }
            if (L.ls >= k * k) {
                if (L.a0 > 0.0f) {
                    const float li = (L.a3 / (float)(int)L.a1) * L.a0 / (float)(k * k);
                    L.color += calc_color(ld3(pl.color), li, 1.0f, L.a2, render_mat<TEX>(S, L));
                }
                L.li++;
                L.ls = -1;
                continue;
            }
            if (start_cansee(L, L.u0, q)) return true;
            have_result = true;
            vis = true;
            continue;
        }
        return false;  // L_DONE
    }
}

// the light loop as its own function: fewer live registers in the caller
template <bool TEX>
__device__ __attribute__((noinline)) bool advance_lights_call(const void* ka, Lane& L, bool have_result, bool vis,
                                                              FanResult fan, Query& q) {
    return advance_lights_body<TEX>(kernel_params(ka), L, have_result, vis, fan, q);
}

// ... the same with the lane state and query as PRIVATE-address-space references (they live in the
// calling kernel's private frame): scratch instead of flat accesses.  Used where the state machine
// is inline in the kernel (single-frame variants); inside the out-of-line advance it cost the batch
// variant spilled registers (rejected list).
#define RT_PRIV __attribute__((address_space(5)))
template <bool TEX>
__device__ __attribute__((noinline)) bool advance_lights_pcall(const void* ka, Lane RT_PRIV& L, bool have_result,
                                                               bool vis, FanResult fan, Query RT_PRIV& q) {
    return advance_lights_body<TEX>(kernel_params(ka), *(Lane*)&L, have_result, vis, fan, *(Query*)&q);
}


// ---- recursion tree ------------------------------------------------------------------------
// Next lobe sample of the glossy frame f (src/main.cpp:209-249): two uniforms per draw from the
// Philox stream (key = rng_seed, counter = (draw, pixel, sample, 0)) in place of rand(); up to
// glossy_ray_count / 4 redraws while the direction points into the surface.  Returns true with the
// sample ray in q and its lobe weight max(pow(dot(reflect, dir), shininess), 0) in cw; false when
// the lobe is done.
__device__ __forceinline__ bool glossy_next_body(const KParams& P, Lane& L, Frame& f, Query& q, float& cw) {
    const v3 r = f.d;
    v3 notr = r;
    if (r.x != 0.0f) {
        notr.y = -r.x;
        notr.x = r.y;
    } else {
        notr.y = -r.z;
        notr.z = r.y;
    }
    const v3 pr1 = cross(r, notr);
    const v3 pr2 = cross(r, pr1);
    while (++f.sample < P.glossy_n) {
        v3 sd;
        int loops = 0;
        do {
            float a, b;
            do {
                uint32_t c[4] = {L.draws++, L.rpix, (uint32_t)L.sample, 0u};
                philox4x32_10(c, P.seed_lo, P.seed_hi);
                a = u01(c[0]);
                b = u01(c[1]);
            } while (a == 0.0f && b == 0.0f && a * a + b * b < 1.0f);
            a = (2.0f * a - 1.0f) * f.gd;
            b = (2.0f * b - 1.0f) * f.gd;
            sd = normalize((r + a * pr1) + b * pr2);
            loops++;
        } while (dot(sd, f.nraw) <= 0.0f && loops < P.glossy_n / 4);
        if (dot(sd, f.nraw) > 0.0f) {
            q.o = f.o + 0.01f * sd;
            q.d = sd;
            q.t = FLT_MAX;
            cw = gmax(powf(dot(r, sd), f.shin), 0.0f);
            return true;
        }
    }
    return false;
}

__device__ __attribute__((noinline)) bool glossy_next_call(const void* ka, Lane& L, Frame& f, Query& q, float& cw) {
    return glossy_next_body(kernel_params(ka), L, f, q, cw);
}

// A getFinalColor node was hit by the path query (qo, qd): record the shading point, start its
// light loop and decide its children (src/main.cpp:131-290) -- the mirror or reflected child after
// the lights (L.desc, weight L.wc), and a frame for a pending refracted ray or a glossy lobe.
template <bool COUNT, bool TEX>
__device__ __forceinline__ void begin_node(const KParams& P, Lane& L, Frame* fr, v3 qo, v3 qd, const Best& b,
                                           Cnt& cnt) {
    const DevScene& S = P.S;
    const Surf s = surface(S, qo, qd, b, TEX, L.level == 0);
    if (COUNT) {
        cnt.hits++;
        if (s.ub) cnt.ub++;
    }
    L.hp = s.p;
    L.nN = normalize(s.n);
    L.refl = reflect(normalize(qd), L.nN);
    L.mat = (b.rec >= 0) ? s.mesh : b.rec;
    if (TEX) L.kd = v3{s.m.kd[0], s.m.kd[1], s.m.kd[2]};
    L.color = v3{0.0f, 0.0f, 0.0f};
    L.lt = L_POINT;
    L.li = 0;
    L.ls = -1;
    L.desc = false;
    if (L.level >= P.max_level) return;
    const DMat& m = s.m;
    const v3 ks{m.ks[0], m.ks[1], m.ks[2]};
    if (m.transp == 1.0f) {
        if (!(ks.x > 0.0f || ks.y > 0.0f || ks.z > 0.0f)) return;
        L.desc = true;
        if (m.shin != 0.0f) {
            // color += ks * reflectColor / glossy_ray_count (src/main.cpp:204-251)
            L.wc = L.w * ((ks * ks) / (float)P.glossy_n);
            if (P.glossy_n > 1) {
                Frame& f = fr[L.nfr++];
                f.mode = FR_GLOSSY;
                f.o = L.hp;
                f.d = L.refl;
                f.w = L.w * (ks / (float)P.glossy_n);
                f.nraw = s.n;
                f.shin = m.shin;
                f.gd = m.gd;
                f.level = L.level + 1;
                f.sample = 0;
            }
        } else {
            L.wc = L.w * (ks * ks);  // color += ks * (0 + ks * child)
        }
        return;
    }
    // transparent: Schlick Fresnel with R0 = transparency, Snell with eta = refraction_factor
    // (src/main.cpp:257-290); the reflected child first, then the refracted one (if traced)
    const v3 l = normalize(qd);
    const v3 n = L.nN;
    const float r = P.refr;
    const float c = fabsf(dot(l, n));
    v3 refr = r * l + (r * c - sqrtf(1.0f - r * r * (1.0f - c * c))) * n;
    refr = normalize(refr);
    const float R0 = m.transp;
    const float reflC = (float)((double)R0 + (double)(1.0f - R0) * pow((double)(1.0f - c), 5.0));
    const float refrC = 1.0f - reflC;
    L.desc = true;
    L.wc = L.w * reflC;
    if (r * r * (1.0f - c * c) <= 1.0f) {
        Frame& f = fr[L.nfr++];
        f.mode = FR_REFRACT;
        f.o = L.hp + 0.01f * refr;
        f.d = refr;
        f.w = L.w * refrC;
        f.level = L.level + 1;
    }
}

// The subtree under the current node is finished: resume the deepest pending branch (true, query
// in q) or report the camera sample complete (false, colour in L.acc).
__device__ __forceinline__ bool next_branch(const KParams& P, const void* ka, Lane& L, Frame* fr, Query& q) {
    while (L.nfr > 0) {
        Frame& f = fr[L.nfr - 1];
        if (f.mode == FR_REFRACT) {
            L.nfr--;
            L.level = f.level;
            L.w = f.w;
            q.o = f.o;
            q.d = f.d;
            q.t = FLT_MAX;
            return true;
        }
        float cw;
        if (glossy_next_call(ka, L, f, q, cw)) {  // reflectColor += child * cw (src/main.cpp:239-240)
            L.level = f.level;
            L.w = f.w * cw;
            return true;
        }
        L.nfr--;
    }
    return false;
}

// ---- jobs ----------------------------------------------------------------------------------
struct JobSrc {
    int mode;  // 0: pixels of the band layout, 1: explicit rays (rt_shade)
    int njobs;
    const rt_ray* rays;
    float* rgb;                      // mode 1 output [n][3]
    unsigned long long* ray_counts;  // mode 1 per-ray counts
    int* counter;                    // global job counter (zeroed per launch)
    int* xq;  // dynamic-fetch kernel, or null: 8 job heads (32-int spacing, zeroed per launch), one
              // per group of blocks sharing an XCD (blockIdx % 8), each over 1/8 of the jobs
    int n_views;    // view batch: njobs = n_views * view_jobs
    int view_jobs;  // jobs of one view (a multiple of 64)
};

// the second kernel argument of the render kernels (see kernel_params)
__device__ __forceinline__ const JobSrc& kernel_jobs(const void* ka) {
    constexpr size_t off = (sizeof(KParams) + alignof(JobSrc) - 1) / alignof(JobSrc) * alignof(JobSrc);
    return *(const JobSrc*)(uniform_kernarg(ka) + off);
}

// Job range of XCD group x: a contiguous run of 8x8 tiles (a horizontal band of the frame), so
// the rays of one XCD touch the geometry of one band and its L2 holds that part of the scene.
// A view batch keeps the split per view: range x holds band x of view 0, then band x of view 1, ...
__device__ __forceinline__ int xq_lo(const JobSrc& J, int x) {
    return J.n_views * (((x * ((J.view_jobs + 63) >> 6)) >> 3) << 6);
}

// Job index of a view batch -> (view, job inside the view): the inverse of the range layout above
// (identity for one view).
__device__ __forceinline__ int view_job(const KParams& P, int g, int& v) {
    v = 0;
    if (P.n_views <= 1) return g;
    const int nt = (P.view_jobs + 63) >> 6;
    int x = 7;
    while (x > 0 && g < P.n_views * (((x * nt) >> 3) << 6)) --x;
    const int lo = ((x * nt) >> 3) << 6;
    const int hi = x == 7 ? P.view_jobs : (((x + 1) * nt) >> 3) << 6;
    const int k = g - P.n_views * lo;
    v = k / (hi - lo);
    return lo + (k - v * (hi - lo));
}

// a new camera sample or explicit ray: the root of a fresh recursion tree
__device__ __forceinline__ void new_tree(Lane& L) {
    L.acc = v3{0.0f, 0.0f, 0.0f};
    L.w = v3{1.0f, 1.0f, 1.0f};
    L.level = 0;
    L.nfr = 0;
    L.lt = L_POINT;
    L.desc = false;
    L.draws = 0u;
    L.shadow = false;
    L.sdist = 0.0f;
}

// the camera ray of pixel rpix's camera sample `sample` (src/main.cpp:350-386); job = the pixel's job
// (its view in a batch)
__device__ __forceinline__ void camera_query(const KParams& P, int job, uint32_t rpix, int sample, Query& q) {
    const int py = (int)(rpix / (uint32_t)P.W);
    const int px = (int)(rpix - (uint32_t)py * (uint32_t)P.W);
    const float ndx = (float)px / (float)P.W * 2.0f - 1.0f;
    const float ndy = (float)py / (float)P.H * 2.0f - 1.0f;
    float sx = ndx, sy = ndy;
    if (P.aa) {
        const int s = sample;
        sx = (s == 0 || s == 2) ? ndx - P.aa_offx : ndx + P.aa_offx;
        sy = (s < 2) ? ndy + P.aa_offy : ndy - P.aa_offy;
    } else if (P.multi) {
        const int per_q = ((P.ms_moves + 1) / 2) * ((P.ms_moves + 1) / 2);
        const int qd = sample / per_q;
        const int r = sample % per_q;
        const int nyv = (P.ms_moves + 1) / 2;
        const int xx = 1 + 2 * (r / nyv);
        const int yy = 1 + 2 * (r % nyv);
        const float qx = (qd == 0 || qd == 2) ? -1.0f : 1.0f;
        const float qy = (qd < 2) ? 1.0f : -1.0f;
        sx = ndx + (P.ms_offx * qx * (float)xx);
        sy = ndy + (P.ms_offy * qy * (float)yy);
    }
    if (P.n_views > 1) {
        int view;
        view_job(P, job, view);
        gen_ray_view(P, view, sx, sy, q.o, q.d);
    } else
        gen_ray(P, sx, sy, q.o, q.d);
    q.t = FLT_MAX;
}

// queue the camera ray of the lane's current sample
__device__ __forceinline__ void queue_camera(const KParams& P, Lane& L, Query& q) {
    camera_query(P, L.job, L.rpix, L.sample, q);
    new_tree(L);
}

// Map a job index to its pixel (8x8 tiles inside the rank's bands): the reference's pixel id and the
// pixel's row in the output (band buffer or final image).  False if outside the image.
__device__ __forceinline__ bool job_pixel(const KParams& P, int gjob, uint32_t& rpix, int& out_row) {
    int view;
    int job = view_job(P, gjob, view);
    if (P.interleave && view >= P.interleave_view) {
        // groups of k = 2^interleave tiles: the group's r-th job is pixel r / nb of its tile r % nb, so the
        // 64 jobs one wave takes lie in k tiles (64 / k pixels of each), and an expensive patch of the image
        // is shared by k waves instead of held by one
        const int kl = P.interleave, nt = P.view_jobs >> 6, b = job >> (6 + kl);
        const int nb = min(1 << kl, nt - (b << kl)), r = job & ((64 << kl) - 1);
        job = (((b << kl) + r % nb) << 6) + r / nb;
    }
    const int tiles_x = (P.W + 7) / 8;
    const int tiles_y_band = (P.band_rows + 7) / 8;
    int tile = job >> 6;
    if (P.centre_first) {
        // the XCD ranges of the upper half (x < 4, rows above the centre) walked from their last tile: every
        // range starts at the rows nearest the image centre, where the long query chains are
        const int nt = P.view_jobs >> 6;
        int x = 7;
        while (x > 0 && tile < ((x * nt) >> 3)) --x;
        if (x < 4) tile = ((x * nt) >> 3) + (((x + 1) * nt) >> 3) - 1 - tile;
    }
    const int lane = job & 63;
    const int tx = tile % tiles_x;
    const int rest = tile / tiles_x;
    const int ty = rest % tiles_y_band;
    const int lb = rest / tiles_y_band;
    const int gb = lb * P.band_count + P.band_rank;
    const int row_in_band = ty * 8 + (lane >> 3);
    const int px = tx * 8 + (lane & 7);
    const int py = gb * P.band_rows + row_in_band;
    rpix = (uint32_t)(py * P.W + px);  // the reference's pixel (x, y), y up
    // band-dense rows of this rank, or the pixel's final row (setPixel: row H-1-y of view v's image,
    // src/screen.cpp:32-38) in the caller's images -- local HBM or another device's, peer-mapped
    out_row = P.out_image ? view * P.H + (P.H - 1 - py) : view * P.view_rows + lb * P.band_rows + row_in_band;
    return (px < P.W) && (row_in_band < P.band_rows) && (py < P.H) && (lb < P.n_local_bands);
}

// Start job `job` on the lane: its first query in q.  False for a padding pixel (the lane stays
// idle and fetches again).
__device__ __forceinline__ bool start_job(const KParams& P, const JobSrc& J, Lane& L, int job, Query& q) {
    L.job = job;
    L.sample = 0;
    if (J.mode == 0) {
        int out_row;
        if (!job_pixel(P, job, L.rpix, out_row)) {
            L.job = -1;
            return false;
        }
        queue_camera(P, L, q);
        return true;
    }
    const rt_ray r = J.rays[job];
    q.o = v3{r.origin[0], r.origin[1], r.origin[2]};
    q.d = v3{r.direction[0], r.direction[1], r.direction[2]};
    q.t = r.t;
    L.rpix = (uint32_t)job;
    new_tree(L);
    L.level = P.shade_level;  // getFinalColor(scene, bvh, ray, level)
    return true;
}

// One cansee segment finished (src/shadow.cpp:41-67): 1 visible, 0 blocked, 2 the next segment
// (past a transparent surface, intensity attenuated) queued in q.
__device__ __forceinline__ int cansee_step(const DevScene& S, Query& q, bool hit, const Best& b, float& sI,
                                           float& sdist) {
    if (S.all_opaque) return hit ? 0 : 1;
    if (!hit || b.t > sdist - 2.0f * 0.0005f) return 1;
    const Surf s = surface(S, q.o, q.d, b);
    if (s.m.transp != 1.0f) {
        sdist -= b.t;
        const float c = fabsf(dot(q.d, s.n));
        const float R0 = s.m.transp;
        sI = (float)((double)sI * (1.0 - ((double)R0 + (double)(1.0f - R0) * pow((double)(1.0f - c), 5.0))));
        if (sdist > 0.0005f) {
            q.o = s.p + 0.0005f * q.d;
            q.t = FLT_MAX;
            return 2;
        }
        return 1;  // loop exit without an opaque blocker
    }
    return 0;
}

// ... out of line, for the kernel's fan samples in scenes with transparent materials
__device__ __attribute__((noinline)) int cansee_step_call(const void* ka, Query& q, bool hit, const Best& b, float& sI,
                                                          float& sdist) {
    return cansee_step(kernel_params(ka).S, q, hit, b, sI, sdist);
}

// A camera sample of pixel job `job` is complete with colour acc: the pixel's samples are summed in its
// output slot in sample order (setPixel of the average, src/main.cpp:358-395).  True if the pixel has
// more samples.
__device__ __forceinline__ bool store_sample(const KParams& P, int job, int sample, v3 acc) {
    uint32_t rpix;
    int out_row;
    job_pixel(P, job, rpix, out_row);
    const int px = (int)(rpix % (uint32_t)P.W);
    float* dst = P.out + ((size_t)out_row * P.W + px) * 3;
    const int nsamples = P.aa ? 4 : (P.multi ? P.sample_size : 1);
    v3 col = acc;
    if (nsamples > 1) {
        const v3 sum = (sample == 0) ? v3{0.0f, 0.0f, 0.0f} : v3{dst[0], dst[1], dst[2]};
        col = sum + acc;
        if (sample + 1 == nsamples) col = P.aa ? col * 0.25f : col * (float)(1.0f / (float)P.sample_size);
    }
    dst[0] = col.x;
    dst[1] = col.y;
    dst[2] = col.z;
    return sample + 1 < nsamples;
}

// The state-machine advance after a finished query (q = that query's ray; hit, b = its result):
// the cansee segment loop, the light loop, the recursion tree, the camera samples and the pixel
// output.  Returns true with the next query in q (L.shadow says which kind); false when the lane's
// job is complete (L.job = -1).
template <bool COUNT, bool TEX, bool PRIVL = false>
__device__ __forceinline__ bool advance_lane(const KParams& P, const JobSrc& J, const void* ka, Lane& L, Frame* fr,
                                             bool hit, const Best& b, FanResult fan, Query& q, Cnt& cnt,
                                             uint32_t job_rays) {
    const DevScene& S = P.S;
    bool lights_have = false, lights_vis = false;
    if (L.shadow) {
        const int r = fan.done ? 1 : cansee_step(S, q, hit, b, L.sI, L.sdist);
        if (r == 2) return true;  // the next segment, same direction
        lights_have = true;
        lights_vis = r == 1;
    } else if (hit) {
        begin_node<COUNT, TEX>(P, L, fr, q.o, q.d, b, cnt);
    }
    bool more;
    if (L.shadow || hit) {
        L.shadow = false;
        if (PRIVL ? advance_lights_pcall<TEX>(ka, *(Lane RT_PRIV*)&L, lights_have, lights_vis, fan, *(Query RT_PRIV*)&q)
                  : advance_lights_call<TEX>(ka, L, lights_have, lights_vis, fan, q))
            return true;
        // every light done: the node's colour, then its mirror / reflected child
        L.acc = L.acc + L.w * L.color;
        if (L.desc) {
            L.w = L.wc;
            L.level++;
            q.o = L.hp + 0.01f * L.refl;
            q.d = L.refl;
            q.t = FLT_MAX;
            return true;
        }
        more = next_branch(P, ka, L, fr, q);
    } else {
        more = next_branch(P, ka, L, fr, q);  // a miss: getFinalColor returns black
    }
    if (more) return true;
    // camera sample complete: the pixel's samples are summed in its output slot, in sample order
    if (J.mode == 0) {
        if (store_sample(P, L.job, L.sample, L.acc)) {
            L.sample++;
            queue_camera(P, L, q);
            return true;
        }
    } else {
        J.rgb[L.job * 3 + 0] = L.acc.x;
        J.rgb[L.job * 3 + 1] = L.acc.y;
        J.rgb[L.job * 3 + 2] = L.acc.z;
        J.ray_counts[L.job] = job_rays;
    }
    L.job = -1;
    return false;
}

// The same advance as an out-of-line call: the lane's state then lives in the call's private frame
// between queries instead of in registers across the traversal loop (kernel variant bit RT_V_CALL).
template <bool COUNT, bool TEX>
__device__ __attribute__((noinline)) bool advance_lane_call(const void* ka, Lane& L, Frame* fr, bool hit, const Best& b,
                                                            FanResult fan, Query& q, Cnt& cnt, uint32_t job_rays) {
    return advance_lane<COUNT, TEX>(kernel_params(ka), kernel_jobs(ka), ka, L, fr, hit, b, fan, q, cnt, job_rays);
}

// Kernel variants (compile-time): bit 0 RT_V_CALL = state machine (and drain lane groups) out of line;
// bit 1 RT_V_NOPF = no node prefetch in the dynamic-fetch traversal; bit 2 RT_V_NOCOOP = no drain lane
// groups; bit 4 RT_V_W4 = compiled for 4 waves per SIMD (128 VGPRs) instead of 2 (256); bit 8 RT_V_FAN =
// light-sample fans.  Every variant renders the same bits; they differ in registers, spills and occupancy.
#define RT_V_CALL 1
#define RT_V_NOPF 2
#define RT_V_NOCOOP 4
#define RT_V_W4 16  // compiled for 4 waves per SIMD (128 VGPRs)
#define RT_V_FAN 256  // dynamic fetch: the spherical-light sample fans compiled in (P.fan)

#define RT_V_W3 8    // compiled for 3 waves per SIMD (168 VGPRs)
#define RT_V_REVISIT 32  // opaque / tree kernels: the re-visit group stack of the other kernels (A/B), not DIRECT
#define RT_V_CHK 64      // tree kernel: the checked build (indices validated and reported, chk_report)
#define RT_V_SPLIT 128   // opaque kernel: a node's shadow segment traced beside its mirror child (split_node)
#define RT_V_W5 512      // opaque kernel: compiled for 5 waves per SIMD (96 VGPRs; with NOCOOP its LDS fits 20 blocks)
#define RT_V_WAVES(V) (((V) & RT_V_W5) ? 5 : ((V) & RT_V_W4) ? 4 : ((V) & RT_V_W3) ? 3 : 2)

// the ray mix of counting builds: a query starts (a cansee segment or light sample, or a camera ray: level 0, not a
// segment) and ends (a camera ray that found nothing)
template <bool COUNT>
__device__ __forceinline__ void count_start(Cnt& cnt, bool shadow, uint32_t level, bool& qcam) {
    if (!COUNT) return;
    if (shadow) cnt.shad++;
    qcam = !shadow && level == 0u;
}
template <bool COUNT>
__device__ __forceinline__ void count_end(Cnt& cnt, bool qcam, bool found) {
    if (COUNT && qcam && !found) cnt.cmiss++;
}

template <bool COUNT, bool TEX, int V>
__device__ __forceinline__ bool advance_v(const KParams& P, const JobSrc& J, const void* ka, Lane& L, Frame* fr,
                                          bool hit, const Best& b, FanResult fan, Query& q, Cnt& cnt,
                                          uint32_t job_rays) {
    if constexpr ((V & RT_V_CALL) != 0)
        return advance_lane_call<COUNT, TEX>(ka, L, fr, hit, b, fan, q, cnt, job_rays);
    else
        return advance_lane<COUNT, TEX, true>(P, J, ka, L, fr, hit, b, fan, q, cnt, job_rays);
}

// ---- whole-traversal persistent kernel ------------------------------------------------------
// Refill between whole traversals: every busy lane traces its query with trace_query8, then
// advances; idle lanes take jobs (one atomic per wave).
template <bool COUNT, bool TEX, int V>
__global__ __launch_bounds__(64, RT_V_WAVES(V)) void persistent_kernel(KParams P, JobSrc J) {
    __shared__ int stack_lds[RT_STACK_SIZE * RT_WAVE];
    __shared__ int s_base;
    const int lane_id = threadIdx.x;
    int* stk = stack_lds + lane_id;
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();  // this kernel's (P, J)
    const unsigned long long t_wave0 = P.wave_trace ? wall_clock64() : 0ull;
    unsigned int wave_jobs = 0;  // jobs this wave took (wave trace)
    const DevScene& S = P.S;
    Frame fr[RT_MAX_DEPTH];
    Lane L;
    L.job = -1;
    L.shadow = false;
    L.sdist = 0.0f;
    Query q;
    Cnt cnt{};
    uint32_t job_rays = 0;  // queries of the lane's current job (rt_shade ray counts)
    bool need_trace = false;
    for (;;) {
        // ---- refill idle lanes (one atomic per wave) ----
        const bool idle = (L.job == -1);
        const unsigned long long want = __ballot(idle);
        if (want) {
            if (lane_id == __ffsll((long long)want) - 1) s_base = atomicAdd(J.counter, __popcll(want));
            wave_jobs += (unsigned int)__popcll(want);
            __builtin_amdgcn_wave_barrier();
            __syncthreads();
            const int base = s_base;
            if (idle) {
                const int job_k = base + __popcll(want & ((1ull << lane_id) - 1ull));
                if (job_k < J.njobs) {
                    need_trace = start_job(P, J, L, job_k, q);
                    job_rays = 0;
                } else {
                    L.job = -2;  // no more work for this lane
                }
            }
            __syncthreads();
        }
        const bool busy = need_trace && L.job >= 0;
        if (!__any(busy)) {
            if (!__any(L.job == -1)) break;  // every lane exhausted
            continue;
        }
        // ---- the one traversal ----
        Best b;
        bool hit = false;
        if (busy) {
            cnt.rays++;
            job_rays++;
            hit = trace_query8<COUNT, 8>(S, q.o, q.d, q.t, L.sdist - 2.0f * 0.0005f, L.shadow || P.use_bvh,
                                         L.shadow && S.all_opaque, b, stk, cnt);
            bool qcam = false;
            count_start<COUNT>(cnt, L.shadow, L.level, qcam);
            count_end<COUNT>(cnt, qcam, hit);
        }
        if (!busy) continue;
        if (COUNT && wave_leader()) cnt.wadv++;
        // ---- advance the state machine until the next query ----
        need_trace = advance_v<COUNT, TEX, V>(P, J, ka, L, fr, hit, b, FanResult{0ull, nullptr, false}, q, cnt, job_rays);
    }
    flush_counters<COUNT>(P, cnt);
    if (P.wave_trace && lane_id == 0) {  // wave trace: (start, end, jobs) per wave, 100 MHz clock
        unsigned long long* w = P.wave_trace + 8 * blockIdx.x;
        w[0] = t_wave0;
        w[1] = wall_clock64();
        w[2] = wave_jobs;
        for (int k = 3; k < 8; ++k) w[k] = 0ull;
    }
}

// ---- dynamic-fetch persistent kernel --------------------------------------------------------
// persistent_kernel above refills a lane only between whole traversals, so a wave runs every
// traversal for as long as its slowest query: on the dragon ~1/5 of the lanes are active per
// node fetch.  Here the traversal is a resumable per-lane state (Trav) advanced one node visit
// per iteration; a lane whose query completes parks as "pending", and once `refill` lanes of the
// wave are pending (or none is still tracing) the wave leaves the traversal loop, advances every
// pending lane's state machine to its next query (or next pixel), and resumes.  Every query is
// still judged with the same arithmetic and (t, key) order as trace_query8, so the image and the
// ray count are bit-identical; only the interleaving of queries within a wave changes.
#define RT_TRAV_NONE 0xFFFFFFFFu

struct Trav {
    v3 o, d, nd, inv;
    float tcull;  // closest hit: the cull distance (the best t so far); any hit: the threshold distance - 2 eps
    Best best;
    RefMask mask;
    uint32_t cur;  // node << 8 | slot mask of the node to visit next; RT_TRAV_NONE: none
    int sp;        // LDS stack depth (groups node << 8 | inner slots not yet visited)
    // postponed leaf work: the record cursor of the current range, then the hit leaf slots
    // (lh) of the last visited node whose records start at lb with 4-bit counts lc
    int rr, rk;
    uint32_t lb, lc, lh;
    bool found, ref, any;
};

__device__ __forceinline__ bool leaf_pending(const Trav& T) { return T.rk > 0 || T.lh != 0u; }

// a traversal state with nothing to walk (a lane without a query this phase)
__device__ __forceinline__ void trav_idle(Trav& T) {
    T.o = T.d = T.nd = T.inv = v3{0.0f, 0.0f, 0.0f};
    T.tcull = 0.0f;
    T.best.t = 0.0f;
    T.best.key = -1;
    T.best.rec = RT_NO_HIT;
    T.mask = RefMask{0u, 0u};
    T.cur = RT_TRAV_NONE;
    T.sp = 0;
    T.rr = T.rk = 0;
    T.lb = T.lc = T.lh = 0u;
    T.found = T.ref = T.any = false;
}

// Query setup: the prologue of trace_query8 (same thresholds and flags).
__device__ __forceinline__ void trav_init_q(const DevScene& S, bool use_bvh, v3 qo, v3 qd, float qt, bool shadow,
                                            float sdist, Trav& T) {
    T.o = qo;
    T.d = qd;
    T.nd = normalize(qd);
    T.inv = safe_inv(qd);
    T.ref = shadow || use_bvh;
    T.any = shadow && S.all_opaque;
    const float thr = sdist - 2.0f * 0.0005f;
    T.best.t = qt;
    T.best.key = -1;
    T.best.rec = RT_NO_HIT;
    T.mask = RefMask{0u, 0u};
    T.tcull = T.any ? thr : qt;  // an any-hit query's threshold (it never moves: the first hit ends it)
    T.found = false;
    T.sp = 0;
    T.lb = 0u;
    T.lc = 0u;
    T.lh = 0u;
    const float dd = dot(qd, qd);
    if (!(fabsf(dd - 1.0f) <= 4e-6f)) {  // non-unit direction: exhaustive (see traverse())
        T.rr = 0;
        T.rk = S.ntri;
        T.cur = RT_TRAV_NONE;
    } else {
        T.rr = 0;
        T.rk = 0;
        T.cur = (S.ntri > 0) ? 0xFFu : RT_TRAV_NONE;
    }
}


__device__ __forceinline__ void node_fetch(const float4* nodes, uint32_t cur, float4 (&g)[RT_NODE_F4]) {
    const float4* np = nodes + (size_t)(cur >> 8) * RT_NODE_SF4;
#pragma unroll
    for (int k = 0; k < RT_NODE_F4; ++k) g[k] = np[k];
}

// One node visit (node in g): box tests of its slots, the next node (whose 128 B are requested
// at once into g), and the hit leaf slots postponed into T.lb/lc/lh.
// PF: the node was prefetched into g by the previous visit (and the next one is prefetched here);
// otherwise it is loaded now (fewer live registers).
// Checked builds (RT_V_CHK, developer diagnosis of a fault): an index about to leave its buffer is reported
// into err[0] (the first: code << 32 | value) and err[1] (a count) and the access is skipped, so the launch
// finishes and says what it found instead of faulting.
__device__ __forceinline__ void chk_report(unsigned long long* err, uint32_t code, uint32_t value) {
    if (!err) return;
    atomicCAS(err, 0ull, ((unsigned long long)code << 32) | value);
    atomicAdd(err + 1, 1ull);
}

// DIRECT (the opaque and tree kernels): the stack holds groups of children, (child_base << 9) | (order << 8) |
// slots (the builders put the inner children in the low slots, bvh_build.h slot_order, so a child's node is
// child_base + slot), and a pop takes the group's next child at once -- front to back along the node's sort
// axis by the ray's direction (order bit) -- where the re-visit form (node << 8) | slots re-tests the parent's
// remaining slots first (one more node visit per pop).  Either walk gives the same lexicographic minimum.
// LOADED (the wavefront trace kernel): the caller issued the node's loads into g before its record test, so
// both memory round trips of a dual step overlap; nothing is prefetched
template <bool COUNT, int NW, bool PF = true, bool DIRECT = false, bool CHK = false, bool LOADED = false>
__device__ __forceinline__ void trav_node(const DevScene& S, Trav& T, int* stk, float4 (&g)[RT_NODE_F4], Cnt& cnt,
                                          unsigned long long* err = nullptr) {
    const uint32_t node = T.cur >> 8;
    if (CHK && node >= (uint32_t)S.nnodes) {
        chk_report(err, 1, T.cur);
        T.cur = RT_TRAV_NONE;
        T.rk = 0;
        T.lh = 0u;
        return;
    }
    if (!PF && !LOADED) node_fetch(S.nodes, T.cur, g);
    const float4 f0 = g[0], f1 = g[1];
    if (COUNT) {
        cnt.nodes++;
        if (wave_leader()) cnt.wnodes++;
    }
    const v3 o = T.o, inv = T.inv;
    const uint32_t w3 = __float_as_uint(f0.w);
    const uint32_t imask = __float_as_uint(f1.z) & 0xFFu;
    const uint32_t lmask = (__float_as_uint(f1.z) >> 8) & 0xFFu;
    const uint32_t child_base = __float_as_uint(f1.x);
    const float bx = pow2f(w3 & 0xFFu) * inv.x, by = pow2f((w3 >> 8) & 0xFFu) * inv.y,
                bz = pow2f((w3 >> 16) & 0xFFu) * inv.z;
    const float ax = (f0.x - o.x) * inv.x, ay = (f0.y - o.y) * inv.y, az = (f0.z - o.z) * inv.z;
    const uint32_t m = (T.cur & 0xFFu) & (imask | lmask), mi = m & imask;
    const float tcull = T.tcull;
    // every slot tested without branches: a slot is hit iff max(t0, 0) <= min(t1, tcull) (= t0 <= t1,
    // t1 >= 0, t0 <= tcull whenever a hit can still be accepted, tcull >= 0); the nearest inner hit
    // is the minimum of (clamped t0's bits, slot) keys (ordering is free: results are order-independent)
    // the near and far plane of an axis by the sign of its direction (fma is monotonic in the plane
    // value: for b > 0 the lo plane gives the smaller t, for b < 0 the hi plane, for b == 0 both are a),
    // so min/max per axis become one selection per plane word; near and far in one packed fma
    const bool sx = __float_as_uint(inv.x) >> 31, sy = __float_as_uint(inv.y) >> 31, sz = __float_as_uint(inv.z) >> 31;
    // the near and far plane words of each axis (PD dwords per plane: 8 slots of 1 or 2 bytes)
    constexpr int PD = RT_PLANES_U8 ? 2 : 4;
    auto dword = [&](int i) {
        const float4 v = g[2 + (i >> 2)];
        return __float_as_uint((i & 3) == 0 ? v.x : (i & 3) == 1 ? v.y : (i & 3) == 2 ? v.z : v.w);
    };
    uint32_t nw[3][PD], fw[3][PD];
    const bool sa[3] = {sx, sy, sz};
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int j = 0; j < PD; ++j) {
            const uint32_t lo = dword(a * PD + j), hi = dword((3 + a) * PD + j);
            nw[a][j] = sa[a] ? hi : lo;
            fw[a][j] = sa[a] ? lo : hi;
        }
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 b2x = {bx, bx}, b2y = {by, by}, b2z = {bz, bz}, a2x = {ax, ax}, a2y = {ay, ay}, a2z = {az, az};
    uint32_t hits = 0u, kbest = 0xFFFFFFFFu;
    uint32_t keys[NW];
    const uint32_t ni = __popc(imask);  // DIRECT: the inner children are slots 0 .. ni - 1 (slot_order)
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        // slot s's value in a plane's words: byte s & 3 of word s >> 2 (U8, one v_cvt_f32_ubyteN), else the half
        // word s & 1 of word s >> 1
        auto pv = [&](const uint32_t* w) {
            if constexpr (RT_PLANES_U8) return (float)((w[s >> 2] >> (8 * (s & 3))) & 0xFFu);
            else return plane_f(w[s >> 1], (s & 1) * 16);
        };
        f2 tx, ty, tz;  // (near, far)
        if constexpr (RT_PLANES_F16 && !RT_PLANES_U8) {  // one v_fma_mix_f32 per plane (the half widened inside the fma)
            tx = f2{fmaf(pv(nw[0]), bx, ax), fmaf(pv(fw[0]), bx, ax)};
            ty = f2{fmaf(pv(nw[1]), by, ay), fmaf(pv(fw[1]), by, ay)};
            tz = f2{fmaf(pv(nw[2]), bz, az), fmaf(pv(fw[2]), bz, az)};
        } else {  // integer planes: converted, then near and far in one packed fma
            tx = __builtin_elementwise_fma(f2{pv(nw[0]), pv(fw[0])}, b2x, a2x);
            ty = __builtin_elementwise_fma(f2{pv(nw[1]), pv(fw[1])}, b2y, a2y);
            tz = __builtin_elementwise_fma(f2{pv(nw[2]), pv(fw[2])}, b2z, a2z);
        }
        const float t0 = fmaxf(fmaxf(tx.x, ty.x), fmaxf(tz.x, 0.0f));
        const float t1 = fminf(fminf(tx.y, ty.y), fminf(tz.y, tcull));
        const bool h = t0 <= t1;
        hits |= h ? (1u << s) : 0u;
        const uint32_t key = (__float_as_uint(t0) & ~7u) | (uint32_t)s;
        if (DIRECT)
            keys[s] = (h && (uint32_t)s < ni) ? key : 0xFFFFFFFFu;  // reduced by a min3 tree below
        else
            kbest = (h && (mi & (1u << s))) ? min(kbest, key) : kbest;
    }
    // the ray's direction along the node's sort axis (slot_order): a group's children are taken from the
    // high slots first when it points back
    const uint32_t back = DIRECT ? ((((uint32_t)sx | ((uint32_t)sy << 1) | ((uint32_t)sz << 2)) >> ((w3 >> 24) & 3u)) & 1u) : 0u;
    if (DIRECT) {
        static_assert(NW == 8, "the key tree assumes 8 slots");
        kbest = min(min(min(keys[0], keys[1]), keys[2]), min(min(keys[3], keys[4]), keys[5]));
        kbest = min(min(kbest, keys[6]), keys[7]);
    }
    hits &= m;
    T.lb = __float_as_uint(f1.y);
    T.lc = __float_as_uint(f1.w);
    T.lh = hits & lmask;
    const uint32_t ih = hits & imask;
    if (COUNT && (T.cur & 0xFFu) != 0xFFu) {
        cnt.rv++;
        cnt.rvk += __popc(T.cur & 0xFFu);
        cnt.rvj += __popc(ih);
    }
    if (ih) {
        const uint32_t sbest = kbest & 7u;  // nearest first (the axis order for the first child too: C3 batch
                                             // 0.462 vs 0.458 ms/frame, 5.51 vs 5.35 node visits per ray)
        const uint32_t rest = ih & ~(1u << sbest);
        if (DIRECT) {
            if (rest) {
                if (CHK && T.sp >= RT_STACK8) {
                    chk_report(err, 2, (uint32_t)T.sp);
                    T.cur = RT_TRAV_NONE;
                    return;
                }
                stk[T.sp * RT_WAVE] = (int)((child_base << 9) | (back << 8) | rest);
                ++T.sp;
            }
            T.cur = ((child_base + sbest) << 8) | 0xFFu;
        } else {
            if (rest) {
                stk[T.sp * RT_WAVE] = (int)((node << 8) | rest);
                ++T.sp;
            }
            const uint32_t rank = __popc(imask & ((1u << sbest) - 1u));
            T.cur = ((child_base + rank) << 8) | 0xFFu;
        }
    } else if (T.sp > 0) {
        if (DIRECT) {
            // the group's next child: the lowest slot along the axis, or the highest for a ray going back
            const uint32_t e = (uint32_t)stk[(T.sp - 1) * RT_WAVE];
            const uint32_t m = e & 0xFFu;
            const uint32_t sl = (e & 0x100u) ? 31u - __clz(m) : (uint32_t)(__ffs(m) - 1);
            const uint32_t left = m & ~(1u << sl);
            if (left) stk[(T.sp - 1) * RT_WAVE] = (int)((e & ~0xFFu) | left);
            else --T.sp;
            T.cur = (((e >> 9) + sl) << 8) | 0xFFu;
        } else {
            --T.sp;
            T.cur = (uint32_t)stk[T.sp * RT_WAVE];
        }
    } else {
        T.cur = RT_TRAV_NONE;
    }
    if (PF && !LOADED && T.cur != RT_TRAV_NONE) node_fetch(S.nodes, T.cur, g);
}

// One postponed leaf record (the loop body of test_records).  The cursor moves to the next hit
// leaf slot when the current range is used up.  Any-hit queries drop the rest of their work on
// the first accepted candidate.
// SLAB: the reference slab tests of candidate culling decided from quotient bounds first (RT_SLAB_FILTER); rl: the
// reference BVH in LDS (RT_REF_LDS)
#ifndef RT_REF_LDS
#define RT_REF_LDS 1
#endif
template <bool COUNT, bool PIN, bool CHK = false, bool SLAB = false>
__device__ __forceinline__ void trav_record(const DevScene& S, Trav& T, Cnt& cnt, unsigned long long* err = nullptr,
                                            SlabCnt* sc = nullptr, const RefLds* rl = nullptr) {
    if (T.rk == 0) {
        const int s = __ffs(T.lh) - 1;
        T.lh &= T.lh - 1u;
        const uint32_t below = s ? (T.lc & ((1u << (4 * s)) - 1u)) : 0u;
        uint32_t nib = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
        nib = (nib * 0x01010101u) >> 24;
        T.rr = (int)(T.lb + nib);
        T.rk = (int)((T.lc >> (4 * s)) & 15u);
        if (T.rk == 0) return;
    }
    if (COUNT && sc) sc->step = 0;
    const int r = T.rr;
    T.rr = r + 1;
    T.rk--;
    if (CHK && (r < 0 || r >= S.ntri)) {
        chk_report(err, 3, (uint32_t)r);
        T.rk = 0;
        T.lh = 0u;
        return;
    }
    float4 r0, r1, r2, r3;
    load_record<PIN>(S.tri + r * 4, r0, r1, r2, r3);
    if (COUNT) {
        cnt.tris++;
        if (wave_leader()) cnt.wtris++;
    }
    float t;
    if (!tri_test(r0, r1, r2, r3, T.o, T.d, T.nd, t)) return;
    const int key = T.ref ? __float_as_int(r3.z) : __float_as_int(r3.y);
    if (T.any ? !(t <= T.tcull) : !(t < T.best.t || (t == T.best.t && key < T.best.key))) return;
    if (T.ref) {
        const uint32_t k0 = (COUNT && sc) ? __popc(T.mask.known) : 0u;
        const bool reach = (RT_REF_LDS && rl) ? leaf_reachable_lds<SLAB>(S, *rl, __float_as_int(r3.w), T.o, T.nd, T.mask)
                                              : leaf_reachable<SLAB>(S, __float_as_int(r3.w), T.o, T.nd, T.mask);
        if (COUNT && sc) {
            sc->step = __popc(T.mask.known) - k0;
            sc->slab += sc->step;
        }
        if (!reach) return;
    }
    T.best.t = t;
    T.best.key = key;
    T.best.rec = r;
    T.found = true;
    if (T.any) {
        T.rk = 0;
        T.lh = 0u;
        T.cur = RT_TRAV_NONE;
    } else {
        T.tcull = t;
    }
}

// ---- cooperative drain traversal -----------------------------------------------------------
// Once the job queue is dry a wave keeps few lanes with a query (tools/wave_trace.py: median 8
// of 64 after the queue runs dry) and each of those walks its query one node or record per
// dependent step: the frame ends with the longest such chain.  coop_group_trace gives each
// remaining query (k <= COOP_Q of them) a group of G = 64/k lanes (power of two) that walks it
// breadth first: each group lane visits one node of the group's pool per step and tests the
// records of that node's hit leaves, so a step covers up to G nodes.  Candidates are judged with
// the owner's arithmetic (tri_test, leaf_reachable) against the group's running best; the best
// is the lexicographic minimum of (t, key) and an any-hit query takes any accepted candidate, so
// every owner ends with the hit its own walk would give (tests/test_gpu_parity.py, RT_COOP=0 vs 1).
#define COOP_POOL 1024  // node groups, split between the lane groups (4 KB: with the 4-KB stack, 16 blocks fit a CU)
#define COOP_Q 16       // queries one drain traversal takes

// query hand-over through LDS: [field][COOP_Q]
enum {
    CQ_OX, CQ_OY, CQ_OZ, CQ_DX, CQ_DY, CQ_DZ, CQ_NX, CQ_NY, CQ_NZ, CQ_IX, CQ_IY, CQ_IZ,
    CQ_THR, CQ_TCULL, CQ_BT, CQ_BKEY, CQ_BREC, CQ_FLAGS, CQ_MK, CQ_MP, CQ_TOP, CQ_RR, CQ_RK, CQ_LB, CQ_LC, CQ_LH,
    CQ_N
};

__device__ __forceinline__ void coop_put(const Trav& T, int* q, int r) {
    const float f[12] = {T.o.x, T.o.y, T.o.z, T.d.x, T.d.y, T.d.z, T.nd.x, T.nd.y, T.nd.z, T.inv.x, T.inv.y, T.inv.z};
#pragma unroll
    for (int i = 0; i < 12; ++i) q[i * COOP_Q + r] = __float_as_int(f[i]);
    q[CQ_THR * COOP_Q + r] = __float_as_int(T.tcull);  // the any-hit threshold (= tcull for any-hit queries)
    q[CQ_TCULL * COOP_Q + r] = __float_as_int(T.tcull);
    q[CQ_BT * COOP_Q + r] = __float_as_int(T.best.t);
    q[CQ_BKEY * COOP_Q + r] = T.best.key;
    q[CQ_BREC * COOP_Q + r] = T.best.rec;
    q[CQ_FLAGS * COOP_Q + r] = (T.found ? 1 : 0) | (T.ref ? 2 : 0) | (T.any ? 4 : 0);
    q[CQ_MK * COOP_Q + r] = (int)T.mask.known;
    q[CQ_MP * COOP_Q + r] = (int)T.mask.pass;
    q[CQ_TOP * COOP_Q + r] = T.sp + (T.cur != RT_TRAV_NONE ? 1 : 0);
    q[CQ_RR * COOP_Q + r] = T.rr;
    q[CQ_RK * COOP_Q + r] = T.rk;
    q[CQ_LB * COOP_Q + r] = (int)T.lb;
    q[CQ_LC * COOP_Q + r] = (int)T.lc;
    q[CQ_LH * COOP_Q + r] = (int)T.lh;
}

// the owner's query after coop_group_trace: its hit, nothing left to walk
__device__ __forceinline__ void coop_get(Trav& T, const int* q, int r) {
    // every field the finished query still needs comes back from LDS, so the owner's traversal
    // registers are dead across coop_group_trace
    T.o = v3{__int_as_float(q[CQ_OX * COOP_Q + r]), __int_as_float(q[CQ_OY * COOP_Q + r]),
             __int_as_float(q[CQ_OZ * COOP_Q + r])};
    T.d = v3{__int_as_float(q[CQ_DX * COOP_Q + r]), __int_as_float(q[CQ_DY * COOP_Q + r]),
             __int_as_float(q[CQ_DZ * COOP_Q + r])};
    T.nd = v3{__int_as_float(q[CQ_NX * COOP_Q + r]), __int_as_float(q[CQ_NY * COOP_Q + r]),
              __int_as_float(q[CQ_NZ * COOP_Q + r])};
    T.best.t = __int_as_float(q[CQ_BT * COOP_Q + r]);
    T.best.key = q[CQ_BKEY * COOP_Q + r];
    T.best.rec = q[CQ_BREC * COOP_Q + r];
    const int flags = q[CQ_FLAGS * COOP_Q + r];
    T.found = (flags & 1) != 0;
    T.ref = (flags & 2) != 0;
    T.any = (flags & 4) != 0;
    T.tcull = __int_as_float(q[CQ_TCULL * COOP_Q + r]);
    T.mask.known = (uint32_t)q[CQ_MK * COOP_Q + r];
    T.mask.pass = (uint32_t)q[CQ_MP * COOP_Q + r];
    T.cur = RT_TRAV_NONE;
    T.sp = 0;
    T.rk = 0;
    T.lh = 0u;
}

__device__ __forceinline__ void lex_min(float& t, int& key, int& rec, float t2, int key2, int rec2) {
    if (t2 < t || (t2 == t && key2 < key)) {
        t = t2;
        key = key2;
        rec = rec2;
    }
}

// Box tests of the slots `slots` of one quantised BVH8 node (the arithmetic of trav_node): hit
// masks of inner and leaf children against the cull distance tc, the node's child base, record
// base and 4-bit record counts.
template <int NW>
__device__ __forceinline__ void node_slot_hits(const float4* np, v3 o, v3 inv, float tc, uint32_t slots, uint32_t& ih,
                                               uint32_t& lh, uint32_t& child_base, uint32_t& tri_base,
                                               uint32_t& counts, uint32_t& imask_out) {
    float4 g[RT_NODE_F4];
#pragma unroll
    for (int k = 0; k < RT_NODE_F4; ++k) g[k] = np[k];
    const float4 f0 = g[0], f1 = g[1];
    const uint32_t w3 = __float_as_uint(f0.w);
    const uint32_t imask = __float_as_uint(f1.z) & 0xFFu;
    const uint32_t lmask = (__float_as_uint(f1.z) >> 8) & 0xFFu;
    child_base = __float_as_uint(f1.x);
    tri_base = __float_as_uint(f1.y);
    counts = __float_as_uint(f1.w);
    imask_out = imask;
    const float bx = pow2f(w3 & 0xFFu) * inv.x, by = pow2f((w3 >> 8) & 0xFFu) * inv.y,
                bz = pow2f((w3 >> 16) & 0xFFu) * inv.z;
    const float ax = (f0.x - o.x) * inv.x, ay = (f0.y - o.y) * inv.y, az = (f0.z - o.z) * inv.z;
    const uint32_t m = slots & (imask | lmask);
    uint32_t hits = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        if (m & (1u << s)) {
            const float tlx = fmaf(node_plane(g, 0, s), bx, ax), thx = fmaf(node_plane(g, 3, s), bx, ax);
            const float tly = fmaf(node_plane(g, 1, s), by, ay), thy = fmaf(node_plane(g, 4, s), by, ay);
            const float tlz = fmaf(node_plane(g, 2, s), bz, az), thz = fmaf(node_plane(g, 5, s), bz, az);
            const float t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fminf(tlz, thz));
            const float t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fmaxf(tlz, thz));
            if (t0 <= t1 && t1 >= 0.0f && t0 <= tc) hits |= 1u << s;
        }
    }
    ih = hits & imask;
    lh = hits & lmask;
}

// exclusive prefix of v over the aligned group of G lanes; group total in `tot`
__device__ __forceinline__ int group_scan(int v, int G, int gl, int& tot) {
    int inc = v;
    for (int off = 1; off < G; off <<= 1) {
        const int u = __shfl_up(inc, off, G);
        if (gl >= off) inc += u;
    }
    tot = __shfl(inc, G - 1, G);
    return inc - v;
}

// The drain traversal.  `om`: lanes that own a query; the r-th owner's query is q[.][r] and its
// node groups (LDS stack, then the node it was about to visit) are pool[r * PC ..].  Results go
// back into q[.][r].
// Returns this lane's (node visits, record tests) and, in counting builds (STEPS), the wave's steps
// with a node visit and with record tests (a step's record tests run one after the other, so a step
// counts as many record steps as its busiest lane tests): the SIMD efficiency of tools/simd_eff.py
// counts the lane groups' steps like the traversal loop's.
template <int NW, bool STEPS = false>
__device__ __forceinline__ uint4 coop_group_trace(const float4* __restrict__ nodes, const float4* __restrict__ tri,
                                               const DRefNode* __restrict__ refn, const int* __restrict__ leaf_path,
                                               int* pool, int* q, unsigned long long om, int reserve) {
    const int lane = (int)(threadIdx.x & 63);
    const int k = __popcll(om);
    int G = 64;
    while (G > 1 && k * G > 64) G >>= 1;
    const int gi = lane / G, gl = lane % G;
    const bool in_group = gi < k;
    const int qi = in_group ? gi : 0;
    const int PC = COOP_POOL * G / 64;
    int* gpool = pool + qi * PC;
    const v3 o{__int_as_float(q[CQ_OX * COOP_Q + qi]), __int_as_float(q[CQ_OY * COOP_Q + qi]),
               __int_as_float(q[CQ_OZ * COOP_Q + qi])};
    const v3 d{__int_as_float(q[CQ_DX * COOP_Q + qi]), __int_as_float(q[CQ_DY * COOP_Q + qi]),
               __int_as_float(q[CQ_DZ * COOP_Q + qi])};
    const v3 nd{__int_as_float(q[CQ_NX * COOP_Q + qi]), __int_as_float(q[CQ_NY * COOP_Q + qi]),
                __int_as_float(q[CQ_NZ * COOP_Q + qi])};
    const v3 inv{__int_as_float(q[CQ_IX * COOP_Q + qi]), __int_as_float(q[CQ_IY * COOP_Q + qi]),
                 __int_as_float(q[CQ_IZ * COOP_Q + qi])};
    const float thr = __int_as_float(q[CQ_THR * COOP_Q + qi]);
    float tcull = __int_as_float(q[CQ_TCULL * COOP_Q + qi]);
    float bt = __int_as_float(q[CQ_BT * COOP_Q + qi]);
    int bkey = q[CQ_BKEY * COOP_Q + qi];
    int brec = q[CQ_BREC * COOP_Q + qi];
    const int flags = q[CQ_FLAGS * COOP_Q + qi];
    bool found = (flags & 1) != 0;
    const bool ref = (flags & 2) != 0, any = (flags & 4) != 0;
    RefMask rm{(uint32_t)q[CQ_MK * COOP_Q + qi], (uint32_t)q[CQ_MP * COOP_Q + qi]};
    int top = q[CQ_TOP * COOP_Q + qi];
    // the owner's postponed leaf work goes to the group's first lane
    int rr = 0, rk = 0;
    uint32_t lb = 0u, lc = 0u, lh = 0u;
    if (gl == 0) {
        rr = q[CQ_RR * COOP_Q + qi];
        rk = q[CQ_RK * COOP_Q + qi];
        lb = (uint32_t)q[CQ_LB * COOP_Q + qi];
        lc = (uint32_t)q[CQ_LC * COOP_Q + qi];
        lh = (uint32_t)q[CQ_LH * COOP_Q + qi];
    }
    uint4 n{0u, 0u, 0u, 0u};
    bool done = !in_group || (any && found);
    for (;;) {
        // ---- this lane's leaf records, against the group's best at the start of the step ----
        float ct = FLT_MAX;
        int ckey = 0x7fffffff, crec = RT_NO_HIT;
        int acc_any = 0;
        const uint32_t tests0 = n.y;
        if (!done) {
            float lt = bt;
            int lkey = bkey;
            for (;;) {
                if (rk == 0) {
                    if (!lh) break;
                    const int s = __ffs(lh) - 1;
                    lh &= lh - 1u;
                    const uint32_t below = s ? (lc & ((1u << (4 * s)) - 1u)) : 0u;
                    uint32_t nib = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
                    nib = (nib * 0x01010101u) >> 24;
                    rr = (int)(lb + nib);
                    rk = (int)((lc >> (4 * s)) & 15u);
                    continue;
                }
                const int r = rr++;
                --rk;
                float4 r0, r1, r2, r3;
                load_record(tri + (size_t)r * 4, r0, r1, r2, r3);
                n.y++;
                float t;
                if (!tri_test(r0, r1, r2, r3, o, d, nd, t)) continue;
                const int key = ref ? __float_as_int(r3.z) : __float_as_int(r3.y);
                bool acc = any ? (t <= thr) : (t < lt || (t == lt && key < lkey));
                if (acc && ref && !leaf_reachable_p(leaf_path, refn, __float_as_int(r3.w), o, nd, rm)) acc = false;
                if (!acc) continue;
                lt = t;
                lkey = key;
                ct = t;
                ckey = key;
                crec = r;
                acc_any = 1;
                if (any) {
                    rk = 0;
                    lh = 0u;
                    break;
                }
            }
        }
        if (STEPS) {  // the busiest lane's record tests of this step
            int m = (int)(n.y - tests0);
            for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
            n.w += (uint32_t)m;
        }
        // ---- group reduction (aligned xor butterfly, stays inside the group) ----
        for (int off = G >> 1; off > 0; off >>= 1) {
            const float t2 = __shfl_xor(ct, off);
            const int k2 = __shfl_xor(ckey, off), r2 = __shfl_xor(crec, off);
            acc_any |= __shfl_xor(acc_any, off);
            lex_min(ct, ckey, crec, t2, k2, r2);
        }
        if (!done && acc_any) {
            if (any) {  // any accepted candidate ends the query
                bt = ct;
                bkey = ckey;
                brec = crec;
                found = true;
                done = true;
            } else if (ct < bt || (ct == bt && ckey < bkey)) {
                bt = ct;
                bkey = ckey;
                brec = crec;
                found = true;
                tcull = bt;
            }
        }
        if (!done && top == 0) done = true;
        if (!__any(!done)) break;
        // ---- nodes: each group lane visits one node of its group's pool ----
        // breadth (up to G nodes) while `reserve` pool slots stay free, else one node per step
        // from the pool top (depth first): a visit grows the pool by at most NW - 1, and depth
        // first by at most (NW - 1) per BVH level, which the reserve covers
        int take = 0;
        if (!done) {
            take = min(G, top);
            take = max(1, min(take, (PC - reserve - top) / (NW - 1)));
        }
        const bool mine = !done && gl < take;
        if (STEPS && __any(mine)) n.z++;
        const uint32_t item = mine ? (uint32_t)gpool[top - 1 - gl] : 0u;
        if (!done) top -= take;
        __syncthreads();
        uint32_t ih = 0u, cb = 0u, imask = 0u;
        if (mine) {
            n.x++;
            node_slot_hits<NW>(nodes + (size_t)(item >> 8) * RT_NODE_SF4, o, inv, any ? thr : tcull, item & 0xFFu, ih, lh, cb,
                               lb, lc, imask);
            rk = 0;
        }
        int ti = 0;
        const int pi = group_scan(__popc(ih), G, gl, ti);
        if (!done) {
            int w = top + pi;
            for (uint32_t m = ih; m; m &= m - 1u) {
                const int s = __ffs(m) - 1;
                if (w < PC) gpool[w] = (int)(((cb + __popc(imask & ((1u << s) - 1u))) << 8) | 0xFFu);
                ++w;
            }
            top = min(PC, top + ti);
        }
        __syncthreads();
    }
    if (in_group && gl == 0) {
        q[CQ_BT * COOP_Q + gi] = __float_as_int(bt);
        q[CQ_BKEY * COOP_Q + gi] = bkey;
        q[CQ_BREC * COOP_Q + gi] = brec;
        q[CQ_FLAGS * COOP_Q + gi] = (found ? 1 : 0) | (ref ? 2 : 0) | (any ? 4 : 0);
        q[CQ_TCULL * COOP_Q + gi] = __float_as_int(tcull);
        q[CQ_MK * COOP_Q + gi] = (int)rm.known;
        q[CQ_MP * COOP_Q + gi] = (int)rm.pass;
    }
    return n;
}

// The drain traversal as an out-of-line call, for the variants whose state machine is out of line
// (RT_V_CALL): the lane groups' registers are the callee's, not added to the traversal loop's.  Every
// argument is wave-uniform and the call is made with every lane active (the phase-B loop's exits are
// wave-uniform), which the lane groups' cross-lane steps need.
template <int NW>
__device__ __attribute__((noinline)) uint4 coop_group_trace_call(const float4* __restrict__ nodes,
                                                                 const float4* __restrict__ tri,
                                                                 const DRefNode* __restrict__ refn,
                                                                 const int* __restrict__ leaf_path, int* pool, int* q,
                                                                 unsigned long long om, int reserve) {
    return coop_group_trace<NW>(nodes, tri, refn, leaf_path, pool, q, om, reserve);
}

// DIRECT stacks (trav_node): the pool entries the lane groups take, one per pending child, (node << 8) | 0xFF,
// then the node about to be visited; returns the count.  direct_pending counts them without writing.
__device__ __forceinline__ int direct_pending(const Trav& T, const int* stk) {
    int n = T.cur != RT_TRAV_NONE ? 1 : 0;
    for (int j = 0; j < T.sp; ++j) n += __popc((uint32_t)stk[j * RT_WAVE] & 0xFFu);
    return n;
}
__device__ __forceinline__ int direct_to_pool(const Trav& T, const int* stk, int* gp) {
    int n = 0;
    for (int j = 0; j < T.sp; ++j) {
        const uint32_t e = (uint32_t)stk[j * RT_WAVE];
        for (uint32_t m = e & 0xFFu; m; m &= m - 1u) gp[n++] = (int)((((e >> 9) + (uint32_t)(__ffs(m) - 1)) << 8) | 0xFFu);
    }
    if (T.cur != RT_TRAV_NONE) gp[n++] = (int)T.cur;
    return n;
}

// Epilogue of trace_query8: the spheres, after every triangle (same order and keys).
__device__ __forceinline__ void trav_finish(const DevScene& S, Trav& T) {
    if (T.any && T.found) return;
    for (int s = 0; s < S.nsph; ++s) {
        const DSph sp_ = S.sph[s];
        float t;
        if (!sphere_test(sp_, T.o, T.d, t)) continue;
        const int key = T.ref ? sp_.key_bvh : S.ntri + s;
        if (T.any ? !(t <= T.tcull) : !(t < T.best.t || (t == T.best.t && key < T.best.key))) continue;
        if (T.ref && !leaf_reachable(S, sp_.leaf, T.o, T.nd, T.mask)) continue;
        T.best.t = t;
        T.best.key = key;
        T.best.rec = -s - 1;
        T.found = true;
        if (T.any) break;
    }
}

// ---- spherical-light fans (dynamic-fetch kernel, all-opaque scenes, P.fan) -------------------
// getSpherelights (src/shadow.cpp:145-215) traces the light's centre and then sl_m * sl_n samples
// (sl_n spokes of sl_m rings) from one shading point, one cansee each.  Traced one after the other by
// the lane that owns the pixel, a 64-sample light keeps that lane busy for 64 traversals while the
// rest of the wave moves on.  Here the lane posts the light as a fan in its wave's LDS table and
// every lane whose traversal slot is free takes samples of any posted fan: the samples of one shading
// point run side by side (nearly the same nodes, so the wave stays coherent) and the pixel waits for
// one traversal's time instead of 64.  A sample is the same cansee query (fan_sample_query restates
// the loop's target arithmetic for sample s); the owner resumes with the visibility mask, and in an
// opaque scene the loop's sums are counts of visible samples, so the result is bit-identical.
#define FAN_SLOTS 8
struct FanTable {
    int owner[FAN_SLOTS];   // lane, -1 free
    int next[FAN_SLOTS];    // next sample to hand out
    int count[FAN_SLOTS];   // samples: centre + sl_m * sl_n (<= 64)
    int done[FAN_SLOTS];    // samples finished
    int traced[FAN_SLOTS];  // samples that needed a query (the owner's ray count)
    int li[FAN_SLOTS];      // the spherical light
    float hx[FAN_SLOTS], hy[FAN_SLOTS], hz[FAN_SLOTS];  // the shading point
    int plane[FAN_SLOTS];                               // 1: a plane light's k * k grid, 0: a spherical light
    unsigned long long vis[FAN_SLOTS];                  // bit s: sample s visible
    float rx[FAN_SLOTS], ry[FAN_SLOTS], rz[FAN_SLOTS];  // plane lights: the owner's normalize(reflected direction)
    unsigned int c2max[FAN_SLOTS];                      // ... the visible samples' largest specular cosine (bits)
    float inten[FAN_SLOTS][64];                         // sample s's cansee intensity (transparent scenes)
    float term[FAN_SLOTS][64];                          // plane lights: visible sample s's hit term
};

// Sample s of a fan (0: the centre; s >= 1: the loop's sample ls = s - 1): the cansee query of
// getSpherelights with the target the loop builds (its perp rotated once per finished spoke).
// False when the target is within SHADOW_ERROR_OFFSET (visible without a query).
__device__ __forceinline__ bool fan_sample_query(const KParams& P, v3 hp, int li, int plane, int s, Query& q,
                                                 float& sdist) {
    v3 target;
    if (plane) {
        // getPlaneLights' grid (src/shadow.cpp:259-299): row i = s / k, column j = s % k, px reached by
        // the loop's additions (py += dy per row, px += dx per column)
        const float4 t = P.plane_tab[li * RT_PLANE_TAB + plane_tab_at(P.plane_k, s)];
        target = v3{t.x, t.y, t.z};
    } else {
    const rt_spherical_light sl = P.S.sl[li];
    const v3 lp = ld3(sl.position);
    target = lp;
    if (s > 0) {
        const int m = P.sl_m, ls = s - 1, j = ls % m, k = ls / m;
        v3 u0 = sphere_perp(hp, lp, sl.radius);
        if (k > 0) {
            const m3 rot = rodrigues(P.sl_sin, P.sl_1mcos, normalize(lp - hp));
            for (int i = 0; i < k; ++i) u0 = mul(rot, u0);
        }
        target = lp + ((float)(m - j) / (float)m) * u0;
    }
    }
    v3 d = target - hp;  // start_cansee
    sdist = length(d);
    d = normalize(d);
    if (!(sdist > 0.0005f)) return false;
    q.o = hp + 0.0005f * d;
    q.d = d;
    q.t = FLT_MAX;
    return true;
}

// A visible sample s of plane-light fan f: its terms of getPlaneLights' sums (src/shadow.cpp:289-305)
// with the loop's own arithmetic -- px reached by the loop's additions (as fan_sample_query), the owner's
// shading point and normalize(reflect) -- so the owner's replay is a sum of finished terms in sample order
// instead of 64 serial normalisations on one lane.  maxCos = max(0, visible samples' cosines), NaN never
// taken: an atomic maximum of the positive cosines' bits (positive floats order as their bits).
__device__ __forceinline__ void fan_plane_term(const KParams& P, FanTable& ft, int f, int s) {
    const float4* tab = P.plane_tab + ft.li[f] * RT_PLANE_TAB;
    const float4 t = tab[plane_tab_at(P.plane_k, s)], nt = tab[RT_PLANE_TAB - 1];
    const v3 px{t.x, t.y, t.z};
    const v3 hp{ft.hx[f], ft.hy[f], ft.hz[f]};
    const v3 normal{nt.x, nt.y, nt.z};
    const float dn = dot(normalize(hp - px), normal);
    ft.term[f][s] = ((dn < 0.0f) ? 0.0f : dn) / length(hp - px);
    // normalize(px - hp) is -normalize(hp - px) bit for bit (a - b == -(b - a), and the products and sums of
    // the dot product and the scaling negate exactly), so its cosine is the negated dot with that vector
    const float c2 = -dot(v3{ft.rx[f], ft.ry[f], ft.rz[f]}, normalize(hp - px));
    if (c2 > 0.0f) atomicMax(&ft.c2max[f], __float_as_uint(c2));
}

// a sample of fan slot f finished: into the fan's mask, then its count (the owner reads the mask
// once the count is complete)
__device__ __forceinline__ void fan_record(FanTable& ft, int f, int s, bool vis, float inten) {
    if (vis) atomicOr(&ft.vis[f], 1ull << s);
    ft.inten[f][s] = inten;
    atomicAdd(&ft.done[f], 1);
}

template <bool COUNT, bool TEX, int V>
__global__ __launch_bounds__(64, RT_V_WAVES(V)) void persistent_df_kernel(KParams, JobSrc) {
    // drain lane groups: inline, or out of line with the out-of-line state machine (RT_V_CALL)
    constexpr bool PF = !(V & RT_V_NOPF), COOP = !(V & RT_V_NOCOOP), FANS = (V & RT_V_FAN) != 0;
    // the kernel's arguments (P, J) are read where each pass uses them (fresh_kernarg), not held in SGPRs
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
    const bool fan_on = FANS && kernel_params(ka).fan;  // (the host sets P.fan only for FANS variants)
    __shared__ int stack_lds[RT_STACK8 * RT_WAVE];
    __shared__ int coop_pool[COOP_POOL];   // drain: node groups of the wave's last queries
    __shared__ int coop_q[CQ_N * COOP_Q];  // drain: those queries
    __shared__ int s_base, s_lim;
    __shared__ FanTable ft;
    const int lane_id = threadIdx.x;
    int* stk = stack_lds + lane_id;
    const unsigned long long t_wave0 = kernel_params(ka).wave_trace ? wall_clock64() : 0ull;
    unsigned int wave_jobs = 0;  // jobs this wave took (wave trace)
    if (FANS) {
        if (lane_id < FAN_SLOTS) ft.owner[lane_id] = -1;
        __syncthreads();
    }
    __shared__ int fan_queue[RT_WAVE];  // lanes waiting for a fan slot, oldest first
    int fq_head = 0, fq_tail = 0;       // (wave-uniform)
    int fq_in = 0;                      // this lane is in the queue
    int own_fan = -1;             // fan slot this lane's state machine waits for
    bool fan_req = false;         // the state machine posted a fan, no free slot yet
    int ray_fan = -1, ray_s = 0;  // the fan sample this lane's traversal slot traces
    float ray_sI = 1.0f, ray_sdist = 0.0f;  // ... its cansee intensity and remaining distance
    Frame fr[RT_MAX_DEPTH];
    Lane L;
    L.job = -1;
    L.shadow = false;
    L.sdist = 0.0f;
    Trav T;
    Cnt cnt{};
    uint32_t job_rays = 0;                       // queries of the lane's current job (rt_shade ray counts)
    int xr = (int)(blockIdx.x & 7), xtried = 0;  // J.xq: the job range this wave draws from, ranges used up
    bool tracing = false;                        // a query is in flight
    bool qcam = false;                           // counting builds: the query in flight is a camera ray
    bool pending = false;                        // a finished query waits for advance_lane
    const int refill_at = kernel_params(ka).refill;
    // wave trace of the drain (after this wave first found the job queue empty)
    unsigned long long t_exh = 0ull;
    unsigned int it_drain = 0, lanes_drain = 0, coop_n = 0, pa_drain = 0;
    for (;;) {
        // ---- phase A: advance the pending lanes, then refill the idle ones ----
        unsigned long long tA = COUNT ? (unsigned long long)clock64() : 0ull;
        const KParams& P = *(const KParams*)fresh_kernarg(ka);
        const JobSrc& J = kernel_jobs(&P);
        const DevScene& S = P.S;
        if (COUNT && P.wave_trace && t_exh) pa_drain++;
        bool start = false;
        Query q;
        bool qshadow = false;  // the new query's kind and cansee distance
        float qsdist = 0.0f;
        // fan samples that finished: into their fan's mask
        if (FANS && pending && ray_fan >= 0) {
            pending = false;
            Query fq;
            fq.o = T.o;
            fq.d = T.d;
            const int r = S.all_opaque ? (T.found ? 0 : 1) : cansee_step_call(ka, fq, T.found, T.best, ray_sI, ray_sdist);
            if (r == 2) {  // past a transparent surface: the sample's next segment
                q = fq;
                start = true;
                qshadow = true;
                qsdist = ray_sdist;
                atomicAdd(&ft.traced[ray_fan], 1);
            } else {
                if (r == 1 && ft.plane[ray_fan]) fan_plane_term(P, ft, ray_fan, ray_s);
                fan_record(ft, ray_fan, ray_s, r == 1, ray_sI);
                ray_fan = -1;
            }
        }
        if (FANS) __syncthreads();
        // the owners of complete fans resume with the mask -- once their own traversal slot is free (a
        // lane waiting on its fan traces other fans' samples; its next query must not replace one)
        bool fan_done = false;
        FanResult fan{0ull, nullptr, false};
        if (FANS && own_fan >= 0 && !tracing && !start && ft.done[own_fan] == ft.count[own_fan]) {
            fan.vis = ft.vis[own_fan];
            fan.inten = S.all_opaque ? nullptr : ft.inten[own_fan];
            fan.term = ft.term[own_fan];
            fan.c2max = __uint_as_float(ft.c2max[own_fan]);
            fan.done = true;
            job_rays += (uint32_t)ft.traced[own_fan];
            ft.owner[own_fan] = -1;
            own_fan = -1;
            fan_done = true;
        }
        if (pending || fan_done) {
            pending = false;
            if (COUNT && wave_leader()) cnt.wadv++;
            q.o = T.o;
            q.d = T.d;
            const int jb = L.job;
            start = advance_v<COUNT, TEX, V>(P, J, ka, L, fr, T.found, T.best, fan, q, cnt, job_rays);
            if (P.job_trace && L.job == -1) {
                P.job_trace[3 * jb + 1] = wall_clock64();
                P.job_trace[3 * jb + 2] = job_rays;
            }
            if (FANS && start && L.ls == -2) {  // posted a fan
                start = false;
                fan_req = true;
            }
            qshadow = L.shadow;
            qsdist = L.sdist;
        }
        if (fan_on) {
            __syncthreads();
            // the fans posted in this pass join the wave's queue; free slots go to the oldest (in
            // lane order, a busy wave's high lanes could wait for ever)
            const bool new_req = fan_req && fq_in == 0;
            const unsigned long long nr = __ballot(new_req);
            if (nr) {
                if (new_req) {
                    fan_queue[(fq_tail + __popcll(nr & ((1ull << lane_id) - 1ull))) & (RT_WAVE - 1)] = lane_id;
                    fq_in = 1;
                }
                fq_tail += __popcll(nr);
                __syncthreads();
            }
            if (fq_head != fq_tail) {
                uint64_t freeslots = __ballot(lane_id < FAN_SLOTS && ft.owner[lane_id] < 0);
                while (fq_head != fq_tail && freeslots) {
                    const int l = fan_queue[fq_head & (RT_WAVE - 1)], f = __ffsll((long long)freeslots) - 1;
                    ++fq_head;
                    freeslots &= freeslots - 1ull;
                    if (lane_id == l) {
                        fq_in = 0;
                        ft.owner[f] = l;
                        ft.next[f] = 0;
                        ft.plane[f] = L.lt == L_PLANE ? 1 : 0;
                        ft.count[f] = L.lt == L_PLANE ? P.plane_k * P.plane_k : 1 + P.sl_m * P.sl_n;
                        ft.done[f] = 0;
                        ft.traced[f] = 0;
                        ft.vis[f] = 0ull;
                        ft.li[f] = L.li;
                        ft.hx[f] = L.hp.x;
                        ft.hy[f] = L.hp.y;
                        ft.hz[f] = L.hp.z;
                        const v3 nr = normalize(L.refl);  // (fan_plane_term's normalize(reflect), once per fan)
                        ft.rx[f] = nr.x;
                        ft.ry[f] = nr.y;
                        ft.rz[f] = nr.z;
                        ft.c2max[f] = 0u;
                        own_fan = f;
                        fan_req = false;
                    }
                }
                __syncthreads();
            }
            // samples of the posted fans to every lane whose traversal slot is free, in slot order
            const bool tfree = !tracing && !start;
            const unsigned long long fl = __ballot(tfree);
            uint64_t pend = __ballot(lane_id < FAN_SLOTS && ft.owner[lane_id] >= 0 && ft.next[lane_id] < ft.count[lane_id]);
            if (fl && pend) {
                const int nfree = __popcll(fl);
                const int rank = __popcll(fl & ((1ull << lane_id) - 1ull));
                int base = 0;
                while (pend && base < nfree) {
                    const int f = __ffsll((long long)pend) - 1;
                    pend &= pend - 1ull;
                    const int nx = ft.next[f];
                    const int take = min(ft.count[f] - nx, nfree - base);
                    if (tfree && rank >= base && rank < base + take) {
                        ray_fan = f;
                        ray_s = nx + (rank - base);
                    }
                    __syncthreads();
                    if (lane_id == 0) ft.next[f] = nx + take;
                    base += take;
                }
                __syncthreads();
            }
            if (tfree && ray_fan >= 0) {
                const v3 hp{ft.hx[ray_fan], ft.hy[ray_fan], ft.hz[ray_fan]};
                ray_sI = 1.0f;
                if (fan_sample_query(P, hp, ft.li[ray_fan], ft.plane[ray_fan], ray_s, q, qsdist)) {
                    start = true;
                    qshadow = true;
                    ray_sdist = qsdist;
                    atomicAdd(&ft.traced[ray_fan], 1);
                } else {  // visible without a query
                    if (ft.plane[ray_fan]) fan_plane_term(P, ft, ray_fan, ray_s);
                    fan_record(ft, ray_fan, ray_s, true, 1.0f);
                    ray_fan = -1;
                }
            }
            __syncthreads();
        }
        const unsigned long long tJ = COUNT ? (unsigned long long)clock64() : 0ull;
        if (COUNT) cnt.cyc_c += tJ - tA;  // state machine
        // a wave whose pixels wait on P.fan_cap fans takes no new pixels: its free lanes trace fan
        // samples, so a cluster of expensive pixels is spread over the wave's lanes instead of each
        // lane carrying one pixel's samples alone (and a wave holds few expensive pixels when the
        // job queue runs dry)
        const bool fan_full = fan_on && __popcll(__ballot(own_fan >= 0 || fan_req)) >= P.fan_cap;
        const bool idle = (L.job == -1) && !start && !tracing && !fan_full;
        const unsigned long long want = __ballot(idle);
        if (want) {
            const int nwant = __popcll(want);
            if (lane_id == __ffsll((long long)want) - 1) {
                if (J.xq) {
                    const int lo = xq_lo(J, xr);
                    s_base = lo + atomicAdd(J.xq + 32 * xr, nwant);
                    s_lim = xr == 7 ? J.njobs : xq_lo(J, xr + 1);
                } else {
                    s_base = atomicAdd(J.counter, nwant);
                    s_lim = J.njobs;
                }
            }
            wave_jobs += (unsigned int)nwant;
            __builtin_amdgcn_wave_barrier();
            __syncthreads();
            const int base = s_base, lim = s_lim;
            if (J.xq && base + nwant >= lim) {  // this group's range is used up: go on to the next
                xr = (xr + 1) & 7;
                ++xtried;
            }
            if (idle) {
                const int job_k = base + __popcll(want & ((1ull << lane_id) - 1ull));
                if (job_k < lim) {
                    if (P.job_trace) P.job_trace[3 * job_k] = wall_clock64();
                    start = start_job(P, J, L, job_k, q);
                    qshadow = false;
                    qsdist = 0.0f;
                    job_rays = 0;
                } else {
                    L.job = (J.xq && xtried < 8) ? -1 : -2;  // -2: no more work for this lane
                }
            }
            __syncthreads();
        }
        if (COUNT) cnt.cyc_d += (unsigned long long)clock64() - tJ;  // job fetch and camera rays
        if (start) {
            cnt.rays++;
            count_start<COUNT>(cnt, qshadow, L.level, qcam);
            if (ray_fan < 0) job_rays++;  // a fan sample counts for its owner's job (ft.traced)
            trav_init_q(S, P.use_bvh != 0, q.o, q.d, q.t, qshadow, qsdist, T);
            tracing = true;
        }
        if (P.wave_trace && !t_exh && __any(L.job == -2)) t_exh = wall_clock64();
        // device-wide fans with samples not yet handed out (waves out of pixels stay to take them)
        if (!__any(tracing)) {
            if (!__any(L.job == -1 || pending || own_fan >= 0 || fan_req)) break;  // every lane exhausted
            continue;
        }
        const bool fans = fan_on && __any(own_fan >= 0 || fan_req);  // lanes of exhausted waves take samples
        // ---- phase B: one node visit or one leaf record per lane and iteration ("if-if"), until
        // enough lanes wait for phase A ----
        unsigned long long tB = 0ull;
        if (COUNT) {
            tB = (unsigned long long)clock64();
            cnt.cyc_a += tB - tA;
        }
        float4 g[RT_NODE_F4];
        if (PF && tracing && T.cur != RT_TRAV_NONE) node_fetch(S.nodes, T.cur, g);
        bool coop_now = false;
        for (;;) {
            if (COUNT) {
                const int ntr = __popcll(__ballot(tracing));  // (wave-wide: before the leader branch)
                if (wave_leader()) cnt.hist[min((ntr - 1) >> 4, 2)]++;
            }
            if (tracing) {
                // a lane whose hit leaf slots are all taken (lh == 0) visits its next node in the
                // same step as its current record (P.dual): both code paths run in every step a
                // wave has lanes in each, so this fills lanes that would idle in one of them
                const bool rec = leaf_pending(T);
                if (rec) trav_record<COUNT, !(V & RT_V_W4)>(S, T, cnt);
                const bool nv = T.cur != RT_TRAV_NONE && (!rec || (P.dual && T.lh == 0u));
                if (nv) trav_node<COUNT, 8, PF>(S, T, stk, g, cnt);
            }
            if (tracing && !leaf_pending(T) && T.cur == RT_TRAV_NONE) {
                trav_finish(S, T);
                count_end<COUNT>(cnt, qcam, T.found);
                tracing = false;
                pending = true;
            }
            if (!__any(tracing)) break;
            if (__popcll(__ballot(pending || L.job == -1 || (!tracing && (fans || own_fan >= 0 || fan_req)))) >= refill_at)
                break;
            if (COUNT && P.wave_trace && t_exh) {
                it_drain++;
                lanes_drain += (unsigned int)__popcll(__ballot(tracing));
            }
            // drain (no lane can take a new job): the remaining queries go to lane groups
            // (coop 2: also in steady state, for the last queries a full-wave refill waits for); the
            // lane groups run after the loop, so their registers do not add to the traversal loop's
            if (COOP && P.coop && ((P.coop == 2 && refill_at == 64) || (!__any(L.job == -1) && __any(L.job == -2))) &&
                __popcll(__ballot(tracing)) <= P.coop_max) {
                coop_now = true;
                break;
            }
        }
        if (COOP && coop_now) {
            const unsigned long long om = __ballot(tracing);
            const int k = __popcll(om);
            int G = 64;
            while (G > 1 && k * G > 64) G >>= 1;
            const int r = __popcll(om & ((1ull << lane_id) - 1ull));
            if (tracing) {
                coop_put(T, coop_q, r);
                int* gp = coop_pool + r * (COOP_POOL * G / 64);
                for (int j = 0; j < T.sp; ++j) gp[j] = stk[j * RT_WAVE];
                if (T.cur != RT_TRAV_NONE) gp[T.sp] = (int)T.cur;
            }
            __syncthreads();
            const uint4 nv =
                (V & RT_V_CALL) ? coop_group_trace_call<8>(S.nodes, S.tri, S.refn, S.leaf_path, coop_pool, coop_q, om,
                                                           P.coop_reserve)
                                : coop_group_trace<8, COUNT>(S.nodes, S.tri, S.refn, S.leaf_path, coop_pool, coop_q, om,
                                                             P.coop_reserve);
            __syncthreads();
            if (COUNT) {
                cnt.nodes += nv.x;
                cnt.tris += nv.y;
                if (wave_leader()) {
                    cnt.wnodes += nv.z;
                    cnt.wtris += nv.w;
                }
            }
            if (tracing) {
                coop_get(T, coop_q, r);
                trav_finish(S, T);
                count_end<COUNT>(cnt, qcam, T.found);
                tracing = false;
                pending = true;
            }
            if (COUNT && P.wave_trace) coop_n++;
        }
        if (COUNT) cnt.cyc_b += (unsigned long long)clock64() - tB;
    }
    const KParams& P = kernel_params(ka);
    flush_counters<COUNT>(P, cnt);
    if (P.wave_trace && lane_id == 0) {  // wave trace, 100 MHz clock: start, end, jobs, drain
        unsigned long long* w = P.wave_trace + 8 * blockIdx.x;
        w[0] = t_wave0;
        w[1] = wall_clock64();
        w[2] = wave_jobs;
        w[3] = t_exh;
        w[4] = it_drain;
        w[5] = lanes_drain;
        w[6] = coop_n;
        w[7] = pa_drain;
    }
}

// ---- the opaque-scene kernel: point and spot lights, mirror recursion --------------------------
// getFinalColor (src/main.cpp:129-301) on a scene whose materials are all opaque (transparency == 1),
// lit only by point and spot lights (src/shadow.cpp:106-131,229-252), without glossy lobes
// (glossy_ray_count == 1) or textures: every node has at most one child (the ks^2-weighted mirror ray)
// and every shadow query is an any-hit cansee of one segment.  The recursion tree is then a chain, the
// light loop a cursor over the point then the spot lights, and the whole per-lane state -- pixel, camera
// sample, recursion level, colour and weights, the shading point -- is 24 dwords that stay in registers:
// the state machine runs inline between traversal steps, with no private-memory frame and no call.
// Its arithmetic is the general state machine's (begin_node, advance_lights_body, the forward colour
// fold), so the image and the ray count are bit-identical (tests/test_gpu_parity.py variant matrix).
struct LiteLane {
    int job;        // >= 0 job; -1 idle (fetch another); -2 no more work (the pixel: job_pixel)
    uint32_t sample : 7;  // camera sample
    uint32_t level : 5;   // recursion level of the current node
    uint32_t desc : 1;    // the current node descends to its mirror child after its lights
    uint32_t shadow : 1;  // the query in flight is a cansee segment
    uint32_t li : 18;     // light cursor: point lights [0, npl), then spot lights
    v3 acc, w;            // sample colour, weight of the current node (its mirror child's: lite_child_weight)
    v3 hp, nN, refl;      // shading point, normalize(normal), reflect
    int mat;              // >= 0 mesh material, < 0 sphere -(s+1)
    v3 color;             // direct light of the current node
};

// The next light of the cursor that needs a cansee segment (true, query in q, cursor on it), or false
// when the node's lights are done.  Lights whose target lies within SHADOW_ERROR_OFFSET are visible
// without a query (src/shadow.cpp:38-40) and spot lights outside their cone contribute nothing
// (src/shadow.cpp:235-237).
template <bool COUNT>
__device__ __forceinline__ bool lite_next_light(const KParams& P, LiteLane& L, Query& q, float& sdist) {
    const DevScene& S = P.S;
    const int nl = S.npl + S.nspot;
    while ((int)L.li < nl) {
        v3 lp, lc;
        if ((int)L.li < S.npl) {
            const rt_point_light pl = S.pl[L.li];
            lp = ld3(pl.position);
            lc = ld3(pl.color);
        } else {
            const DSpot sp = S.spot[L.li - S.npl];
            lp = ld3(sp.pos);
            lc = ld3(sp.color);
            if (!(dot(normalize(ld3(sp.dir)), normalize(L.hp - lp)) > sp.cos_angle)) {
                L.li++;
                continue;
            }
        }
        v3 d = lp - L.hp;  // start_cansee
        sdist = length(d);
        d = normalize(d);
        if (sdist > 0.0005f) {
            q.o = L.hp + 0.0005f * d;
            q.d = d;
            q.t = FLT_MAX;
            return true;
        }
        // visible without a query (cansee's loop condition fails at once): the light counts at once
        const v3 ldir = normalize(lp - L.hp);
        const float cosL = fabsf(dot(L.nN, ldir));
        const float d2 = dot(normalize(L.refl), ldir);
        L.color += calc_color(lc, 1.0f, cosL, (0.0f < d2) ? d2 : 0.0f, load_mat(S, L.mat));
        L.li++;
    }
    return false;
}

// the light under the cursor was visible: its calcColor into the node's colour
__device__ __forceinline__ void lite_light_visible(const KParams& P, LiteLane& L) {
    const DevScene& S = P.S;
    v3 lp, lc;
    if ((int)L.li < S.npl) {
        const rt_point_light pl = S.pl[L.li];
        lp = ld3(pl.position);
        lc = ld3(pl.color);
    } else {
        const DSpot sp = S.spot[L.li - S.npl];
        lp = ld3(sp.pos);
        lc = ld3(sp.color);
    }
    const v3 ldir = normalize(lp - L.hp);
    const float cosL = fabsf(dot(L.nN, ldir));
    const float d2 = dot(normalize(L.refl), ldir);
    L.color += calc_color(lc, 1.0f, cosL, (0.0f < d2) ? d2 : 0.0f, load_mat(S, L.mat));
}

// color += ks * reflectColor (/ glossy_ray_count with shininess): the mirror child's weight from the node's
// weight (unchanged since its begin_node) and material, evaluated when the node descends rather than kept
__device__ __forceinline__ v3 lite_child_weight(const KParams& P, const LiteLane& L) {
    const DMat m = load_mat(P.S, L.mat);
    const v3 ks{m.ks[0], m.ks[1], m.ks[2]};
    return (m.shin != 0.0f) ? L.w * ((ks * ks) / (float)P.glossy_n) : L.w * (ks * ks);
}

// The state-machine advance of the opaque-scene kernel after a finished query (q = its ray, hit / b =
// its result): true with the next query in q (sdist: its cansee distance), false when the job is done.
template <bool COUNT>
__device__ __forceinline__ bool lite_advance(const KParams& P, LiteLane& L, bool hit, const Best& b, Query& q,
                                             float& sdist, Cnt& cnt) {
    const DevScene& S = P.S;
    bool node_done;
    if (L.shadow) {
        // cansee in an opaque scene: visible iff no candidate at t <= distance - 2 * SHADOW_ERROR_OFFSET
        if (!hit) lite_light_visible(P, L);
        L.li++;
        L.shadow = false;
        node_done = true;
    } else if (hit) {
        // begin_node (src/main.cpp:131-256), the opaque branch
        const Surf s = surface(S, q.o, q.d, b, false, L.level == 0);
        if (COUNT) {
            cnt.hits++;
            if (s.ub) cnt.ub++;
        }
        L.hp = s.p;
        L.nN = normalize(s.n);
        L.refl = reflect(normalize(q.d), L.nN);
        L.mat = (b.rec >= 0) ? s.mesh : b.rec;
        L.color = v3{0.0f, 0.0f, 0.0f};
        L.li = 0;
        L.desc = false;
        if (L.level < P.max_level) {
            const v3 ks{s.m.ks[0], s.m.ks[1], s.m.ks[2]};
            if (ks.x > 0.0f || ks.y > 0.0f || ks.z > 0.0f) L.desc = true;
        }
        node_done = true;
    } else {
        node_done = false;  // a miss: getFinalColor returns black, the camera sample is complete
    }
    if (node_done) {
        if (lite_next_light<COUNT>(P, L, q, sdist)) {
            L.shadow = true;
            return true;
        }
        L.acc = L.acc + L.w * L.color;  // every light done: the node's colour, then its mirror child
        if (L.desc) {
            L.w = lite_child_weight(P, L);
            L.level++;
            q.o = L.hp + 0.01f * L.refl;
            q.d = L.refl;
            q.t = FLT_MAX;
            return true;
        }
    }
    // camera sample complete
    if (store_sample(P, L.job, L.sample, L.acc)) {
        L.sample++;
        uint32_t rpix;
        int out_row;
        job_pixel(P, L.job, rpix, out_row);
        camera_query(P, L.job, rpix, L.sample, q);
        L.acc = v3{0.0f, 0.0f, 0.0f};
        L.w = v3{1.0f, 1.0f, 1.0f};
        L.level = 0;
        L.desc = false;
        L.shadow = false;
        return true;
    }
    L.job = -1;
    return false;
}

// ---- SPLIT: a node's shadow segment traced beside its mirror child (RT_V_SPLIT) ----
// The lane above walks its pixel's chain one query per full-wave phase: camera ray, the node's cansee segment,
// the mirror ray, its segment, ... -- 2 (max_level + 1) dependent phases, so a single frame ends with the waves
// that hold the longest chains (profiles/r04/job_trace_C3_frame_interleave16.log: a job started at 5 us ends
// with the frame).  The segment does not feed the chain: a node's colour needs its visibility, the mirror ray
// does not.  With one light (point or spot) the lane writes each node's shading point, material and light term
// (the light's calcColor, were it visible) to a per-lane frame in device memory, posts the segment and walks on
// with the mirror ray; a free lane of the wave (its job done, or the owner itself once its chain has ended)
// traces the segment and sets the node's result bits in LDS.  When the chain has ended and every segment is
// resolved, the owner folds its nodes in level order with the same expressions as lite_advance -- colour =
// 0 + term if visible, acc = acc + w * colour, w = lite_child_weight -- and stores the sample, so the values,
// their order and the ray count are unchanged.  Between phases the lane keeps 3 dwords instead of LiteLane's 24.
struct SplitLane {
    int job;                 // >= 0 job; -1 idle (fetch another or take a segment); -2 no more work
    uint32_t sample : 7;     // camera sample
    uint32_t level : 5;      // level of the node the lane's own query looks for
    uint32_t cdone : 1;      // the sample's mirror chain has ended (segments may be outstanding)
    uint32_t tk : 1;         // the query in flight is the segment of lane tk_owner's node tk_level
    uint32_t tk_owner : 6;
    uint32_t tk_level : 4;
    uint32_t nlev : 5;       // nodes of the sample in the frame: levels 0 .. nlev - 1
    uint32_t untaken : 16;   // levels whose segment is posted and not taken
    uint32_t posted : 16;    // levels with a segment
};

// frame of lane `lane`'s node `level`: (shading point, material), (colour, or the light term of a posted segment)
__device__ __forceinline__ float4* split_frame(const KParams& P, int lane, int level) {
    return P.frames + ((size_t)level * P.frame_slots + blockIdx.x * RT_WAVE + lane) * 2;
}

// the scene's one light (src/shadow.cpp: point lights first, then spot lights)
__device__ __forceinline__ void split_light(const DevScene& S, v3& lp, v3& lc) {
    if (S.npl > 0) {
        const rt_point_light pl = S.pl[0];
        lp = ld3(pl.position);
        lc = ld3(pl.color);
    } else {
        const DSpot sp = S.spot[0];
        lp = ld3(sp.pos);
        lc = ld3(sp.color);
    }
}

// start_cansee toward the light (lite_next_light): false if the light lies within SHADOW_ERROR_OFFSET
__device__ __forceinline__ bool split_segment(v3 hp, v3 lp, Query& q, float& sdist) {
    v3 d = lp - hp;
    sdist = length(d);
    d = normalize(d);
    if (!(sdist > 0.0005f)) return false;
    q.o = hp + 0.0005f * d;
    q.d = d;
    q.t = FLT_MAX;
    return true;
}

// the i-th (0-based) set bit of m (i < popcount(m))
__device__ __forceinline__ int nth_set(uint64_t m, int i) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const int c = __popcll(m & ((1ull << w) - 1ull));
        if (i >= c) {
            i -= c;
            m >>= w;
            pos += w;
        }
    }
    return pos;
}

// The lane's own query (camera or mirror ray) finished: its node into the frame, its segment posted, and true
// with the mirror ray in q; false when the chain ends (a miss, the last level, or no specular colour).
template <bool COUNT>
__device__ __forceinline__ bool split_node(const KParams& P, SplitLane& L, int lane, bool hit, const Best& b, Query& q,
                                           Cnt& cnt) {
    const DevScene& S = P.S;
    if (!hit) {
        L.cdone = 1;
        return false;
    }
    const Surf s = surface(S, q.o, q.d, b, false, L.level == 0);
    if (COUNT) {
        cnt.hits++;
        if (s.ub) cnt.ub++;
    }
    const v3 hp = s.p, nN = normalize(s.n), refl = reflect(normalize(q.d), nN);
    const int mat = (b.rec >= 0) ? s.mesh : b.rec;
    v3 lp, lc, color{0.0f, 0.0f, 0.0f};
    split_light(S, lp, lc);
    bool post = false;
    const bool lit = (S.npl > 0) || dot(normalize(ld3(S.spot[0].dir)), normalize(hp - lp)) > S.spot[0].cos_angle;
    if (lit) {
        Query sq;
        float sd;
        post = split_segment(hp, lp, sq, sd);
        const v3 ldir = normalize(lp - hp);  // lite_light_visible
        const float cosL = fabsf(dot(nN, ldir));
        const float d2 = dot(normalize(refl), ldir);
        const v3 t = calc_color(lc, 1.0f, cosL, (0.0f < d2) ? d2 : 0.0f, load_mat(S, mat));
        if (post) color = t;   // folded as 0 + t once the segment finds the light visible
        else color += t;       // visible without a query
    }
    float4* f = split_frame(P, lane, L.level);
    f[0] = make_float4(hp.x, hp.y, hp.z, __int_as_float(mat));
    f[1] = make_float4(color.x, color.y, color.z, 0.0f);
    if (post) {
        L.untaken |= 1u << L.level;
        L.posted |= 1u << L.level;
    }
    L.nlev = L.level + 1;
    if (L.level < P.max_level) {
        const v3 ks{s.m.ks[0], s.m.ks[1], s.m.ks[2]};
        if (ks.x > 0.0f || ks.y > 0.0f || ks.z > 0.0f) {
            L.level++;
            q.o = hp + 0.01f * refl;
            q.d = refl;
            q.t = FLT_MAX;
            return true;
        }
    }
    L.cdone = 1;
    return false;
}

// the posted segment of lane `owner`'s node `level`, rebuilt from its shading point
__device__ __forceinline__ void split_take(const KParams& P, int owner, int level, Query& q, float& sdist) {
    const float4 a = split_frame(P, owner, level)[0];
    v3 lp, lc;
    split_light(P.S, lp, lc);
    split_segment(v3{a.x, a.y, a.z}, lp, q, sdist);
}

// the sample's colour: its nodes in level order (lite_advance's fold; res: LDS result bits, done | visible << 16)
__device__ __forceinline__ v3 split_fold(const KParams& P, const SplitLane& L, int lane, uint32_t res) {
    v3 acc{0.0f, 0.0f, 0.0f}, w{1.0f, 1.0f, 1.0f};
    for (int l = 0; l < (int)L.nlev; ++l) {
        const float4* f = split_frame(P, lane, l);
        const float4 a = f[0], c = f[1];
        v3 color{c.x, c.y, c.z};
        if ((L.posted >> l) & 1u) {
            const v3 zero{0.0f, 0.0f, 0.0f};
            color = ((res >> (16 + l)) & 1u) ? zero + color : zero;
        }
        acc = acc + w * color;
        if (l + 1 < (int)L.nlev) {  // lite_child_weight of node l
            const DMat m = load_mat(P.S, __float_as_int(a.w));
            const v3 ks{m.ks[0], m.ks[1], m.ks[2]};
            w = (m.shin != 0.0f) ? w * ((ks * ks) / (float)P.glossy_n) : w * (ks * ks);
        }
    }
    return acc;
}

template <bool COUNT, int V>
__global__ __launch_bounds__(64, RT_V_WAVES(V)) void persistent_opaque_kernel(KParams, JobSrc) {
    constexpr bool PF = !(V & RT_V_NOPF), COOP = !(V & RT_V_NOCOOP), DIRECT = !(V & RT_V_REVISIT);
    constexpr bool SPLIT = (V & RT_V_SPLIT) != 0;
    // the kernel's arguments are read where each phase uses them (fresh_kernarg), not held in SGPRs
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
#define RT_FRESH const KParams& P = *(const KParams*)fresh_kernarg(ka); const DevScene& S = P.S
    __shared__ int stack_lds[RT_STACK8 * RT_WAVE];
    __shared__ int coop_pool[COOP ? COOP_POOL : 1];   // drain lane groups (COOP): node groups of the wave's last queries
    __shared__ int coop_q[COOP ? CQ_N * COOP_Q : 1];  // ... and those queries
    __shared__ int s_base, s_lim;
    __shared__ RefLds ref_lds;             // the reference BVH's boxes and leaf paths (candidate culling)
    __shared__ uint32_t split_res[SPLIT ? RT_WAVE : 1];  // SPLIT: per owner lane, segments done | visible << 16
    const int lane_id = threadIdx.x;
    int* stk = stack_lds + lane_id;
    if (RT_REF_LDS) {
        ref_lds_load(kernel_params(ka).S, ref_lds, lane_id);
        __syncthreads();
    }
    const unsigned long long t_wave0 = (COUNT && kernel_params(ka).wave_trace) ? wall_clock64() : 0ull;
    unsigned int wave_jobs = 0;
    std::conditional_t<SPLIT, SplitLane, LiteLane> L;
    L.job = -1;
    if constexpr (SPLIT) {
        L.tk = 0;
        L.cdone = 0;
        L.untaken = L.posted = 0;
    } else {
        L.shadow = false;
    }
    Trav T;
    Cnt cnt{};
    SlabCnt slab{};
    int xr = (int)(blockIdx.x & 7), xtried = 0;
    bool tracing = false, pending = false;
    bool qcam = false;  // counting builds: the query in flight is a camera ray
    unsigned long long t_exh = 0ull;
    unsigned int it_drain = 0, lanes_drain = 0, coop_n = 0, pa_drain = 0;  // wave trace, counting builds only
    uint32_t qn0 = 0, qr0 = 0;  // counting builds: the lane's node / record counts when its query started
    uint32_t nph = 0;           // counting builds with a phase trace: the wave's traversal phases so far
    for (;;) {
        // ---- phase A: advance the pending lanes, then refill the idle ones ----
        unsigned long long tA = COUNT ? (unsigned long long)clock64() : 0ull;
        RT_FRESH;
        const JobSrc& J = kernel_jobs(&P);
        if (COUNT && P.wave_trace && t_exh) pa_drain++;
        bool start = false, qshadow = false;
        Query q;
        float qsdist = 0.0f;
        if constexpr (SPLIT) {
            if (COUNT) {
                const bool ap = __any(pending);
                if (ap && wave_leader()) cnt.wadv++;
            }
            // a taken segment finished: its visibility to the owner (visible iff no candidate)
            if (pending && L.tk) {
                pending = false;
                atomicOr(&split_res[L.tk_owner], (1u << L.tk_level) | (T.found ? 0u : (1u << (16 + L.tk_level))));
                L.tk = 0;
            }
            __syncthreads();
            // the lane's own camera / mirror query finished: its node into the frame, the mirror ray next
            if (pending) {
                pending = false;
                q.o = T.o;
                q.d = T.d;
                start = split_node<COUNT>(P, L, lane_id, T.found, T.best, q, cnt);
            }
            // the chain has ended: its own untaken segments first, then the fold once every segment is resolved
            if (L.job >= 0 && L.cdone && !start) {
                if (L.untaken) {
                    const int lv = __ffs(L.untaken) - 1;
                    L.untaken &= L.untaken - 1u;
                    split_take(P, lane_id, lv, q, qsdist);
                    L.tk = 1;
                    L.tk_owner = lane_id;
                    L.tk_level = lv;
                    start = qshadow = true;
                } else {
                    const uint32_t r = split_res[lane_id];
                    if ((r & 0xFFFFu) == L.posted) {
                        const v3 acc = split_fold(P, L, lane_id, r);
                        const int jb = L.job;
                        if (store_sample(P, L.job, L.sample, acc)) {
                            L.sample++;
                            uint32_t rpix;
                            int out_row;
                            job_pixel(P, L.job, rpix, out_row);
                            camera_query(P, L.job, rpix, L.sample, q);
                            L.level = 0;
                            L.cdone = 0;
                            L.nlev = 0;
                            L.untaken = L.posted = 0;
                            split_res[lane_id] = 0u;
                            start = true;
                        } else {
                            L.job = -1;
                            if (COUNT && P.job_trace) P.job_trace[3 * jb + 1] = wall_clock64();
                        }
                    }
                }
            }
            // free lanes take posted segments: the oldest of each owner, owners in lane order
            {
                const bool fr = L.job < 0 && !start;
                const uint32_t ut = L.untaken;
                const unsigned long long om = __ballot(ut != 0u), fm = __ballot(fr);
                if (om && fm) {
                    const int n = min(__popcll(om), __popcll(fm));
                    const int rf = __popcll(fm & ((1ull << lane_id) - 1ull));
                    const int ro = __popcll(om & ((1ull << lane_id) - 1ull));
                    const int owner = nth_set(om, (fr && rf < n) ? rf : 0);
                    const uint32_t out = (uint32_t)__shfl((int)ut, owner);
                    if (fr && rf < n) {
                        const int lv = __ffs(out) - 1;
                        split_take(P, owner, lv, q, qsdist);
                        L.tk = 1;
                        L.tk_owner = owner;
                        L.tk_level = lv;
                        start = qshadow = true;
                    }
                    if (ut && ro < n) L.untaken = ut & (ut - 1u);
                }
            }
        } else if (pending) {
            pending = false;
            if (COUNT && wave_leader()) cnt.wadv++;
            q.o = T.o;
            q.d = T.d;
            const int jb = L.job;
            start = lite_advance<COUNT>(P, L, T.found, T.best, q, qsdist, cnt);
            qshadow = L.shadow;
            if (COUNT && P.job_trace && L.job == -1) P.job_trace[3 * jb + 1] = wall_clock64();
        }
        const unsigned long long tJ = COUNT ? (unsigned long long)clock64() : 0ull;
        if (COUNT) cnt.cyc_c += tJ - tA;
        const bool idle = (L.job == -1) && !start && !tracing;
        const unsigned long long want = __ballot(idle);
        if (want) {
            const int nwant = __popcll(want);
            if (lane_id == __ffsll((long long)want) - 1) {
                const int lo = xq_lo(J, xr);
                s_base = lo + atomicAdd(J.xq + 32 * xr, nwant);
                s_lim = xr == 7 ? J.njobs : xq_lo(J, xr + 1);
            }
            wave_jobs += (unsigned int)nwant;
            __builtin_amdgcn_wave_barrier();
            __syncthreads();
            const int base = s_base, lim = s_lim;
            if (base + nwant >= lim) {  // this group's range is used up: go on to the next
                xr = (xr + 1) & 7;
                ++xtried;
            }
            if (idle) {
                const int job_k = base + __popcll(want & ((1ull << lane_id) - 1ull));
                if (job_k < lim) {
                    if (COUNT && P.job_trace) P.job_trace[3 * job_k] = wall_clock64();
                    int out_row;
                    L.job = job_k;
                    uint32_t rpix;
                    if (job_pixel(P, job_k, rpix, out_row)) {
                        if (COUNT && P.job_trace) P.job_trace[3 * job_k + 2] = rpix;  // the job's pixel id y * W + x
                        L.sample = 0;
                        camera_query(P, job_k, rpix, 0, q);
                        L.level = 0;
                        if constexpr (SPLIT) {
                            L.cdone = 0;
                            L.nlev = 0;
                            L.untaken = L.posted = 0;
                            split_res[lane_id] = 0u;
                        } else {
                            L.acc = v3{0.0f, 0.0f, 0.0f};
                            L.w = v3{1.0f, 1.0f, 1.0f};
                            L.desc = false;
                            L.shadow = false;
                        }
                        qshadow = false;
                        qsdist = 0.0f;
                        start = true;
                    } else {
                        L.job = -1;  // a padding pixel
                    }
                } else {
                    L.job = xtried < 8 ? -1 : -2;
                }
            }
            __syncthreads();
        }
        if (COUNT) cnt.cyc_d += (unsigned long long)clock64() - tJ;
        // full-wave phases: no lane traces across phase A, so the traversal state is rebuilt for every lane
        // here (a new query, or an empty walk) and nothing of it has to be kept across the state machine
        // (phases that end once some queries are done, the others tracing on across the state machine:
        // C3 frame 1.35-1.64 vs 1.25 ms at refill 32 / 16 / 8 / 2, profiles/r04/ab_r04g_refill.log)
        {
            Trav Tn;
            if (start) {
                cnt.rays++;
                count_start<COUNT>(cnt, qshadow, L.level, qcam);
                trav_init_q(S, P.use_bvh != 0, q.o, q.d, q.t, qshadow, qsdist, Tn);
                tracing = true;
                // counting builds: queries whose direction is not unit walk every record (debug counter 28)
                // (wave trace 1 only: these per-query atomics on one word would distort the other traces' clocks)
                if (COUNT && P.wave_trace && !P.phase_trace && Tn.cur == RT_TRAV_NONE && Tn.rk > 0)
                    atomicAdd(P.stats + RT_STATS_EXTRA + 12, 1ull);
                if (COUNT) {
                    qn0 = cnt.nodes;
                    qr0 = cnt.tris;
                }
            } else {
                trav_idle(Tn);
            }
            T = Tn;
        }
        if (COUNT && P.wave_trace && !t_exh && __any(L.job == -2)) t_exh = wall_clock64();
        if (!__any(tracing)) {
            // every lane exhausted (SPLIT: an owner waits only on a segment some lane is tracing)
            if (!__any(L.job == -1 || pending || (SPLIT && L.job >= 0))) break;
            continue;
        }
        // ---- phase B: one node visit and / or one leaf record per lane and iteration ----
        unsigned long long tB = 0ull;
        if (COUNT) {
            tB = (unsigned long long)clock64();
            cnt.cyc_a += tB - tA;
        }
        float4 g[RT_NODE_F4];
        if (PF && tracing && T.cur != RT_TRAV_NONE) node_fetch(S.nodes, T.cur, g);
        bool to_coop = false;  // the loop ended for the lane groups (not for a partial refill)
        unsigned long long t_ph = 0ull;
        uint32_t ntr_ph = 0, it_ph = 0;
        if (COUNT && P.phase_trace) {
            t_ph = wall_clock64();
            ntr_ph = (uint32_t)__popcll(__ballot(tracing));
        }
        int it_prio = 0;  // (wave-uniform) this phase's iterations, for P.prio_iters
        for (;;) {
            if (COUNT && P.phase_trace) ++it_ph;
            // a phase still tracing after prio_iters iterations holds the wave's slowest queries: issue first
            if (P.prio_iters > 0 && ++it_prio == P.prio_iters) __builtin_amdgcn_s_setprio(2);
            if (COUNT) {
                const int ntr = __popcll(__ballot(tracing));
                if (wave_leader()) cnt.hist[min((ntr - 1) >> 4, 2)]++;
            }
            if (tracing) {
                const bool rec = leaf_pending(T);
                if (rec) trav_record<COUNT, true, false, true>(S, T, cnt, nullptr, COUNT ? &slab : nullptr, &ref_lds);
                if (COUNT) {  // the wave's ref_slab executions this step: the most any lane did
                    const uint32_t ns = rec ? slab.step : 0u;
                    uint32_t w = 0u;
                    for (uint32_t k = 0; k < 8u; ++k) w += __ballot(ns > k) ? 1u : 0u;
                    if (wave_leader()) slab.wslab += w;
                }
                const bool nv = T.cur != RT_TRAV_NONE && (!rec || (P.dual && T.lh == 0u));
                if (COUNT) {
                    slab.iters++;
                    if (nv && rec) slab.both++;
                    if (!nv && T.cur != RT_TRAV_NONE) slab.blocked++;
                }
                if (nv) trav_node<COUNT, 8, PF, DIRECT>(S, T, stk, g, cnt);
            }
            if (tracing && !leaf_pending(T) && T.cur == RT_TRAV_NONE) {
                trav_finish(S, T);
                count_end<COUNT>(cnt, qcam, T.found);
                if (COUNT && qcam && !T.found) {
                    cnt.cmn += cnt.nodes - qn0;
                    cnt.cmr += cnt.tris - qr0;
                }
                tracing = false;
                pending = true;
                // counting builds: the longest queries (debug counters 29 / 30: most node visits / records of one
                // query, 31: queries with more than 512 node visits)
                if (COUNT && P.wave_trace && !P.phase_trace) {
                    atomicMax(P.stats + RT_STATS_EXTRA + 13, (unsigned long long)(cnt.nodes - qn0));
                    atomicMax(P.stats + RT_STATS_EXTRA + 14, (unsigned long long)(cnt.tris - qr0));
                    if (cnt.nodes - qn0 > 512u) atomicAdd(P.stats + RT_STATS_EXTRA + 15, 1ull);
                }
            }
            // full-wave phases (refill 64, the batch and few-sample policy of the general kernel): the phase
            // ends when no lane traces
            if (!__any(tracing)) break;
            if (COUNT && P.wave_trace && t_exh) {
                it_drain++;
                lanes_drain += (unsigned int)__popcll(__ballot(tracing));
            }
            // drain (no lane can take a new job): the wave's last queries walked by lane groups, as in
            // persistent_df_kernel (coop 2: also the last ones a full-wave refill waits for).  The lane
            // groups run after the loop, so their registers do not add to the traversal loop's
            if (COOP && P.coop && (P.coop == 2 || (!__any(L.job == -1) && __any(L.job == -2)))) {
                const int ntr = __popcll(__ballot(tracing));
                if (ntr <= P.coop_max) {
                    if (!DIRECT) {
                        to_coop = true;
                        break;
                    }
                    // a DIRECT stack expands into one pool entry per pending child: the groups take the
                    // queries once every one fits its share of the pool above the depth-first reserve
                    int G = 64;
                    while (G > 1 && ntr * G > 64) G >>= 1;
                    if (!__any(tracing && direct_pending(T, stk) > COOP_POOL * G / 64 - P.coop_reserve)) {
                        to_coop = true;
                        break;
                    }
                }
            }
        }
        if (COOP && to_coop) {
            const unsigned long long om = __ballot(tracing);
            const int k = __popcll(om);
            int G = 64;
            while (G > 1 && k * G > 64) G >>= 1;
            const int r = __popcll(om & ((1ull << lane_id) - 1ull));
            if (tracing) {
                coop_put(T, coop_q, r);
                int* gp = coop_pool + r * (COOP_POOL * G / 64);
                if (DIRECT) {
                    coop_q[CQ_TOP * COOP_Q + r] = direct_to_pool(T, stk, gp);
                } else {
                    for (int j = 0; j < T.sp; ++j) gp[j] = stk[j * RT_WAVE];
                    if (T.cur != RT_TRAV_NONE) gp[T.sp] = (int)T.cur;
                }
            }
            __syncthreads();
            const uint4 nv =
                coop_group_trace<8, COUNT>(S.nodes, S.tri, S.refn, S.leaf_path, coop_pool, coop_q, om, P.coop_reserve);
            __syncthreads();
            if (COUNT) {
                cnt.nodes += nv.x;
                cnt.tris += nv.y;
                if (wave_leader()) {
                    cnt.wnodes += nv.z;
                    cnt.wtris += nv.w;
                }
            }
            if (tracing) {
                coop_get(T, coop_q, r);
                trav_finish(S, T);
                count_end<COUNT>(cnt, qcam, T.found);
                tracing = false;
                pending = true;
            }
            if (COUNT && P.wave_trace) coop_n++;
        }
        if (P.prio_iters > 0 && it_prio >= P.prio_iters) __builtin_amdgcn_s_setprio(0);
        if (COUNT && P.phase_trace) {
            if (lane_id == 0 && nph < RT_PHASE_EV) {
                unsigned long long* w = P.phase_trace + ((size_t)blockIdx.x * RT_PHASE_EV + nph) * 2;
                // times relative to the wave's start (wave trace word 0), in 40 bits
                w[0] = (t_ph - t_wave0) | ((unsigned long long)ntr_ph << 48);
                w[1] = (wall_clock64() - t_wave0) | ((unsigned long long)it_ph << 40) |
                       ((unsigned long long)(to_coop ? 1 : 0) << 63);
            }
            ++nph;
        }
        if (COUNT) cnt.cyc_b += (unsigned long long)clock64() - tB;
    }
    const KParams& P = kernel_params(ka);
    flush_counters<COUNT>(P, cnt);
    flush_slab_counters<COUNT>(P, slab);
    if (COUNT && P.wave_trace && lane_id == 0) {  // traces: counting build only
        unsigned long long* w = P.wave_trace + 8 * blockIdx.x;
        w[0] = t_wave0;
        w[1] = wall_clock64();
        w[2] = wave_jobs;
        w[3] = t_exh;
        w[4] = it_drain;
        w[5] = lanes_drain;
        w[6] = coop_n;
        w[7] = pa_drain;
    }
#undef RT_FRESH
}

// ---- the recursion-tree kernel: transparent materials and every light type, lane state in registers ----
// getFinalColor (src/main.cpp:129-301) on any scene without glossy lobes (glossy_ray_count == 1, or no
// glossy material) and without textures, whose spherical and plane lights take at most 64 samples: the C4
// and C5 configurations.  It is the opaque kernel's inline, register-resident state machine extended with
//   * the transparent reflect + refract tree (src/main.cpp:257-290): the reflected child is walked at once,
//     the refracted one is a pending frame on a per-lane stack in device memory (48 B, written only when a
//     transparent node is shaded: the stack is depth-first, so it never holds more than max_level frames);
//   * the cansee segment loop past transparent surfaces (src/shadow.cpp:41-67) for point and spot lights;
//   * spherical and plane lights as wave-shared fans (FanTable, as in persistent_df_kernel): the owner posts
//     the light, the wave's free lanes trace its samples, the owner folds their results in sample order.
// The general state machine keeps a 42-dword lane image and its frames in private memory around an
// out-of-line call (C5: ~170 GB of scratch writes per 4K frame); here the ~26 dwords below stay in VGPRs.
// Every expression is the general machine's (begin_node, advance_lights_body, next_branch, cansee_step,
// the fan folds), so images and ray counts are bit-identical (tests/test_gpu_parity.py variant matrix).
struct TreeLane {
    int job;               // >= 0 job; -1 idle; -2 no more work
    uint32_t sample : 6;   // camera sample (< 64)
    uint32_t level : 4;    // recursion level of the current node (max_level < 16)
    uint32_t desc : 1;     // the current node descends to its mirror / reflected child after its lights
    uint32_t shadow : 1;   // the lane's own query in flight is a cansee segment (point / spot light)
    uint32_t nfr : 4;      // pending refracted rays on the lane's frame stack
    uint32_t li : 16;      // light cursor over point, spherical, spot, then plane lights (getFinalColor's order)
    v3 acc, w;             // sample colour; weight of the current node
    v3 hp, nN, refl;       // shading point, normalize(normal), reflect
    int mat;               // >= 0 mesh material, < 0 sphere -(s+1)
    v3 color;              // direct light of the current node
    float rc;              // transparent node: the reflected child's Fresnel weight R
};

// one refracted ray pending on the lane's stack (the general machine's FR_REFRACT frame)
__device__ __forceinline__ float4* tree_frame(const KParams& P, int f) {
    return P.frames + ((size_t)f * P.frame_slots + blockIdx.x * RT_WAVE + (threadIdx.x & 63)) * 3;
}

// a point or spot light under the cursor was visible with cansee intensity sI: its calcColor
__device__ __forceinline__ void tree_light_visible(const KParams& P, TreeLane& L, float sI) {
    const DevScene& S = P.S;
    v3 lp, lc;
    if ((int)L.li < S.npl) {
        const rt_point_light pl = S.pl[L.li];
        lp = ld3(pl.position);
        lc = ld3(pl.color);
    } else {
        const DSpot sp = S.spot[L.li - S.npl - S.nsl];
        lp = ld3(sp.pos);
        lc = ld3(sp.color);
    }
    const v3 ldir = normalize(lp - L.hp);
    const float cosL = fabsf(dot(L.nN, ldir));
    const float d2 = dot(normalize(L.refl), ldir);
    L.color += calc_color(lc, sI, cosL, (0.0f < d2) ? d2 : 0.0f, load_mat(S, L.mat));
}

// A finished fan of the spherical or plane light under the cursor: getSpherelights' / getPlaneLights' sums
// replayed in sample order from the samples' visibility, intensities and (plane) hit terms, as
// advance_lights_body folds them (src/shadow.cpp:145-226, 255-321).
__device__ __forceinline__ void tree_fan_light(const KParams& P, TreeLane& L, const FanResult& fan) {
    const DevScene& S = P.S;
    const DMat m = load_mat(S, L.mat);
    const int li = (int)L.li;
    if (li < S.npl + S.nsl) {
        const rt_spherical_light sl = S.sl[li - S.npl];
        float a0, a1;
        if (!fan.inten) {
            const float nv = (float)__popcll(fan.vis >> 1);
            a0 = 1.0f + nv;
            a1 = (float)(fan.vis & 1ull) + nv;
        } else {
            a0 = fan.inten[0];
            a1 = (fan.vis & 1ull) ? 1.0f : 0.0f;
            for (int s = 1; s <= P.sl_m * P.sl_n; ++s)
                if ((fan.vis >> s) & 1ull) {
                    a1 += 1.0f;
                    a0 += fan.inten[s];
                }
        }
        if (a1 > 0.0f) {
            const v3 ldir = normalize(ld3(sl.position) - L.hp);
            const float cosL = fabsf(dot(L.nN, ldir));
            const float d2 = dot(normalize(L.refl), ldir);
            L.color += calc_color(ld3(sl.color), a0 / (float)P.sl_count, cosL, (0.0f < d2) ? d2 : 0.0f, m);
        }
    } else {
        const rt_plane_light pl = S.plane[li - S.npl - S.nsl - S.nspot];
        const int k = P.plane_k;
        // the visible samples' terms (and intensities) summed in sample order, as the loop of src/shadow.cpp:
        // 284-299 adds them: every sample's LDS word is read in blocks of 8 (no read waits on the previous add) and
        // an invisible sample leaves the sums as they are (a select, not an add of 0); the count is exact in float.
        // (The per-sample loop with a branch and a dependent LDS read per sample: C5 137.7 vs 129.5 ms,
        // profiles/r06/ab_r06p*.log)
        const unsigned long long vis = fan.vis;  // (bits of samples >= k * k are never set)
        const float a1 = (float)__popcll(vis);
        float a0 = 0.0f, a3 = fan.inten ? 0.0f : a1;
#pragma unroll 1
        for (int s0 = 0; s0 < k * k; s0 += 8) {
            float tv[8], iv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                tv[j] = fan.term[s0 + j];
                iv[j] = fan.inten ? fan.inten[s0 + j] : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const bool v = (vis >> (s0 + j)) & 1ull;
                a0 = v ? a0 + tv[j] : a0;
                if (fan.inten) a3 = v ? a3 + iv[j] : a3;
            }
        }
        if (a0 > 0.0f) {
            const float lin = (a3 / (float)(int)a1) * a0 / (float)(k * k);
            L.color += calc_color(ld3(pl.color), lin, 1.0f, fan.c2max, m);
        }
    }
}

// The next light of the cursor that needs work: 1 = the lane's own cansee segment (point / spot light)
// queued in q with its distance and intensity; 2 = a fan to post (spherical light, or a plane light the
// shading point is in front of); 0 = the node's lights are done.  Lights visible without a query
// (target within SHADOW_ERROR_OFFSET) count at once; spot lights outside their cone and plane lights
// behind the point contribute nothing (src/shadow.cpp:235-237, 270-272).
__device__ __forceinline__ int tree_next_light(const KParams& P, TreeLane& L, Query& q, float& sdist, float& sI) {
    const DevScene& S = P.S;
    const int n_ps = S.npl + S.nsl, n_pss = n_ps + S.nspot, nl = n_pss + S.nplane;
    while ((int)L.li < nl) {
        const int li = (int)L.li;
        if (li >= S.npl && li < n_ps) return 2;
        if (li >= n_pss) {
            const rt_plane_light pl = S.plane[li - n_pss];
            const v3 w = ld3(pl.width), h = ld3(pl.height), lpos = ld3(pl.position);
            const v3 normal = normalize(cross(w, h));
            if (dot(normalize(L.hp - (lpos + 0.5f * (w + h))), normal) > 0.0f) return 2;
            L.li++;
            continue;
        }
        v3 lp;
        if (li < S.npl) {
            lp = ld3(S.pl[li].position);
        } else {
            const DSpot sp = S.spot[li - n_ps];
            lp = ld3(sp.pos);
            if (!(dot(normalize(ld3(sp.dir)), normalize(L.hp - lp)) > sp.cos_angle)) {
                L.li++;
                continue;
            }
        }
        v3 d = lp - L.hp;  // start_cansee
        sdist = length(d);
        d = normalize(d);
        sI = 1.0f;
        if (sdist > 0.0005f) {
            q.o = L.hp + 0.0005f * d;
            q.d = d;
            q.t = FLT_MAX;
            return 1;
        }
        tree_light_visible(P, L, 1.0f);
        L.li++;
    }
    return 0;
}

enum { TA_DONE = 0, TA_QUERY = 1, TA_FAN = 2 };

// The tree kernel's advance after a finished query or fan: `vis` = the lane's own cansee result (its
// shadow query ended: 1 visible, 0 blocked), `fan` = the completed fan of the light under the cursor,
// else the path query (q = its ray, hit / b = its result) ended.  TA_QUERY with the next query in q
// (sdist / sI: a cansee segment's distance and intensity), TA_FAN when a fan is to be posted, TA_DONE when
// the job is complete.
template <bool COUNT, bool CHK = false>
__device__ __forceinline__ int tree_advance(const KParams& P, TreeLane& L, int vis, const FanResult& fan, bool hit,
                                            const Best& b, Query& q, float& sdist, float& sI, Cnt& cnt) {
    const DevScene& S = P.S;
    bool node_done = true;
    unsigned long long* err = CHK ? P.stats + RT_STATS_EXTRA + 8 : nullptr;
    if (CHK && !fan.done && !L.shadow && hit && !(b.rec >= 0 ? b.rec < S.ntri : (-b.rec - 1) < S.nsph)) {
        chk_report(err, 7, (uint32_t)b.rec);
        hit = false;
    }
    if (fan.done) {
        tree_fan_light(P, L, fan);
        L.li++;
    } else if (L.shadow) {
        if (vis) tree_light_visible(P, L, sI);
        L.li++;
        L.shadow = false;
    } else if (hit) {
        // begin_node (src/main.cpp:131-290)
        const Surf s = surface(S, q.o, q.d, b, false, L.level == 0);
        if (COUNT) {
            cnt.hits++;
            if (s.ub) cnt.ub++;
        }
        L.hp = s.p;
        L.nN = normalize(s.n);
        L.refl = reflect(normalize(q.d), L.nN);
        L.mat = (b.rec >= 0) ? s.mesh : b.rec;
        L.color = v3{0.0f, 0.0f, 0.0f};
        L.li = 0;
        L.desc = false;
        if (L.level < P.max_level) {
            const v3 ks{s.m.ks[0], s.m.ks[1], s.m.ks[2]};
            if (s.m.transp == 1.0f) {
                if (ks.x > 0.0f || ks.y > 0.0f || ks.z > 0.0f) L.desc = true;
            } else {
                // Schlick Fresnel with R0 = transparency, Snell with eta = refraction_factor: the reflected
                // child after the lights, the refracted one (if traced) pushed
                const v3 l = normalize(q.d);
                const v3 n = L.nN;
                const float r = P.refr;
                const float c = fabsf(dot(l, n));
                v3 refr = r * l + (r * c - sqrtf(1.0f - r * r * (1.0f - c * c))) * n;
                refr = normalize(refr);
                const float R0 = s.m.transp;
                const float reflC = (float)((double)R0 + (double)(1.0f - R0) * pow((double)(1.0f - c), 5.0));
                const float refrC = 1.0f - reflC;
                L.desc = true;
                L.rc = reflC;
                if (CHK && (int)L.nfr >= max(1, P.max_level)) {
                    chk_report(err, 4, L.nfr);
                } else if (r * r * (1.0f - c * c) <= 1.0f) {
                    const v3 fo = L.hp + 0.01f * refr, fw = L.w * refrC;
                    float4* fp = tree_frame(P, (int)L.nfr);
                    fp[0] = make_float4(fo.x, fo.y, fo.z, __int_as_float((int)L.level + 1));
                    fp[1] = make_float4(refr.x, refr.y, refr.z, 0.0f);
                    fp[2] = make_float4(fw.x, fw.y, fw.z, 0.0f);
                    L.nfr++;
                }
            }
        }
    } else {
        node_done = false;  // a miss: getFinalColor returns black
    }
    if (node_done) {
        const int r = tree_next_light(P, L, q, sdist, sI);
        if (r == 1) {
            L.shadow = true;
            return TA_QUERY;
        }
        if (r == 2) return TA_FAN;
        L.acc = L.acc + L.w * L.color;  // every light done: the node's colour, then its child
        if (L.desc) {
            const DMat m = load_mat(S, L.mat);
            if (m.transp == 1.0f) {
                const v3 ks{m.ks[0], m.ks[1], m.ks[2]};
                L.w = (m.shin != 0.0f) ? L.w * ((ks * ks) / (float)P.glossy_n) : L.w * (ks * ks);
            } else {
                L.w = L.w * L.rc;
            }
            L.level++;
            q.o = L.hp + 0.01f * L.refl;
            q.d = L.refl;
            q.t = FLT_MAX;
            return TA_QUERY;
        }
    }
    // the subtree is finished: the deepest pending refracted ray (next_branch)
    if (L.nfr > 0) {
        L.nfr--;
        const float4* fp = tree_frame(P, (int)L.nfr);
        const float4 f0 = fp[0], f1 = fp[1], f2 = fp[2];
        L.level = (uint32_t)__float_as_int(f0.w);
        L.w = v3{f2.x, f2.y, f2.z};
        q.o = v3{f0.x, f0.y, f0.z};
        q.d = v3{f1.x, f1.y, f1.z};
        q.t = FLT_MAX;
        return TA_QUERY;
    }
    // camera sample complete
    if (CHK) {
        uint32_t rpix;
        int out_row;
        job_pixel(P, L.job, rpix, out_row);
        const int rows = P.out_image ? max(1, P.n_views) * P.H : (P.view_rows > 0 ? max(1, P.n_views) * P.view_rows : 0x7FFFFFFF);
        // rpix is the reference's pixel id y * W + x of one view: below W * H
        if (out_row < 0 || out_row >= rows || rpix >= (uint32_t)P.W * (uint32_t)P.H) {
            chk_report(err, 5, (uint32_t)out_row);
            L.job = -1;
            return TA_DONE;
        }
    }
    if (store_sample(P, L.job, L.sample, L.acc)) {
        L.sample++;
        uint32_t rpix;
        int out_row;
        job_pixel(P, L.job, rpix, out_row);
        camera_query(P, L.job, rpix, L.sample, q);
        L.acc = v3{0.0f, 0.0f, 0.0f};
        L.w = v3{1.0f, 1.0f, 1.0f};
        L.level = 0;
        L.desc = false;
        return TA_QUERY;
    }
    L.job = -1;
    return TA_DONE;
}

template <bool COUNT, int V>
__global__ __launch_bounds__(64, RT_V_WAVES(V)) void persistent_tree_kernel(KParams, JobSrc) {
    constexpr bool PF = !(V & RT_V_NOPF), DIRECT = !(V & RT_V_REVISIT), CHK = (V & RT_V_CHK) != 0;
    const void* ka = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
#define RT_FRESH const KParams& P = *(const KParams*)fresh_kernarg(ka); const DevScene& S = P.S
    __shared__ int stack_lds[RT_STACK8 * RT_WAVE];
    __shared__ int s_base, s_lim;
    __shared__ FanTable ft;
    __shared__ int fan_queue[RT_WAVE];  // lanes waiting for a fan slot, oldest first
    __shared__ RefLds ref_lds;          // the reference BVH's boxes and leaf paths (candidate culling)
    const int lane_id = threadIdx.x;
    int* stk = stack_lds + lane_id;
    if (RT_REF_LDS) ref_lds_load(kernel_params(ka).S, ref_lds, lane_id);
    if (lane_id < FAN_SLOTS) ft.owner[lane_id] = -1;
    __syncthreads();
    int fq_head = 0, fq_tail = 0;  // (wave-uniform)
    bool fq_in = false;            // this lane is in the fan queue
    int own_fan = -1;              // fan slot this lane's state machine waits for
    bool fan_req = false;          // the state machine posted a fan, no free slot yet
    int ray_fan = -1, ray_s = 0;   // the fan sample this lane's traversal slot traces
    float qsI = 1.0f, qsdist = 0.0f;  // cansee intensity / remaining distance of the segment in flight
    TreeLane L;
    L.job = -1;
    L.shadow = false;
    L.nfr = 0;
    Trav T;
    Cnt cnt{};
    int xr = (int)(blockIdx.x & 7), xtried = 0;
    bool tracing = false, pending = false;
    bool qcam = false;  // counting builds: the query in flight is a camera ray
    for (;;) {
        unsigned long long tA = COUNT ? (unsigned long long)clock64() : 0ull;
        RT_FRESH;
        const JobSrc& J = kernel_jobs(&P);
        bool start = false, qshadow = false;
        Query q;
        // ---- a finished cansee segment (the lane's own, or a fan sample): next segment, or its result ----
        unsigned long long tE = COUNT ? (unsigned long long)clock64() : 0ull;
        int vis = 0;
        if (pending && (ray_fan >= 0 || L.shadow)) {
            q.o = T.o;
            q.d = T.d;
            const int r = S.all_opaque ? (T.found ? 0 : 1) : cansee_step(S, q, T.found, T.best, qsI, qsdist);
            if (r == 2) {  // past a transparent surface: the segment loop goes on
                pending = false;
                start = true;
                qshadow = true;
            } else if (ray_fan >= 0) {
                pending = false;
                if (r == 1 && ft.plane[ray_fan]) fan_plane_term(P, ft, ray_fan, ray_s);
                fan_record(ft, ray_fan, ray_s, r == 1, qsI);
                ray_fan = -1;
            } else {
                vis = r;
            }
        }
        __syncthreads();
        if (COUNT) {
            const unsigned long long t = (unsigned long long)clock64();
            cnt.cyc_e += t - tE;
            tE = t;
        }
        // ---- owners of complete fans resume once their traversal slot is free ----
        FanResult fan{0ull, nullptr, false, nullptr, 0.0f};
        if (own_fan >= 0 && !tracing && !start && ft.done[own_fan] == ft.count[own_fan]) {
            fan.vis = ft.vis[own_fan];
            fan.inten = S.all_opaque ? nullptr : ft.inten[own_fan];
            fan.term = ft.term[own_fan];
            fan.c2max = __uint_as_float(ft.c2max[own_fan]);
            fan.done = true;
            ft.owner[own_fan] = -1;
            own_fan = -1;
        }
        if (pending || fan.done) {
            pending = false;
            if (COUNT && wave_leader()) cnt.wadv++;
            if (!fan.done && !L.shadow) {
                q.o = T.o;
                q.d = T.d;
            }
            const int jb = L.job;
            const int r = tree_advance<COUNT, CHK>(P, L, vis, fan, T.found, T.best, q, qsdist, qsI, cnt);
            if (r == TA_QUERY) {
                start = true;
                qshadow = L.shadow;
            } else if (r == TA_FAN) {
                fan_req = true;
            }
            if (COUNT && P.job_trace && L.job == -1) P.job_trace[3 * jb + 1] = wall_clock64();
        }
        __syncthreads();
        if (COUNT) {
            const unsigned long long t = (unsigned long long)clock64();
            cnt.cyc_f += t - tE;
            tE = t;
        }
        // ---- fan slots to the oldest posters, then samples to every lane whose traversal slot is free ----
        {
            const bool new_req = fan_req && !fq_in;
            const unsigned long long nr = __ballot(new_req);
            if (nr) {
                if (new_req) {
                    fan_queue[(fq_tail + __popcll(nr & ((1ull << lane_id) - 1ull))) & (RT_WAVE - 1)] = lane_id;
                    fq_in = true;
                }
                fq_tail += __popcll(nr);
                __syncthreads();
            }
            if (fq_head != fq_tail) {
                uint64_t freeslots = __ballot(lane_id < FAN_SLOTS && ft.owner[lane_id] < 0);
                while (fq_head != fq_tail && freeslots) {
                    const int l = fan_queue[fq_head & (RT_WAVE - 1)], f = __ffsll((long long)freeslots) - 1;
                    ++fq_head;
                    freeslots &= freeslots - 1ull;
                    if (lane_id == l) {
                        const bool plane = (int)L.li >= S.npl + S.nsl;
                        fq_in = false;
                        ft.owner[f] = l;
                        ft.next[f] = 0;
                        ft.plane[f] = plane ? 1 : 0;
                        ft.count[f] = plane ? P.plane_k * P.plane_k : 1 + P.sl_m * P.sl_n;
                        ft.done[f] = 0;
                        ft.traced[f] = 0;
                        ft.vis[f] = 0ull;
                        ft.li[f] = plane ? (int)L.li - S.npl - S.nsl - S.nspot : (int)L.li - S.npl;
                        ft.hx[f] = L.hp.x;
                        ft.hy[f] = L.hp.y;
                        ft.hz[f] = L.hp.z;
                        const v3 nr = normalize(L.refl);  // (fan_plane_term's normalize(reflect), once per fan)
                        ft.rx[f] = nr.x;
                        ft.ry[f] = nr.y;
                        ft.rz[f] = nr.z;
                        ft.c2max[f] = 0u;
                        own_fan = f;
                        fan_req = false;
                    }
                }
                __syncthreads();
            }
            const bool tfree = !tracing && !start;
            const unsigned long long fl = __ballot(tfree);
            uint64_t pend =
                __ballot(lane_id < FAN_SLOTS && ft.owner[lane_id] >= 0 && ft.next[lane_id] < ft.count[lane_id]);
            if (fl && pend) {
                const int nfree = __popcll(fl);
                const int rank = __popcll(fl & ((1ull << lane_id) - 1ull));
                int base = 0;
                while (pend && base < nfree) {
                    const int f = __ffsll((long long)pend) - 1;
                    pend &= pend - 1ull;
                    const int nx = ft.next[f];
                    const int take = min(ft.count[f] - nx, nfree - base);
                    if (tfree && rank >= base && rank < base + take) {
                        ray_fan = f;
                        ray_s = nx + (rank - base);
                    }
                    __syncthreads();
                    if (lane_id == 0) ft.next[f] = nx + take;
                    base += take;
                }
                __syncthreads();
            }
            if (CHK && tfree && ray_fan >= 0 && (ray_fan >= FAN_SLOTS || ray_s < 0 || ray_s >= 64)) {
                chk_report(P.stats + RT_STATS_EXTRA + 8, 6, (uint32_t)(ray_fan << 8 | ray_s));
                ray_fan = -1;
            }
            if (tfree && ray_fan >= 0) {
                const v3 hp{ft.hx[ray_fan], ft.hy[ray_fan], ft.hz[ray_fan]};
                qsI = 1.0f;
                if (fan_sample_query(P, hp, ft.li[ray_fan], ft.plane[ray_fan], ray_s, q, qsdist)) {
                    start = true;
                    qshadow = true;
                } else {  // visible without a query
                    if (ft.plane[ray_fan]) fan_plane_term(P, ft, ray_fan, ray_s);
                    fan_record(ft, ray_fan, ray_s, true, 1.0f);
                    ray_fan = -1;
                }
            }
            __syncthreads();
        }
        const unsigned long long tJ = COUNT ? (unsigned long long)clock64() : 0ull;
        if (COUNT) {
            cnt.cyc_c += tJ - tA;
            cnt.cyc_g += tJ - tE;
        }
        // ---- new pixels for idle lanes (none while the wave's pixels wait on fan_cap fans) ----
        const bool fan_full = __popcll(__ballot(own_fan >= 0 || fan_req)) >= P.fan_cap;
        const bool idle = (L.job == -1) && !start && !tracing && !fan_full;
        const unsigned long long want = __ballot(idle);
        if (want) {
            const int nwant = __popcll(want);
            if (lane_id == __ffsll((long long)want) - 1) {
                const int lo = xq_lo(J, xr);
                s_base = lo + atomicAdd(J.xq + 32 * xr, nwant);
                s_lim = xr == 7 ? J.njobs : xq_lo(J, xr + 1);
            }
            __builtin_amdgcn_wave_barrier();
            __syncthreads();
            const int base = s_base, lim = s_lim;
            if (base + nwant >= lim) {  // this group's range is used up: go on to the next
                xr = (xr + 1) & 7;
                ++xtried;
            }
            if (idle) {
                const int job_k = base + __popcll(want & ((1ull << lane_id) - 1ull));
                if (job_k < lim) {
                    if (COUNT && P.job_trace) P.job_trace[3 * job_k] = wall_clock64();
                    int out_row;
                    L.job = job_k;
                    uint32_t rpix;
                    if (job_pixel(P, job_k, rpix, out_row)) {
                        L.sample = 0;
                        camera_query(P, job_k, rpix, 0, q);
                        L.acc = v3{0.0f, 0.0f, 0.0f};
                        L.w = v3{1.0f, 1.0f, 1.0f};
                        L.level = 0;
                        L.desc = false;
                        L.shadow = false;
                        L.nfr = 0;
                        qshadow = false;
                        start = true;
                    } else {
                        L.job = -1;  // a padding pixel
                    }
                } else {
                    L.job = xtried < 8 ? -1 : -2;
                }
            }
            __syncthreads();
        }
        if (COUNT) cnt.cyc_d += (unsigned long long)clock64() - tJ;
        // full-wave phases: the traversal state is rebuilt for every lane (a new query or an empty walk)
        {
            Trav Tn;
            if (start) {
                cnt.rays++;
                count_start<COUNT>(cnt, qshadow, L.level, qcam);
                trav_init_q(S, P.use_bvh != 0, q.o, q.d, q.t, qshadow, qsdist, Tn);
                tracing = true;
            } else {
                trav_idle(Tn);
            }
            T = Tn;
        }
        if (!__any(tracing)) {
            if (!__any(L.job == -1 || pending || own_fan >= 0 || fan_req)) break;  // every lane exhausted
            continue;
        }
        // ---- one node visit and / or one leaf record per lane and iteration, until no lane traces ----
        unsigned long long tB = 0ull;
        if (COUNT) {
            tB = (unsigned long long)clock64();
            cnt.cyc_a += tB - tA;
        }
        float4 g[RT_NODE_F4];
        if (PF && tracing && T.cur != RT_TRAV_NONE) node_fetch(S.nodes, T.cur, g);
        for (;;) {
            if (COUNT) {
                const int ntr = __popcll(__ballot(tracing));
                if (wave_leader()) cnt.hist[min((ntr - 1) >> 4, 2)]++;
            }
            if (tracing) {
                const bool rec = leaf_pending(T);
                unsigned long long* err = CHK ? P.stats + RT_STATS_EXTRA + 8 : nullptr;
                if (rec) trav_record<COUNT, true, CHK, true>(S, T, cnt, err, nullptr, &ref_lds);
                const bool nv = T.cur != RT_TRAV_NONE && (!rec || (P.dual && T.lh == 0u));
                if (nv) trav_node<COUNT, 8, PF, DIRECT, CHK>(S, T, stk, g, cnt, err);
            }
            if (tracing && !leaf_pending(T) && T.cur == RT_TRAV_NONE) {
                trav_finish(S, T);
                count_end<COUNT>(cnt, qcam, T.found);
                tracing = false;
                pending = true;
            }
            if (!__any(tracing)) break;
        }
        if (COUNT) cnt.cyc_b += (unsigned long long)clock64() - tB;
    }
    const KParams& P = kernel_params(ka);
    flush_counters<COUNT>(P, cnt);
#undef RT_FRESH
}

// BoundingVolumeHierarchy::intersect(ray, hitInfo, useBVH) per ray (rt_intersect): the same
// trace_query8 and surface() as the renderer.
__global__ __launch_bounds__(64) void intersect_kernel(DevScene S, const rt_ray* rays, int n, int use_bvh,
                                                       rt_hit* hits) {
    __shared__ int stack_lds[RT_STACK_SIZE * RT_WAVE];
    const int i = blockIdx.x * 64 + threadIdx.x;
    int* stk = stack_lds + threadIdx.x;
    if (i >= n) return;
    const rt_ray r = rays[i];
    const v3 o{r.origin[0], r.origin[1], r.origin[2]};
    const v3 d{r.direction[0], r.direction[1], r.direction[2]};
    Best b;
    Cnt cnt{};
    const bool hit = trace_query8<false, 8>(S, o, d, r.t, 0.0f, use_bvh != 0, false, b, stk, cnt);
    rt_hit h;
    h.hit = hit ? 1 : 0;
    h.t = hit ? b.t : r.t;
    if (hit) {
        const Surf s = surface(S, o, d, b);
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

}  // namespace rt
