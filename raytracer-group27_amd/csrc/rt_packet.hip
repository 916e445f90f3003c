// rt_packet.hip -- primary rays as wave-coherent packets (included by rt_runtime.hip after
// rt_megakernel.hip).
//
// One 64-lane wave takes one 8x8 pixel tile and traces its 64 camera rays (src/main.cpp:350-354,
// Trackball::generateRay framework/src/trackball.cpp:87-98) through the quantised wide BVH as ONE
// packet: the wave walks a single shared node sequence, so every node and triangle record is one
// wave-uniform (scalar) fetch instead of 64 divergent gathers, and each lane still judges its own
// ray with the reference arithmetic (slab culling, plane/edge triangle test, (t, key) order).
// A lane takes part in a subtree only while its own box tests admit it, so its candidate set is
// exactly the one the single-ray walk would test; the result (closest t, record) is therefore
// the same bits.  The megakernels then start every pixel from its stored primary hit.
//
// Stack: (node, lane mask) pairs in LDS, written by every lane with the same value (no barrier).

namespace rt {

#define PK_STACK 256

template <bool COUNT, int NW>
__global__ __launch_bounds__(64, 4) void primary_packet_kernel(KParams P, float* __restrict__ pre_t,
                                                               int* __restrict__ pre_rec, int ntiles) {
    __shared__ int s_node[PK_STACK];
    __shared__ unsigned long long s_mask[PK_STACK];
    const int lane = (int)threadIdx.x;
    const DevScene& S = P.S;
    const bool REF = P.use_bvh != 0;
    unsigned int nrays = 0;
    Cnt cnt{};  // counting builds: per-ray node visits / records (the single-ray definition)
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int job = tile * 64 + lane;
        Lane L;
        L.sample = 0;
        const bool ok = job_pixel(P, job, L);
        v3 o{0.0f, 0.0f, 0.0f}, d{0.0f, 0.0f, 1.0f};
        if (ok) {
            queue_camera(P, L);
            o = L.qo;
            d = L.qd;
        }
        const bool unit = ok && (fabsf(dot(d, d) - 1.0f) <= 4e-6f);
        const v3 nd = normalize(d);
        const v3 inv = safe_inv(d);
        Best best;
        best.t = FLT_MAX;
        best.key = -1;
        best.rec = RT_NO_HIT;
        RefMask rmask{0u, 0u};
        bool found = false;
        int sp = 0;
        const unsigned long long live = __ballot(unit);
        if (live && S.ntri > 0) {
            s_node[0] = 0;
            s_mask[0] = live;
            sp = 1;
        }
        while (sp > 0) {
            --sp;
            const int node = __builtin_amdgcn_readfirstlane(s_node[sp]);
            const unsigned long long m = s_mask[sp];
            const bool act = (m >> lane) & 1ull;
            if (COUNT && act) cnt.nodes++;
            const float4* np = S.nodes + (size_t)node * 8;
            const float4 f0 = np[0], f1 = np[1], qlx = np[2], qly = np[3], qlz = np[4], qhx = np[5], qhy = np[6],
                         qhz = np[7];
            const uint32_t w3 = __float_as_uint(f0.w);
            const uint32_t imask = __float_as_uint(f1.z) & 0xFFu;
            const uint32_t lmask = (__float_as_uint(f1.z) >> 8) & 0xFFu;
            const uint32_t counts = __float_as_uint(f1.w);
            const uint32_t child_base = __float_as_uint(f1.x);
            const uint32_t tri_base = __float_as_uint(f1.y);
            const float bx = pow2f(w3 & 0xFFu) * inv.x, by = pow2f((w3 >> 8) & 0xFFu) * inv.y,
                        bz = pow2f((w3 >> 16) & 0xFFu) * inv.z;
            const float ax = (f0.x - o.x) * inv.x, ay = (f0.y - o.y) * inv.y, az = (f0.z - o.z) * inv.z;
            const float tcull = best.t;
            float tn[NW];
            uint32_t hits = 0;
#pragma unroll
            for (int s = 0; s < NW; ++s) {
                tn[s] = FLT_MAX;
                if (act && ((imask | lmask) & (1u << s))) {
                    const int wi = s >> 1, sh = (s & 1) * 16;
                    auto q = [&](const float4& f) {
                        const uint32_t wv = __float_as_uint(wi == 0 ? f.x : wi == 1 ? f.y : wi == 2 ? f.z : f.w);
                        return (float)((wv >> sh) & 0xFFFFu);
                    };
                    const float tlx = fmaf(q(qlx), bx, ax), thx = fmaf(q(qhx), bx, ax);
                    const float tly = fmaf(q(qly), by, ay), thy = fmaf(q(qhy), by, ay);
                    const float tlz = fmaf(q(qlz), bz, az), thz = fmaf(q(qhz), bz, az);
                    const float t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fminf(tlz, thz));
                    const float t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fmaxf(tlz, thz));
                    if (t0 <= t1 && t1 >= 0.0f && t0 <= tcull) {
                        hits |= 1u << s;
                        tn[s] = t0;
                    }
                }
            }
            // leaf slots, in slot order: every record once per wave, tested by the lanes that hit it
#pragma unroll
            for (int s = 0; s < NW; ++s) {
                if (!(lmask & (1u << s))) continue;
                const unsigned long long ms = __ballot((hits >> s) & 1u);
                if (!ms) continue;
                const bool mine = (ms >> lane) & 1ull;
                const uint32_t below = s ? (counts & ((1u << (4 * s)) - 1u)) : 0u;
                uint32_t nib = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
                nib = (nib * 0x01010101u) >> 24;
                const int first = (int)(tri_base + nib);
                const int cnt_s = (int)((counts >> (4 * s)) & 15u);
                for (int r = first; r < first + cnt_s; ++r) {
                    const float4* tp = S.tri + (size_t)r * 4;
                    const float4 r0 = tp[0], r1 = tp[1], r2 = tp[2], r3 = tp[3];
                    if (!mine) continue;
                    if (COUNT) cnt.tris++;
                    float t;
                    if (!tri_test(r0, r1, r2, r3, o, d, nd, t)) continue;
                    const int key = REF ? __float_as_int(r3.z) : __float_as_int(r3.y);
                    if (!(t < best.t || (t == best.t && key < best.key))) continue;
                    if (REF && !leaf_reachable(S, __float_as_int(r3.w), o, nd, rmask)) continue;
                    best.t = t;
                    best.key = key;
                    best.rec = r;
                    found = true;
                }
            }
            // inner slots: push far to near (the order key is the first admitted lane's entry t)
            float key_s[NW];
            unsigned long long msk[NW];
            uint32_t rem = 0;
#pragma unroll
            for (int s = 0; s < NW; ++s) {
                msk[s] = 0ull;
                key_s[s] = 0.0f;
                if (!(imask & (1u << s))) continue;
                // lanes whose best hit moved closer than this child's entry drop out here
                const unsigned long long ms = __ballot(((hits >> s) & 1u) && tn[s] <= best.t);
                if (!ms) continue;
                msk[s] = ms;
                const int fl = __ffsll((long long)ms) - 1;
                key_s[s] = __shfl(tn[s], fl);
                rem |= 1u << s;
            }
            while (rem) {
                int sel = -1;
                float kmax = -FLT_MAX;
#pragma unroll
                for (int s = 0; s < NW; ++s) {
                    if ((rem & (1u << s)) && (sel < 0 || key_s[s] > kmax)) {
                        sel = s;
                        kmax = key_s[s];
                    }
                }
                rem &= ~(1u << sel);
                if (sp < PK_STACK) {
                    unsigned long long ms = 0ull;
#pragma unroll
                    for (int s = 0; s < NW; ++s)
                        if (s == sel) ms = msk[s];
                    s_node[sp] = (int)(child_base + __popc(imask & ((1u << sel) - 1u)));
                    s_mask[sp] = ms;
                    ++sp;
                }
            }
        }
        if (unit) {
            // spheres after every triangle (trav_finish order)
            for (int s = 0; s < S.nsph; ++s) {
                const DSph sp_ = S.sph[s];
                float t;
                if (!sphere_test(sp_, o, d, t)) continue;
                const int key = REF ? sp_.key_bvh : S.ntri + s;
                if (!(t < best.t || (t == best.t && key < best.key))) continue;
                if (REF && !leaf_reachable(S, sp_.leaf, o, nd, rmask)) continue;
                best.t = t;
                best.key = key;
                best.rec = -s - 1;
                found = true;
            }
            pre_t[job] = best.t;
            pre_rec[job] = found ? best.rec : RT_NO_HIT;
            ++nrays;
        } else if (ok) {
            pre_rec[job] = RT_PRE_NONE;
        }
    }
    for (int off = 32; off > 0; off >>= 1) nrays += __shfl_xor(nrays, off);
    if (lane == 0 && nrays) atomicAdd(P.stats + 0, (unsigned long long)nrays);
    if (COUNT) flush_counters<COUNT>(P, cnt);
}

}  // namespace rt
