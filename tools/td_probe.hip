// Developer probe (not part of the library): what a divergent gather costs the vector memory pipe.
// Each wave runs `iters` steps; in a step the lanes below `active` load one 128-B "node" (8 x dwordx4, as
// node_fetch does) from a pseudo-random line of a buffer of `bytes`, the next line depending on the data
// (a dependent walk, like a traversal).  Time per step against the active lane count shows whether the
// memory pipe's cost follows the active lanes or the instruction.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/td_probe tools/td_probe.hip
// Run:   tools/td_probe [blocks] [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

__global__ __launch_bounds__(64) void walk(const float4* __restrict__ buf, unsigned nlines, int iters, int active,
                                           float* out) {
    const int lane = threadIdx.x;
    unsigned line = (blockIdx.x * 64u + (unsigned)lane) * 2654435761u % nlines;
    float acc = 0.0f;
    if (lane < active) {
        for (int i = 0; i < iters; ++i) {
            const float4* p = buf + (size_t)line * 8;
            float4 g[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = p[k];
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 8; ++k) s += g[k].x + g[k].y + g[k].z + g[k].w;
            acc += s;
            // the next line depends on the loaded data (a dependent walk); the data are small integers
            line = (line * 1103515245u + 12345u + (unsigned)s) % nlines;
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

// The same walk with the nodes gathered cooperatively: gather k has lane i fetch 16-B chunk (i & 7) of the node
// of lane 8k + (i >> 3) into LDS, so one instruction touches 8 lines instead of 64, and a wave with A active
// lanes issues ceil(A / 8) gathers instead of 8; each lane then reads its own node back (8 x ds_read_b128).
// SWZ: chunk c of node s sits at entry s * 8 + (c ^ (s & 7)), so the 8 lanes of a read-back quad-group hit 8
// different bank groups (unswizzled, every lane's chunk k is in the same one)
template <bool SWZ>
__global__ __launch_bounds__(64) void walk_coop(const float4* __restrict__ buf, unsigned nlines, int iters, int active,
                                                float* out) {
    __shared__ float4 st[64 * 8];
    const int lane = threadIdx.x;
    unsigned line = (blockIdx.x * 64u + (unsigned)lane) * 2654435761u % nlines;
    float acc = 0.0f;
    const int ngather = (active + 7) >> 3;
    for (int i = 0; i < iters; ++i) {
        for (int k = 0; k < ngather; ++k) {
            const int src = 8 * k + (lane >> 3);
            const unsigned l = (unsigned)__shfl((int)line, src);
            const int c = lane & 7;
            if (src < active) st[src * 8 + (SWZ ? (c ^ (src & 7)) : c)] = buf[(size_t)l * 8 + c];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane < active) {
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float4 g = st[lane * 8 + (SWZ ? (k ^ (lane & 7)) : k)];
                s += g.x + g.y + g.z + g.w;
            }
            acc += s;
            line = (line * 1103515245u + 12345u + (unsigned)s) % nlines;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    out[blockIdx.x * 64 + lane] = acc;
}

// The swizzled cooperative walk with LDS-DMA: gather k is one global_load_lds_dwordx4 whose lane i writes LDS entry
// 64k + i (the instruction's destination is wave-uniform base + 16 B x lane), so the swizzle goes on the source:
// entry 8s + j receives chunk j ^ (s & 7) of node s.  No VGPR holds the node on its way to LDS.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;
__global__ __launch_bounds__(64) void walk_glds(const float4* __restrict__ buf, unsigned nlines, int iters, int active,
                                                float* out) {
    __shared__ float4 st[64 * 8];
    const int lane = threadIdx.x;
    unsigned line = (blockIdx.x * 64u + (unsigned)lane) * 2654435761u % nlines;
    float acc = 0.0f;
    const int ngather = (active + 7) >> 3;
    for (int i = 0; i < iters; ++i) {
        for (int k = 0; k < ngather; ++k) {
            const int src = 8 * k + (lane >> 3);
            const unsigned l = (unsigned)__shfl((int)line, src);
            const int c = (lane & 7) ^ (src & 7);
            if (src < active)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(buf + (size_t)l * 8 + c), (lds_ptr_t)(st + 64 * k), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the DMA has landed in LDS
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane < active) {
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float4 g = st[lane * 8 + (k ^ (lane & 7))];
                s += g.x + g.y + g.z + g.w;
            }
            acc += s;
            line = (line * 1103515245u + 12345u + (unsigned)s) % nlines;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    out[blockIdx.x * 64 + lane] = acc;
}

// 64-B records (4 x dwordx4) per active lane, per-lane gathers (R = 0) or LDS-DMA with 16 records per
// instruction (R = 1): the record step of a traversal
template <int R>
__global__ __launch_bounds__(64) void walk_rec(const float4* __restrict__ buf, unsigned nlines, int iters, int active,
                                               float* out) {
    __shared__ float4 st[64 * 4];
    const int lane = threadIdx.x;
    const unsigned nrec = nlines * 2;
    unsigned rec = (blockIdx.x * 64u + (unsigned)lane) * 2654435761u % nrec;
    float acc = 0.0f;
    const int ngather = (active + 15) >> 4;
    for (int i = 0; i < iters; ++i) {
        float4 g[4];
        if (R == 0) {
            if (lane < active) {
#pragma unroll
                for (int k = 0; k < 4; ++k) g[k] = buf[(size_t)rec * 4 + k];
            }
        } else {
            for (int k = 0; k < ngather; ++k) {
                const int src = 16 * k + (lane >> 2);
                const unsigned r = (unsigned)__shfl((int)rec, src);
                const int c = (lane & 3) ^ ((src >> 2) & 3);
                if (src < active)
                    __builtin_amdgcn_global_load_lds((gbl_ptr_t)(buf + (size_t)r * 4 + c), (lds_ptr_t)(st + 64 * k), 16, 0, 0);
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (lane < active) {
#pragma unroll
                for (int k = 0; k < 4; ++k) g[k] = st[lane * 4 + (k ^ ((lane >> 2) & 3))];
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (lane < active) {
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 4; ++k) s += g[k].x + g[k].y + g[k].z + g[k].w;
            acc += s;
            rec = (rec * 1103515245u + 12345u + (unsigned)s) % nrec;
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
    const size_t sizes[] = {16u << 10, 2u << 20, 64u << 20, 1024u << 20};
    const int actives[] = {64, 32, 16, 8, 1};
    float4* buf;
    float* out;
    const size_t maxb = sizes[3];
    CHECK(hipMalloc(&buf, maxb));
    CHECK(hipMemset(buf, 0, maxb));
    CHECK(hipMalloc(&out, (size_t)blocks * 64 * sizeof(float)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::printf("blocks %d, iters %d: ns per wave step (one 128-B node per active lane)\n", blocks, iters);
    std::printf("%16s", "gather / buffer");
    for (int act : actives) std::printf("  active %2d", act);
    std::printf("   (lines/us chip-wide at 64 | at 8)\n");
    const char* names[] = {"lane", "coop", "cswz", "glds", "rec ", "rgld"};
    for (int coop = 0; coop < 6; ++coop)
    for (size_t bytes : sizes) {
        const unsigned nlines = (unsigned)(bytes / 128);
        std::printf("%s%10zu K", names[coop], bytes >> 10);
        double t64 = 0, t8 = 0;
        for (int act : actives) {
            auto k = coop == 5 ? walk_rec<1> : coop == 4 ? walk_rec<0> : coop == 3 ? walk_glds
                   : coop == 2 ? walk_coop<true> : coop ? walk_coop<false> : walk;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, buf, nlines, iters / 10, act, out);  // warm
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, buf, nlines, iters, act, out);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            CHECK(hipGetLastError());
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double ns_step = ms * 1e6 / iters;  // every wave runs `iters` steps concurrently
            if (act == 64) t64 = (double)blocks * 64 * iters / (ms * 1e3);
            if (act == 8) t8 = (double)blocks * 8 * iters / (ms * 1e3);
            std::printf("  %9.1f", ns_step);
        }
        std::printf("   (%.0f | %.0f)\n", t64, t8);
    }
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
