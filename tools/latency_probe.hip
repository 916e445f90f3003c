// Developer tool: dependent-load latency on one wave (pointer chase), for a working set that fits
// L1 / L2 / MALL / only HBM -- the per-step cost floor of a traversal step.
// Build: hipcc --offload-arch=gfx950 -O2 tools/latency_probe.hip -o tools/latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>

__global__ void chase(const unsigned* __restrict__ next, unsigned start, int steps, unsigned* out,
                      unsigned long long* cycles) {
    unsigned p = start + (threadIdx.x >> 6);  // per-lane value (0 for one wave): vector loads, as in the traversal
    const unsigned long long t0 = wall_clock64();
    for (int i = 0; i < steps; ++i) p = next[p];
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[0] = p;
        cycles[0] = t1 - t0;
    }
}

int main() {
    const size_t sizes[] = {16u << 10, 1u << 20, 3u << 20, 64u << 20, 192u << 20, 1024u << 20};
    for (size_t bytes : sizes) {
        const size_t n = bytes / 4;
        const size_t stride = 32;  // 128-B lines
        const size_t lines = n / stride;
        std::vector<unsigned> order(lines);
        for (size_t i = 0; i < lines; ++i) order[i] = (unsigned)i;
        std::shuffle(order.begin(), order.end(), std::mt19937(7));
        std::vector<unsigned> next(n, 0);
        for (size_t i = 0; i < lines; ++i) next[order[i] * stride] = order[(i + 1) % lines] * stride;
        unsigned *d, *o;
        unsigned long long* c;
        hipMalloc(&d, n * 4);
        hipMalloc(&o, 4);
        hipMalloc(&c, 8);
        hipMemcpy(d, next.data(), n * 4, hipMemcpyHostToDevice);
        const int steps = 20000;
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, order[0] * (unsigned)stride, steps, o, c);  // warm
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, order[0] * (unsigned)stride, steps, o, c);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long cyc = 0;
        hipMemcpy(&cyc, c, 8, hipMemcpyDeviceToHost);
        printf("working set %8zu KB: %.0f ns per dependent load (events), %.0f (wall_clock64 x10 ns)\n", bytes >> 10,
               ms * 1e6 / steps, cyc * 10.0 / steps);
        hipFree(d);
        hipFree(o);
        hipFree(c);
    }
    return 0;
}
