// Developer tool: host BVH build stages on a synthetic 800k-triangle knot (timing + structure hash).
// g++ -O3 -std=c++17 -pthread -I raytracer-group27_amd/csrc tools/bvh_build_time.cpp raytracer-group27_amd/csrc/bvh_build.cpp
#include <chrono>
#include <cstdio>
#include <cmath>
#include <vector>
#include "bvh_build.h"
using namespace rt;
int main() {
    // torus-knot-ish synthetic triangles like the dragon proxy: 800k tris
    const int U = 2000, V = 200;
    std::vector<float> pos;
    pos.reserve((size_t)U * V * 18);
    auto P = [&](int i, int j, float* o) {
        const float u = 6.2831853f * i / U, v = 6.2831853f * j / V;
        const float p = 2, q = 3;
        const float r = std::cos(q * u) + 2;
        const float cx = r * std::cos(p * u), cy = r * std::sin(p * u), cz = -std::sin(q * u);
        o[0] = cx + 0.3f * std::cos(v); o[1] = cy + 0.3f * std::sin(v); o[2] = cz + 0.3f * std::cos(v + u);
    };
    for (int i = 0; i < U; ++i) for (int j = 0; j < V; ++j) {
        float a[3], b[3], c[3], d[3];
        P(i, j, a); P(i + 1, j, b); P(i + 1, j + 1, c); P(i, j + 1, d);
        for (float* t : {a, b, c}) pos.insert(pos.end(), t, t + 3);
        for (float* t : {a, c, d}) pos.insert(pos.end(), t, t + 3);
    }
    const int ntri = (int)(pos.size() / 9);
    auto t0 = std::chrono::steady_clock::now();
    RefBvh ref = build_ref_bvh(pos.data(), ntri, nullptr, 0, 4);
    auto t1 = std::chrono::steady_clock::now();
    Bvh2 b2 = build_bvh2(pos.data(), ntri, 1e-4f, 4);  // build_bvh2 x3
    auto ta = std::chrono::steady_clock::now();
    { Bvh2 bx = build_bvh2(pos.data(), ntri, 1e-4f, 4); }
    auto tb = std::chrono::steady_clock::now();
    std::printf("second bvh2 %.1f ms\n", std::chrono::duration<double, std::milli>(tb - ta).count());
    auto t2 = std::chrono::steady_clock::now();
    Bvh8 b8 = build_bvh8(b2, 8);
    auto t3 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::printf("ntri %d: ref %.1f ms, bvh2 %.1f ms, bvh8 %.1f ms (depth %d)\n", ntri, ms(t0, t1), ms(t1, t2), ms(t2, t3), b8.max_depth);
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) { const unsigned char* c = (const unsigned char*)p; for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; } };
    mix(b8.nodes.data(), b8.nodes.size() * 4); mix(b8.order.data(), b8.order.size() * 4);
    mix(ref.tri_key.data(), ref.tri_key.size() * 4); mix(ref.tri_leaf.data(), ref.tri_leaf.size() * 4);
    for (auto& n : ref.nodes) { mix(&n.lower, sizeof(n.lower)); mix(&n.upper, sizeof(n.upper)); }
    std::printf("hash %016llx nodes8 %zu\n", h, b8.nodes.size() / 32);
}

