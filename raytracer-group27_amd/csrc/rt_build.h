// rt_build.h -- rt_create's GPU scene build (rt_build.hip): reference BVH, BVH2, BVH8 and records.
#pragma once
#include <string>

#include "bvh_build.h"

namespace rt {

struct GpuBuild {
    RefBvh ref;            // the reference BVH's nodes, leaf paths and sphere keys (triangle keys are in the records)
    void* tri = nullptr;   // device: ntri x 64-B triangle records in BVH8 leaf order (hipMalloc, caller frees)
    void* nodes = nullptr; // device: nnodes x 128-B BVH8 nodes (hipMalloc, caller frees)
    int nnodes = 0, max_depth = 0;
    int bvh2_nodes = 0, bvh2_depth = 0;
    double ms[4] = {0, 0, 0, 0};
};

// Builds on the current device from host positions [ntri][3][3] and spheres [nsph][4]; false (with
// err) when the scene does not suit the GPU path (too few objects, degenerate large ranges) or on a
// HIP error -- the caller then builds on the host.
bool gpu_build(const float* positions, int ntri, const float* sph4, int nsph, GpuBuild& out, std::string& err);

}  // namespace rt
