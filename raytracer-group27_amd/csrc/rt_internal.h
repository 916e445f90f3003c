// rt_internal.h -- shared host-side declarations between the C++ ingest code and the HIP runtime.
#pragma once
#include <string>

namespace rt {
void set_error(const std::string& msg);
}

#define RT_MAX_DEPTH 16        // frames of the recursion stack (reference default depth 5, configs <= 8)
#define RT_STACK_SIZE 40       // BVH2 traversal stack entries per lane (BVH depth <= 37, bvh_build.cpp)
#define RT_STACK8 12           // dynamic-fetch kernel: BVH8 group-stack entries per lane (BVH8 depth <= 13;
                               // the 800k-triangle dragon proxy has depth 7); deeper trees run the whole-traversal kernel
#define RT_MAX_REF_NODES 31    // depth-4 binary reference BVH
#define RT_WAVE 64
#define RT_STATS_EXTRA (16 + 8 * 16)  // d_stats: 16 counters, the 8 per-XCD job heads, then 16 more counters
