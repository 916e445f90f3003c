// rt_schedule.hip -- primary pass + longest-first job order for the persistent render kernels
// (included by rt_runtime.hip after rt_megakernel.hip).
//
// Why: the persistent kernels hand out pixels from one counter in tile order.  A pixel's path is
// a sequence of dependent queries interleaved with 63 other lanes, so its latency under load is
// long (~0.1-1 ms on the dragon) while its cost is wildly uneven: a background pixel is one
// query, a mirror pixel up to ~10.  Handed out in image order, the last mirror pixels start late
// and the chip drains for the length of their paths: on C3 the first wave retires at 48 % of the
// kernel time and the mean wave lives 65 % of it (tools/wave_trace.py).
//
// Here a lean first kernel traces every pixel's camera ray (tile-coherent, one ray per lane) and
// stores the primary hit; a scan + scatter orders the jobs "primary hit" first, "miss" last; the
// persistent kernel then takes jobs in that order and starts each pixel from its stored primary
// hit.  Longest-processing-time-first: the expensive paths start at once and the cheap misses
// fill the drain.  Every query keeps its reference arithmetic, so images and ray counts are
// bit-identical (only the schedule changes).

namespace rt {

// one camera ray per pixel (sample 0; only used when a pixel has one sample)
template <bool COUNT, int BW>
__global__ __launch_bounds__(64) void primary_kernel(KParams P, float* __restrict__ pre_t, int* __restrict__ pre_rec,
                                                     int* __restrict__ tile_hits, int ntiles) {
    __shared__ int stack_lds[RT_STACK_SIZE * RT_WAVE];
    const int lane = (int)threadIdx.x;
    int* stk = stack_lds + lane;
    Cnt cnt{};
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int job = tile * 64 + lane;
        Lane L;
        L.sample = 0;
        const bool ok = job_pixel(P, job, L);
        bool hit = false;
        if (ok) {
            queue_camera(P, L);
            Best b;
            hit = trace_query8<COUNT, BW>(P.S, L.qo, L.qd, L.qt, 0.0f, P.use_bvh != 0, false, b, stk, cnt);
            pre_t[job] = b.t;
            pre_rec[job] = hit ? b.rec : RT_NO_HIT;
            cnt.rays++;
        }
        const int h = __popcll(__ballot(hit));
        if (lane == 0) tile_hits[tile] = h;
    }
    flush_counters<COUNT>(P, cnt);  // one atomic per wave (rays, and the counting-build counters)
}

// exclusive prefix sum of the per-tile hit counts (one block of 1024 threads; total at [ntiles])
__global__ __launch_bounds__(1024) void tile_scan_kernel(const int* __restrict__ tile_hits, int* __restrict__ tile_off,
                                                         int ntiles) {
    __shared__ int part[1024];
    const int t = (int)threadIdx.x;
    const int per = (ntiles + 1023) / 1024;
    const int b = t * per, e = min(ntiles, b + per);
    int s = 0;
    for (int i = b; i < e; ++i) s += tile_hits[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan of the partial sums
        const int v = (t >= d) ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - s;
    for (int i = b; i < e; ++i) {
        tile_off[i] = run;
        run += tile_hits[i];
    }
    if (t == 1023) tile_off[ntiles] = part[1023];
}

// job order: hits first (tile order, lane order inside a tile), then misses and padding jobs
__global__ __launch_bounds__(64) void job_order_kernel(const int* __restrict__ pre_rec, const int* __restrict__ tile_off,
                                                       int* __restrict__ order, KParams P, int ntiles) {
    const int lane = (int)threadIdx.x;
    const int total_hits = tile_off[ntiles];
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int job = tile * 64 + lane;
        Lane L;
        const bool ok = job_pixel(P, job, L);
        const bool hit = ok && pre_rec[job] != RT_NO_HIT;
        const unsigned long long hm = __ballot(hit);
        const unsigned long long below = (1ull << lane) - 1ull;
        const int hoff = tile_off[tile];
        if (hit) {
            order[hoff + __popcll(hm & below)] = job;
        } else {
            const int moff = total_hits + (tile * 64 - hoff);  // misses of earlier tiles come first
            order[moff + __popcll(~hm & below)] = job;
        }
    }
}

// ---- cost-ordered schedule (RT_SCHED=2) ----------------------------------------------------
// Jobs ordered by the number of queries each pixel took in the previous frame of the same
// launch geometry, most expensive first (16 log2 buckets, a stable radix partition: per-block
// histograms, one scan, per-block scatter; no global atomics).
#define CS_BUCKETS 16
#define CS_BLOCK 1024

__device__ __forceinline__ int cost_bucket(int c) {
    const int b = (c <= 1) ? 0 : (31 - __clz(c));
    return (CS_BUCKETS - 1) - min(CS_BUCKETS - 1, b);  // bucket 0 = most expensive
}

__global__ __launch_bounds__(CS_BLOCK) void cost_hist_kernel(const int* __restrict__ cost, int njobs,
                                                             int* __restrict__ block_hist) {
    __shared__ int h[CS_BUCKETS];
    const int t = (int)threadIdx.x;
    if (t < CS_BUCKETS) h[t] = 0;
    __syncthreads();
    const int j = blockIdx.x * CS_BLOCK + t;
    if (j < njobs) atomicAdd(&h[cost_bucket(cost[j])], 1);
    __syncthreads();
    if (t < CS_BUCKETS) block_hist[t * gridDim.x + blockIdx.x] = h[t];  // bucket-major
}

// exclusive scan of block_hist[bucket][block] in place (one block)
__global__ __launch_bounds__(1024) void cost_scan_kernel(int* __restrict__ a, int n) {
    __shared__ int part[1024];
    const int t = (int)threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int b = t * per, e = min(n, b + per);
    int s = 0;
    for (int i = b; i < e; ++i) s += a[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = (t >= d) ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - s;
    for (int i = b; i < e; ++i) {
        const int x = a[i];
        a[i] = run;
        run += x;
    }
}

// order[offset of (bucket, block) + rank inside the block] = job; ranks by lane-ordered ballots
__global__ __launch_bounds__(CS_BLOCK) void cost_scatter_kernel(const int* __restrict__ cost, int njobs,
                                                                const int* __restrict__ block_off,
                                                                int* __restrict__ order) {
    __shared__ int wave_cnt[CS_BLOCK / 64][CS_BUCKETS];
    const int t = (int)threadIdx.x, w = t >> 6, lane = t & 63;
    const int j = blockIdx.x * CS_BLOCK + t;
    const int b = (j < njobs) ? cost_bucket(cost[j]) : -1;
    int rank = 0;
    for (int k = 0; k < CS_BUCKETS; ++k) {
        const unsigned long long m = __ballot(b == k);
        if (b == k) rank = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wave_cnt[w][k] = __popcll(m);
    }
    __syncthreads();
    if (b >= 0) {
        int before = 0;  // same bucket in earlier waves of the block
        for (int v = 0; v < w; ++v) before += wave_cnt[v][b];
        order[block_off[b * gridDim.x + blockIdx.x] + before + rank] = j;
    }
}

}  // namespace rt
