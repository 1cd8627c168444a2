// schedule.hip -- scenario launch order for the next batched solve.
//
// PDHG iteration counts of a scenario change slowly from one PH iteration to the next (warm
// starts), so the previous solve's counts predict the next one's work.  Launching scenarios
// heaviest-first (longest-processing-time order) shortens the grid's tail, and it places
// scenarios of similar work side by side in the lane-local kernel's multi-scenario waves, where a
// wave runs until its slowest scenario converges.
//
// One single-workgroup counting sort on the iteration count in units of the check interval
// (every count is a multiple of it): LDS histogram, descending exclusive scan, scatter.  Stream-
// ordered behind the solve, no host round trip.  The order inside a bucket is whatever the LDS
// atomics produce; it does not matter for results because scenarios never interact in a solve.
#include "phg_internal.h"

namespace phg {

constexpr int kBuckets = 4096;

__global__ __launch_bounds__(1024) void schedule_kernel(const int* iters, int S, int unit, int* order) {
    __shared__ int cnt[kBuckets];
    __shared__ int wsum[16];
    const int tid = threadIdx.x;
    for (int b = tid; b < kBuckets; b += 1024) cnt[b] = 0;
    __syncthreads();
    auto bucket = [&](int s) {
        // descending: the heaviest scenarios get the lowest bucket index
        const int u = iters[s] / unit;
        return kBuckets - 1 - min(u, kBuckets - 1);
    };
    for (int s = tid; s < S; s += 1024) atomicAdd(&cnt[bucket(s)], 1);
    __syncthreads();
    // exclusive scan of 4096 counts: 4 per thread, then a scan of the 1024 thread totals
    int v[4], tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = cnt[tid * 4 + i]; tot += v[i]; }
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if ((tid & 63) >= o) incl += t;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = incl;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < (tid >> 6); ++w) base += wsum[w];
    int run = base + incl - tot;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) { cnt[tid * 4 + i] = run; run += v[i]; }
    __syncthreads();
    for (int s = tid; s < S; s += 1024) order[atomicAdd(&cnt[bucket(s)], 1)] = s;
}

hipError_t schedule_launch(const int* iters, int S, int unit, int* order, hipStream_t st) {
    hipLaunchKernelGGL(schedule_kernel, dim3(1), dim3(1024), 0, st, iters, S, unit > 0 ? unit : 1, order);
    return hipGetLastError();
}

}  // namespace phg
