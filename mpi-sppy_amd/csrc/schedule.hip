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
// The atomics are wave-aggregated (wave_add) and each thread's count loads are batched.
#include "phg_internal.h"

namespace phg {

constexpr int kBuckets = 4096;

// cnt[b] += (number of lanes of the wave with bucket b), for every b present in the wave; returns
// the old cnt[b] plus the lane's rank among those lanes (b < 0: inactive lane, returns -1).  One
// LDS atomic per distinct bucket of the wave instead of one per lane.
__device__ __forceinline__ int wave_add(int* cnt, int b) {
    int out = -1;
    unsigned long long todo = __builtin_amdgcn_ballot_w64(b >= 0);
    while (todo) {
        const int leader = __builtin_ctzll(todo);
        const int bl = __shfl(b, leader, 64);
        const unsigned long long m = __builtin_amdgcn_ballot_w64(b == bl);
        int base = 0;
        if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&cnt[bl], __builtin_popcountll(m));
        base = __shfl(base, leader, 64);
        if (b == bl) out = base + __builtin_popcountll(m & ((1ull << (threadIdx.x & 63)) - 1ull));
        todo &= ~m;
    }
    return out;
}

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
    // warm-started iteration counts fall into a handful of buckets, so per-lane LDS atomics would
    // serialise on the same few addresses: the lanes of a wave that share a bucket are counted by
    // one atomic of their leader (wave_add), which also hands each lane its rank inside the group
    // (eight scenarios per thread per step: their count loads are issued together, so a pass costs
    // ~S / 8192 global-load round trips instead of S / 1024)
    constexpr int U = 8;
    auto pass = [&](auto f) {
        for (int s0 = 0; s0 < S; s0 += 1024 * U) {
            int bk[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int s = s0 + u * 1024 + tid;
                bk[u] = s < S ? bucket(s) : -1;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) f(s0 + u * 1024 + tid, bk[u]);
        }
    };
    pass([&](int, int b) { wave_add(cnt, b); });
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
    pass([&](int s, int b) {
        const int pos = wave_add(cnt, b);
        if (b >= 0) order[pos] = s;
    });
}

hipError_t schedule_launch(const int* iters, int S, int unit, int* order, hipStream_t st) {
    hipLaunchKernelGGL(schedule_kernel, dim3(1), dim3(1024), 0, st, iters, S, unit > 0 ? unit : 1, order);
    return hipGetLastError();
}

}  // namespace phg
