// schedule.h -- the scenario launch order for the next batched solve, as a workgroup device
// function (schedule.hip's own launch, and the extra workgroup of the pipelined node-sum launch,
// ph_update.hip node_sums_kernel HEADX).
//
// PDHG iteration counts of a scenario change slowly from one PH iteration to the next (warm
// starts), so the previous solve's counts predict the next one's work.  Launching scenarios
// heaviest-first (longest-processing-time order) shortens the grid's tail, and it places scenarios
// of similar work side by side in the lane-local kernel's multi-scenario waves, where a wave runs
// until its slowest scenario converges.
//
// A counting sort on the iteration count in units of the check interval (every count is a multiple
// of it): LDS histogram, descending exclusive scan, scatter -- per-lane LDS atomics (a wave-
// aggregated form, one atomic per distinct bucket per wave with its peers found by ballot, measured
// 2.5x slower on farmer 10 000: 25.7 vs 10.3 us; the counts spread over ~20 buckets per wave).  The
// order inside a bucket is whatever the LDS atomics produce; it does not matter for results because
// scenarios never interact in a solve.
#pragma once
#include "phg_internal.h"

namespace phg {

constexpr int kSchedBuckets = 4096;

// NT threads (whole waves, dividing kSchedBuckets); B: rows of counts read at once per lane (B
// loads in flight instead of one dependent L2 round trip per row: the 256-thread form; the
// 1 024-thread launch reads them one by one -- 8 at once measured 13.9 vs 10.3 us on farmer
// 10 000); cnt: kSchedBuckets ints of LDS, wsum: NT / 64 ints of LDS.  Every thread of the
// workgroup must call it.
template <int NT, int B>
__device__ __forceinline__ void schedule_block(const int* __restrict__ iters, int S, int unit, int* __restrict__ order,
                                               int* cnt, int* wsum) {
    static_assert(NT % 64 == 0 && kSchedBuckets % NT == 0, "whole waves, whole bucket slices");
    constexpr int PER = kSchedBuckets / NT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    for (int b = tid; b < kSchedBuckets; b += NT) cnt[b] = 0;
    __syncthreads();
    auto bucket = [&](int s) {
        // descending: the heaviest scenarios get the lowest bucket index
        const int u = iters[s] / unit;
        return kSchedBuckets - 1 - min(u, kSchedBuckets - 1);
    };
    // pass 0: histogram; pass 1: scatter (cnt then holds each bucket's next free slot)
    for (int pass = 0; pass < 2; ++pass) {
        for (int s0 = tid; s0 < S; s0 += NT * B) {
            int bk[B];
#pragma unroll
            for (int j = 0; j < B; ++j) {
                const int s = s0 + j * NT;
                bk[j] = s < S ? bucket(s) : 0;
            }
#pragma unroll
            for (int j = 0; j < B; ++j) {
                const int s = s0 + j * NT;
                if (s < S) {
                    const int slot = atomicAdd(&cnt[bk[j]], 1);
                    if (pass == 1) order[slot] = s;
                }
            }
        }
        __syncthreads();
        if (pass == 1) break;
        // exclusive scan of the bucket counts: PER per thread, then the thread totals
        int v[PER], tot = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) { v[i] = cnt[tid * PER + i]; tot += v[i]; }
        int incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        if (lane == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < (tid >> 6); ++w) base += wsum[w];
        int run = base + incl - tot;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; ++i) { cnt[tid * PER + i] = run; run += v[i]; }
        __syncthreads();
    }
}

}  // namespace phg
