// stream_sync.h -- cross-workgroup primitives of the multi-workgroup PDHG kernels
// (pdhg_stream.hip, pdhg_border.hip), gfx950.
//
// Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1): values other
// workgroups read are stored sc1 (write-through) and EVERY load of them is an sc1 load; each
// workgroup signals with one agent-scope add by one lane behind a workgroup barrier that follows
// every wave's vmcnt(0); the consumer polls with sc1 loads and its other waves load after a
// workgroup barrier; one 1024-thread workgroup per CU (<= 128 VGPRs: the CU's 16 wave slots).
#pragma once
#include <cstdlib>

#include "wave_ops.h"

namespace phg {

// K > 1 workgroups per scenario are launched cooperatively (hipLaunchCooperativeKernel: the
// runtime guarantees co-residency or fails).  PHG_COOP=0: a plain launch of the same grid -- every
// workgroup is resident anyway (one per CU, grid <= the CU count, nothing else on the device), and
// the bounded waits of scen_barrier / the granule reads turn a missing co-resident into an error,
// never a hang.  For rocprofv3: its kernel-trace teardown segfaults after any cooperative launch
// (tools/repro/coop_exit.hip: a 64-thread cooperative kernel alone reproduces it, the plain launch
// of the same kernel does not), so UC is profiled with PHG_COOP=0.
inline bool coop_launch_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("PHG_COOP");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

// write-through (sc1) store and L1-bypassing (sc1) load of the values other workgroups read
__device__ __forceinline__ void put(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double get(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// barrier of the K workgroups of one slot: cnt[0] counts arrivals (monotonic within the launch,
// zeroed before it); target = (barrier number) * K.  The wait is bounded (~0.5 s): past it the
// workgroup reports failure and sets the device error flag, so the grid always drains.
__device__ __forceinline__ bool scen_barrier(unsigned* cnt, unsigned target, int* err) {
    __shared__ int s_ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int ok = 1;
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 23)) {
                ok = 0;
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// p[0] + p[s] + ... + p[(cnt - 1) s] added in that order (the same bits as the plain loop), the
// LDS loads issued eight at a time instead of one dependent load per add; cnt >= 1
__device__ __forceinline__ double ordered_sum(const double* p, int s, int cnt) {
    double acc = p[0];
    int q = 1;
    for (; q + 8 <= cnt; q += 8) {
        double r[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = p[(q + i) * s];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += r[i];
    }
    for (; q < cnt; ++q) acc += p[q * s];
    return acc;
}

// workgroup sum of V values (V <= 16), same bits in every thread; fixed order: wave partials in
// wave order, added by thread k < V for value k (in place, red[k NW]) and read back by every thread
template <int NT, int V>
__device__ __forceinline__ void wg_sum(double (&v)[V], double* red) {
    constexpr int NW = NT / 64;
    gsum_many<64, V>(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < V; ++k) red[k * NW + w] = v[k];
    __syncthreads();
    if (threadIdx.x < V) {
        double r[NW];
#pragma unroll
        for (int u = 0; u < NW; ++u) r[u] = red[threadIdx.x * NW + u];
        double t = r[0];
#pragma unroll
        for (int u = 1; u < NW; ++u) t += r[u];
        red[threadIdx.x * NW] = t;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = red[k * NW];
    __syncthreads();
}

}  // namespace phg
