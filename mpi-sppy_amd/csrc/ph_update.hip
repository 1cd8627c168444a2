// ph_update.hip -- fused PH node-average / dual-weight / convergence kernels.
//
// Restates, for all local scenarios at once and with deterministic fixed-order reductions
// (no floating-point atomics):
//   _Compute_Xbar     mpisppy/phbase.py:32-112   node sums of prob_coeff*x and prob_coeff*x^2
//   Update_W          mpisppy/phbase.py:301-326  W += rho (x - xbar)
//   convergence_diff  mpisppy/phbase.py:349-371  (1/P) sum_v  sum_{s in v,k} |x - xbar| / count_v
// Two launches per PH iteration.  Node sums are reduced per "segment" (a contiguous scenario range
// inside one node) and then, by the last workgroup, per node in segment order; the cross-GPU
// all-reduce (RCCL) of the 2*N_tot node sums and of the 2*P+2 convergence partials happens
// between / after the kernels (see include/phg.h).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "phg_internal.h"
#include "ph_sums.h"
#include "schedule.h"

namespace phg {

// Handed-off partials are published write-through: every store of them is an agent-scope (sc1)
// store, so no workgroup needs an agent-scope release (buffer_wbl2, a write-back of the XCD's whole
// L2 -- ~0.4 us per workgroup per XCD, serialised, measured on the PH-update sweep).  The consumer
// side keeps its agent-scope acquire (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores,
// every storing wave's vmcnt(0), a workgroup barrier, then the counter add; acquire, then loads).
__device__ __forceinline__ void publish(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// "Last workgroup done" hand-off: every storing wave drains its (published) stores, lane 0 takes a
// ticket; the workgroup whose ticket is last acquires at agent scope and finishes the reduction in
// a FIXED order, so the result does not depend on which workgroup arrived last.  That workgroup
// also re-zeroes the counter for the next (stream-ordered) launch.
__device__ __forceinline__ bool last_workgroup(unsigned* counter) {
    __shared__ unsigned s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = prev == gridDim.x - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_last = last ? 1u : 0u;
    }
    __syncthreads();
    return s_last != 0u;
}

// conv = (1/P) sum_v convpart[2v] / convpart[2v+1] (phbase.py:349-371; virtual ranks with no
// nonants contribute 0) -- +inf while convpart[2P+2] (the flag a W update sets) is 0, i.e. before
// the first W update: no convergence metric exists yet.  One 256-thread workgroup, fixed-order tree
// over the virtual ranks; every thread returns the same value (the same bits wherever computed).
__device__ double conv_value_block(const double* convpart, int P, double* red) {
    double t = 0.0;
    for (int v = threadIdx.x; v < P; v += 256)
        if (convpart[2 * v + 1] > 0.0) t += convpart[2 * v] / convpart[2 * v + 1];
    red[threadIdx.x] = t;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    const double v = convpart[2 * P + 2] > 0.0 ? red[0] / (double)P : INFINITY;
    __syncthreads();
    return v;
}

// gate = {conv, not optimal, NaN} (the status counts ride in convpart[2P], [2P+1]).  The same
// three values go to fine-grained pinned host memory followed (drained, publish_host_gate) by the
// sequence number `seq` in word 3 of slot seq mod 2 of the [2][4] ring: the host polls that word,
// so no event has to pass through the GPU's queue (two slots: a solve's fused tail, ph_tail.h, may
// publish the NEXT value before the host has read this one).  Called by one thread.
__device__ void publish_gate(double conv, const double* convpart, int P, double* gate, double* gate_host,
                             double seq) {
    const double g[3] = {conv, convpart[2 * P], convpart[2 * P + 1]};
    for (int i = 0; i < 3; ++i) gate[i] = g[i];
    if (gate_host) publish_host_gate(gate_host, g[0], g[1], g[2], seq);
}

__device__ void conv_gate_block(const double* convpart, int P, double* gate, double* gate_host, double seq) {
    __shared__ double red[256];
    const double conv = conv_value_block(convpart, P, red);
    if (threadIdx.x == 0) publish_gate(conv, convpart, P, gate, gate_host, seq);
}

// "Last K workgroups" hand-off: as last_workgroup, but the K workgroups that arrive last all
// return a rank r in [0, K) (the others -1) once EVERY workgroup has arrived, so a final reduction
// too large for one workgroup is split K ways by rank -- deterministic, since the work of rank r
// does not depend on which workgroup holds it.  The K ranked workgroups spin only on arrivals of
// workgroups that are already running (K is far below the resident capacity).  finish_k() re-arms
// the counters for the next launch once all K are done.
// (total: the workgroups that take a ticket -- the whole grid unless it carries extra ones)
__device__ __forceinline__ int last_k_workgroups(unsigned* counter, int K, int total) {
    __shared__ int s_rank;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int rank = (int)prev - (total - K);
        if (rank >= 0) {
            while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)total)
                __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        s_rank = rank;
    }
    __syncthreads();
    return s_rank;
}

__device__ __forceinline__ void finish_k(unsigned* counter, unsigned* done, int K) {
    __syncthreads();
    if (threadIdx.x == 0) {
        // relaxed: the counters are only re-read by the next (stream-ordered) launch
        if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)K - 1) {
            __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Node sums (first half of _Compute_Xbar).  One workgroup per node segment (a contiguous scenario
// range inside one node, sized on the host so that large batches get ~256 segments per level) and
// 256-nonant column chunk (blockIdx.y; wide nodes get several workgroups per segment, so the
// number of loads in flight does not depend on the final reduction's segment count);
// thread t handles nonant k = t % klen of scenarios s0 + t / klen + q*i (q = 256 / klen lanes per
// nonant) -> coalesced rows of xN, 8 rows in flight per thread.  The last K workgroups then add
// every node's segment partials in segment order (element range split K ways):
// nodesum[e] = sum p x, nodesum[N_tot + e] = sum p x^2 (the buffer the cross-GPU all-reduce sums).
template <bool NTL = false>
__device__ __forceinline__ void node_sum_partials(const PhArgs& a) {
    __shared__ double sh[2 * 512];
    const int tid = threadIdx.x;
    const NodeSeg sg = a.seg[blockIdx.x];
    double* out = a.segpart + (long)blockIdx.x * 2 * a.maxk;
    // element pairs with 16-byte loads when every row's slice starts 16-byte aligned (even N,
    // offset and length) and the probability is per node: thread (k2, so) adds nonants 2 k2, 2 k2 + 1
    // of rows s0 + so + j q2 (eight rows in flight), then the q2 row lanes are added in order
    // (ph_sums.h: the per-thread sums, shared with the solve tail's one-wave form)
    const bool pairs = nsum_pairs(a, sg);
    for (int k0 = 256 * (int)blockIdx.y; k0 < sg.klen; k0 += 256 * (int)gridDim.y) {
        const NsumThread th = nsum_thread(pairs, sg.klen, k0, sg.s1 - sg.s0, tid);
        double r[4];
        nsum_thread_sums<NTL>(a, sg, k0, th, pairs, r);
        nsum_stage(sh, th, pairs, r);
        __syncthreads();
        if (tid < th.kl) {
            double t1 = 0.0, t2 = 0.0;
            for (int j = 0; j < th.q; ++j) { t1 += sh[j * th.kl + tid]; t2 += sh[512 + j * th.kl + tid]; }
            publish(&out[k0 + tid], t1);
            publish(&out[a.maxk + k0 + tid], t2);
        }
        __syncthreads();
    }
}

// final node sums of elements [e_lo, e_hi) (rank `rank` of K): per node, its segments' partials in
// segment order, written with the given store -- MODE 0: plain; 1: sc1, and x-bar / x-sq-bar too
// (ph_step_kernel); 2: sc1, node sums only (other workgroups of the same launch read them); 3:
// plain, and kept in `stash` (LDS, [2][256]) when the rank has <= 256 elements (the one-hop HEADX
// writes x-bar from there once it knows conv)
template <int MODE>
__device__ __forceinline__ void node_sum_final(const PhArgs& a, double* nodesum, int rank, int K,
                                               double* stash = nullptr) {
    const int tid = threadIdx.x;
    // elements [e_lo, e_hi) of this rank; T lanes per element (power of two <= 64), each summing
    // every T-th segment of the node, then a fixed xor-butterfly over the T lanes: wide enough to
    // hide the L2 latency when there are few elements per rank, one lane per element otherwise
    const int e_lo = (int)((long)a.N_tot * rank / K), e_hi = (int)((long)a.N_tot * (rank + 1) / K);
    const int ne = e_hi - e_lo;
    int T = 1;
    while (T < 64 && T * 2 * ne <= 256) T *= 2;
    const int E = 256 / T;
    const int sub = tid % T;
    for (int e0 = e_lo; e0 < e_hi; e0 += E) {
        const int e = e0 + tid / T;
        double t1 = 0.0, t2 = 0.0;
        if (e < e_hi) {
            // node g with node_off[g] <= e < node_off[g] + level_len[level[g]]
            int lo = 0, hi = a.n_nodes - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (a.node_off[mid] <= e) lo = mid; else hi = mid - 1;
            }
            const int i = e - a.node_off[lo];
#pragma unroll 8
            for (int g = a.node_first_seg[lo] + sub; g < a.node_first_seg[lo + 1]; g += T) {
                t1 += a.segpart[(long)g * 2 * a.maxk + i];
                t2 += a.segpart[(long)g * 2 * a.maxk + a.maxk + i];
            }
        }
        for (int o = 1; o < T; o <<= 1) {
            t1 += __shfl_xor(t1, o, 64);
            t2 += __shfl_xor(t2, o, 64);
        }
        if (e < e_hi && sub == 0) {
            if (MODE == 1 || MODE == 2) {
                publish(&nodesum[e], t1);
                publish(&nodesum[a.N_tot + e], t2);
                if (MODE == 1) {
                    publish(&a.xbar[e], t1);
                    publish(&a.xsqbar[e], t2);
                }
            } else {
                nodesum[e] = t1;
                nodesum[a.N_tot + e] = t2;
                if (MODE == 3 && ne <= 256) {
                    stash[e - e_lo] = t1;
                    stash[256 + e - e_lo] = t2;
                }
            }
        }
    }
}

// Folded W update (PdhgArgs::fold_w): the solve prologue left each scenario's sum |x - xbar|
// (conv_s) and the status of the solve that produced x (fold_st).  Conv segment b's partials:
// fixed-order sums over its scenario range, published for conv_partials_final.
// FoldHead: a thread's first element of the segment, loaded ahead (node_sums_kernel issues it before
// the node-sum pass over x, so the two load latencies overlap) and added in the same order as the loop
struct FoldHead {
    double v = 0.0;
    int st = 0;
    bool on = false;
};

__device__ __forceinline__ FoldHead fold_conv_head(const PhArgs& a, int b) {
    FoldHead h;
    const int s = a.cseg_s0[b] + (int)threadIdx.x;
    if (s < a.cseg_s1[b]) {
        h.v = a.conv_s[s];
        h.st = a.fold_st[s];
        h.on = true;
    }
    return h;
}

__device__ void fold_conv_segment(const PhArgs& a, int b, FoldHead h = FoldHead{}, bool pre = false) {
    __shared__ double red[4];
    __shared__ int bad[8];
    const int tid = threadIdx.x;
    const int s0 = a.cseg_s0[b], s1 = a.cseg_s1[b];
    if (!pre) h = fold_conv_head(a, b);
    double acc = 0.0;
    int nb = 0, nn = 0;
    if (h.on) {
        acc += h.v;
        nb += h.st != 0;
        nn += h.st == 2;
    }
    for (int s = s0 + tid + 256; s < s1; s += 256) {
        acc += a.conv_s[s];
        const int st = a.fold_st[s];
        nb += st != 0;
        nn += st == 2;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        acc += __shfl_xor(acc, o, 64);
        nb += __shfl_xor(nb, o, 64);
        nn += __shfl_xor(nn, o, 64);
    }
    if ((tid & 63) == 0) { red[tid >> 6] = acc; bad[tid >> 6] = nb; bad[4 + (tid >> 6)] = nn; }
    __syncthreads();
    if (tid == 0) {
        publish(&a.csegpart[b], ((red[0] + red[1]) + red[2]) + red[3]);
        publish(&a.csegbad[2 * b], bad[0] + bad[1] + bad[2] + bad[3]);
        publish(&a.csegbad[2 * b + 1], bad[4] + bad[5] + bad[6] + bad[7]);
    }
    __syncthreads();
}

// virtual ranks up to which the HEADX ranks each form conv themselves (their LDS copy of the partials)
constexpr int kHeadxOneHopP = 128;

// a thread's conv segment (g = vr_first[0] + tid) loaded ahead for conv_partials_final (P = 1,
// <= 256 segments: one per thread) -- the same element the loop would read, added in the same order
struct ConvPre {
    double v = 0.0;
    int b = 0, n = 0;
    bool on = false;
};

__device__ __forceinline__ ConvPre conv_pre_load(const PhArgs& a) {
    ConvPre p;
    const int g = a.vr_first[0] + (int)threadIdx.x;
    if (g < a.vr_first[1]) {
        p.v = a.csegpart[g];
        p.on = true;
    }
    if ((int)threadIdx.x < a.n_cseg) {
        p.b = a.csegbad[2 * threadIdx.x];
        p.n = a.csegbad[2 * threadIdx.x + 1];
    }
    return p;
}

// the last workgroup's part of convergence_diff (declared here, defined below)
__device__ __forceinline__ void conv_partials_final(const PhArgs& a, double* convpart, const ConvPre* pre = nullptr);

// HEADX (phg_ph_step on one GPU with the folded update): the x-bar head rides along -- the last of
// the K ranks to finish (every node sum published) reduces the conv partials, computes conv
// exactly as xbar_head_kernel does from the same buffer, publishes the gate and, unless conv is
// below head_thr, copies the node sums into x-bar / x-sq-bar: one launch instead of two.
//
// (PhArgs::onehop -- PHG_HEADX_ONEHOP, default on -- for up to kHeadxOneHopP virtual ranks: the K ranks skip that second
// meeting -- each computes conv itself and writes its own elements' x-bar; see below.)
//
// HEADX with PhArgs::sched_order set: the grid has one more column of workgroups, whose first
// (blockIdx.x == n_seg, blockIdx.y == 0) computes the next solve's launch order (schedule.h) beside
// the node sums -- nothing else reads or waits for it in this launch, and it takes no ticket.
template <bool NTL, bool HEADX>
__global__ __launch_bounds__(256) void node_sums_kernel(PhArgs a, double* nodesum, double head_thr, int first) {
    if constexpr (HEADX) {
        if ((int)blockIdx.x >= a.n_seg) {
            __shared__ int s_cnt[kSchedBuckets];
            __shared__ int s_wsum[4];
            if (blockIdx.y == 0) schedule_block<256, 4>(a.sched_iters, a.S, a.sched_unit, a.sched_order, s_cnt, s_wsum);
            return;
        }
    }
    // folded update pending: its conv segments ride along (the packed buffer's partials region);
    // the first one's loads go out before the pass over x
    const bool fold_here = a.fold_conv && blockIdx.y == 0 && (int)blockIdx.x < a.n_cseg;
    FoldHead fh;
    if (fold_here) fh = fold_conv_head(a, blockIdx.x);
    node_sum_partials<NTL>(a);
    if (fold_here) {
        fold_conv_segment(a, blockIdx.x, fh, true);
        for (int b = blockIdx.x + a.n_seg; b < a.n_cseg; b += a.n_seg) fold_conv_segment(a, b);
    }
    const int total = a.n_seg * (int)gridDim.y;
    const int K = min(a.n_final, total);
    const int rank = last_k_workgroups(a.ticket, K, total);
    if (rank < 0) return;
    if constexpr (!HEADX) {
        node_sum_final<0>(a, nodesum, rank, K);
        if (a.fold_conv && rank == K - 1) {
            __syncthreads();
            conv_partials_final(a, nodesum + 2 * (long)a.N_tot);
        }
        finish_k(a.ticket, a.ticket + 2, K);
    } else {
        __shared__ double red256[256];
        __shared__ int s_last;
        double* convpart = nodesum + 2 * (long)a.N_tot;
        if (a.onehop && a.P <= kHeadxOneHopP) {
            // one hop: every rank forms the conv partials and conv itself (conv_partials_final and
            // conv_value_block over the same inputs in the same fixed order: the same bits in every
            // rank) and writes the x-bar of its own elements, so the ranks never meet again --
            // rank 0 stores the partials and publishes the gate; the counters are re-armed by the
            // last rank out (finish_k)
            // The node sums go first with the conv segments' partials already in flight (P = 1, one
            // segment per thread: ConvPre), so the two load latencies overlap; x-bar is written
            // from the LDS stash once conv is known.
            __shared__ double s_cp[2 * kHeadxOneHopP + 3];
            __shared__ double s_xb[512];
            const int ncp = 2 * a.P + 3;
            const bool pre = a.fold_conv && a.P == 1 && a.n_cseg <= 256;
            ConvPre cpre;
            if (pre) cpre = conv_pre_load(a);
            node_sum_final<3>(a, nodesum, rank, K, s_xb);
            if (a.fold_conv) {
                conv_partials_final(a, s_cp, pre ? &cpre : nullptr);
            } else {
                for (int i = threadIdx.x; i < ncp; i += 256) s_cp[i] = convpart[i];
            }
            __syncthreads();
            const double conv = first ? INFINITY : conv_value_block(s_cp, a.P, red256);
            if (rank == 0) {
                if (a.fold_conv)
                    for (int i = threadIdx.x; i < ncp; i += 256) convpart[i] = s_cp[i];
                if (threadIdx.x == 0) publish_gate(conv, s_cp, a.P, a.gate, a.gate_host, a.gate_seq);
            }
            if (conv >= head_thr) {
                const int e_lo = (int)((long)a.N_tot * rank / K), e_hi = (int)((long)a.N_tot * (rank + 1) / K);
                const int ne = e_hi - e_lo;
                for (int i = threadIdx.x; i < ne; i += 256) {
                    a.xbar[e_lo + i] = ne <= 256 ? s_xb[i] : nodesum[e_lo + i];
                    a.xsqbar[e_lo + i] = ne <= 256 ? s_xb[256 + i] : nodesum[a.N_tot + e_lo + i];
                }
            }
            finish_k(a.ticket, a.ticket + 2, K);
            return;
        }
        node_sum_final<2>(a, nodesum, rank, K);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned prev = __hip_atomic_fetch_add(a.ticket + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = prev == (unsigned)K - 1;
            if (s_last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        if (!s_last) return;
        if (a.fold_conv) conv_partials_final(a, convpart);
        __syncthreads();
        const double conv = first ? INFINITY : conv_value_block(convpart, a.P, red256);
        if (threadIdx.x == 0) publish_gate(conv, convpart, a.P, a.gate, a.gate_host, a.gate_seq);
        if (conv >= head_thr)
            for (long j = threadIdx.x; j < a.N_tot; j += 256) {
                a.xbar[j] = nodesum[j];
                a.xsqbar[j] = nodesum[a.N_tot + j];
            }
        __syncthreads();
        if (threadIdx.x == 0) {   // every rank is past both counters: re-arm them for the next launch
            __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ticket + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// fixed-order sum of v[first..last) by all 256 threads of the workgroup (same result in every thread)
__device__ __forceinline__ double block_sum_reg(double t, double* red);
__device__ __forceinline__ double block_sum_range(const double* v, int first, int last, double* red) {
    const int tid = threadIdx.x;
    double t = 0.0;
    for (int g = first + tid; g < last; g += 256) t += v[g];
    return block_sum_reg(t, red);
}

// the fixed-order workgroup sum of every thread's t (block_sum_range's tree)
__device__ __forceinline__ double block_sum_reg(double t, double* red) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = t;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

// Update_W + Update_z (smoothed PH only) + convergence_diff (local half) + the solve-status summary.  One workgroup per
// convergence segment (scenario range inside one virtual rank): xbar from the (all-reduced) node
// sums, W += rho (x - xbar), sum |x - xbar|, and the number of scenarios whose last solve did not
// reach the KKT tolerance / failed numerically.  The last workgroup reduces the segment partials
// per virtual rank (fixed order) into convpart[2v], convpart[2v+1] = (sum, count) and
// convpart[2P], convpart[2P+1] = the two status counts; workgroup 0 publishes xbar / xsqbar.
// ROOT_ONLY (two-stage trees, checked on the host: PhArgs::root_only): the x-bar of element e is nodesum[e mod N], tracked per
// thread by increments instead of the per-element index array (4 fewer bytes and one dependent load
// less per element); multistage trees read xidx.
//
// HEAD (phg_ph_head, the pipelined PH iteration): `convpart` holds the PREVIOUS iteration's
// partials, all-reduced together with this iteration's node sums in one exchange buffer.  Every
// workgroup first computes that iteration's convergence metric (the same fixed-order tree, so the
// same bits in every workgroup and as phg_conv_finish); workgroup 0 publishes it (device gate +
// pinned host word); and if it is below `head_thr` the whole grid returns -- PH had converged
// before the solve that followed it, so this update must not happen (phbase.py:1008-1010).  The
// partials of THIS update then overwrite convpart (by the last workgroup, after every workgroup
// has read the old ones).
// W update of convergence segment b (see w_update_kernel): W += rho (x - x-bar), its sum |x - x-bar|
// and the segment's status counts, published for the final reduction.  Ends with a workgroup barrier
// (a workgroup may run several segments).
template <bool ROOT_ONLY>
__device__ __forceinline__ void w_update_segment(const PhArgs& a, int b, const double* nodesum) {
    __shared__ double red[4];
    __shared__ int bad[8];
    const int tid = threadIdx.x;
    const int s0 = a.cseg_s0[b], s1 = a.cseg_s1[b];
    const long e0 = (long)s0 * a.N, e1 = (long)s1 * a.N;
    double acc = 0.0;
    auto upd = [&](long e, double xv, double xb, double w, double r) {
        const double d = xv - xb;
        // variable probability: W of a zero-probability nonant stays 0 (prob0_mask)
        a.W[e] = (a.pcv && a.pcv[e] == 0.0) ? 0.0 : w + r * d;
        if (a.smooth_on) a.Z[e] += a.beta[e] * (xv - a.Z[e]);   // Update_z (smoothed PH)
        return fabs(d);
    };
    long e = e0 + tid;
    // ROOT_ONLY: k = e mod N, advanced by dk = 256 mod N (< N) per 256-element stride
    const int dk = ROOT_ONLY ? 256 % a.N : 0;
    int k = ROOT_ONLY ? (int)(e % a.N) : 0;
    auto adv = [&](int kk) { kk += dk; return kk >= a.N ? kk - a.N : kk; };
    if (ROOT_ONLY && !a.smooth_on && !a.pcv) {
        // two-stage fast path: 16-byte loads / stores of element PAIRS (hipMalloc'd arrays: pair
        // (e, e + 1) is 16-byte aligned for even e), four pairs in flight per thread; an odd first
        // or last element of the segment is done by thread 0
        long b = e0;
        if (b & 1) {
            if (tid == 0) acc += upd(b, a.xN[b], nodesum[(int)(b % a.N)], a.W[b], a.rho_k ? a.rho_k[(int)(b % a.N)] : a.rho[b]);
            ++b;
        }
        const long npair = (e1 - b) >> 1;
        if (((e1 - b) & 1) && tid == 0) {
            const long l = e1 - 1;
            acc += upd(l, a.xN[l], nodesum[(int)(l % a.N)], a.W[l], a.rho_k ? a.rho_k[(int)(l % a.N)] : a.rho[l]);
        }
        const double2* X2 = reinterpret_cast<const double2*>(a.xN + b);
        const double2* R2 = reinterpret_cast<const double2*>(a.rho + b);
        double2* W2 = reinterpret_cast<double2*>(a.W + b);
        const int N = a.N;
        const int dk2 = 512 % N;   // k advance per 256-pair stride
        int kp = (int)((b + 2L * tid) % N);
        auto adv2 = [&](int kk) { kk += dk2; return kk >= N ? kk - N : kk; };
        auto nxt = [&](int kk) { return kk + 1 == N ? 0 : kk + 1; };
        long pp = tid;
        // RK: rho the same in every scenario -- its two values come from the [N] copy (cached), not
        // from a third S*N stream
        auto pairs = [&](auto rkc) {
            constexpr bool RK = decltype(rkc)::value;
            auto rho2 = [&](long q, int k0) {
                if constexpr (RK) return make_double2(a.rho_k[k0], a.rho_k[nxt(k0)]);
                else return R2[q];
            };
            for (; pp + 3 * 256 < npair; pp += 4 * 256) {
                double2 xv[4], wv[4], rv[4];
                double xb0[4], xb1[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    xv[u] = X2[pp + u * 256];
                    wv[u] = W2[pp + u * 256];
                    rv[u] = rho2(pp + u * 256, kp);
                    xb0[u] = nodesum[kp];
                    xb1[u] = nodesum[nxt(kp)];
                    kp = adv2(kp);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double d0 = xv[u].x - xb0[u], d1 = xv[u].y - xb1[u];
                    W2[pp + u * 256] = make_double2(fma(rv[u].x, d0, wv[u].x), fma(rv[u].y, d1, wv[u].y));
                    acc += fabs(d0) + fabs(d1);
                }
            }
            for (; pp < npair; pp += 256) {
                const double2 xv = X2[pp], wv = W2[pp], rv = rho2(pp, kp);
                const double d0 = xv.x - nodesum[kp], d1 = xv.y - nodesum[nxt(kp)];
                W2[pp] = make_double2(fma(rv.x, d0, wv.x), fma(rv.y, d1, wv.y));
                acc += fabs(d0) + fabs(d1);
                kp = adv2(kp);
            }
        };
        if (a.rho_k) pairs(std::true_type{});
        else pairs(std::false_type{});
        e = e1;   // the generic loops below are skipped
    }
    // four elements in flight per thread (all loads before the stores), then the remainder
    for (; e + 3 * 256 < e1; e += 4 * 256) {
        double xv[4], xb[4], w[4], r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long f = e + u * 256;
            xv[u] = a.xN[f];
            if constexpr (ROOT_ONLY) { xb[u] = nodesum[k]; k = adv(k); }
            else xb[u] = nodesum[a.xidx[f]];
            w[u] = a.W[f];
            r[u] = a.rho_k ? a.rho_k[(int)(f % a.N)] : a.rho[f];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += upd(e + u * 256, xv[u], xb[u], w[u], r[u]);
    }
    for (; e < e1; e += 256) {
        double xb;
        if constexpr (ROOT_ONLY) { xb = nodesum[k]; k = adv(k); }
        else xb = nodesum[a.xidx[e]];
        acc += upd(e, a.xN[e], xb, a.W[e], a.rho_k ? a.rho_k[(int)(e % a.N)] : a.rho[e]);
    }
    int nb = 0, nn = 0;
    if (a.status)
        for (int s = s0 + tid; s < s1; s += 256) {
            const int st = a.status[s];
            nb += st != 0;
            nn += st == 2;
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        acc += __shfl_xor(acc, o, 64);
        nb += __shfl_xor(nb, o, 64);
        nn += __shfl_xor(nn, o, 64);
    }
    if ((tid & 63) == 0) { red[tid >> 6] = acc; bad[tid >> 6] = nb; bad[4 + (tid >> 6)] = nn; }
    __syncthreads();
    if (tid == 0) {
        publish(&a.csegpart[b], ((red[0] + red[1]) + red[2]) + red[3]);
        publish(&a.csegbad[2 * b], bad[0] + bad[1] + bad[2] + bad[3]);
        publish(&a.csegbad[2 * b + 1], bad[4] + bad[5] + bad[6] + bad[7]);
    }
    __syncthreads();
}

// the last workgroup's part of convergence_diff: segment partials per virtual rank (fixed order)
// into convpart[2v], convpart[2v+1] = (sum, count); the status counts; the flag
__device__ __forceinline__ void conv_partials_final(const PhArgs& a, double* convpart, const ConvPre* pre) {
    __syncthreads();
    __shared__ double red[4];
    __shared__ int bad[8];
    const int tid = threadIdx.x;
    for (int v = 0; v < a.P; ++v) {
        const int g0 = a.vr_first[v], g1 = a.vr_first[v + 1];
        double t;
        if (pre) {   // (P = 1, one segment per thread, loaded ahead)
            double u = 0.0;
            if (pre->on) u += pre->v;
            t = block_sum_reg(u, red);
        } else {
            t = block_sum_range(a.csegpart, g0, g1, red);
        }
        if (tid == 0) {
            convpart[2 * v] = t;
            convpart[2 * v + 1] = g1 > g0 ? (double)(a.cseg_s1[g1 - 1] - a.cseg_s0[g0]) * (double)a.N : 0.0;
        }
    }
    {
        int tb = 0, tn = 0;
        if (pre) {
            tb = pre->b;
            tn = pre->n;
        } else {
            for (int g = tid; g < a.n_cseg; g += 256) { tb += a.csegbad[2 * g]; tn += a.csegbad[2 * g + 1]; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            tb += __shfl_xor(tb, o, 64);
            tn += __shfl_xor(tn, o, 64);
        }
        __syncthreads();
        if ((tid & 63) == 0) { bad[tid >> 6] = tb; bad[4 + (tid >> 6)] = tn; }
        __syncthreads();
        if (tid == 0) {
            convpart[2 * a.P] = (double)(bad[0] + bad[1] + bad[2] + bad[3]);
            convpart[2 * a.P + 1] = (double)(bad[4] + bad[5] + bad[6] + bad[7]);
            convpart[2 * a.P + 2] = 1.0;   // the partials are a W update's
        }
    }
}

template <bool ROOT_ONLY, bool HEAD>
__global__ __launch_bounds__(256) void w_update_kernel(PhArgs a, const double* nodesum, double* convpart,
                                                       double head_thr, int first) {
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    if (!HEAD && a.skip_gate && a.skip_gate[0] < a.skip_below) return;   // grid-uniform (flush_fold)
    if constexpr (HEAD) {
        __shared__ double red256[256];
        // first PH iteration: no update precedes it, whatever the buffer holds
        const double conv = first ? INFINITY : conv_value_block(convpart, a.P, red256);
        if (b == 0 && tid == 0) publish_gate(conv, convpart, a.P, a.gate, a.gate_host, a.gate_seq);
        if (conv < head_thr) return;   // grid-uniform: no workgroup touches the tickets
    }
    w_update_segment<ROOT_ONLY>(a, b, nodesum);
    if (b == 0)
        for (int j = tid; j < a.N_tot; j += 256) {
            a.xbar[j] = nodesum[j];
            a.xsqbar[j] = nodesum[a.N_tot + j];
        }
    if (!last_workgroup(a.ticket + 1)) return;
    conv_partials_final(a, convpart);
    if (!HEAD && a.gate) {   // single GPU: nothing to all-reduce, finish convergence_diff here
        __syncthreads();
        conv_gate_block(convpart, a.P, a.gate, a.gate_host, a.gate_seq);
    }
}

// Single-GPU PH step (phg_ph_step): the pipelined head (phg_ph_head) and the node sums in ONE launch,
// for batches where no cross-GPU exchange sits between them (one GPU) and the tree is two-stage with
// one virtual rank, no smoothing and no variable probability (PhArgs::fusable).  Grid = the node-sum
// grid.  Every workgroup first computes the previous update's conv from `packed` (the same tree, the
// same bits as phg_ph_head / phg_conv_finish) and the whole grid returns if it is below head_thr;
// workgroup 0 publishes it.  Then the node-sum partials (node_sums_kernel's pass over x); the LAST K
// workgroups to arrive (every other has finished: they spin only on running workgroups) form the node
// sums and x-bar of their element ranges, meet at a counter of the K, and each applies the W update
// to a K-th of the convergence segments (w_update_segment, the same loops and partials as the
// two-launch path: the same bits) -- x is read again from the caches, not from HBM at these sizes;
// the last of the K reduces the segment partials (conv_partials_final) and re-arms the counters.  Replaces node sums + W update (phbase.py:32-112,
// :301-326, the local half of :349-371): one launch, x streamed from HBM once.
__global__ __launch_bounds__(256) void ph_step_kernel(PhArgs a, double* packed, double head_thr, int first) {
    __shared__ double red256[256];
    __shared__ int s_last;
    double* nodesum = packed;
    double* convpart = packed + 2 * (long)a.N_tot;
    const int tid = threadIdx.x;
    const double conv = first ? INFINITY : conv_value_block(convpart, a.P, red256);
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) publish_gate(conv, convpart, a.P, a.gate, a.gate_host, a.gate_seq);
    if (conv < head_thr) return;   // grid-uniform
    node_sum_partials(a);
    // K: enough workgroups for the W update (the node sums' own final reduction needs far fewer,
    // PhArgs::n_final), still far below the resident capacity (the ranked ones spin)
    const int K = min(min(128, a.n_cseg), (int)(gridDim.x * gridDim.y));
    const int rank = last_k_workgroups(a.fticket, K, (int)(gridDim.x * gridDim.y));
    if (rank < 0) return;
    node_sum_final<1>(a, nodesum, rank, K);
    // the K ranks meet: every node sum / x-bar published (sc1 stores, drained) before the W update
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_fetch_add(a.fticket + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(a.fticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)K)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // W update of this rank's convergence segments, exactly as w_update_kernel's workgroups do
    // them (same per-segment loops and partials, so the same bits as the two-launch path)
    const int b0 = (int)((long)a.n_cseg * rank / K), b1 = (int)((long)a.n_cseg * (rank + 1) / K);
    for (int b = b0; b < b1; ++b) w_update_segment<true>(a, b, nodesum);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.fticket + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == (unsigned)K - 1;
        if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!s_last) return;
    conv_partials_final(a, convpart);
    __syncthreads();
    if (tid == 0) {   // every rank is past all three counters: re-arm them for the next launch
        __hip_atomic_store(a.fticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.fticket + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.fticket + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Folded PH iteration, the part before the solve (phg_ph_head with the fold on): conv of the
// previous update from the all-reduced partials (the same tree as everywhere: same bits), published
// by workgroup 0; unless it is below thr, xbar / xsqbar from the all-reduced node sums.  The W update
// itself runs in the next solve's prologue (PdhgArgs::fold_w).  Grid: N_tot / 2048 workgroups.
__global__ __launch_bounds__(256) void xbar_head_kernel(PhArgs a, const double* packed, double thr, int first) {
    __shared__ double red256[256];
    const double conv = first ? INFINITY : conv_value_block(packed + 2 * (long)a.N_tot, a.P, red256);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        publish_gate(conv, packed + 2 * (long)a.N_tot, a.P, a.gate, a.gate_host, a.gate_seq);
    if (conv < thr) return;
    for (long j = (long)blockIdx.x * 256 + threadIdx.x; j < a.N_tot; j += (long)gridDim.x * 256) {
        a.xbar[j] = packed[j];
        a.xsqbar[j] = packed[a.N_tot + j];
    }
}

hipError_t xbar_head_launch(const PhArgs& a, const double* packed, double thr, int first, hipStream_t st) {
    const int g = (int)std::min<long>(64, std::max<long>(1, ((long)a.N_tot + 2047) / 2048));
    hipLaunchKernelGGL(xbar_head_kernel, dim3(g), dim3(256), 0, st, a, packed, thr, first);
    return hipGetLastError();
}

// the conv partials of a folded update on their own (the drain after the last pipelined iteration,
// phg_fold_partials): conv segments, then the last workgroup's per-virtual-rank reduction
__global__ __launch_bounds__(256) void fold_conv_kernel(PhArgs a, double* convpart) {
    fold_conv_segment(a, blockIdx.x);
    if (!last_workgroup(a.ticket + 1)) return;
    conv_partials_final(a, convpart);
}

hipError_t fold_conv_launch(const PhArgs& a, double* convpart, hipStream_t st) {
    hipLaunchKernelGGL(fold_conv_kernel, dim3(a.n_cseg), dim3(256), 0, st, a, convpart);
    return hipGetLastError();
}

hipError_t ph_step_launch(const PhArgs& a, double* packed, double thr, int first, hipStream_t st) {
    hipLaunchKernelGGL(ph_step_kernel, dim3(a.n_seg, (a.maxk + 255) / 256), dim3(256), 0, st, a, packed, thr, first);
    return hipGetLastError();
}

// per-scenario objective value with the current W / xbar / rho (pyo.value(objfct))
__global__ void eval_obj_kernel(int S, int n, int N, const double* x, const double* c,
                                const double* obj_off, const int* nonant_col, const double* xN,
                                const double* W, const double* rho, const double* xbar,
                                const int* xidx, int w_on, int prox_on, double sense,
                                const double* Z, const double* Psm, int smooth_on, double* out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    double f = 0.0;
    for (int j = 0; j < n; ++j) f += c[(long)s * n + j] * x[(long)s * n + j];
    double t = 0.0;
    for (int k = 0; k < N; ++k) {
        const long e = (long)s * N + k;
        const double xv = xN[e];
        if (w_on) t += W[e] * xv;
        if (prox_on) {
            const double xb = xbar[xidx[e]];
            t += 0.5 * rho[e] * (xv * xv - 2.0 * xb * xv + xb * xb);
            if (smooth_on) {
                const double z = Z[e];
                t += 0.5 * Psm[e] * (xv * xv - 2.0 * z * xv + z * z);
            }
        }
    }
    // c is min-form: model objective = sense * (c.x + off) ; PH terms enter with the model sense
    out[s] = sense * (f + obj_off[s]) + sense * t;
}

// out[s*N + k] = row[k] for every s (xhat candidate broadcast, phg_fix_from)
__global__ void broadcast_row_kernel(const double* row, int N, int S, double* out) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < (long)S * N) out[e] = row[e % N];
}

// out[e] = s[e] * d[e]: the unscaled solution from the scaled warm-start state (x = xs * dc,
// y = ys * dr -- the same product the PDHG epilogues would store), materialised on demand
__global__ void unscale_kernel(const double* sv, const double* d, long cnt, double* out) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < cnt) out[e] = sv[e] * d[e];
}

hipError_t unscale_launch(const double* sv, const double* d, long cnt, double* out, hipStream_t st) {
    if (cnt <= 0) return hipSuccess;
    hipLaunchKernelGGL(unscale_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, sv, d, cnt, out);
    return hipGetLastError();
}

hipError_t broadcast_row_launch(const double* row, int N, int S, double* out, hipStream_t st) {
    const long tot = (long)S * N;
    hipLaunchKernelGGL(broadcast_row_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, row, N, S, out);
    return hipGetLastError();
}

__global__ void conv_gate_kernel(const double* __restrict__ convpart, int P, double* gate, double* gate_host,
                                 double seq) {
    conv_gate_block(convpart, P, gate, gate_host, seq);
}

hipError_t conv_gate_launch(const double* convpart, int P, double* gate, double* gate_host, double seq,
                            hipStream_t st) {
    hipLaunchKernelGGL(conv_gate_kernel, dim3(1), dim3(256), 0, st, convpart, P, gate, gate_host, seq);
    return hipGetLastError();
}

// nontemporal loads of x in the node sums (x is read once there) when x is far larger than the
// caches: S N = 1e8 (1e6 x 100), node sums 159.6 vs 177.2 us (4.5 -> 5.2 TB/s); farmer 10k (x just
// written by the solve, cache-resident) keeps plain loads.  PHG_NODESUM_NT=0 / 1 forces either
static bool node_sums_nontemporal(const PhArgs& a) {
    static const int ntenv = [] { const char* e = std::getenv("PHG_NODESUM_NT"); return e ? std::atoi(e) : -1; }();
    return ntenv >= 0 ? ntenv == 1 : (long)a.S * a.N >= 10000000L;
}

hipError_t node_sums_launch(const PhArgs& a, double* nodesum, hipStream_t st) {
    const bool ntl = node_sums_nontemporal(a);
    const dim3 grid(a.n_seg, (a.maxk + 255) / 256);
    if (ntl) hipLaunchKernelGGL((node_sums_kernel<true, false>), grid, dim3(256), 0, st, a, nodesum, 0.0, 0);
    else hipLaunchKernelGGL((node_sums_kernel<false, false>), grid, dim3(256), 0, st, a, nodesum, 0.0, 0);
    return hipGetLastError();
}

// node sums + the x-bar head of the folded pipelined iteration in one launch (node_sums_kernel
// HEADX; one GPU: packed is the handle's own buffer, nothing is exchanged between the two)
hipError_t node_sums_head_launch(const PhArgs& a, double* packed, double thr, int first, hipStream_t st) {
    const bool ntl = node_sums_nontemporal(a);
    const dim3 grid(a.n_seg + (a.sched_order ? 1 : 0), (a.maxk + 255) / 256);
    if (ntl) hipLaunchKernelGGL((node_sums_kernel<true, true>), grid, dim3(256), 0, st, a, packed, thr, first);
    else hipLaunchKernelGGL((node_sums_kernel<false, true>), grid, dim3(256), 0, st, a, packed, thr, first);
    return hipGetLastError();
}

hipError_t w_update_launch(const PhArgs& a, const double* nodesum, double* convpart, hipStream_t st) {
    if (a.root_only)
        hipLaunchKernelGGL((w_update_kernel<true, false>), dim3(a.n_cseg), dim3(256), 0, st, a, nodesum, convpart, 0.0, 0);
    else
        hipLaunchKernelGGL((w_update_kernel<false, false>), dim3(a.n_cseg), dim3(256), 0, st, a, nodesum, convpart, 0.0, 0);
    return hipGetLastError();
}

// packed = [2 N_tot node sums | 2P+2 partials | flag] (phg_api.hip: phg_handle::packed)
hipError_t ph_head_launch(const PhArgs& a, double* packed, double thr, int first, hipStream_t st) {
    double* cp = packed + 2 * (long)a.N_tot;
    if (a.root_only)
        hipLaunchKernelGGL((w_update_kernel<true, true>), dim3(a.n_cseg), dim3(256), 0, st, a, packed, cp, thr, first);
    else
        hipLaunchKernelGGL((w_update_kernel<false, true>), dim3(a.n_cseg), dim3(256), 0, st, a, packed, cp, thr, first);
    return hipGetLastError();
}

hipError_t eval_obj_launch(int S, int n, int N, const double* x, const double* c, const double* obj_off,
                           const int* nonant_col, const double* xN, const double* W, const double* rho,
                           const double* xbar, const int* xidx, int w_on, int prox_on, double sense,
                           const double* Z, const double* Psm, int smooth_on, double* out, hipStream_t st) {
    hipLaunchKernelGGL(eval_obj_kernel, dim3((S + 127) / 128), dim3(128), 0, st, S, n, N, x, c, obj_off,
                       nonant_col, xN, W, rho, xbar, xidx, w_on, prox_on, sense, Z, Psm, smooth_on, out);
    return hipGetLastError();
}

}  // namespace phg
