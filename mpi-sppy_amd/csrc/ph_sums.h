// ph_sums.h -- the node-sum arithmetic of _Compute_Xbar (mpisppy/phbase.py:32-112), shared by the
// 256-thread node-sum workgroups of ph_update.hip and the one-wave emulation of them in the solve's
// tail (ph_tail.h), so the two produce the same bits: every multiply-add here is spelled out
// (contraction off, explicit fma), and both callers add the rows of a thread into its accumulators
// in the same order.
#pragma once
#include "phg_internal.h"

namespace phg {

// one row (probability p, nonant x) into a thread's accumulators: s1 += p x, s2 += (p x) x
__device__ __forceinline__ void nsum_add(double& s1, double& s2, double p, double x) {
#pragma clang fp contract(off)
    const double px = p * x;
    s1 = s1 + px;
    s2 = fma(px, x, s2);
}

// the fixed pairing of a thread's eight accumulators
__device__ __forceinline__ double nsum_tree8(const double* t) {
#pragma clang fp contract(off)
    return ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
}

// The row plan of virtual thread `tid` of a 256-thread node-sum workgroup on the 256-nonant chunk
// k0 of a segment (node_sum_partials): in the paired form thread (k2, so) adds nonants k0 + 2 k2,
// + 1 of rows s0 + so + i q; in the scalar form thread (k, so) nonant k0 + k.  Row i goes into
// accumulator i mod 8 while it lies in a full block of eight (the workgroup's main loop), the
// remainder rows into accumulator 0, in increasing i.
struct NsumThread {
    bool active;
    int kk;       // k2 (paired) or k (scalar)
    int so;       // first row offset
    int q;        // row stride
    int kl;       // nonants of the chunk
    int nr;       // rows of this thread
    int nfull;    // full blocks of eight
};

__device__ __forceinline__ NsumThread nsum_thread(bool pairs, int klen, int k0, int len, int tid) {
    NsumThread t;
    t.kl = min(256, klen - k0);
    const int w = pairs ? t.kl / 2 : t.kl;   // threads per row
    t.q = 256 / w;
    t.kk = tid % w;
    t.so = tid / w;
    t.active = t.so < t.q;
    t.nr = (t.active && t.so < len) ? (len - t.so + t.q - 1) / t.q : 0;
    const int d = len - t.so - 7 * t.q;      // full block b exists while so + (8 b + 7) q < len
    t.nfull = (t.active && d > 0) ? (d + 8 * t.q - 1) / (8 * t.q) : 0;
    return t;
}

// the paired form applies when every row's slice starts 16-byte aligned and the probability is per node
__device__ __forceinline__ bool nsum_pairs(const PhArgs& a, const NodeSeg& sg) {
    return (a.N % 2 == 0) && (sg.kofs % 2 == 0) && (sg.klen % 2 == 0) && !a.pcv;
}

// One virtual thread's sums (the 256-thread node-sum workgroup's per-thread loops): r = {s1, s1', s2,
// s2'} in the paired form (nonants 2 kk, 2 kk + 1), {s1, -, s2, -} in the scalar form.  Eight rows
// in flight per step (fixed pairing: deterministic), then the remainder: every load issued first,
// then the rows added in row order into accumulator 0 (small segments are all remainder: one round
// trip instead of one per row).  NTL: nontemporal loads of x (read once, large batches).
template <bool NTL>
__device__ __forceinline__ void nsum_thread_sums(const PhArgs& a, const NodeSeg& sg, int k0, const NsumThread& th,
                                                 bool pairs, double* r) {
    r[0] = r[1] = r[2] = r[3] = 0.0;
    if (!th.active) return;
    constexpr int R = 8;
    const int q = th.q;
    auto pr = [&](int s) { return a.pc[(long)s * a.L + sg.level]; };
    int s = sg.s0 + th.so;
    if (pairs) {
        const long kg = sg.kofs + k0 + 2 * th.kk;
        auto ld = [&](int s_) {
            const double2* p = reinterpret_cast<const double2*>(a.xN + (long)s_ * a.N + kg);
            if constexpr (NTL) {
                typedef double d2v __attribute__((ext_vector_type(2)));
                const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
                return double2(v.x, v.y);
            } else {
                return *p;
            }
        };
        double ta[R], tb[R], ua[R], ub[R];
#pragma unroll
        for (int u = 0; u < R; ++u) ta[u] = tb[u] = ua[u] = ub[u] = 0.0;
        for (; s + (R - 1) * q < sg.s1; s += R * q) {
            double2 xv[R];
            double p[R];
#pragma unroll
            for (int u = 0; u < R; ++u) { xv[u] = ld(s + u * q); p[u] = pr(s + u * q); }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                nsum_add(ta[u], ua[u], p[u], xv[u].x);
                nsum_add(tb[u], ub[u], p[u], xv[u].y);
            }
        }
        {
            double2 xv[R];
            double p[R];
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (s + u * q < sg.s1) { xv[u] = ld(s + u * q); p[u] = pr(s + u * q); }
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (s + u * q < sg.s1) {
                    nsum_add(ta[0], ua[0], p[u], xv[u].x);
                    nsum_add(tb[0], ub[0], p[u], xv[u].y);
                }
        }
        r[0] = nsum_tree8(ta);
        r[1] = nsum_tree8(tb);
        r[2] = nsum_tree8(ua);
        r[3] = nsum_tree8(ub);
    } else {
        const long kg = sg.kofs + k0 + th.kk;
        auto px = [&](int s_, double& p, double& xv) {
            xv = a.xN[(long)s_ * a.N + kg];
            p = a.pcv ? a.pcv[(long)s_ * a.N + kg] : pr(s_);
        };
        double t1[R], t2[R];
#pragma unroll
        for (int u = 0; u < R; ++u) t1[u] = t2[u] = 0.0;
        for (; s + (R - 1) * q < sg.s1; s += R * q) {
            double p[R], xv[R];
#pragma unroll
            for (int u = 0; u < R; ++u) px(s + u * q, p[u], xv[u]);
#pragma unroll
            for (int u = 0; u < R; ++u) nsum_add(t1[u], t2[u], p[u], xv[u]);
        }
        {
            double p[R], xv[R];
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (s + u * q < sg.s1) px(s + u * q, p[u], xv[u]);
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (s + u * q < sg.s1) nsum_add(t1[0], t2[0], p[u], xv[u]);
        }
        r[0] = nsum_tree8(t1);
        r[2] = nsum_tree8(t2);
    }
}

// a thread's sums into the workgroup's staging array sh[2][512] (sh[so][k] = the thread's partial of
// nonant k), whose q rows the chunk's first kl threads then add in row order
__device__ __forceinline__ void nsum_stage(double* sh, const NsumThread& th, bool pairs, const double* r) {
    if (!th.active) return;
    if (pairs) {
        const int b = th.so * th.kl + 2 * th.kk;
        sh[b] = r[0];
        sh[b + 1] = r[1];
        sh[512 + b] = r[2];
        sh[512 + b + 1] = r[3];
    } else {
        const int b = th.so * th.kl + th.kk;
        sh[b] = r[0];
        sh[512 + b] = r[2];
    }
}

}  // namespace phg
