// ph_tail.h -- the PH update fused into the end of the lane-local solve (pdhg_local.hip).
//
// In the pipelined PH iteration (phbase.update_and_solve) the solve of iteration k is followed by
// the node sums of its x (_Compute_Xbar, mpisppy/phbase.py:32-112) and, on one GPU, by the x-bar
// head (the convergence metric of update k from the folded W update's per-scenario partials,
// phbase.py:349-371, the gate of solve k+1 and x-bar of iteration k+1).  Launched as a kernel of its
// own that work costs a dependent-kernel boundary and a launch ramp.  Here it runs at the end of the
// solve's own launch, as a chain of "last arrival does the work" hand-offs -- no wave ever waits for
// another:
//   1. every wave, after its epilogue (its x stores write-through, drained), counts its scenarios
//      into their node segments (one counter per segment and tree level, PhArgs::seg) and their
//      convergence segments (PhArgs::cseg_*);
//   2. the wave that completes a segment computes the segment's partial sums -- exactly what
//      node_sums_kernel's 256-thread workgroup computes for it (the same per-thread sums of
//      ph_sums.h, the four 64-lane quarters of that workgroup run by one wave) -- or the conv
//      segment's sum |x - x-bar| and status counts (fold_conv_segment's), publishes them
//      write-through and counts one finished unit;
//   3. the wave that finishes the last unit runs the final reduction: every node sum in
//      node_sum_final's order (a host-built slot plan, TailArgs::fin, puts each element's T
//      strided partial sums in T aligned lanes), the convergence partials (conv_partials_final's
//      order) and -- one GPU -- the convergence metric (conv_value_block's tree), the gate and the
//      next x-bar into a staging buffer (the current x-bar where conv < convthresh: the reference's
//      break before Update_W, phbase.py:1008-1010), which phg_ph_step commits.
// Every sum is associated as in the separate launches, so the results are the separate launches'
// bit for bit.  Hand-offs as in node_sums_kernel (MI355X_MICROARCH.md, inter-workgroup
// visibility): handed-off stores are sc1 (write-through), drained by s_waitcnt vmcnt(0) before the
// counter add; the consumer takes ONE agent-scope acquire, then plain loads.  Each counter is
// re-zeroed by the wave that completes it (every add of this launch has happened by then), so the
// next stream-ordered launch starts from zero; no wave spins, so no wave can give up.
#pragma once
#include "phg_internal.h"
#include "ph_sums.h"
#include "wave_ops.h"

namespace phg {

__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one wave's butterfly sum, xor 32 ... 1 (the per-wave step of the 256-thread reductions; every
// lane the same bits)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ void tail_acquire() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------- 2. node segment
// node_sum_partials (ph_update.hip) of segment g by one wave: virtual thread tid = lane + 64 p of
// the workgroup in quarter p.  RMAX: rows per virtual thread up to which every load of the four
// quarters is issued at once (farmer: a 64-scenario segment is <= 4 rows per thread); beyond it the
// quarters run one after another through the workgroup's own loops.
template <int RMAX>
__device__ void tail_seg_partial(const PhArgs& a, int g, double* sh, bool generic) {
    const int lane = threadIdx.x;
    const NodeSeg sg = a.seg[g];
    double* out = a.segpart + (long)g * 2 * a.maxk;
    const bool pairs = nsum_pairs(a, sg);
    const int len = sg.s1 - sg.s0;
    for (int k0 = 0; k0 < sg.klen; k0 += 256) {
        NsumThread th[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) th[p] = nsum_thread(pairs, sg.klen, k0, len, lane + 64 * p);
        const int kl = th[0].kl, q = th[0].q;
        if (!generic && len <= RMAX * q && pairs) {
            double2 xv[4][RMAX];
            double pr[4][RMAX];
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int i = 0; i < RMAX; ++i) {
                    const int s = sg.s0 + th[p].so + i * q;
                    const int sc = i < th[p].nr ? s : sg.s0;   // (rows past the thread's: a valid row, unused)
                    xv[p][i] = *reinterpret_cast<const double2*>(a.xN + (long)sc * a.N + sg.kofs + k0 + 2 * th[p].kk);
                    pr[p][i] = a.pc[(long)sc * a.L + sg.level];
                }
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                double ta[8], tb[8], ua[8], ub[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) ta[u] = tb[u] = ua[u] = ub[u] = 0.0;
#pragma unroll
                for (int i = 0; i < RMAX; ++i) {
                    if (i < th[p].nr) {
                        if (i < 8 * th[p].nfull) {   // a full block of eight: accumulator i mod 8
                            nsum_add(ta[i & 7], ua[i & 7], pr[p][i], xv[p][i].x);
                            nsum_add(tb[i & 7], ub[i & 7], pr[p][i], xv[p][i].y);
                        } else {                     // the remainder: accumulator 0
                            nsum_add(ta[0], ua[0], pr[p][i], xv[p][i].x);
                            nsum_add(tb[0], ub[0], pr[p][i], xv[p][i].y);
                        }
                    }
                }
                const double r[4] = {nsum_tree8(ta), nsum_tree8(tb), nsum_tree8(ua), nsum_tree8(ub)};
                nsum_stage(sh, th[p], true, r);
            }
        } else {
            for (int p = 0; p < 4; ++p) {   // (the plan recomputed: no dynamically indexed local array)
                const NsumThread tp = nsum_thread(pairs, sg.klen, k0, len, lane + 64 * p);
                double r[4];
                nsum_thread_sums<false>(a, sg, k0, tp, pairs, r);
                nsum_stage(sh, tp, pairs, r);
            }
        }
        __syncthreads();   // (a one-wave workgroup: orders the LDS stores before the loads)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int tid = lane + 64 * p;
            if (tid < kl) {
                double t1 = 0.0, t2 = 0.0;
                for (int j = 0; j < q; ++j) { t1 += sh[j * kl + tid]; t2 += sh[512 + j * kl + tid]; }
                st_sc1(&out[k0 + tid], t1);
                st_sc1(&out[a.maxk + k0 + tid], t2);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------- 2'. conv segment
// fold_conv_segment (ph_update.hip) of conv segment b by one wave: the sum of the folded update's
// per-scenario |x - x-bar| (lane-strided over the 256 virtual threads, a butterfly per quarter, the
// four quarters in order) and the solve-status counts
__device__ void tail_cseg_partial(const PhArgs& a, int b) {
    const int lane = threadIdx.x;
    const int s0 = a.cseg_s0[b], s1 = a.cseg_s1[b];
    double r[4];
    int nb = 0, nn = 0;
    if (s1 - s0 <= 256) {   // one scenario per virtual thread: every load at once
        double v[4];
        int st[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int s = s0 + lane + 64 * p;
            const int sc = s < s1 ? s : s0;
            v[p] = a.conv_s[sc];
            st[p] = a.fold_st[sc];
            if (!(s < s1)) { v[p] = 0.0; st[p] = 0; }
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            r[p] = wave_sum(0.0 + v[p]);
            nb += st[p] != 0;
            nn += st[p] == 2;
        }
    } else {
        for (int p = 0; p < 4; ++p) {
            double acc = 0.0;
            for (int s = s0 + lane + 64 * p; s < s1; s += 256) {
                acc += a.conv_s[s];
                const int st = a.fold_st[s];
                nb += st != 0;
                nn += st == 2;
            }
            r[p] = wave_sum(acc);
        }
    }
    nb = wave_sum(nb);
    nn = wave_sum(nn);
    if (lane == 0) {
        st_sc1(&a.csegpart[b], ((r[0] + r[1]) + r[2]) + r[3]);
        st_sc1(&a.csegbad[2 * b], nb);
        st_sc1(&a.csegbad[2 * b + 1], nn);
    }
}

// ---------------------------------------------------------------------------- 3. final
// node_sum_final's sums: fin slot v = lane + 64 q holds {element e (< 0: empty), first segment, terms J
// | stride T << 16, position i of e in its node}; the slot adds its J strided segment partials in
// order, then the xor butterfly over its T aligned lanes (o < T) gives node_sum_final's bits in the
// element's first lane.  Every load the final needs is issued in a few batches (the wave's loads
// after the acquire miss the XCD's L2: each dependent round trip is a microsecond or more), and
// every store comes after the last load.
constexpr int kTailJ = 12;    // strided terms of a slot loaded at once (more: a second round)
constexpr int kTailQ = 8;     // slot passes held in registers (512 slots; more: the plan in rounds)
constexpr int kTailP = 128;   // virtual ranks the final keeps in LDS (host-checked)

__device__ __forceinline__ void tail_fin_sum(const PhArgs& p, const int4& f, double& t1, double& t2) {
    const int e = f.x, g0 = f.y, J = f.z & 0xFFFF, T = f.z >> 16, i = f.w;
    t1 = t2 = 0.0;
    if (e < 0) return;
    double v1[kTailJ], v2[kTailJ];
#pragma unroll
    for (int j = 0; j < kTailJ; ++j) {
        const long gj = (long)(j < J ? g0 + j * T : g0) * 2 * p.maxk;
        v1[j] = p.segpart[gj + i];
        v2[j] = p.segpart[gj + p.maxk + i];
    }
#pragma unroll
    for (int j = 0; j < kTailJ; ++j)
        if (j < J) { t1 += v1[j]; t2 += v2[j]; }
    for (int j = kTailJ; j < J; ++j) {
        const long gj = (long)(g0 + j * T) * 2 * p.maxk;
        t1 += p.segpart[gj + i];
        t2 += p.segpart[gj + p.maxk + i];
    }
}

__device__ void tail_final(const TailArgs& tl, double* lds) {
    const int lane = threadIdx.x;
    const PhArgs& p = tl.ph;
    double* cp = tl.out + 2 * (long)p.N_tot;
    const int4* fin = reinterpret_cast<const int4*>(tl.fin);
    const int nq = tl.n_fin / 64;
    // -- round 1: the status counts, the slot plan and the ranks' conv-segment ranges
    int tb = 0, tn = 0;
    for (int g = lane; g < p.n_cseg; g += 64) { tb += p.csegbad[2 * g]; tn += p.csegbad[2 * g + 1]; }
    int4 pl[kTailQ];
#pragma unroll
    for (int q = 0; q < kTailQ; ++q) pl[q] = q < nq ? fin[q * 64 + lane] : make_int4(-1, 0, 0, 0);
    // -- convergence partials (conv_partials_final): per virtual rank v, block_sum_range over its conv
    // segments -- a lane-strided sum per virtual thread, a butterfly per quarter, the quarters in
    // order; sum, count and ratio kept in LDS (lds[256 + v], lds[384 + 2 v], + 1) until the stores
    for (int v = 0; v < p.P; ++v) {
        const int g0 = p.vr_first[v], g1 = p.vr_first[v + 1];
        double r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double t = 0.0;
            for (int g = g0 + lane + 64 * q; g < g1; g += 256) t += p.csegpart[g];
            r[q] = wave_sum(t);
        }
        const double sum = ((r[0] + r[1]) + r[2]) + r[3];
        const double cnt = g1 > g0 ? (double)(p.cseg_s1[g1 - 1] - p.cseg_s0[g0]) * (double)p.N : 0.0;
        if (lane == 0) {
            lds[256 + v] = cnt > 0.0 ? sum / cnt : 0.0;   // (a rank without nonants adds nothing)
            lds[384 + 2 * v] = sum;
            lds[384 + 2 * v + 1] = cnt;
        }
    }
    tb = wave_sum(tb);
    tn = wave_sum(tn);
    double conv = INFINITY;
    if (tl.mode == 1) {
        // conv_value_block: virtual thread t adds the ratios of ranks t, t + 256, ...; then the
        // halving tree red[t] += red[t + w], w = 128 ... 1
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int t = lane + 64 * q;
            lds[t] = t < p.P ? lds[256 + t] : 0.0;
        }
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            for (int t = lane; t < w; t += 64) lds[t] += lds[t + w];
            __syncthreads();
        }
        conv = lds[0] / (double)p.P;
    }
    const bool keep = tl.mode == 1 && !(conv >= tl.thr);   // below convthresh: x-bar stays
    // -- node sums (node_sum_final's order), two slot passes per round of loads
    auto do_pass = [&](const int4& f, int v, double t1, double t2) {
        const int T = f.z >> 16;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double u1 = __shfl_xor(t1, o, 64), u2 = __shfl_xor(t2, o, 64);
            if (o < T) { t1 += u1; t2 += u2; }
        }
        const int e = f.x;
        if (e >= 0 && (v % T) == 0) {
            tl.out[e] = t1;
            tl.out[p.N_tot + e] = t2;
            if (tl.mode == 1) {
                tl.xbar_next[e] = keep ? tl.xbar_cur[e] : t1;
                tl.xbar_next[p.N_tot + e] = keep ? tl.xbar_cur[p.N_tot + e] : t2;
            }
        }
    };
#pragma unroll
    for (int q = 0; q < kTailQ; q += 2) {
        if (q >= nq) break;
        double a1, a2, b1, b2;
        tail_fin_sum(p, pl[q], a1, a2);
        tail_fin_sum(p, pl[q + 1], b1, b2);
        do_pass(pl[q], q * 64 + lane, a1, a2);
        do_pass(pl[q + 1], (q + 1) * 64 + lane, b1, b2);
    }
    for (int q = kTailQ; q < nq; ++q) {   // (plans beyond the registers' passes)
        const int4 f = fin[q * 64 + lane];
        double a1, a2;
        tail_fin_sum(p, f, a1, a2);
        do_pass(f, q * 64 + lane, a1, a2);
    }
    // -- the convergence partials, then the gate (one GPU): device copy for the next gated launch,
    // pinned host ring for the host
    if (lane == 0) {
        for (int v = 0; v < p.P; ++v) {
            cp[2 * v] = lds[384 + 2 * v];
            cp[2 * v + 1] = lds[384 + 2 * v + 1];
        }
        cp[2 * p.P] = (double)tb;
        cp[2 * p.P + 1] = (double)tn;
        cp[2 * p.P + 2] = 1.0;   // the partials are a W update's
        if (tl.mode == 1) {
            tl.gate[0] = conv;
            tl.gate[1] = (double)tb;
            tl.gate[2] = (double)tn;
            publish_host_gate(tl.gate_host, conv, (double)tb, (double)tn, tl.seq);   // (slot seq mod 2)
        }
    }
}

// ---------------------------------------------------------------------------- the tail
// run by every wave of the grid after its last epilogue; its G groups held scenarios scen[q] (-1:
// none).  lds: the wave's dynamic LDS (its cold state is dead by now; >= 1 024 doubles)
template <int G>
__device__ __forceinline__ void ph_tail_end(const TailArgs& tl, const int (&scen)[G], double* lds) {
    const int lane = threadIdx.x;
    const PhArgs& p = tl.ph;
    constexpr int LPS = 64 / G;
    const int grp = lane / LPS;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores are out
    const unsigned long long t_arrive = tl.prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // 1. count this wave's scenarios into their units: lane grp * LPS + l counts group grp's scenario
    //    into its level-l node segment (l < L) or, at l = L, its conv segment
    int unit = -1;    // the unit this lane completed: node segment g, or n_seg + conv segment b
    {
        int s = -1;
#pragma unroll
        for (int q = 0; q < G; ++q) s = grp == q ? scen[q] : s;
        const int l = lane % LPS;
        if (s >= 0 && l <= p.L) {
            const bool cs = l == p.L;
            const int u = cs ? tl.scen_cseg[s] : tl.scen_seg[(long)s * p.L + l];
            unsigned* c = cs ? tl.csegcnt + u : tl.segcnt + u;
            const int size = cs ? p.cseg_s1[u] - p.cseg_s0[u] : p.seg[u].s1 - p.seg[u].s0;
            const unsigned prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev + 1u == (unsigned)size) {
                unit = cs ? p.n_seg + u : u;
                __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-armed
            }
        }
    }
    unsigned long long done = __ballot(unit >= 0);
    if (!done) return;
    // 2. this wave completed units: their producers' stores are visible after one acquire
    tail_acquire();
    int n_units = 0;
    while (done) {
        const int src = __builtin_ctzll(done);
        done &= done - 1ull;
        const int u = __shfl(unit, src, 64);
        if (u < p.n_seg) tail_seg_partial<4>(p, u, lds, tl.generic != 0);
        else tail_cseg_partial(p, u - p.n_seg);
        ++n_units;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the partials are out
    int last = 0;
    if (lane == 0) {
        const unsigned prev = __hip_atomic_fetch_add(tl.done, (unsigned)n_units, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev + (unsigned)n_units == (unsigned)(p.n_seg + p.n_cseg);
        if (last) __hip_atomic_store(tl.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-armed
    }
    if (!__shfl(last, 0, 64)) return;
    // 3. every unit is in: the final reduction
    tail_acquire();
    const unsigned long long t_final = tl.prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
    tail_final(tl, lds);
    if (tl.prof) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            tl.prof[0] = t_arrive;
            tl.prof[1] = t_final;
            tl.prof[2] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

}  // namespace phg
