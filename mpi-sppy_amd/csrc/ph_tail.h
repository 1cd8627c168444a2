// ph_tail.h -- the PH update fused into the end of the lane-local solve (pdhg_local.hip).
//
// In the pipelined PH iteration (phbase.update_and_solve) the solve of iteration k is followed by
// the node sums of its x (_Compute_Xbar, mpisppy/phbase.py:32-112) and, on one GPU, by the x-bar
// head (the convergence metric of update k from the folded W update's per-scenario partials,
// phbase.py:349-371, the gate of solve k+1 and x-bar of iteration k+1).  Launched as a kernel of its
// own that work costs a dependent-kernel boundary and a launch ramp (~25 us between two solves on
// farmer 10k, ~16 us of it the node-sum kernel).  Here it runs at the END of the solve's own launch:
// each wave, once it has no work left, drains its stores and adds to a counter; the LAST T waves to
// arrive (tail ranks, as node_sums_kernel's last-K workgroups: every other wave has finished, so the
// few still running are all resident) wait for the count to reach the grid, then
//   1. node-sum partials of the node segments and the folded update's conv-segment partials
//      (tail rank t takes segments t, t + T, ...), published write-through;
//   2. the last R of them to arrive wait for all T, then each forms the
//      convergence partials (the same fixed-order sums in every rank), adds its slice of the
//      node sums in segment order into the packed buffer, and -- one GPU -- writes the next x-bar
//      into a staging buffer (the current x-bar where conv < convthresh: the reference's break
//      before Update_W, phbase.py:1008-1010) that phg_ph_step commits; rank 0 publishes the gate.
// Hand-offs as in node_sums_kernel (MI355X_MICROARCH.md, inter-workgroup visibility): every
// handed-off store is an sc1 (write-through) store drained by s_waitcnt vmcnt(0) before the counter
// add; the consumer polls the counter, takes ONE agent-scope acquire, then reads with plain loads
// (batched: a first version read with sc1 atomic loads, which the compiler issued one at a time --
// +54 us per launch on farmer 10k).  All spins are bounded (a give-up sets an error word and the
// wave leaves; the grid always drains).  The sums are deterministic
// (fixed orders); their association differs from node_sums_kernel's, so a pipelined trajectory
// with the tail agrees with the statement-by-statement one to rounding, not bit for bit.
#pragma once
#include "phg_internal.h"
#include "wave_ops.h"

namespace phg {

__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one wave's butterfly sum (every lane the same bits)
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

// lane 0 waits until *cnt >= target (bounded: ~2^22 polls of ~64 cycles each, seconds); false on
// a give-up, which also sets the error word
__device__ __forceinline__ bool tail_wait(unsigned* cnt, unsigned target, unsigned* err) {
    int ok = 1;
    if (threadIdx.x == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++spins > (1u << 22)) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (ok) {   // agent-scope acquire: this CU's L1 holds no stale copy of the handed-off bytes
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    return __shfl(ok, 0, 64) != 0;
}

// the whole tail, run at the end of every wave of the grid (one 64-lane wave per workgroup) after
// its last epilogue; lds: >= 128 doubles of the wave's dynamic LDS (its cold state is dead by now)
__device__ __forceinline__ void ph_tail_end(const TailArgs& tl, double* lds) {
    const int lane = threadIdx.x;
    const PhArgs& p = tl.ph;
    unsigned* cnt = tl.cnt;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores are out
    int t = -1;
    // PHG_TAIL_PROF stamps (100 MHz): [0] the last wave's arrival, [1] rank 0 past the wait,
    // [2] rank 0 done with its partials, [3] final rank 0 past the second wait, [4] its stores done
    auto stamp = [&](int i) {
        if (tl.prof && lane == 0) tl.prof[i] = __builtin_amdgcn_s_memrealtime();
    };
    if (lane == 0) {
        const unsigned prev = __hip_atomic_fetch_add(cnt + 0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = (int)prev - (tl.W - tl.T);
        if (tl.prof && prev == (unsigned)tl.W - 1) tl.prof[0] = __builtin_amdgcn_s_memrealtime();
    }
    t = __shfl(t, 0, 64);
    if (t < 0) return;
    if (!tail_wait(cnt + 0, (unsigned)tl.W, cnt + 3)) return;
    if (t == 0) stamp(1);
    // ---------------------------------------------------------------- 1. partials
    // this rank's conv segment (one per rank when n_cseg <= T and a segment has <= 128 scenarios:
    // its loads issued now, with the node segment's, and reduced after -- one round trip for both)
    const bool cpre = p.n_cseg <= tl.T && (t >= p.n_cseg || p.cseg_s1[t] - p.cseg_s0[t] <= 128);
    double cv[2] = {0.0, 0.0};
    int cst[2] = {0, 0};
    if (cpre && t < p.n_cseg) {
        const int s0 = p.cseg_s0[t], s1 = p.cseg_s1[t];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int s = s0 + lane + 64 * h;
            const int sc = s < s1 ? s : s0;
            cv[h] = p.conv_s[sc];
            cst[h] = p.fold_st[sc];
            if (!(s < s1)) { cv[h] = 0.0; cst[h] = 0; }
        }
    }
    for (int g = t; g < p.n_seg; g += tl.T) {
        const NodeSeg sg = p.seg[g];
        double* out = p.segpart + (long)g * 2 * p.maxk;
        for (int k0 = 0; k0 < sg.klen; k0 += 64) {
            const int kl = min(64, sg.klen - k0);
            const int q = 64 / kl;                 // lanes per element
            const int k = lane % kl, so = lane / kl;
            double s1 = 0.0, s2 = 0.0;
            if (so < q) {
                const long kg = sg.kofs + k0 + k;
                // 32 rows per lane in flight (a farmer segment, 64 scenarios x 2 lanes per element,
                // in ONE round trip), accumulated into 8 sums by row mod 8 (fixed pairing)
                constexpr int RB = 32, R = 8;
                double t1[R], t2[R];
#pragma unroll
                for (int u = 0; u < R; ++u) t1[u] = t2[u] = 0.0;
                int s = sg.s0 + so;
                for (; s < sg.s1; s += RB * q) {
                    double xv[RB], pr[RB];
#pragma unroll
                    for (int u = 0; u < RB; ++u) {   // (rows past the segment: a valid row, weight 0)
                        const int su = s + u * q;
                        const int sc = su < sg.s1 ? su : sg.s0;
                        xv[u] = p.xN[(long)sc * p.N + kg];
                        pr[u] = p.pcv ? p.pcv[(long)sc * p.N + kg] : p.pc[(long)sc * p.L + sg.level];
                        pr[u] = su < sg.s1 ? pr[u] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < RB; ++u) {
                        const double px = pr[u] * xv[u];
                        t1[u % R] += px;
                        t2[u % R] = fma(px, xv[u], t2[u % R]);
                    }
                }
                s1 = ((t1[0] + t1[1]) + (t1[2] + t1[3])) + ((t1[4] + t1[5]) + (t1[6] + t1[7]));
                s2 = ((t2[0] + t2[1]) + (t2[2] + t2[3])) + ((t2[4] + t2[5]) + (t2[6] + t2[7]));
            }
            lds[lane] = s1;
            lds[64 + lane] = s2;
            __syncthreads();   // (a one-wave workgroup: orders the LDS stores before the loads)
            if (lane < kl) {
                double a1 = 0.0, a2 = 0.0;
                for (int j = 0; j < q; ++j) { a1 += lds[j * kl + lane]; a2 += lds[64 + j * kl + lane]; }
                st_sc1(&out[k0 + lane], a1);
                st_sc1(&out[p.maxk + k0 + lane], a2);
            }
            __syncthreads();
        }
    }
    // the folded update's conv segments: sum |x - xbar| and the status counts of its solve
    if (cpre && t < p.n_cseg) {   // (the order of the loop below: lane-strided, then the butterfly)
        const double acc = wave_sum(cv[0] + cv[1]);
        const int nb = wave_sum((int)(cst[0] != 0) + (int)(cst[1] != 0));
        const int nn = wave_sum((int)(cst[0] == 2) + (int)(cst[1] == 2));
        if (lane == 0) {
            st_sc1(&p.csegpart[t], acc);
            st_sc1(&p.csegbad[2 * t], nb);
            st_sc1(&p.csegbad[2 * t + 1], nn);
        }
    }
    for (int b = t; !cpre && b < p.n_cseg; b += tl.T) {
        const int s0 = p.cseg_s0[b], s1 = p.cseg_s1[b];
        double acc = 0.0;
        int nb = 0, nn = 0;
        for (int s = s0 + lane; s < s1; s += 64) {
            acc += p.conv_s[s];
            const int st = p.fold_st[s];
            nb += st != 0;
            nn += st == 2;
        }
        acc = wave_sum(acc);
        nb = wave_sum(nb);
        nn = wave_sum(nn);
        if (lane == 0) {
            st_sc1(&p.csegpart[b], acc);
            st_sc1(&p.csegbad[2 * b], nb);
            st_sc1(&p.csegbad[2 * b + 1], nn);
        }
    }
    // ---------------------------------------------------------------- arrival, ranks
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t == 0) stamp(2);
    int rank = -1;
    if (lane == 0) {
        const unsigned prev = __hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rank = (int)prev - (tl.T - tl.R);
    }
    rank = __shfl(rank, 0, 64);
    if (rank < 0) return;
    if (!tail_wait(cnt + 1, (unsigned)tl.T, cnt + 3)) return;
    if (rank == 0) stamp(3);
    // ---------------------------------------------------------------- 2. final (rank of R)
    double* cp = tl.out + 2 * (long)p.N_tot;
    // this rank's slice of the node sums: TL lanes per element, each adding every TL-th segment of
    // the element's node, then a fixed butterfly
    const int e_lo = (int)((long)p.N_tot * rank / tl.R), e_hi = (int)((long)p.N_tot * (rank + 1) / tl.R);
    const int ne = e_hi - e_lo;
    int TL = 1;
    while (TL < 64 && TL * 2 * ne <= 64) TL *= 2;
    const int E = 64 / TL;
    const int sub = lane % TL;
    auto node_sum = [&](int e, double& a1, double& a2) {
        a1 = a2 = 0.0;
        if (e < e_hi) {
            int lo = 0, hi = p.n_nodes - 1;   // node g with node_off[g] <= e
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (p.node_off[mid] <= e) lo = mid; else hi = mid - 1;
            }
            const int i = e - p.node_off[lo];
#pragma unroll 8
            for (int g = p.node_first_seg[lo] + sub; g < p.node_first_seg[lo + 1]; g += TL) {
                a1 += p.segpart[(long)g * 2 * p.maxk + i];
                a2 += p.segpart[(long)g * 2 * p.maxk + p.maxk + i];
            }
        }
        for (int o = 1; o < TL; o <<= 1) {
            a1 += __shfl_xor(a1, o, 64);
            a2 += __shfl_xor(a2, o, 64);
        }
    };
    // one virtual rank and <= 128 conv segments (the usual case): their partials loaded first, then
    // this rank's node sums (one pass when its slice fits), both in flight together
    const bool fastc = p.P == 1 && p.n_cseg <= 128;
    const bool one_pass = ne <= E;
    double cA[2] = {0.0, 0.0};
    int bA[4] = {0, 0, 0, 0};
    if (fastc) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int g = lane + 64 * h;
            const int gc = g < p.n_cseg ? g : 0;
            cA[h] = p.csegpart[gc];
            bA[2 * h] = p.csegbad[2 * gc];
            bA[2 * h + 1] = p.csegbad[2 * gc + 1];
            if (!(g < p.n_cseg)) { cA[h] = 0.0; bA[2 * h] = bA[2 * h + 1] = 0; }
        }
    }
    double f1 = 0.0, f2 = 0.0;
    if (one_pass) node_sum(e_lo + lane / TL, f1, f2);
    // convergence partials: per virtual rank v (sum |x - xbar|, count) in fixed order; the status
    // counts; the flag -- the same sums in every rank
    double conv = 0.0;
    int tb = 0, tn = 0;
    for (int v = 0; v < p.P; ++v) {
        const int g0 = p.vr_first[v], g1 = p.vr_first[v + 1];
        double sv = 0.0;
        if (fastc) sv = cA[0] + cA[1];
        else
            for (int g = g0 + lane; g < g1; g += 64) sv += p.csegpart[g];
        sv = wave_sum(sv);
        const double c = g1 > g0 ? (double)(p.cseg_s1[g1 - 1] - p.cseg_s0[g0]) * (double)p.N : 0.0;
        if (c > 0.0) conv += sv / c;
        if (rank == 0 && lane == 0) {
            cp[2 * v] = sv;
            cp[2 * v + 1] = c;
        }
    }
    if (fastc) {
        tb = bA[0] + bA[2];
        tn = bA[1] + bA[3];
    } else {
        for (int g = lane; g < p.n_cseg; g += 64) {
            tb += p.csegbad[2 * g];
            tn += p.csegbad[2 * g + 1];
        }
    }
    tb = wave_sum(tb);
    tn = wave_sum(tn);
    conv /= (double)p.P;
    if (rank == 0 && lane == 0) {
        cp[2 * p.P] = (double)tb;
        cp[2 * p.P + 1] = (double)tn;
        cp[2 * p.P + 2] = 1.0;   // the partials are a W update's
    }
    const bool keep = tl.mode == 1 && !(conv >= tl.thr);   // below convthresh: x-bar stays
    auto put = [&](int e, double a1, double a2) {
        if (e < e_hi && sub == 0) {
            tl.out[e] = a1;
            tl.out[p.N_tot + e] = a2;
            if (tl.mode == 1) {
                tl.xbar_next[e] = keep ? tl.xbar_cur[e] : a1;
                tl.xbar_next[p.N_tot + e] = keep ? tl.xbar_cur[p.N_tot + e] : a2;
            }
        }
    };
    if (one_pass) {
        put(e_lo + lane / TL, f1, f2);
    } else {
        for (int e0 = e_lo; e0 < e_hi; e0 += E) {
            node_sum(e0 + lane / TL, f1, f2);
            put(e0 + lane / TL, f1, f2);
        }
    }
    if (tl.prof && rank == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(4);
    }
    // ---------------------------------------------------------------- gate (one GPU), re-arm
    if (tl.mode == 1 && rank == 0 && lane == 0) {
        tl.gate[0] = conv;
        tl.gate[1] = (double)tb;
        tl.gate[2] = (double)tn;
        double* gh = tl.gate_host + 4 * ((long long)tl.seq & 1);   // (the host reads slot seq mod 2)
        __hip_atomic_store(&gh[0], conv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&gh[1], (double)tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&gh[2], (double)tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __hip_atomic_store(&gh[3], tl.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (lane == 0 &&
        __hip_atomic_fetch_add(cnt + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)tl.R - 1) {
        // every rank is past both waits: re-arm for the next (stream-ordered) launch
        __hip_atomic_store(cnt + 0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace phg
