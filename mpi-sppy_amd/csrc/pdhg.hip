// pdhg.hip -- batched restarted PDHG for PH scenario subproblems on gfx950.
//
// Replaces the per-scenario external-solver call of SPOpt.solve_one (mpisppy/spopt.py:184-231)
// for every local scenario at once.  One 64-lane wavefront = one scenario = one workgroup:
//   * the scenario's scaled matrix lives in VGPRs for the whole solve (CSR slots for A x,
//     CSC slots for A^T y, "dense" rows dealt round-robin over the wave),
//   * the iterates x, y are staged in LDS only for the two gathers per iteration,
//   * every reduction (dense rows, KKT norms, objectives) is a 64-lane DPP/permlane all-reduce
//     (wave_ops.h; deterministic: all lanes end with the same bits),
//   * each wave restarts / terminates on its own, so scenarios never wait for each other.
//
// Problem per scenario (min-form, PH terms of mpisppy/phbase.py:670-760):
//   min (c + w_on W - prox_on rho xbar)^T x + prox_on 1/2 sum rho x_N^2
//   s.t. rl <= A x <= ru, cl <= x <= cu
// Algorithm: PDHG (Chambolle-Pock) on the Ruiz + Pock-Chambolle scaled problem with the
// diagonal Hessian treated exactly in the primal prox, constant step eta/||A||, PDLP-style
// adaptive restarts to the average/current iterate (beta 0.2 / 0.8 / 0.25) with primal-weight
// updates, and a relative KKT termination test on the UNscaled problem.
#include "phg_internal.h"
#include "wave_ops.h"

namespace phg {

template <int K>
__device__ __forceinline__ void wsum_many(double (&v)[K]) { gsum_many<64, K>(v); }

template <int CPL, int KCS, int RPL, int KRS, int D, int KD>
__global__ __launch_bounds__(64) void pdhg_kernel(PdhgArgs a) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (PdhgArgs::gate)
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int s = a.order ? a.order[blockIdx.x] : blockIdx.x;
    const int l = threadIdx.x;
    double* xl = smem;               // [n_pad]  x staged for the row gathers
    double* yl = smem + a.n_pad;     // [m]      y staged for the column gathers
    const Layout& L = a.lay;
    const long sn = (long)s * a.n, sm = (long)s * a.m, snz = (long)s * a.nnz, sN = (long)s * a.N;

    // ------------------------------------------------------------------ columns owned by lane
    int cj[CPL];
    double x[CPL], c[CPL], q[CPL], lo[CPL], hi[CPL], dcs[CPL], aty[CPL], xsum[CPL], atysum[CPL], xr[CPL];
    double cv[CPL][KCS];
    int cr[CPL][KCS];
    double prox_const = 0.0;   // sum rho/2 xbar^2 (min-form objective constant of the prox term)
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int j = L.col_of[l * CPL + k];
        cj[k] = j;
        x[k] = c[k] = q[k] = lo[k] = hi[k] = aty[k] = xsum[k] = atysum[k] = xr[k] = 0.0;
        dcs[k] = 1.0;
#pragma unroll
        for (int t = 0; t < KCS; ++t) { cv[k][t] = 0.0; cr[k][t] = 0; }
        if (j >= 0) {
            const long b = sn + j;
            const double d = a.dc[b];
            double cc = a.c[b], qq = 0.0;
            double lo_ = a.cl[b], hi_ = a.cu[b];
            const int kk = L.col_nonant[j];
            if (kk >= 0) {
                const long t = sN + kk;
                ph_terms(a, t, kk, cc, qq, prox_const);
                if (a.fix_nonants) fixed_box(a, t, d, lo_, hi_);
            }
            dcs[k] = d;
            c[k] = cc * d;
            q[k] = qq * d * d;
            lo[k] = lo_;
            hi[k] = hi_;
            x[k] = clampd((a.warm & 1) ? a.xs_in[b] : 0.0, lo_, hi_);
#pragma unroll
            for (int t = 0; t < KCS; ++t) {
                const int idx = (l * CPL + k) * KCS + t;
                const int p = L.cent_p[idx];
                if (p >= 0) { cv[k][t] = a.vals[snz + p]; cr[k][t] = L.cent_row[idx]; }
            }
        }
    }
    // ------------------------------------------------------------------ rows owned by lane
    int ri[RPL], rd[RPL];
    double y[RPL], ax[RPL], rlo[RPL], rhi[RPL], drs[RPL], ysum[RPL], axsum[RPL], yr[RPL];
    double rv[RPL][KRS];
    int rc[RPL][KRS];
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
        const int i = L.row_of[l * RPL + r];
        ri[r] = i;
        rd[r] = L.row_dense[l * RPL + r];
        y[r] = ax[r] = rlo[r] = rhi[r] = ysum[r] = axsum[r] = yr[r] = 0.0;
        drs[r] = 1.0;
#pragma unroll
        for (int t = 0; t < KRS; ++t) { rv[r][t] = 0.0; rc[r][t] = 0; }
        if (i >= 0) {
            const long b = sm + i;
            row_bounds(a, i, b, rlo[r], rhi[r]);
            drs[r] = a.dr[b];
            y[r] = (a.warm & 1) ? a.ys_in[b] : 0.0;
            if (!fin(rlo[r])) y[r] = fmin(y[r], 0.0);   // a warm dual must fit the row's bounds
            if (!fin(rhi[r])) y[r] = fmax(y[r], 0.0);
#pragma unroll
            for (int t = 0; t < KRS; ++t) {
                const int idx = (l * RPL + r) * KRS + t;
                const int p = L.rent_p[idx];
                if (p >= 0) { rv[r][t] = a.vals[snz + p]; rc[r][t] = L.rent_col[idx]; }
            }
        }
    }
    double dv[D > 0 ? D : 1][KD];
    int dcl[D > 0 ? D : 1][KD];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int t = 0; t < KD; ++t) {
            const int idx = (d * 64 + l) * KD + t;
            const int p = L.dent_p[idx];
            dv[d][t] = p >= 0 ? a.vals[snz + p] : 0.0;
            dcl[d][t] = p >= 0 ? L.dent_col[idx] : 0;
        }

    // y must have the right sign for its row (projection invariant) even when warm-started
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
        if (!fin(rlo[r])) y[r] = fmin(y[r], 0.0);
        if (!fin(rhi[r])) y[r] = fmax(y[r], 0.0);
    }

    auto gather_ax = [&](double (&out)[RPL]) {
        double dsum[D > 0 ? D : 1];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < KD; ++t) acc += dv[d][t] * xl[dcl[d][t]];
            dsum[d] = acc;
        }
        if constexpr (D > 0) wsum_many<D>(dsum);
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < KRS; ++t) acc += rv[r][t] * xl[rc[r][t]];
#pragma unroll
            for (int d = 0; d < D; ++d)
                if (rd[r] == d) acc = dsum[d];
            out[r] = acc;
        }
    };
    auto gather_aty = [&](double (&out)[CPL]) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < KCS; ++t) acc += cv[k][t] * yl[cr[k][t]];
            out[k] = acc;
        }
    };
    auto put_x = [&](const double (&v)[CPL]) {
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (cj[k] >= 0) xl[cj[k]] = v[k];
    };
    auto put_y = [&](const double (&v)[RPL]) {
#pragma unroll
        for (int r = 0; r < RPL; ++r)
            if (ri[r] >= 0) yl[ri[r]] = v[r];
    };

    // ------------------------------------------------------------------ scalars
    // ||c'|| (unscaled, incl. PH terms), ||b|| (unscaled), prox constant
    double red0[2];
    {
        double c2 = 0.0;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (cj[k] >= 0) { const double cu_ = c[k] / dcs[k]; c2 += cu_ * cu_; }
        red0[0] = c2;
        red0[1] = prox_const;
        wsum_many<2>(red0);
    }
    const double cnorm = sqrt(red0[0]);
    prox_const = red0[1];
    const double bnorm = a.bnorm[s];
    const double eta = a.eta[s];
    double omega;
    if ((a.warm & 2) && a.omega_in[s] > 0.0) {
        omega = a.omega_in[s];
    } else {
        // PDLP init: ||c_hat|| / ||b_hat|| in the scaled space
        double rr[2];
        double c2 = 0.0, b2 = 0.0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) c2 += c[k] * c[k];
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            if (ri[r] >= 0) {
                if (fin(rlo[r])) b2 += rlo[r] * rlo[r];
                if (fin(rhi[r])) b2 += rhi[r] * rhi[r];
            }
        }
        rr[0] = c2; rr[1] = b2;
        wsum_many<2>(rr);
        const double cn = sqrt(rr[0]), bn = sqrt(rr[1]);
        omega = (cn > 1e-10 && bn > 1e-10) ? cn / bn : 1.0;
        if ((a.warm & 4) && a.omega_in[s] > 0.0) omega = sqrt(omega * a.omega_in[s]);   // blend
    }
    double tau = eta / omega, sig = eta * omega;

    // initial products
    put_x(x);
    put_y(y);
    __syncthreads();
    gather_ax(ax);
    gather_aty(aty);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CPL; ++k) xr[k] = x[k];
#pragma unroll
    for (int r = 0; r < RPL; ++r) yr[r] = y[r];

    // KKT pieces: [0] ||pr||^2 scaled, [1] ||dres||^2 scaled, [2] ||pr_u||^2, [3] ||dres_u||^2,
    //             [4] pobj, [5] dobj
    auto kkt_local = [&](const double (&xx)[CPL], const double (&at)[CPL], const double (&yy)[RPL],
                         const double (&axx)[RPL], double* o) {
        double p2 = 0, d2 = 0, pu2 = 0, du2 = 0, po = 0, dob = 0;
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            if (ri[r] >= 0) {
                const double pr = axx[r] - clampd(axx[r], rlo[r], rhi[r]);
                p2 += pr * pr;
                const double pu = pr / drs[r];
                pu2 += pu * pu;
                if (fin(rlo[r])) dob += rlo[r] * fmax(yy[r], 0.0);
                if (fin(rhi[r])) dob += rhi[r] * fmin(yy[r], 0.0);
            }
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            if (cj[k] >= 0) {
                const double rc_ = c[k] + q[k] * xx[k] - at[k];
                double dres = 0.0;
                if (!fin(lo[k]) && rc_ > 0.0) dres += rc_;
                if (!fin(hi[k]) && rc_ < 0.0) dres += rc_;
                d2 += dres * dres;
                const double du = dres / dcs[k];
                du2 += du * du;
                po += c[k] * xx[k] + 0.5 * q[k] * xx[k] * xx[k];
                if (fin(lo[k])) dob += lo[k] * fmax(rc_, 0.0);
                if (fin(hi[k])) dob += hi[k] * fmin(rc_, 0.0);
                dob -= 0.5 * q[k] * xx[k] * xx[k];
            }
        }
        o[0] = p2; o[1] = d2; o[2] = pu2; o[3] = du2; o[4] = po; o[5] = dob;
    };
    auto rel_of = [&](const double* o) {
        const double p = sqrt(o[2]) / (1.0 + bnorm);
        const double d = sqrt(o[3]) / (1.0 + cnorm);
        const double g = fabs(o[4] - o[5]) /
                         gap_den(o[4], o[5], a.gap_const ? a.obj_off[s] + (a.prox_on ? prox_const : 0.0) : 0.0);
        return fmax(fmax(p, d), g);
    };
    auto wkkt_of = [&](const double* o, double w) {
        const double g = o[4] - o[5];
        return sqrt(w * w * o[0] + o[1] / (w * w) + g * g);
    };

    double kkt_restart, kkt_prev = INFINITY;
    {
        double o[6];
        kkt_local(x, aty, y, ax, o);
        wsum_many<6>(o);
        kkt_restart = wkkt_of(o, omega);
    }
    int it = 0, since = 0, cnt = 0;
    int st = 1;
    double rel_final = INFINITY;
    bool final_avg = false;
    const int chk = a.check_every;

    while (it < a.max_iter) {
        for (int kk = 0; kk < chk; ++kk) {
            // primal step (exact prox of the diagonal quadratic + box)
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const double xn = clampd((x[k] - tau * (c[k] - aty[k])) / (1.0 + tau * q[k]), lo[k], hi[k]);
                x[k] = xn;
                xsum[k] += xn;
            }
            put_x(x);
            __syncthreads();
            // dual step with extrapolation A(2x+ - x) = 2 A x+ - A x
            double axn[RPL];
            gather_ax(axn);
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
                const double g = y[r] - sig * (2.0 * axn[r] - ax[r]);
                const double yn = fmax(g + sig * rlo[r], 0.0) + fmin(g + sig * rhi[r], 0.0);
                y[r] = (ri[r] >= 0) ? yn : 0.0;
                ax[r] = axn[r];
                ysum[r] += y[r];
                axsum[r] += axn[r];
            }
            put_y(y);
            __syncthreads();
            gather_aty(aty);
#pragma unroll
            for (int k = 0; k < CPL; ++k) atysum[k] += aty[k];
        }
        it += chk;
        since += chk;
        cnt += chk;

        // ---------------------------------------------------------- restart / termination check
        const double inv = 1.0 / (double)cnt;
        double xa[CPL], ata[CPL], ya[RPL], axa[RPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) { xa[k] = xsum[k] * inv; ata[k] = atysum[k] * inv; }
#pragma unroll
        for (int r = 0; r < RPL; ++r) { ya[r] = ysum[r] * inv; axa[r] = axsum[r] * inv; }
        double o[12];
        kkt_local(x, aty, y, ax, o);
        kkt_local(xa, ata, ya, axa, o + 6);
        wsum_many<12>(o);
        const double rel_cur = rel_of(o), rel_avg = rel_of(o + 6);
        if (rel_cur <= a.eps || rel_avg <= a.eps || !(rel_cur == rel_cur)) {
            if (!(rel_cur == rel_cur)) { st = 2; rel_final = rel_cur; break; }
            final_avg = rel_avg < rel_cur;
            rel_final = final_avg ? rel_avg : rel_cur;
            st = 0;
            break;
        }
        const double k_cur = wkkt_of(o, omega), k_avg = wkkt_of(o + 6, omega);
        const bool use_avg = k_avg < k_cur;
        const double cand = use_avg ? k_avg : k_cur;
        const bool restart = (cand <= a.beta_suf * kkt_restart) ||
                             (cand <= a.beta_nec * kkt_restart && cand > kkt_prev) ||
                             ((double)since >= a.beta_art * (double)it);
        kkt_prev = cand;
        if (restart) {
            if (use_avg) {
#pragma unroll
                for (int k = 0; k < CPL; ++k) x[k] = xa[k];
#pragma unroll
                for (int r = 0; r < RPL; ++r) y[r] = ya[r];
            }
            // primal weight update (theta = 0.5) from the movement since the last restart
            double mv[2] = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < CPL; ++k) { const double d = x[k] - xr[k]; mv[0] += d * d; }
#pragma unroll
            for (int r = 0; r < RPL; ++r) { const double d = y[r] - yr[r]; mv[1] += d * d; }
            wsum_many<2>(mv);
            const double dx = sqrt(mv[0]), dy = sqrt(mv[1]);
            omega = primal_weight(omega, dx * dx, dy * dy, a.theta);
            tau = eta / omega;
            sig = eta * omega;
            // exact products at the restart point
            __syncthreads();
            put_x(x);
            put_y(y);
            __syncthreads();
            gather_ax(ax);
            gather_aty(aty);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < CPL; ++k) { xr[k] = x[k]; xsum[k] = 0.0; atysum[k] = 0.0; }
#pragma unroll
            for (int r = 0; r < RPL; ++r) { yr[r] = y[r]; ysum[r] = 0.0; axsum[r] = 0.0; }
            cnt = 0;
            since = 0;
            kkt_restart = cand;
            kkt_prev = INFINITY;
        }
    }

    // ------------------------------------------------------------------ outputs
    if (st == 1) {
        // iteration limit: report the better of current / average
        const double inv = cnt > 0 ? 1.0 / (double)cnt : 0.0;
        if (cnt > 0) {
            double xa[CPL], ata[CPL], ya[RPL], axa[RPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k) { xa[k] = xsum[k] * inv; ata[k] = atysum[k] * inv; }
#pragma unroll
            for (int r = 0; r < RPL; ++r) { ya[r] = ysum[r] * inv; axa[r] = axsum[r] * inv; }
            double o[12];
            kkt_local(x, aty, y, ax, o);
            kkt_local(xa, ata, ya, axa, o + 6);
            wsum_many<12>(o);
            final_avg = rel_of(o + 6) < rel_of(o);
            rel_final = final_avg ? rel_of(o + 6) : rel_of(o);
        }
    }
    if (final_avg && cnt > 0) {
        const double inv = 1.0 / (double)cnt;
#pragma unroll
        for (int k = 0; k < CPL; ++k) { x[k] = xsum[k] * inv; aty[k] = atysum[k] * inv; }
#pragma unroll
        for (int r = 0; r < RPL; ++r) { y[r] = ysum[r] * inv; ax[r] = axsum[r] * inv; }
    }
    double o[6];
    kkt_local(x, aty, y, ax, o);
    wsum_many<6>(o);
    const double offs = a.obj_off[s] + (a.prox_on ? prox_const : 0.0);
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        if (cj[k] >= 0) {
            const long b = sn + cj[k];
            a.xs[b] = x[k];
            const double xu = x[k] * dcs[k];
            if (a.x_out) a.x_out[b] = xu;
            const int kk = L.col_nonant[cj[k]];
            if (kk >= 0) a.xN[sN + kk] = xu;
        }
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
        if (ri[r] >= 0) {
            const long b = sm + ri[r];
            a.ys[b] = y[r];
            if (a.y_out) a.y_out[b] = y[r] * drs[r];
        }
    }
    if (l == 0) {
        a.omega[s] = omega;
        a.obj[s] = a.sense * (o[4] + offs);
        a.bound[s] = a.sense * (o[5] + offs);
        a.kkt[s] = rel_final;
        a.iters[s] = it;
        a.iters_acc[s] += it;
        a.status[s] = st;
    }
}

// ----------------------------------------------------------------------------- dispatch
struct Variant {
    int CPL, KCS, RPL, KRS, D, KD;
    void (*fn)(PdhgArgs);
};

#define PHG_V(a_, b_, c_, d_, e_, f_) {a_, b_, c_, d_, e_, f_, pdhg_kernel<a_, b_, c_, d_, e_, f_>}
static const Variant kVariants[] = {
    PHG_V(1, 4, 1, 4, 1, 1),
    PHG_V(1, 4, 1, 8, 2, 1),
    PHG_V(2, 4, 2, 4, 2, 1),
    PHG_V(2, 4, 2, 8, 2, 1),
    PHG_V(2, 8, 2, 8, 4, 2),
    PHG_V(4, 4, 4, 8, 4, 2),
};
#undef PHG_V

int pdhg_num_variants() { return (int)(sizeof(kVariants) / sizeof(kVariants[0])); }

void pdhg_variant_shape(int v, int* out6) {
    const Variant& V = kVariants[v];
    out6[0] = V.CPL; out6[1] = V.KCS; out6[2] = V.RPL; out6[3] = V.KRS; out6[4] = V.D; out6[5] = V.KD;
}

hipError_t pdhg_launch(int v, const PdhgArgs& a, hipStream_t stream) {
    const size_t lds = (size_t)(a.n_pad + a.m) * sizeof(double);
    hipLaunchKernelGGL(kVariants[v].fn, dim3(a.S), dim3(64), lds, stream, a);
    return hipGetLastError();
}

}  // namespace phg
