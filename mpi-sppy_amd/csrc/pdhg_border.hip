// pdhg_border.hip -- batched PDHG for scenario LPs / QPs too large for one workgroup whose
// constraint matrix is bordered block-diagonal (block-angular): column blocks coupled only through
// a few linking rows.  Unit commitment is the type (one block per generating unit,
// demand and reserve rows coupling them); the host finds the blocks (phg_api.hip:
// build_border_layout) and falls back to the range-split kernel (pdhg_stream.hip) when it finds
// none.  Same algorithm, restart rule, termination test and outputs as the other PDHG kernels
// (replaces SPOpt.solve_one, mpisppy/spopt.py:184-231, for every local scenario).  Mapping:
//
//   * a slot of K workgroups (one 1024-thread workgroup per CU) solves one scenario at a time,
//     taking scenarios from a queue heaviest first; workgroup k owns a group of whole blocks -- its
//     columns and every row whose columns it owns ("local rows") -- and keeps their CSR / CSC
//     slices in LDS (values loaded per scenario);
//   * the NL linking rows are replicated: every workgroup holds their y (thread l < NL, registers,
//     and an LDS copy for A^T y); their A x is the one cross-workgroup step of a PDHG iteration --
//     each workgroup publishes the partial sums over its columns (sc1 stores), ONE slot barrier,
//     and every workgroup adds the K partials in workgroup order, so all hold the same bits and
//     take the same decisions (a double-buffered exchange: no second barrier);
//   * everything else (x, local y, A x, A^T y, running sums) is owned by one workgroup: plain
//     loads and stores, ordered by workgroup barriers;
//   * per-scenario sums (KKT norms, objectives, primal-weight movement) every check_every
//     iterations through the same workgroup-partials pattern (linking rows counted by workgroup 0).
//
// Roofline: per PDHG iteration a workgroup moves its slice's vectors (x, y, sums, bounds: L2-
// resident at these sizes), gathers from LDS, and exchanges NL doubles; the slot barrier sets the
// floor (MI355X_MICROARCH.md: a few us per cross-CU barrier), so the time per iteration is
// latency-bound and reported against HBM on the SURVEY 8(d)1 algorithmic bytes.
#include "phg_internal.h"
#include "wave_ops.h"
#include "stream_sync.h"

#ifndef PHG_GGET_SLEEP
#define PHG_GGET_SLEEP 1   // granule poll interval, s_sleep units of 64 cycles (UC 64: 3 and 8 measured 1-3 % slower)
#endif

namespace phg {

template <int NT>
__global__ __launch_bounds__(NT) void pdhg_border_kernel(PdhgArgs a) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (PdhgArgs::gate)
    __shared__ double red[16 * (NT / 64)];
    __shared__ int s_w;
    extern __shared__ __attribute__((aligned(16))) double dyn[];   // (16 B: vector gathers)
    const StreamLayout& L = a.st;
    const BorderLayout& B = a.bd;
    const int K = L.K;
    const int slot = blockIdx.x / K, kw = blockIdx.x % K;
    const int t = threadIdx.x;
    const BorderGroup G = B.grp[kw];
    const int NL = B.nlink;
    const int nc = G.nc, nr = G.nr;
    // ------------------------------------------------------------------ LDS slice (per launch)
    double* lrv = dyn;                               // [nrz_max] local rows' values, CSR order
    double* lkv = lrv + B.nrz_max;                   // [nlz_max] linking rows' values on owned columns
    double* lcv = lkv + B.nlz_max;                   // [ncz_max] owned columns' values, CSC order
    double* yl = lcv + B.ncz_max;                    // [NL] linking rows' y (current)
    double* ylx = yl + NL;                           // [NL] linking rows' y running sums (checks)
    int* lcol = reinterpret_cast<int*>(ylx + NL);    // [C_max] owned columns
    int* lrow = lcol + B.C_max;                      // [R_max] local rows
    int* lrp = lrow + B.R_max;                       // [R_max + 1]
    int* lci = lrp + B.R_max + 1;                    // [nrz_max] column of each local-row entry
    int* lkp = lci + B.nrz_max;                      // [NL + 1]
    int* lkc = lkp + NL + 1;                         // [nlz_max] column of each linking-row entry
    int* lcp = lkc + B.nlz_max;                      // [C_max + 1]
    int* lri = lcp + B.C_max + 1;                    // [ncz_max] row: >= 0 local row, -(l + 1) linking row l
    for (int q = t; q < nc; q += NT) lcol[q] = B.col_list[G.c0 + q];
    for (int q = t; q < nr; q += NT) lrow[q] = B.row_list[G.r0 + q];
    for (int q = t; q <= nr; q += NT) lrp[q] = B.rptr[G.rp0 + q];
    for (int q = t; q < G.nrz; q += NT) lci[q] = B.rcol[G.rz0 + q];
    for (int q = t; q <= NL; q += NT) lkp[q] = B.lptr[G.lp0 + q];
    for (int q = t; q < G.nlz; q += NT) lkc[q] = B.lcol[G.lz0 + q];
    for (int q = t; q <= nc; q += NT) lcp[q] = B.cptr[G.cp0 + q];
    for (int q = t; q < G.ncz; q += NT) lri[q] = B.crow[G.cz0 + q];

    double* part = L.part + (long)slot * K * 16;
    unsigned* bar = L.ctrl + kCtrlBar + 2 * slot;
    unsigned* mbox = L.ctrl + kCtrlBar + 2 * L.slots + slot;
    unsigned nbar = 0, xc = 0;
    bool alive = true;
    auto barrier = [&]() {
        if (K == 1) { __syncthreads(); return; }
        ++nbar;
        if (!scen_barrier(bar, nbar * (unsigned)K, L.err)) alive = false;
    };
    auto scen_sum = [&](auto& v) {
        constexpr int V = sizeof(v) / sizeof(double);
        wg_sum<NT, V>(v, red);
        if (K == 1) return;
        if (t < V) put(&part[kw * 16 + t], v[t]);
        barrier();
#pragma unroll
        for (int u = 0; u < V; ++u) {
            double acc = get(&part[u]);
            for (int q = 1; q < K; ++q) acc += get(&part[q * 16 + u]);
            v[u] = acc;
        }
        barrier();   // the partials are reused by the next scen_sum
    };
    // linking-row partials (thread l < NL) -> the K-workgroup sum, same bits everywhere
    auto exchange = [&](double v) {
        if (K == 1) return v;
        double* buf = B.plink + ((long)slot * 2 + (xc & 1u)) * K * NL;
        ++xc;
        if (t < NL) put(&buf[kw * NL + t], v);
        barrier();
        double acc = 0.0;
        if (t < NL) {
            acc = get(&buf[t]);
            for (int q = 1; q < K; ++q) acc += get(&buf[q * NL + t]);
        }
        return acc;
    };
    bool vals_loaded = false;

    while (true) {
    // ------------------------------------------------------------------ next scenario of the slot
    if (kw == 0 && t == 0) {
        const unsigned w = __hip_atomic_fetch_add(L.ctrl + kCtrlHead, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_w = (int)w;
        if (K > 1) __hip_atomic_store(mbox, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (K > 1) {
        barrier();
        if (kw != 0 && t == 0) s_w = (int)__hip_atomic_load(mbox, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int wi = s_w;
    if (!alive || wi >= a.S) break;
    const int s = a.order ? a.order[wi] : wi;
    const long sn = (long)s * a.n, sm = (long)s * a.m, sN = (long)s * a.N;
    if (L.vstride != 0 || !vals_loaded) {
        const double* rv = L.rvals + (long)s * L.vstride;
        for (int q = t; q < G.nrz; q += NT) lrv[q] = rv[B.rperm[G.rz0 + q]];
        for (int q = t; q < G.nlz; q += NT) lkv[q] = rv[B.lperm[G.lz0 + q]];
        for (int q = t; q < G.ncz; q += NT) lcv[q] = rv[B.cperm[G.cz0 + q]];
        vals_loaded = true;
    }
    double* X = a.xs + sn;            // owned columns only: plain accesses inside the workgroup
    double* Y = a.ys + sm;
    double* XS = L.xsum + sn;
    double* YS = L.ysum + sm;
    double* CS = L.cs + sn;
    double* QS = L.qs + sn;
    double* LO = L.lo + sn;
    double* HI = L.hi + sn;
    double* ATY = L.aty + sn;
    double* XR = L.xr + sn;
    double* AXO = L.axo + sm;
    double* YR = L.yr + sm;
    auto rowb = [&](int i, double& lo, double& hi) { row_bounds(a, i, sm + i, lo, hi); };
    auto ax_loc = [&](const double* xv, int q) {
        double acc = 0.0;
        for (int p = lrp[q]; p < lrp[q + 1]; ++p) acc = fma(lrv[p], xv[lci[p]], acc);
        return acc;
    };
    auto ax_link = [&](const double* xv) {
        double acc = 0.0;
        if (t < NL)
            for (int p = lkp[t]; p < lkp[t + 1]; ++p) acc = fma(lkv[p], xv[lkc[p]], acc);
        return acc;
    };
    auto aty_col = [&](const double* yv, const double* ylv, int q) {
        double acc = 0.0;
        for (int p = lcp[q]; p < lcp[q + 1]; ++p) {
            const int r = lri[p];
            acc = fma(lcv[p], r >= 0 ? yv[r] : ylv[-r - 1], acc);
        }
        return acc;
    };

    // ------------------------------------------------------------------ prologue
    double c2 = 0.0, prox_const = 0.0, cs2 = 0.0, b2 = 0.0;
    for (int q = t; q < nc; q += NT) {
        const int j = lcol[q];
        const long b = sn + j;
        const double d = a.dc[b];
        double cc = a.c[b], qq = 0.0;
        double lo_ = a.cl[b], hi_ = a.cu[b];
        const int kk = a.lay.col_nonant[j];
        if (kk >= 0) {
            ph_terms(a, sN + kk, kk, cc, qq, prox_const);
            if (a.fix_nonants) fixed_box(a, sN + kk, d, lo_, hi_);
        }
        c2 += cc * cc;
        const double csj = cc * d;
        cs2 += csj * csj;
        CS[j] = csj;
        QS[j] = qq * d * d;
        LO[j] = lo_;
        HI[j] = hi_;
        const double x0 = clampd((a.warm & 1) ? a.xs_in[b] : 0.0, lo_, hi_);
        X[j] = x0;
        XR[j] = x0;
        XS[j] = 0.0;
    }
    for (int q = t; q < nr; q += NT) {
        const int i = lrow[q];
        double lo_, hi_;
        rowb(i, lo_, hi_);
        double yy = (a.warm & 1) ? a.ys_in[sm + i] : 0.0;
        if (!fin(lo_)) yy = fmin(yy, 0.0); else b2 += lo_ * lo_;
        if (!fin(hi_)) yy = fmax(yy, 0.0); else b2 += hi_ * hi_;
        Y[i] = yy;
        YR[i] = yy;
        YS[i] = 0.0;
    }
    // linking row t: replicated state in registers of thread t
    double l_lo = 0.0, l_hi = 0.0, l_y = 0.0, l_ys = 0.0, l_yr = 0.0, l_ax = 0.0, l_dr = 1.0;
    int l_i = 0;
    if (t < NL) {
        l_i = B.link_rows[t];
        rowb(l_i, l_lo, l_hi);
        l_dr = a.dr[sm + l_i];
        double yy = (a.warm & 1) ? a.ys_in[sm + l_i] : 0.0;
        if (!fin(l_lo)) yy = fmin(yy, 0.0); else if (kw == 0) b2 += l_lo * l_lo;
        if (!fin(l_hi)) yy = fmax(yy, 0.0); else if (kw == 0) b2 += l_hi * l_hi;
        l_y = l_yr = yy;
        yl[t] = yy;
    }
    double omega, cnorm;
    {
        double rr[4] = {c2, prox_const, cs2, b2};
        scen_sum(rr);   // (its workgroup barriers also order the prologue's stores)
        cnorm = sqrt(rr[0]);
        prox_const = rr[1];
        const double cn = sqrt(rr[2]), bn = sqrt(rr[3]);
        omega = (cn > 1e-10 && bn > 1e-10) ? cn / bn : 1.0;
        if ((a.warm & 2) && a.omega_in[s] > 0.0) omega = a.omega_in[s];
        else if ((a.warm & 4) && a.omega_in[s] > 0.0) omega = sqrt(omega * a.omega_in[s]);
    }
    const double bnorm = a.bnorm[s], eta = a.eta[s];
    double tau = eta / omega, sig = eta * omega;
    auto products = [&]() {   // A x and A^T y at the current point (after a workgroup barrier)
        for (int q = t; q < nr; q += NT) AXO[lrow[q]] = ax_loc(X, q);
        l_ax = exchange(ax_link(X));
        for (int q = t; q < nc; q += NT) ATY[lcol[q]] = aty_col(Y, yl, q);
    };
    products();

    // KKT pieces of the current iterate (inv = 0) or of the average (inv = 1 / cnt), see
    // pdhg_stream.hip: [0] ||pr||^2 scaled, [1] ||dres||^2 scaled, [2] ||pr||^2, [3] ||dres||^2
    // unscaled, [4] pobj, [5] dobj; linking rows counted by workgroup 0
    auto kkt_part = [&](bool avg, double inv, double l_axs, double* o) {
        double v[6] = {0, 0, 0, 0, 0, 0};
        auto row_terms = [&](double axx, double yy, double lo_, double hi_, double dr) {
            const double pr = axx - clampd(axx, lo_, hi_);
            v[0] += pr * pr;
            const double pu = pr / dr;
            v[2] += pu * pu;
            if (fin(lo_)) v[5] += lo_ * fmax(yy, 0.0);
            if (fin(hi_)) v[5] += hi_ * fmin(yy, 0.0);
        };
        for (int q = t; q < nr; q += NT) {
            const int i = lrow[q];
            double lo_, hi_;
            rowb(i, lo_, hi_);
            row_terms(avg ? ax_loc(XS, q) * inv : AXO[i], avg ? YS[i] * inv : Y[i], lo_, hi_, a.dr[sm + i]);
        }
        if (kw == 0 && t < NL) row_terms(avg ? l_axs * inv : l_ax, avg ? l_ys * inv : l_y, l_lo, l_hi, l_dr);
        for (int q = t; q < nc; q += NT) {
            const int j = lcol[q];
            const double xx = avg ? XS[j] * inv : X[j];
            const double at = avg ? aty_col(YS, ylx, q) * inv : ATY[j];
            const double ck = CS[j], qk = QS[j], lo_ = LO[j], hi_ = HI[j];
            const double rc_ = ck + qk * xx - at;
            double dres = 0.0;
            if (!fin(lo_) && rc_ > 0.0) dres += rc_;
            if (!fin(hi_) && rc_ < 0.0) dres += rc_;
            v[1] += dres * dres;
            const double du = dres / a.dc[sn + j];
            v[3] += du * du;
            const double hq = 0.5 * qk * xx * xx;
            v[4] += ck * xx + hq;
            if (fin(lo_)) v[5] += lo_ * fmax(rc_, 0.0);
            if (fin(hi_)) v[5] += hi_ * fmin(rc_, 0.0);
            v[5] -= hq;
        }
#pragma unroll
        for (int u = 0; u < 6; ++u) o[u] = v[u];
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
        kkt_part(false, 0.0, 0.0, o);
        scen_sum(o);
        kkt_restart = wkkt_of(o, omega);
    }
    int it = 0, since = 0, cnt = 0, st = 1;
    double rel_final = INFINITY, pobj = 0.0, dobj = 0.0;
    bool use_avg_final = false;
    const int chk = a.check_every;

    while (alive) {
        for (int kk = 0; kk < chk && alive; ++kk) {
            for (int q = t; q < nc; q += NT) {
                const int j = lcol[q];
                const double ip = 1.0 / (1.0 + tau * QS[j]);
                const double xn = clampd(fma(tau, ATY[j] - CS[j], X[j]) * ip, LO[j], HI[j]);
                X[j] = xn;
                XS[j] += xn;
            }
            __syncthreads();
            // dual step: A (2 x+ - x) = 2 A x+ - A x
            for (int q = t; q < nr; q += NT) {
                const int i = lrow[q];
                double lo_, hi_;
                rowb(i, lo_, hi_);
                const double axn = ax_loc(X, q);
                const double g = Y[i] - sig * (2.0 * axn - AXO[i]);
                const double yn = fmax(fma(sig, lo_, g), 0.0) + fmin(fma(sig, hi_, g), 0.0);
                AXO[i] = axn;
                Y[i] = yn;
                YS[i] += yn;
            }
            const double axn_l = exchange(ax_link(X));   // the iteration's one slot barrier
            if (t < NL) {
                const double g = l_y - sig * (2.0 * axn_l - l_ax);
                l_y = fmax(fma(sig, l_lo, g), 0.0) + fmin(fma(sig, l_hi, g), 0.0);
                l_ax = axn_l;
                l_ys += l_y;
                yl[t] = l_y;
            }
            __syncthreads();
            for (int q = t; q < nc; q += NT) ATY[lcol[q]] = aty_col(Y, yl, q);
        }
        if (!alive) break;
        it += chk;
        since += chk;
        cnt += chk;

        const double inv = 1.0 / (double)cnt;
        const double l_axs = exchange(ax_link(XS));   // A x of the linking rows at the average
        // the average's linking-row y sums beside the current y (kkt_part reads ylx for the
        // average's A^T y; yl keeps the current y that the next iteration's A^T y reads)
        if (t < NL) ylx[t] = l_ys;
        __syncthreads();
        double oc[6], oa[6];
        kkt_part(false, 0.0, 0.0, oc);
        kkt_part(true, inv, l_axs, oa);
        {
            double both[12];
#pragma unroll
            for (int u = 0; u < 6; ++u) { both[u] = oc[u]; both[6 + u] = oa[u]; }
            scen_sum(both);
#pragma unroll
            for (int u = 0; u < 6; ++u) { oc[u] = both[u]; oa[u] = both[6 + u]; }
        }
        const double rel_cur = rel_of(oc), rel_avg = rel_of(oa);
        const bool nan = !(rel_cur == rel_cur);
        if (nan || rel_cur <= a.eps || rel_avg <= a.eps || it >= a.max_iter) {
            use_avg_final = !nan && rel_avg < rel_cur;
            rel_final = use_avg_final ? rel_avg : rel_cur;
            pobj = use_avg_final ? oa[4] : oc[4];
            dobj = use_avg_final ? oa[5] : oc[5];
            st = nan ? 2 : ((rel_cur <= a.eps || rel_avg <= a.eps) ? 0 : 1);
            break;
        }
        const double k_cur = wkkt_of(oc, omega), k_avg = wkkt_of(oa, omega);
        const bool use_avg = k_avg < k_cur;
        const double cand = use_avg ? k_avg : k_cur;
        const bool restart = (cand <= a.beta_suf * kkt_restart) ||
                             (cand <= a.beta_nec * kkt_restart && cand > kkt_prev) ||
                             ((double)since >= a.beta_art * (double)it);
        kkt_prev = cand;
        if (restart) {
            double mv[2] = {0.0, 0.0};
            for (int q = t; q < nc; q += NT) {
                const int j = lcol[q];
                const double xv = use_avg ? XS[j] * inv : X[j];
                const double d = xv - XR[j];
                mv[0] += d * d;
                XR[j] = xv;
                X[j] = xv;
                XS[j] = 0.0;
            }
            for (int q = t; q < nr; q += NT) {
                const int i = lrow[q];
                const double yv = use_avg ? YS[i] * inv : Y[i];
                const double d = yv - YR[i];
                mv[1] += d * d;
                YR[i] = yv;
                Y[i] = yv;
                YS[i] = 0.0;
            }
            if (t < NL) {
                const double yv = use_avg ? l_ys * inv : l_y;
                const double d = yv - l_yr;
                if (kw == 0) mv[1] += d * d;
                l_yr = l_y = yv;
                l_ys = 0.0;
                yl[t] = yv;
            }
            scen_sum(mv);
            omega = primal_weight(omega, mv[0], mv[1], a.theta);
            tau = eta / omega;
            sig = eta * omega;
            cnt = 0;
            since = 0;
            kkt_restart = cand;
            kkt_prev = INFINITY;
            if (use_avg) products();   // exact products at the new point
        }
    }
    // a scenario given up (a co-resident workgroup missing: the bounded wait expired) reports status 2;
    // its x is NOT a consistent iterate -- columns without a linking-row entry may already have taken
    // the next iteration's primal step -- and callers treat status 2 as a failed solve
    if (!alive) { st = 2; rel_final = NAN; }

    // ------------------------------------------------------------------ outputs
    const double inv = cnt > 0 ? 1.0 / (double)cnt : 0.0;
    for (int q = t; q < nc; q += NT) {
        const int j = lcol[q];
        const long b = sn + j;
        const double xv = use_avg_final ? XS[j] * inv : X[j];
        X[j] = xv;
        const double xu = xv * a.dc[b];
        if (a.x_out) a.x_out[b] = xu;
        const int kk = a.lay.col_nonant[j];
        if (kk >= 0) a.xN[sN + kk] = xu;
    }
    for (int q = t; q < nr; q += NT) {
        const int i = lrow[q];
        const long b = sm + i;
        const double yv = use_avg_final ? YS[i] * inv : Y[i];
        Y[i] = yv;
        if (a.y_out) a.y_out[b] = yv * a.dr[b];
    }
    if (kw == 0 && t < NL) {
        const long b = sm + l_i;
        const double yv = use_avg_final ? l_ys * inv : l_y;
        Y[l_i] = yv;
        if (a.y_out) a.y_out[b] = yv * a.dr[b];
    }
    if (kw == 0 && t == 0) {
        const double offs = a.obj_off[s] + (a.prox_on ? prox_const : 0.0);
        a.omega[s] = omega;
        a.obj[s] = a.sense * (pobj + offs);
        a.bound[s] = a.sense * (dobj + offs);
        a.kkt[s] = rel_final;
        a.iters[s] = it;
        a.iters_acc[s] += it;
        a.status[s] = st;
    }
    if (!alive) break;
    __syncthreads();   // the LDS values / linking copies are rewritten by the next scenario
    }   // scenario queue
}

// ----------------------------------------------------------------------------- register-resident
// The same solve with every owned element's state in registers (512-thread workgroups, see the
// dispatch; E = 2: 254 VGPRs, no spills -- E = 4 spills ~100): thread t owns columns t + e NT and
// local rows t + e NT (e < E); x and y of the group live in LDS (Xl, Yl, indexed by local position)
// for the gathers, so a PDHG iteration touches memory only for the linking-row exchange -- the
// memory-resident kernel above moves each iteration's vectors through L2 / HBM (PMC: ~1.7 TB per
// UC launch at S = 64).  Needs C_max, R_max <= E NT (the host picks E, or this variant is not used).
template <int NT, int E, bool PROF>
__global__ __launch_bounds__(NT) void pdhg_border_reg_kernel(PdhgArgs a) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (PdhgArgs::gate)
    // PROF (PHG_BORDER_PROF=1, diagnostic): wall-clock split of a PDHG iteration as wave 0 of each
    // workgroup sees it (s_memrealtime, 100 MHz), [10] per workgroup: primal, publish + local dual,
    // hop-1 wait, row sums + mid, hop-2 wait, linking dual + settle + A^T y, checks, the rest
    // (queue, prologue, outputs), PDHG iterations, scenarios
    unsigned long long pf[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pf_last = 0, pf_it = 0, pf_sc = 0;
    if constexpr (PROF) pf_last = __builtin_amdgcn_s_memrealtime();
    auto PF = [&](int i) {
        if constexpr (PROF) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            pf[i] += now - pf_last;
            pf_last = now;
        }
    };
    __shared__ double red[16 * (NT / 64)];
    __shared__ int s_w;
    extern __shared__ double dyn[];
    const StreamLayout& L = a.st;
    const BorderLayout& B = a.bd;
    const int K = L.K;
    const int slot = blockIdx.x / K, kw = blockIdx.x % K;
    const int t = threadIdx.x;
    const BorderGroup G = B.grp[kw];
    const int NL = B.nlink;
    const int nc = G.nc, nr = G.nr;
    double* lrv = dyn;                               // [nrz_max]
    double* lkv = lrv + B.nrz_max;                   // [nlz_max]
    double* lcv = lkv + B.nlz_max;                   // [ncz_max]
    double* Xl = lcv + B.ncz_max;                    // [C_max] x of the owned columns (local position)
    double* Yl = Xl + B.C_max;                       // [R_max] y of the local rows
    double* yl = Yl + B.R_max;                       // [NL] linking rows' y, right after the local rows'
    double* xtmp = yl + NL;                          // [xtmp_len] staged cross-workgroup partials
    // every row / column segment padded to a multiple of 4 entries (value 0, index 0: the host's
    // build_border_layout), the index arrays 16-byte aligned: a gather reads 4 indices and 4 values
    // per step with vector LDS loads and issues the 4 x / y loads together
    int* lci = reinterpret_cast<int*>(xtmp + B.xtmp_len);   // [nrz_max] local column position
    int* lkc = lci + B.nrz_max;                      // [nlz_max] local column position
    int* lri = lkc + B.nlz_max;                      // [ncz_max] local row position, or -(l + 1)
    int* lrp = lri + B.ncz_max;                      // [R_max + 1]
    int* lkp = lrp + B.R_max + 1;                    // [NL + 1]
    int* lcp = lkp + NL + 1;                         // [C_max + 1]
    for (int q = t; q <= nr; q += NT) lrp[q] = B.rptr[G.rp0 + q];
    for (int q = t; q < G.nrz; q += NT) lci[q] = B.rcl[G.rz0 + q];
    for (int q = t; q <= NL; q += NT) lkp[q] = B.lptr[G.lp0 + q];
    for (int q = t; q < G.nlz; q += NT) lkc[q] = B.lcl[G.lz0 + q];
    for (int q = t; q <= nc; q += NT) lcp[q] = B.cptr[G.cp0 + q];
    // column entries' rows as positions in Yl: local row r, or R_max + l for linking row l
    for (int q = t; q < G.ncz; q += NT) {
        const int r = B.crl[G.cz0 + q];
        lri[q] = r >= 0 ? r : B.R_max - r - 1;
    }
    // padding entries point at position 0 (value 0): zero every x / y slot once, so a slot this group
    // never owns (Yl[0] of a group without local rows) is a finite 0 and fma(0, v, acc) = acc holds
    // (each thread zeroes the positions t + e NT it owns later, so no barrier is needed before those)
    for (int q = t; q < B.C_max + B.R_max; q += NT) Xl[q] = 0.0;
    // owned elements of this thread (fixed for the launch)
    int jc[E], ir[E];
    bool cv_[E], rv_[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int q = t + e * NT;
        cv_[e] = q < nc;
        rv_[e] = q < nr;
        jc[e] = cv_[e] ? B.col_list[G.c0 + q] : 0;
        ir[e] = rv_[e] ? B.row_list[G.r0 + q] : 0;
    }

    unsigned* bar = L.ctrl + kCtrlBar + 2 * slot;
    unsigned* mbox = L.ctrl + kCtrlBar + 2 * L.slots + slot;
    unsigned nbar = 0;
    bool alive = true;
    auto barrier = [&]() {   // counter barrier: only for the per-scenario mailbox
        if (K == 1) { __syncthreads(); return; }
        ++nbar;
        if (!scen_barrier(bar, nbar * (unsigned)K, L.err)) alive = false;
    };
    // Cross-workgroup sums as data-tagged granules (cdna_hip_programming.md Guideline 16, R2): a
    // double is two 8-byte {tag = epoch, 32-bit half} words, each one sc1 store; a reader re-reads
    // the pair until both tags are the epoch -- no counter, no drain, no barrier.  Every reading
    // thread loads ONE pair, so a hop costs one round trip (the counter barrier and K dependent
    // partial loads cost ~10 us of a ~14 us iteration, measured in-kernel).  Epochs count the hops
    // of each kind (zeroed buffers every launch); buffers are double-buffered by epoch parity: a
    // workgroup rewrites a parity only after a later hop that every workgroup joins after reading
    // this one.  A bounded spin that gives up sets s_dead; callers read it after a barrier.
    __shared__ int s_dead;
    if (t == 0) s_dead = 0;
    unsigned long long* G1 = reinterpret_cast<unsigned long long*>(B.plink);            // [slots][2][NL][K][2]
    unsigned long long* G2 = G1 + (long)L.slots * 2 * NL * K * 2;                         // [slots][2][NL][2]
    unsigned long long* GS = G2 + (long)L.slots * 2 * NL * 2;                             // [slots][2][K][16][2]
    unsigned ex_ep = 0, ss_ep = 0;
    auto gput = [&](unsigned long long* g, unsigned ep, double v) {
        const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
        const unsigned long long tag = (unsigned long long)ep << 32;
        __hip_atomic_store(g, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto gget = [&](const unsigned long long* g, unsigned ep) {
        unsigned long long lo = 0, hi = 0;
        for (unsigned spins = 0;; ++spins) {
            lo = __hip_atomic_load(const_cast<unsigned long long*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hi = __hip_atomic_load(const_cast<unsigned long long*>(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(lo >> 32) == ep && (unsigned)(hi >> 32) == ep) break;
            if (spins > (1u << 24)) {
                s_dead = 1;
                __hip_atomic_store(L.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(PHG_GGET_SLEEP);
        }
        return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
    };
    // scenario sum of V <= 16 values: workgroup sums -> one granule hop -> every workgroup adds the
    // K partials in workgroup order from LDS (same bits everywhere)
    auto scen_sum = [&](auto& v) {
        constexpr int V = sizeof(v) / sizeof(double);
        wg_sum<NT, V>(v, red);
        if (K == 1) return;
        const unsigned ep = ++ss_ep;
        unsigned long long* g = GS + ((long)slot * 2 + (ep & 1u)) * K * 16 * 2;
        if (t < V) gput(g + ((long)kw * 16 + t) * 2, ep, v[t]);
        for (int u = t; u < V * K; u += NT) xtmp[u] = gget(g + ((long)(u / V) * 16 + u % V) * 2, ep);
        __syncthreads();
        // value u's K partials in workgroup order by thread u (in place), then read by every thread
        if (t < V) xtmp[t] = ordered_sum(xtmp + t, V, K);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < V; ++u) v[u] = xtmp[u];
        __syncthreads();
        if (s_dead) alive = false;
    };
    // linking-row sums (thread l < NL holds workgroup kw's partial of row l): reduce-scatter then
    // allgather, two granule hops -- workgroup l mod K owns row l, reads the K partials (one pair
    // per thread), adds them in workgroup order and publishes the sum; every workgroup reads the NL
    // sums.  Returns row t's sum (threads t < NL); the caller follows with settle().
    auto exchange = [&](double v) {
        if (K == 1) return v;
        const unsigned ep = ++ex_ep;
        unsigned long long* g1 = G1 + ((long)slot * 2 + (ep & 1u)) * NL * K * 2;
        unsigned long long* g2 = G2 + ((long)slot * 2 + (ep & 1u)) * NL * 2;
        if (t < NL) gput(g1 + ((long)t * K + kw) * 2, ep, v);
        const int nown = (NL - kw + K - 1) / K;   // rows kw, kw + K, ...
        for (int u = t; u < nown * K; u += NT) xtmp[u] = gget(g1 + ((long)(kw + K * (u / K)) * K + u % K) * 2, ep);
        __syncthreads();
        if (t < nown) gput(g2 + (long)(kw + K * t) * 2, ep, ordered_sum(xtmp + t * K, 1, K));
        return t < NL ? gget(g2 + (long)t * 2, ep) : 0.0;
    };
    // the same exchange split around independent work (the PDHG iteration): ex_publish stores this
    // workgroup's linking-row partials (hop 1 starts), ex_complete reads them back, publishes the row
    // sums (hop 2 starts), runs mid() -- work that needs this call's workgroup barrier but not the
    // linking rows' sums -- and returns the sum of row t.  The same arithmetic in the same order as
    // exchange(): the same bits.
    auto ex_publish = [&](double v) -> unsigned {
        if (K == 1) return 0u;
        const unsigned ep = ++ex_ep;
        unsigned long long* g1 = G1 + ((long)slot * 2 + (ep & 1u)) * NL * K * 2;
        if (t < NL) gput(g1 + ((long)t * K + kw) * 2, ep, v);
        return ep;
    };
    auto ex_complete = [&](unsigned ep, double v, auto mid) {
        if (K == 1) {
            __syncthreads();
            mid();
            return v;
        }
        unsigned long long* g1 = G1 + ((long)slot * 2 + (ep & 1u)) * NL * K * 2;
        unsigned long long* g2 = G2 + ((long)slot * 2 + (ep & 1u)) * NL * 2;
        const int nown = (NL - kw + K - 1) / K;
        for (int u = t; u < nown * K; u += NT) xtmp[u] = gget(g1 + ((long)(kw + K * (u / K)) * K + u % K) * 2, ep);
        __syncthreads();
        PF(2);
        if (t < nown) gput(g2 + (long)(kw + K * t) * 2, ep, ordered_sum(xtmp + t * K, 1, K));
        mid();
        PF(3);
        const double r = t < NL ? gget(g2 + (long)t * 2, ep) : 0.0;
        PF(4);
        return r;
    };
    auto settle = [&]() {   // after an exchange: one workgroup barrier, then the give-up flag
        __syncthreads();
        if (s_dead) alive = false;
    };
    // sum over a padded segment [p0, p1) of val[p] * vec[idx[p]], 4 entries per step, in entry order
    // (a padding entry adds fma(0, v, acc) = acc: the same bits as the unpadded loop)
    auto gather4 = [&](const double* val, const int* idx, const double* vec, int p0, int p1) {
        double acc = 0.0;
        for (int p = p0; p < p1; p += 4) {
            const int4 ix = *reinterpret_cast<const int4*>(idx + p);
            const double2 v0 = *reinterpret_cast<const double2*>(val + p);
            const double2 v1 = *reinterpret_cast<const double2*>(val + p + 2);
            const double x0 = vec[ix.x], x1 = vec[ix.y], x2 = vec[ix.z], x3 = vec[ix.w];
            acc = fma(v0.x, x0, acc);
            acc = fma(v0.y, x1, acc);
            acc = fma(v1.x, x2, acc);
            acc = fma(v1.y, x3, acc);
        }
        return acc;
    };
    auto ax_loc = [&](int q) { return gather4(lrv, lci, Xl, lrp[q], lrp[q + 1]); };   // A x of local row q from Xl
    auto ax_link = [&]() { return t < NL ? gather4(lkv, lkc, Xl, lkp[t], lkp[t + 1]) : 0.0; };
    auto aty_col = [&](int q) { return gather4(lcv, lri, Yl, lcp[q], lcp[q + 1]); };   // A^T y of column q (Yl, yl)
    bool vals_loaded = false;
    // owned columns with no linking-row entry (their A^T y needs only the local y)
    __syncthreads();   // lcp / lri in LDS
    bool loc_[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        loc_[e] = true;
        if (cv_[e])
            for (int p = lcp[t + e * NT]; p < lcp[t + e * NT + 1]; ++p) loc_[e] = loc_[e] && lri[p] < B.R_max;
    }

    // Split solves (BorderLayout::slice > 0; the launch has more scenarios than slots): a fresh
    // scenario still running after slice x check_every PDHG iterations while the queue's first pass
    // is not exhausted is suspended at that check -- its iterate, running sums, restart point and
    // restart / step state saved -- and re-queued behind the first pass, so a slot that drew a heavy
    // scenario late does not hold the launch: every scenario starts within the first pass, and the
    // heavy ones then run to the end one per slot.  Resuming restores the state and recomputes A x /
    // A^T y with the same gathers and sums: the same iterates, bits and iteration counts as an
    // uninterrupted solve.  Queue codes: s (fresh), S + s (resumed), 2 S (no work left).
    // (only workgroup 0's lane 0 waits here; the slot's other workgroups wait in the mailbox barrier,
    // whose bound (~2^23 polls) is far above any first-pass wait: a scenario suspends or finishes
    // within one solve of at most max_iter iterations)
    // (L.err is cleared with the queue words at every launch: pdhg_border_launch.)  A suspended
    // scenario carries status 2 until a slot resumes and finishes it, so one this slot gives up on
    // reports a failed solve.
    auto requeued = [&](int j) -> int {   // the j-th suspended scenario, or 2 S once every scenario is done
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        auto queued = [&]() -> int {
            return j < a.S ? __hip_atomic_load(B.requeue + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        };
        while (true) {
            int v = queued();
            if (v != 0) return a.S + v - 1;
            const bool over =
                __hip_atomic_load(L.ctrl + kCtrlDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)a.S ||
                __hip_atomic_load(L.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            const bool late = __builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull;   // 30 s (100 MHz)
            if (over || late) {
                v = queued();   // published between the two reads: resume it
                if (v != 0) return a.S + v - 1;
                if (late) __hip_atomic_store(L.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return 2 * a.S;
            }
            __builtin_amdgcn_s_sleep(8);
        }
    };

    while (true) {
    if (kw == 0 && t == 0) {
        const unsigned w = __hip_atomic_fetch_add(L.ctrl + kCtrlHead, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int code = 2 * a.S;
        if ((int)w < a.S) code = a.order ? a.order[w] : (int)w;
        else if (B.slice > 0) code = requeued((int)w - a.S);
        s_w = code;
        if (K > 1) __hip_atomic_store(mbox, (unsigned)code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (K > 1) {
        barrier();
        if (kw != 0 && t == 0) s_w = (int)__hip_atomic_load(mbox, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int code = s_w;
    if (!alive || code >= 2 * a.S) break;
    const bool resumed = code >= a.S;
    const int s = resumed ? code - a.S : code;
    if (resumed) {   // the suspending slot's stores (released before it re-queued s): acquire
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    const long sn = (long)s * a.n, sm = (long)s * a.m, sN = (long)s * a.N;
    // PROF: per scenario {first start, end, iterations, splits} after the workgroup items
    unsigned long long* pf_scen = a.prof ? a.prof + (size_t)gridDim.x * 10 + (size_t)s * 4 : nullptr;
    if constexpr (PROF)
        if (kw == 0 && t == 0 && !resumed) pf_scen[0] = __builtin_amdgcn_s_memrealtime();
    double* SV = B.susp + (long)s * 8;   // suspended state: omega, kkt_restart, kkt_prev, it, since, cnt
    if (L.vstride != 0 || !vals_loaded) {   // (position -1: a padding entry, value 0)
        const double* rvs = L.rvals + (long)s * L.vstride;
        auto val = [&](int pp) { return pp >= 0 ? rvs[pp] : 0.0; };
        for (int q = t; q < G.nrz; q += NT) lrv[q] = val(B.rperm[G.rz0 + q]);
        for (int q = t; q < G.nlz; q += NT) lkv[q] = val(B.lperm[G.lz0 + q]);
        for (int q = t; q < G.ncz; q += NT) lcv[q] = val(B.cperm[G.cz0 + q]);
        vals_loaded = true;
    }
    double* XR = L.xr + sn;          // restart points (owner-only, touched at restarts)
    double* YR = L.yr + sm;

    // ------------------------------------------------------------------ prologue
    double x[E], xs[E], aty[E], cs[E], qs[E], ip[E], lo[E], hi[E];
    double y[E], ys[E], axo[E], rlo[E], rhi[E];
    double c2 = 0.0, prox_const = 0.0, cs2 = 0.0, b2 = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        x[e] = xs[e] = aty[e] = cs[e] = qs[e] = lo[e] = hi[e] = 0.0;
        ip[e] = 1.0;
        if (cv_[e]) {
            const int j = jc[e];
            const long b = sn + j;
            const double d = a.dc[b];
            double cc = a.c[b], qq = 0.0;
            double lo_ = a.cl[b], hi_ = a.cu[b];
            const int kk = a.lay.col_nonant[j];
            if (kk >= 0) {
                ph_terms(a, sN + kk, kk, cc, qq, prox_const);
                if (a.fix_nonants) fixed_box(a, sN + kk, d, lo_, hi_);
            }
            c2 += cc * cc;
            cs[e] = cc * d;
            cs2 += cs[e] * cs[e];
            qs[e] = qq * d * d;
            lo[e] = lo_;
            hi[e] = hi_;
            if (resumed) {   // (XR holds the suspended solve's restart point)
                x[e] = a.xs[b];
                xs[e] = L.xsum[b];
            } else {
                x[e] = clampd((a.warm & 1) ? a.xs_in[b] : 0.0, lo_, hi_);
                XR[j] = x[e];
            }
            Xl[t + e * NT] = x[e];
        }
        y[e] = ys[e] = axo[e] = rlo[e] = rhi[e] = 0.0;
        if (rv_[e]) {
            const int i = ir[e];
            row_bounds(a, i, sm + i, rlo[e], rhi[e]);
            double yy = (a.warm & 1) ? a.ys_in[sm + i] : 0.0;
            if (!fin(rlo[e])) yy = fmin(yy, 0.0); else b2 += rlo[e] * rlo[e];
            if (!fin(rhi[e])) yy = fmax(yy, 0.0); else b2 += rhi[e] * rhi[e];
            if (resumed) {
                yy = a.ys[sm + i];
                ys[e] = L.ysum[sm + i];
            } else {
                YR[i] = yy;
            }
            y[e] = yy;
            Yl[t + e * NT] = yy;
        }
    }
    double l_lo = 0.0, l_hi = 0.0, l_y = 0.0, l_ys = 0.0, l_yr = 0.0, l_ax = 0.0, l_dr = 1.0;
    int l_i = 0;
    if (t < NL) {
        l_i = B.link_rows[t];
        row_bounds(a, l_i, sm + l_i, l_lo, l_hi);
        l_dr = a.dr[sm + l_i];
        double yy = (a.warm & 1) ? a.ys_in[sm + l_i] : 0.0;
        if (!fin(l_lo)) yy = fmin(yy, 0.0); else if (kw == 0) b2 += l_lo * l_lo;
        if (!fin(l_hi)) yy = fmax(yy, 0.0); else if (kw == 0) b2 += l_hi * l_hi;
        l_y = l_yr = yy;
        if (resumed) {   // (the linking rows' restart point is kept in YR by the suspending slot)
            l_y = a.ys[sm + l_i];
            l_ys = L.ysum[sm + l_i];
            l_yr = YR[l_i];
        }
        yl[t] = l_y;
    }
    double omega, cnorm;
    {
        double rr[4] = {c2, prox_const, cs2, b2};
        scen_sum(rr);
        cnorm = sqrt(rr[0]);
        prox_const = rr[1];
        const double cn = sqrt(rr[2]), bn = sqrt(rr[3]);
        omega = (cn > 1e-10 && bn > 1e-10) ? cn / bn : 1.0;
        if ((a.warm & 2) && a.omega_in[s] > 0.0) omega = a.omega_in[s];
        else if ((a.warm & 4) && a.omega_in[s] > 0.0) omega = sqrt(omega * a.omega_in[s]);
        if (resumed) omega = SV[0];
    }
    const double bnorm = a.bnorm[s], eta = a.eta[s];
    double tau = eta / omega, sig = eta * omega;
    auto step_coefs = [&]() {
#pragma unroll
        for (int e = 0; e < E; ++e) ip[e] = 1.0 / (1.0 + tau * qs[e]);
    };
    step_coefs();
    auto products = [&]() {   // A x, A^T y at the current point (Xl, Yl, yl current; after a barrier)
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (rv_[e]) axo[e] = ax_loc(t + e * NT);
        l_ax = exchange(ax_link());
        settle();
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (cv_[e]) aty[e] = aty_col(t + e * NT);
    };
    products();

    // KKT pieces (pdhg_stream.hip); avg: the products of the running sums staged through Xl / Yl
    auto kkt_part = [&](bool avg, double inv, const double* axa, const double* ata, double l_axs, double* o) {
        double v[6] = {0, 0, 0, 0, 0, 0};
        auto row_terms = [&](double axx, double yy, double lo_, double hi_, double dr) {
            const double pr = axx - clampd(axx, lo_, hi_);
            v[0] += pr * pr;
            const double pu = pr / dr;
            v[2] += pu * pu;
            if (fin(lo_)) v[5] += lo_ * fmax(yy, 0.0);
            if (fin(hi_)) v[5] += hi_ * fmin(yy, 0.0);
        };
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (rv_[e])
                row_terms(avg ? axa[e] * inv : axo[e], avg ? ys[e] * inv : y[e], rlo[e], rhi[e], a.dr[sm + ir[e]]);
        if (kw == 0 && t < NL) row_terms(avg ? l_axs * inv : l_ax, avg ? l_ys * inv : l_y, l_lo, l_hi, l_dr);
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (cv_[e]) {
                const double xx = avg ? xs[e] * inv : x[e];
                const double at = avg ? ata[e] * inv : aty[e];
                const double rc_ = cs[e] + qs[e] * xx - at;
                double dres = 0.0;
                if (!fin(lo[e]) && rc_ > 0.0) dres += rc_;
                if (!fin(hi[e]) && rc_ < 0.0) dres += rc_;
                v[1] += dres * dres;
                const double du = dres / a.dc[sn + jc[e]];
                v[3] += du * du;
                const double hq = 0.5 * qs[e] * xx * xx;
                v[4] += cs[e] * xx + hq;
                if (fin(lo[e])) v[5] += lo[e] * fmax(rc_, 0.0);
                if (fin(hi[e])) v[5] += hi[e] * fmin(rc_, 0.0);
                v[5] -= hq;
            }
#pragma unroll
        for (int u = 0; u < 6; ++u) o[u] = v[u];
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
    int it = 0, since = 0, cnt = 0, st = 1;
    if (resumed) {
        kkt_restart = SV[1];
        kkt_prev = SV[2];
        it = (int)SV[3];
        since = (int)SV[4];
        cnt = (int)SV[5];
    } else {
        double o[6];
        kkt_part(false, 0.0, nullptr, nullptr, 0.0, o);
        scen_sum(o);
        kkt_restart = wkkt_of(o, omega);
    }
    bool suspend = false;
    double rel_final = INFINITY, pobj = 0.0, dobj = 0.0;
    bool use_avg_final = false;
    const int chk = a.check_every;

    // primal step of owned column e (A^T y in aty)
    auto primal = [&](int e) {
        const double xn = clampd(fma(tau, aty[e] - cs[e], x[e]) * ip[e], lo[e], hi[e]);
        x[e] = xn;
        xs[e] += xn;
        Xl[t + e * NT] = xn;
    };
    PF(7);
    while (alive) {
        PF(6);
        // pre: the columns without a linking entry took this iteration's primal step already, during
        // the previous iteration's second hop (never across a check: their A^T y is final there)
        bool pre = false;
        for (int kk = 0; kk < chk && alive; ++kk) {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (cv_[e] && !(pre && loc_[e])) primal(e);
            __syncthreads();
            PF(0);
            // the iteration's one cross-workgroup step, overlapped: the linking-row partials go out
            // first; the local rows' dual step runs during hop 1, the A^T y of the columns without a
            // linking-row entry during hop 2 (it needs only the local y, visible after the exchange's
            // barrier); the other columns' A^T y after the linking y.  Same operations as before,
            // reordered: the same bits (test_border_matches_block_kernel)
            const double axl = ax_link();
            const unsigned ep = ex_publish(axl);
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (rv_[e]) {
                    const double axn = ax_loc(t + e * NT);
                    const double g = y[e] - sig * (2.0 * axn - axo[e]);
                    const double yn = fmax(fma(sig, rlo[e], g), 0.0) + fmin(fma(sig, rhi[e], g), 0.0);
                    axo[e] = axn;
                    y[e] = yn;
                    ys[e] += yn;
                    Yl[t + e * NT] = yn;
                }
            PF(1);
            pre = kk + 1 < chk;
            const double axn_l = ex_complete(ep, axl, [&]() {
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (cv_[e] && loc_[e]) {
                        aty[e] = aty_col(t + e * NT);
                        // the next iteration's primal step of this column: its A^T y is complete
                        // (no linking row), and every read of Xl of this iteration has passed the
                        // exchange's barrier
                        if (pre) primal(e);
                    }
            });
            if (t < NL) {
                const double g = l_y - sig * (2.0 * axn_l - l_ax);
                l_y = fmax(fma(sig, l_lo, g), 0.0) + fmin(fma(sig, l_hi, g), 0.0);
                l_ax = axn_l;
                l_ys += l_y;
                yl[t] = l_y;
            }
            settle();
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (cv_[e] && !loc_[e]) aty[e] = aty_col(t + e * NT);
            PF(5);
        }
        if (!alive) break;
        it += chk;
        since += chk;
        cnt += chk;

        const double inv = 1.0 / (double)cnt;
        // products at the average: stage the running sums in Xl / Yl / yl, gather, restore
        double axa[E], ata[E];
        __syncthreads();   // every ATY gather of the last iteration is done with Yl
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (cv_[e]) Xl[t + e * NT] = xs[e];
            if (rv_[e]) Yl[t + e * NT] = ys[e];
        }
        if (t < NL) yl[t] = l_ys;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e) {
            axa[e] = rv_[e] ? ax_loc(t + e * NT) : 0.0;
            ata[e] = cv_[e] ? aty_col(t + e * NT) : 0.0;
        }
        const double l_axs = exchange(ax_link());
        settle();   // every gather of the staged sums is done
        if (!alive) break;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (cv_[e]) Xl[t + e * NT] = x[e];
            if (rv_[e]) Yl[t + e * NT] = y[e];
        }
        if (t < NL) yl[t] = l_y;
        double oc[6], oa[6];
        kkt_part(false, 0.0, nullptr, nullptr, 0.0, oc);
        kkt_part(true, inv, axa, ata, l_axs, oa);
        {
            // [12]: 1 when workgroup 0 decides to suspend the solve at this check (split solves):
            // the same decision in every workgroup of the slot
            double both[13];
#pragma unroll
            for (int u = 0; u < 6; ++u) { both[u] = oc[u]; both[6 + u] = oa[u]; }
            both[12] = 0.0;
            if (B.slice > 0 && !resumed && kw == 0 && t == 0 && it >= B.slice * chk &&
                __hip_atomic_load(L.ctrl + kCtrlHead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)a.S)
                both[12] = 1.0;
            scen_sum(both);   // (its workgroup barriers also publish the restored Xl / Yl)
#pragma unroll
            for (int u = 0; u < 6; ++u) { oc[u] = both[u]; oa[u] = both[6 + u]; }
            suspend = both[12] > 0.5;
        }
        const double rel_cur = rel_of(oc), rel_avg = rel_of(oa);
        const bool nan = !(rel_cur == rel_cur);
        if (nan || rel_cur <= a.eps || rel_avg <= a.eps || it >= a.max_iter) {
            use_avg_final = !nan && rel_avg < rel_cur;
            rel_final = use_avg_final ? rel_avg : rel_cur;
            pobj = use_avg_final ? oa[4] : oc[4];
            dobj = use_avg_final ? oa[5] : oc[5];
            st = nan ? 2 : ((rel_cur <= a.eps || rel_avg <= a.eps) ? 0 : 1);
            suspend = false;   // terminated at this check: nothing to resume
            break;
        }
        const double k_cur = wkkt_of(oc, omega), k_avg = wkkt_of(oa, omega);
        const bool use_avg = k_avg < k_cur;
        const double cand = use_avg ? k_avg : k_cur;
        const bool restart = (cand <= a.beta_suf * kkt_restart) ||
                             (cand <= a.beta_nec * kkt_restart && cand > kkt_prev) ||
                             ((double)since >= a.beta_art * (double)it);
        kkt_prev = cand;
        if (restart) {
            double mv[2] = {0.0, 0.0};
#pragma unroll
            for (int e = 0; e < E; ++e) {
                if (cv_[e]) {
                    const int j = jc[e];
                    const double xv = use_avg ? xs[e] * inv : x[e];
                    const double d = xv - XR[j];
                    mv[0] += d * d;
                    XR[j] = xv;
                    x[e] = xv;
                    xs[e] = 0.0;
                    Xl[t + e * NT] = xv;
                }
                if (rv_[e]) {
                    const int i = ir[e];
                    const double yv = use_avg ? ys[e] * inv : y[e];
                    const double d = yv - YR[i];
                    mv[1] += d * d;
                    YR[i] = yv;
                    y[e] = yv;
                    ys[e] = 0.0;
                    Yl[t + e * NT] = yv;
                }
            }
            if (t < NL) {
                const double yv = use_avg ? l_ys * inv : l_y;
                const double d = yv - l_yr;
                if (kw == 0) mv[1] += d * d;
                l_yr = l_y = yv;
                l_ys = 0.0;
                yl[t] = yv;
            }
            scen_sum(mv);
            omega = primal_weight(omega, mv[0], mv[1], a.theta);
            tau = eta / omega;
            sig = eta * omega;
            step_coefs();
            cnt = 0;
            since = 0;
            kkt_restart = cand;
            kkt_prev = INFINITY;
            if (use_avg) products();
        }
        if (suspend) break;
    }
    // a scenario given up (a co-resident workgroup missing: the bounded wait expired) reports status 2;
    // its x is NOT a consistent iterate -- columns without a linking-row entry may already have taken
    // the next iteration's primal step -- and callers treat status 2 as a failed solve
    if (!alive) { st = 2; rel_final = NAN; }

    if (alive && suspend) {   // save the solve's state, release it, re-queue the scenario
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (cv_[e]) {
                a.xs[sn + jc[e]] = x[e];
                L.xsum[sn + jc[e]] = xs[e];
            }
            if (rv_[e]) {
                a.ys[sm + ir[e]] = y[e];
                L.ysum[sm + ir[e]] = ys[e];
            }
        }
        if (kw == 0 && t < NL) {
            a.ys[sm + l_i] = l_y;
            L.ysum[sm + l_i] = l_ys;
            YR[l_i] = l_yr;
        }
        if (kw == 0 && t == 0) {
            SV[0] = omega;
            SV[1] = kkt_restart;
            SV[2] = kkt_prev;
            SV[3] = (double)it;
            SV[4] = (double)since;
            SV[5] = (double)cnt;
            // provisional outputs of a suspended solve: a failed solve (status 2, NaN KKT) unless the
            // slot that resumes it overwrites them -- a scenario no slot resumes (its waiting slot gave
            // up: requeued()) is then reported as failed, never with the previous launch's values
            a.status[s] = 2;
            a.kkt[s] = NAN;
            if constexpr (PROF) pf_scen[3] += 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        barrier();   // every workgroup of the slot has released its part
        if (kw == 0 && t == 0) {
            const unsigned j = __hip_atomic_fetch_add(L.ctrl + kCtrlTail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(B.requeue + j, s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!alive) break;
        __syncthreads();
        continue;
    }

    // ------------------------------------------------------------------ outputs
    const double inv = cnt > 0 ? 1.0 / (double)cnt : 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (cv_[e]) {
            const int j = jc[e];
            const long b = sn + j;
            const double xv = use_avg_final ? xs[e] * inv : x[e];
            a.xs[b] = xv;
            const double xu = xv * a.dc[b];
            if (a.x_out) a.x_out[b] = xu;
            const int kk = a.lay.col_nonant[j];
            if (kk >= 0) a.xN[sN + kk] = xu;
        }
        if (rv_[e]) {
            const long b = sm + ir[e];
            const double yv = use_avg_final ? ys[e] * inv : y[e];
            a.ys[b] = yv;
            if (a.y_out) a.y_out[b] = yv * a.dr[b];
        }
    }
    if (kw == 0 && t < NL) {
        const long b = sm + l_i;
        const double yv = use_avg_final ? l_ys * inv : l_y;
        a.ys[b] = yv;
        if (a.y_out) a.y_out[b] = yv * a.dr[b];
    }
    if (kw == 0 && t == 0) {
        const double offs = a.obj_off[s] + (a.prox_on ? prox_const : 0.0);
        a.omega[s] = omega;
        a.obj[s] = a.sense * (pobj + offs);
        a.bound[s] = a.sense * (dobj + offs);
        a.kkt[s] = rel_final;
        a.iters[s] = it;
        a.iters_acc[s] += it;
        a.status[s] = st;
        if (B.slice > 0) __hip_atomic_fetch_add(L.ctrl + kCtrlDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (PROF) {
            pf_scen[1] = __builtin_amdgcn_s_memrealtime();
            pf_scen[2] = (unsigned long long)it;
        }
    }
    if constexpr (PROF) {
        PF(7);
        pf_it += it;
        ++pf_sc;
    }
    if (!alive) break;
    __syncthreads();
    }   // scenario queue
    if constexpr (PROF) {   // lane u of wave 0 stores item u (vector stores)
        const int lane = t & 63;
        if (t < 64) {
            unsigned long long v = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) v = lane == u ? pf[u] : v;
            v = lane == 8 ? pf_it : (lane == 9 ? pf_sc : v);
            if (lane < 10) a.prof[(size_t)blockIdx.x * 10 + lane] = v;
        }
    }
}

// ----------------------------------------------------------------------------- dispatch
constexpr int kBorderNT = 1024;

// granule words of the register variant: G1 [slots][2][NL][K][2], G2 [slots][2][NL][2], GS [slots][2][K][16][2]
size_t pdhg_border_granule_words(const BorderLayout& B, const StreamLayout& L) {
    return (size_t)L.slots * 2 * 2 * ((size_t)B.nlink * L.K + B.nlink + 16 * (size_t)L.K);
}

size_t pdhg_border_lds_bytes(const BorderLayout& B) {
    if (B.reg)   // register-resident: x / y in LDS, no column / row lists
        return (size_t)(B.nrz_max + B.nlz_max + B.ncz_max + B.C_max + B.R_max + B.nlink + B.xtmp_len) * sizeof(double) +
               (size_t)(B.R_max + 1 + B.nrz_max + B.nlink + 1 + B.nlz_max + B.C_max + 1 + B.ncz_max) * sizeof(int);
    return (size_t)(B.nrz_max + B.nlz_max + B.ncz_max + 2 * B.nlink) * sizeof(double) +
           (size_t)(B.C_max + B.R_max + B.R_max + 1 + B.nrz_max + B.nlink + 1 + B.nlz_max + B.C_max + 1 + B.ncz_max) *
               sizeof(int);
}

// register-resident variant: 512-thread workgroups (launch bounds allow 256 VGPRs: the owned
// elements' state stays in registers), E = 2 elements per thread; its LDS request is padded
// past half a CU's 160 KB so that, like the 1024-thread kernels, it runs one workgroup per CU (the
// hand-off protocol of stream_sync.h is measured for that)
constexpr int kBorderRegNT = 512;
constexpr size_t kOnePerCuLds = 82 * 1024;

int pdhg_border_max_per_thread() { return 2 * kBorderRegNT; }   // elements per workgroup (E = 2: no spills)

hipError_t pdhg_border_launch(const PdhgArgs& a, hipStream_t stream) {
    const StreamLayout& L = a.st;
    hipError_t e = hipMemsetAsync(L.ctrl, 0, (size_t)(kCtrlBar + 3 * L.slots) * sizeof(unsigned), stream);
    if (e != hipSuccess) return e;
    // the give-up flag too: a timeout in an earlier launch must not end this one's waits at once
    e = hipMemsetAsync(L.err, 0, sizeof(int), stream);
    if (e != hipSuccess) return e;
    if (a.bd.reg && a.bd.slice > 0) {   // split solves: the re-queue starts empty
        e = hipMemsetAsync(a.bd.requeue, 0, (size_t)a.S * sizeof(int), stream);
        if (e != hipSuccess) return e;
    }
    if (a.bd.reg && L.K > 1) {   // tagged granules start from tag 0 every launch
        e = hipMemsetAsync(a.bd.plink, 0, pdhg_border_granule_words(a.bd, L) * sizeof(unsigned long long), stream);
        if (e != hipSuccess) return e;
    }
    const dim3 grid((unsigned)L.slots * (unsigned)L.K), block(a.bd.reg ? kBorderRegNT : kBorderNT);
    const size_t lds = a.bd.reg ? std::max(pdhg_border_lds_bytes(a.bd), kOnePerCuLds) : pdhg_border_lds_bytes(a.bd);
    PdhgArgs copy = a;
    void* args[] = {&copy};
    const void* fn = !a.bd.reg ? (const void*)pdhg_border_kernel<kBorderNT>
                     : a.prof ? (const void*)pdhg_border_reg_kernel<kBorderRegNT, 2, true>
                              : (const void*)pdhg_border_reg_kernel<kBorderRegNT, 2, false>;
    if (L.K == 1 || !coop_launch_enabled()) return hipLaunchKernel(fn, grid, block, args, lds, stream);
    return hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)lds, stream);
}

}  // namespace phg
