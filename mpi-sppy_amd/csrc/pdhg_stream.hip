// pdhg_stream.hip -- batched PDHG for scenario LPs / QPs far larger than a workgroup's LDS
// (UC-shaped: n, m ~ 2e4, nnz ~ 6e4 per scenario), on gfx950.
//
// Same algorithm, restart rule, termination test and outputs as the other PDHG kernels (replaces
// SPOpt.solve_one, mpisppy/spopt.py:184-231, for every local scenario).  Mapping:
//
//   * K workgroups of NT threads per scenario (grid S * K; K from the host so the grid fills the
//     chip even at tens of scenarios); workgroup k owns a contiguous range of rows and of columns
//     (split by nonzeros on the host);
//   * NOTHING of the scenario stays on chip between iterations: iterates, running sums, costs,
//     bounds and the CSR / CSC values are streamed from memory every PDHG iteration -- the HBM
//     streaming path of SURVEY 8(d)1;
//   * one PDHG iteration = primal step on owned columns (A^T y from the CSC), a cross-workgroup
//     barrier, dual step on owned rows (A x from the CSR), a barrier, A^T y of the new y on owned
//     columns.  Values other workgroups read (x, y, the running sums, reduction partials) are
//     stored sc1 (write-through) and EVERY load of them is an sc1 load (L2-served, never L1), the
//     barrier counter is one agent-scope add per workgroup behind a workgroup barrier and is
//     polled with sc1 loads: the hand-off MI355X_MICROARCH.md measures valid WITHOUT an agent
//     acquire (row 1 of its table, one workgroup per CU -- 1024-thread workgroups at <= 128
//     VGPRs are exactly that), which would otherwise cost ~1.7 us per CU per barrier;
//   * per-scenario sums (KKT norms, objectives, primal-weight movement) are workgroup sums
//     published per workgroup and added by EVERY workgroup in workgroup order: all K workgroups
//     hold the same bits and take the same restart / termination decisions;
//   * every barrier wait is bounded: past ~0.5 s of spinning the scenario is abandoned with status
//     2 and a device error flag (the grid always drains).  K > 1 needs the scenario's workgroups
//     co-resident: the host launches cooperatively (hipLaunchCooperativeKernel fails rather than
//     over-subscribing).
#include "phg_internal.h"
#include "wave_ops.h"
#include "stream_sync.h"

namespace phg {

template <int NT, bool RES>
__global__ __launch_bounds__(NT) void pdhg_stream_kernel(PdhgArgs a) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (PdhgArgs::gate)
    __shared__ double red[16 * (NT / 64)];
    __shared__ int s_w;
    extern __shared__ double dyn[];
    const StreamLayout& L = a.st;
    const int K = L.K;
    const int slot = blockIdx.x / K, kw = blockIdx.x % K;
    const int t = threadIdx.x;
    const int r0 = L.row_first[kw], r1 = L.row_first[kw + 1];
    const int c0 = L.col_first[kw], c1 = L.col_first[kw + 1];
    const int p0 = L.rowptr[r0], q0 = L.colptr[c0];      // first nonzero of the owned rows / columns
    const int nr = L.rowptr[r1] - p0, nc = L.colptr[c1] - q0;
    // resident slice (RES): the owned rows' CSR and the owned columns' CSC, values per scenario
    double* lrv = dyn;
    double* lcv = lrv + L.nr_max;
    int* lrp = reinterpret_cast<int*>(lcv + L.nc_max);
    int* lci = lrp + L.R_max + 1;
    int* lcp = lci + L.nr_max;
    int* lri = lcp + L.C_max + 1;
    if (RES) {
        for (int i = t; i <= r1 - r0; i += NT) lrp[i] = L.rowptr[r0 + i] - p0;
        for (int q = t; q < nr; q += NT) lci[q] = L.colidx[p0 + q];
        for (int j = t; j <= c1 - c0; j += NT) lcp[j] = L.colptr[c0 + j] - q0;
        for (int q = t; q < nc; q += NT) lri[q] = L.rowidx[q0 + q];
    }
    double* part = L.part + (long)slot * K * 16;
    unsigned* bar = L.ctrl + kCtrlBar + 2 * slot;
    unsigned* mbox = L.ctrl + kCtrlBar + 2 * L.slots + slot;
    unsigned nbar = 0;
    bool alive = true;
    auto barrier = [&]() {
        if (K == 1) { __syncthreads(); return; }
        ++nbar;
        if (!scen_barrier(bar, nbar * (unsigned)K, L.err)) alive = false;
    };
    // scenario sum of V values: workgroup sums published, then every workgroup adds all K in order
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
    bool vals_loaded = false;

    // the slot's K workgroups take scenarios from one queue, heaviest first (a.order), until it is
    // empty: workgroup 0 dequeues and publishes the index in the slot's mailbox
    while (true) {
    if (kw == 0 && t == 0) {
        const unsigned w = __hip_atomic_fetch_add(L.ctrl + kCtrlHead, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_w = (int)w;
        if (K > 1) __hip_atomic_store(mbox, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (K > 1) {
        barrier();   // the mailbox is published (its next write follows this scenario's barriers)
        if (kw != 0 && t == 0) s_w = (int)__hip_atomic_load(mbox, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int wi = s_w;
    if (!alive || wi >= a.S) break;
    const int s = a.order ? a.order[wi] : wi;
    const long sn = (long)s * a.n, sm = (long)s * a.m, sN = (long)s * a.N;
    const double* rv = L.rvals + (long)s * L.vstride;
    const double* cv = L.cvals + (long)s * L.vstride;
    if (RES && (L.vstride != 0 || !vals_loaded)) {
        for (int q = t; q < nr; q += NT) lrv[q] = rv[p0 + q];
        for (int q = t; q < nc; q += NT) lcv[q] = cv[q0 + q];
        vals_loaded = true;
    }
    __syncthreads();
    double* X = a.xs + sn;            // current x (published), the solve's output copy
    double* Y = a.ys + sm;
    double* XS = L.xsum + sn;         // running sums since the last restart (published)
    double* YS = L.ysum + sm;
    double* CS = L.cs + sn;           // scaled cost with the PH terms
    double* QS = L.qs + sn;           // scaled prox diagonal
    double* LO = L.lo + sn;           // scaled column bounds (fixed nonants applied)
    double* HI = L.hi + sn;
    double* ATY = L.aty + sn;         // A^T y of the current y, owned columns
    double* XR = L.xr + sn;           // restart point
    double* AXO = L.axo + sm;         // A x of the current x, owned rows
    double* YR = L.yr + sm;
    auto rowb = [&](int i, double& lo, double& hi) { row_bounds(a, i, sm + i, lo, hi); };

    // ------------------------------------------------------------------ prologue (owned elements)
    double c2 = 0.0, prox_const = 0.0, cs2 = 0.0, b2 = 0.0;
    for (int j = c0 + t; j < c1; j += NT) {
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
        put(&X[j], x0);
        XR[j] = x0;
        put(&XS[j], 0.0);
    }
    for (int i = r0 + t; i < r1; i += NT) {
        double lo_, hi_;
        rowb(i, lo_, hi_);
        double yy = (a.warm & 1) ? a.ys_in[sm + i] : 0.0;
        if (!fin(lo_)) yy = fmin(yy, 0.0); else b2 += lo_ * lo_;
        if (!fin(hi_)) yy = fmax(yy, 0.0); else b2 += hi_ * hi_;
        put(&Y[i], yy);
        YR[i] = yy;
        put(&YS[i], 0.0);
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
    }
    const double bnorm = a.bnorm[s], eta = a.eta[s];
    double tau = eta / omega, sig = eta * omega;

    // products of the published x / y for the owned rows / columns
    auto ax_row = [&](const double* xv, int i) {
        double acc = 0.0;
        if (RES) {
            for (int p = lrp[i - r0]; p < lrp[i - r0 + 1]; ++p) acc = fma(lrv[p], get(&xv[lci[p]]), acc);
        } else {
            for (int p = L.rowptr[i]; p < L.rowptr[i + 1]; ++p) acc = fma(rv[p], get(&xv[L.colidx[p]]), acc);
        }
        return acc;
    };
    auto aty_col = [&](const double* yv, int j) {
        double acc = 0.0;
        if (RES) {
            for (int p = lcp[j - c0]; p < lcp[j - c0 + 1]; ++p) acc = fma(lcv[p], get(&yv[lri[p]]), acc);
        } else {
            for (int p = L.colptr[j]; p < L.colptr[j + 1]; ++p) acc = fma(cv[p], get(&yv[L.rowidx[p]]), acc);
        }
        return acc;
    };
    barrier();   // x, y published
    for (int i = r0 + t; i < r1; i += NT) AXO[i] = ax_row(X, i);
    for (int j = c0 + t; j < c1; j += NT) ATY[j] = aty_col(Y, j);

    // KKT pieces of the current iterate (inv = 0) or of the average (inv = 1 / cnt; its products
    // from the published running sums), owned elements, then summed over the scenario:
    // [0] ||pr||^2 scaled, [1] ||dres||^2 scaled, [2] ||pr||^2, [3] ||dres||^2 unscaled, [4] pobj, [5] dobj
    auto kkt_part = [&](bool avg, double inv, double* o) {
        double v[6] = {0, 0, 0, 0, 0, 0};
        for (int i = r0 + t; i < r1; i += NT) {
            double lo_, hi_;
            rowb(i, lo_, hi_);
            const double axx = avg ? ax_row(XS, i) * inv : AXO[i];
            const double yy = avg ? get(&YS[i]) * inv : get(&Y[i]);
            const double pr = axx - clampd(axx, lo_, hi_);
            v[0] += pr * pr;
            const double pu = pr / a.dr[sm + i];
            v[2] += pu * pu;
            if (fin(lo_)) v[5] += lo_ * fmax(yy, 0.0);
            if (fin(hi_)) v[5] += hi_ * fmin(yy, 0.0);
        }
        for (int j = c0 + t; j < c1; j += NT) {
            const double xx = avg ? get(&XS[j]) * inv : get(&X[j]);
            const double at = avg ? aty_col(YS, j) * inv : ATY[j];
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
        kkt_part(false, 0.0, o);
        scen_sum(o);
        kkt_restart = wkkt_of(o, omega);
    }
    int it = 0, since = 0, cnt = 0, st = 1;
    double rel_final = INFINITY, pobj = 0.0, dobj = 0.0;
    bool use_avg_final = false;
    const int chk = a.check_every;

    while (alive) {
        for (int kk = 0; kk < chk && alive; ++kk) {
            // primal step on owned columns (A^T y of the current y in ATY)
            for (int j = c0 + t; j < c1; j += NT) {
                const double ip = 1.0 / (1.0 + tau * QS[j]);
                const double xn = clampd(fma(tau, ATY[j] - CS[j], get(&X[j])) * ip, LO[j], HI[j]);
                put(&X[j], xn);
                put(&XS[j], get(&XS[j]) + xn);
            }
            barrier();
            // dual step on owned rows: A (2 x+ - x) = 2 A x+ - A x
            for (int i = r0 + t; i < r1; i += NT) {
                double lo_, hi_;
                rowb(i, lo_, hi_);
                const double axn = ax_row(X, i);
                const double g = get(&Y[i]) - sig * (2.0 * axn - AXO[i]);
                const double yn = fmax(fma(sig, lo_, g), 0.0) + fmin(fma(sig, hi_, g), 0.0);
                AXO[i] = axn;
                put(&Y[i], yn);
                put(&YS[i], get(&YS[i]) + yn);
            }
            barrier();
            for (int j = c0 + t; j < c1; j += NT) ATY[j] = aty_col(Y, j);
        }
        if (!alive) break;
        it += chk;
        since += chk;
        cnt += chk;

        const double inv = 1.0 / (double)cnt;
        double oc[6], oa[6];
        kkt_part(false, 0.0, oc);
        kkt_part(true, inv, oa);
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
            // new point (own elements), its movement since the last restart, published
            double mv[2] = {0.0, 0.0};
            for (int j = c0 + t; j < c1; j += NT) {
                const double xv = use_avg ? get(&XS[j]) * inv : get(&X[j]);
                const double d = xv - XR[j];
                mv[0] += d * d;
                XR[j] = xv;
                put(&X[j], xv);
                put(&XS[j], 0.0);
            }
            for (int i = r0 + t; i < r1; i += NT) {
                const double yv = use_avg ? get(&YS[i]) * inv : get(&Y[i]);
                const double d = yv - YR[i];
                mv[1] += d * d;
                YR[i] = yv;
                put(&Y[i], yv);
                put(&YS[i], 0.0);
            }
            scen_sum(mv);   // (its barriers also publish the new point)
            omega = primal_weight(omega, mv[0], mv[1], a.theta);
            tau = eta / omega;
            sig = eta * omega;
            cnt = 0;
            since = 0;
            kkt_restart = cand;
            kkt_prev = INFINITY;
            if (use_avg) {   // exact products at the new point
                for (int i = r0 + t; i < r1; i += NT) AXO[i] = ax_row(X, i);
                for (int j = c0 + t; j < c1; j += NT) ATY[j] = aty_col(Y, j);
            }
        }
    }
    if (!alive) { st = 2; rel_final = NAN; }

    // ------------------------------------------------------------------ outputs (owned elements)
    const double inv = cnt > 0 ? 1.0 / (double)cnt : 0.0;
    for (int j = c0 + t; j < c1; j += NT) {
        const long b = sn + j;
        const double xv = use_avg_final ? get(&XS[j]) * inv : get(&X[j]);
        put(&X[j], xv);
        const double xu = xv * a.dc[b];
        if (a.x_out) a.x_out[b] = xu;
        const int kk = a.lay.col_nonant[j];
        if (kk >= 0) a.xN[sN + kk] = xu;
    }
    for (int i = r0 + t; i < r1; i += NT) {
        const long b = sm + i;
        const double yv = use_avg_final ? get(&YS[i]) * inv : get(&Y[i]);
        put(&Y[i], yv);
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
    }   // scenario queue
}

// ----------------------------------------------------------------------------- dispatch
constexpr int kStreamNT = 1024;

int pdhg_stream_threads() { return kStreamNT; }

size_t pdhg_stream_lds_bytes(const StreamLayout& L) {
    if (!L.res) return 0;
    return (size_t)(L.nr_max + L.nc_max) * sizeof(double) +
           (size_t)(L.R_max + 1 + L.nr_max + L.C_max + 1 + L.nc_max) * sizeof(int);
}

// workgroups that can be resident at once (for the co-residency of a scenario's K workgroups)
hipError_t pdhg_stream_capacity(int* out) {
    int dev = 0, cus = 0, per = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pdhg_stream_kernel<kStreamNT, false>, kStreamNT, 0);
    if (e != hipSuccess) return e;
    // a 1024-thread workgroup at <= 128 VGPRs fills a CU's 16 wave slots: one per CU, whatever the
    // occupancy API says (the barriers' hand-off protocol is measured for one per CU)
    *out = std::min(per, 1) * cus;
    return hipSuccess;
}

hipError_t pdhg_stream_launch(const PdhgArgs& a, hipStream_t stream) {
    const StreamLayout& L = a.st;
    // queue head, barrier counters and mailboxes start from zero every launch
    hipError_t e = hipMemsetAsync(L.ctrl, 0, (size_t)(kCtrlBar + 3 * L.slots) * sizeof(unsigned), stream);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(L.err, 0, sizeof(int), stream);   // the give-up flag too (per launch)
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)L.slots * (unsigned)L.K), block(kStreamNT);
    const size_t lds = pdhg_stream_lds_bytes(L);
    const void* fn = L.res ? (const void*)pdhg_stream_kernel<kStreamNT, true> : (const void*)pdhg_stream_kernel<kStreamNT, false>;
    PdhgArgs copy = a;
    void* args[] = {&copy};
    if (L.K == 1 || !coop_launch_enabled()) return hipLaunchKernel(fn, grid, block, args, lds, stream);
    return hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)lds, stream);
}

}  // namespace phg
