// pdhg_mfma.hip -- batched PDHG for scenario LPs / QPs that SHARE their constraint matrix, with
// A x and A^T y of 16 scenarios at a time on the fp64 matrix cores (v_mfma_f64_16x16x4_f64).
//
// Same algorithm, restart rule, termination test and outputs as pdhg_local.hip (replaces
// SPOpt.solve_one, mpisppy/spopt.py:184-231, for every local scenario).  Used when every scenario
// has the same A -- only costs, bounds and right-hand sides differ, e.g. hydro's inflows
// (examples/hydro/hydro.py:79-152) -- and A is small enough (n, m <= 16: one 16 x 16 tile) for
// the iterates of 16 scenarios and A's MFMA fragments to stay in registers:
//
//   * one wave = 16 scenarios, the MFMA's N dimension (scenario = lane & 15);
//   * a vector of length 16 T (x: columns, y: rows) is held as T tiles in the MFMA's f64 C/D
//     layout: lane l, register j of tile t holds element 16 t + (l >> 4) + 4 j of scenario l & 15
//     (cdna_hip_programming.md: f64 C/D col = lane & 15, row = (lane >> 4) + 4 reg);
//   * that layout IS the B operand of the next product: register j of a tile is B[k = l >> 4][n]
//     for the k-step covering elements 16 t + 4 j + k, so A x -> dual step -> A^T y -> primal step
//     never moves data between lanes; the A operand of each k-step is a fixed fragment of the
//     scaled shared matrix, built once per batch (phg_api.hip: build_mfma_fragments) and held in
//     registers (16 x 4 fragments that are all zero are skipped);
//   * per-scenario sums (KKT norms, objectives, primal-weight movement) add a lane's own elements
//     and then the scenario's 4 lanes (l, l^16, l^32, l^48) with v_permlane16/32_swap.
//
// Roofline: fp64 matrix-core bound, 2 * 16 TM * 16 TN * 2 flops per scenario per PDHG iteration
// for the two products as executed dense (SURVEY 8(d)2, F = 4 m n S) -- on MI355X the fp64 MFMA
// rate equals the fp64 VALU rate (78.6 TF), so what the matrix cores buy here is 16 scenarios per
// wave with every operand in registers, not a faster multiply.
#include "phg_internal.h"
#include "wave_ops.h"

namespace phg {

using d4 = __attribute__((ext_vector_type(4))) double;

// sum over the 4 lanes holding one scenario (same bits in all four)
template <int K>
__device__ __forceinline__ void ssum_many(double (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = swap16_add(v[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = swap32_add(v[k]);
}

template <int TM, int TN>
struct MCold {
    static constexpr int KC = 4 * TN, KR = 4 * TM;
    static constexpr int XR = 0, Q = KC, IDC = 2 * KC, C = 3 * KC, YR = 4 * KC, IDR = YR + KR, BLO = IDR + KR,
                         BHI = BLO + KR, SC = BHI + KR;
    enum { CNORM = 0, BNORM, ETA, PROX, OMEGA, KRST, KPREV, TP, TD, W2, IW2, KOFF, NSC };   // KOFF: gap_den's K
    static constexpr int N = SC + NSC;
};

// WATCH (diagnostic, PHG_WATCH_SCEN): the watched scenario's every check printed
template <int TM, int TN, bool WATCH>
__global__ __launch_bounds__(64, 2) void pdhg_mfma_kernel(PdhgArgs a) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (PdhgArgs::gate)
    constexpr int KC = 4 * TN, KR = 4 * TM, NF = 4 * TM * TN;
    using CI = MCold<TM, TN>;
    extern __shared__ double cold[];
    const int lane = threadIdx.x;
    const int g = lane >> 4;                       // lane row: element offset inside a tile row block
    auto CS = [&](int item) -> double& { return cold[item * 64 + lane]; };
    // per-scenario scalars: one slot per scenario, written with the same bits by its 4 lanes
    auto SS = [&](int item) -> double& { return cold[CI::SC * 64 + item * 16 + (lane & 15)]; };
    const int w_raw = blockIdx.x * 16 + (lane & 15);
    const bool valid = w_raw < a.S;
    const int w = valid ? w_raw : a.S - 1;         // a tail lane mirrors the last item, writes nothing
    const int s = a.order ? a.order[w] : w;
    const int* col_nonant = a.lay.col_nonant;
    auto colof = [&](int k) { return 16 * (k >> 2) + g + 4 * (k & 3); };
    auto rowof = [&](int r) { return 16 * (r >> 2) + g + 4 * (r & 3); };

    // ------------------------------------------------------------------ A fragments
    double fa[NF], fb[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        fa[f] = a.mf.frag[(long)f * 64 + lane];
        fb[f] = a.mf.frag[(long)(NF + f) * 64 + lane];
    }
    const unsigned long long nza = a.mf.nz_ax, nzb = a.mf.nz_aty;

    // ------------------------------------------------------------------ columns
    double x[KC], aty[KC], lo[KC], hi[KC], ip[KC], tip[KC], ctip[KC], xsum[KC];
    double prox_const = 0.0, c2 = 0.0, cs2 = 0.0;
    {
        const long sn = (long)s * a.n, sN = (long)s * a.N;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            seq();
            const int j = colof(k);
            x[k] = aty[k] = lo[k] = hi[k] = xsum[k] = 0.0;
            double cs = 0.0, qs = 0.0;
            CS(CI::IDC + k) = 0.0;
            if (j < a.n) {
                const long b = sn + j;
                const double d = a.dc[b];
                double cc = a.c[b], qq = 0.0;
                double lo_ = a.cl[b], hi_ = a.cu[b];
                const int kk = col_nonant[j];
                if (kk >= 0) {
                    const long t = sN + kk;
                    ph_terms(a, t, kk, cc, qq, prox_const);
                    if (a.fix_nonants) fixed_box(a, t, d, lo_, hi_);
                }
                c2 += cc * cc;
                CS(CI::IDC + k) = 1.0 / d;
                cs = cc * d;
                qs = qq * d * d;
                lo[k] = lo_;
                hi[k] = hi_;
                x[k] = clampd((a.warm & 1) ? a.xs_in[b] : 0.0, lo_, hi_);
            }
            cs2 += cs * cs;
            CS(CI::XR + k) = x[k];
            CS(CI::Q + k) = qs;
            CS(CI::C + k) = cs;
        }
    }
    // ------------------------------------------------------------------ rows
    double y[KR], ax[KR], rlo[KR], rhi[KR], ysum[KR];
    double b2 = 0.0;
    {
        const long sm = (long)s * a.m;
#pragma unroll
        for (int r = 0; r < KR; ++r) {
            seq();
            const int i = rowof(r);
            y[r] = ax[r] = rlo[r] = rhi[r] = ysum[r] = 0.0;
            CS(CI::IDR + r) = 0.0;
            if (i < a.m) {
                const long b = sm + i;
                CS(CI::IDR + r) = 1.0 / a.dr[b];
                row_bounds(a, i, b, rlo[r], rhi[r]);
                double yy = (a.warm & 1) ? a.ys_in[b] : 0.0;
                if (!fin(rlo[r])) yy = fmin(yy, 0.0); else b2 += rlo[r] * rlo[r];
                if (!fin(rhi[r])) yy = fmax(yy, 0.0); else b2 += rhi[r] * rhi[r];
                y[r] = yy;
            }
            CS(CI::YR + r) = y[r];
            CS(CI::BLO + r) = rlo[r];
            CS(CI::BHI + r) = rhi[r];
        }
    }

    // ------------------------------------------------------------------ products (MFMA)
    auto mv_ax = [&](const double (&xx)[KC], double (&o)[KR]) {
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int u = 0; u < TN; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int f = (t * TN + u) * 4 + j;
                    if ((nza >> f) & 1ull) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[f], xx[u * 4 + j], acc, 0, 0, 0);
                }
#pragma unroll
            for (int j = 0; j < 4; ++j) o[t * 4 + j] = acc[j];
        }
    };
    auto mv_aty = [&](const double (&yy)[KR], double (&o)[KC]) {
#pragma unroll
        for (int u = 0; u < TN; ++u) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int t = 0; t < TM; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int f = (u * TM + t) * 4 + j;
                    if ((nzb >> f) & 1ull) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[f], yy[t * 4 + j], acc, 0, 0, 0);
                }
#pragma unroll
            for (int j = 0; j < 4; ++j) o[u * 4 + j] = acc[j];
        }
    };

    // ------------------------------------------------------------------ scalars
    double omega;
    {
        double rr[4] = {c2, prox_const, cs2, b2};
        ssum_many<4>(rr);
        SS(CI::CNORM) = sqrt(rr[0]);
        SS(CI::PROX) = rr[1];
        SS(CI::KOFF) = a.gap_const ? a.obj_off[s] + (a.prox_on ? rr[1] : 0.0) : 0.0;
        const double cn = sqrt(rr[2]), bn = sqrt(rr[3]);
        omega = (cn > 1e-10 && bn > 1e-10) ? cn / bn : 1.0;
        if ((a.warm & 2) && a.omega_in[s] > 0.0) omega = a.omega_in[s];
        else if ((a.warm & 4) && a.omega_in[s] > 0.0) omega = sqrt(omega * a.omega_in[s]);
    }
    const double eta = a.eta[s];
    SS(CI::BNORM) = a.bnorm[s];
    SS(CI::ETA) = eta;
    {
        const double tp = a.eps * (1.0 + a.bnorm[s]), td = a.eps * (1.0 + SS(CI::CNORM));
        SS(CI::TP) = tp * tp;
        SS(CI::TD) = td * td;
    }
    double tau = eta / omega, sig = eta * omega;
    auto rescale_bounds = [&]() {
#pragma unroll
        for (int r = 0; r < KR; ++r) { rlo[r] = -sig * CS(CI::BLO + r); rhi[r] = -sig * CS(CI::BHI + r); }
    };
    auto step_coefs = [&]() {
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            ip[k] = 1.0 / (1.0 + tau * CS(CI::Q + k));
            tip[k] = tau * ip[k];
            ctip[k] = CS(CI::C + k) * tip[k];
        }
    };
    rescale_bounds();
    step_coefs();
    mv_ax(x, ax);
    mv_aty(y, aty);

    // KKT pieces of an iterate (see pdhg_local.hip): [0] restart metric w/o gap, [2] ||pr||^2,
    // [3] ||dres||^2 (unscaled), [4] primal objective, [5] dual objective; padded slots are zeros
    auto kkt_part = [&](auto xf, auto atf, auto yf, auto axf, double* t) {
#pragma unroll
        for (int u = 0; u < 6; ++u) t[u] = 0.0;
        double pr2 = 0.0, dr2 = 0.0;
#pragma unroll
        for (int r = 0; r < KR; ++r) {
            seq();
            const double axx = axf(r), yy = yf(r);
            const double bl = CS(CI::BLO + r), bu = CS(CI::BHI + r);
            const double pr = axx - clampd(axx, bl, bu);
            pr2 += pr * pr;
            const double pu = pr * CS(CI::IDR + r);
            t[2] += pu * pu;
            if (fin(bl)) t[5] += bl * fmax(yy, 0.0);
            if (fin(bu)) t[5] += bu * fmin(yy, 0.0);
        }
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            seq();
            const double xx = xf(k);
            const double qk = CS(CI::Q + k);
            const double ck = CS(CI::C + k);
            const double rc_ = ck + qk * xx - atf(k);
            double dres = 0.0;
            if (!fin(lo[k]) && rc_ > 0.0) dres += rc_;
            if (!fin(hi[k]) && rc_ < 0.0) dres += rc_;
            dr2 += dres * dres;
            const double du = dres * CS(CI::IDC + k);
            t[3] += du * du;
            const double hq = 0.5 * qk * xx * xx;
            t[4] += ck * xx + hq;
            if (fin(lo[k])) t[5] += lo[k] * fmax(rc_, 0.0);
            if (fin(hi[k])) t[5] += hi[k] * fmin(rc_, 0.0);
            t[5] -= hq;
        }
        t[0] = fma(SS(CI::W2), pr2, dr2 * SS(CI::IW2));
    };
    auto kkt_both = [&](bool avg, double inv, double* oc, double* oa) {
        double t[12];
        kkt_part([&](int k) { return x[k]; }, [&](int k) { return aty[k]; }, [&](int r) { return y[r]; },
                 [&](int r) { return ax[r]; }, t);
        if (avg) {
            double axa[KR], ata[KC];
            mv_ax(xsum, axa);
            mv_aty(ysum, ata);
            kkt_part([&](int k) { return xsum[k] * inv; }, [&](int k) { return ata[k] * inv; },
                     [&](int r) { return ysum[r] * inv; }, [&](int r) { return axa[r] * inv; }, t + 6);
            ssum_many<12>(t);
        } else {
            ssum_many<6>(*reinterpret_cast<double(*)[6]>(t));
        }
#pragma unroll
        for (int u = 0; u < 6; ++u) oc[u] = t[u];
        if (avg)
#pragma unroll
            for (int u = 0; u < 6; ++u) oa[u] = t[6 + u];
    };
    auto rel_of = [&](const double* o) {
        const double p = sqrt(o[2]) / (1.0 + SS(CI::BNORM));
        const double d = sqrt(o[3]) / (1.0 + SS(CI::CNORM));
        const double gg = fabs(o[4] - o[5]) / gap_den(o[4], o[5], SS(CI::KOFF));
        return fmax(fmax(p, d), gg);
    };
    auto converged = [&](const double* o) {
        return o[2] <= SS(CI::TP) && o[3] <= SS(CI::TD) &&
               fabs(o[4] - o[5]) <= a.eps * gap_den(o[4], o[5], SS(CI::KOFF));
    };
    auto wkkt2_of = [&](const double* o) {
        const double gg = o[4] - o[5];
        return fma(gg, gg, o[0]);
    };

    SS(CI::OMEGA) = omega;
    SS(CI::W2) = omega * omega;
    SS(CI::IW2) = 1.0 / (omega * omega);
    {
        double o[6];
        kkt_both(false, 0.0, o, o);
        SS(CI::KRST) = wkkt2_of(o);
        SS(CI::KPREV) = INFINITY;
    }
    int it = 0, since = 0, cnt = 0;
    bool live = true;
    const int chk = a.check_every;

    auto finish = [&](bool use_avg, double inv, double rel, double pobj, double dobj, int st) {
        if (!valid) return;
        const int sl = launder(s);
        const long sn = (long)sl * a.n, sm = (long)sl * a.m, sN = (long)sl * a.N;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            seq();
            const int j = colof(k);
            if (j < a.n) {
                const long b = sn + j;
                const double xv = use_avg ? xsum[k] * inv : x[k];
                a.xs[b] = xv;
                const double xu = xv * a.dc[b];
                if (a.x_out) a.x_out[b] = xu;
                const int kk = col_nonant[j];
                if (kk >= 0) a.xN[sN + kk] = xu;
            }
        }
#pragma unroll
        for (int r = 0; r < KR; ++r) {
            seq();
            const int i = rowof(r);
            if (i < a.m) {
                const long b = sm + i;
                const double yv = use_avg ? ysum[r] * inv : y[r];
                a.ys[b] = yv;
                if (a.y_out) a.y_out[b] = yv * a.dr[b];
            }
        }
        if (g == 0) {
            const double offs = a.obj_off[sl] + (a.prox_on ? SS(CI::PROX) : 0.0);
            a.omega[sl] = SS(CI::OMEGA);
            a.obj[sl] = a.sense * (pobj + offs);
            a.bound[sl] = a.sense * (dobj + offs);
            a.kkt[sl] = rel;
            a.iters[sl] = it;
            a.iters_acc[sl] += it;
            a.status[sl] = st;
        }
    };

    while (wave_any(live)) {
        auto step = [&]() {
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const double xn = vmin(vmax(fma(aty[k], tip[k], fma(x[k], ip[k], -ctip[k])), lo[k]), hi[k]);
                x[k] = xn;
                xsum[k] += xn;
            }
            double axn[KR];
            mv_ax(x, axn);
#pragma unroll
            for (int r = 0; r < KR; ++r) {
                const double gg = y[r] - sig * (2.0 * axn[r] - ax[r]);
                y[r] = gg - vmin(vmax(gg, rhi[r]), rlo[r]);
                ax[r] = axn[r];
                ysum[r] += y[r];
            }
            mv_aty(y, aty);
        };
#pragma unroll 1
        for (int kk = 0; kk < chk; kk += 2) {
            step();
            step();
        }
        it += chk;
        since += chk;
        cnt += chk;

        const double inv = 1.0 / (double)cnt;
        double oc[6], oa[6];
        kkt_both(true, inv, oc, oa);
        const bool nan = !(oc[2] + oc[3] + oc[4] + oc[5] == oc[2] + oc[3] + oc[4] + oc[5]);
        const bool ok_cur = converged(oc), ok_avg = converged(oa);
        const bool term = live && (nan || ok_cur || ok_avg);
        const bool cap = live && !term && it >= a.max_iter;
        if (term || cap) {
            const double rel_cur = rel_of(oc), rel_avg = rel_of(oa);
            const bool ua = !nan && rel_avg < rel_cur;
            finish(ua, inv, ua ? rel_avg : rel_cur, ua ? oa[4] : oc[4], ua ? oa[5] : oc[5],
                   nan ? 2 : (term ? 0 : 1));
            live = false;
        }
        if (!wave_any(live)) break;

        const double k_cur = wkkt2_of(oc), k_avg = wkkt2_of(oa);
        const bool use_avg = k_avg < k_cur;
        const double cand = use_avg ? k_avg : k_cur;
        const double krst = SS(CI::KRST);
        const bool restart = live && ((cand <= a.beta_suf * a.beta_suf * krst) ||
                                      (cand <= a.beta_nec * a.beta_nec * krst && cand > SS(CI::KPREV)) ||
                                      ((double)since >= a.beta_art * (double)it));
        if constexpr (WATCH) {
            if (live && valid && s == a.watch && g == 0)
                printf("PHG_WATCH s %d it %d since %d kc %.6e ka %.6e krst %.6e kprev %.6e rst %d ua %d om %.6e "
                       "pres2 %.6e dres2 %.6e tp %.3e td %.3e pobj %.15e dobj %.15e koff %.6e\n",
                       s, it, since, k_cur, k_avg, krst, SS(CI::KPREV), (int)restart, (int)use_avg, omega, oc[2], oc[3],
                       SS(CI::TP), SS(CI::TD), oc[4], oc[5], SS(CI::KOFF));
        }
        SS(CI::KPREV) = cand;
        if (wave_any(restart)) {
            const bool ra = restart && use_avg;
            if (wave_any(ra)) {
#pragma unroll
                for (int k = 0; k < KC; ++k) x[k] = ra ? xsum[k] * inv : x[k];
#pragma unroll
                for (int r = 0; r < KR; ++r) y[r] = ra ? ysum[r] * inv : y[r];
                // exact products at the new point (a wave-wide MFMA; scenarios that keep their
                // point recompute the same values)
                mv_ax(x, ax);
                mv_aty(y, aty);
            }
            double mv[2] = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < KC; ++k) { const double t = x[k] - CS(CI::XR + k); mv[0] += t * t; }
#pragma unroll
            for (int r = 0; r < KR; ++r) { const double t = y[r] - CS(CI::YR + r); mv[1] += t * t; }
            ssum_many<2>(mv);
            if (restart) {
                omega = primal_weight(SS(CI::OMEGA), mv[0], mv[1], a.theta);
                const double et = SS(CI::ETA);
                tau = et / omega;
                sig = et * omega;
                rescale_bounds();
                step_coefs();
#pragma unroll
                for (int k = 0; k < KC; ++k) { CS(CI::XR + k) = x[k]; xsum[k] = 0.0; }
#pragma unroll
                for (int r = 0; r < KR; ++r) { CS(CI::YR + r) = y[r]; ysum[r] = 0.0; }
                SS(CI::OMEGA) = omega;
                SS(CI::W2) = omega * omega;
                SS(CI::IW2) = 1.0 / (omega * omega);
                SS(CI::KRST) = cand;
                SS(CI::KPREV) = INFINITY;
                cnt = 0;
                since = 0;
            }
        }
    }
}

// ----------------------------------------------------------------------------- dispatch
struct MfmaVariant {
    int TM, TN;
    void (*fn)(PdhgArgs);
    void (*fn_watch)(PdhgArgs);
};

#define PHG_M(m_, n_) {m_, n_, pdhg_mfma_kernel<m_, n_, false>, pdhg_mfma_kernel<m_, n_, true>}
// smallest tile grid that holds (m, n) first
// one 16 x 16 tile: 224 VGPRs, no spills; the 16 x 32 / 32 x 16 grids spill 220-324 bytes per
// lane (8 TM TN fragments + 8 x 4 TN + 5 x 4 TM iterate values per lane), so they are left out
static const MfmaVariant kMfmaVariants[] = {
    PHG_M(1, 1),
};
#undef PHG_M

int pdhg_mfma_num_variants() { return (int)(sizeof(kMfmaVariants) / sizeof(kMfmaVariants[0])); }

void pdhg_mfma_variant_shape(int v, int* out2) {
    out2[0] = kMfmaVariants[v].TM;
    out2[1] = kMfmaVariants[v].TN;
}

size_t pdhg_mfma_lds_bytes(int v) {
    const MfmaVariant& V = kMfmaVariants[v];
    // per-lane vector items + per-scenario scalars (MCold): 17.4 KB for one tile, so LDS admits the
    // 2 waves per SIMD the registers allow (8 per CU; per-lane scalars made it 21.5 KB: 7 per CU)
    return ((size_t)(4 * 4 * V.TN + 4 * 4 * V.TM) * 64 + (size_t)MCold<1, 1>::NSC * 16) * sizeof(double);
}

hipError_t pdhg_mfma_launch(int v, const PdhgArgs& a, hipStream_t stream) {
    const MfmaVariant& V = kMfmaVariants[v];
    hipLaunchKernelGGL(a.watch >= 0 ? V.fn_watch : V.fn, dim3((a.S + 15) / 16), dim3(64), pdhg_mfma_lds_bytes(v), stream, a);
    return hipGetLastError();
}

}  // namespace phg
