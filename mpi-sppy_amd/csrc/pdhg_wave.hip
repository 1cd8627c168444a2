// pdhg_wave.hip -- batched PDHG with ONE WAVEFRONT PER SCENARIO for shared-matrix scenario LPs/QPs
// of a few hundred columns (gfx950).
//
// Same algorithm, restart rule and outputs as pdhg_block.hip (replaces SPOpt.solve_one,
// mpisppy/spopt.py:184-231, for every local scenario), for the batches whose constraint matrix is the
// same in every scenario -- sslp_15_45_10 (examples/sslp/model/ReferenceModel.py:77-78: only the
// client-presence right-hand sides vary; 705 x 60, 1 364 nonzeros).  The workgroup kernel solves one
// such scenario per 256-thread workgroup and pays three workgroup barriers per PDHG iteration for ~5 k
// flops; here:
//
//   * a workgroup of WPG waves solves WPG scenarios, one per wave, and the waves never wait for each
//     other after the prologue: every sum of a PDHG iteration is inside the wave (LDS traffic of one
//     wave is executed in order, so a compiler barrier orders it; no s_barrier in the loop);
//   * the scaled matrix -- the same for every scenario -- is held ONCE per workgroup in LDS, in piece
//     order: row pieces of <= 8 consecutive CSR entries ([slot][entry][lane]) for A x, and each
//     column's <= CE entries ([slot][lane][entry], one 16-byte read for CE = 2) for A^T y, which is
//     column-local (no partials);
//   * each lane owns CPL columns (x, running sum, scaled cost, box in registers) and RPL rows; the
//     wave's x and y sit in LDS for the gathers; q / 1 / (1 + tau q) exist only for the NSL column
//     slots that hold nonants (the engine's quadratic terms are the PH prox / smoothing terms, on
//     nonants only; the host puts the nonant columns into the first slots).
//
// The pieces and their summation order are those of the workgroup kernel's register-piece variant,
// so A x and A^T y return the same bits; the KKT reductions are wave sums (gsum<64>) instead of
// workgroup sums, so restart decisions can differ in the last bits of the norms.
#include "phg_internal.h"
#include "wave_ops.h"

namespace phg {

// orders a wave's LDS stores before its later loads (DS instructions of one wave execute in order:
// only the compiler must not move them)
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

template <int CPL, int RPL, int PPT, int CE, int NSL, int WPG>
__global__ __launch_bounds__(64 * WPG, 8 / WPG) void pdhg_wave_kernel(PdhgArgs a) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (PdhgArgs::gate)
    constexpr int RE = 8;
    constexpr int RMAX = 8;   // pieces per row (<= 64 entries; checked on the host)
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const WaveLayout& V = a.wv;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double* rvs = smem;                          // [PPT][RE][64] row-piece values (shared)
    double* cvs = rvs + PPT * RE * 64;           // [CPL][64][CE] column values (shared)
    int* xis = reinterpret_cast<int*>(cvs + CPL * 64 * CE);   // [PPT][RE][64] row-piece x positions (shared)
    int* cis = xis + PPT * RE * 64;              // [CPL][64][CE] column entry rows (shared)
    double* xl = reinterpret_cast<double*>(cis + CPL * 64 * CE) + (long)w * V.wave_doubles;   // [CPL*64] x by position
    double* yl = xl + V.n_pad;                   // [m_pad]
    double* rp = yl + V.m_pad;                   // [PPT*64] row-piece partials
    for (int e = threadIdx.x; e < PPT * RE * 64; e += 64 * WPG) rvs[e] = V.rvals[e];
    for (int e = threadIdx.x; e < CPL * 64 * CE; e += 64 * WPG) cvs[e] = V.cvals[e];
    for (int e = threadIdx.x; e < PPT * RE * 64; e += 64 * WPG) xis[e] = V.ridx[e];
    for (int e = threadIdx.x; e < CPL * 64 * CE; e += 64 * WPG) cis[e] = V.cidx[e];
    __syncthreads();   // the only workgroup barrier: the waves are independent from here on
    const int item = blockIdx.x * WPG + w;
    if (item >= a.S) return;
    const int s = a.order ? a.order[item] : item;
    const long sn = (long)s * a.n, sm = (long)s * a.m, sN = (long)s * a.N;

    // ------------------------------------------------------------------ columns owned
    double x[CPL], c[CPL], lo[CPL], hi[CPL], xsum[CPL];
    double q[NSL > 0 ? NSL : 1], ip[NSL > 0 ? NSL : 1];
    double prox_const = 0.0, c2 = 0.0;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int j = V.col_of[k * 64 + lane];
        x[k] = c[k] = lo[k] = hi[k] = xsum[k] = 0.0;
        if (k < NSL) q[k] = 0.0;
        if (j >= 0) {
            const long b = sn + j;
            const double d = a.dc[b];
            double cc = a.c[b], qq = 0.0;
            double lo_ = a.cl[b], hi_ = a.cu[b];
            const int kk = a.lay.col_nonant[j];
            if (kk >= 0) {   // (the host placed every nonant into a slot k < NSL)
                const long tt = sN + kk;
                ph_terms(a, tt, kk, cc, qq, prox_const);
                if (a.fix_nonants) fixed_box(a, tt, d, lo_, hi_);
            }
            c2 += cc * cc;
            c[k] = cc * d;
            if (k < NSL) q[k] = qq * d * d;
            lo[k] = lo_;
            hi[k] = hi_;
            x[k] = clampd((a.warm & 1) ? a.xs_in[b] : 0.0, lo_, hi_);
            a.xs[b] = x[k];
        }
    }
    // ------------------------------------------------------------------ rows owned
    int ri[RPL], rf[RPL], rn[RPL];
    double y[RPL], ax[RPL], rlo[RPL], rhi[RPL], ysum[RPL];
    double b2 = 0.0;
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
        const int i = V.row_of[r * 64 + lane];
        ri[r] = i;
        rf[r] = V.row_pfirst[r * 64 + lane];
        rn[r] = V.row_pcnt[r * 64 + lane];
        y[r] = ax[r] = rlo[r] = rhi[r] = ysum[r] = 0.0;
        if (i >= 0) {
            const long b = sm + i;
            row_bounds(a, i, b, rlo[r], rhi[r]);
            double yy = (a.warm & 1) ? a.ys_in[b] : 0.0;
            if (!fin(rlo[r])) yy = fmin(yy, 0.0); else b2 += rlo[r] * rlo[r];
            if (!fin(rhi[r])) yy = fmax(yy, 0.0); else b2 += rhi[r] * rhi[r];
            y[r] = yy;
            a.ys[b] = yy;
        }
    }

    // ------------------------------------------------------------------ products through LDS
    auto put_x = [&](auto f) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) xl[k * 64 + lane] = f(k);   // (empty positions hold 0)
    };
    auto cur_x = [&](int k) { return x[k]; };
    auto put_y = [&](const double (&v)[RPL]) {
#pragma unroll
        for (int r = 0; r < RPL; ++r)
            if (ri[r] >= 0) yl[ri[r]] = v[r];
    };
    // column k of A^T y for the y in yl (the workgroup kernel's column-local order: entries in CSC
    // order from 0)
    auto aty_col = [&](int k) {
        double acc = 0.0;
#pragma unroll
        for (int e = 0; e < CE; ++e) acc = fma(cvs[(k * 64 + lane) * CE + e], yl[cis[(k * 64 + lane) * CE + e]], acc);
        return acc;
    };
    // A x for the x in xl: pieces -> rp, then row owners add their pieces left to right
    auto spmv_ax = [&](double (&out)[RPL]) {
#pragma unroll
        for (int ps = 0; ps < PPT; ++ps) {
            double acc = 0.0;
#pragma unroll
            for (int e = 0; e < RE; ++e) acc = fma(rvs[(ps * RE + e) * 64 + lane], xl[xis[(ps * RE + e) * 64 + lane]], acc);
            rp[ps * 64 + lane] = acc;
        }
        wsync();
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            double pv[RMAX];
#pragma unroll
            for (int u = 0; u < RMAX; ++u) pv[u] = u < rn[r] ? rp[rf[r] + u] : 0.0;
            double t = 0.0;
#pragma unroll
            for (int u = 0; u < RMAX; ++u) t += pv[u];   // (+0.0 past the row's pieces: the same sum)
            out[r] = t;
        }
        wsync();   // partials consumed before the next pieces overwrite them
    };

    // ------------------------------------------------------------------ scalars
    double omega, cnorm;
    {
        double rr[4] = {c2, prox_const, 0.0, b2};
#pragma unroll
        for (int k = 0; k < CPL; ++k) rr[2] += c[k] * c[k];
        gsum_many<64, 4>(rr);
        cnorm = sqrt(rr[0]);
        prox_const = rr[1];
        const double cn_ = sqrt(rr[2]), bn = sqrt(rr[3]);
        omega = (cn_ > 1e-10 && bn > 1e-10) ? cn_ / bn : 1.0;
        if ((a.warm & 2) && a.omega_in[s] > 0.0) omega = a.omega_in[s];
        else if ((a.warm & 4) && a.omega_in[s] > 0.0) omega = sqrt(omega * a.omega_in[s]);
    }
    const double bnorm = a.bnorm[s];
    const double eta = a.eta[s];
    double tau = eta / omega, sig = eta * omega;
#pragma unroll
    for (int k = 0; k < NSL; ++k) ip[k] = 1.0 / (1.0 + tau * q[k]);
    put_x(cur_x);
    put_y(y);
    wsync();
    spmv_ax(ax);

    // KKT pieces of one iterate (see pdhg_block.hip), reduced over the wave; the iterate's A^T y is
    // formed column by column from the y in yl (at), its A x given (axx)
    auto kkt = [&](auto xf, const double (&yy)[RPL], const double (&axx)[RPL], double* o) {
        double v[6] = {0, 0, 0, 0, 0, 0};
        const int sl = launder(s);
        const long sn_ = (long)sl * a.n, sm_ = (long)sl * a.m;
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            seq();
            if (ri[r] >= 0) {
                const double pr = axx[r] - clampd(axx[r], rlo[r], rhi[r]);
                v[0] += pr * pr;
                const double pu = pr / a.dr[sm_ + ri[r]];
                v[2] += pu * pu;
                if (fin(rlo[r])) v[5] += rlo[r] * fmax(yy[r], 0.0);
                if (fin(rhi[r])) v[5] += rhi[r] * fmin(yy[r], 0.0);
            }
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            seq();
            const int j = launder(V.col_of[k * 64 + lane]);
            if (j >= 0) {
                const double xx = xf(k), qk = k < NSL ? q[k < NSL ? k : 0] : 0.0;
                const double rc_ = c[k] + qk * xx - aty_col(k);
                double dres = 0.0;
                if (!fin(lo[k]) && rc_ > 0.0) dres += rc_;
                if (!fin(hi[k]) && rc_ < 0.0) dres += rc_;
                v[1] += dres * dres;
                const double du = dres / a.dc[sn_ + j];
                v[3] += du * du;
                v[4] += c[k] * xx + 0.5 * qk * xx * xx;
                if (fin(lo[k])) v[5] += lo[k] * fmax(rc_, 0.0);
                if (fin(hi[k])) v[5] += hi[k] * fmin(rc_, 0.0);
                v[5] -= 0.5 * qk * xx * xx;
            }
        }
        gsum_many<64, 6>(v);
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
    auto wkkt_of = [&](const double* o, double om) {
        const double g = o[4] - o[5];
        return sqrt(om * om * o[0] + o[1] / (om * om) + g * g);
    };

    double kkt_restart, kkt_prev = INFINITY;
    {
        double o[6];
        kkt([&](int k) { return x[k]; }, y, ax, o);
        kkt_restart = wkkt_of(o, omega);
    }
    int it = 0, since = 0, cnt = 0, st = 1;
    double rel_final = INFINITY, pobj = 0.0, dobj = 0.0;
    bool use_avg_final = false;
    const int chk = a.check_every;

    while (true) {
#pragma unroll 1
        for (int kk = 0; kk < chk; ++kk) {
            // primal step (A^T y of the y in yl, formed per column)
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const double g = fma(tau, aty_col(k) - c[k], x[k]);
                // raw v_max / v_min: no NaN canonicalisation of the loop-invariant bounds (wave_ops.h)
                const double xn = vmin(vmax(k < NSL ? g * ip[k < NSL ? k : 0] : g, lo[k]), hi[k]);
                x[k] = xn;
                xsum[k] += xn;
            }
            put_x(cur_x);
            wsync();
            double axn[RPL];
            spmv_ax(axn);
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
                const double g = y[r] - sig * (2.0 * axn[r] - ax[r]);
                y[r] = fmax(fma(sig, rlo[r], g), 0.0) + fmin(fma(sig, rhi[r], g), 0.0);   // 0 on empty slots
                ax[r] = axn[r];
                ysum[r] += y[r];
            }
            put_y(y);
            wsync();
        }
        it += chk;
        since += chk;
        cnt += chk;

        // ---------------------------------------------------------- restart / termination check
        const double inv = 1.0 / (double)cnt;
        double oc[6], oa[6];
        kkt([&](int k) { return x[k]; }, y, ax, oc);
        {   // the average iterate (every check, as the workgroup kernel): its products through LDS
            double ya[RPL], axa[RPL];
#pragma unroll
            for (int r = 0; r < RPL; ++r) ya[r] = ysum[r] * inv;
            put_x([&](int k) { return xsum[k] * inv; });
            put_y(ya);
            wsync();
            spmv_ax(axa);
            kkt([&](int k) { return xsum[k] * inv; }, ya, axa, oa);
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
            if (use_avg) {
#pragma unroll
                for (int k = 0; k < CPL; ++k) x[k] = xsum[k] * inv;
#pragma unroll
                for (int r = 0; r < RPL; ++r) y[r] = ysum[r] * inv;
            }
            double mv[2] = {0.0, 0.0};
            {
                const int sl = launder(s);
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    seq();
                    const int j = launder(V.col_of[k * 64 + lane]);
                    if (j >= 0) {
                        const long b = (long)sl * a.n + j;
                        const double d = x[k] - a.xs[b];
                        mv[0] += d * d;
                        a.xs[b] = x[k];
                    }
                }
#pragma unroll
                for (int r = 0; r < RPL; ++r) {
                    seq();
                    if (ri[r] >= 0) {
                        const long b = (long)sl * a.m + ri[r];
                        const double d = y[r] - a.ys[b];
                        mv[1] += d * d;
                        a.ys[b] = y[r];
                    }
                }
            }
            gsum_many<64, 2>(mv);
            omega = primal_weight(omega, mv[0], mv[1], a.theta);
            tau = eta / omega;
            sig = eta * omega;
#pragma unroll
            for (int k = 0; k < NSL; ++k) ip[k] = 1.0 / (1.0 + tau * q[k]);
#pragma unroll
            for (int k = 0; k < CPL; ++k) xsum[k] = 0.0;
#pragma unroll
            for (int r = 0; r < RPL; ++r) ysum[r] = 0.0;
            cnt = 0;
            since = 0;
            kkt_restart = cand;
            kkt_prev = INFINITY;
        }
        // x, y back into LDS (the average's products used it); A x of the point the iteration
        // continues from: recomputed after a restart to the average, else still in ax
        put_x(cur_x);
        put_y(y);
        wsync();
        if (restart && use_avg) spmv_ax(ax);
    }

    // ------------------------------------------------------------------ outputs
    const double inv = cnt > 0 ? 1.0 / (double)cnt : 0.0;
    const double offs = a.obj_off[s] + (a.prox_on ? prox_const : 0.0);
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int j = V.col_of[k * 64 + lane];
        if (j >= 0) {
            const long b = sn + j;
            const double xv = use_avg_final ? xsum[k] * inv : x[k];
            a.xs[b] = xv;
            const double xu = xv * a.dc[b];
            if (a.x_out) a.x_out[b] = xu;
            const int kk = a.lay.col_nonant[j];
            if (kk >= 0) a.xN[sN + kk] = xu;
        }
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
        if (ri[r] >= 0) {
            const long b = sm + ri[r];
            const double yv = use_avg_final ? ysum[r] * inv : y[r];
            a.ys[b] = yv;
            if (a.y_out) a.y_out[b] = yv * a.dr[b];
        }
    }
    if (lane == 0) {
        a.omega[s] = omega;
        a.obj[s] = a.sense * (pobj + offs);
        a.bound[s] = a.sense * (dobj + offs);
        a.kkt[s] = rel_final;
        a.iters[s] = it;
        a.iters_acc[s] += it;
        a.status[s] = st;
    }
}

// ----------------------------------------------------------------------------- dispatch
struct WaveVariant {
    int CPL, RPL, PPT, CE, NSL, WPG;
    void (*fn)(PdhgArgs);
};
#define PHG_W(a_, b_, c_, d_, e_, f_) {a_, b_, c_, d_, e_, f_, pdhg_wave_kernel<a_, b_, c_, d_, e_, f_>}
// preference order: fewest column slots first
static const WaveVariant kWaveVariants[] = {
    PHG_W(12, 1, 3, 2, 1, 4),    // sslp_15_45_10: 705 columns (15 nonants), 60 rows, 180 row pieces
    PHG_W(16, 1, 4, 2, 1, 4),    // <= 1024 columns, 64 rows, 256 row pieces
};
#undef PHG_W

int pdhg_wave_num_variants() { return (int)(sizeof(kWaveVariants) / sizeof(kWaveVariants[0])); }

void pdhg_wave_variant_shape(int v, int* out6) {
    const WaveVariant& V = kWaveVariants[v];
    out6[0] = V.CPL; out6[1] = V.RPL; out6[2] = V.PPT; out6[3] = V.CE; out6[4] = V.NSL; out6[5] = V.WPG;
}

size_t pdhg_wave_lds_bytes(int v, int wave_doubles) {
    const WaveVariant& V = kWaveVariants[v];
    const size_t ent = (size_t)V.PPT * 8 * 64 + (size_t)V.CPL * 64 * V.CE;   // values (double) + indices (int)
    return ent * (sizeof(double) + sizeof(int)) + (size_t)V.WPG * wave_doubles * sizeof(double);
}

hipError_t pdhg_wave_launch(int v, const PdhgArgs& a, hipStream_t stream) {
    const WaveVariant& V = kWaveVariants[v];
    const size_t lds = pdhg_wave_lds_bytes(v, a.wv.wave_doubles);
    hipLaunchKernelGGL(V.fn, dim3((a.S + V.WPG - 1) / V.WPG), dim3(64 * V.WPG), lds, stream, a);
    return hipGetLastError();
}

}  // namespace phg
