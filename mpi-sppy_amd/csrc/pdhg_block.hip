// pdhg_block.hip -- batched PDHG for scenario LPs/QPs too large for one wavefront (gfx950).
//
// Same algorithm, restart rule and outputs as pdhg.hip / pdhg_local.hip (replaces
// SPOpt.solve_one, mpisppy/spopt.py:184-231, for every local scenario), mapped for n, m in the
// hundreds to thousands (sslp: 705 x 60, netdes: 2940 x 1520):
//
//   * one workgroup of NT = 256 / 512 / 1024 threads per scenario; the iterates x, y and the
//     SpMV partial sums live in LDS, per-column / per-row state in registers (CPL / RPL slots);
//   * A x and A^T y are CSR / CSC SpMVs over "pieces" of <= 8 consecutive entries of a row /
//     column.  Piece p belongs to thread p % NT (slot p / NT); its values are STREAMED from memory
//     every iteration in a piece-major layout [slot][entry][thread], so a wave's loads are
//     coalesced 512-byte rows (the HBM-bound streaming path of SURVEY 8(d)1); when every scenario
//     has the same matrix the layout is stored once and served from L2 / MALL;
//   * a row's pieces are consecutive, so the row owner adds its pieces' partials from LDS in a
//     fixed order (deterministic, no atomics); four workgroup barriers per PDHG iteration.
#include "phg_internal.h"
#include "wave_ops.h"

namespace phg {

// workgroup all-reduce of K <= 16 values: DPP wave sums, wave partials to LDS, thread k adds value
// k's NT/64 partials in wave order, every thread reads the K totals back (same bits everywhere)
template <int NT, int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double* red) {
    constexpr int NW = NT / 64;
    static_assert(K <= 16, "block_sum scratch holds 16 values");
    gsum_many<64, K>(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[k * NW + w] = v[k];
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        double t = red[k * NW];
#pragma unroll 1
        for (int u = 1; u < NW; ++u) t += red[k * NW + u];
        red[16 * NW + k] = t;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = red[16 * NW + k];
}

// sum of a row's (column's) cnt piece partials, left to right (the owner's fixed order).  (Issuing
// the loads four at a time with predicated tails measured slower on sslp: 12.0 -> 15.2 ms.)
__device__ __forceinline__ double piece_sum(const double* p, int cnt) {
    double acc = 0.0;
#pragma unroll 1
    for (int u = 0; u < cnt; ++u) acc += p[u];
    return acc;
}
// the same sum with the (<= 8) partials' loads issued together, added in the same order (PS
// variants; + 0.0 past the row's pieces leaves the sum unchanged)
__device__ __forceinline__ double piece_sum8(const double* p, int cnt) {
    if (cnt > 8) return piece_sum(p, cnt);
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = u < cnt ? p[u] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
    return acc;
}

// RE / CE > 0: every row (column) piece slot holds at most RE (CE) entries, and the thread's piece
// values and LDS indices are loaded into registers once, in the prologue -- the matrix is constant
// over the solve, so the iterations read only LDS (x, y, partials).  RE = CE = 0: values and
// indices are re-read from memory every iteration (the streaming form, for pieces that do not fit
// the register budget).  Both forms add the same products in the same order (padding entries are
// fma(0, x[0], acc) = acc), so they return the same bits.
//
// CL: every column is ONE piece, held by the thread and slot that own the column (QPT == CPL;
// checked on the host) -- so A^T y needs no partials in LDS and no workgroup barrier: three
// barriers per PDHG iteration instead of four (sslp: every column has <= 2 entries; netdes <= 3).
//
// VS: the delta value form (BlockLayout::vscale) -- the pieces hold unscaled values and the scenario's
// scaling is applied on the fly: x and y enter the LDS as dc x and dr y, A x leaves as dr (A (dc x)),
// A^T y as dc (A^T (dr y)).
//
// UN: the unit form (BlockLayout::rcode) -- VS with every constant entry +-1: the entry codes and the
// scenario's varying entry rows sit in LDS; an entry fma's its x (y) with +-1 built from the code's
// sign bit or, on a varying row, with its value -- the delta form's products, bit for bit.
//
// SEG = 8 / 16: the row-segment form (BlockLayout built by build_block_layout's segment planner) --
// every row's pieces sit in an aligned segment of 1, 2, 4, 8 (or 16) consecutive lanes of one wave,
// in the piece slot of the row's own slot (PPT == RPL; row_pcnt = the segment length, the row owned
// by the segment's first lane), so a row sum is a DPP butterfly over its segment inside the wave: no
// partials in LDS and no workgroup barrier between the pieces and the row owners -- two barriers per
// PDHG iteration instead of three.  The segment sums add the pieces pairwise ((p0 + p1) + (p2 +
// p3)) + ..., a different order from the sequential piece_sum.
template <int NT, int CPL, int RPL, int PPT, int QPT, int RE, int CE, bool CL, bool VS, bool PS = false,
          bool UN = false, int SEG = 0>
__global__ __launch_bounds__(NT) void pdhg_block_kernel(PdhgArgs a) {
    static_assert(!CL || QPT == CPL, "column-local A^T y needs one piece slot per column slot");
    static_assert(SEG == 0 || ((SEG == 8 || SEG == 16) && PPT == RPL), "row segments: piece slot r holds row slot r's rows");
    static_assert(!UN || (VS && RE == 0 && CE == 0), "the unit form is a streaming delta-form variant");
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (PdhgArgs::gate)
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const BlockLayout& B = a.blk;
    const int t = threadIdx.x;
    const int s = a.order ? a.order[blockIdx.x] : blockIdx.x;
    double* xl = smem;                   // [n_pad]
    double* yl = xl + B.n_pad;           // [m_pad]
    double* zl = yl + B.m_pad;           // [2] zl[0] = 0.0: the unit form's padding entries read it
    double* rp = zl + 2;                 // [PPT*NT] row-piece partials
    double* cp = rp + PPT * NT;          // [QPT*NT] column-piece partials
    double* red = cp + QPT * NT;         // [16 * (NT/64 + 1)] reduction scratch
    const long sn = (long)s * a.n, sm = (long)s * a.m, sN = (long)s * a.N;
    const double* rv = B.rvals + (long)s * B.vstride_r;
    const double* cv = B.cvals + (long)s * B.vstride_c;
    // delta form (BlockLayout::rdrow): entry rows with a varying entry come from the scenario's blocks
    const double* rvd = B.rvd ? B.rvd + (long)s * B.dstride_r : nullptr;
    const double* cvd = B.cvd ? B.cvd + (long)s * B.dstride_c : nullptr;
    // value of piece entry e (entry row R = e / NT, uniform over the workgroup)
    auto rval = [&](int e, int R) {
        const int d = B.rdrow[R];
        return d >= 0 ? rvd[(long)d * NT + t] : rv[e];
    };
    auto cval = [&](int e, int R) {
        const int d = B.cdrow[R];
        return d >= 0 ? cvd[(long)d * NT + t] : cv[e];
    };
    // UN: the scenario's varying entry rows [nd_r + nd_c][NT] and the codes [er + ec] in LDS.  Every
    // thread reads back only its own entries (e % NT == t), so no barrier is needed before use.
    double* dl = red + 16 * (NT / 64 + 1);
    short* codes = reinterpret_cast<short*>(dl + (UN ? (B.nd_r + B.nd_c) * NT : 0));
    if constexpr (UN) {
        for (int i = t; i < B.nd_r * NT; i += NT) dl[i] = rvd[i];
        for (int i = t; i < B.nd_c * NT; i += NT) dl[B.nd_r * NT + i] = cvd[i];
        for (int i = t; i < B.er; i += NT) codes[i] = B.rcode[i];
        for (int i = t; i < B.ec; i += NT) codes[B.er + i] = B.ccode[i];
    }
    // UN product of code cd (entry row with varying-row index d) with the LDS vector v
    // (code = LDS byte address of the x / y element, bit 0 the value's sign; padding: zl)
    if constexpr (UN) {
        if (t == 0) zl[0] = 0.0;   // read after the first products() barrier
    }
    // the varying entry rows as bit masks (their block index = the set bits below them, as
    // build_block_values numbers them): uniform scalar arithmetic instead of a kernarg load per entry row
    unsigned rdm = 0, cdm = 0;
    if constexpr (UN) {
#pragma unroll
        for (int R = 0; R < 32; ++R) {
            rdm |= B.rdrow[R] >= 0 ? 1u << R : 0u;
            cdm |= B.cdrow[R] >= 0 ? 1u << R : 0u;
        }
    }
    auto drow_of = [](unsigned msk, int R) {
        return (msk >> R) & 1u ? __builtin_popcount(msk & ((1u << R) - 1u)) : -1;
    };
    auto unit_fma = [&](int cd, int d, int drow0, double acc, int tq) {
        const unsigned cu = (unsigned)(unsigned short)cd;
        const double v = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(smem) + (cu & 0xFFF8u));
        if (d >= 0) return fma(dl[(drow0 + d) * NT + tq], v, acc);
        // +-1.0 built from the sign bit: fma(+-1, v, acc), the delta form's bits
        return fma(__hiloint2double((int)(0x3FF00000u | (cu << 31)), 0), v, acc);
    };

    // ------------------------------------------------------------------ columns owned
    int cj[CPL], cf[CPL], cn[CPL];
    // restart reference points live in the xs / ys state arrays (each thread reads back only the
    // elements it wrote), not in registers
    double x[CPL], aty[CPL], c[CPL], q[CPL], lo[CPL], hi[CPL], ip[CPL], xsum[CPL];
    double dcs[VS ? CPL : 1], drs[VS ? RPL : 1];   // VS: the scenario's column / row scaling
    double prox_const = 0.0, c2 = 0.0;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int j = B.col_of[k * NT + t];
        cj[k] = j;
        cf[k] = B.col_pfirst[k * NT + t];
        cn[k] = B.col_pcnt[k * NT + t];
        x[k] = aty[k] = c[k] = q[k] = lo[k] = hi[k] = xsum[k] = 0.0;
        if constexpr (VS) dcs[k] = 0.0;
        if (j >= 0) {
            const long b = sn + j;
            const double d = a.dc[b];
            if constexpr (VS) dcs[k] = d;
            double cc = a.c[b], qq = 0.0;
            double lo_ = a.cl[b], hi_ = a.cu[b];
            const int kk = a.lay.col_nonant[j];
            if (kk >= 0) {
                const long tt = sN + kk;
                ph_terms(a, tt, kk, cc, qq, prox_const);
                if (a.fix_nonants) fixed_box(a, tt, d, lo_, hi_);
            }
            c2 += cc * cc;
            c[k] = cc * d;
            q[k] = qq * d * d;
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
        const int i = B.row_of[r * NT + t];
        ri[r] = i;
        rf[r] = B.row_pfirst[r * NT + t];
        rn[r] = B.row_pcnt[r * NT + t];
        y[r] = ax[r] = rlo[r] = rhi[r] = ysum[r] = 0.0;
        if constexpr (VS) drs[r] = 0.0;
        if (i >= 0) {
            const long b = sm + i;
            if constexpr (VS) drs[r] = a.dr[b];
            row_bounds(a, i, b, rlo[r], rhi[r]);
            double yy = (a.warm & 1) ? a.ys_in[b] : 0.0;
            if (!fin(rlo[r])) yy = fmin(yy, 0.0); else b2 += rlo[r] * rlo[r];
            if (!fin(rhi[r])) yy = fmax(yy, 0.0); else b2 += rhi[r] * rhi[r];
            y[r] = yy;
            a.ys[b] = yy;
        }
    }

    // ------------------------------------------------------------------ register-resident pieces
    constexpr int RE1 = RE > 0 ? RE : 1, CE1 = CE > 0 ? CE : 1;
    double rvr[RE > 0 ? PPT : 1][RE1], cvr[CE > 0 ? QPT : 1][CE1];
    int rir[RE > 0 ? PPT : 1][RE1], cir[CE > 0 ? QPT : 1][CE1];
    if constexpr (RE > 0) {
        int off = 0;
#pragma unroll
        for (int ps = 0; ps < PPT; ++ps) {
            const int kk = B.rk[ps];
#pragma unroll
            for (int k = 0; k < RE; ++k) {
                const int e = off + k * NT + t;
                rvr[ps][k] = k < kk ? rval(e, off / NT + k) : 0.0;
                rir[ps][k] = k < kk ? B.ridx[e] : 0;
            }
            off += kk * NT;
        }
    }
    if constexpr (CE > 0) {
        int off = 0;
#pragma unroll
        for (int ps = 0; ps < QPT; ++ps) {
            const int kk = B.ck[ps];
#pragma unroll
            for (int k = 0; k < CE; ++k) {
                const int e = off + k * NT + t;
                cvr[ps][k] = k < kk ? cval(e, off / NT + k) : 0.0;
                cir[ps][k] = k < kk ? B.cidx[e] : 0;
            }
            off += kk * NT;
        }
    }

    // ------------------------------------------------------------------ SpMVs through LDS
    // A x for the x currently in xl: pieces -> rp, barrier, row owners add their pieces
    // tq: the thread index laundered at every product, so the per-thread LDS addresses of the pieces
    // are re-formed in the iteration (one add each) instead of being hoisted out of the PDHG loop --
    // held across it they spilled (netdes: 5 scratch reloads per PDHG iteration, the HBM traffic of
    // round 3's 14.3 KB per scenario-iteration)
    auto spmv_ax = [&](double (&out)[RPL]) {
        const int tq = launder(t);
        int off = 0;
#pragma unroll
        for (int ps = 0; ps < PPT; ++ps) {
            double acc = 0.0;
            if constexpr (RE > 0) {
#pragma unroll
                for (int k = 0; k < RE; ++k) acc = fma(rvr[ps][k], xl[rir[ps][k]], acc);
            } else {
                const int kk = B.rk[ps];
#pragma unroll 2
                for (int k = 0; k < kk; ++k) {
                    const int e = off + k * NT + tq;
                    if constexpr (UN) acc = unit_fma(codes[e], drow_of(rdm, off / NT + k), 0, acc, tq);
                    else acc = fma(rval(e, off / NT + k), xl[B.ridx[e]], acc);
                }
                off += kk * NT;
            }
            if constexpr (SEG > 0) {
                // the segment's sum in its first lane: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
                // row_mirror (every lane of an aligned group ends with the same bits: a + b = b + a)
                const double v1 = acc + dpp_d<0xB1>(acc);
                const double v2 = v1 + dpp_d<0x4E>(v1);
                const double v3 = v2 + dpp_d<0x141>(v2);
                const int L = rn[ps];   // 0 on lanes that own no row: their sum is 0 (their y stays 0)
                double t_ = L >= 8 ? v3 : (L >= 4 ? v2 : (L >= 2 ? v1 : (L == 1 ? acc : 0.0)));
                if constexpr (SEG == 16) {
                    const double v4 = v3 + dpp_d<0x140>(v3);
                    t_ = L >= 16 ? v4 : t_;
                }
                out[ps] = VS ? t_ * drs[ps] : t_;
            } else {
                rp[ps * NT + t] = acc;
            }
        }
        if constexpr (SEG == 0) {
            __syncthreads();
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
                const double t_ = PS ? piece_sum8(rp + rf[r], rn[r]) : piece_sum(rp + rf[r], rn[r]);
                out[r] = VS ? t_ * drs[r] : t_;
            }
        }
    };
    // A^T y for the y currently in yl
    auto spmv_aty = [&](double (&out)[CPL]) {
        const int tq = launder(t);
        int off = 0;
#pragma unroll
        for (int ps = 0; ps < QPT; ++ps) {
            double acc = 0.0;
            if constexpr (CE > 0) {
#pragma unroll
                for (int k = 0; k < CE; ++k) acc = fma(cvr[ps][k], yl[cir[ps][k]], acc);
            } else {
                const int kk = B.ck[ps];
#pragma unroll 2
                for (int k = 0; k < kk; ++k) {
                    const int e = off + k * NT + tq;
                    if constexpr (UN) acc = unit_fma(codes[B.er + e], drow_of(cdm, off / NT + k), B.nd_r, acc, tq);
                    else acc = fma(cval(e, off / NT + k), yl[B.cidx[e]], acc);
                }
                off += kk * NT;
            }
            if constexpr (CL) out[ps] = VS ? acc * dcs[ps] : 0.0 + acc;   // (the same bits as a one-piece piece_sum)
            else cp[ps * NT + t] = acc;
        }
        if constexpr (!CL) {
            __syncthreads();
#pragma unroll
            for (int k = 0; k < CPL; ++k) out[k] = VS ? piece_sum(cp + cf[k], cn[k]) * dcs[k] : piece_sum(cp + cf[k], cn[k]);
        }
    };
    auto put_x = [&](const double (&v)[CPL]) {
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (cj[k] >= 0) xl[cj[k]] = VS ? v[k] * dcs[k] : v[k];
    };
    auto put_y = [&](const double (&v)[RPL]) {
#pragma unroll
        for (int r = 0; r < RPL; ++r)
            if (ri[r] >= 0) yl[ri[r]] = VS ? v[r] * drs[r] : v[r];
    };
    // products at the current point (x, y): ends with every partial consumed
    auto products = [&]() {
        __syncthreads();
        put_x(x);
        put_y(y);
        __syncthreads();
        spmv_ax(ax);
        spmv_aty(aty);
        __syncthreads();
    };

    // ------------------------------------------------------------------ scalars
    double omega, cnorm;
    {
        double rr[4] = {c2, prox_const, 0.0, b2};
#pragma unroll
        for (int k = 0; k < CPL; ++k) rr[2] += c[k] * c[k];
        block_sum<NT, 4>(rr, red);
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
    for (int k = 0; k < CPL; ++k) ip[k] = 1.0 / (1.0 + tau * q[k]);
    products();

    // KKT pieces of one iterate (see pdhg.hip), reduced over the workgroup
    auto kkt = [&](const double (&xx)[CPL], const double (&at)[CPL], const double (&yy)[RPL],
                   const double (&axx)[RPL], double* o) {
        double v[6] = {0, 0, 0, 0, 0, 0};
        const int sl = launder(s);
        const long sn_ = (long)sl * a.n, sm_ = (long)sl * a.m;
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            seq();
            if (ri[r] >= 0) {
                const double pr = axx[r] - clampd(axx[r], rlo[r], rhi[r]);
                v[0] += pr * pr;
                // (VS: the scaling is already in a register -- no per-check load or address to keep)
                const double pu = pr / (VS ? drs[r] : a.dr[sm_ + ri[r]]);
                v[2] += pu * pu;
                if (fin(rlo[r])) v[5] += rlo[r] * fmax(yy[r], 0.0);
                if (fin(rhi[r])) v[5] += rhi[r] * fmin(yy[r], 0.0);
            }
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            seq();
            if (cj[k] >= 0) {
                const double rc_ = c[k] + q[k] * xx[k] - at[k];
                double dres = 0.0;
                if (!fin(lo[k]) && rc_ > 0.0) dres += rc_;
                if (!fin(hi[k]) && rc_ < 0.0) dres += rc_;
                v[1] += dres * dres;
                const double du = dres / (VS ? dcs[k] : a.dc[sn_ + cj[k]]);
                v[3] += du * du;
                v[4] += c[k] * xx[k] + 0.5 * q[k] * xx[k] * xx[k];
                if (fin(lo[k])) v[5] += lo[k] * fmax(rc_, 0.0);
                if (fin(hi[k])) v[5] += hi[k] * fmin(rc_, 0.0);
                v[5] -= 0.5 * q[k] * xx[k] * xx[k];
            }
        }
        block_sum<NT, 6>(v, red);
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
        kkt(x, aty, y, ax, o);
        kkt_restart = wkkt_of(o, omega);
    }
    int it = 0, since = 0, cnt = 0, st = 1;
    double rel_final = INFINITY, pobj = 0.0, dobj = 0.0;
    bool use_avg_final = false;
    const int chk = a.check_every;

    while (true) {
        for (int kk = 0; kk < chk; ++kk) {
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const double xn = clampd(fma(tau, aty[k] - c[k], x[k]) * ip[k], lo[k], hi[k]);
                x[k] = xn;
                xsum[k] += xn;
            }
            put_x(x);
            __syncthreads();
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
            __syncthreads();
            spmv_aty(aty);
        }
        it += chk;
        since += chk;
        cnt += chk;

        // ---------------------------------------------------------- restart / termination check
        const double inv = 1.0 / (double)cnt;
        double oc[6], oa[6];
        kkt(x, aty, y, ax, oc);
        // the average iterate at every check: on these LP relaxations (sslp, netdes) evaluating
        // it at every 3rd / 6th check only (as the lane-local kernel does) measured 1.3-2.6x the
        // PDHG iterations and 1.4-8x the time per launch
        constexpr bool avg = true;
        if (!avg) {
            oa[0] = oa[1] = oa[2] = oa[3] = INFINITY;
            oa[4] = INFINITY;
            oa[5] = -INFINITY;
        } else {
            double xa[CPL], ya[RPL], ata[CPL], axa[RPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k) xa[k] = xsum[k] * inv;
#pragma unroll
            for (int r = 0; r < RPL; ++r) ya[r] = ysum[r] * inv;
            __syncthreads();
            put_x(xa);
            put_y(ya);
            __syncthreads();
            spmv_ax(axa);
            spmv_aty(ata);
            kkt(xa, ata, ya, axa, oa);
        }
        const double rel_cur = rel_of(oc), rel_avg = avg ? rel_of(oa) : INFINITY;
        const bool nan = !(rel_cur == rel_cur);
        if (nan || rel_cur <= a.eps || rel_avg <= a.eps || it >= a.max_iter) {
            use_avg_final = !nan && rel_avg < rel_cur;
            rel_final = use_avg_final ? rel_avg : rel_cur;
            pobj = use_avg_final ? oa[4] : oc[4];
            dobj = use_avg_final ? oa[5] : oc[5];
            st = nan ? 2 : ((rel_cur <= a.eps || rel_avg <= a.eps) ? 0 : 1);
            break;
        }
        const double k_cur = wkkt_of(oc, omega), k_avg = avg ? wkkt_of(oa, omega) : INFINITY;
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
                    if (cj[k] >= 0) {
                        const long b = (long)sl * a.n + cj[k];
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
            block_sum<NT, 2>(mv, red);
            const double dx = sqrt(mv[0]), dy = sqrt(mv[1]);
            omega = primal_weight(omega, dx * dx, dy * dy, a.theta);
            tau = eta / omega;
            sig = eta * omega;
#pragma unroll
            for (int k = 0; k < CPL; ++k) { ip[k] = 1.0 / (1.0 + tau * q[k]); xsum[k] = 0.0; }
#pragma unroll
            for (int r = 0; r < RPL; ++r) ysum[r] = 0.0;
            cnt = 0;
            since = 0;
            kkt_restart = cand;
            kkt_prev = INFINITY;
        }
        // A x, A^T y at a new point (restart to the average); otherwise the registers still hold
        // the products of the current point (what a recomputation would return, bit for bit)
        if (restart && use_avg) products();
        else __syncthreads();
    }

    // ------------------------------------------------------------------ outputs
    const double inv = cnt > 0 ? 1.0 / (double)cnt : 0.0;
    const double offs = a.obj_off[s] + (a.prox_on ? prox_const : 0.0);
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        if (cj[k] >= 0) {
            const long b = sn + cj[k];
            const double xv = use_avg_final ? xsum[k] * inv : x[k];
            a.xs[b] = xv;
            const double xu = xv * a.dc[b];
            if (a.x_out) a.x_out[b] = xu;
            const int kk = a.lay.col_nonant[cj[k]];
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
    if (t == 0) {
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
struct BlockVariant {
    int NT, CPL, RPL, PPT, QPT, RE, CE, CL, VS, PS, UN, SEG;
    void (*fn)(PdhgArgs);
};

#define PHG_B(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 0, 0, 0, 0, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, false, false>}
#define PHG_BC(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 1, 0, 0, 0, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, true, false>}
#define PHG_BR(a_, b_, c_, d_, e_, f_, g_, h_) {a_, b_, c_, d_, e_, f_, g_, h_, 0, 0, 0, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, f_, g_, h_, false>}
// row piece sums with their loads issued together (default; PHG_PSUM=0 skips them, A/B)
#define PHG_BRP(a_, b_, c_, d_, e_, f_, g_, h_) {a_, b_, c_, d_, e_, f_, g_, h_, 0, 1, 0, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, f_, g_, h_, false, true>}
// the delta value form (unscaled shared pieces, scaling on the fly)
#define PHG_BV(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 0, 1, 0, 0, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, false, true>}
#define PHG_BCV(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 1, 1, 0, 0, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, true, true>}
// the unit form of the delta value form (BlockLayout::rcode): chosen at value time, not by the planner
#define PHG_BCVU(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 1, 1, 0, 1, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, true, true, false, true>}
#define PHG_BVU(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 0, 1, 0, 1, 0, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, false, true, false, true>}
// row segments of <= SEG lanes (rows of <= 8 / 16 pieces; PHG_BLOCK_SEG=0 skips them)
#define PHG_BRS(a_, b_, c_, d_, e_, f_, g_, h_) {a_, b_, c_, d_, e_, f_, g_, h_, 0, 0, 0, 8, pdhg_block_kernel<a_, b_, c_, d_, e_, f_, g_, h_, false, false, false, 8>}
#define PHG_BCVS(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 1, 1, 0, 0, 16, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, true, true, false, false, 16>}
#define PHG_BCVUS(a_, b_, c_, d_, e_) {a_, b_, c_, d_, e_, 0, 0, 1, 1, 0, 1, 16, pdhg_block_kernel<a_, b_, c_, d_, e_, 0, 0, true, true, false, true, 16>}
// preference order: smallest workgroup that holds the problem
static const BlockVariant kBlockVariants[] = {
    PHG_BRS(256, 3, 1, 1, 3, 8, 2, true),   // sslp: 180 row pieces in 15 8-lane + 45 2-lane segments
    PHG_BRP(256, 3, 1, 2, 3, 8, 2, true),   // sslp: ... row piece sums' loads issued together (PHG_PSUM=0: not)
    PHG_BR(256, 3, 1, 2, 3, 8, 2, true),    // sslp-like: register-resident pieces, column-local A^T y
    PHG_BR(256, 3, 1, 2, 3, 8, 2, false),   // the same with A^T y through LDS partials
    PHG_B(256, 3, 1, 2, 3),      // sslp-like: n <= 768, m <= 256
    PHG_B(256, 4, 4, 4, 4),      // n, m, pieces <= 1024
    PHG_B(512, 4, 4, 4, 4),      // <= 2048
    PHG_BC(1024, 3, 2, 3, 3),    // netdes-like with column-local A^T y (streamed values)
    PHG_B(1024, 3, 2, 3, 3),     // netdes-like: n <= 3072, m <= 2048
    PHG_B(1024, 4, 4, 4, 4),     // <= 4096
    // delta value form
    PHG_BV(256, 3, 1, 2, 3),
    PHG_BV(256, 4, 4, 4, 4),
    PHG_BV(512, 4, 4, 4, 4),
    PHG_BCVS(1024, 3, 2, 2, 3),  // netdes: rows in lane segments (<= 16 lanes; 1 910 of 2 048)
    PHG_BCV(1024, 3, 2, 3, 3),   // netdes (only the vubs' u_e vary).  (Its row piece sums with the
                                 // loads issued together, PHG_BCVP: 58.0 vs 42.0 ms per PH iteration
                                 // at 1 024 -- 372 B/lane of spills at 128 VGPRs -- not kept)
    PHG_BV(1024, 3, 2, 3, 3),
    PHG_BV(1024, 4, 4, 4, 4),
    // unit twins of the delta-form variants (same shapes; build_block_values switches to them)
    PHG_BVU(256, 3, 1, 2, 3),
    PHG_BVU(256, 4, 4, 4, 4),
    PHG_BVU(512, 4, 4, 4, 4),
    PHG_BCVU(1024, 3, 2, 3, 3),
    PHG_BCVUS(1024, 3, 2, 2, 3),
    PHG_BVU(1024, 3, 2, 3, 3),
    PHG_BVU(1024, 4, 4, 4, 4),
};
#undef PHG_B
#undef PHG_BR
#undef PHG_BC
#undef PHG_BV
#undef PHG_BCV
#undef PHG_BRP
#undef PHG_BCVU
#undef PHG_BRS
#undef PHG_BCVS
#undef PHG_BCVUS
#undef PHG_BVU

int pdhg_block_num_variants() { return (int)(sizeof(kBlockVariants) / sizeof(kBlockVariants[0])); }

void pdhg_block_variant_shape(int v, int* out12) {
    int* out9 = out12;
    const BlockVariant& V = kBlockVariants[v];
    out9[0] = V.NT; out9[1] = V.CPL; out9[2] = V.RPL; out9[3] = V.PPT; out9[4] = V.QPT; out9[5] = V.RE; out9[6] = V.CE;
    out9[7] = V.CL;
    out9[8] = V.VS;
    out9[9] = V.PS;
    out9[10] = V.UN;
    out9[11] = V.SEG;
}

// UN variants add the varying entry rows (nd doubles per thread) and the er + ec 16-bit codes
size_t pdhg_block_lds_bytes(int v, int n_pad, int m_pad, int nd, int ecodes) {
    const BlockVariant& V = kBlockVariants[v];
    const size_t base = (size_t)(n_pad + m_pad + 2 + V.PPT * V.NT + V.QPT * V.NT + 16 * (V.NT / 64 + 1)) * sizeof(double);
    return V.UN ? base + (size_t)nd * V.NT * sizeof(double) + (size_t)ecodes * sizeof(short) : base;
}

hipError_t pdhg_block_launch(int v, const PdhgArgs& a, hipStream_t stream) {
    const BlockVariant& V = kBlockVariants[v];
    const size_t lds = pdhg_block_lds_bytes(v, a.blk.n_pad, a.blk.m_pad, a.blk.nd_r + a.blk.nd_c, a.blk.er + a.blk.ec);
    hipLaunchKernelGGL(V.fn, dim3(a.S), dim3(V.NT), lds, stream, a);
    return hipGetLastError();
}

}  // namespace phg

namespace phg {

// piece-major value copies: out[s][e] = vals[s][perm[e]] (0 where perm < 0); grid (ceil(E/256), S')
__global__ void piece_gather_kernel(const double* vals, int nnz, const int* perm, int E, double* out) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const long s = blockIdx.y;
    if (e >= E) return;
    const int p = perm[e];
    out[s * E + e] = p >= 0 ? vals[s * nnz + p] : 0.0;
}

hipError_t piece_gather_launch(const double* vals, int nnz, const int* perm, int E, int S, double* out,
                               hipStream_t st) {
    hipLaunchKernelGGL(piece_gather_kernel, dim3((E + 255) / 256, S), dim3(256), 0, st, vals, nnz, perm, E, out);
    return hipGetLastError();
}

}  // namespace phg
