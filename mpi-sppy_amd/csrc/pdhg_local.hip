// pdhg_local.hip -- register-resident batched PDHG for block-structured scenario LPs/QPs (gfx950).
//
// Same algorithm and outputs as pdhg.hip (restarted PDHG, PDLP-style restarts and primal weight,
// relative-KKT termination on the unscaled problem; it replaces SPOpt.solve_one,
// mpisppy/spopt.py:184-231, for every local scenario at once), but with a different mapping of a
// scenario onto the wavefront, chosen when the sparsity pattern allows it:
//
//   * a scenario owns an aligned group of LPS = 16, 32 or 64 lanes, so one wave solves 64/LPS
//     scenarios side by side (farmer cm=10: 30 crop blocks -> 32 lanes, two scenarios per wave);
//   * every non-coupling row sits in the lane that owns ALL of its columns, so A x and A^T y for it
//     are register FMAs over a dense RPL x CPL block -- no LDS, no gathers, no barriers;
//   * the D coupling rows are replicated in every lane of the group; their A x is one
//     gsum<LPS> all-reduce (DPP row rotations + gfx950 permlane swaps, wave_ops.h) per iteration.
//
// So one PDHG iteration is ~100 fp64 VALU instructions and one short DPP chain per wave, with no
// memory traffic at all between the prologue (load the scenario) and the epilogue (store x, y).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ph_tail.h"
#include "phg_internal.h"
#include "wave_ops.h"

namespace phg {

// Per-lane "cold" state (read only at the every-`check_every` restart/termination test) lives in
// LDS as [item][lane] doubles -- conflict-free ds_read_b64 -- so the registers hold only what the
// PDHG iteration itself touches.  Lane items: XR / YR restart point, Q diagonal, C scaled cost,
// IDC / IDR inverse scalings (unscaled residuals), BLO / BHI the scaled row bounds (the registers
// hold them times -sigma).  Group items (the same value in every lane of a scenario's group, stored
// once per group and read as an LDS broadcast): the coupling rows' restart point, inverse scaling
// and bounds, and the scalars (CNORM, BNORM, ...).  12.5 KB per wave (farmer).
template <int CPL, int RPL, int D>
struct Cold {
    static constexpr int DD = D > 0 ? D : 1;
    // lane items
    static constexpr int XR = 0, Q = CPL, IDC = 2 * CPL, C = 3 * CPL, YR = 4 * CPL, IDR = YR + RPL, BLO = IDR + RPL,
                         BHI = BLO + RPL, NL = BHI + RPL;
    // group items
    static constexpr int YDR = 0, IDRD = DD, DLO = 2 * DD, DHI = 3 * DD, SC = 4 * DD;
    // KRST / KPREV hold SQUARED weighted KKT errors; TP / TD the squared termination thresholds
    // (eps (1 + ||b||))^2, (eps (1 + ||c||))^2; W2 / IW2 = omega^2, 1 / omega^2
    // KOFF: the objective constant of the gap test (PdhgArgs::gap_const)
    enum { CNORM = 0, BNORM, ETA, PROX, OMEGA, KRST, KPREV, TP, TD, W2, IW2, KOFF, NSC };
    static constexpr int NG = SC + NSC;
};
template <int LPS, int CPL, int RPL, int D>
constexpr size_t local_lds_bytes() {
    using CI = Cold<CPL, RPL, D>;
    return (size_t)(CI::NL * 64 + (64 / LPS) * CI::NG) * sizeof(double);
}

// One work item per group, grid = items / G.  (Round 3's persistent work-queue grid was measured
// slower and hung once; it is gone.)  PROF: the PHG_LOCAL_PROF diagnostic's clock reads and
// per-wave stores, a separate instantiation so the default kernel carries none of them.
//
// MB / MC: the block slots (bit r*CPL + k) and coupling slots (bit d*CPL + k) that hold an entry in
// at least one lane (computed on the host from the layout; all ones = the generic kernel).  A slot
// empty in every lane is dropped at compile time -- its register and its multiply-by-zero FMA in
// A x, A^T y and the check's products (farmer: 8 of 24 per iteration; every crop's lane has the
// same 4-column / 2-row block pattern and one coupling entry).  The sums are bit-identical to the
// generic kernel's (the dropped terms are fma(0, v, acc) = acc).
// Waves per SIMD.  Three fit the LDS (12.5 KB per wave on farmer) and, with the step
// coefficients re-derived after every check instead of held across it, 168 registers with a few
// prologue spills -- but measured on MI355X that is 0.345-0.350 ms per farmer-10k launch against
// 0.342 ms at two waves (the kernel is VALU-issue-bound, not latency-bound), so two it is.
// WV = 1 (the "lone-wave" instantiation, small shards): when the grid has no more waves than the chip
// has SIMDs, every wave runs alone on its SIMD whatever the register budget, so that build may take
// the whole register file (__launch_bounds__(64, 1)): the check keeps its per-element loads
// unserialised (no seq(): nothing else competes for the registers) and the scheduler interleaves
// its elements.  The arithmetic is the same operation for operation (the same bits).
#ifndef PHG_LOCAL_WAVES
#define PHG_LOCAL_WAVES 2
#endif
#ifndef PHG_SEQ_CHECK
#define PHG_SEQ_CHECK 0
#endif

// (xs dc) - xbar, each operation rounded on its own (the folded W update must see the bits of the
// epilogue's xN = xs dc)
__device__ __forceinline__ double x_minus_xbar(double xs, double dc, double xbar) {
#pragma clang fp contract(off)
    const double x = xs * dc;
    return x - xbar;
}

template <int LPS, int CPL, int RPL, int D, bool PROF, unsigned MB, unsigned MC, unsigned long long BI,
          unsigned long long BF, unsigned QM, int WV>
__global__ __launch_bounds__(64, WV) void pdhg_local_kernel(PdhgArgs a) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // PH converged: skip (see PdhgArgs::gate)
    extern __shared__ double cold[];
    constexpr int G = 64 / LPS;                    // scenarios per wave
    constexpr int DD = D > 0 ? D : 1;
    using CI = Cold<CPL, RPL, D>;
    const int lane = threadIdx.x;
    const int gl = lane % LPS;                     // lane inside the scenario's group
    const int grp = lane / LPS;
    auto CS = [&](int item) -> double& { return cold[item * 64 + lane]; };
    auto GS = [&](int item) -> double& { return cold[CI::NL * 64 + grp * CI::NG + item]; };
    // the primal step is x+ = clamp(x ip + A^T y tip - ctip) with ip = 1 / (1 + tau q),
    // tip = tau ip, ctip = c tip (re-derived whenever tau changes; c itself is read from LDS):
    // 2 instead of 3 fp64 ops per column, for 2 more registers per column -- only where they
    // fit (the widest variants would spill; they keep x+ = clamp((x + tau (A^T y - c)) ip))
    constexpr bool FOLD = RPL * CPL + D * CPL <= 12;
    // FOLDT (pattern-specialised kernels with <= 8 occupied slots): tau ip folded into the matrix as
    // well -- blkt = blk tip, cft = cf tip, re-derived with the step coefficients -- so the primal
    // step is one FMA chain clamp(fma(x, ip, -ctip) + sum blkt y) per column: A^T y itself is no
    // longer formed in the iteration (the checks re-form it), 1 fp64 instruction less per column
    constexpr bool FOLDT = FOLD && (__builtin_popcount(MB) + __builtin_popcount(MC) <= 8);

    // ------------------------------------------------------------------ per-group state
    int s = 0;                                     // scenario of the group's current work item
    double x[CPL], aty[CPL], c[CPL], lo[CPL], hi[CPL], ip[CPL], tip[CPL], ctip[CPL], xsum[CPL];
    double y[RPL], ax[RPL], rlo[RPL], rhi[RPL], ysum[RPL];
    double blk[RPL][CPL];
    double blkt[FOLDT ? RPL : 1][FOLDT ? CPL : 1];
    double yd[DD], axd[DD], dlo[DD], dhi[DD], ydsum[DD];
    double cf[DD][CPL];
    double cft[FOLDT ? DD : 1][FOLDT ? CPL : 1];
#pragma unroll
    for (int k = 0; k < CPL; ++k) { x[k] = aty[k] = c[k] = lo[k] = hi[k] = ip[k] = tip[k] = ctip[k] = xsum[k] = 0.0; }
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
        y[r] = ax[r] = rlo[r] = rhi[r] = ysum[r] = 0.0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) blk[r][k] = 0.0;
    }
#pragma unroll
    for (int d = 0; d < DD; ++d) {
        yd[d] = axd[d] = dlo[d] = dhi[d] = ydsum[d] = 0.0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) cf[d][k] = 0.0;
    }
    double omega = 1.0, tau = 0.0, sig = 0.0;
    int it = 0, since = 0, cnt = 0;
    int chk_mod = 0;   // the group's checks so far, modulo avg_every (avg: chk_mod == 0 at a check)

    // ------------------------------------------------------------------ products
    // (loops fully unrolled: the mask tests fold to constants)
    auto bon = [](int r, int k) { return ((MB >> (r * CPL + k)) & 1u) != 0u; };
    auto con = [](int d, int k) { return ((MC >> (d * CPL + k)) & 1u) != 0u; };
    // BI: bound sides infinite in every occupied lane slot of every scenario (host-verified,
    // local_inf_mask in phg_api.hip): the projection onto them is the identity, so its v_max / v_min
    // is dropped at compile time (bit-identical: max(v, -inf) = v, min(v, +inf) = v).  Bits: column
    // slot k lower 0 + k, upper 16 + k; row slot r lower 32 + r, upper 40 + r; coupling row d lower
    // 48 + d, upper 52 + d.  Farmer: 5 of the 14 clamps per PDHG iteration (sold / purchased
    // quantities have no upper bound, every row one infinite side)
    auto binf = [](int bit) { return ((BI >> bit) & 1ull) != 0ull; };
    // BF: bound sides FINITE in every occupied slot of every scenario (host-verified, local_fin_mask;
    // rows that fixing the nonants frees never count).  fin_side(bit, v) is then a compile-time
    // constant for every side in BI or BF -- the check's finiteness tests and their selects vanish
    // (the same values: fin(v) is what they would have returned)
    auto fin_side = [](int bit, double v) {
        if (((BI >> bit) & 1ull) != 0ull) return false;
        if (((BF >> bit) & 1ull) != 0ull) return true;
        return fin(v);
    };
    auto clampx = [&](int k, double v) {
        if (!binf(k)) v = vmax(v, lo[k]);
        if (!binf(16 + k)) v = vmin(v, hi[k]);
        return v;
    };
    // g - clamp(g, -sig hi, -sig lo) with the infinite sides' no-op dropped (rlo / rhi hold -sig
    // times the bounds: an infinite upper bound is -inf there, an infinite lower one +inf)
    auto dproj = [&](double g, double nhi, double nlo, int blo, int bhi) {
        double t = g;
        if (!binf(bhi)) t = vmax(t, nhi);
        if (!binf(blo)) t = vmin(t, nlo);
        return g - t;
    };
    // One-sided rows (compile time: one side in BF, the other in BI -- never a row the fixing of the
    // nonants frees): the row's A x is held in offset form w = A x - b (b its finite bound), which the
    // row sum forms for free (its FMA chain starts from -b, roff), so the dual step is
    //   y+ = max(y - sig (2 w+ - w), 0)   (lower bound)  /  min(..., 0)  (upper bound)
    // -- 3 instructions instead of 4 (the same projection; its roundings differ in the last bits)
    auto one_lo = [&](int r) { return ((BF >> (32 + r)) & 1ull) && ((BI >> (40 + r)) & 1ull); };
    auto one_hi = [&](int r) { return ((BF >> (40 + r)) & 1ull) && ((BI >> (32 + r)) & 1ull); };
    auto one_sided = [&](int r) { return one_lo(r) || one_hi(r); };
    double roff[RPL];
#pragma unroll
    for (int r = 0; r < RPL; ++r) roff[r] = 0.0;
    // The same for the coupling rows (bits 48 + d lower, 52 + d upper): their offset -b rides on the
    // group's lane 0 only (roffd: -b there, 0 elsewhere), so the group all-reduce returns A x - b.
    // A coupling row whose columns are all nonants (farmer's total acreage) is freed when the
    // nonants are fixed, so its finite side is in BF only for the variant the host picks for solves
    // WITHOUT fixed nonants (phg_api.hip local_variant_free)
    auto cone_lo = [&](int d) { return ((BF >> (48 + d)) & 1ull) && ((BI >> (52 + d)) & 1ull); };
    auto cone_hi = [&](int d) { return ((BF >> (52 + d)) & 1ull) && ((BI >> (48 + d)) & 1ull); };
    auto cone_sided = [&](int d) { return cone_lo(d) || cone_hi(d); };
    double roffd[DD];
#pragma unroll
    for (int d = 0; d < DD; ++d) roffd[d] = 0.0;
    // row r of the block times a column vector f(k) (first term a product, then FMAs; one-sided rows
    // in offset form: every term an FMA onto -b)
    auto brow = [&](int r, auto f) {
        if (one_sided(r)) {
            double acc = roff[r];
#pragma unroll
            for (int k = 0; k < CPL; ++k)
                if (bon(r, k)) acc = fma(blk[r][k], f(k), acc);
            return acc;
        }
        double acc = 0.0;
        bool first = true;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (bon(r, k)) { acc = first ? blk[r][k] * f(k) : fma(blk[r][k], f(k), acc); first = false; }
        return acc;
    };
    auto crow = [&](int d, auto f) {
        double acc = 0.0;
        bool first = true;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (con(d, k)) { acc = first ? cf[d][k] * f(k) : fma(cf[d][k], f(k), acc); first = false; }
        return acc;
    };
    // an iterate's coupling partial, in offset form on one-sided coupling rows (every term an FMA
    // onto roffd)
    auto crow_it = [&](int d, auto f) {
        if (!cone_sided(d)) return crow(d, f);
        double acc = roffd[d];
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (con(d, k)) acc = fma(cf[d][k], f(k), acc);
        return acc;
    };
    // column k of [block; coupling]^T times (row vector g(r), coupling vector h(d))
    auto bcol = [&](int k, auto g, auto h) {
        double acc = 0.0;
        bool first = true;
#pragma unroll
        for (int r = 0; r < RPL; ++r)
            if (bon(r, k)) { acc = first ? blk[r][k] * g(r) : fma(blk[r][k], g(r), acc); first = false; }
#pragma unroll
        for (int d = 0; d < D; ++d)
            if (con(d, k)) { acc = first ? cf[d][k] * h(d) : fma(cf[d][k], h(d), acc); first = false; }
        return acc;
    };
    auto mv_ax = [&](const double (&xx)[CPL], double (&o)[RPL], double (&od)[DD]) {
#pragma unroll
        for (int r = 0; r < RPL; ++r) o[r] = brow(r, [&](int k) { return xx[k]; });
        if constexpr (D > 0) {
            double t[D];
#pragma unroll
            for (int d = 0; d < D; ++d) t[d] = crow_it(d, [&](int k) { return xx[k]; });
            gsum_many<LPS, D>(t);
#pragma unroll
            for (int d = 0; d < D; ++d) od[d] = t[d];
        }
    };
    auto mv_aty = [&](const double (&yy)[RPL], const double (&yyd)[DD], double (&o)[CPL]) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) o[k] = bcol(k, [&](int r) { return yy[r]; }, [&](int d) { return yyd[d]; });
    };
    // row bounds are held pre-multiplied by -sig (the dual step; re-derived from the LDS copy at
    // restarts), so the dual projection is one v_max_f64 + one v_min_f64 without modifiers
    auto rescale_bounds = [&]() {
#pragma unroll
        for (int r = 0; r < RPL; ++r) { rlo[r] = -sig * CS(CI::BLO + r); rhi[r] = -sig * CS(CI::BHI + r); }
#pragma unroll
        for (int d = 0; d < D; ++d) { dlo[d] = -sig * GS(CI::DLO + d); dhi[d] = -sig * GS(CI::DHI + d); }
    };
    // QM: the column slots that can carry a quadratic term (a nonant's prox / smoothing diagonal, set
    // on the host from the slot tables); every other slot has q = 0 at compile time: ip = 1 without
    // the division, no q terms in the checks (the same values: 1 / (1 + tau 0) = 1, q x = 0)
    auto qon = [](int k) { return ((QM >> k) & 1u) != 0u; };
    auto step_coefs = [&]() {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            ip[k] = qon(k) ? 1.0 / (1.0 + tau * CS(CI::Q + k)) : 1.0;
            if constexpr (FOLD) {
                tip[k] = tau * ip[k];
                ctip[k] = CS(CI::C + k) * tip[k];
            }
            if constexpr (FOLDT) {
#pragma unroll
                for (int r = 0; r < RPL; ++r) blkt[r][k] = blk[r][k] * tip[k];
#pragma unroll
                for (int d = 0; d < D; ++d) cft[d][k] = cf[d][k] * tip[k];
            }
        }
    };

    // KKT pieces of an iterate over the scenario (group): [0] omega^2 ||pr||^2 + ||dres||^2 /
    // omega^2 on the scaled problem (PDLP's restart metric without the gap term), [1] unused,
    // [2] ||pr||^2 unscaled, [3] ||dres||^2 unscaled, [4] primal objective, [5] dual objective.  The iterate is given element-wise (xf, atf: column k; yf, axf: local row r;
    // axdp: coupling row d's LOCAL partial of A x) so the average iterate is never materialised in
    // registers.  Padded column / row slots hold zeros everywhere, so no per-element branches.
    // element-by-element order in the check (see kkt_part); dropped in the lone-wave build, and
    // since round 6 in the two-wave build too (PHG_SEQ_CHECK=0: the check then fits in 212 VGPRs
    // without spills; farmer 10k time to conv 0.775-0.777 vs 0.784 s, the same 5 185 PH iterations
    // and bits, the per-iteration line within noise -- profiles/r06/seq_check_ab.json)
    auto sq = []() {
        if constexpr (WV > 1 && PHG_SEQ_CHECK) seq();
    };
    constexpr int KT = 5 + DD;   // reduced values per iterate
    // slot of coupling row d's A x partial: 1 (free in the reduced vector), then 6, 7, ...
    auto cslot = [](int d) { return d == 0 ? 1 : 5 + d; };
    auto kkt_part = [&](auto xf, auto atf, auto yf, auto axf, auto axdp, double* t) {
#pragma unroll
        for (int u = 0; u < KT; ++u) t[u] = 0.0;
        double pr2 = 0.0, dr2 = 0.0;
        // element by element (seq() stops the scheduler from hoisting every element's loads and
        // products at once, which would hold them all in registers beside the hot state)
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            sq();
            const double axx = axf(r), yy = yf(r);
            const double bl = CS(CI::BLO + r), bu = CS(CI::BHI + r);
            // (one-sided rows: axx is the offset form A x - b)
            const double pr = one_lo(r) ? vmin(axx, 0.0) : one_hi(r) ? vmax(axx, 0.0) : axx - clampd(axx, bl, bu);
            pr2 += pr * pr;
            const double pu = pr * CS(CI::IDR + r);
            t[2] += pu * pu;
            if (fin_side(32 + r, bl)) t[5] += bl * vmax(yy, 0.0);
            if (fin_side(40 + r, bu)) t[5] += bu * vmin(yy, 0.0);
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            sq();
            const double xx = xf(k);
            const double qk = qon(k) ? CS(CI::Q + k) : 0.0;
            const double ck = FOLD ? CS(CI::C + k) : c[k];
            const double rc_ = qon(k) ? ck + qk * xx - atf(k) : ck - atf(k);
            double dres = 0.0;
            if (!fin_side(k, lo[k]) && rc_ > 0.0) dres += rc_;
            if (!fin_side(16 + k, hi[k]) && rc_ < 0.0) dres += rc_;
            dr2 += dres * dres;
            const double du = dres * CS(CI::IDC + k);
            t[3] += du * du;
            const double hq = qon(k) ? 0.5 * qk * xx * xx : 0.0;
            t[4] += qon(k) ? ck * xx + hq : ck * xx;
            if (fin_side(k, lo[k])) t[5] += lo[k] * vmax(rc_, 0.0);
            if (fin_side(16 + k, hi[k])) t[5] += hi[k] * vmin(rc_, 0.0);
            if (qon(k)) t[5] -= hq;
        }
        t[0] = fma(GS(CI::SC + CI::W2), pr2, dr2 * GS(CI::SC + CI::IW2));
#pragma unroll
        for (int d = 0; d < D; ++d) t[cslot(d)] = axdp(d);
    };
    // replicated coupling rows, added once after the group reduction
    // (off: the activities given are an iterate's, in offset form on one-sided coupling rows; the
    // average's are plain sums)
    auto kkt_coupling = [&](double* t, auto ydf, double scale, bool off) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            sq();
            const double axx = t[cslot(d)] * scale, yy = ydf(d);
            const double bl = GS(CI::DLO + d), bu = GS(CI::DHI + d);
            const double pr = cone_lo(d) ? vmin(off ? axx : axx - bl, 0.0)
                            : cone_hi(d) ? vmax(off ? axx : axx - bu, 0.0)
                                         : axx - clampd(axx, bl, bu);
            t[0] = fma(GS(CI::SC + CI::W2), pr * pr, t[0]);
            const double pu = pr * GS(CI::IDRD + d);
            t[2] += pu * pu;
            if (fin_side(48 + d, bl)) t[5] += bl * vmax(yy, 0.0);
            if (fin_side(52 + d, bu)) t[5] += bu * vmin(yy, 0.0);
        }
    };
    // the current iterate (its coupling products are already reduced: lane 0 of the group
    // contributes them) and, with AVG, the average iterate: one group reduction for both
    // the current iterate's coupling products are already group sums (axd): only its 5 other
    // values go through the reduction (adding the other lanes' zeros would return axd unchanged)
    auto kkt_both = [&](bool avg, double inv, double* oc, double* oa) {
        double t[2 * KT];
        kkt_part([&](int k) { return x[k]; }, [&](int k) { return aty[k]; }, [&](int r) { return y[r]; },
                 [&](int r) { return ax[r]; }, [&](int d) { return 0.0; }, t);
        if (avg) {
            kkt_part([&](int k) { return xsum[k] * inv; },
                     [&](int k) {
                         return bcol(k, [&](int r) { return ysum[r]; }, [&](int d) { return ydsum[d]; }) * inv;
                     },
                     [&](int r) { return ysum[r] * inv; },
                     [&](int r) {
                         // (offset form on the one-sided rows, as the current iterate's ax)
                         return one_sided(r) ? fma(brow(r, [&](int k) { return xsum[k]; }) - roff[r], inv, roff[r])
                                             : brow(r, [&](int k) { return xsum[k]; }) * inv;
                     },
                     [&](int d) { return crow(d, [&](int k) { return xsum[k]; }); },
                     t + KT);
            double u[5 + KT] = {t[0], t[2], t[3], t[4], t[5]};
#pragma unroll
            for (int q = 0; q < KT; ++q) u[5 + q] = t[KT + q];
            gsum_many<LPS, 5 + KT>(u);
            t[0] = u[0]; t[2] = u[1]; t[3] = u[2]; t[4] = u[3]; t[5] = u[4];
#pragma unroll
            for (int q = 0; q < KT; ++q) t[KT + q] = u[5 + q];
        } else {
            double u[5] = {t[0], t[2], t[3], t[4], t[5]};
            gsum_many<LPS, 5>(u);
            t[0] = u[0]; t[2] = u[1]; t[3] = u[2]; t[4] = u[3]; t[5] = u[4];
        }
#pragma unroll
        for (int d = 0; d < D; ++d) t[cslot(d)] = axd[d];
        kkt_coupling(t, [&](int d) { return yd[d]; }, 1.0, true);
#pragma unroll
        for (int u = 0; u < 6; ++u) oc[u] = t[u];
        if (avg) {
            kkt_coupling(t + KT, [&](int d) { return ydsum[d] * inv; }, inv, false);
#pragma unroll
            for (int u = 0; u < 6; ++u) oa[u] = t[KT + u];
        }
    };
    // relative KKT error (reported in the epilogue only)
    auto rel_of = [&](const double* o) {
        const double p = sqrt(o[2]) / (1.0 + GS(CI::SC + CI::BNORM));
        const double d = sqrt(o[3]) / (1.0 + GS(CI::SC + CI::CNORM));
        const double g = fabs(o[4] - o[5]) / gap_den(o[4], o[5], GS(CI::SC + CI::KOFF));
        return fmax(fmax(p, d), g);
    };
    // rel_of(o) <= eps without square roots or divisions
    auto converged = [&](const double* o) {
        return o[2] <= GS(CI::SC + CI::TP) && o[3] <= GS(CI::SC + CI::TD) &&
               fabs(o[4] - o[5]) <= a.eps * gap_den(o[4], o[5], GS(CI::SC + CI::KOFF));
    };
    // squared primal-weighted KKT error (PDLP's restart metric)
    auto wkkt2_of = [&](const double* o) {
        const double g = o[4] - o[5];
        return fma(g, g, o[0]);
    };

    // ------------------------------------------------------------------ load one scenario
    // (the group's lanes only; everything the iteration and the checks read is (re)initialised).
    // Branch-free: the constant data comes from the lane image (coalesced, no index chain), the
    // slot tables give the columns / rows / nonants of the dynamic data (warm start, W, rho, xbar),
    // read at clamped indices and masked, so every load of the scenario is in flight at once.  The
    // arithmetic is the round-3 prologue's, operation for operation (the same bits).
    constexpr int I_DC = 0, I_C = CPL, I_CL = 2 * CPL, I_CU = 3 * CPL, I_IDR = 4 * CPL, I_RL = 4 * CPL + RPL,
                  I_RU = 4 * CPL + 2 * RPL, I_B = 4 * CPL + 3 * RPL;
    constexpr int NB = __builtin_popcount(MB);
    auto bidx = [](int r, int k) { return __builtin_popcount(MB & ((1u << (r * CPL + k)) - 1u)); };
    auto cidx = [](int d, int k) { return __builtin_popcount(MC & ((1u << (d * CPL + k)) - 1u)); };
    auto load = [&](int sc) {
        s = sc;
        KP ka = kargs();
        const int n_ = ka->n, m_ = ka->m, N_ = ka->N, warm = ka->warm, fold = ka->fold_w;
        const long sn = (long)s * n_, sm = (long)s * m_, sN = (long)s * N_;
        const double* img = ka->loc.img + (long)s * ka->loc.ni * LPS + gl;
        const bool wx = (warm & 1) || fold;
        // slot tables
        int jj[CPL], kq[CPL], ii[RPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            jj[k] = ka->loc.col_of[gl * CPL + k];
            kq[k] = ka->loc.slot_kk[gl * CPL + k];
        }
#pragma unroll
        for (int r = 0; r < RPL; ++r) ii[r] = ka->loc.row_of[gl * RPL + r];
        // every load of the scenario
        double dd[CPL], cc[CPL], lo_[CPL], hi_[CPL], xw[CPL], wv[CPL], rv[CPL], xb[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            dd[k] = img[(I_DC + k) * LPS];
            cc[k] = img[(I_C + k) * LPS];
            lo_[k] = img[(I_CL + k) * LPS];
            hi_[k] = img[(I_CU + k) * LPS];
            const long b = sn + (jj[k] >= 0 ? jj[k] : 0);
            xw[k] = wx ? ka->xs_in[b] : 0.0;
            const int kk = kq[k] >= 0 ? kq[k] : 0;
            const long t = sN + kk;
            wv[k] = ka->W[t];
            rv[k] = ka->rho_k ? ka->rho_k[kk] : ka->rho[t];
            xb[k] = ka->xbar[ka->root_only ? kk : ka->xidx[t]];
        }
        double idr[RPL], rl_[RPL], ru_[RPL], yw[RPL];
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            idr[r] = img[(I_IDR + r) * LPS];
            rl_[r] = img[(I_RL + r) * LPS];
            ru_[r] = img[(I_RU + r) * LPS];
            yw[r] = (warm & 1) ? ka->ys_in[sm + (ii[r] >= 0 ? ii[r] : 0)] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < RPL; ++r)
#pragma unroll
            for (int k = 0; k < CPL; ++k) blk[r][k] = bon(r, k) ? img[(I_B + bidx(r, k)) * LPS] : 0.0;
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int k = 0; k < CPL; ++k) cf[d][k] = con(d, k) ? img[(I_B + NB + cidx(d, k)) * LPS] : 0.0;
        double ci[DD][3], yc[DD];
        int irow[DD];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const double* cim = ka->loc.cimg + ((long)s * D + d) * 3;
            ci[d][0] = cim[0];
            ci[d][1] = cim[1];
            ci[d][2] = cim[2];
            irow[d] = ka->loc.cpl_row[d];
            yc[d] = (warm & 1) && irow[d] >= 0 ? ka->ys_in[sm + irow[d]] : 0.0;
        }
        // columns
        double prox_const = 0.0, c2 = 0.0, dsum = 0.0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const bool occ = jj[k] >= 0;
            const double d = dd[k];
            double c_ = cc[k], qq = 0.0, clo = lo_[k], chi = hi_[k];
            const double xs0 = occ ? xw[k] : 0.0;
            if (kq[k] >= 0) {
                const long t = sN + kq[k];
                double w = wv[k];
                const double r_ = rv[k], xbv = xb[k];
                if (fold) {   // Update_W (phbase.py:301-326) of the x this solve starts from
                    // the epilogue's xN = xs * dc, rounded as it was: x - xbar without FMA contraction
                    const double dv = x_minus_xbar(xs0, d, xbv);
                    w = fma(r_, dv, w);
                    ka->W_rw[t] = w;
                    dsum += fabs(dv);
                }
                // ph_terms_w (phg_internal.h) on the preloaded rho / xbar, the same operations
                if (ka->w_on) c_ += w;
                if (ka->prox_on) {
                    c_ -= r_ * xbv;
                    qq = r_;
                    prox_const += 0.5 * r_ * xbv * xbv;
                    if (ka->smooth_on) {
                        const double p = ka->Psm[t], z = ka->Z[t];
                        c_ -= p * z;
                        qq += p;
                        prox_const += 0.5 * p * z * z;
                    }
                }
                if (ka->fix_nonants) {
                    const double v = ka->fixed[t];
                    const double wd = ka->fix_tol * fmax(1.0, fabs(v));
                    clo = (v - wd) / d;
                    chi = (v + wd) / d;
                }
            }
            c2 += c_ * c_;
            CS(CI::IDC + k) = occ ? 1.0 / d : 1.0;
            c[k] = c_ * d;
            lo[k] = clo;
            hi[k] = chi;
            x[k] = clampd((warm & 1) ? xs0 : 0.0, clo, chi);
            xsum[k] = aty[k] = 0.0;
            CS(CI::XR + k) = x[k];
            CS(CI::Q + k) = qq * d * d;
        }
        // rows
        double b2 = 0.0;
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            const bool occ = ii[r] >= 0;
            double lo = rl_[r], hi = ru_[r];
            if (ka->fix_nonants && occ && ka->row_fixed && ka->row_fixed[ii[r]]) { lo = -INFINITY; hi = INFINITY; }
            double yy = occ ? yw[r] : 0.0;
            if (!fin_side(32 + r, lo)) yy = fmin(yy, 0.0); else b2 += lo * lo;
            if (!fin_side(40 + r, hi)) yy = fmax(yy, 0.0); else b2 += hi * hi;
            y[r] = yy;
            ax[r] = ysum[r] = 0.0;
            rlo[r] = lo;
            rhi[r] = hi;
            roff[r] = one_lo(r) ? -lo : one_hi(r) ? -hi : 0.0;
            CS(CI::IDR + r) = idr[r];
            CS(CI::YR + r) = y[r];
            CS(CI::BLO + r) = lo;
            CS(CI::BHI + r) = hi;
        }
        double b2d = 0.0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const bool occ = irow[d] >= 0;
            double lo = ci[d][1], hi = ci[d][2];
            if (ka->fix_nonants && occ && ka->row_fixed && ka->row_fixed[irow[d]]) { lo = -INFINITY; hi = INFINITY; }
            double yy = yc[d];
            if (occ) {
                if (!fin_side(48 + d, lo)) yy = fmin(yy, 0.0); else b2d += lo * lo;
                if (!fin_side(52 + d, hi)) yy = fmax(yy, 0.0); else b2d += hi * hi;
            }
            yd[d] = yy;
            axd[d] = ydsum[d] = 0.0;
            dlo[d] = lo;
            dhi[d] = hi;
            roffd[d] = gl == 0 ? (cone_lo(d) ? -lo : cone_hi(d) ? -hi : 0.0) : 0.0;
            GS(CI::IDRD + d) = ci[d][0];
            GS(CI::YDR + d) = yd[d];
            GS(CI::DLO + d) = lo;
            GS(CI::DHI + d) = hi;
        }
        // ||c'|| (unscaled, incl. PH terms), prox constant, initial primal weight ||c_hat||/||b_hat||
        {
            double rr[5] = {c2, prox_const, 0.0, b2, dsum};
#pragma unroll
            for (int k = 0; k < CPL; ++k) rr[2] += c[k] * c[k];
            gsum_many<LPS, 5>(rr);
            if (fold && gl == 0) {   // (write-through: the tail waves read them in this launch)
                if (ka->tl.mode) {
                    st_sc1(&ka->conv_s[s], rr[4]);
                    st_sc1(&ka->fold_st[s], ka->status_in[s]);
                } else {   // (plain stores without the tail: write-through stores cost ~0.3 ms per
                           // launch at 1e6 scenarios, the PH-update sweep)
                    ka->conv_s[s] = rr[4];
                    ka->fold_st[s] = ka->status_in[s];
                }
            }
            rr[3] += b2d;
            GS(CI::SC + CI::CNORM) = sqrt(rr[0]);
            GS(CI::SC + CI::PROX) = rr[1];
            GS(CI::SC + CI::KOFF) = ka->gap_const ? ka->obj_off[s] + (ka->prox_on ? rr[1] : 0.0) : 0.0;
            const double cn = sqrt(rr[2]), bn = sqrt(rr[3]);
            omega = (cn > 1e-10 && bn > 1e-10) ? cn / bn : 1.0;
            const double om_in = (warm & 6) ? ka->omega_in[s] : 0.0;
            if ((warm & 2) && om_in > 0.0) omega = om_in;
            else if ((warm & 4) && om_in > 0.0) omega = sqrt(omega * om_in);   // blend
        }
        const double eta = ka->eta[s], bnorm = ka->bnorm[s];
        GS(CI::SC + CI::BNORM) = bnorm;
        GS(CI::SC + CI::ETA) = eta;
        {
            const double tp = ka->eps * (1.0 + bnorm), td = ka->eps * (1.0 + GS(CI::SC + CI::CNORM));
            GS(CI::SC + CI::TP) = tp * tp;
            GS(CI::SC + CI::TD) = td * td;
        }
        tau = eta / omega;
        sig = eta * omega;
        rescale_bounds();
#pragma unroll
        for (int k = 0; k < CPL; ++k) CS(CI::C + k) = c[k];
        step_coefs();
        mv_ax(x, ax, axd);
        mv_aty(y, yd, aty);
        GS(CI::SC + CI::OMEGA) = omega;
        GS(CI::SC + CI::W2) = omega * omega;
        GS(CI::SC + CI::IW2) = 1.0 / (omega * omega);
        {
            double o[6];
            kkt_both(false, 0.0, o, o);
            GS(CI::SC + CI::KRST) = wkkt2_of(o);
            GS(CI::SC + CI::KPREV) = INFINITY;
        }
        it = 0;
        since = 0;
        cnt = 0;
        chk_mod = 0;
    };

    // epilogue of a group that has terminated (st 0 optimal, 1 iteration limit, 2 NaN)
    auto finish = [&](bool use_avg, double inv, double rel, double pobj, double dobj, int st) {
        KP ka = kargs();
        const int sl = launder(s);
        const long sn = (long)sl * ka->n, sm = (long)sl * ka->m, sN = (long)sl * ka->N;
        const double* img = ka->loc.img + (long)sl * ka->loc.ni * LPS + gl;
        double* xo = ka->x_out;
        double* yo = ka->y_out;
        // every load first (tables, scaling), then the stores: a store may alias a later load, so
        // interleaving them would serialise one round trip per element
        int jj[CPL], kq[CPL], ii[RPL], irow[DD];
        double dcv[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            jj[k] = ka->loc.col_of[gl * CPL + k];
            kq[k] = ka->loc.slot_kk[gl * CPL + k];
            dcv[k] = img[(I_DC + k) * LPS];
        }
#pragma unroll
        for (int r = 0; r < RPL; ++r) ii[r] = ka->loc.row_of[gl * RPL + r];
#pragma unroll
        for (int d = 0; d < D; ++d) irow[d] = ka->loc.cpl_row[d];
        const double offs = ka->obj_off[sl] + (ka->prox_on ? GS(CI::SC + CI::PROX) : 0.0);
        const double sg = ka->sense;
        double* xs_ = ka->xs;
        double* xN_ = ka->xN;
        const bool tl_on = ka->tl.mode != 0;
        double* ys_ = ka->ys;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            if (jj[k] >= 0) {
                const long b = sn + jj[k];
                const double xv = use_avg ? xsum[k] * inv : x[k];
                xs_[b] = xv;
                const double xu = xv * dcv[k];
                if (xo) xo[b] = xu;
                if (kq[k] >= 0) {   // (write-through only when the tail reads them in this launch)
                    if (tl_on) st_sc1(&xN_[sN + kq[k]], xu);
                    else xN_[sN + kq[k]] = xu;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            if (ii[r] >= 0) {
                const long b = sm + ii[r];
                const double yv = use_avg ? ysum[r] * inv : y[r];
                ys_[b] = yv;
                if (yo) yo[b] = yv * ka->dr[b];
            }
        }
        if (gl == 0) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                if (irow[d] >= 0) {
                    const long b = sm + irow[d];
                    const double yv = use_avg ? ydsum[d] * inv : yd[d];
                    ys_[b] = yv;
                    if (yo) yo[b] = yv * ka->dr[b];
                }
            }
            ka->omega[sl] = GS(CI::SC + CI::OMEGA);
            ka->obj[sl] = sg * (pobj + offs);
            ka->bound[sl] = sg * (dobj + offs);
            ka->kkt[sl] = rel;
            ka->iters[sl] = it;
            ka->iters_acc[sl] += it;
            ka->status[sl] = st;
        }
    };

    // next work item of this group (group-uniform): the group's one item of this workgroup (and
    // nothing after it)
    int taken = 0;
    auto fetch = [&]() -> int { return taken++ ? a.S : (int)blockIdx.x * G + grp; };

    bool valid = true, live = false;   // valid: the group may still receive work
    const int chk = a.check_every;
    // PdhgArgs::prof: cycles in the PDHG iterations, in the checks (of which the KKT part and the
    // restart block), in loads; checks (uniform per wave)
    unsigned long long pf_it = 0, pf_chk = 0, pf_load = 0, pf_n = 0, pf_t1 = 0, pf_kkt = 0, pf_rst = 0;
    // and the wave's start / end on the 100 MHz constant clock (s_memrealtime): the occupancy timeline
    const unsigned long long pf_w0 = PROF ? __builtin_amdgcn_s_memrealtime() : 0ull;
    for (;;) {
        unsigned long long pf_t0 = 0;
        if constexpr (PROF) {
            pf_t0 = clock64();
            if (pf_t1) pf_chk += pf_t0 - pf_t1;
        }
        const bool need = valid && !live;
        if (wave_any(need)) {
            if (need) {
                const int w = fetch();
                if (w < a.S) {
                    const int* ord = kargs()->order;
                    load(ord ? ord[w] : w);
                    live = true;
                } else {
                    valid = false;
                }
            }
        }
        if constexpr (PROF) {
            const unsigned long long now = clock64();
            pf_load += now - pf_t0;
            pf_t0 = now;
        }
        if (!wave_any(live)) break;
        // two PDHG iterations per trip (check_every is even): the A x / A x+ hand-over is a
        // register rename instead of copies
        auto step = [&](auto sumc) {
            constexpr bool SUM = decltype(sumc)::value;
            // primal step: exact prox of the diagonal quadratic + box (1/(1+tau q) precomputed)
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                double xn;
                if constexpr (FOLDT) {
                    double acc = fma(x[k], ip[k], -ctip[k]);
#pragma unroll
                    for (int r = 0; r < RPL; ++r)
                        if (bon(r, k)) acc = fma(blkt[r][k], y[r], acc);
#pragma unroll
                    for (int d = 0; d < D; ++d)
                        if (con(d, k)) acc = fma(cft[d][k], yd[d], acc);
                    xn = clampx(k, acc);
                } else if constexpr (FOLD) {
                    xn = clampx(k, fma(aty[k], tip[k], fma(x[k], ip[k], -ctip[k])));
                } else {
                    xn = clampx(k, fma(tau, aty[k] - c[k], x[k]) * ip[k]);
                }
                x[k] = xn;
                if constexpr (SUM) xsum[k] += xn;
            }
            // dual step with extrapolation A(2x+ - x) = 2 A x+ - A x (empty row slots stay 0:
            // zero block row and zero bounds)
            double axn[RPL], axdn[DD];
            mv_ax(x, axn, axdn);
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
                // y+ = max(g + sig lo, 0) + min(g + sig hi, 0) = g - clamp(g, -sig hi, -sig lo)
                if (one_lo(r)) {
                    y[r] = vmax(fma(-sig, fma(2.0, axn[r], -ax[r]), y[r]), 0.0);
                } else if (one_hi(r)) {
                    y[r] = vmin(fma(-sig, fma(2.0, axn[r], -ax[r]), y[r]), 0.0);
                } else {
                    const double g = y[r] - sig * (2.0 * axn[r] - ax[r]);
                    y[r] = dproj(g, rhi[r], rlo[r], 32 + r, 40 + r);
                }
                ax[r] = axn[r];
                if constexpr (SUM) ysum[r] += y[r];
            }
#pragma unroll
            for (int d = 0; d < D; ++d) {
                if (cone_lo(d)) {
                    yd[d] = vmax(fma(-sig, fma(2.0, axdn[d], -axd[d]), yd[d]), 0.0);
                } else if (cone_hi(d)) {
                    yd[d] = vmin(fma(-sig, fma(2.0, axdn[d], -axd[d]), yd[d]), 0.0);
                } else {
                    const double g = yd[d] - sig * (2.0 * axdn[d] - axd[d]);
                    yd[d] = dproj(g, dhi[d], dlo[d], 48 + d, 52 + d);
                }
                axd[d] = axdn[d];
                if constexpr (SUM) ydsum[d] += yd[d];
            }
            if constexpr (!FOLDT) mv_aty(y, yd, aty);
        };
        // the running sums of the average iterate take every second iterate only (the average of
        // the even iterates: still an ergodic PDHG average, and a restart candidate like any other
        // point) -- 7 of ~62 fp64 instructions per PDHG iteration on farmer saved in the other step.
        // (Every fourth iterate, round 6: the xhat evaluation's fixed-nonant solves of farmer 10k
        // then no longer all reach the tolerance -- test_farmer_converged_ph_vs_ef[10000] -- so no.)
        // The only loop compiled: with the every-iterate and windowed loops beside it the scheduler
        // did worse (end of round 4: 0.2623 vs 0.2666 ms per launch, the same iterations bit for bit)
#pragma unroll 1
        for (int kk = 0; kk < chk; kk += 2) {
            step(std::false_type{});
            step(std::true_type{});
        }
        it += chk;
        since += chk;
        cnt += chk / 2;
        if constexpr (PROF) {
            pf_t1 = clock64();
            pf_it += pf_t1 - pf_t0;
            ++pf_n;
        }

        // ---------------------------------------------------------- restart / termination check
        const double inv = 1.0 / (double)cnt;
        double oc[6], oa[6];
        // the average iterate's KKT (products of the running sums: ~half the check) every
        // avg_every-th check of the group -- uniform over the wave, the check's reductions are
        // group-local but the products are wave-wide
        // ((it / chk) % avg_every == 0, counted instead of divided: a runtime integer division and
        // modulo on the VALU were ~40 instructions per check)
        chk_mod = chk_mod + 1 >= a.avg_every ? 0 : chk_mod + 1;
        const bool avg = wave_any(live && chk_mod == 0);
        if constexpr (FOLDT) mv_aty(y, yd, aty);   // not formed in the iterations
        kkt_both(avg, inv, oc, oa);
        if constexpr (PROF) pf_kkt += clock64() - pf_t1;
        if (!avg)
#pragma unroll
            for (int u = 0; u < 6; ++u) oa[u] = u == 4 ? INFINITY : (u == 5 ? -INFINITY : INFINITY);
        const bool nan = !(oc[2] + oc[3] + oc[4] + oc[5] == oc[2] + oc[3] + oc[4] + oc[5]);
        const bool ok_cur = converged(oc), ok_avg = avg && converged(oa);
        const bool term = live && (nan || ok_cur || ok_avg);
        const bool cap = live && !term && it >= a.max_iter;
        if (term || cap) {
            const double rel_cur = rel_of(oc), rel_avg = rel_of(oa);
            const bool ua = !nan && rel_avg < rel_cur;
            finish(ua, inv, ua ? rel_avg : rel_cur, ua ? oa[4] : oc[4], ua ? oa[5] : oc[5],
                   nan ? 2 : (term ? 0 : 1));
            live = false;
        }
        if (!wave_any(live)) continue;   // (refill or exit at the top)

        const double k_cur = wkkt2_of(oc), k_avg = wkkt2_of(oa);
        const bool use_avg = k_avg < k_cur;
        const double cand = use_avg ? k_avg : k_cur;
        const double krst = GS(CI::SC + CI::KRST);
        const bool restart = live && ((cand <= a.beta_suf * a.beta_suf * krst) ||
                                      (cand <= a.beta_nec * a.beta_nec * krst && cand > GS(CI::SC + CI::KPREV)) ||
                                      ((double)since >= a.beta_art * (double)it));
#ifdef PHG_LOCAL_WATCH
        if constexpr (PROF) {   // PHG_WATCH_SCEN (diagnostic build, -DPHG_LOCAL_WATCH): one scenario's
                                // restart / primal-weight history.  Not in the default PROF build: the
                                // printf's registers spilled it (~2 KB per lane) and distorted the splits
            if (live && gl == 0 && s == a.watch)
                printf("PHG_WATCH s %d it %d since %d avg %d kc %.6e ka %.6e krst %.6e kprev %.6e rst %d ua %d "
                       "om %.6e pres2 %.6e dres2 %.6e tp %.3e td %.3e pobj %.15e dobj %.15e\n",
                       s, it, since, (int)avg, k_cur, k_avg, krst, GS(CI::SC + CI::KPREV), (int)restart, (int)use_avg,
                       omega, oc[2], oc[3], GS(CI::SC + CI::TP), GS(CI::SC + CI::TD), oc[4], oc[5]);
        }
#endif
        if (live) GS(CI::SC + CI::KPREV) = cand;
        const unsigned long long pf_r0 = PROF ? clock64() : 0ull;
        if (wave_any(restart)) {
            const bool ra = restart && use_avg;
            if (wave_any(ra)) {
#pragma unroll
                for (int k = 0; k < CPL; ++k) x[k] = ra ? xsum[k] * inv : x[k];
#pragma unroll
                for (int r = 0; r < RPL; ++r) y[r] = ra ? ysum[r] * inv : y[r];
#pragma unroll
                for (int d = 0; d < D; ++d) yd[d] = ra ? ydsum[d] * inv : yd[d];
                // exact products at the new point; groups that keep their point recompute the same
                mv_ax(x, ax, axd);
                mv_aty(y, yd, aty);
            }
            // primal weight update from the movement since the last restart
            double mv[2] = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < CPL; ++k) { const double t = x[k] - CS(CI::XR + k); mv[0] += t * t; }
#pragma unroll
            for (int r = 0; r < RPL; ++r) { const double t = y[r] - CS(CI::YR + r); mv[1] += t * t; }
            gsum_many<LPS, 2>(mv);
#pragma unroll
            for (int d = 0; d < D; ++d) { const double t = yd[d] - GS(CI::YDR + d); mv[1] += t * t; }
            if (restart) {
                omega = primal_weight(GS(CI::SC + CI::OMEGA), mv[0], mv[1], a.theta);
                const double et = GS(CI::SC + CI::ETA);
                tau = et / omega;
                sig = et * omega;
                rescale_bounds();
                step_coefs();
#pragma unroll
                for (int k = 0; k < CPL; ++k) { CS(CI::XR + k) = x[k]; xsum[k] = 0.0; }
#pragma unroll
                for (int r = 0; r < RPL; ++r) { CS(CI::YR + r) = y[r]; ysum[r] = 0.0; }
#pragma unroll
                for (int d = 0; d < D; ++d) { GS(CI::YDR + d) = yd[d]; ydsum[d] = 0.0; }
                GS(CI::SC + CI::OMEGA) = omega;
                GS(CI::SC + CI::W2) = omega * omega;
                GS(CI::SC + CI::IW2) = 1.0 / (omega * omega);
                GS(CI::SC + CI::KRST) = cand;
                GS(CI::SC + CI::KPREV) = INFINITY;
                cnt = 0;
                since = 0;
            }
        }
        if constexpr (PROF) pf_rst += clock64() - pf_r0;
    }
    if (PROF && lane < 10) {   // (lane-indexed: a vector store)
        const unsigned long long pf_w1 = __builtin_amdgcn_s_memrealtime();
        // where the wave ran: HW_ID (SIMD [5:4], CU [11:8], SH [12], SE [15:13]) and the XCD
        unsigned hwid = 0, xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const unsigned long long v = lane == 0 ? pf_it : lane == 1 ? pf_chk : lane == 2 ? pf_load : lane == 3 ? pf_kkt
                                   : lane == 4 ? pf_rst : lane == 5 ? pf_n : lane == 6 ? pf_w0 : lane == 7 ? pf_w1
                                   : lane == 8 ? (unsigned long long)hwid : (unsigned long long)xcc;
        a.prof[(size_t)blockIdx.x * 10 + lane] = v;
    }
    // the pipelined iteration's PH update: the waves that complete its units run it (ph_tail.h)
    if (a.tl.mode) {
        int scen[G];
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const int w = (int)blockIdx.x * G + q;   // (fetch: this workgroup's one item per group)
            const int* ord = kargs()->order;
            scen[q] = w < a.S ? (ord ? ord[w] : w) : -1;
        }
        ph_tail_end<G>(a.tl, scen, cold);
    }
}

// ----------------------------------------------------------------------------- lane image
// LocalLayout::img / cimg of a batch (phg_load_batch, after prep_kernel has scaled it): one
// workgroup per scenario; the item order is the kernel's (I_DC ... I_B, then the MB / MC entries in
// slot order).  Empty slots: dc 1, everything else 0.
__global__ __launch_bounds__(256) void local_image_kernel(PdhgArgs a, int LPS, int CPL, int RPL, int D, unsigned MB,
                                                          unsigned MC, double* img, double* cimg) {
    const int s = blockIdx.x;
    const int NB = __builtin_popcount(MB), NC = __builtin_popcount(MC);
    const int ni = 4 * CPL + 3 * RPL + NB + NC;
    const long sn = (long)s * a.n, sm = (long)s * a.m, snz = (long)s * a.nnz;
    const LocalLayout& L = a.loc;
    for (int e = threadIdx.x; e < ni * LPS; e += 256) {
        const int item = e / LPS, gl = e % LPS;
        double v = 0.0;
        if (item < 4 * CPL) {
            const int f = item / CPL, k = item % CPL;
            const int j = L.col_of[gl * CPL + k];
            if (j < 0) v = f == 0 ? 1.0 : 0.0;
            else v = f == 0 ? a.dc[sn + j] : f == 1 ? a.c[sn + j] : f == 2 ? a.cl[sn + j] : a.cu[sn + j];
        } else if (item < 4 * CPL + 3 * RPL) {
            const int f = (item - 4 * CPL) / RPL, r = (item - 4 * CPL) % RPL;
            const int i = L.row_of[gl * RPL + r];
            if (i >= 0) v = f == 0 ? 1.0 / a.dr[sm + i] : f == 1 ? a.rl[sm + i] : a.ru[sm + i];
        } else {
            int q = item - (4 * CPL + 3 * RPL);
            const bool cpl = q >= NB;
            unsigned msk = cpl ? MC : MB;
            if (cpl) q -= NB;
            for (int u = 0; u < q; ++u) msk &= msk - 1u;   // drop the q lowest set bits
            const int bit = __builtin_ctz(msk);
            const int k = bit % CPL, rd = bit / CPL;
            const int p = cpl ? L.cpl_p[(rd * LPS + gl) * CPL + k] : L.blk_p[(gl * RPL + rd) * CPL + k];
            if (p >= 0) v = a.vals[snz + p];
        }
        img[((long)s * ni + item) * LPS + gl] = v;
    }
    if (threadIdx.x < 3 * D) {
        const int d = threadIdx.x / 3, f = threadIdx.x % 3;
        const int i = L.cpl_row[d];
        double v = 0.0;
        if (i >= 0) v = f == 0 ? 1.0 / a.dr[sm + i] : f == 1 ? a.rl[sm + i] : a.ru[sm + i];
        cimg[((long)s * D + d) * 3 + f] = v;
    }
}

// items per lane of variant v's image (LocalLayout::ni)
int pdhg_local_image_items(int v);

hipError_t pdhg_local_image_launch(int v, const PdhgArgs& a, double* img, double* cimg, hipStream_t stream);

// ----------------------------------------------------------------------------- executed work
// fp64 operations ONE lane issues per PDHG iteration in the hot loop of a variant (x 100; an FMA
// counts 2, an add / mul / max / min 1), restating the step's compile-time structure above:
//   primal step per column slot: FOLDT fma(x, ip, -ctip) + one FMA per occupied block / coupling
//     entry; FOLD two FMAs; else sub, FMA, mul -- then the clamps whose side is not infinite (BI);
//   A x: per row slot its occupied entries (one-sided rows: all FMAs onto the offset; else a mul
//     and FMAs), per coupling row a mul, FMAs and the log2(LPS) adds of the group sum;
//   dual step: one-sided rows 2 FMAs + 1 clamp, else 2 FMAs + the finite-side clamps + 1 sub;
//   A^T y (not FOLDT) per column a mul and FMAs; running sums (every second iterate) 1/2 per element.
// tools/loop_ops.py checks it against the compiled inner loop (the compiler turns the first DPP
// step's add into an FMA that re-forms the coupling product: +1 per coupling row in the ISA).
constexpr int local_loop_ops(int LPS, int CPL, int RPL, int D, unsigned MB, unsigned MC, unsigned long long BI,
                             unsigned long long BF) {
    const bool FOLD = RPL * CPL + D * CPL <= 12;
    const bool FOLDT = FOLD && (__builtin_popcount(MB) + __builtin_popcount(MC) <= 8);
    auto bon = [&](int r, int k) { return ((MB >> (r * CPL + k)) & 1u) != 0u; };
    auto con = [&](int d, int k) { return ((MC >> (d * CPL + k)) & 1u) != 0u; };
    auto inf = [&](int bit) { return ((BI >> bit) & 1ull) != 0ull; };
    auto finb = [&](int bit) { return ((BF >> bit) & 1ull) != 0ull; };
    int ops = 0;   // x 2: half-ops of the stride-2 running sums
    for (int k = 0; k < CPL; ++k) {
        int e = 0;
        for (int r = 0; r < RPL; ++r) e += bon(r, k);
        for (int d = 0; d < D; ++d) e += con(d, k);
        if (FOLDT) ops += 2 * (2 + 2 * e);
        else if (FOLD) ops += 2 * 4;
        else ops += 2 * 4;
        ops += 2 * ((inf(k) ? 0 : 1) + (inf(16 + k) ? 0 : 1));
        if (!FOLDT) ops += 2 * (e > 0 ? 2 * e - 1 : 0);   // A^T y
        ops += 1;                                         // x running sum
    }
    for (int r = 0; r < RPL; ++r) {
        int e = 0;
        for (int k = 0; k < CPL; ++k) e += bon(r, k);
        const bool one = (finb(32 + r) && inf(40 + r)) || (finb(40 + r) && inf(32 + r));
        ops += 2 * (one ? 2 * e : (e > 0 ? 2 * e - 1 : 0));
        ops += 2 * (one ? 5 : 4 + (inf(32 + r) ? 0 : 1) + (inf(40 + r) ? 0 : 1) + 1);
        ops += 1;
    }
    int lg = 0;
    for (int l = LPS; l > 1; l >>= 1) ++lg;
    for (int d = 0; d < D; ++d) {
        int e = 0;
        for (int k = 0; k < CPL; ++k) e += con(d, k);
        const bool one = (finb(48 + d) && inf(52 + d)) || (finb(52 + d) && inf(48 + d));   // offset form
        ops += 2 * ((one ? 2 * e : (e > 0 ? 2 * e - 1 : 0)) + lg);
        ops += 2 * (one ? 5 : 4 + (inf(48 + d) ? 0 : 1) + (inf(52 + d) ? 0 : 1) + 1);
        ops += 1;
    }
    return ops * 50;
}

// ----------------------------------------------------------------------------- dispatch
struct LocalVariant {
    int LPS, CPL, RPL, D;
    unsigned MB, MC;           // compiled-in block / coupling slot masks (all ones: generic)
    unsigned long long BI;     // compiled-in infinite bound sides (0: generic)
    unsigned long long BF;     // compiled-in finite bound sides (0: tested at run time)
    unsigned QM;               // column slots that can hold a quadratic term (all ones: generic)
    size_t lds;                // dynamic LDS per wave (Cold layout)
    void (*fn)(PdhgArgs);
    void (*fn_prof)(PdhgArgs);   // PROF: PdhgArgs::prof set (PHG_LOCAL_PROF)
    void (*fn1)(PdhgArgs);       // the lone-wave build (WV = 1), or null
    void (*fn1_prof)(PdhgArgs);
};

#define PHG_LK(a_, b_, c_, d_, p_, mb_, mc_, bi_, bf_, qm_, w_) \
    pdhg_local_kernel<a_, b_, c_, d_, p_, mb_, mc_, bi_, bf_, qm_, w_>
#define PHG_LM(a_, b_, c_, d_, mb_, mc_, bi_, bf_, qm_)                                                  \
    {a_, b_, c_, d_, mb_, mc_, bi_, bf_, qm_, local_lds_bytes<a_, b_, c_, d_>(),                            \
     PHG_LK(a_, b_, c_, d_, false, mb_, mc_, bi_, bf_, qm_, PHG_LOCAL_WAVES),                               \
     PHG_LK(a_, b_, c_, d_, true, mb_, mc_, bi_, bf_, qm_, PHG_LOCAL_WAVES), nullptr, nullptr}
// ... with a lone-wave build beside it
#define PHG_LM1(a_, b_, c_, d_, mb_, mc_, bi_, bf_, qm_)                                                 \
    {a_, b_, c_, d_, mb_, mc_, bi_, bf_, qm_, local_lds_bytes<a_, b_, c_, d_>(),                            \
     PHG_LK(a_, b_, c_, d_, false, mb_, mc_, bi_, bf_, qm_, PHG_LOCAL_WAVES),                               \
     PHG_LK(a_, b_, c_, d_, true, mb_, mc_, bi_, bf_, qm_, PHG_LOCAL_WAVES),                                \
     PHG_LK(a_, b_, c_, d_, false, mb_, mc_, bi_, bf_, qm_, 1), PHG_LK(a_, b_, c_, d_, true, mb_, mc_, bi_, bf_, qm_, 1)}
#define PHG_L(a_, b_, c_, d_) PHG_LM(a_, b_, c_, d_, (1u << (c_ * b_)) - 1u, (1u << ((d_ > 0 ? d_ : 1) * b_)) - 1u, 0ull, 0ull, (1u << b_) - 1u)
// farmer's infinite sides: columns 2, 3 (QuantitySuperQuotaSold, QuantityPurchased) above; row 0
// (cattle feed, >=) above, row 1 (limit sold, <= 0) below; the total-acreage row (<=) below
#define PHG_FARMER_BI ((1ull << 18) | (1ull << 19) | (1ull << 40) | (1ull << 33) | (1ull << 48))
// farmer's finite sides (local_fin_mask): every column lower bound, DevotedAcreage / SubQuota upper
// bounds, the cattle-feed row's lower and the limit-sold row's upper side (the acreage coupling row
// is freed when the nonants are fixed, so it stays a run-time test)
#define PHG_FARMER_BF 0x2010003000full
// shapes ordered by preference: fewest lanes per scenario first, then smallest register footprint;
// the generic kernel of every shape first, then pattern-specialised ones
static const LocalVariant kLocalVariants[] = {
    PHG_L(16, 4, 2, 1),
    PHG_L(16, 4, 3, 1),
    PHG_L(16, 4, 4, 2),
    PHG_L(32, 4, 2, 1),
    PHG_L(32, 4, 3, 1),
    PHG_L(32, 4, 4, 2),
    PHG_L(64, 4, 2, 1),
    PHG_L(64, 4, 3, 1),
    PHG_L(64, 4, 4, 2),
    // one column per lane, every row a coupling row: small dense-coupled scenarios (hydro,
    // examples/hydro/hydro.py:79-152: 16 columns, 10 rows, every row spanning 2-5 stages' columns)
    PHG_L(16, 1, 1, 10),
    // farmer (examples/farmer/farmer.py:157-203): per crop lane, columns DevotedAcreage, SubQuota,
    // SuperQuota, Purchased; rows cattle feed (all four) and limit sold (no Purchased); the
    // total-acreage coupling row on DevotedAcreage only
    PHG_LM(16, 4, 2, 1, 0x7Fu, 0x1u, 0ull, 0ull, 0xFu),
    PHG_LM(32, 4, 2, 1, 0x7Fu, 0x1u, 0ull, 0ull, 0xFu),
    PHG_LM(64, 4, 2, 1, 0x7Fu, 0x1u, 0ull, 0ull, 0xFu),
    // ... and its infinite bound sides
    PHG_LM(16, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, 0ull, 0xFu),
    PHG_LM(32, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, 0ull, 0xFu),
    PHG_LM(64, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, 0ull, 0xFu),
    // ... its finite ones, and the nonant (DevotedAcreage) in column slot 0 only
    PHG_LM1(16, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, PHG_FARMER_BF, 0x1u),
    PHG_LM1(32, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, PHG_FARMER_BF, 0x1u),
    PHG_LM1(64, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, PHG_FARMER_BF, 0x1u),
    // ... and, for solves whose nonants are NOT fixed (phg_api.hip local_variant_free), the total-
    // acreage coupling row's finite upper side: its A x in offset form, one dual-step instruction
    // fewer per PDHG iteration
    PHG_LM1(16, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, PHG_FARMER_BF | (1ull << 52), 0x1u),
    PHG_LM1(32, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, PHG_FARMER_BF | (1ull << 52), 0x1u),
    PHG_LM1(64, 4, 2, 1, 0x7Fu, 0x1u, PHG_FARMER_BI, PHG_FARMER_BF | (1ull << 52), 0x1u),
    // hydro's: no row local to a lane (the block slot dropped), all 10 coupling slots
    PHG_LM1(16, 1, 1, 10, 0x0u, 0x3FFu, 0ull, 0ull, 0x1u),
};
#undef PHG_FARMER_BI
#undef PHG_FARMER_BF
#undef PHG_L
#undef PHG_LM
#undef PHG_LM1
#undef PHG_LK
constexpr int kLocalShapes = 10;   // the generic entries; the planner walks these

int pdhg_local_num_variants() { return kLocalShapes; }

// the variant to run for shape v and the layout's slot masks: the specialised entry of that shape
// with the fewest slots that still covers every occupied one, else the generic kernel
int pdhg_local_pick_masked(int v, unsigned mb, unsigned mc, unsigned long long bi, unsigned long long bf,
                           unsigned qm) {
    const LocalVariant& S0 = kLocalVariants[v];
    int best = v, bits = __builtin_popcount(S0.MB) + __builtin_popcount(S0.MC);
    int inf = 0;
    const int total = (int)(sizeof(kLocalVariants) / sizeof(kLocalVariants[0]));
    for (int u = kLocalShapes; u < total; ++u) {
        const LocalVariant& V = kLocalVariants[u];
        if (V.LPS != S0.LPS || V.CPL != S0.CPL || V.RPL != S0.RPL || V.D != S0.D) continue;
        if ((mb & ~V.MB) || (mc & ~V.MC) || (V.BI & ~bi)) continue;   // every dropped clamp must be a no-op
        if (V.BF & ~bf) continue;                                      // every side assumed finite must be
        if (qm & ~V.QM) continue;                                      // every quadratic slot kept
        const int b = __builtin_popcount(V.MB) + __builtin_popcount(V.MC);
        const int f = __builtin_popcountll(V.BI) + __builtin_popcountll(V.BF) + (32 - __builtin_popcount(V.QM));
        if (b < bits || (b == bits && f > inf)) { best = u; bits = b; inf = f; }
    }
    return best;
}

void pdhg_local_variant_masks(int v, unsigned* out2) {
    out2[0] = kLocalVariants[v].MB;
    out2[1] = kLocalVariants[v].MC;
}

void pdhg_local_variant_shape(int v, int* out4) {
    const LocalVariant& V = kLocalVariants[v];
    out4[0] = V.LPS; out4[1] = V.CPL; out4[2] = V.RPL; out4[3] = V.D;
}

size_t pdhg_local_lds_bytes(int v) { return kLocalVariants[v].lds; }

int pdhg_local_loop_ops(int v) {
    const LocalVariant& V = kLocalVariants[v];
    return local_loop_ops(V.LPS, V.CPL, V.RPL, V.D, V.MB, V.MC, V.BI, V.BF);
}

// SIMDs of the current device (4 per CU): a grid of at most this many one-wave workgroups runs every
// wave alone on its SIMD
static int device_simds() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    return 4 * cus;
}

// the lone-wave build is taken when the variant has one and the grid fits the chip's SIMDs one wave
// each (small shards: farmer 10 000 over 4 or 8 GPUs); PHG_LOCAL_LONE=0 / 1 forces it off / on
bool pdhg_local_lone(int v, int S) {
    const LocalVariant& V = kLocalVariants[v];
    if (!V.fn1) return false;
    static const int force = [] { const char* e = std::getenv("PHG_LOCAL_LONE"); return e ? std::atoi(e) : -1; }();
    if (force >= 0) return force > 0;
    static int simds = -1;
    if (simds < 0) simds = device_simds();
    const int G = 64 / V.LPS;
    return (S + G - 1) / G <= simds;
}

hipError_t pdhg_local_launch(int v, const PdhgArgs& a, hipStream_t stream) {
    const LocalVariant& V = kLocalVariants[v];
    const int G = 64 / V.LPS;
    const size_t lds = pdhg_local_lds_bytes(v);
    const int grid = (a.S + G - 1) / G;
    const bool lone = pdhg_local_lone(v, a.S);
    void (*fn)(PdhgArgs) = lone ? (a.prof ? V.fn1_prof : V.fn1) : (a.prof ? V.fn_prof : V.fn);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64), lds, stream, a);   // (TailArgs::W = grid)
    return hipGetLastError();
}

int pdhg_local_image_items(int v) {
    const LocalVariant& V = kLocalVariants[v];
    return 4 * V.CPL + 3 * V.RPL + __builtin_popcount(V.MB) + __builtin_popcount(V.MC);
}

hipError_t pdhg_local_image_launch(int v, const PdhgArgs& a, double* img, double* cimg, hipStream_t stream) {
    const LocalVariant& V = kLocalVariants[v];
    hipLaunchKernelGGL(local_image_kernel, dim3(a.S), dim3(256), 0, stream, a, V.LPS, V.CPL, V.RPL, V.D, V.MB, V.MC,
                       img, cimg);
    return hipGetLastError();
}

}  // namespace phg
