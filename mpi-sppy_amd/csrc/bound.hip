// bound.hip -- a dual bound for every scenario that is valid whatever the solve's status
// (phg_opts.safe_bound).
//
// The reference takes each subproblem's outer bound from its solver (spopt.py:225-230,
// results.Problem[0].Lower_bound) and sums p_s * bound_s in Ebound (spopt.py:377-422) -- Iter0's
// trivial bound and the Lagrangian spoke's outer bound (lagrangian_bounder.py:21-44).  A first-order
// solve that stops at its iteration limit leaves a dual iterate that is not dual feasible: its
// "dual objective" is no bound.  This kernel turns ANY dual iterate y into a certificate by weak
// duality.  For the scaled subproblem  min c'x + 1/2 x'Qx  s.t. rl <= A x <= ru,  cl <= x <= cu
// (Q diagonal, the PH prox) and any y whose sign matches a finite row bound (y_i > 0 needs rl_i,
// y_i < 0 needs ru_i),
//     f(x) >= sum_i [y_i > 0 ? y_i rl_i : y_i ru_i] + sum_j min_{L_j <= x_j <= U_j} (r_j x_j + q_j/2 x_j^2)
// for every feasible x, with r = c' - A^T y and [L, U] ANY box holding the feasible set: the column
// bounds, an infinite side replaced by one the rows imply (computed on the host from the caller's
// data, slightly widened against round-off).  The only way to get -inf is then a column with q_j = 0,
// no finite bound on one side and its reduced cost pointing that way; such a reduced cost is
// repaired by moving the duals of the column's rows toward zero (which keeps their signs valid and
// changes other columns' reduced costs only by finite charges against their bounds).  If that cannot
// zero it, the scenario's bound is -inf: no finite certificate from this iterate.
//
// Applied to the scenarios that did NOT reach the KKT tolerance (status 1 / 2); the others keep the
// PDHG epilogue's dual objective (safe_bound = 2: to every scenario).  One 256-thread workgroup per scenario; duals and reduced costs in per-scenario scratch; the repair
// (a handful of columns on farmer: the Purchased columns, whose only row is the cattle-feed row) is
// sequential in one thread; sums are fixed-order block reductions (deterministic).
#include "phg_internal.h"
#include "wave_ops.h"

namespace phg {

__device__ __forceinline__ double block_sum256(double v, double* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const double t = ((red[0] + red[1]) + red[2]) + red[3];
    __syncthreads();
    return t;
}

__global__ __launch_bounds__(256) void safe_bound_kernel(PdhgArgs a, SafeBoundArgs b) {
    if (a.gate && a.gate[0] < a.gate_below) return;   // the solve was gated off: nothing to bound
    __shared__ double red[4];
    const int s = blockIdx.x, tid = threadIdx.x;
    // a scenario that reached the KKT tolerance keeps the solve's own dual objective -- a solver's
    // bound at optimality, as a CPU solver reports it at its tolerances; charging that iterate's
    // tolerance-level reduced costs against implied bounds would only loosen it (farmer: up to
    // 1.5e-6 relative, sold quantities capped at ~1e5)
    // (phg_opts.safe_bound = 2, SafeBoundArgs::all: every scenario -- a certificate at any eps)
    if (a.status[s] == 0 && !b.all) return;
    const int n = a.n, m = a.m;
    const long sn = (long)s * n, sm = (long)s * m, snz = (long)s * a.nnz, sN = (long)s * a.N;
    double* Y = b.Y + sm;
    double* R = b.R + sn;
    const double* v = a.vals + snz;                    // scaled values A_hat = Dr A Dc
    // scaled column box: the bound, or the implied one where the bound is infinite
    auto colbox = [&](int j, double& L, double& U) {
        const double d = a.dc[sn + j];
        L = a.cl[sn + j];
        U = a.cu[sn + j];
        if (!fin(L) && fin(b.ilo[sn + j])) L = b.ilo[sn + j] / d;
        if (!fin(U) && fin(b.ihi[sn + j])) U = b.ihi[sn + j] / d;
    };
    // scaled cost and prox diagonal of column j with the PH terms of the solve (ph_terms)
    auto cost = [&](int j, double& cc, double& qq, double& pc) {
        const double d = a.dc[sn + j];
        cc = a.c[sn + j];
        qq = 0.0;
        const int kk = a.lay.col_nonant[j];
        if (kk >= 0) ph_terms(a, sN + kk, kk, cc, qq, pc);
        cc *= d;
        qq *= d * d;
    };
    // 1. duals (scaled space: y_hat r_hat = y r), sign-projected onto the finite row bounds
    for (int i = tid; i < m; i += 256) {
        double y = a.ys[sm + i];
        if (y > 0.0 && !fin(a.rl[sm + i])) y = 0.0;
        if (y < 0.0 && !fin(a.ru[sm + i])) y = 0.0;
        Y[i] = y;
    }
    __syncthreads();
    // 2. reduced costs r = c_hat - A_hat^T y_hat (CSC of the shared pattern)
    for (int j = tid; j < n; j += 256) {
        double cc, qq, pc = 0.0;
        cost(j, cc, qq, pc);
        double aty = 0.0;
        for (int t = b.colptr[j]; t < b.colptr[j + 1]; ++t) aty = fma(v[b.csc_p[t]], Y[b.rowidx[t]], aty);
        R[j] = cc - aty;
    }
    __syncthreads();
    // 3. repair the reduced costs of columns with no finite bound on the side they point to
    if (tid == 0 && b.nf > 0) {
        for (int pass = 0; pass < 4; ++pass) {
            bool any = false;
            for (int f = 0; f < b.nf; ++f) {
                const int j = b.free_col[f];
                double cc, qq, pc = 0.0, L, U;
                cost(j, cc, qq, pc);
                if (qq > 0.0) continue;                 // the prox term bounds it already
                colbox(j, L, U);
                const double r = R[j];
                double need = 0.0;
                int dir = 0;                            // +1: raise r (U = inf), -1: lower it (L = -inf)
                if (r < 0.0 && !fin(U)) { need = -r; dir = 1; }
                else if (r > 0.0 && !fin(L)) { need = r; dir = -1; }
                if (dir == 0) continue;
                any = true;
                for (int t = b.colptr[j]; t < b.colptr[j + 1] && need > 0.0; ++t) {
                    const int i = b.rowidx[t];
                    const double av = v[b.csc_p[t]];
                    const double cap = dir * av * Y[i];   // how much moving y_i to 0 changes r_j
                    if (!(cap > 0.0)) continue;
                    const double del = fmin(need, cap);
                    const double y0 = Y[i];
                    const double y1 = del == cap ? 0.0 : y0 - dir * del / av;
                    Y[i] = y1;
                    const double dy = y1 - y0;
                    for (int p = b.rowptr[i]; p < b.rowptr[i + 1]; ++p) R[b.colidx[p]] -= v[p] * dy;
                    need -= del;
                }
            }
            if (!any) break;
        }
    }
    __syncthreads();
    // 4. the certificate: row terms + per-column minima (+ the objective constant)
    double t = 0.0, prox = 0.0;
    for (int i = tid; i < m; i += 256) {
        const double y = Y[i];
        if (y > 0.0) t += y * a.rl[sm + i];
        else if (y < 0.0) t += y * a.ru[sm + i];
    }
    for (int j = tid; j < n; j += 256) {
        double cc, qq, L, U;
        cost(j, cc, qq, prox);
        colbox(j, L, U);
        const double r = R[j];
        if (qq > 0.0) {
            const double xs = fmin(fmax(-r / qq, L), U);
            t += r * xs + 0.5 * qq * xs * xs;
        } else {
            // a reduced cost the repair left at round-off level counts as zero
            const double tol = 1e-12 * (1.0 + fabs(cc));
            if (r > 0.0) t += fin(L) ? r * L : (r <= tol ? 0.0 : -INFINITY);
            else if (r < 0.0) t += fin(U) ? r * U : (-r <= tol ? 0.0 : -INFINITY);
        }
    }
    t = block_sum256(t, red);
    prox = block_sum256(prox, red);
    if (tid == 0) {
        double d = t + a.obj_off[s] + (a.prox_on ? prox : 0.0);
        if (!(d == d)) d = -INFINITY;                   // a NaN iterate certifies nothing
        a.bound[s] = a.sense * d;
    }
}

hipError_t safe_bound_launch(const PdhgArgs& a, const SafeBoundArgs& b, hipStream_t st) {
    hipLaunchKernelGGL(safe_bound_kernel, dim3(a.S), dim3(256), 0, st, a, b);
    return hipGetLastError();
}

}  // namespace phg
