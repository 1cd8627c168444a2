#include <algorithm>
// prep.hip -- one-time per-batch preconditioning of the scenario LPs (runs at phg_load_batch).
//
// For every scenario (one 256-thread workgroup each): Ruiz equilibration (inf-norm, 10 passes),
// then one Pock-Chambolle (alpha = 1) pass, which bounds ||A_hat||_2 <= 1; then a power
// iteration on A_hat^T A_hat estimates ||A_hat||_2 for the PDHG step eta = 0.99/||A_hat||.
// Bounds are scaled in place (cl/dc, cu/dc, rl*dr, ru*dr); c is kept unscaled because the PH
// terms are added to it on the fly inside the solver.
#include "phg_internal.h"

namespace phg {

__device__ __forceinline__ double block_sum(double v, double* red) {
    // 256 threads = 4 waves; deterministic: wave butterflies, then wave 0 adds the 4 partials
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    const double t = ((red[0] + red[1]) + red[2]) + red[3];
    __syncthreads();
    return t;
}

__global__ __launch_bounds__(256) void prep_kernel(PrepArgs a) {
    __shared__ double red[4];
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    const int n = a.n, m = a.m, nnz = a.nnz;
    double* v = a.vals + (long)s * nnz;
    double* dc = a.dc + (long)s * n;
    double* dr = a.dr + (long)s * m;
    double* sc = a.scratch + (long)s * (2 * n + 2 * m);
    double* rs = sc;           // [m]
    double* cs = sc + m;       // [n]
    double* pv = sc + m + n;   // [n]
    double* pw = pv + n;       // [m]
    for (int j = tid; j < n; j += 256) dc[j] = 1.0;
    for (int i = tid; i < m; i += 256) dr[i] = 1.0;
    __syncthreads();
    for (int pass = 0; pass <= a.ruiz_iters; ++pass) {
        const bool pock = (pass == a.ruiz_iters);
        for (int i = tid; i < m; i += 256) {
            double acc = 0.0;
            for (int p = a.rowptr[i]; p < a.rowptr[i + 1]; ++p)
                acc = pock ? acc + fabs(v[p]) : fmax(acc, fabs(v[p]));
            rs[i] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
        }
        for (int j = tid; j < n; j += 256) {
            double acc = 0.0;
            for (int t = a.colptr[j]; t < a.colptr[j + 1]; ++t) {
                const double av = fabs(v[a.csc_p[t]]);
                acc = pock ? acc + av : fmax(acc, av);
            }
            cs[j] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
        }
        __syncthreads();
        for (int p = tid; p < nnz; p += 256) v[p] *= rs[a.row_of_p[p]] * cs[a.colidx[p]];
        for (int j = tid; j < n; j += 256) dc[j] *= cs[j];
        for (int i = tid; i < m; i += 256) dr[i] *= rs[i];
        __syncthreads();
    }
    // power iteration for ||A_hat||_2
    for (int j = tid; j < n; j += 256) pv[j] = 1.0;
    __syncthreads();
    double sig2 = 0.0;
    for (int itp = 0; itp < a.power_iters; ++itp) {
        for (int i = tid; i < m; i += 256) {
            double acc = 0.0;
            for (int p = a.rowptr[i]; p < a.rowptr[i + 1]; ++p) acc += v[p] * pv[a.colidx[p]];
            pw[i] = acc;
        }
        __syncthreads();
        double part = 0.0;
        for (int j = tid; j < n; j += 256) {
            double acc = 0.0;
            for (int t = a.colptr[j]; t < a.colptr[j + 1]; ++t) acc += v[a.csc_p[t]] * pw[a.row_of_p[a.csc_p[t]]];
            cs[j] = acc;
            part += acc * acc;
        }
        const double nrm = sqrt(block_sum(part, red));
        sig2 = nrm;   // ||A^T A v|| with ||v|| = 1  -> sigma_max^2 estimate
        const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
        for (int j = tid; j < n; j += 256) pv[j] = cs[j] * inv;
        __syncthreads();
    }
    const double anorm = sqrt(fmax(sig2, 1e-300));
    // scale bounds; ||b|| of the unscaled finite row bounds
    double b2 = 0.0;
    for (int i = tid; i < m; i += 256) {
        const long b = (long)s * m + i;
        const double l_ = a.rl[b], u_ = a.ru[b];
        if (fabs(l_) < 1e300) b2 += l_ * l_;
        if (fabs(u_) < 1e300) b2 += u_ * u_;
        a.rl[b] = l_ * dr[i];
        a.ru[b] = u_ * dr[i];
    }
    for (int j = tid; j < n; j += 256) {
        const long b = (long)s * n + j;
        a.cl[b] = a.cl[b] / dc[j];
        a.cu[b] = a.cu[b] / dc[j];
    }
    const double bn = sqrt(block_sum(b2, red));
    if (tid == 0) {
        a.eta[s] = 0.99 / fmax(anorm, 1e-12);
        a.bnorm[s] = bn;
    }
}

// new column bounds of a loaded batch (phg_set_col_bounds): scaled as prep_kernel scales them
__global__ void scale_cols_kernel(double* cl, double* cu, const double* dc, long cnt) {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < cnt; e += (long)gridDim.x * blockDim.x) {
        cl[e] = cl[e] / dc[e];
        cu[e] = cu[e] / dc[e];
    }
}

hipError_t scale_cols_launch(double* cl, double* cu, const double* dc, long cnt, hipStream_t stream) {
    const int grid = (int)std::min<long>(1024, (cnt + 255) / 256);
    hipLaunchKernelGGL(scale_cols_kernel, dim3(std::max(1, grid)), dim3(256), 0, stream, cl, cu, dc, cnt);
    return hipGetLastError();
}

hipError_t prep_launch(const PrepArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(prep_kernel, dim3(a.S), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace phg
