// ph_update.hip -- fused PH node-average / dual-weight / convergence kernels.
//
// Restates, for all local scenarios at once and with deterministic fixed-order reductions
// (no floating-point atomics):
//   _Compute_Xbar     mpisppy/phbase.py:32-112   node sums of prob_coeff*x and prob_coeff*x^2
//   Update_W          mpisppy/phbase.py:301-326  W += rho (x - xbar)
//   convergence_diff  mpisppy/phbase.py:349-371  (1/P) sum_v  sum_{s in v,k} |x - xbar| / count_v
// Node sums are reduced per "segment" (a contiguous scenario range inside one node) and then
// per node in segment order; the cross-GPU all-reduce (RCCL) of the 2*N_tot node sums and of the
// 2*P convergence partials happens between the kernels (see include/phg.h).
#include "phg_internal.h"

namespace phg {

// one workgroup per node segment; thread t handles nonant k = t % klen of scenarios
// s0 + t / klen + q*i  (q = 256 / klen lanes per nonant) -> coalesced rows of xN
__global__ __launch_bounds__(256) void node_partial_kernel(PhArgs a) {
    __shared__ double sh[2 * 256];
    const NodeSeg sg = a.seg[blockIdx.x];
    const int tid = threadIdx.x;
    double* out = a.segpart + (long)blockIdx.x * 2 * a.maxk;
    for (int k0 = 0; k0 < sg.klen; k0 += 256) {
        const int kl = min(256, sg.klen - k0);
        const int q = 256 / kl;
        const int k = tid % kl;
        const int so = tid / kl;
        double s1 = 0.0, s2 = 0.0;
        if (so < q) {
            const int kg = sg.kofs + k0 + k;
            for (int s = sg.s0 + so; s < sg.s1; s += q) {
                const double xv = a.xN[(long)s * a.N + kg];
                const double p = a.pc[(long)s * a.L + sg.level];
                s1 += p * xv;
                s2 += p * xv * xv;
            }
        }
        sh[tid] = s1;
        sh[256 + tid] = s2;
        __syncthreads();
        if (tid < kl) {
            double t1 = 0.0, t2 = 0.0;
            for (int j = 0; j < q; ++j) { t1 += sh[j * kl + tid]; t2 += sh[256 + j * kl + tid]; }
            out[k0 + tid] = t1;
            out[a.maxk + k0 + tid] = t2;
        }
        __syncthreads();
    }
}

// one thread per (node, i): add that node's segment partials in segment order
__global__ void node_final_kernel(PhArgs a, double* nodesum) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.N_tot) return;
    // find the node g with node_off[g] <= e < node_off[g] + level_len[level[g]]
    int lo = 0, hi = a.n_nodes - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.node_off[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const int g = lo;
    const int i = e - a.node_off[g];
    double t1 = 0.0, t2 = 0.0;
    for (int sg = a.node_first_seg[g]; sg < a.node_first_seg[g + 1]; ++sg) {
        t1 += a.segpart[(long)sg * 2 * a.maxk + i];
        t2 += a.segpart[(long)sg * 2 * a.maxk + a.maxk + i];
    }
    nodesum[e] = t1;
    nodesum[a.N_tot + e] = t2;
}

// one workgroup per convergence segment (scenario range inside one virtual rank):
// xbar from the (all-reduced) node sums, W update, sum |x - xbar|
__global__ __launch_bounds__(256) void w_update_kernel(PhArgs a, const double* nodesum) {
    __shared__ double red[4];
    const int b = blockIdx.x;
    const long e0 = (long)a.cseg_s0[b] * a.N, e1 = (long)a.cseg_s1[b] * a.N;
    double acc = 0.0;
    for (long e = e0 + threadIdx.x; e < e1; e += 256) {
        const double xb = nodesum[a.xidx[e]];
        const double d = a.xN[e] - xb;
        a.W[e] += a.rho[e] * d;
        acc += fabs(d);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) a.csegpart[b] = ((red[0] + red[1]) + red[2]) + red[3];
    // the first workgroup also publishes xbar / xsqbar
    if (b == 0)
        for (int j = threadIdx.x; j < a.N_tot; j += 256) {
            a.xbar[j] = nodesum[j];
            a.xsqbar[j] = nodesum[a.N_tot + j];
        }
}

__global__ void conv_final_kernel(PhArgs a, double* convpart) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= a.P) return;
    double t = 0.0, cnt = 0.0;
    for (int b = a.vr_first[v]; b < a.vr_first[v + 1]; ++b) {
        t += a.csegpart[b];
        cnt += (double)(a.cseg_s1[b] - a.cseg_s0[b]) * (double)a.N;
    }
    convpart[2 * v] = t;
    convpart[2 * v + 1] = cnt;
}

// per-scenario objective value with the current W / xbar / rho (pyo.value(objfct))
__global__ void eval_obj_kernel(int S, int n, int N, const double* x, const double* c,
                                const double* obj_off, const int* nonant_col, const double* xN,
                                const double* W, const double* rho, const double* xbar,
                                const int* xidx, int w_on, int prox_on, double sense,
                                double* out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    double f = 0.0;
    for (int j = 0; j < n; ++j) f += c[(long)s * n + j] * x[(long)s * n + j];
    double t = 0.0;
    for (int k = 0; k < N; ++k) {
        const long e = (long)s * N + k;
        const double xv = xN[e];
        if (w_on) t += W[e] * xv;
        if (prox_on) {
            const double xb = xbar[xidx[e]];
            t += 0.5 * rho[e] * (xv * xv - 2.0 * xb * xv + xb * xb);
        }
    }
    // c is min-form: model objective = sense * (c.x + off) ; PH terms enter with the model sense
    out[s] = sense * (f + obj_off[s]) + sense * t;
}

hipError_t node_sums_launch(const PhArgs& a, double* nodesum, hipStream_t st) {
    hipLaunchKernelGGL(node_partial_kernel, dim3(a.n_seg), dim3(256), 0, st, a);
    hipLaunchKernelGGL(node_final_kernel, dim3((a.N_tot + 255) / 256), dim3(256), 0, st, a, nodesum);
    return hipGetLastError();
}

hipError_t w_update_launch(const PhArgs& a, const double* nodesum, double* convpart, hipStream_t st) {
    hipLaunchKernelGGL(w_update_kernel, dim3(a.n_cseg), dim3(256), 0, st, a, nodesum);
    hipLaunchKernelGGL(conv_final_kernel, dim3((a.P + 255) / 256), dim3(256), 0, st, a, convpart);
    return hipGetLastError();
}

hipError_t eval_obj_launch(int S, int n, int N, const double* x, const double* c, const double* obj_off,
                           const int* nonant_col, const double* xN, const double* W, const double* rho,
                           const double* xbar, const int* xidx, int w_on, int prox_on, double sense,
                           double* out, hipStream_t st) {
    hipLaunchKernelGGL(eval_obj_kernel, dim3((S + 127) / 128), dim3(128), 0, st, S, n, N, x, c, obj_off,
                       nonant_col, xN, W, rho, xbar, xidx, w_on, prox_on, sense, out);
    return hipGetLastError();
}

}  // namespace phg
