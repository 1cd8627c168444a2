// hbm_probe.hip -- ceilings for the PH-update access patterns on MI355X (NOT the product: a
// measurement tool).  Over S*N = 1e8 doubles (800 MB per array):
//   read      : grid-stride 16-byte loads of one array, summed (the node-sum pass's traffic)
//   read_nt   : the same with nontemporal loads
//   update    : W = W + r (x - c) with 16-byte loads/stores (x, W, r read, W written: the W update)
//   update_nt : the same with nontemporal loads / stores
//   copy      : y = x (the guide's 6.3 TB/s reference pattern)
// Build: hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o tools/_diag/hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double v2d __attribute__((ext_vector_type(2)));

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const v2d* __restrict__ x, long n2, double* out) {
    double acc = 0.0;
    const long stride = (long)gridDim.x * 256;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n2; i += U * stride) {
        v2d v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(x + i + u * stride) : x[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y;
    }
    for (; i < n2; i += stride) { const v2d v = x[i]; acc += v.x + v.y; }
    if (acc == 12345.678) out[0] = acc;   // keeps the loads
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void update_kernel(const v2d* __restrict__ x, const v2d* __restrict__ r,
                                                     v2d* __restrict__ w, long n2, double c) {
    const long stride = (long)gridDim.x * 256;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n2; i += U * stride) {
        v2d xv[U], rv[U], wv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + u * stride;
            xv[u] = NT ? __builtin_nontemporal_load(x + k) : x[k];
            rv[u] = NT ? __builtin_nontemporal_load(r + k) : r[k];
            wv[u] = NT ? __builtin_nontemporal_load(w + k) : w[k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const v2d o = v2d{fma(rv[u].x, xv[u].x - c, wv[u].x), fma(rv[u].y, xv[u].y - c, wv[u].y)};
            if (NT) __builtin_nontemporal_store(o, w + i + u * stride);
            else w[i + u * stride] = o;
        }
    }
    for (; i < n2; i += stride) {
        const v2d xv = x[i], rv = r[i], wv = w[i];
        w[i] = v2d{fma(rv.x, xv.x - c, wv.x), fma(rv.y, xv.y - c, wv.y)};
    }
}

__global__ __launch_bounds__(256) void copy_kernel(const v2d* __restrict__ x, v2d* __restrict__ y, long n2) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) y[i] = x[i];
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 100000000L;
    const long n2 = n / 2;
    double *x, *r, *w, *y, *out;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&r, n * 8));
    CK(hipMalloc(&w, n * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(x, 0, n * 8));
    CK(hipMemset(r, 0, n * 8));
    CK(hipMemset(w, 0, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int k = 0; k < 3; ++k) launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int k = 0; k < reps; ++k) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
        std::printf("%-28s %9.1f us  %7.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
    };
    const double B = (double)n * 8;
    for (int grid : {8192, 16384, 32768, 65536}) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "read U8 grid %d", grid);
        timeit(nm, B, [&] { read_kernel<8, false><<<grid, 256>>>((const v2d*)x, n2, out); });
        std::snprintf(nm, sizeof nm, "read_nt U4 grid %d", grid);
        timeit(nm, B, [&] { read_kernel<4, true><<<grid, 256>>>((const v2d*)x, n2, out); });
        std::snprintf(nm, sizeof nm, "read_nt U8 grid %d", grid);
        timeit(nm, B, [&] { read_kernel<8, true><<<grid, 256>>>((const v2d*)x, n2, out); });
        std::snprintf(nm, sizeof nm, "read_nt U16 grid %d", grid);
        timeit(nm, B, [&] { read_kernel<16, true><<<grid, 256>>>((const v2d*)x, n2, out); });
        std::snprintf(nm, sizeof nm, "update U4 grid %d", grid);
        timeit(nm, 4 * B, [&] { update_kernel<4, false><<<grid, 256>>>((const v2d*)x, (const v2d*)r, (v2d*)w, n2, 0.5); });
        std::snprintf(nm, sizeof nm, "update_nt U2 grid %d", grid);
        timeit(nm, 4 * B, [&] { update_kernel<2, true><<<grid, 256>>>((const v2d*)x, (const v2d*)r, (v2d*)w, n2, 0.5); });
        std::snprintf(nm, sizeof nm, "update_nt U4 grid %d", grid);
        timeit(nm, 4 * B, [&] { update_kernel<4, true><<<grid, 256>>>((const v2d*)x, (const v2d*)r, (v2d*)w, n2, 0.5); });
        std::snprintf(nm, sizeof nm, "update_nt U8 grid %d", grid);
        timeit(nm, 4 * B, [&] { update_kernel<8, true><<<grid, 256>>>((const v2d*)x, (const v2d*)r, (v2d*)w, n2, 0.5); });
        std::snprintf(nm, sizeof nm, "copy grid %d", grid);
        timeit(nm, 2 * B, [&] { copy_kernel<<<grid, 256>>>((const v2d*)x, (v2d*)y, n2); });
    }
    return 0;
}
