// Minimal reproducer for the UC-under-rocprofv3 exit segfault: one trivial kernel
// launched with hipLaunchCooperativeKernel (mode 1) or with a plain launch (mode 0), synchronised,
// then a normal process exit.  Run plain and under `rocprofv3 --kernel-trace --stats`: a crash only
// in the cooperative + profiler combination isolates the teardown fault from libphg.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void touch(int* p) { if (threadIdx.x == 0) p[blockIdx.x] = (int)blockIdx.x; }

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 1;
    int* d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 2;
    void* args[] = {&d};
    hipError_t e;
    if (mode) {
        e = hipLaunchCooperativeKernel((const void*)touch, dim3(64), dim3(64), args, 0, 0);
    } else {
        hipLaunchKernelGGL(touch, dim3(64), dim3(64), 0, 0, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    int h[64];
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("mode %d: %s, h[63] = %d\n", mode, hipGetErrorString(e), h[63]);
    (void)hipFree(d);
    return e == hipSuccess ? 0 : 1;
}
