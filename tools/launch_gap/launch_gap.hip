// Kernel-boundary cost on this GPU: back-to-back dependent launches on one stream (no host sync in
// between), for a trivial kernel and for one that leaves `mb` MiB of dirty lines in L2, plain and
// captured in a hipGraph.  Prints the average period per launch.  (Diagnostic for DESIGN.md (d).)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void touch(double* p, long n, double v) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v + i;
}

struct Big { double* p; long n; double v; double pad[197]; };   // 1 616 B, the size of PdhgArgs
__global__ void touch_big(Big b) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += (long)gridDim.x * blockDim.x) b.p[i] = b.v + i + b.pad[i & 7];
}

// big kernel arguments, optionally with a timing event pair around every launch (bench.py's form)
static double run_big(hipStream_t s, double* buf, long n, int grid, int reps, bool events) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int per = 20;
    std::vector<hipEvent_t> ev(2 * per * (reps + 3));
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    Big g{};
    g.p = buf; g.n = n;
    int k = 0;
    auto one = [&](int i) {
        g.v = i;
        if (events) CK(hipEventRecord(ev[k++], s));
        hipLaunchKernelGGL(touch_big, dim3(grid), dim3(256), 0, s, g);
        if (events) CK(hipEventRecord(ev[k++], s));
    };
    for (int w = 0; w < 3; ++w) for (int i = 0; i < per; ++i) one(i);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) for (int i = 0; i < per; ++i) one(i);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3 / (reps * per);
}

static double run(hipStream_t s, double* buf, long n, int grid, int reps, bool graph) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipGraphExec_t ge = nullptr;
    const int per = 20;
    if (graph) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < per; ++i) hipLaunchKernelGGL(touch, dim3(grid), dim3(256), 0, s, buf, n, (double)i);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    for (int w = 0; w < 3; ++w) {
        if (graph) CK(hipGraphLaunch(ge, s));
        else for (int i = 0; i < per; ++i) hipLaunchKernelGGL(touch, dim3(grid), dim3(256), 0, s, buf, n, (double)i);
    }
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) {
        if (graph) CK(hipGraphLaunch(ge, s));
        else for (int i = 0; i < per; ++i) hipLaunchKernelGGL(touch, dim3(grid), dim3(256), 0, s, buf, n, (double)i);
    }
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3 / (reps * per);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    double* buf;
    const long nmax = 4l << 20;   // 32 MiB of doubles
    CK(hipMalloc(&buf, nmax * sizeof(double)));
    const long sizes[] = {1, 1l << 17, 1l << 18, 4l << 20};   // 8 B, 1 MiB, 2 MiB, 32 MiB
    for (long n : sizes)
        for (int graph = 0; graph < 2; ++graph) {
            const int grid = n < 256 ? 1 : 1024;
            printf("write %9.3f MiB  %-6s  %7.2f us per launch\n", n * 8.0 / (1 << 20), graph ? "graph" : "stream",
                   run(s, buf, n, grid, 50, graph));
        }
    for (long n : sizes)
        for (int events = 0; events < 2; ++events) {
            const int grid = n < 256 ? 1 : 1024;
            printf("write %9.3f MiB  big-args%s  %7.2f us per launch\n", n * 8.0 / (1 << 20), events ? "+events" : "       ",
                   run_big(s, buf, n, grid, 50, events));
        }
    return 0;
}
