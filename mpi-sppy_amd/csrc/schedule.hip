// schedule.hip -- the scenario launch order for the next batched solve, on its own launch (one
// 1 024-thread workgroup; the sort itself is schedule.h).  Stream-ordered behind the solve, no host
// round trip.  On one GPU with the folded update, shards of <= 16 384 scenarios, the pipelined
// node-sum launch carries the same sort as an extra 256-thread workgroup instead (ph_update.hip
// node_sums_kernel HEADX, phg_api.hip sched_pending), so no launch of its own is paid there.
#include "schedule.h"

namespace phg {

__global__ __launch_bounds__(1024) void schedule_kernel(const int* iters, int S, int unit, int* order) {
    __shared__ int cnt[kSchedBuckets];
    __shared__ int wsum[16];
    schedule_block<1024, 1>(iters, S, unit, order, cnt, wsum);
}

hipError_t schedule_launch(const int* iters, int S, int unit, int* order, hipStream_t st) {
    hipLaunchKernelGGL(schedule_kernel, dim3(1), dim3(1024), 0, st, iters, S, unit > 0 ? unit : 1, order);
    return hipGetLastError();
}

}  // namespace phg
