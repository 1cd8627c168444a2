// wave_ops.h -- register-only cross-lane reductions for gfx950 (CDNA4, wave64).
//
// gsum<LPS>(v) is an ALL-reduce (sum) over aligned groups of LPS lanes (16, 32 or 64) that never
// touches the LDS crossbar:
//   * within each 16-lane DPP row: a rotate-and-add butterfly (row_ror:8,4,2,1);
//   * across rows: v_permlane16_swap (rows 0<->1, 2<->3) and v_permlane32_swap (halves), both new
//     in gfx950, each followed by one add.
// Every step adds two partials that are the same pair of values in both lanes that hold them
// (IEEE addition is commutative), so every lane of a group ends with the SAME bits, and the
// summation tree is fixed (deterministic run to run).
#pragma once
#include <hip/hip_runtime.h>

namespace phg {

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// rows (0,1) and (2,3) exchanged: returns own + partner-row value, same bits in both rows
__device__ __forceinline__ double swap16_add(double v) {
#pragma clang fp contract(off)
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}

__device__ __forceinline__ double swap32_add(double v) {
#pragma clang fp contract(off)
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}

// all-reduce over groups of LPS lanes; K independent values interleaved for ILP
//
// Contraction is OFF here: a partial that is a single product (farmer's coupling row: one entry per
// lane) would otherwise be fused into the first DPP add -- fma(a_i, b_i, round(a_j b_j)) in lane i,
// fma(a_j, b_j, round(a_i b_i)) in lane j -- and the lanes of a group would disagree in the last bit,
// then on the restart / termination decisions that every lane takes from these sums (round 6: a
// farmer 10k prox-QP ran to the 2e5-iteration cap at a gap its split group could no longer close)
template <int LPS, int K>
__device__ __forceinline__ void gsum_many(double (&v)[K]) {
#pragma clang fp contract(off)
    static_assert(LPS == 16 || LPS == 32 || LPS == 64, "group of 16, 32 or 64 lanes");
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_d<0x128>(v[k]);   // row_ror:8
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_d<0x124>(v[k]);   // row_ror:4
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_d<0x122>(v[k]);   // row_ror:2
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_d<0x121>(v[k]);   // row_ror:1
    if constexpr (LPS >= 32) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = swap16_add(v[k]);
    }
    if constexpr (LPS >= 64) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = swap32_add(v[k]);
    }
}

template <int LPS>
__device__ __forceinline__ double gsum(double v) {
    double t[1] = {v};
    gsum_many<LPS, 1>(t);
    return t[0];
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) {
    return fmin(fmax(v, lo), hi);
}

// clamp by compare + select: no NaN canonicalisation of the (loop-invariant) bounds on every use,
// which IEEE-mode fmin/fmax pay; a NaN v passes through (the KKT test catches it)
__device__ __forceinline__ double clamp_sel(double v, double lo, double hi) {
    v = v < lo ? lo : v;
    return v > hi ? hi : v;
}

// raw v_max_f64 / v_min_f64: IEEE-mode fmax/fmin must quiet signalling NaNs, so the compiler
// re-canonicalises every operand it cannot prove canonical (loop-carried bounds included: one
// extra v_max_f64 per operand per use).  Our operands come from arithmetic or are finite/inf
// bounds, never sNaN, so the bare instructions are exact here.
__device__ __forceinline__ double vmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmin(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// opaque to the optimiser: stops loop-invariant code motion from hoisting address arithmetic /
// loads used only by the rarely-run check and epilogue code into registers held across the
// hot loop
template <class T>
__device__ __forceinline__ T launder(T v) {
    asm volatile("" : "+v"(v));
    return v;
}

// compiler-only memory barrier: orders the surrounding memory accesses as written
__device__ __forceinline__ void seq() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ bool fin(double v) { return fabs(v) < 1e300; }

// wave-uniform "any lane true"
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

}  // namespace phg
