// k10s_common.h — shared definitions for the MI355X batched-ensemble engine.
//
// The per-replica simulation (k10s_engine.h) is written once as __host__ __device__ code:
//   * on gfx950 one 64-lane wavefront owns one replica (K10S_LANES = 64).  Event handling is
//     executed wave-uniformly (every lane computes the same values; stores of equal values to
//     equal addresses coalesce), and the node scans of the scheduling hot path are split over
//     the 64 lanes with DPP/ds_swizzle shuffles for the reductions;
//   * the host-side check build (tests/hostcheck) compiles the same code with one lane so the
//     engine's logic can be diffed against the CPU oracle without a GPU.  It is test-only and
//     is never reachable from the product C ABI (include/k10s.h), which requires a GPU.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define K10S_HD __host__ __device__ __forceinline__
#define K10S_D __device__ __forceinline__
#define K10S_HD_NOINL __host__ __device__ __attribute__((noinline)) inline
#define K10S_HD_FLEX __host__ __device__
#else
#define K10S_HD inline
#define K10S_D inline
#define K10S_HD_NOINL inline
#define K10S_HD_FLEX inline
#endif

// Device-side inlining policy (tuning knob, semantics-neutral): K10S_SPLIT >= 1 keeps the cold
// handlers (autoscalers, metrics) out of line, >= 2 also the api-server / storage / node handlers,
// >= 3 also the queue/heap helpers, so the hot loop's register allocation is not sized by them.
#ifndef K10S_SPLIT
#define K10S_SPLIT 2
#endif
// K10S_COLD / K10S_WARM / K10S_HELPER: function qualifiers following K10S_SPLIT
#if K10S_SPLIT >= 1
#define K10S_COLD K10S_HD_NOINL
#else
#define K10S_COLD K10S_HD
#endif
#if K10S_SPLIT >= 2
#define K10S_WARM K10S_HD_NOINL
#else
#define K10S_WARM K10S_HD
#endif
#if K10S_SPLIT >= 3
#define K10S_HELPER K10S_HD_NOINL
#else
#define K10S_HELPER K10S_HD
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define K10S_DEVICE 1
#define K10S_LANES 64
#else
#define K10S_DEVICE 0
#define K10S_LANES 1
#endif

namespace k10s {

// ---- bit casts -------------------------------------------------------------------------------
K10S_HD uint64_t f2u(double x) {
#if K10S_DEVICE
    return (uint64_t)__double_as_longlong(x);
#else
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
#endif
}
K10S_HD double u2f(uint64_t u) {
#if K10S_DEVICE
    return __longlong_as_double((long long)u);
#else
    double x;
    memcpy(&x, &u, 8);
    return x;
#endif
}
K10S_HD bool is_nan(double x) { return x != x; }

// Rust f64::total_cmp key: monotone in the IEEE total order (core/num/f64.rs).
K10S_HD int64_t total_key(double x) {
    int64_t b = (int64_t)f2u(x);
    b ^= (int64_t)(((uint64_t)(b >> 63)) >> 1);
    return b;
}
// Unsigned key, monotone for non-NaN scores (argmax of LeastAllocated scores).  Never 0 for a
// non-NaN input, so 0 doubles as "no candidate".
K10S_HD uint64_t score_key(double x) {
    uint64_t b = f2u(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// Rust `as` casts
K10S_HD uint64_t f64_as_u64(double x) {
    if (is_nan(x) || x <= 0.0) return 0;
    if (x >= 18446744073709551616.0) return ~0ull;
    return (uint64_t)x;
}
K10S_HD double fmin_rs(double a, double b) {  // f64::min: NaN-ignoring
    if (is_nan(a)) return b;
    if (is_nan(b)) return a;
    return a < b ? a : b;
}
K10S_HD double fmax_rs(double a, double b) {
    if (is_nan(a)) return b;
    if (is_nan(b)) return a;
    return a > b ? a : b;
}

// ---- lanes -----------------------------------------------------------------------------------
K10S_HD int lane_id() {
#if K10S_DEVICE
    return (int)(threadIdx.x & 63);
#else
    return 0;
#endif
}

#if K10S_DEVICE
K10S_D uint64_t shfl_xor_u64(uint64_t v, int m) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = (uint32_t)__shfl_xor((int)lo, m, 64);
    hi = (uint32_t)__shfl_xor((int)hi, m, 64);
    return ((uint64_t)hi << 32) | lo;
}
#endif

// Reduce (key, idx) to the lexicographic max over the wave; every lane gets the result.
K10S_HD void wave_argmax(uint64_t& key, int32_t& idx) {
#if K10S_DEVICE
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t ok = shfl_xor_u64(key, m);
        int32_t oi = __shfl_xor(idx, m, 64);
        if (ok > key || (ok == key && oi > idx)) {
            key = ok;
            idx = oi;
        }
    }
#else
    (void)key;
    (void)idx;
#endif
}
K10S_HD int32_t wave_min_i32(int32_t v) {
#if K10S_DEVICE
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        int32_t o = __shfl_xor(v, m, 64);
        v = o < v ? o : v;
    }
#endif
    return v;
}
K10S_HD uint32_t wave_sum_u32(uint32_t v) {
#if K10S_DEVICE
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
#endif
    return v;
}
// Make a value provably wave-uniform for the compiler (it already is by construction).
K10S_HD uint32_t uniform_u32(uint32_t v) {
#if K10S_DEVICE
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
#else
    return v;
#endif
}
K10S_HD void wave_sync() {
#if K10S_DEVICE
    __syncthreads();  // one wavefront per workgroup: orders cross-lane global writes (cheap)
#endif
}

}  // namespace k10s
