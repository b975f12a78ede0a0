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
#define K10S_UNROLL _Pragma("unroll")
#else
#define K10S_UNROLL
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
// K10S_TIME_KEY_ID = 1: the key is the value's bit pattern itself.  For every value without the
// sign bit (+0.0 ... +inf, positive NaNs) total_cmp's transform is the identity, and -0.0 maps to
// INT64_MIN, still below all of them; only two distinct negative values (or negative NaNs) would
// compare the wrong way round.  The default event-loop kernel (k10s_kernels.hip) is compiled with 1
// and runs only scenarios whose every event time is such a value: trace timestamps, durations,
// network delays and tick intervals carry no sign (times_nonneg, k10s_builder.cpp), so every
// clock + delay is one too; any other scenario runs the second kernel copy, compiled with 0 (the
// full transform).  Saves the transform's five VALU instructions on every key (emit, consume, the
// heap's sift steps, the source list): C3 1,297 -> 1,280 ms, profiles/r03_k1_time_key_ab.json.
#ifndef K10S_TIME_KEY_ID
#define K10S_TIME_KEY_ID 0
#endif
K10S_HD int64_t total_key(double x) {
    int64_t b = (int64_t)f2u(x);
#if !K10S_TIME_KEY_ID
    b ^= (int64_t)(((uint64_t)(b >> 63)) >> 1);
#endif
    return b;
}
// Unsigned key, monotone for non-NaN scores (argmax of LeastAllocated scores).  Never 0 for a
// non-NaN input, so 0 doubles as "no candidate".
K10S_HD uint64_t score_key(double x) {
    uint64_t b = f2u(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// Histogram bin of an estimator value (K10S_HIST_BINS log2 bins, include/k10s.h).
K10S_HD uint32_t hist_bin(double x) {
    if (!(x >= 0.0009765625)) return 0;  // < 2^-10, NaN
    const int32_t e = (int32_t)((f2u(x) >> 52) & 0x7FF) - 1023;
    return e >= 20 ? 31u : (uint32_t)(e + 11);
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
// K10S_LANE_OPAQUE: the lane index is re-read at each use (an empty asm the compiler cannot hoist),
// so lane-dependent masks are recomputed where needed instead of being held in SGPR pairs across
// the event loop (where they are spilled around every out-of-line handler call).  Tuning knob.
#ifndef K10S_LANE_OPAQUE
#define K10S_LANE_OPAQUE 1   // C3 +1.7 % (profiles/r02_v13_sgpr_live_ab.json)
#endif
K10S_HD int lane_id() {
#if K10S_DEVICE
#if K10S_LANE_OPAQUE
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return (int)(t & 63);
#else
    return (int)(threadIdx.x & 63);
#endif
#else
    return 0;
#endif
}

#if K10S_DEVICE
// Cross-lane exchange without LDS: DPP and gfx950 permlane swaps (VALU only; __shfl_xor would be
// ds_bpermute through the LDS crossbar, ~100 cycles per step).  Step S pairs each lane with one
// partner; xpair<S>(v, a, b) returns the two values of the pair (own and partner, in some order),
// so combining a and b with a commutative, associative operation and repeating for S = 0..k-1
// leaves every lane of each 2^(k+1)-lane group with the group's reduction:
//   S=0 quad xor 1, S=1 quad xor 2, S=2 half-row mirror (8 lanes), S=3 row mirror (16 lanes),
//   S=4 permlane16 swap (32 lanes), S=5 permlane32 swap (64 lanes).
template <int S>
K10S_D void xpair(uint32_t v, uint32_t& a, uint32_t& b) {
    if constexpr (S < 4) {
        constexpr int ctrl = S == 0 ? 0xB1 : S == 1 ? 0x4E : S == 2 ? 0x141 : 0x140;
        a = v;
        b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, 0xF, 0xF, false);
    } else if constexpr (S == 4) {
        auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        a = r[0];
        b = r[1];
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        a = r[0];
        b = r[1];
    }
}
K10S_D uint64_t join64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// one reduction step of a lexicographic (key, idx) max
template <int S>
K10S_D void argmax_step(uint64_t& key, int32_t& idx) {
    uint32_t la, lb, ha, hb, ia, ib;
    xpair<S>((uint32_t)key, la, lb);
    xpair<S>((uint32_t)(key >> 32), ha, hb);
    xpair<S>((uint32_t)idx, ia, ib);
    const uint64_t ka = join64(la, ha), kb = join64(lb, hb);
    const bool tb = kb > ka || (kb == ka && (int32_t)ib > (int32_t)ia);
    key = tb ? kb : ka;
    idx = (int32_t)(tb ? ib : ia);
}
// one reduction step of a lexicographic (key signed 64, seq, payload) min
template <int S>
K10S_D void keymin_step(int64_t& key, uint32_t& seq, uint32_t& pay) {
    uint32_t la, lb, ha, hb, sa, sb, pa, pb;
    xpair<S>((uint32_t)(uint64_t)key, la, lb);
    xpair<S>((uint32_t)((uint64_t)key >> 32), ha, hb);
    xpair<S>(seq, sa, sb);
    xpair<S>(pay, pa, pb);
    const int64_t ka = (int64_t)join64(la, ha), kb = (int64_t)join64(lb, hb);
    const bool tb = kb < ka || (kb == ka && sb < sa);
    key = tb ? kb : ka;
    seq = tb ? sb : sa;
    pay = tb ? pb : pa;
}
#endif

// Reduce (key, idx) to the lexicographic max over the wave; every lane gets the result.
K10S_HD void wave_argmax(uint64_t& key, int32_t& idx) {
#if K10S_DEVICE
    argmax_step<0>(key, idx);
    argmax_step<1>(key, idx);
    argmax_step<2>(key, idx);
    argmax_step<3>(key, idx);
    argmax_step<4>(key, idx);
    argmax_step<5>(key, idx);
#else
    (void)key;
    (void)idx;
#endif
}
#if K10S_DEVICE
template <int S>
K10S_D uint32_t max_step(uint32_t v) {
    uint32_t a, b;
    xpair<S>(v, a, b);
    return a > b ? a : b;
}
template <int S>
K10S_D int32_t min_step_i32(int32_t v) {
    uint32_t a, b;
    xpair<S>((uint32_t)v, a, b);
    return (int32_t)a < (int32_t)b ? (int32_t)a : (int32_t)b;
}
template <int S>
K10S_D uint32_t sum_step(uint32_t v) {
    uint32_t a, b;
    xpair<S>(v, a, b);
    return a + b;
}
template <int S>
K10S_D uint64_t max_step64(uint64_t v) {
    uint32_t la, lb, ha, hb;
    xpair<S>((uint32_t)v, la, lb);
    xpair<S>((uint32_t)(v >> 32), ha, hb);
    const uint64_t a = join64(la, ha), b = join64(lb, hb);
    return a > b ? a : b;
}
#endif
K10S_HD uint32_t wave_max_u32(uint32_t v) {
#if K10S_DEVICE
    v = max_step<0>(v); v = max_step<1>(v); v = max_step<2>(v);
    v = max_step<3>(v); v = max_step<4>(v); v = max_step<5>(v);
#endif
    return v;
}
K10S_HD uint64_t wave_max_u64(uint64_t v) {
#if K10S_DEVICE
    v = max_step64<0>(v); v = max_step64<1>(v); v = max_step64<2>(v);
    v = max_step64<3>(v); v = max_step64<4>(v); v = max_step64<5>(v);
#endif
    return v;
}
K10S_HD bool wave_any(bool b) {
#if K10S_DEVICE
    return __ballot(b) != 0;
#else
    return b;
#endif
}
K10S_HD int32_t wave_min_i32(int32_t v) {
#if K10S_DEVICE
    v = min_step_i32<0>(v); v = min_step_i32<1>(v); v = min_step_i32<2>(v);
    v = min_step_i32<3>(v); v = min_step_i32<4>(v); v = min_step_i32<5>(v);
#endif
    return v;
}
K10S_HD uint32_t wave_sum_u32(uint32_t v) {
#if K10S_DEVICE
    v = sum_step<0>(v); v = sum_step<1>(v); v = sum_step<2>(v);
    v = sum_step<3>(v); v = sum_step<4>(v); v = sum_step<5>(v);
#endif
    return v;
}
K10S_HD uint64_t wave_or_u64(uint64_t v) {   // every lane gets the OR over the wave
#if K10S_DEVICE
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32), a, b;
    xpair<0>(lo, a, b); lo = a | b; xpair<0>(hi, a, b); hi = a | b;
    xpair<1>(lo, a, b); lo = a | b; xpair<1>(hi, a, b); hi = a | b;
    xpair<2>(lo, a, b); lo = a | b; xpair<2>(hi, a, b); hi = a | b;
    xpair<3>(lo, a, b); lo = a | b; xpair<3>(hi, a, b); hi = a | b;
    xpair<4>(lo, a, b); lo = a | b; xpair<4>(hi, a, b); hi = a | b;
    xpair<5>(lo, a, b); lo = a | b; xpair<5>(hi, a, b); hi = a | b;
    return join64(lo, hi);
#else
    return v;
#endif
}
// Make a value provably wave-uniform for the compiler (it already is by construction).
K10S_HD uint32_t uniform_u32(uint32_t v) {
#if K10S_DEVICE
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
#else
    return v;
#endif
}
K10S_HD uint64_t uniform_u64(uint64_t v) {
    return (uint64_t)uniform_u32((uint32_t)v) | ((uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32);
}
K10S_HD double uniform_f64(double v) { return u2f(uniform_u64(f2u(v))); }
K10S_HD void wave_sync() {
#if K10S_DEVICE
    __syncthreads();  // one wavefront per workgroup: orders cross-lane global writes (cheap)
#endif
}

}  // namespace k10s
