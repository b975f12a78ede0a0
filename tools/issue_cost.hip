// tools/issue_cost.hip — VALU issue cost per instruction kind on gfx950 (tooling, not product).
//
// One launch per kind: 256 CUs x 32 waves (8 per SIMD, the engine's occupancy), each wave runs
// ITER iterations of a block of 16 independent instructions of that kind (8 accumulator chains of
// 2, so issue — not dependency latency — bounds it).  SIMD cycles per instruction =
// kernel time x clock / (instructions per SIMD).  Build: hipcc --offload-arch=gfx950 -O3
// tools/issue_cost.hip -o build/issue_cost; run: build/issue_cost (prints one JSON line).
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITER 4096

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ __launch_bounds__(64) void cost_kernel(float* out, int n) {
    // 8 independent 64-bit register pairs per lane
    double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
    for (int it = 0; it < n; it++) {
#define OPF64ADD(i) asm volatile("v_add_f64 %0, %0, %0" : "+v"(d##i));
#define OPF64FMA(i) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d##i));
#define OPRCP(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(d##i));
#define OPADD32(i) asm volatile("v_add_u32 %0, %0, %0" : "+v"(*((int*)&d##i)));
#define OPSHR64(i) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(d##i));
#define OPCMP64(i) asm volatile("v_cmp_lt_i64 vcc, %0, %0" : : "v"(d##i) : "vcc");
#define OPRFL(i) { int s_; asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(s_) : "v"(*((int*)&d##i))); }
#define OPDPP(i) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(*((int*)&d##i)));
#define OPCVT(i) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d##i) : "v"(*((int*)&d##i)));
#define OPMUL32(i) asm volatile("v_mul_lo_u32 %0, %0, %0" : "+v"(*((int*)&d##i)));
        if constexpr (K == 0) { REP8(OPF64ADD) REP8(OPF64ADD) }
        if constexpr (K == 1) { REP8(OPF64FMA) REP8(OPF64FMA) }
        if constexpr (K == 2) { REP8(OPRCP) REP8(OPRCP) }
        if constexpr (K == 3) { REP8(OPADD32) REP8(OPADD32) }
        if constexpr (K == 4) { REP8(OPSHR64) REP8(OPSHR64) }
        if constexpr (K == 5) { REP8(OPCMP64) REP8(OPCMP64) }
        if constexpr (K == 6) { REP8(OPRFL) REP8(OPRFL) }
        if constexpr (K == 7) { REP8(OPDPP) REP8(OPDPP) }
        if constexpr (K == 8) { REP8(OPCVT) REP8(OPCVT) }
        if constexpr (K == 9) { REP8(OPMUL32) REP8(OPMUL32) }
    }
    out[blockIdx.x * 64 + threadIdx.x] = (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
}

template <int K>
static float run(float* out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(cost_kernel<K>, dim3(blocks), dim3(64), 0, 0, out, 16);  // warm up
    hipEventRecord(a);
    hipLaunchKernelGGL(cost_kernel<K>, dim3(blocks), dim3(64), 0, 0, out, ITER);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const int blocks = 256 * 32;  // 8 waves per SIMD
    float* out;
    hipMalloc(&out, blocks * 64 * sizeof(float));
    const char* names[] = {"v_add_f64", "v_fma_f64", "v_rcp_f64", "v_add_u32", "v_lshrrev_b64", "v_cmp_lt_i64",
                           "v_readfirstlane_b32", "v_mov_b32_dpp", "v_cvt_f64_u32", "v_mul_lo_u32"};
    float ms[10];
    ms[0] = run<0>(out, blocks);
    ms[1] = run<1>(out, blocks);
    ms[2] = run<2>(out, blocks);
    ms[3] = run<3>(out, blocks);
    ms[4] = run<4>(out, blocks);
    ms[5] = run<5>(out, blocks);
    ms[6] = run<6>(out, blocks);
    ms[7] = run<7>(out, blocks);
    ms[8] = run<8>(out, blocks);
    ms[9] = run<9>(out, blocks);
    // instructions per SIMD = waves per SIMD (8) x ITER x 16; cycles at the clock the run reports
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    printf("{\"clock_mhz\": %.0f, \"waves_per_simd\": 8, \"cycles_per_wave64_instr\": {", clk_khz / 1e3);
    for (int k = 0; k < 10; k++) {
        const double cyc = ms[k] * 1e-3 * clk_khz * 1e3 / (8.0 * ITER * 16);
        printf("%s\"%s\": %.2f", k ? ", " : "", names[k], cyc);
    }
    printf("}}\n");
    return 0;
}
