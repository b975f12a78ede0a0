// k10s_kernels.hip — gfx950 kernels of the batched-ensemble engine.
//
//   k10s_init_kernel      one 64-lane wavefront per replica: KubernetriksSimulation::initialize
//   k10s_run_kernel       one 64-lane wavefront per replica: the dslab step loop with every
//                         handler; the scheduling hot path (Fit + LeastAllocated + argmax over the
//                         node cache) is lane-parallel, everything else wave-uniform
//   k10s_schedule_kernel  unit-parity surface: R independent schedule_one calls, one wave each
//
// No MFMA: nothing on this path is a dense contraction.  The scheduler's node cache is one packed
// u64 per node in HBM (cpu << 40 | ram: 8 B/node; the wide u32 + u64 SoA, 12 B/node, in the
// plugins copy), read coalesced (lane l reads 4 consecutive nodes per 256-node step), reductions by
// cross-lane shuffles (DPP/permlane).
// Built with -ffp-contract=off and without fast-math: the f64 score arithmetic must round exactly
// like the Rust reference (correctly rounded division, no FMA contraction).
#include <hip/hip_runtime.h>

#include <mutex>

#define K10S_KERNEL_TU 1
// The score-plugin profile path (k10s_replica_params.score_plugins other than LeastAllocated
// alone) is compiled only into the second copy of the event-loop kernels, k10s_kernels_plugins.hip
// (same code, renamed symbols); an engine launches that copy only when one of its replicas needs
// it, so the default kernel's register allocation never pays for the extension.
#ifndef K10S_SCORE_PLUGINS
#define K10S_SCORE_PLUGINS 0
#endif
// Event-time keys as the raw bit pattern (k10s_common.h total_key): this copy runs only scenarios
// whose event times carry no sign bit (make_layout: packed only when times_nonneg); the plugins
// copy keeps the full total_cmp transform.
#ifndef K10S_TIME_KEY_ID
#define K10S_TIME_KEY_ID 1
#endif
#include "k10s_engine.h"

using namespace k10s;

// Occupancy knob for the event-loop kernel (0 = compiler default).  amdgpu_waves_per_eu(n) caps
// the register allocation so that n waves fit per SIMD.
#ifndef K10S_WAVES_PER_EU
#define K10S_WAVES_PER_EU 8
#endif
#if K10S_WAVES_PER_EU > 0
#define K10S_RUN_BOUNDS __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(K10S_WAVES_PER_EU)))
#else
#define K10S_RUN_BOUNDS __launch_bounds__(64)
#endif

// Stage replica r's header between HBM and the LDS working copy k10s_hdr (dword-wise, 64 lanes).
__device__ __forceinline__ void hdr_copy(uint32_t* dst, const uint32_t* src) {
    constexpr uint32_t W = sizeof(RepHdr) / 4;
    static_assert(sizeof(RepHdr) % 4 == 0, "RepHdr must be a whole number of dwords");
    for (uint32_t i = threadIdx.x; i < W; i += 64) dst[i] = src[i];
    __syncthreads();
}
// Through the opaque constant pointer (K10S_DC): the copy-out after the event loop recomputes the
// address instead of keeping the copy-in's 4 SGPRs live (and spilled around every handler call)
// across the whole loop.
__device__ __forceinline__ uint32_t* hdr_global(uint32_t r) {
#if K10S_DEVICE
    return (uint32_t*)(K10S_DC.base + (uint64_t)r * K10S_DC.L.stride + K10S_DC.L.hdr);
#else
    return (uint32_t*)(k10s_dc.base + (uint64_t)r * k10s_dc.L.stride + k10s_dc.L.hdr);
#endif
}

// The replica's region and hot sections as absolute addresses in LDS (k10s_engine.h k10s_sec).
__device__ __forceinline__ void sec_setup(uint32_t r) {
#if K10S_DEVICE
    const uint32_t l = threadIdx.x;
    if (l < (uint32_t)K10S_NSEC) {
        const Layout& L = K10S_DC.L;
        const uint64_t b = (uint64_t)(K10S_DC.base + (uint64_t)r * L.stride);
        const uint64_t off = l == SEC_POD ? L.pod : l == SEC_NODE ? L.node : l == SEC_SLOT ? L.slot : l == SEC_FQ ? L.fq
                           : l == SEC_HEAP ? L.heap : l == SEC_SNODE ? L.s_node : l == SEC_PRES ? L.s_present
                           : l == SEC_AQ ? L.aq : l == SEC_UQ ? L.uq : 0;
        k10s_sec[l] = l == SEC_PARAMS ? (uint64_t)(K10S_DC.params + r) : b + off;
    }
    __syncthreads();
#else
    (void)r;
#endif
}

__global__ __launch_bounds__(64) void k10s_init_kernel(uint32_t n_replicas) {
    uint32_t r = blockIdx.x;
    if (r >= n_replicas) return;
    sec_setup(r);
    Ctx c;
    init_replica(c);
    __syncthreads();
    hdr_copy(hdr_global(r), (const uint32_t*)&k10s_hdr);
}

__global__ K10S_RUN_BOUNDS void k10s_run_kernel(uint32_t n_replicas, int mode, double until_time, double max_time,
                                                uint64_t budget, uint32_t* active) {
    uint32_t r = blockIdx.x;
    if (r >= n_replicas) return;
#if K10S_WALL
    // tooling builds only: launch wall-time placement of each replica (100 MHz realtime counter,
    // hardware ids) in the profile slots, for the finish-time spread of one resident round
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
#endif
    sec_setup(r);
    hdr_copy((uint32_t*)&k10s_hdr, hdr_global(r));
    Ctx c;
    int more = run_replica(c, mode, until_time, max_time, budget);
    (void)more;
#if K10S_WALL
    if (threadIdx.x == 0) {
        k10s_hdr.prof[0] = w0;
        k10s_hdr.prof[1] = __builtin_amdgcn_s_memrealtime();
        k10s_hdr.prof[2] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
        k10s_hdr.prof[3] = (uint32_t)__builtin_amdgcn_s_getreg((15 << 11) | 20);   // XCC_ID
    }
#endif
    __syncthreads();
    hdr_copy(hdr_global(r), (const uint32_t*)&k10s_hdr);
#if K10S_BEACON
    if (threadIdx.x == 0)   // word 13: the header is written back
        __hip_atomic_store(k10s_beacon + (uint64_t)r * K10S_BEACON_WORDS + 13, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    (void)active;   // the same pointer, read after the loop through the constant block
#if K10S_DEVICE
    if (more && threadIdx.x == 0) atomicAdd(K10S_DC.active, 1u);
    // a replica stopped at a capacity the reference does not have (a generated-name universe, the
    // event heap, the scheduler queues): the host recompiles the batch with it doubled and replays it
    // (k10s_host.cpp regrow)
    if (threadIdx.x == 0) {
        const uint32_t ec = k10s_hdr.error_code;
        if (ec == K10S_ERR_NAME_BOUND || ec == K10S_ERR_HEAP_FULL || ec == K10S_ERR_QUEUE_FULL) K10S_DC.active[1] = 1u;
    }
#endif
}

#ifndef K10S_PLUGINS_TU
__global__ __launch_bounds__(64) void k10s_schedule_kernel(const uint32_t* __restrict__ alloc_cpu,
                                                             const uint64_t* __restrict__ alloc_ram,
                                                             const uint64_t* __restrict__ present, uint32_t n_nodes,
                                                             uint32_t node_stride, const uint32_t* __restrict__ req_cpu,
                                                             const uint64_t* __restrict__ req_ram, double weight,
                                                             uint32_t n_problems, int32_t* out_node, int32_t* out_status) {
    uint32_t r = blockIdx.x;
    if (r >= n_problems) return;
    const uint64_t off = (uint64_t)r * node_stride;
    const uint32_t rc = req_cpu[r];
    const uint64_t rr = req_ram[r];
    int32_t chosen = -1;
    int st;
    uint32_t cnt = 0;
    for (uint32_t w = threadIdx.x; w < (n_nodes + 63) / 64; w += 64) {
        uint64_t bits = present[(off >> 6) + w];
        if ((w + 1) * 64 > n_nodes) bits &= (n_nodes & 63) ? ((1ull << (n_nodes & 63)) - 1) : ~0ull;
        cnt += (uint32_t)__popcll(bits);
    }
    cnt = wave_sum_u32(cnt);
    if (rc == 0 && rr == 0) st = K10S_SCHED_REQUESTED_RESOURCES_ARE_ZEROS;
    else if (cnt == 0) st = K10S_SCHED_NO_NODES_IN_CLUSTER;
    else st = schedule_scan(alloc_cpu + off, alloc_ram + off, present + (off >> 6), n_nodes, rc, rr, weight, &chosen);
    if (threadIdx.x == 0) {
        out_status[r] = st;
        out_node[r] = st == K10S_SCHED_OK ? chosen : -1;
    }
}

// ScorePlugin surface: out[i] = 0.0 + LeastAllocated(alloc[i], req[i]) * weight, the scheduler's
// per-plugin accumulation (kube_scheduler.rs:113-138) for one (pod, node) pair per element.
__global__ __launch_bounds__(256) void k10s_score_kernel(const uint32_t* __restrict__ alloc_cpu,
                                                         const uint64_t* __restrict__ alloc_ram,
                                                         const uint32_t* __restrict__ req_cpu,
                                                         const uint64_t* __restrict__ req_ram, double weight,
                                                         uint64_t n, double* __restrict__ out) {
#if K10S_DEVICE
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = 0.0 + la_score_d(alloc_cpu[i], alloc_ram[i], req_cpu[i], req_ram[i]) * weight;
#endif
}

#endif  // !K10S_PLUGINS_TU

// ---- launchers (called from k10s_host.cpp) -------------------------------------------------------
// The launch constants live in the one __constant__ block k10s_dc, so every engine launch first
// copies its block (from pinned host memory, stream-ordered) and then launches; engines of a device
// share one stream (k10s_host.cpp), and the mutex keeps each (copy, launch) pair adjacent in it.
static std::mutex g_launch_mu;

static hipError_t upload(const DevConst* h_dc, hipStream_t s) {
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(k10s_dc), h_dc, sizeof(DevConst), 0, hipMemcpyHostToDevice, s);
}

// The launchers take the constant block as an untyped pointer: the second copy of this file
// (k10s_kernels_plugins.hip) compiles every engine type in its own namespace, so only C-level
// types cross between the translation units.
hipError_t k10s_launch_init(const void* h_dcv, uint32_t n_replicas, hipStream_t s) {
    const DevConst* h_dc = (const DevConst*)h_dcv;
    std::lock_guard<std::mutex> g(g_launch_mu);
    hipError_t e = upload(h_dc, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k10s_init_kernel, dim3(n_replicas), dim3(64), 0, s, n_replicas);
    return hipGetLastError();
}

hipError_t k10s_launch_run(const void* h_dcv, uint32_t n_replicas, int mode, double until_time, double max_time,
                           uint64_t budget, uint32_t* d_active, hipStream_t s) {
    const DevConst* h_dc = (const DevConst*)h_dcv;
    std::lock_guard<std::mutex> g(g_launch_mu);
    hipError_t e = upload(h_dc, s);
    if (e != hipSuccess) return e;
    void* board = nullptr;
    e = hipGetSymbolAddress(&board, HIP_SYMBOL(k10s_fair_board));
    if (e == hipSuccess) e = hipMemsetAsync(board, 0, sizeof(k10s_fair_board), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k10s_run_kernel, dim3(n_replicas), dim3(64), 0, s, n_replicas, mode, until_time, max_time,
                       budget, d_active);
    return hipGetLastError();
}

#if K10S_BEACON && defined(K10S_PLUGINS_TU)
// tooling builds only: the plugins copy's beacon pointer (its own device symbol, k10s_beacon_plugins)
hipError_t k10s_beacon_set_plugins(void* d) { return hipMemcpyToSymbol(HIP_SYMBOL(k10s_beacon), &d, sizeof d); }
#endif
#if K10S_BEACON && !defined(K10S_PLUGINS_TU)
hipError_t k10s_beacon_set_plugins(void* d);
// tooling builds only: host-mapped beacon memory for n_replicas replicas; returns its host address.
// Both kernel copies get the pointer (a wide-layout or plugin engine launches the plugins copy).
extern "C" void* k10s_debug_beacon_alloc(uint32_t n_replicas) {
    void* h = nullptr;
    void* d = nullptr;
    const size_t bytes = sizeof(uint32_t) * K10S_BEACON_WORDS * (size_t)n_replicas;
    if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    memset(h, 0xFF, bytes);
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return nullptr;
    if (hipMemcpyToSymbol(HIP_SYMBOL(k10s_beacon), &d, sizeof d) != hipSuccess) return nullptr;
    if (k10s_beacon_set_plugins(d) != hipSuccess) return nullptr;
    return h;
}
#endif

#ifndef K10S_PLUGINS_TU
hipError_t k10s_launch_schedule(const uint32_t* alloc_cpu, const uint64_t* alloc_ram, const uint64_t* present,
                                uint32_t n_nodes, uint32_t node_stride, const uint32_t* req_cpu, const uint64_t* req_ram,
                                double weight, uint32_t n_problems, int32_t* out_node, int32_t* out_status,
                                hipStream_t s) {
    hipLaunchKernelGGL(k10s_schedule_kernel, dim3(n_problems), dim3(64), 0, s, alloc_cpu, alloc_ram, present, n_nodes,
                       node_stride, req_cpu, req_ram, weight, n_problems, out_node, out_status);
    return hipGetLastError();
}

hipError_t k10s_launch_score(const uint32_t* alloc_cpu, const uint64_t* alloc_ram, const uint32_t* req_cpu,
                             const uint64_t* req_ram, double weight, uint64_t n, double* out, hipStream_t s) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k10s_score_kernel, dim3((uint32_t)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, s, alloc_cpu,
                       alloc_ram, req_cpu, req_ram, weight, n, out);
    return hipGetLastError();
}
#endif  // !K10S_PLUGINS_TU
