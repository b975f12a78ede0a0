// k10s_host.cpp — C ABI (include/k10s.h) of the MI355X engine: scenario compilation, device
// memory, launches, result readback.  Requires a HIP device; there is no CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/k10s.h"
#include "k10s_builder.h"
#include "k10s_front_check.h"
#include "k10s_results.h"

using namespace k10s;

hipError_t k10s_launch_init(const void* h_dc, uint32_t n_replicas, hipStream_t s);
hipError_t k10s_launch_run(const void* h_dc, uint32_t n_replicas, int mode, double until_time, double max_time,
                           uint64_t budget, uint32_t* d_active, hipStream_t s);
// the same two kernels with the score-plugin profile path compiled in (k10s_kernels_plugins.hip)
hipError_t k10s_launch_init_plugins(const void* h_dc, uint32_t n_replicas, hipStream_t s);
hipError_t k10s_launch_run_plugins(const void* h_dc, uint32_t n_replicas, int mode, double until_time,
                                   double max_time, uint64_t budget, uint32_t* d_active, hipStream_t s);
hipError_t k10s_launch_schedule(const uint32_t* alloc_cpu, const uint64_t* alloc_ram, const uint64_t* present,
                                uint32_t n_nodes, uint32_t node_stride, const uint32_t* req_cpu, const uint64_t* req_ram,
                                double weight, uint32_t n_problems, int32_t* out_node, int32_t* out_status,
                                hipStream_t s);
hipError_t k10s_launch_score(const uint32_t* alloc_cpu, const uint64_t* alloc_ram, const uint32_t* req_cpu,
                             const uint64_t* req_ram, double weight, uint64_t n, double* out, hipStream_t s);

namespace {
thread_local std::string g_err;

int32_t set_err(int32_t code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(x)                                                                           \
    do {                                                                                    \
        hipError_t _e = (x);                                                                \
        if (_e != hipSuccess) return set_err(K10S_E_HIP, std::string(#x ": ") + hipGetErrorString(_e)); \
    } while (0)
}  // namespace

// Everything one compiled batch owns on the device and the host.  Kept apart from the handle so a
// regrown batch (more generated names, see regrow below) can take the handle's place in one swap.
struct EngineCore {
    HostScenario hs;
    Scenario dsc;       // device view
    Layout L;
    uint32_t R = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    void* d_scen = nullptr;
    uint8_t* d_state = nullptr;
    Params* d_params = nullptr;
    uint32_t* d_active = nullptr;  // [0] replicas with work left, [1] a replica stopped at a name bound
    uint32_t* h_active = nullptr;  // pinned
    RepHdr* h_hdr = nullptr;       // pinned staging for the replica headers (results / profile readback),
                                   // allocated at create; hdr_mu serializes its fill-and-read
    DevConst* h_dc = nullptr;      // pinned launch constants
    std::vector<Params> params;
    bool plugins = false;          // some replica's profile is not LeastAllocated alone
    bool wide = false;             // launch the wide-cache kernel copy (k10s_kernels_plugins.hip): a
                                   // plugin replica, or a node cache that is not packed (L.packed == 0)
};

// One call that advanced the replicas since the last initialize: a regrown batch replays them.
struct RunCall {
    int32_t mode;
    double until_time, max_time;
    uint64_t budget;
    bool single;   // one launch (k10s_engine_step_async) rather than a launch loop (k10s_engine_run)
};

struct k10s_engine : EngineCore {
    std::mutex hdr_mu;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // what the batch was compiled from (a regrow recompiles it with larger name universes)
    std::string text;
    std::vector<uint8_t> blob;
    k10s_capacities caps;
    std::vector<RunCall> history;
    uint32_t regrows = 0;   // batches recompiled by regrow since create
};

// All engines of a device launch on one stream: the launch constants are one __constant__ block per
// device (k10s_kernels.hip), so launches of different engines must not overlap.
static hipStream_t engine_stream(int device) {
    static std::mutex mu;
    static std::vector<hipStream_t> streams;
    std::lock_guard<std::mutex> g(mu);
    if ((int)streams.size() <= device) streams.resize(device + 1, nullptr);
    if (!streams[device] && hipStreamCreateWithFlags(&streams[device], hipStreamNonBlocking) != hipSuccess)
        streams[device] = nullptr;
    return streams[device];
}

static void core_free(EngineCore& e) {
    (void)hipSetDevice(e.device);
    if (e.d_scen) (void)hipFree(e.d_scen);
    if (e.d_state) (void)hipFree(e.d_state);
    if (e.d_params) (void)hipFree(e.d_params);
    if (e.d_active) (void)hipFree(e.d_active);
    if (e.h_active) (void)hipHostFree(e.h_active);
    if (e.h_hdr) (void)hipHostFree(e.h_hdr);
    if (e.h_dc) (void)hipHostFree(e.h_dc);
    e.d_scen = nullptr;
    e.d_state = nullptr;
    e.d_params = nullptr;
    e.d_active = e.h_active = nullptr;
    e.h_hdr = nullptr;
    e.h_dc = nullptr;   // e.stream is the device's shared engine stream: not destroyed
}

static void engine_free(k10s_engine* e) {
    if (!e) return;
    core_free(*e);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    delete e;
}

// A failed regrow that had to release the replaced batch's state leaves the engine without one.
static int32_t live(const EngineCore& e) {
    if (e.d_state) return K10S_OK;
    return set_err(K10S_E_CAPACITY, "engine state was released by a regrow that then failed (device memory); "
                                    "destroy the engine");
}

static int32_t core_init(EngineCore& e) {
    if (int32_t rc = live(e)) return rc;
    HIPCHK(hipSetDevice(e.device));
    HIPCHK(hipMemsetAsync(e.d_active, 0, 8, e.stream));
    HIPCHK((e.wide ? k10s_launch_init_plugins : k10s_launch_init)(e.h_dc, e.R, e.stream));
    HIPCHK(hipStreamSynchronize(e.stream));
    return K10S_OK;
}

// Compile the scenario and allocate + initialize the batch.  params: n_replicas entries, or NULL for
// the scenario defaults.  Returns K10S_OK or an error code (message in g_err); on failure the core
// holds nothing the caller must free beyond what core_free releases.
// reclaim (a regrow only): the batch this one replaces.  When the new replica state does not fit
// the free device memory beside reclaim's but fits in its place, reclaim's state is freed first
// (reclaim->d_state becomes NULL: the caller's results are then lost if this create fails).
static int32_t core_create(EngineCore& e, const char* text, const uint8_t* blob, uint64_t blob_len,
                           const k10s_replica_params* params, uint32_t n_replicas, const k10s_capacities& c,
                           int32_t device, EngineCore* reclaim = nullptr) {
    e.device = device;
    e.R = n_replicas;
    std::string err;
    if (!build_scenario(text, c.group_name_bound, c.ca_name_bound, e.hs, err, blob, blob_len))
        return set_err(K10S_E_INVALID, "scenario: " + err);
    e.params.resize(n_replicas);
    for (uint32_t r = 0; r < n_replicas; r++) {
        if (params) {
            e.params[r] = params[r];
        } else {
            e.params[r] = e.hs.defaults;
            e.params[r].seed = e.hs.defaults.seed + r;
        }
        e.params[r].ca_max_node_count = e.hs.defaults.ca_max_node_count;  // fixed by the node pool
        if (e.params[r].score_plugins != K10S_SCORE_LEAST_ALLOCATED) e.plugins = true;
        const std::string perr = params_error(e.params[r], e.hs);
        if (!perr.empty()) return set_err(K10S_E_INVALID, "params[" + std::to_string(r) + "]: " + perr);
    }
    // the node cache is packed unless some replica needs the wide SoA (k10s_capacities.node_cache)
    const bool tnn = times_nonneg(e.hs, e.params.data(), n_replicas);
    e.L = make_layout(e.hs, c, !e.plugins && tnn, tnn);
    e.wide = e.plugins || !e.L.packed;
    if (hipSetDevice(device) != hipSuccess) return set_err(K10S_E_HIP, "hipSetDevice");
    if (!(e.stream = engine_stream(device))) return set_err(K10S_E_HIP, "hipStreamCreate");
    Scenario offs;
    std::vector<uint8_t> img = pack_scenario(e.hs, offs);
    if (hipMalloc(&e.d_scen, img.size()) != hipSuccess) return set_err(K10S_E_HIP, "hipMalloc scenario");
    if (hipMemcpy(e.d_scen, img.data(), img.size(), hipMemcpyHostToDevice) != hipSuccess)
        return set_err(K10S_E_HIP, "upload scenario");
    e.dsc = rebase_scenario(offs, (const uint8_t*)e.d_scen);
    size_t bytes = (size_t)e.L.stride * n_replicas;
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    const size_t old_b = (reclaim && reclaim->d_state) ? (size_t)reclaim->L.stride * reclaim->R : 0;
    const size_t here_b = free_b;   // free beside the batch being replaced
    free_b += old_b;                // ... and in its place
    if (bytes + (64ull << 20) > free_b && c.delay_fifo == 0 && e.L.cap_fq > 512) {
        // the default rings grow with the node count (up to 8 x 8,192 x 32 B = 2 MiB per replica): when
        // that does not fit, fall back to 512-entry rings (a fuller ring only spills to the heap)
        k10s_capacities c512 = c;
        c512.delay_fifo = 512;
        e.L = make_layout(e.hs, c512, !e.plugins && tnn, tnn);
        bytes = (size_t)e.L.stride * n_replicas;
    }
    if (bytes + (64ull << 20) > free_b)
        return set_err(K10S_E_CAPACITY, "replica state (" + std::to_string(bytes >> 20) + " MiB) exceeds free device memory");
    if (old_b && bytes + (64ull << 20) > here_b) {   //  room only in the replaced batch's place
        (void)hipFree(reclaim->d_state);
        reclaim->d_state = nullptr;
    }
    if (hipMalloc(&e.d_state, bytes) != hipSuccess) return set_err(K10S_E_HIP, "hipMalloc replica state");
    if (hipMalloc(&e.d_params, sizeof(Params) * n_replicas) != hipSuccess) return set_err(K10S_E_HIP, "hipMalloc params");
    if (hipMemcpy(e.d_params, e.params.data(), sizeof(Params) * n_replicas, hipMemcpyHostToDevice) != hipSuccess)
        return set_err(K10S_E_HIP, "upload params");
    if (hipMalloc(&e.d_active, 64) != hipSuccess) return set_err(K10S_E_HIP, "hipMalloc active");
    if (hipHostMalloc(&e.h_active, 64) != hipSuccess) return set_err(K10S_E_HIP, "hipHostMalloc");
    std::memset(e.h_active, 0, 64);
    if (hipHostMalloc(&e.h_hdr, sizeof(RepHdr) * (size_t)e.R) != hipSuccess) return set_err(K10S_E_HIP, "hipHostMalloc");
    if (hipHostMalloc(&e.h_dc, sizeof(DevConst)) != hipSuccess) return set_err(K10S_E_HIP, "hipHostMalloc");
    std::memset(e.h_dc, 0, sizeof(DevConst));
    e.h_dc->sc = e.dsc;
    e.h_dc->L = e.L;
    e.h_dc->params = e.d_params;
    e.h_dc->base = e.d_state;
    e.h_dc->active = e.d_active;
    return core_init(e);
}

// One launch over every replica (no sync); h_active[0..1] receive the launch's flags when it is done.
static int32_t core_launch(EngineCore& e, const RunCall& rc) {
    if (int32_t r = live(e)) return r;
    HIPCHK(hipSetDevice(e.device));
    HIPCHK(hipMemsetAsync(e.d_active, 0, 4, e.stream));   // word 1 (a growable stop) stays set until a regrow
    HIPCHK((e.wide ? k10s_launch_run_plugins : k10s_launch_run)(e.h_dc, e.R, rc.mode, rc.until_time, rc.max_time,
                                                                 rc.budget, e.d_active, e.stream));
    HIPCHK(hipMemcpyAsync(e.h_active, e.d_active, 8, hipMemcpyDeviceToHost, e.stream));
    return K10S_OK;
}

// One recorded call: a single launch, or launches until no replica has work left.
static int32_t core_call(EngineCore& e, const RunCall& rc) {
    for (;;) {
        int32_t r = core_launch(e, rc);
        if (r != K10S_OK) return r;
        HIPCHK(hipStreamSynchronize(e.stream));
        if (rc.single || rc.budget == 0 || e.h_active[0] == 0) return K10S_OK;
    }
}

// All replica headers into the engine's pinned staging buffer (one strided DMA; a pageable
// destination would be copied through a bounce buffer).  The caller holds e->hdr_mu across the fill
// and its reads of h_hdr, so concurrent read-back calls on one engine do not interleave.
static int32_t read_all_hdrs(EngineCore* e) {
    if (int32_t rc = live(*e)) return rc;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpy2DAsync(e->h_hdr, sizeof(RepHdr), e->d_state + e->L.hdr, e->L.stride, sizeof(RepHdr), e->R,
                            hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return K10S_OK;
}

// Engine capacities the reference does not have.  The reference's containers grow without a bound:
// the event queue (dslab-core's BinaryHeap), the active queue and the unschedulable map
// (scheduler.rs:45, 49), and the generated names — the HPA's pods "{group}_{total_created}"
// (kube_horizontal_pod_autoscaler.rs:178-182, api_server.rs:421) and the cluster autoscaler's nodes
// "{group}_{k}" (kube_cluster_autoscaler.rs).  The engine sizes each replica's state ahead of time
// (name rank = index; k10s_capacities), and a replica that outgrows one of them stops
// with K10S_ERR_HEAP_FULL, K10S_ERR_QUEUE_FULL or K10S_ERR_NAME_BOUND.  The run kernel flags such a
// stop (active word 1); this recompiles the batch with every exhausted capacity doubled and replays
// every call since the last initialize on it, until no replica stops there.  Every replica is
// deterministic, so the others come out identical; the handle keeps its identity (name tables and
// replica_bytes may grow).  A capacity at its maximum (2^20 names per universe, 2^30 heap or queue
// entries) is left as the replica's error.
// Memory: the regrown batch is allocated beside the current one when both fit, else in its place
// (core_create's reclaim); if it fits neither way the engine keeps the stopped results and the run
// returns K10S_E_CAPACITY.  K10S_ERR_CA_BUFFER is not regrown: its buffers are sized from the node
// pool and the pod count (cap_act >= max(ca_max_node_count, N) + 16 actions per decision, cap_undo =
// P + 16 moved pods), which no decision can exceed, so it marks a broken invariant, not a limit.
#define K10S_NAME_BOUND_MAX (1u << 20)
#define K10S_QUEUE_CAP_MAX (1u << 30)
static uint32_t grow2(uint32_t cur, uint32_t floor_, uint32_t max_) {
    return std::min<uint32_t>(2 * std::max<uint32_t>(cur, floor_), max_);
}
static int32_t regrow(k10s_engine* e) {
    for (;;) {
        if (e->h_active[1] == 0) return K10S_OK;
        bool grow_ca = false, grow_group = false, grow_heap = false, grow_queue = false;
        {
            std::lock_guard<std::mutex> g(e->hdr_mu);
            int32_t rc = read_all_hdrs(e);
            if (rc != K10S_OK) return rc;
            for (uint32_t r = 0; r < e->R; r++) {
                const uint32_t code = e->h_hdr[r].error_code;
                if (code == K10S_ERR_NAME_BOUND) {
                    if (e->h_hdr[r].error_kind == K10S_EV_PS_CA_REQ) grow_ca = true;
                    else grow_group = true;
                } else if (code == K10S_ERR_HEAP_FULL) {
                    grow_heap = true;
                } else if (code == K10S_ERR_QUEUE_FULL) {
                    grow_queue = true;
                }
            }
        }
        k10s_capacities c = e->caps;   // the batch's effective capacities
        c.group_name_bound = e->hs.group_bound;
        c.ca_name_bound = e->hs.ca_bound;
        c.event_heap = e->L.cap_heap;
        c.active_queue = e->L.cap_aq;
        c.unschedulable = e->L.cap_uq;
        bool grown = false;
        if (grow_group && c.group_name_bound < K10S_NAME_BOUND_MAX) {
            c.group_name_bound = grow2(c.group_name_bound, 32, K10S_NAME_BOUND_MAX);
            grown = true;
        }
        if (grow_ca && c.ca_name_bound < K10S_NAME_BOUND_MAX) {
            c.ca_name_bound = grow2(c.ca_name_bound, 32, K10S_NAME_BOUND_MAX);
            grown = true;
        }
        if (grow_heap && c.event_heap < K10S_QUEUE_CAP_MAX) {
            c.event_heap = grow2(c.event_heap, 64, K10S_QUEUE_CAP_MAX);
            grown = true;
        }
        if (grow_queue && (c.active_queue < K10S_QUEUE_CAP_MAX || c.unschedulable < K10S_QUEUE_CAP_MAX)) {
            c.active_queue = grow2(c.active_queue, 16, K10S_QUEUE_CAP_MAX);   // (which one filled is not
            c.unschedulable = grow2(c.unschedulable, 16, K10S_QUEUE_CAP_MAX);  // recorded: both grow)
            grown = true;
        }
        if (!grown) {   // every stop is at a maximum: they stay the replicas' errors
            e->h_active[1] = 0;
            HIPCHK(hipSetDevice(e->device));
            HIPCHK(hipMemsetAsync(e->d_active + 1, 0, 4, e->stream));
            return K10S_OK;
        }
        EngineCore n;
        int32_t rc = core_create(n, e->text.c_str(), e->blob.empty() ? nullptr : e->blob.data(), e->blob.size(),
                                 e->params.data(), e->R, c, e->device, e);
        for (size_t i = 0; rc == K10S_OK && i < e->history.size(); i++) rc = core_call(n, e->history[i]);
        if (rc != K10S_OK) {
            const std::string m = g_err;
            core_free(n);
            if (e->d_state) {   // the stopped batch is intact: keep its results readable
                e->h_active[1] = 0;
                (void)hipMemsetAsync(e->d_active + 1, 0, 4, e->stream);
            }
            return set_err(rc, "regrow: " + m);
        }
        std::lock_guard<std::mutex> g(e->hdr_mu);
        std::swap(static_cast<EngineCore&>(*e), n);
        core_free(n);
        e->caps = c;
        e->regrows += 1;
    }
}

extern "C" {

const char* k10s_last_error(void) { return g_err.c_str(); }
#ifndef K10S_BUILD_ID
#define K10S_BUILD_ID "dev"
#endif
const char* k10s_version(void) { return "k10s-mi355x 0.2 (gfx950) build " K10S_BUILD_ID; }

int32_t k10s_schedule_one_batch(const uint32_t* alloc_cpu, const uint64_t* alloc_ram, const uint64_t* present_bits,
                                uint32_t n_nodes, uint32_t node_stride, const uint32_t* req_cpu, const uint64_t* req_ram,
                                double weight, uint32_t n_problems, int32_t* out_node, int32_t* out_status,
                                void* stream) {
    if (n_problems == 0) return K10S_OK;
    if (!alloc_cpu || !alloc_ram || !present_bits || !req_cpu || !req_ram || !out_node || !out_status)
        return set_err(K10S_E_INVALID, "null pointer");
    if (node_stride % 64 != 0 || node_stride < n_nodes) return set_err(K10S_E_INVALID, "node_stride must be a multiple of 64 and >= n_nodes");
    if (((uintptr_t)alloc_cpu & 15) || ((uintptr_t)alloc_ram & 15) || ((uintptr_t)present_bits & 7))
        return set_err(K10S_E_INVALID, "alloc_cpu / alloc_ram must be 16-byte aligned (present_bits 8-byte)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return set_err(K10S_E_NO_DEVICE, "no HIP device");
    HIPCHK(k10s_launch_schedule(alloc_cpu, alloc_ram, present_bits, n_nodes, node_stride, req_cpu, req_ram, weight,
                                n_problems, out_node, out_status, (hipStream_t)stream));
    return K10S_OK;
}

int32_t k10s_score_batch(const uint32_t* alloc_cpu, const uint64_t* alloc_ram, const uint32_t* req_cpu,
                         const uint64_t* req_ram, double weight, uint64_t n, double* out_score, void* stream) {
    if (n == 0) return K10S_OK;
    if (!alloc_cpu || !alloc_ram || !req_cpu || !req_ram || !out_score) return set_err(K10S_E_INVALID, "null pointer");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return set_err(K10S_E_NO_DEVICE, "no HIP device");
    HIPCHK(k10s_launch_score(alloc_cpu, alloc_ram, req_cpu, req_ram, weight, n, out_score, (hipStream_t)stream));
    return K10S_OK;
}

}  // extern "C"

struct k10s_scheduler {
    int device = 0;
    uint32_t max_nodes = 0, max_problems = 0, stride = 0;
    hipStream_t stream = nullptr;
    uint32_t* d_cpu = nullptr;
    uint64_t* d_ram = nullptr;
    uint64_t* d_bits = nullptr;
    uint32_t* d_rc = nullptr;
    uint64_t* d_rr = nullptr;
    int32_t* d_out = nullptr;  // [2 * max_problems]: node, status
};

static void scheduler_free(k10s_scheduler* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    for (void* p : {(void*)s->d_cpu, (void*)s->d_ram, (void*)s->d_bits, (void*)s->d_rc, (void*)s->d_rr, (void*)s->d_out})
        if (p) (void)hipFree(p);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

static int32_t scheduler_alloc(k10s_scheduler* s) {
    HIPCHK(hipSetDevice(s->device));
    HIPCHK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    const uint64_t cells = (uint64_t)s->stride * s->max_problems;
    HIPCHK(hipMalloc(&s->d_cpu, 4 * cells));
    HIPCHK(hipMalloc(&s->d_ram, 8 * cells));
    HIPCHK(hipMalloc(&s->d_bits, cells / 8));
    HIPCHK(hipMalloc(&s->d_rc, 4ull * s->max_problems));
    HIPCHK(hipMalloc(&s->d_rr, 8ull * s->max_problems));
    HIPCHK(hipMalloc(&s->d_out, 8ull * s->max_problems));
    return K10S_OK;
}

extern "C" {

k10s_scheduler* k10s_scheduler_create(uint32_t max_nodes, uint32_t max_problems, int32_t device) {
    if (max_nodes == 0 || max_problems == 0) {
        set_err(K10S_E_INVALID, "max_nodes and max_problems must be > 0");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_err(K10S_E_NO_DEVICE, "no HIP device: the k10s scheduler runs only on the GPU");
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        set_err(K10S_E_INVALID, "device index out of range");
        return nullptr;
    }
    auto* s = new k10s_scheduler();
    s->device = device;
    s->max_nodes = max_nodes;
    s->max_problems = max_problems;
    s->stride = (max_nodes + 63) / 64 * 64;
    if (scheduler_alloc(s) != K10S_OK) {
        std::string m = g_err;
        scheduler_free(s);
        set_err(K10S_E_CAPACITY, m);
        return nullptr;
    }
    return s;
}

void k10s_scheduler_destroy(k10s_scheduler* s) { scheduler_free(s); }

int32_t k10s_scheduler_schedule(k10s_scheduler* s, const uint32_t* alloc_cpu, const uint64_t* alloc_ram,
                                const uint64_t* present_bits, uint32_t n_nodes, const uint32_t* req_cpu,
                                const uint64_t* req_ram, double weight, uint32_t n_problems, int32_t* out_node,
                                int32_t* out_status) {
    if (!s) return set_err(K10S_E_INVALID, "null scheduler");
    if (n_problems == 0) return K10S_OK;
    if (!alloc_cpu || !alloc_ram || !req_cpu || !req_ram || !out_node || !out_status)
        return set_err(K10S_E_INVALID, "null pointer");
    if (n_nodes > s->max_nodes || n_problems > s->max_problems)
        return set_err(K10S_E_CAPACITY, "n_nodes/n_problems exceed the scheduler's capacity");
    HIPCHK(hipSetDevice(s->device));
    const uint32_t words = (n_nodes + 63) / 64, dwords = s->stride / 64;
    if (n_nodes > 0) {
        HIPCHK(hipMemcpy2DAsync(s->d_cpu, 4ull * s->stride, alloc_cpu, 4ull * n_nodes, 4ull * n_nodes, n_problems,
                                hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipMemcpy2DAsync(s->d_ram, 8ull * s->stride, alloc_ram, 8ull * n_nodes, 8ull * n_nodes, n_problems,
                                hipMemcpyHostToDevice, s->stream));
        if (present_bits) {
            HIPCHK(hipMemcpy2DAsync(s->d_bits, 8ull * dwords, present_bits, 8ull * words, 8ull * words, n_problems,
                                    hipMemcpyHostToDevice, s->stream));
        } else {
            HIPCHK(hipMemsetAsync(s->d_bits, 0xFF, 8ull * dwords * n_problems, s->stream));
        }
    }
    HIPCHK(hipMemcpyAsync(s->d_rc, req_cpu, 4ull * n_problems, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(s->d_rr, req_ram, 8ull * n_problems, hipMemcpyHostToDevice, s->stream));
    HIPCHK(k10s_launch_schedule(s->d_cpu, s->d_ram, s->d_bits, n_nodes, s->stride, s->d_rc, s->d_rr, weight, n_problems,
                                s->d_out, s->d_out + s->max_problems, s->stream));
    HIPCHK(hipMemcpyAsync(out_node, s->d_out, 4ull * n_problems, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipMemcpyAsync(out_status, s->d_out + s->max_problems, 4ull * n_problems, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return K10S_OK;
}

k10s_engine* k10s_engine_create(const char* scenario_text, const k10s_replica_params* params, uint32_t n_replicas,
                                const k10s_capacities* caps, int32_t device) {
    return k10s_engine_create_bulk(scenario_text, nullptr, 0, params, n_replicas, caps, device);
}

k10s_engine* k10s_engine_create_bulk(const char* scenario_text, const void* pods_blob, uint64_t blob_len,
                                     const k10s_replica_params* params, uint32_t n_replicas,
                                     const k10s_capacities* caps, int32_t device) {
    if (!scenario_text || n_replicas == 0) {
        set_err(K10S_E_INVALID, "scenario_text is NULL or n_replicas == 0");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_err(K10S_E_NO_DEVICE, "no HIP device: the k10s engine runs only on the GPU");
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        set_err(K10S_E_INVALID, "device index out of range");
        return nullptr;
    }
    auto* e = new k10s_engine();
    std::memset(&e->caps, 0, sizeof e->caps);
    if (caps) e->caps = *caps;
    e->text = scenario_text;
    if (pods_blob && blob_len) e->blob.assign((const uint8_t*)pods_blob, (const uint8_t*)pods_blob + blob_len);
    const int32_t rc = core_create(*e, scenario_text, e->blob.empty() ? nullptr : e->blob.data(), e->blob.size(),
                                   params, n_replicas, e->caps, device);
    if (rc == K10S_OK) {
        (void)hipEventCreate(&e->ev0);
        (void)hipEventCreate(&e->ev1);
        return e;
    }
    const std::string m = g_err;
    engine_free(e);
    set_err(rc, m);
    return nullptr;
}

void k10s_engine_destroy(k10s_engine* e) { engine_free(e); }

int32_t k10s_engine_default_params(const k10s_engine* e, k10s_replica_params* out) {
    if (!e || !out) return set_err(K10S_E_INVALID, "null");
    *out = e->hs.defaults;
    return K10S_OK;
}

int32_t k10s_engine_reset(k10s_engine* e) {
    if (!e) return set_err(K10S_E_INVALID, "null");
    e->history.clear();
    return core_init(*e);
}

int32_t k10s_engine_step_async(k10s_engine* e, int32_t mode, double until_time, double max_time,
                               uint64_t max_events_per_launch) {
    if (!e) return set_err(K10S_E_INVALID, "null");
    if (mode != K10S_RUN_UNTIL_ALL_FINISHED && mode != K10S_RUN_UNTIL_TIME) return set_err(K10S_E_INVALID, "bad mode");
    const RunCall rc{mode, until_time, max_time, max_events_per_launch, true};
    e->history.push_back(rc);
    return core_launch(*e, rc);
}

int32_t k10s_engine_sync(k10s_engine* e) {
    if (!e) return set_err(K10S_E_INVALID, "null");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    return regrow(e);
}

int32_t k10s_engine_run(k10s_engine* e, int32_t mode, double until_time, double max_time,
                        uint64_t max_events_per_launch, double* elapsed_ms) {
    if (!e) return set_err(K10S_E_INVALID, "null");
    if (mode != K10S_RUN_UNTIL_ALL_FINISHED && mode != K10S_RUN_UNTIL_TIME) return set_err(K10S_E_INVALID, "bad mode");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipEventRecord(e->ev0, e->stream));
    const RunCall rc{mode, until_time, max_time, max_events_per_launch, false};
    e->history.push_back(rc);
    int32_t r = core_call(*e, rc);
    if (r == K10S_OK) r = regrow(e);
    if (r != K10S_OK) return r;
    HIPCHK(hipEventRecord(e->ev1, e->stream));
    HIPCHK(hipEventSynchronize(e->ev1));
    if (elapsed_ms) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e->ev0, e->ev1));
        *elapsed_ms = ms;
    }
    return K10S_OK;
}

int32_t k10s_engine_results(const k10s_engine* ce, k10s_replica_result* out) {
    if (!ce || !out) return set_err(K10S_E_INVALID, "null");
    k10s_engine* e = const_cast<k10s_engine*>(ce);
    std::lock_guard<std::mutex> g(e->hdr_mu);
    int32_t rc = read_all_hdrs(e);
    if (rc != K10S_OK) return rc;
    for (uint32_t r = 0; r < e->R; r++) hdr_to_result(e->h_hdr[r], out[r]);
    return K10S_OK;
}

int32_t k10s_engine_profile(const k10s_engine* ce, uint64_t* out) {
    if (!ce || !out) return set_err(K10S_E_INVALID, "null");
    k10s_engine* e = const_cast<k10s_engine*>(ce);
    std::lock_guard<std::mutex> g(e->hdr_mu);
    int32_t rc = read_all_hdrs(e);
    if (rc != K10S_OK) return rc;
    for (uint32_t r = 0; r < e->R; r++)
        for (int i = 0; i < K10S_PROF_SLOTS; i++) out[(size_t)r * K10S_PROF_SLOTS + i] = e->h_hdr[r].prof[i];
    return K10S_OK;
}

uint32_t k10s_engine_profile_width(void) { return K10S_PROF_SLOTS; }

static int32_t read_hdr(const k10s_engine* e, uint32_t r, RepHdr& h) {
    if (r >= e->R) return set_err(K10S_E_INVALID, "replica index out of range");
    if (int32_t rc = live(*e)) return rc;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpy(&h, e->d_state + (size_t)r * e->L.stride + e->L.hdr, sizeof h, hipMemcpyDeviceToHost));
    return K10S_OK;
}

int32_t k10s_engine_event_log(const k10s_engine* e, uint32_t r, k10s_log_entry* out, uint32_t cap, uint32_t* n) {
    if (!e || !n) return set_err(K10S_E_INVALID, "null");
    RepHdr h;
    int32_t rc = read_hdr(e, r, h);
    if (rc) return rc;
    uint32_t k = e->L.cap_log ? (h.log_n < cap ? h.log_n : cap) : 0;
    if (k) HIPCHK(hipMemcpy(out, e->d_state + (size_t)r * e->L.stride + e->L.log, sizeof(k10s_log_entry) * k,
                            hipMemcpyDeviceToHost));
    *n = k;
    return K10S_OK;
}

int32_t k10s_engine_gauges(const k10s_engine* e, uint32_t r, k10s_gauge_row* out, uint32_t cap, uint32_t* n) {
    if (!e || !n) return set_err(K10S_E_INVALID, "null");
    RepHdr h;
    int32_t rc = read_hdr(e, r, h);
    if (rc) return rc;
    uint32_t k = e->L.cap_gauge ? (h.gauge_n < cap ? h.gauge_n : cap) : 0;
    if (k) HIPCHK(hipMemcpy(out, e->d_state + (size_t)r * e->L.stride + e->L.gauge, sizeof(k10s_gauge_row) * k,
                            hipMemcpyDeviceToHost));
    *n = k;
    return K10S_OK;
}

int32_t k10s_engine_placements(const k10s_engine* e, uint32_t r, k10s_placement* out, uint32_t cap, uint32_t* n) {
    if (!e || !n) return set_err(K10S_E_INVALID, "null");
    RepHdr h;
    int32_t rc = read_hdr(e, r, h);
    if (rc) return rc;
    uint32_t k = e->L.cap_place ? (h.place_n < cap ? h.place_n : cap) : 0;
    if (k) HIPCHK(hipMemcpy(out, e->d_state + (size_t)r * e->L.stride + e->L.place, sizeof(k10s_placement) * k,
                            hipMemcpyDeviceToHost));
    *n = k;
    return K10S_OK;
}

int32_t k10s_engine_pod_records(const k10s_engine* e, uint32_t r, k10s_pod_record* out, uint32_t cap, uint32_t* n) {
    if (!e || !n) return set_err(K10S_E_INVALID, "null");
    if (r >= e->R) return set_err(K10S_E_INVALID, "replica index out of range");
    if (int32_t rc = live(*e)) return rc;
    uint32_t k = e->L.rec_on ? (e->hs.n_pods < cap ? e->hs.n_pods : cap) : 0;
    HIPCHK(hipSetDevice(e->device));
    if (k) HIPCHK(hipMemcpy(out, e->d_state + (size_t)r * e->L.stride + e->L.prec, sizeof(k10s_pod_record) * k,
                            hipMemcpyDeviceToHost));
    *n = k;
    return K10S_OK;
}

int32_t k10s_engine_group_sizes(const k10s_engine* e, uint32_t r, uint32_t* created, uint32_t* total, uint32_t cap,
                                uint32_t* n) {
    if (!e || !n) return set_err(K10S_E_INVALID, "null");
    if (r >= e->R) return set_err(K10S_E_INVALID, "replica index out of range");
    if (int32_t rc = live(*e)) return rc;
    uint32_t G = (uint32_t)e->hs.group_names.size();
    uint32_t k = G < cap ? G : cap;
    std::vector<GroupState> gs(G);
    HIPCHK(hipSetDevice(e->device));
    if (G) HIPCHK(hipMemcpy(gs.data(), e->d_state + (size_t)r * e->L.stride + e->L.grp, sizeof(GroupState) * G,
                            hipMemcpyDeviceToHost));
    for (uint32_t g = 0; g < k; g++) {
        created[g] = gs[g].registered ? gs[g].created_count : 0;
        total[g] = gs[g].total_created;
    }
    *n = k;
    return K10S_OK;
}

uint32_t k10s_engine_num_nodes(const k10s_engine* e) { return e ? e->hs.n_nodes : 0; }
uint32_t k10s_engine_num_pods(const k10s_engine* e) { return e ? e->hs.n_pods : 0; }
uint32_t k10s_engine_num_groups(const k10s_engine* e) { return e ? (uint32_t)e->hs.group_names.size() : 0; }
const char* k10s_engine_node_name(const k10s_engine* e, uint32_t i) {
    return (e && i < e->hs.n_nodes) ? e->hs.node_names[i].c_str() : "";
}
const char* k10s_engine_pod_name(const k10s_engine* e, uint32_t i) {
    return (e && i < e->hs.n_pods) ? e->hs.pod_names[i].c_str() : "";
}
const char* k10s_engine_group_name(const k10s_engine* e, uint32_t i) {
    return (e && i < e->hs.group_names.size()) ? e->hs.group_names[i].c_str() : "";
}
uint64_t k10s_engine_replica_bytes(const k10s_engine* e) { return e ? e->L.stride : 0; }
int32_t k10s_engine_name_bounds(const k10s_engine* e, uint32_t* group_bound, uint32_t* ca_bound) {
    if (!e || !group_bound || !ca_bound) return set_err(K10S_E_INVALID, "null");
    *group_bound = e->hs.group_bound;
    *ca_bound = e->hs.ca_bound;
    return K10S_OK;
}
int32_t k10s_engine_check_fronts(const k10s_engine* e, uint32_t replica, int32_t* result) {
    if (!e || !result) return set_err(K10S_E_INVALID, "null");
    RepHdr h;
    if (int32_t rc = read_hdr(e, replica, h)) return rc;
    *result = 0;
    if (!e->L.front) return K10S_OK;
    const uint32_t N = e->dsc.n_nodes;
    const uint32_t nb = std::min<uint32_t>((N + 63u) / 64u, 64u);
    std::vector<uint64_t> sn(N), fv((size_t)nb * K10S_FR_K);
    std::vector<uint8_t> fi((size_t)nb * K10S_FR_K);
    const uint8_t* base = e->d_state + (size_t)replica * e->L.stride;
    HIPCHK(hipMemcpy(sn.data(), base + e->L.s_node, 8 * (size_t)N, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(fv.data(), base + e->L.fr_val, 8 * fv.size(), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(fi.data(), base + e->L.fr_idx, fi.size(), hipMemcpyDeviceToHost));
    *result = k10s_front_check(sn.data(), fv.data(), fi.data(), N, h.fr_dirty, h.fr_over, K10S_FR_K);
    return K10S_OK;
}
uint32_t k10s_engine_node_entry_bytes(const k10s_engine* e) { return e ? (e->L.packed ? 8u : 12u) : 0u; }
int32_t k10s_engine_capacities(const k10s_engine* e, k10s_capacities* out, uint32_t* regrows) {
    if (!e || !out) return set_err(K10S_E_INVALID, "null");
    *out = e->caps;
    out->event_heap = e->L.cap_heap;
    out->active_queue = e->L.cap_aq;
    out->unschedulable = e->L.cap_uq;
    out->group_name_bound = e->hs.group_bound;
    out->ca_name_bound = e->hs.ca_bound;
    out->delay_fifo = e->L.cap_fq ? e->L.cap_fq : K10S_FIFO_OFF;
    if (regrows) *regrows = e->regrows;
    return K10S_OK;
}

}  // extern "C"
