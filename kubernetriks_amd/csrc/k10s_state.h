// k10s_state.h — device-resident layout of a compiled scenario and of per-replica state.
//
// Scenario tables (read-only, shared by every replica on a GPU) are indexed by name rank:
// node index n = rank of the node's name among all node names, pod index p = rank of the pod's
// name among all pod names (byte order, == Rust String order).  So "iterate n ascending" is the
// BTreeMap<String, Node> order the reference's scheduler scans, and "iterate p ascending" is the
// BTreeSet<String> order of its pod sets.  A unified rank u covers node and pod names together
// (the api server keeps pod names in its node-removal set, api_server.rs:343).
//
// Per-replica state is one contiguous region per replica (stride = Layout::stride), SoA inside:
// the scheduler cache (s_cpu u32[N], s_ram u64[N], s_present bit[N]) is the hot scan target,
// 12 B/node + 1 bit, read coalesced by the 64 lanes of the replica's wavefront.
#pragma once

#include "../../include/k10s.h"
#include "../../include/k10s_events.h"
#include "k10s_common.h"

// Device address spaces (gfx950): the compiled scenario is immutable for a launch, so its tables
// are read through constant-address-space pointers (scalar loads through the scalar cache when
// the index is wave-uniform); per-replica state is global memory.  Host code (and the device pass
// of the host-only translation units) sees plain pointers of the same size.
#if K10S_DEVICE && defined(K10S_KERNEL_TU)
#define K10S_RO(T) const __attribute__((address_space(4))) T*
#define K10S_GB(T) __attribute__((address_space(1))) T*
#else
#define K10S_RO(T) const T*
#define K10S_GB(T) T*
#endif

namespace k10s {

struct TraceEv {          // one client-emitted trace event (simulator.rs:234-253)
    double time;
    uint32_t seq;         // dslab event id: 2 + position in (cluster trace ++ workload trace), both
                          // stable-sorted by timestamp (generic.rs:78, 105)
    uint32_t kind;        // K10S_EV_AS_* kind delivered to the api server
    uint32_t arg;         // node def / node idx / pod idx / group idx
    uint32_t wpos;        // workload event: its position in the trace file (generation order);
                          // cluster event: K10S_TRACE_CLUSTER
};
#define K10S_TRACE_CLUSTER 0xFFFFFFFFu

enum : uint8_t {
    POD_HAS_DEF = 1,      // created by the trace or a pod group (else: only named by remove_pod)
    POD_HAS_DUR = 2,      // running_duration is Some
    POD_PERTURB = 4,      // trace pod: subject to seed perturbation
};
enum : uint8_t { GF_HAS_TCPU = 1, GF_HAS_TRAM = 2, GF_TMPL_HAS_DUR = 4 };
enum : uint8_t { MODEL_NONE = 0, MODEL_CONSTANT = 1, MODEL_POD_GROUP = 2 };

struct Scenario {
    uint32_t n_nodes, n_pods, n_uids, n_defs, n_slots, n_pool, n_default, n_trace;
    uint32_t n_groups, n_ca_groups, group_bound, ca_bound, n_units;
    uint32_t ca_enabled, hpa_enabled;
    uint32_t first_dynamic_seq;
    uint32_t n_cluster_trace, n_workload_trace;
    uint64_t total_pods_in_trace, total_nodes_in_trace;

    K10S_RO(uint32_t) node_uid;      // [N]
    K10S_RO(uint32_t) def_node;      // [D] node idx of node instance def
    K10S_RO(uint32_t) def_cpu;       // [D] capacity
    K10S_RO(uint64_t) def_ram;
    K10S_RO(int32_t) def_ca_group;   // [D] "node_group" label -> CA group idx (-1 none, -2 unknown)
    K10S_RO(uint8_t) def_ca_origin;  // [D] label origin == "cluster autoscaler"
    K10S_RO(uint32_t) pod_uid;       // [P]
    K10S_RO(uint32_t) pod_cpu;       // [P] requests
    K10S_RO(uint64_t) pod_ram;
    K10S_RO(double) pod_dur;
    K10S_RO(uint8_t) pod_flags;
    K10S_RO(int32_t) pod_group;      // [P] pod group idx or -1
    K10S_RO(uint32_t) pod_key;       // [P] perturbation key (workload-trace position)
    K10S_RO(uint32_t) default_defs;  // [n_default] defs of default-cluster nodes, slot order
    K10S_RO(TraceEv) trace;          // [n_trace] merged (time, seq) order
    K10S_RO(uint32_t) wl_pods_upto;  // [n_workload_trace + 1] create_pod events among the first k

    // pod groups (name order)
    K10S_RO(uint32_t) g_initial;
    K10S_RO(uint32_t) g_max;
    K10S_RO(uint32_t) g_cpu;
    K10S_RO(uint64_t) g_ram;
    K10S_RO(uint8_t) g_flags;
    K10S_RO(double) g_tcpu;
    K10S_RO(double) g_tram;
    K10S_RO(uint8_t) g_cpu_kind;
    K10S_RO(uint8_t) g_ram_kind;
    K10S_RO(double) g_cpu_usage;
    K10S_RO(double) g_ram_usage;
    K10S_RO(uint32_t) g_cpu_uoff;
    K10S_RO(uint32_t) g_cpu_ucnt;
    K10S_RO(uint32_t) g_ram_uoff;
    K10S_RO(uint32_t) g_ram_ucnt;
    K10S_RO(uint32_t) g_pod;         // [G*group_bound] pod idx of "{g}_{k}"
    K10S_RO(uint32_t) g_pos;         // [G*group_bound] name-order position of k within the group
    K10S_RO(uint32_t) g_sorted_k;    // [G*group_bound] k at name-order position j
    K10S_RO(double) unit_dur;
    K10S_RO(double) unit_load;

    // cluster-autoscaler node groups (name order; cluster_autoscaler.rs:175-200)
    K10S_RO(uint8_t) ca_has_max;
    K10S_RO(uint64_t) ca_max;
    K10S_RO(uint32_t) ca_def;        // [CG*ca_bound] def of "{group}_{k}", k = 1..ca_bound
    K10S_RO(uint32_t) ca_cpu;
    K10S_RO(uint64_t) ca_ram;
};

// Replica parameters as consumed by the device (k10s_replica_params with derived fields).
typedef k10s_replica_params Params;

struct Estimator {          // `average` 0.15 concatenate!(Min, Max, Mean, Variance) + log2 bins
    uint64_t n;
    double mn, mx, avg, sum2;
    uint32_t hist[K10S_HIST_BINS];
};
K10S_HD void est_reset(Estimator& e) {
    e.n = 0;
    e.mn = __builtin_inf();
    e.mx = -__builtin_inf();
    e.avg = 0.0;
    e.sum2 = 0.0;
    for (int i = 0; i < K10S_HIST_BINS; i++) e.hist[i] = 0;
}
K10S_HELPER void est_add(Estimator& e, double x) {
    e.hist[hist_bin(x)] += 1;
    e.mn = fmin_rs(e.mn, x);
    e.mx = fmax_rs(e.mx, x);
    e.n += 1;
    double nf = (double)e.n;
    double delta_n = (x - e.avg) / nf;
    e.avg += delta_n;
    e.sum2 += delta_n * delta_n * nf * (nf - 1.0);
}

struct HeapEv {             // dslab Event {id, time, dst, data}, 32 B
    double time;
    uint32_t seq;
    uint16_t kind;
    int16_t slot;           // node component for N_* kinds
    uint32_t a;             // pod idx / node idx / group idx
    uint32_t b;             // node idx / def id / alloc cpu / flags
    double x;               // event time field (assign/finish/removal/add/start) or alloc ram bits
};

// Delay-class FIFOs of the event queue (k10s_engine.h): events emitted with the same constant
// delay are emitted in (time, id) order, so each class is an already-sorted run.
#define K10S_NFQ 8
#define K10S_NSRC (K10S_NFQ + 2)   // the FIFO classes, the trace stream, the heap
// One entry of the sorted source list: the head (time key, id) of event source `src`.
struct SrcEnt {
    int64_t key;
    uint32_t seq;
    uint32_t src;
};
// The head of every delay-class ring lives in the working header (LDS on the device): ring
// positions [fq.head, fq.wend) are held in a K10S_FQW-entry window, the rest in the HBM ring, and a
// drained window is refilled K10S_FQW entries at a time by one lane-parallel load.
#ifndef K10S_FQW
#define K10S_FQW 4
#endif
static_assert((K10S_FQW & (K10S_FQW - 1)) == 0 && K10S_FQW <= 64, "K10S_FQW: power of two <= 64");
// The top levels of the event heap (K10S_HEAP_TOP entries: 1 + 64 at the default arity 64) live in
// the working header too; the HBM heap array holds positions >= K10S_HEAP_TOP only.
// Arity of the dslab event heap (k10s_engine.h): 8 (top 3 levels in LDS) or 16 / 32 / 64 (top 2
// levels in LDS; a level's children are loaded by that many lanes at once).
#ifndef K10S_HEAP_D
#define K10S_HEAP_D 64
#endif
#if K10S_HEAP_D == 8
#define K10S_HEAP_TOP 73
#else
#define K10S_HEAP_TOP (1 + K10S_HEAP_D)
#endif
static_assert(K10S_HEAP_D == 8 || K10S_HEAP_D == 16 || K10S_HEAP_D == 32 || K10S_HEAP_D == 64, "K10S_HEAP_D");

struct QInfo {              // QueuedPodInfo (queue.rs:13-27), 24 B
    double timestamp;
    double initial;
    uint32_t attempts;
    uint32_t pod;
};
// The scheduler's action queue (Rust BinaryHeap restatement, k10s_engine.h aq_*): positions
// [0, K10S_AQ_TOP) (the top levels of the binary heap) live in the working header (LDS on the
// device), the rest in the replica's HBM array.  0 = all in HBM.  Default 15 (levels 0-3, 360 B of
// LDS): pops and pushes of the cycle's queue touch HBM only below level 3 (profiles/r02_v5_knobs_ab.json).
#ifndef K10S_AQ_TOP
#define K10S_AQ_TOP 15
#endif

#ifndef K10S_PROF
#define K10S_PROF 0
#endif
#define K10S_PROF_KIND0 16   // prof[16 + k]: dispatch cycles of kind k; prof[16 + 46 + k]: count
#if K10S_PROF
#define K10S_PROF_SLOTS (K10S_PROF_KIND0 + 2 * K10S_EV_NUM_KINDS)
#else
#define K10S_PROF_SLOTS 8
#endif

// One delay-class ring's counters, read together (one 16-B LDS read for head / tail / window end).
struct alignas(16) FqRing {
    uint32_t head, tail;   // ring positions (wrapping counters)
    uint32_t wend;         // the LDS window holds positions [head, wend)
    uint32_t pad;
    double last;           // time of the newest entry (the run stays sorted)
    double pad2;
};
static_assert(sizeof(FqRing) == 32, "FqRing must be 32 B");

#define K10S_FR_K 8   // front slots per 64-node block of the packed node cache (k10s_engine.h front_scan)

struct RepHdr {
    double clock;            // clock, next_seq and error_code: one 16-B LDS read in emit
    uint32_t next_seq;
    uint32_t error_code;
    uint32_t trace_cursor;
    uint32_t heap_size;
    uint32_t aq_size;
    uint32_t uq_size;
    uint32_t s_node_count;
    uint32_t ps_node_count;
    uint32_t as_node_count;
    uint32_t pool_head;
    uint32_t pool_count;
    uint32_t status;
    uint32_t error_kind;
    uint32_t error_seq;
    double error_time;
    uint64_t counters[K10S_NUM_COUNTERS];
    Estimator est[3];
    double ca_last_cycle_time;
    uint32_t ca_n_act;
    uint32_t log_n;
    uint32_t place_n;
    uint32_t flags;
    uint32_t unsched_cache_count;
    uint32_t cur_kind, cur_seq;   // event being handled (panic attribution)
    uint32_t gauge_n;             // gauge rows recorded
    uint64_t g_cur_nodes, g_cur_pods, g_pods_q;   // GaugeMetrics counters (collector.rs:169-190)
    // event queue: delay-class FIFO rings (head/tail counters, newest time; a non-empty ring's head
    // entry is fq_win[ring * K10S_FQW + (fq[ring].head & (K10S_FQW - 1))]) and the cached root of the
    // heap (valid while heap_size > 0)
    FqRing fq[K10S_NFQ];
    HeapEv heap_top;
    HeapEv cur_ev;                // a trace event being handled (passed to its handler by reference)
    double tr_time;               // cached head of the shared trace stream (valid while
    uint32_t tr_seq;              // trace_cursor < n_trace)
    uint32_t run_flags;           // this launch: bit 0 runs allowed (no event budget), bit 1 until-time mode
    double run_limit;             // this launch's time limit (until_time or max_time): window events stay below
    uint32_t trace_prefix;        // workload events at file positions >= this are not in this
                                  // replica's trace (k10s_replica_params.workload_prefix; ~0 = all)
    uint32_t tr_skip;             // workload events skipped so far: the replica's id of a later
                                  // workload event is its scenario id minus tr_skip
    int64_t pods_left;            // total_pods_in_trace - terminated_pods (the termination rule)
    // the event sources' heads in (time, id) order (k10s_engine.h "source list"): entries
    // [0, sl_n) are the non-empty sources, sl[0] holds the next event; sl_dirty marks sources whose
    // head an emission changed (an empty ring got its first entry, a new heap root)
    SrcEnt sl[K10S_NSRC];
    uint32_t sl_n, sl_dirty;
    uint32_t unsched_missing;     // PS unscheduled-pod cache entries whose pod left storage (PF_UNSCHED
                                  // without PF_IN_PS): scale_up_info would panic on them
                                  // (persistent_storage.rs:137-145)
    uint32_t stale_fin;           // canceled pod-finish events still in the heap (lazy cancel): while 0,
                                  // a popped N_POD_FINISHED is live without reading its pod's line
    uint32_t pend_rm_n;           // bits set in the api server's removal set (pend_rm): while 0, an
                                  // assignment request needs no read of it
    uint32_t ps_rm_n;             // pods storage dropped on a removal request (PS_REMOVE_POD_REQ): while
                                  // 0, every PodStartedRunning finds its pod in storage (below)
    uint32_t cyc_fails;           // attempts of the previous scheduling cycle that found no node: the cycle
                                  // runs the batched fit pass (k10s_engine.h fit_tile) only after one
    uint32_t aq_sorted;           // the action queue is in sorted mode (k10s_engine.h aq_push): positions
    uint32_t aq_head;             // [aq_head, aq_head + aq_size) hold it in strictly ascending timestamp
    int64_t aq_last;              // order; aq_last = the newest entry's key (total_key)
    int64_t uq_tail;              // total_key of the unschedulable map's last entry's timestamp
                                  // (k10s_engine.h uq_insert); INT64_MAX = not known
    uint64_t fr_dirty;            // 64-node blocks whose front is stale (front_scan rebuilds them)
    uint64_t fr_over;             // blocks whose front has more than K10S_FR_K entries (scanned whole)
    HeapEv fq_win[K10S_NFQ * K10S_FQW];
    HeapEv heap_lds[K10S_HEAP_TOP];
#if K10S_AQ_TOP
    QInfo aq_lds[K10S_AQ_TOP];
#endif
    // cycle attribution of the event loop (K10S_PROF builds only, zero otherwise): PROF_* phases,
    // then per event kind the dispatch cycles and the count (K10S_PROF builds only hold those)
    uint64_t prof[K10S_PROF_SLOTS];
};

struct GroupState {         // HPA PodGroupInfo + metrics/usage-model state of one pod group
    double creation_time;
    double util_cpu, util_ram;        // last pod-metrics tick (collector.rs:263-337)
    double cpu_last_start, ram_last_start;   // PodGroupResourceUsageModel step state
    uint32_t cpu_idx, ram_idx;
    uint32_t registered;              // HPA received RegisterPodGroup
    uint32_t created_count;           // created_pods.len()
    uint32_t total_created;
    uint32_t running;                 // running pods of this group on created nodes
    uint32_t has_metric;              // pod_utilization_metrics contains the group
    uint32_t created_at_as;           // AS handled the CreatePodGroupRequest
};

struct CAAct {
    uint32_t up;            // 1 = ScaleUp(node def), 0 = ScaleDown(node)
    uint32_t arg;           // def id (up) / node idx (down)
};

// NF_CA_ORIGIN: the node instance stored in PS carries origin = "cluster autoscaler"; its PS
// assignment set is kept as a list (ps_head / ps_link) for the CA's scale-down
enum : uint8_t { NF_S_ASSIGN = 1, NF_PS_PRESENT = 2, NF_CA_ORIGIN = 4 };
enum : uint8_t { PF_IN_S = 1, PF_IN_PS = 2, PF_UNSCHED = 4 };

// Per-pod state: every field an event handler touches for one pod, in one 64-B line.
struct PodState {
    uint32_t req_cpu;       // requests (seed-perturbed per replica)
    uint8_t flags;          // PF_IN_PS / PF_UNSCHED: in storage / in the PS unscheduled cache
    uint8_t sflag;          // PF_IN_S: in the scheduler's cache (its own byte, so that
                            // S_POD_SCHEDULE_REQ sets it with a store, no read of the line)
    uint8_t pad0[2];
    uint64_t req_ram;
    double dur;
    int32_t s_assigned;     // scheduler cache pod.status.assigned_node (node idx or -1)
    int32_t ps_assigned;    // storage pod.status.assigned_node
    uint32_t ps_aepoch;     // member of PS assignments[ps_assigned] iff == that node's epoch
    int32_t run_slot;       // node component running it (running_pods), or -1
    uint32_t spare0, spare1;  // unused (round 2 kept a per-component running list here)
    uint32_t finish_seq;    // id of its pending PodFinishedRunning self-event (0 = none/canceled)
    int32_t cancel_slot;    // canceled_pods membership: (slot, slot generation)
    uint32_t cancel_gen;
    uint32_t pad1;
};
static_assert(sizeof(PodState) == 64, "PodState must be one 64-B line");

// Cold per-node state (persistent-storage copy, api-server maps): 32 B.
struct NodeState {
    uint8_t flags;          // NF_*
    uint8_t pad0[3];
    uint32_t ps_cpu;        // PS allocatable
    uint64_t ps_ram;
    uint32_t ps_def;        // node instance stored in PS
    uint32_t ps_epoch;      // bumped by every PS add_node
    int32_t as_slot;        // created_nodes: node component, or -1
    int32_t pend_def;       // pending_node_creation_requests: def, or -1
};
static_assert(sizeof(NodeState) == 32, "NodeState must be 32 B");

// Node component (pool context) state: 32 B.
struct SlotState {
    int32_t node;           // runtime node idx, -1 when back in the pool
    uint32_t def;
    uint32_t gen;           // bumped on reclaim (clears canceled_pods)
    int32_t running;        // pods running on the component (node removal sweeps only if > 0)
    double rtime;           // removal_time
    uint32_t removed;
    uint32_t pad;
};
static_assert(sizeof(SlotState) == 32, "SlotState must be 32 B");

// Offsets (bytes) of per-replica arrays within one replica's region.
struct Layout {
    uint64_t stride;
    uint64_t hdr;
    uint64_t s_cpu, s_ram, s_present;    // hot scheduler-cache SoA (scan target; wide layout)
    uint64_t s_node;                     // packed layout: u64 per node, cpu << 40 | ram (k10s_engine.h nc_*)
    uint64_t fr_val, fr_idx;             // per 64-node block: its index-aware front (k10s_engine.h
                                         // front_scan), K10S_FR_K packed entries + their node offsets
    uint64_t s_bcpu, s_bram;             // per-block maxima of the present nodes' allocatable
    uint64_t s_ccpu, s_cram;             // scheduler-cache capacity SoA (MostAllocated, an extension)
    uint64_t node, pend_rm, pod, prec, slot, pool_ring;
    uint64_t grp, grp_bits;
    uint64_t cag, ca_act, ca_cpu, ca_ram, ca_undo;
    // cluster autoscaler only (0 bytes otherwise): the PS unscheduled-pod cache as a bitmap over pod
    // indices (name order), the PS-present CA-origin nodes as a bitmap over node indices, the PS
    // assignment sets of CA-origin nodes as intrusive lists, and a gather/sort scratch of 2·P entries
    uint64_t ca_ubits, ca_live, ps_head, ps_link, ca_list;
    uint64_t heap, aq, uq, log, place, fq;
    uint64_t gauge, g_cpu, g_ram;        // gauge rows; node-component allocatable per slot
    uint32_t cap_fq;      // entries per delay-class ring (power of two; 0 = no rings)
    uint32_t pruned;      // 1: block bounds maintained, exact pruned scan where it applies
    uint32_t cap_heap, cap_aq, cap_uq, cap_act, cap_log, cap_place, cap_undo, rec_on;
    uint32_t words_nodes, words_uids, words_group, words_pods;
    uint32_t bshift;      // block = 2^bshift consecutive node indices (>= 64, <= 64 blocks)
    uint32_t nblocks;
    uint32_t cap_gauge;   // gauge rows per replica (0 = gauge recorder off)
    uint32_t stall;       // 1: stall guard on (k10s_capacities.stall_guard)
    uint32_t packed;      // 1: node cache packed in s_node (8 B per node); 0: wide SoA s_cpu / s_ram
    uint32_t tnonneg;     // 1: every event time of the scenario and its replicas' parameters is >= 0
                          // (times_nonneg): no emission can precede the clock
    uint32_t front;       // 1: the packed cache keeps per-block fronts (<= 64 blocks of 64 nodes)
    uint32_t pad_front;
};

// Everything a launch reads but never writes, as one block (device: __constant__ memory).
struct DevConst {
    Scenario sc;
    Layout L;
    K10S_RO(Params) params;   // [n_replicas]
    K10S_GB(uint8_t) base;    // replica regions, stride L.stride
    uint32_t* active;         // count of replicas with work left after a budgeted launch
};

}  // namespace k10s
