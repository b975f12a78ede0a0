/*
 * k10s.h — C ABI of the MI355X batched-ensemble engine for kubernetriks' scheduling hot path.
 *
 * Plain C (bindgen-friendly): explicit-width integers, POD structs, caller-owned host buffers,
 * engine-owned device memory behind an opaque handle.  No torch types, no HIP types.  The Rust
 * binding a maintainer would add is in INTEGRATION.md.
 *
 * Two surfaces, mirroring the reference's drop-in boundary:
 *
 *  (1) k10s_schedule_one_batch — replaces, for R independent problems at once,
 *        trait PodSchedulingAlgorithm { fn schedule_one(&self, pod: &Pod,
 *            nodes: &BTreeMap<String, Node>) -> Result<String, ScheduleError>; }
 *      src/core/scheduler/interface.rs:14-23, implemented by KubeScheduler::schedule_one
 *      (src/core/scheduler/kube_scheduler.rs:68-151) with Fit + LeastAllocatedResources
 *      (src/core/scheduler/plugin.rs:34-63).  Nodes are passed in name order (BTreeMap order);
 *      the result is the chosen node's index in that order instead of its String name.
 *
 *  (2) k10s_engine_* — replaces the per-replica event loop that drives it:
 *        KubernetriksSimulation::{new, initialize, run_with_callbacks, step_until_time,
 *        step_for_duration}   src/simulator.rs:68-275, 355-401
 *        RunUntilAllPodsAreFinishedCallbacks::on_step   src/simulation_callbacks.rs:86-91
 *      for thousands of independent replicas per GPU (one wavefront per replica).
 *
 * Errors: every function returns K10S_OK (0) or a negative K10S_E_* code; a reference
 * `panic!` inside one replica is not an ABI error — it stops that replica and is reported in
 * k10s_replica_result.error_code (K10S_PANIC_*), like the reference process would abort.
 * Threading: one handle per device; a handle is not thread-safe (the read-back calls
 * k10s_engine_results / k10s_engine_profile serialize among themselves on one handle).
 */
#ifndef K10S_H
#define K10S_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- schedule_one status (ScheduleError, interface.rs:7-11) ------------------------------ */
#define K10S_SCHED_OK 0
#define K10S_SCHED_NO_NODES_IN_CLUSTER 1
#define K10S_SCHED_NO_SUFFICIENT_RESOURCES 2
#define K10S_SCHED_REQUESTED_RESOURCES_ARE_ZEROS 3

/* ---- ABI error codes -------------------------------------------------------------------- */
#define K10S_OK 0
#define K10S_E_INVALID (-1)       /* bad argument / malformed scenario (message via k10s_last_error) */
#define K10S_E_NO_DEVICE (-2)     /* no HIP device: the engine never falls back to the CPU */
#define K10S_E_HIP (-3)           /* HIP runtime error */
#define K10S_E_CAPACITY (-4)      /* requested capacities do not fit device memory */
#define K10S_E_STATE (-5)         /* call not valid in the handle's current state */

/* ---- per-replica status ------------------------------------------------------------------ */
#define K10S_REPLICA_RUNNING 0    /* paused (event budget or until-time reached) */
#define K10S_REPLICA_FINISHED 1   /* all trace pods terminated at a clock multiple of 1000 */
#define K10S_REPLICA_ERROR 2      /* reference panic or engine capacity overflow: see error_code */
#define K10S_REPLICA_TIME_LIMIT 3 /* next event beyond the run's max_time guard */
#define K10S_REPLICA_STALLED 4    /* opt-in stall guard (k10s_capacities.stall_guard): at a gauge tick
                                     the trace was exhausted and only the periodic ticks were pending
                                     (no running pod will finish, no node event, no CA/HPA), so the
                                     replica can only retry its unschedulable pods forever and would
                                     reach TIME_LIMIT; it stops there instead */

/* ---- per-replica error codes (reference panic sites) ------------------------- */
#define K10S_PANIC_NONE 0
#define K10S_PANIC_POOL_EXHAUSTED 1        /* node_component_pool.rs:56-59 */
#define K10S_PANIC_DUPLICATE_NODE 2        /* api_server.rs:73-78, persistent_storage.rs:76-81 */
#define K10S_PANIC_DUPLICATE_POD 3         /* persistent_storage.rs:89-94 */
#define K10S_PANIC_MISSING_POD 4           /* any pods.get(...).unwrap() on an absent pod */
#define K10S_PANIC_MISSING_NODE 5          /* any nodes/created_nodes.get(...).unwrap() on an absent node */
#define K10S_PANIC_BIND_REMOVED_NODE 6     /* node_component.rs:190-202 */
#define K10S_PANIC_MISSING_ASSIGNMENTS 7   /* scheduler assignments.get_mut(node).unwrap() */
#define K10S_PANIC_USAGE_MODEL 8           /* resource usage model construction/poll panics */
#define K10S_PANIC_HPA_UNREGISTERED 9      /* horizontal_pod_autoscaler.rs:214 */
#define K10S_PANIC_CA_GROUP 10             /* kube_cluster_autoscaler.rs:297-299 */
#define K10S_PANIC_GROUP_DURATION 11       /* api_server.rs:406-409 */
#define K10S_PANIC_MISSING_PENDING 12      /* api_server.rs:98-101 */
#define K10S_PANIC_REMOVE_OTHER_NODE 13    /* node_component.rs:248-254 */
#define K10S_PANIC_UNKNOWN_PROFILE 14      /* kube_scheduler.rs:95 */
#define K10S_PANIC_NEGATIVE_DELAY 15       /* dslab-core add_event: an event emitted with a negative (or NaN)
                                              delay, i.e. into the past (a negative pod duration, network
                                              delay or tick interval reaching an emission) */
#define K10S_ERR_HEAP_FULL 100             /* engine capacity: event heap (regrown, k10s_engine_name_bounds) */
#define K10S_ERR_QUEUE_FULL 101            /* engine capacity: scheduler queues (regrown) */
#define K10S_ERR_NAME_BOUND 102            /* engine capacity: generated-name universe bound (regrown) */
#define K10S_ERR_SEQ_OVERFLOW 103          /* engine capacity: 2^32 event ids in one replica */
#define K10S_ERR_CA_BUFFER 104             /* CA action buffers: sized so no decision can fill them (an
                                              invariant, k10s_host.cpp regrow), never regrown */
#define K10S_ERR_NODE_CACHE_RANGE 105      /* engine capacity: a packed node-cache entry would exceed its
                                              field (allocatable cpu >= 2^24 or ram >= 2^40 after a
                                              release; cannot happen while allocatable <= capacity) */
#define K10S_ERR_INVARIANT 106             /* host check build only: an invariant a device shortcut relies
                                              on was violated (never expected) */
#define K10S_ERR_EXEC_GUARD 107            /* K10S_EXEC_CHECK tooling builds only: a lane-parallel helper
                                              was entered without the whole wave live, or a bounded
                                              loop exceeded its bound; error_kind = site id */

/* ---- counters (printer.rs:90-101 + engine throughput counters) ---------------------------- */
enum k10s_counter {
    K10S_C_TOTAL_NODES_IN_TRACE = 0,
    K10S_C_TOTAL_PODS_IN_TRACE,
    K10S_C_PODS_SUCCEEDED,
    K10S_C_PODS_UNSCHEDULABLE,
    K10S_C_PODS_FAILED,
    K10S_C_PODS_REMOVED,
    K10S_C_TOTAL_SCALED_UP_NODES,
    K10S_C_TOTAL_SCALED_DOWN_NODES,
    K10S_C_TOTAL_SCALED_UP_PODS,
    K10S_C_TOTAL_SCALED_DOWN_PODS,
    K10S_C_PROCESSED_NODES,  /* InternalMetrics.processed_nodes (collector.rs:80) */
    K10S_C_TERMINATED_PODS,  /* InternalMetrics.terminated_pods (collector.rs:84) */
    K10S_C_PLACEMENTS,       /* successful schedule_one calls (scheduler.rs:309-320) */
    K10S_C_ATTEMPTS,         /* schedule_one calls reaching the filter (kube_scheduler.rs:89) */
    K10S_C_EVENTS,           /* delivered (non-canceled) events */
    K10S_C_NODES_SCANNED,    /* Σ |scheduler cache| over attempts: algorithmic scan volume */
    K10S_C_NODES_READ,       /* scheduler-cache entries actually read (block bounds, scanned blocks,
                                bound maintenance): the pruned scan's real volume, engine-only */
    K10S_C_REQUEUED,         /* unschedulable_pods entries moved back to the action queue by any
                                policy (scheduler.rs:174-185): the retry volume under backlog */
    K10S_C_FLUSHED,          /* ... of which by the 30-s flush of entries older than 300 s (188-203) */
    K10S_NUM_COUNTERS
};

/* Fixed log2 bins of every value an estimator sees (engine addition; the reference keeps only
   the four estimators).  Bin 0: x < 2^-10 s (also 0, negatives, NaN); bin k in 1..30:
   2^(k-11) <= x < 2^(k-10); bin 31: x >= 2^20 s.  The bin is read off the f64 exponent, so it is
   exact and identical on the host restatement.  Summed over replicas and over ranks (RCCL). */
#define K10S_HIST_BINS 32

/* `average` 0.15 Min/Max/Mean/Variance estimator state (collector.rs:15-74) + histogram */
typedef struct k10s_estimator {
    uint64_t n;
    double min, max, mean, sum2; /* population variance = sum2 / n */
    uint32_t hist[K10S_HIST_BINS];
} k10s_estimator;

#define K10S_EST_POD_DURATION 0
#define K10S_EST_POD_SCHEDULE_TIME 1
#define K10S_EST_POD_QUEUE_TIME 2

typedef struct k10s_replica_result {
    uint32_t status;        /* K10S_REPLICA_* */
    uint32_t error_code;    /* K10S_PANIC_* / K10S_ERR_* */
    uint32_t error_kind;    /* event kind (k10s_events.h) being handled at the error */
    uint32_t error_seq;     /* id of that event */
    double error_time;
    double clock;           /* simulation time of the last delivered event (dslab time()) */
    uint64_t counters[K10S_NUM_COUNTERS];
    k10s_estimator est[3];
    uint32_t unschedulable_len;  /* scheduler unschedulable_pods.len() (stale entries included) */
    uint32_t active_len;         /* scheduler action_queue.len() */
    uint32_t node_count_as, node_count_ps, node_count_s;
    uint32_t log_len, placements_len, flags;  /* flags bit0: event log overflow, bit1: placement log overflow */
} k10s_replica_result;

/* Per-replica parameters (scheduler-parameter sweeps, seed-perturbed traces).  Fields mirror
   SimulationConfig (config.rs:13-37) and the CA/HPA algorithm configs; k10s_default_params fills
   them from the scenario. */
typedef struct k10s_replica_params {
    double scheduling_cycle_interval;
    double as_to_ps_network_delay, ps_to_sched_network_delay, sched_to_as_network_delay;
    double as_to_node_network_delay, as_to_ca_network_delay, as_to_hpa_network_delay;
    double ca_scan_interval, ca_scale_down_utilization_threshold;
    double hpa_scan_interval, hpa_target_threshold_tolerance;
    double score_weight;                 /* LeastAllocatedResources weight (kube_scheduler.rs:55) */
    uint32_t enable_unscheduled_pods_conditional_move;
    uint32_t perturb;                    /* 0: trace as given; 1: seed-perturbed durations/requests */
    uint64_t seed;
    uint64_t ca_max_node_count;          /* read-only here (fixed by the scenario's node pool) */
    /* Score plugins of the default profile (kube_scheduler.rs:44-61: a weighted sum over the enabled
       score plugins, starting from 0.0): bit 0 LeastAllocatedResources (weight score_weight), bit 1
       MostAllocatedResources (weight most_allocated_weight).  The reference registry
       (plugin.rs:13-23) has only LeastAllocatedResources, so bit 1 is an extension (DESIGN.md §3,
       parity against the oracle's restatement only).  0 is refused (no score plugin: every
       filtered node scores 0.0).  Default K10S_SCORE_LEAST_ALLOCATED. */
    double most_allocated_weight;
    uint32_t score_plugins;
    /* Replica-specific trace length: the replica runs the scenario as if its workload trace held only
       its first workload_prefix events (generic.rs order, before the timestamp sort); 0 = all.  Lets
       one engine batch replicas whose traces are prefixes of one master trace, e.g. C2's per-replica
       ceil(U * 10000) pods (tests/test_determinism.rs:49-68).  Ids, total_pods_in_trace and the
       termination rule are those of the shortened trace. */
    uint32_t workload_prefix;
} k10s_replica_params;
#define K10S_SCORE_LEAST_ALLOCATED 1u
#define K10S_SCORE_MOST_ALLOCATED 2u

/* Capacities of per-replica engine structures (0 = derive from the scenario). */
typedef struct k10s_capacities {
    uint32_t event_heap, active_queue, unschedulable, group_name_bound, ca_name_bound;
    uint32_t event_log, placement_log;   /* parity mode logs; 0 = off */
    uint32_t pod_records;                /* 1 = keep per-pod start/finish/removal times */
    uint32_t delay_fifo;                 /* entries per delay-class event ring: 0 = default (the node
                                            count rounded up to a power of two, within [512, 8192]:
                                            8 rings x 32 B x that many entries per replica, up to 2 MiB;
                                            when the replicas' state would not fit the free device
                                            memory, the default falls back to 512 entries),
                                            K10S_FIFO_OFF = every event in the heap */
    uint32_t pruned_scan;                /* 0 = every attempt scans every node (default);
                                            1 = exact block-bound pruned scan where it applies
                                             */
    uint32_t gauge_log;                  /* rows of the 5-s gauge recorder kept per replica; 0 = off */
    uint32_t stall_guard;                /* 1 = stop a run-until-all-finished replica that can no longer
                                            make progress with K10S_REPLICA_STALLED; 0 = off (reference
                                            behaviour: it runs to max_time) */
    uint32_t node_cache;                 /* layout of the scheduler's node cache (the scan target):
                                            K10S_NODE_CACHE_AUTO (0) = packed, one u64 per node (cpu in
                                            bits 40-63, ram in bits 0-39: 8 B per node and scan), when
                                            every node definition has cpu < 2^24 and ram < 2^40, no
                                            replica uses a score plugin beyond LeastAllocated,
                                            pruned_scan is off and no event time carries a sign bit
                                            (trace timestamps, durations, delays, tick intervals: the
                                            packed kernel keys times by their bit pattern); otherwise
                                            wide.  K10S_NODE_CACHE_WIDE (1)
                                            = always the u32 cpu + u64 ram SoA (12 B per node).  Results
                                            are identical either way. */
} k10s_capacities;
#define K10S_NODE_CACHE_AUTO 0u
#define K10S_NODE_CACHE_WIDE 1u

/* One row of the gauge recorder (MetricsCollector::record_gauge_metrics, collector.rs:352-407,
   written every 5 s of simulated time as the reference's gauge CSV).  The two node averages sum
   over the api server's created nodes in name order (the reference sums in HashMap order). */
typedef struct k10s_gauge_row {
    double time;
    uint64_t current_nodes, current_pods, pods_in_scheduling_queues;
    double node_average_cpu_utilization, node_average_ram_utilization;
    double cluster_total_cpu_utilization, cluster_total_ram_utilization;
} k10s_gauge_row;
#define K10S_FIFO_OFF 0xFFFFFFFFu

/* Parity event-log entry: one delivered event (time, id order). */
typedef struct k10s_log_entry {
    double time;
    uint32_t seq;
    uint16_t kind;   /* k10s_event_kind */
    int16_t slot;    /* node component (pool slot) for N_* kinds, else -1 */
    int32_t pod;     /* pod index (name order) or -1 */
    int32_t node;    /* node index (name order) or -1 */
} k10s_log_entry;

typedef struct k10s_placement {
    double assign_time;
    int32_t pod, node;
} k10s_placement;

typedef struct k10s_pod_record {
    double t_running, t_finished, t_removed;  /* NaN when absent */
    uint32_t state;                           /* 0 none, 1 in storage, 2 succeeded, 3 removed */
    uint32_t pad;
} k10s_pod_record;

/* (1) --------------------------------------------------------------------------------------
 * R independent schedule_one calls.  All pointers are DEVICE pointers.  Problem r sees nodes
 * [r*node_stride, r*node_stride + n_nodes) in name order; present_bits marks which of them are in
 * the scheduler cache (bit i of word (r*node_stride + i)/64 — node_stride must be a multiple
 * of 64).  Writes out_node[r] (index within the problem, -1 on error) and out_status[r].
 * Buffer contract (the scan reads 4 consecutive nodes per lane with 16-byte vector loads):
 * alloc_cpu and alloc_ram must be 16-byte aligned and hold n_problems * node_stride elements
 * (every row padded to node_stride; padding values are ignored), present_bits
 * n_problems * node_stride / 64 words.  A misaligned pointer returns K10S_E_INVALID.
 * stream: a hipStream_t or NULL.  Returns K10S_OK or a negative K10S_E_* code. */
int32_t k10s_schedule_one_batch(const uint32_t* alloc_cpu, const uint64_t* alloc_ram,
                                const uint64_t* present_bits, uint32_t n_nodes, uint32_t node_stride,
                                const uint32_t* req_cpu, const uint64_t* req_ram, double weight,
                                uint32_t n_problems, int32_t* out_node, int32_t* out_status,
                                void* stream);

/* (1b) -------------------------------------------------------------------------------------
 * ScorePlugin surface: replaces `ScorePlugin::score(&self, pod: &Pod, node: &Node) -> f64`
 * (src/core/scheduler/plugin.rs:25-31) for LeastAllocatedResources (plugin.rs:52-63), applied
 * the way KubeScheduler accumulates it (0.0 + score * weight, kube_scheduler.rs:113-138), for n
 * independent (node allocatable, pod request) pairs.  Element i: out_score[i] = 0.0 +
 * LeastAllocated(alloc_cpu[i], alloc_ram[i], req_cpu[i], req_ram[i]) * weight, bit-identical to
 * the values k10s_schedule_one_batch and the engine compare (NaN for a 0/0 resource term).
 * Callers guarantee req <= alloc per element (the Fit filter ran first, as in the reference).
 * All pointers are DEVICE pointers.  Returns K10S_OK or a negative K10S_E_* code. */
int32_t k10s_score_batch(const uint32_t* alloc_cpu, const uint64_t* alloc_ram, const uint32_t* req_cpu,
                         const uint64_t* req_ram, double weight, uint64_t n, double* out_score,
                         void* stream);

/* (1') Host-buffer form of (1) for hosts without HIP bindings (the Rust PodSchedulingAlgorithm
 * adapter in INTEGRATION.md): a handle owns device buffers for up to max_problems problems of up
 * to max_nodes nodes.  k10s_scheduler_schedule takes HOST arrays — problem r's nodes are
 * alloc_cpu/alloc_ram[r*n_nodes .. r*n_nodes + n_nodes) in name order; present_bits (may be NULL
 * = every node present) holds ceil(n_nodes/64) words per problem — copies them to the device,
 * runs the same kernel as (1) and blocks until out_node/out_status (host, [n_problems]) are
 * written.  PCIe-inclusive; meant for one cycle's worth of pods, not for throughput. */
typedef struct k10s_scheduler k10s_scheduler;
k10s_scheduler* k10s_scheduler_create(uint32_t max_nodes, uint32_t max_problems, int32_t device);
void k10s_scheduler_destroy(k10s_scheduler* s);
int32_t k10s_scheduler_schedule(k10s_scheduler* s, const uint32_t* alloc_cpu, const uint64_t* alloc_ram,
                                const uint64_t* present_bits, uint32_t n_nodes, const uint32_t* req_cpu,
                                const uint64_t* req_ram, double weight, uint32_t n_problems, int32_t* out_node,
                                int32_t* out_status);

/* (2) -------------------------------------------------------------------------------------- */
typedef struct k10s_engine k10s_engine;

/* Compile a scenario (DESIGN.md §Scenario format) into device tables and allocate n_replicas
 * replicas on `device`.  params may be NULL (defaults; replica r gets seed = scenario seed + r
 * and perturb = 0).  caps may be NULL.  Returns NULL on failure (k10s_last_error). */
k10s_engine* k10s_engine_create(const char* scenario_text, const k10s_replica_params* params,
                                uint32_t n_replicas, const k10s_capacities* caps, int32_t device);
/* Same as k10s_engine_create, plus binary trace blocks for traces too large for one text line per
   event (host converters: kubernetriks_amd/scenario.py pods_blob / nodes_blob, trace_soa.py).  The
   blob is a sequence of self-delimiting little-endian SoA blocks with nothing after the last one:
     "K10SPOD1" | u64 n | f64 ts[n] | u32 cpu[n] | u32 pad (n odd) | u64 ram[n] | f64 duration[n]
       (NaN = long-running) | u32 name_off[n + 1] | name bytes[name_off[n]]        -> create_pod
     "K10SNOD1" | u64 n | f64 ts[n] | u32 cpu[n] | u32 pad (n odd) | u64 ram[n] | u32 op[n]
       (0 create_node with capacity cpu/ram, 1 remove_node) | u32 pad (n odd)
       | u32 name_off[n + 1] | name bytes                                           -> cluster events
   Names are non-empty and contain none of " \t\n\v\f\r#=".  The events of each block are
   appended after the text's lines of the same trace (workload / cluster), in block order (= trace
   position for the stable timestamp sort, generic.rs:78-107, and for seed perturbation). */
k10s_engine* k10s_engine_create_bulk(const char* scenario_text, const void* pods_blob, uint64_t blob_len,
                                     const k10s_replica_params* params, uint32_t n_replicas,
                                     const k10s_capacities* caps, int32_t device);
void k10s_engine_destroy(k10s_engine* e);

/* Scenario-derived defaults for replica parameters. */
int32_t k10s_engine_default_params(const k10s_engine* e, k10s_replica_params* out);

/* Reset every replica to the initialized state (KubernetriksSimulation::initialize). */
int32_t k10s_engine_reset(k10s_engine* e);

#define K10S_RUN_UNTIL_ALL_FINISHED 0   /* run_with_callbacks(RunUntilAllPodsAreFinished) */
#define K10S_RUN_UNTIL_TIME 1           /* step_until_time(until_time) */

/* Advance every replica.  Each launch processes at most max_events_per_launch delivered events
 * per replica (0 = unbounded) and the call loops launches until no replica is RUNNING-with-work.
 * max_time guards runaway runs in mode 0 (replica -> TIME_LIMIT).  Blocks until done.
 * If elapsed_ms is not NULL it receives the device time of the run (HIP events). */
int32_t k10s_engine_run(k10s_engine* e, int32_t mode, double until_time, double max_time,
                        uint64_t max_events_per_launch, double* elapsed_ms);

/* Launch one bounded pass (no host loop, no sync) on the engine stream; *active receives, after
 * completion, the number of replicas that still have work.  For benches/profilers. */
int32_t k10s_engine_step_async(k10s_engine* e, int32_t mode, double until_time, double max_time,
                               uint64_t max_events_per_launch);
int32_t k10s_engine_sync(k10s_engine* e);

int32_t k10s_engine_results(const k10s_engine* e, k10s_replica_result* out /* [n_replicas] */);
/* Gauge rows of one replica (k10s_capacities.gauge_log > 0): the first min(cap, recorded) rows;
   *n = rows copied.  Result flags bit2 marks a gauge log overflow. */
int32_t k10s_engine_gauges(const k10s_engine* e, uint32_t replica, k10s_gauge_row* out, uint32_t cap,
                           uint32_t* n);
int32_t k10s_engine_event_log(const k10s_engine* e, uint32_t replica, k10s_log_entry* out, uint32_t cap,
                              uint32_t* n);
int32_t k10s_engine_placements(const k10s_engine* e, uint32_t replica, k10s_placement* out, uint32_t cap,
                               uint32_t* n);
int32_t k10s_engine_pod_records(const k10s_engine* e, uint32_t replica, k10s_pod_record* out, uint32_t cap,
                                uint32_t* n);
/* HPA pod-group state: created_pods.len() and total_created per group (name order). */
int32_t k10s_engine_group_sizes(const k10s_engine* e, uint32_t replica, uint32_t* created, uint32_t* total,
                                uint32_t cap, uint32_t* n);

/* Generated-name universes of the compiled batch: names per pod group ("{group}_{k}", the HPA's pods)
   and per CA node group ("{group}_{k}").  k10s_capacities.group_name_bound / ca_name_bound set the
   first universe (0 = derived from the scenario).  The reference bounds neither
   (kube_horizontal_pod_autoscaler.rs:178-182, api_server.rs:421), nor its event queue and scheduler
   queues (dslab-core's BinaryHeap, scheduler.rs:45, 49).  When a replica outgrows a universe
   (K10S_ERR_NAME_BOUND), the event heap (K10S_ERR_HEAP_FULL) or the active queue / unschedulable
   map (K10S_ERR_QUEUE_FULL), k10s_engine_run / k10s_engine_sync recompile the batch with every
   exhausted capacity doubled (up to 2^20 names per universe, 2^30 heap or queue entries) and replay
   every run and step call since the last initialize, so results equal the reference's.
   * Memory: the regrown batch is allocated beside the current one if both fit, else in its place;
     if neither fits, the call returns K10S_E_CAPACITY and the stopped results stay readable.  If the
     regrow released the current state and then failed, every later call on the engine returns
     K10S_E_CAPACITY (destroy it).
   * Timing: elapsed_ms of k10s_engine_run includes the regrow and its replays (k10s_engine_capacities
     reports how many regrows happened).
   * Names: the name tables below then describe the regrown batch.  A pointer returned by
     k10s_engine_node_name / k10s_engine_pod_name / k10s_engine_group_name before a run or sync is
     invalid after one that regrew: re-read the names after every run. */
int32_t k10s_engine_name_bounds(const k10s_engine* e, uint32_t* group_bound, uint32_t* ca_bound);
/* The batch's effective capacities (after any regrow): event_heap, active_queue, unschedulable and
   the two name bounds as compiled (derived values filled in), delay_fifo = entries per ring
   (K10S_FIFO_OFF when off), the other fields as given at create.  *regrows (may be NULL) = batches
   recompiled by regrow since create. */
int32_t k10s_engine_capacities(const k10s_engine* e, k10s_capacities* out, uint32_t* regrows);
/* Test support: checks replica `replica`'s per-block Pareto fronts of the packed node cache against
   its node cache (every block not marked stale holds exactly its front).
   *result = blocks checked, -(1 + the first block that breaks it), or 0 when the batch keeps no
   fronts (a cache of up to 512 or more than 4,096 nodes, or not packed). */
int32_t k10s_engine_check_fronts(const k10s_engine* e, uint32_t replica, int32_t* result);

/* Name tables of the compiled scenario (index -> name), for mapping logs back to names.  The
   returned strings belong to the engine and stay valid until the next run / sync that regrows the
   batch (k10s_engine_name_bounds) or k10s_engine_destroy. */
uint32_t k10s_engine_num_nodes(const k10s_engine* e);
uint32_t k10s_engine_num_pods(const k10s_engine* e);
uint32_t k10s_engine_num_groups(const k10s_engine* e);
const char* k10s_engine_node_name(const k10s_engine* e, uint32_t idx);
const char* k10s_engine_pod_name(const k10s_engine* e, uint32_t idx);
const char* k10s_engine_group_name(const k10s_engine* e, uint32_t idx);

/* Per-replica device-state footprint in bytes and device pointer of replica r's scheduler
   cache SoA (for profiling tools). */
uint64_t k10s_engine_replica_bytes(const k10s_engine* e);
/* Bytes per node of the scheduler's node cache that every scheduling attempt reads: 8 (packed) or
   12 (wide: u32 cpu + u64 ram); see k10s_capacities.node_cache.  0 for a null engine. */
uint32_t k10s_engine_node_entry_bytes(const k10s_engine* e);

/* Tooling: per-replica cycle attribution of the event loop, 8 words per replica
   (loop, select, consume, dispatch, scheduling cycle, scan, scans, bound maintenance; s_memtime
   cycles).  All zero unless the library was built with -DK10S_PROF=1 (variant builds only). */
int32_t k10s_engine_profile(const k10s_engine* e, uint64_t* out /* [n_replicas * width] */);
/* Slots per replica k10s_engine_profile writes (8 in product builds; more in K10S_PROF builds). */
uint32_t k10s_engine_profile_width(void);

const char* k10s_last_error(void);
const char* k10s_version(void);

#ifdef __cplusplus
}
#endif
#endif /* K10S_H */
