// k10s_builder.h — compile a scenario text into the integer tables of k10s_state.h (host side).
//
// What the reference does with strings and ordered maps, this does once per scenario:
//   * every node / pod name that can exist in a replica gets a rank in byte order
//     (trace names, default-cluster names `{prefix}_{k}` simulator.rs:303-344, cluster-autoscaler
//     names `{template}_{k}` kube_cluster_autoscaler.rs:100-105, pod-group names `{group}_{k}`
//     api_server.rs:421 / kube_horizontal_pod_autoscaler.rs:435-438, bounded);
//   * the cluster trace then the workload trace are stably sorted by timestamp
//     (generic.rs:78,105) and given dslab ids 2.. in emission order (simulator.rs:234-253), then
//     merged into one (time, id)-ordered stream shared by all replicas;
//   * the node pool size is max concurrent trace nodes + CA max_node_count (simulator.rs:211-230).
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "k10s_state.h"

namespace k10s {

struct HostScenario {
    // sizes / flags
    uint32_t n_nodes = 0, n_pods = 0, n_uids = 0, n_slots = 0, n_pool = 0, n_default = 0;
    uint32_t group_bound = 0, ca_bound = 0;
    bool ca_enabled = false, hpa_enabled = false;
    uint64_t total_pods_in_trace = 0, total_nodes_in_trace = 0;
    uint32_t n_cluster_trace = 0;           // cluster-trace events (ids 2 .. 2 + n_cluster_trace - 1)
    std::vector<uint32_t> wl_pods_upto;     // [W + 1] create_pod events among the first k workload events
    Params defaults;

    std::vector<std::string> node_names, pod_names, group_names, ca_group_names;
    std::vector<uint32_t> node_uid, pod_uid;
    std::vector<uint32_t> def_node, def_cpu;
    std::vector<uint64_t> def_ram;
    std::vector<int32_t> def_ca_group;
    std::vector<uint8_t> def_ca_origin;
    std::vector<uint32_t> pod_cpu, pod_key;
    std::vector<uint64_t> pod_ram;
    std::vector<double> pod_dur;
    std::vector<uint8_t> pod_flags;
    std::vector<int32_t> pod_group;
    std::vector<uint32_t> default_defs;
    std::vector<TraceEv> trace;
    // pod groups
    std::vector<uint32_t> g_initial, g_max, g_cpu;
    std::vector<uint64_t> g_ram;
    std::vector<uint8_t> g_flags, g_cpu_kind, g_ram_kind;
    std::vector<double> g_tcpu, g_tram, g_cpu_usage, g_ram_usage;
    std::vector<uint32_t> g_cpu_uoff, g_cpu_ucnt, g_ram_uoff, g_ram_ucnt;
    std::vector<uint32_t> g_pod, g_pos, g_sorted_k;
    std::vector<double> unit_dur, unit_load;
    // CA groups
    std::vector<uint8_t> ca_has_max;
    std::vector<uint64_t> ca_max;
    std::vector<uint32_t> ca_def, ca_cpu;
    std::vector<uint64_t> ca_ram;
};

// Parse + compile.  group_bound / ca_bound: 0 = derive.  Returns false with a message on
// malformed or unsupported input.
// `bulk` / `bulk_len`: optional K10S_PODS_MAGIC blob of create_pod workload events (include/k10s.h,
// k10s_engine_create_bulk), appended after the text's workload lines in blob order.
bool build_scenario(const std::string& text, uint32_t group_bound, uint32_t ca_bound, HostScenario& out,
                    std::string& err, const uint8_t* bulk = nullptr, uint64_t bulk_len = 0);

// Point a device-side Scenario view at arrays laid out by `pack_scenario` in one buffer.
// pack_scenario returns the byte image; the Scenario's pointers are offsets relative to `base`.
std::vector<uint8_t> pack_scenario(const HostScenario& hs, Scenario& view_offsets);
Scenario rebase_scenario(const Scenario& view_offsets, const uint8_t* base);

// allow_packed: false when some replica needs the wide node cache (a score plugin beyond
// LeastAllocated: the plugin kernel reads capacities from the wide SoA) or the general event-time
// key (!times_nonneg): the packed layout runs in the default kernel, which keys times by their bits.
Layout make_layout(const HostScenario& hs, const k10s_capacities& caps, bool allow_packed, bool tnonneg);
// Every event time of the scenario under these replica parameters carries no sign bit (trace
// timestamps, pod and usage-unit durations, network delays, tick intervals; -0.0 allowed), so the
// default kernel's bit-pattern time key orders them like total_cmp (k10s_common.h total_key).
bool times_nonneg(const HostScenario& hs, const Params* params, uint32_t n_params);
// Every node definition fits the packed node-cache entry (cpu < 2^24, ram < 2^40).
bool nodes_packable(const HostScenario& hs);

// Caller-supplied replica parameters the engine cannot run: "" when valid, else the reason.
std::string params_error(const Params& p, const HostScenario& hs);

}  // namespace k10s
