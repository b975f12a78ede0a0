/*
 * oracle/oracle.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * A single-threaded CPU restatement of kubernetriks' scheduling hot path and the per-replica
 * event loop that drives it (reference: jellythefish/kubernetriks, Rust, built on dslab-core
 * git rev 4ea3b3a).  It is the parity CHECKER for the MI355X engine: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.  Nothing in the product
 * (kubernetriks_amd/, include/k10s.h) links or calls it.
 *
 * It deliberately keeps the reference's data structures where they define semantics:
 * string-keyed ordered maps (Rust BTreeMap/BTreeSet byte order), a (time, id) event queue with
 * lazy cancellation (dslab-core), a verbatim replica of Rust std BinaryHeap sift order for the
 * scheduler's active queue, and the scheduler's per-call Vec/BTreeMap score table.
 *
 * Parity pinning: the Rust reference cannot be built here (no cargo/rustc; dslab-core is an
 * un-vendored git dependency) — see DESIGN.md.  This restatement is pinned by the golden values
 * transcribed from the reference's own tests (tests/golden/, tests/test_oracle_golden.py).
 * Third-party semantics restated from their published algorithms (parity unpinned where no
 * reference test covers them): dslab-core event order/cancel, Rust BinaryHeap sift order for
 * equal timestamps, `average` 0.15 estimators.
 *
 * Every handler cites the reference file:line it follows.
 */
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <queue>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../include/k10s_events.h"

namespace orc {

struct RefPanic : std::runtime_error {
    using std::runtime_error::runtime_error;
};
[[noreturn]] static void panic(const std::string& m) { throw RefPanic(m); }

/* Rust f64::total_cmp (core/num/f64.rs): flip the magnitude bits of negatives, compare as i64. */
static inline int64_t total_key(double x) {
    int64_t b;
    std::memcpy(&b, &x, 8);
    b ^= (int64_t)(((uint64_t)(b >> 63)) >> 1);
    return b;
}
static inline int total_cmp(double a, double b) {
    int64_t ka = total_key(a), kb = total_key(b);
    return ka < kb ? -1 : (ka > kb ? 1 : 0);
}

/* Rust `as` casts: f64 -> unsigned saturates, NaN -> 0. */
static inline uint64_t f64_as_u64(double x) {
    if (std::isnan(x) || x <= 0.0) return 0;
    if (x >= 18446744073709551616.0) return UINT64_MAX;
    return (uint64_t)x;
}

/* ------------------------------------------------------------------------------------------ */
/* `average` 0.15 estimators: concatenate!(Min, Max, Mean, Variance) (collector.rs:15-21).     */
/* Mean: n += 1; avg += (x - avg) / n.  Variance: sum2 += d*d*n*(n-1), d = (x - avg_old)/n.    */
/* ------------------------------------------------------------------------------------------ */
/* Engine addition (no reference counterpart): 32 log2 bins of the same values, include/k10s.h
   K10S_HIST_BINS.  Bin 0: x < 2^-10 or NaN; k: 2^(k-11) <= x < 2^(k-10); 31: x >= 2^20. */
static int hist_bin(double x) {
    if (!(x >= 0.0009765625)) return 0;
    int e = std::ilogb(x);
    return e >= 20 ? 31 : e + 11;
}
/* GaugeMetrics (collector.rs:169-190): the three counters the api server / scheduler maintain */
struct GaugeMetrics {
    uint64_t current_nodes = 0, current_pods = 0, pods_in_scheduling_queues = 0;
};
struct Estimator {
    uint64_t n = 0;
    double mn = INFINITY, mx = -INFINITY, avg = 0.0, sum2 = 0.0;
    uint32_t hist[32] = {};
    void add(double x) {
        hist[hist_bin(x)] += 1;
        mn = std::fmin(mn, x);
        mx = std::fmax(mx, x);
        n += 1;
        double nf = (double)n;
        double delta_n = (x - avg) / nf;
        avg += delta_n;
        sum2 += delta_n * delta_n * nf * (nf - 1.0);
    }
    double mean() const { return n == 0 ? NAN : avg; }
    double population_variance() const { return n < 1 ? NAN : sum2 / (double)n; }
};

/* ------------------------------------------------------------------------------------------ */
/* Data model (core/common.rs, node.rs, pod.rs, resource_usage/ files)                         */
/* ------------------------------------------------------------------------------------------ */
struct UsageModelConfig {           /* ResourceUsageModelConfig, resource_usage/interface.rs:15 */
    int kind = 0;                   /* 1 = "constant", 2 = "pod_group" */
    double usage = 0.0;             /* constant.rs:8-10 */
    std::vector<std::pair<double, double>> seq;  /* pod_group.rs UsageUnit {duration, total_load} */
};
struct RuntimeUsageConfig {         /* RuntimeResourcesUsageModelConfig, common.rs:54-57 */
    bool has_cpu = false, has_ram = false;
    UsageModelConfig cpu, ram;
};

struct Node {
    std::string name;
    std::map<std::string, std::string> labels;
    uint32_t cap_cpu = 0, alloc_cpu = 0;
    uint64_t cap_ram = 0, alloc_ram = 0;
};

struct Pod {
    std::string name;
    std::map<std::string, std::string> labels;
    uint32_t cpu = 0;
    uint64_t ram = 0;
    bool has_dur = false;
    double dur = 0.0;
    bool has_usage = false;
    RuntimeUsageConfig usage;
    std::string assigned_node;
    /* label "pod_group_creation_time" = f64 to_string(), parsed back exactly (A.8): carried as f64 */
    bool has_group_ct = false;
    double group_ct = 0.0;
    /* conditions (pod.rs:63-68) kept only as the times tests read */
    double t_created = NAN, t_scheduled = NAN, t_running = NAN, t_finished = NAN, t_removed = NAN;
    int sched_status = -1; /* 1 = PodScheduled True, 0 = False */
};

/* ResourceUsageModel instances (resource_usage/constant.rs, pod_group.rs) */
struct UsageModel {
    int kind = 0;
    double usage = 0.0;
    std::vector<std::pair<double, double>> seq;
    double last_unit_start_time = 0.0, last_poll_time = 0.0;
    size_t idx = 0;
    /* pod_group.rs:192-201 */
    double current_usage(double time, bool has_count, size_t pod_count) {
        if (kind == 1) return usage;
        if (time < last_poll_time) panic("Trying to get current usage of time which is behind last poll time");
        last_poll_time = time;
        if (!has_count) panic("pod_count.unwrap() on None");
        /* step_usage_until_current_time, pod_group.rs:172-182 */
        while (last_unit_start_time + seq[idx].first <= time) {
            last_unit_start_time += seq[idx].first;
            idx = (idx + 1) % seq.size();
        }
        double load = seq[idx].second;
        return std::fmin(1.0, load / (double)pod_count);
    }
};
static UsageModel model_from_config(const UsageModelConfig& c, bool has_ct, double creation_time) {
    UsageModel m;
    m.kind = c.kind;
    m.usage = c.usage;
    m.seq = c.seq;
    if (c.kind == 2) {
        if (!has_ct) panic("pod_group_creation_time.unwrap() on None");  /* helpers.rs:41 */
        if (m.seq.empty()) panic("empty usage sequence");
        m.last_unit_start_time = creation_time;
        m.last_poll_time = creation_time;
    }
    return m;
}

struct PodGroup {                    /* horizontal_pod_autoscaler/interface.rs:19-33 */
    std::string name;
    uint64_t initial = 0, max_count = 0;
    Pod tmpl;
    bool has_tcpu = false, has_tram = false;
    double tcpu = 0.0, tram = 0.0;
    RuntimeUsageConfig usage;
};
struct PodGroupInfo {                /* interface.rs:37-45 */
    double creation_time = 0.0;
    std::set<std::string> created_pods;
    uint64_t total_created = 0;
    std::shared_ptr<PodGroup> group;
};

struct CAGroup {                     /* cluster_autoscaler/interface.rs:8-18 */
    bool has_max = false;
    uint64_t max_count = 0, current_count = 0, total_allocated = 0;
    Node tmpl;
};

struct Config {
    double scheduling_cycle_interval = 10.0;
    bool cond_move = false;
    double as_to_ps = 0, ps_to_sched = 0, sched_to_as = 0, as_to_node = 0, as_to_ca = 0, as_to_hpa = 0;
    bool ca_enabled = false;
    double ca_scan_interval = 10.0;
    uint64_t ca_max_node_count = 0;
    double ca_threshold = 0.5;
    std::vector<std::pair<std::string, CAGroup>> ca_groups;  /* config order */
    bool hpa_enabled = false;
    double hpa_scan_interval = 60.0;
    double hpa_tolerance = 0.1;
    double score_weight = 1.0;      /* LeastAllocatedResources weight, kube_scheduler.rs:55 */
    /* score plugins of the default profile: bit 0 LeastAllocatedResources, bit 1 MostAllocatedResources
       (an extension: not in the reference registry, plugin.rs:13-23) */
    uint32_t score_plugins = 1;
    double most_allocated_weight = 1.0;
};

struct DefaultGroup {
    bool has_count = false;
    uint64_t count = 1;
    Node tmpl;  /* name may be empty */
};

struct TraceEvent {
    double ts;
    int kind;  /* K10S_EV_AS_* destination kinds */
    Node node;
    std::string name;
    Pod pod;
    std::shared_ptr<PodGroup> group;
};

/* ------------------------------------------------------------------------------------------ */
/* Rust std BinaryHeap<QueuedPodInfo> (alloc/collections/binary_heap): push = sift_up(0, n);   */
/* pop = swap last into root, sift_down_to_bottom(0), sift_up.  Ord for QueuedPodInfo:         */
/* other.timestamp.total_cmp(&self.timestamp) (queue.rs:29-33), so "a <= b" <=> a.ts >= b.ts. */
/* ------------------------------------------------------------------------------------------ */
struct QueuedPodInfo {
    double timestamp = 0.0;
    uint64_t attempts = 0;
    double initial_attempt_timestamp = 0.0;
    std::string pod_name;
};
static inline bool qpi_le(const QueuedPodInfo& a, const QueuedPodInfo& b) {
    /* a <= b  <=>  cmp(a, b) != Greater, cmp(a,b) = b.ts.total_cmp(a.ts) */
    return total_cmp(b.timestamp, a.timestamp) != 1;
}
struct RustBinaryHeap {
    std::vector<QueuedPodInfo> data;
    size_t sift_up(size_t start, size_t pos) {
        QueuedPodInfo elem = std::move(data[pos]);
        while (pos > start) {
            size_t parent = (pos - 1) / 2;
            if (qpi_le(elem, data[parent])) break;
            data[pos] = std::move(data[parent]);
            pos = parent;
        }
        data[pos] = std::move(elem);
        return pos;
    }
    void sift_down_to_bottom(size_t pos) {
        size_t end = data.size();
        size_t start = pos;
        QueuedPodInfo elem = std::move(data[pos]);
        size_t child = 2 * pos + 1;
        size_t lim = end >= 2 ? end - 2 : 0;
        while (child <= lim && end >= 2) {
            child += qpi_le(data[child], data[child + 1]) ? 1 : 0;
            data[pos] = std::move(data[child]);
            pos = child;
            child = 2 * pos + 1;
        }
        if (child == end - 1) {
            data[pos] = std::move(data[child]);
            pos = child;
        }
        data[pos] = std::move(elem);
        sift_up(start, pos);
    }
    void push(QueuedPodInfo x) {
        size_t old_len = data.size();
        data.push_back(std::move(x));
        sift_up(0, old_len);
    }
    bool pop(QueuedPodInfo& out) {
        if (data.empty()) return false;
        QueuedPodInfo item = std::move(data.back());
        data.pop_back();
        if (!data.empty()) {
            std::swap(item, data[0]);
            sift_down_to_bottom(0);
        }
        out = std::move(item);
        return true;
    }
    size_t size() const { return data.size(); }
};

/* UnschedulablePodKey (queue.rs:49-75): (insert_timestamp total_cmp, pod_name) */
struct UnschedKey {
    std::string pod_name;
    double insert_timestamp;
    bool operator<(const UnschedKey& o) const {
        int c = total_cmp(insert_timestamp, o.insert_timestamp);
        if (c != 0) return c < 0;
        return pod_name < o.pod_name;
    }
};

/* ------------------------------------------------------------------------------------------ */
/* KubeScheduler::schedule_one (kube_scheduler.rs:68-151) with Fit (plugin.rs:34-45) and       */
/* LeastAllocatedResources (plugin.rs:52-63).                                                  */
/* ------------------------------------------------------------------------------------------ */
enum SchedErr { SE_OK = 0, SE_NO_NODES = 1, SE_NO_SUFFICIENT = 2, SE_ZEROS = 3 };

static double least_allocated_score(const Pod& pod, const Node& node) {
    double cpu_score = (double)(uint32_t)(node.alloc_cpu - pod.cpu) * 100.0 / (double)node.alloc_cpu;
    double ram_score = (double)(uint64_t)(node.alloc_ram - pod.ram) * 100.0 / (double)node.alloc_ram;
    return (cpu_score + ram_score) / 2.0;
}

/* MostAllocatedResources (extension, no reference counterpart): kube-scheduler's MostAllocated
   strategy with requested = capacity - allocatable, per resource (cap - alloc + request) * 100 / cap,
   the two averaged as plugin.rs:52-63 averages its terms; wrapping u32/u64 arithmetic. */
static double most_allocated_score(const Pod& pod, const Node& node) {
    double cpu_score = (double)(uint32_t)(node.cap_cpu - node.alloc_cpu + pod.cpu) * 100.0 / (double)node.cap_cpu;
    double ram_score = (double)(uint64_t)(node.cap_ram - node.alloc_ram + pod.ram) * 100.0 / (double)node.cap_ram;
    return (cpu_score + ram_score) / 2.0;
}

struct ScoreProfile {                 /* the default profile's score plugins (kube_scheduler.rs:44-61) */
    uint32_t plugins = 1;             /* bit 0 LeastAllocatedResources, bit 1 MostAllocatedResources */
    double w_la = 1.0, w_ma = 1.0;
};

static int schedule_one(const Pod& pod, const std::map<std::string, Node>& nodes, const ScoreProfile& prof,
                        std::string& out) {
    if (pod.cpu == 0 && pod.ram == 0) return SE_ZEROS;                /* 74-76 */
    if (nodes.empty()) return SE_NO_NODES;                             /* 78-80 */
    auto lab = pod.labels.find("scheduler_name");                      /* 82-87 */
    if (lab != pod.labels.end() && lab->second != "default_scheduler")
        panic("profiles.get(pod_scheduler).unwrap() on unknown profile");
    std::vector<const Node*> filtered;                                 /* 89 */
    filtered.reserve(nodes.size());
    for (auto& kv : nodes) filtered.push_back(&kv.second);
    {   /* Fit::filter */
        std::vector<const Node*> f2;
        for (const Node* n : filtered)
            if (pod.cpu <= n->alloc_cpu && pod.ram <= n->alloc_ram) f2.push_back(n);
        filtered.swap(f2);
    }
    if (filtered.empty()) return SE_NO_SUFFICIENT;                     /* 109-111 */
    std::map<std::string, std::pair<const Node*, double>> node_scores; /* 113 */
    /* 115-138: one pass per score plugin in profile order, node_scores[name] += score * weight */
    if (prof.plugins & 1u)
        for (const Node* n : filtered) {
            auto it = node_scores.find(n->name);
            if (it == node_scores.end()) it = node_scores.emplace(n->name, std::make_pair(n, 0.0)).first;
            double s = least_allocated_score(pod, *n) * prof.w_la;
            it->second.second += s;
        }
    if (prof.plugins & 2u)
        for (const Node* n : filtered) {
            auto it = node_scores.find(n->name);
            if (it == node_scores.end()) it = node_scores.emplace(n->name, std::make_pair(n, 0.0)).first;
            double s = most_allocated_score(pod, *n) * prof.w_ma;
            it->second.second += s;
        }
    const std::string* assigned = &filtered[0]->name;                   /* 140-148 */
    double max_score = node_scores.at(*assigned).second;
    for (auto& kv : node_scores) {
        double score = kv.second.second;
        if (score >= max_score) {
            assigned = &kv.second.first->name;
            max_score = score;
        }
    }
    out = *assigned;
    return SE_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* dslab-core event queue restated: Event{id, time = clock + delay}; pop min (time, id);       */
/* cancel_event = lazy skip; ids from one global counter.                                      */
/* ------------------------------------------------------------------------------------------ */
struct CAAction { bool up; Node node; std::string name; };
struct ScaleUpInfo { std::vector<Pod> unscheduled_pods; };
struct ScaleDownInfo {
    std::vector<Node> nodes;
    std::unordered_map<std::string, Pod> pods_on_autoscaled_nodes;
    std::unordered_map<std::string, std::set<std::string>> assignments;
};

struct Ev {
    double time = 0.0;
    uint64_t id = 0;
    int kind = 0;
    int slot = -1;                 /* node component (pool context) for N_* kinds */
    std::string pod, node;
    double t = 0.0;                /* assign/finish/removal/add/start/not_scheduled time */
    bool flag = false;             /* removed flag; has_assigned for remove-pod response */
    std::shared_ptr<Node> node_obj;
    std::shared_ptr<Pod> pod_obj;
    std::shared_ptr<PodGroup> group;
    std::shared_ptr<PodGroupInfo> group_info;
    std::shared_ptr<ScaleUpInfo> up;
    std::shared_ptr<ScaleDownInfo> down;
};
struct EvCmp {
    bool operator()(const std::shared_ptr<Ev>& a, const std::shared_ptr<Ev>& b) const {
        int c = total_cmp(a->time, b->time);
        if (c != 0) return c > 0;
        return a->id > b->id;
    }
};

struct RunningPodInfo {             /* node_component.rs:24-31 */
    bool has_event = false;
    uint64_t event_id = 0;
    bool has_group = false;
    std::string group;
    uint32_t cpu = 0;
    uint64_t ram = 0;
    bool has_cpu_model = false, has_ram_model = false;
    UsageModel cpu_model, ram_model;
};
struct NodeComponent {              /* node_component.rs:33-47 */
    bool has_runtime = false;
    Node node;
    std::unordered_map<std::string, RunningPodInfo> running_pods;
    std::unordered_set<std::string> canceled_pods;
    bool removed = false;
    double removal_time = 0.0;
};

struct LogEntry { uint64_t id; double time; int kind; std::string pod, node; int slot; };
struct Placement { std::string pod, node; double assign_time; };

struct Counters {
    uint64_t total_nodes_in_trace = 0, total_pods_in_trace = 0, pods_succeeded = 0,
             pods_unschedulable = 0, pods_failed = 0, pods_removed = 0, total_scaled_up_nodes = 0,
             total_scaled_down_nodes = 0, total_scaled_up_pods = 0, total_scaled_down_pods = 0,
             processed_nodes = 0, terminated_pods = 0;
    uint64_t placements = 0, attempts = 0, events = 0;
    uint64_t requeued = 0, flushed = 0; /* unschedulable -> action queue moves (all / flush) */
};

class Sim {
public:
    Config cfg;
    std::vector<DefaultGroup> default_cluster;
    std::vector<TraceEvent> cluster_trace, workload_trace;

    /* dslab state */
    double clock = 0.0;
    uint64_t next_id = 0;
    std::priority_queue<std::shared_ptr<Ev>, std::vector<std::shared_ptr<Ev>>, EvCmp> queue;
    std::unordered_set<uint64_t> canceled;

    /* api server (api_server.rs:28-44) */
    std::deque<int> pool;
    std::map<std::string, Node> pending_node_creation;
    std::set<std::string> pending_node_removal, pending_pod_removal;
    std::map<std::string, int> created_nodes;
    std::vector<NodeComponent> comps;

    /* persistent storage (persistent_storage.rs:31-47) */
    std::map<std::string, Node> ps_nodes;
    std::map<std::string, Pod> ps_pods;
    std::unordered_map<std::string, std::set<std::string>> ps_assignments;
    std::map<std::string, Pod> succeeded_pods;
    std::map<std::string, Pod> removed_pods;   /* records for tests; not reference state */
    std::set<std::string> unscheduled_cache;

    /* scheduler (scheduler.rs:30-54) */
    std::map<std::string, Node> s_nodes;
    std::map<std::string, Pod> s_pods;
    std::unordered_map<std::string, std::set<std::string>> s_assignments;
    RustBinaryHeap action_queue;
    std::map<UnschedKey, QueuedPodInfo> unschedulable;

    /* cluster autoscaler */
    double ca_last_cycle_time = 0.0;
    std::map<std::string, CAGroup> ca_groups;

    /* hpa */
    std::map<std::string, PodGroupInfo> hpa_groups;

    /* metrics collector (collector.rs) */
    GaugeMetrics gauge;                 /* collector.rs:169-190 */
    size_t gauge_cap = 0;               /* rows kept (0 = gauge recording off) */
    std::vector<std::array<double, 8>> gauge_rows;
    Counters c;
    Estimator pod_duration, sched_latency, queue_time;
    std::map<std::string, std::pair<Estimator, Estimator>> pod_utilization;

    /* outputs */
    bool log_events = false;
    std::vector<LogEntry> log;
    std::vector<Placement> placements;
    bool panicked = false;
    std::string panic_msg;
    uint64_t panic_event_id = 0;
    double panic_time = 0.0;

    /* ------------------------------------------------------------------ */
    /* dslab-core SimulationState::add_event (rev 4ea3b3a, not vendored; restated): an event with a
       negative delay — one in the past — is refused with a panic ("Event delay is negative! It is not
       allowed to add events from the past."); `delay >= 0.` is false for NaN too. */
    std::shared_ptr<Ev> emit(int kind, double delay) {
        if (!(delay >= 0.0)) panic("Event delay is negative! It is not allowed to add events from the past.");
        auto e = std::make_shared<Ev>();
        e->kind = kind;
        e->id = next_id++;
        e->time = clock + delay;
        queue.push(e);
        return e;
    }
    void cancel(uint64_t id) { canceled.insert(id); }

    /* next non-canceled event (not popped); nullptr if none */
    std::shared_ptr<Ev> peek() {
        while (!queue.empty()) {
            auto e = queue.top();
            if (canceled.count(e->id)) {
                canceled.erase(e->id);
                queue.pop();
                continue;
            }
            return e;
        }
        return nullptr;
    }

    void initialize();
    bool step();
    int run_until_all_finished(double max_time);
    void step_until_time(double t);

    void dispatch(Ev& e);
    void on_metrics(Ev& e);
    void on_as(Ev& e);
    void on_ps(Ev& e);
    void on_sched(Ev& e);
    void on_node(Ev& e);
    void on_ca(Ev& e);
    void on_hpa(Ev& e);

    /* scheduler helpers (scheduler.rs:118-244) */
    void s_move_pods_to_active(const std::vector<UnschedKey>& keys);
    void s_move_all();
    void s_move_if(std::function<bool(uint32_t, uint64_t)> check);
    void s_move_freed(uint32_t cpu, uint64_t ram);
    void s_release(const Pod& pod);
    void run_scheduling_cycle(double t);
    void ps_clean_up(const Pod& pod);
    std::vector<CAAction> ca_autoscale(std::shared_ptr<ScaleUpInfo> up, std::shared_ptr<ScaleDownInfo> down);
    void collect_pod_metrics(double t);
    int add_node_component(const std::string& name);
};

/* ---------------------------------------------------------------------------------------- */
/* simulator.rs:68-275 — construction + initialize                                            */
/* ---------------------------------------------------------------------------------------- */
void Sim::initialize() {
    /* simulator.rs:150-161: metrics collector emits id 0 (pod metrics) and id 1 (gauge) */
    emit(K10S_EV_M_POD_METRICS_TICK, 0.0);
    emit(K10S_EV_M_GAUGE_TICK, 0.0);

    if (cfg.ca_enabled) {   /* ClusterAutoscaler::new, cluster_autoscaler.rs:163-211 */
        if (cfg.ca_groups.empty()) panic("node groups cannot be empty for CA");
        for (auto& kv : cfg.ca_groups) {
            if (kv.first.empty()) panic("CA node group template needs a name");
            CAGroup g = kv.second;
            g.tmpl.alloc_cpu = g.tmpl.cap_cpu;
            g.tmpl.alloc_ram = g.tmpl.cap_ram;
            g.tmpl.labels["origin"] = "cluster autoscaler";
            g.tmpl.labels["node_group"] = kv.first;
            g.current_count = 0;
            g.total_allocated = 0;
            if (!ca_groups.emplace(kv.first, g).second) panic("unique node group name should be used");
        }
    }

    /* simulator.rs:211-230: pool capacity = max concurrent trace nodes + CA max_node_count */
    {
        std::vector<TraceEvent> ct = cluster_trace;
        std::stable_sort(ct.begin(), ct.end(), [](const TraceEvent& a, const TraceEvent& b) { return a.ts < b.ts; });
        int64_t count = 0, mx = 0;  /* max_nodes_in_trace, simulator.rs:51-65 */
        for (auto& e : ct) {
            if (e.kind == K10S_EV_AS_CREATE_NODE_REQ) count++;
            else if (e.kind == K10S_EV_AS_REMOVE_NODE_REQ) count--;
            mx = std::max(count, mx);
        }
        uint64_t max_nodes = (uint64_t)mx + (cfg.ca_enabled ? cfg.ca_max_node_count : 0);
        for (uint64_t i = 0; i < max_nodes; i++) {
            comps.emplace_back();
            pool.push_back((int)comps.size() - 1);
        }
    }

    /* initialize_default_cluster, simulator.rs:303-344 */
    uint64_t total_nodes = 0;
    for (auto& g : default_cluster) {
        uint64_t cnt = g.has_count ? g.count : 1;
        std::vector<Node> to_add;
        if (cnt == 1 && !g.tmpl.name.empty()) {
            to_add.push_back(g.tmpl);
        } else {
            std::string prefix = g.tmpl.name.empty() ? std::string("default_node") : g.tmpl.name;
            for (uint64_t k = 0; k < cnt; k++) {
                Node n = g.tmpl;
                n.name = prefix + "_" + std::to_string(total_nodes);
                to_add.push_back(n);
                total_nodes++;
            }
        }
        gauge.current_nodes += to_add.size();   /* simulator.rs:339-342 */
        for (auto& n0 : to_add) {   /* KubernetriksSimulation::add_node, simulator.rs:277-301 */
            Node n = n0;
            n.alloc_cpu = n.cap_cpu;
            n.alloc_ram = n.cap_ram;
            if (ps_nodes.count(n.name)) panic("Trying to add node to persistent storage which already exists");
            ps_nodes[n.name] = n;
            ps_assignments[n.name] = {};
            if (created_nodes.count(n.name)) panic("Trying to add node to api server which already exists");
            comps.emplace_back();
            int slot = (int)comps.size() - 1;
            comps[slot].has_runtime = true;
            comps[slot].node = n;
            created_nodes[n.name] = slot;
            s_nodes[n.name] = n;
        }
    }

    /* simulator.rs:234-253: cluster trace events then workload trace events, each stably sorted
       by timestamp (generic.rs:78,105), emitted by the client context at delay = ts. */
    auto emit_trace = [&](std::vector<TraceEvent>& tr, bool cluster) {
        std::stable_sort(tr.begin(), tr.end(), [](const TraceEvent& a, const TraceEvent& b) { return a.ts < b.ts; });
        for (auto& te : tr) {
            auto e = emit(te.kind, te.ts);
            if (te.kind == K10S_EV_AS_CREATE_NODE_REQ) {
                if (cluster) c.total_nodes_in_trace++;
                Node n = te.node;
                n.alloc_cpu = n.cap_cpu;  /* generic.rs:112 */
                n.alloc_ram = n.cap_ram;
                e->node_obj = std::make_shared<Node>(n);
                e->node = n.name;
            } else if (te.kind == K10S_EV_AS_REMOVE_NODE_REQ) {
                e->node = te.name;
            } else if (te.kind == K10S_EV_AS_CREATE_POD_REQ) {
                if (!cluster) c.total_pods_in_trace++;
                e->pod_obj = std::make_shared<Pod>(te.pod);
                e->pod = te.pod.name;
            } else if (te.kind == K10S_EV_AS_REMOVE_POD_REQ) {
                e->pod = te.name;
            } else if (te.kind == K10S_EV_AS_CREATE_GROUP_REQ) {
                e->group = te.group;
            }
        }
    };
    emit_trace(cluster_trace, true);
    emit_trace(workload_trace, false);

    /* Scheduler::start, scheduler.rs:78-81 */
    emit(K10S_EV_S_RUN_CYCLE, 0.0);
    emit(K10S_EV_S_FLUSH, 0.0);
    if (cfg.ca_enabled) emit(K10S_EV_CA_TICK, 0.0);      /* cluster_autoscaler.rs:217-224 */
    if (cfg.hpa_enabled) emit(K10S_EV_HPA_TICK, 0.0);    /* horizontal_pod_autoscaler.rs:149-156 */
}

bool Sim::step() {
    auto e = peek();
    if (!e) return false;
    queue.pop();
    clock = e->time;
    c.events++;
    if (log_events) log.push_back({e->id, e->time, e->kind, e->pod, e->node, e->slot});
    dispatch(*e);
    return true;
}

/* RunUntilAllPodsAreFinishedCallbacks::on_step (simulation_callbacks.rs:86-91) + the loop of
   run_with_callbacks (simulator.rs:359-361).  Returns 0 finished, 1 time limit, 2 panic,
   3 queue empty. */
int Sim::run_until_all_finished(double max_time) {
    try {
        for (;;) {
            if (std::fmod(clock, 1000.0) == 0.0 && c.terminated_pods >= c.total_pods_in_trace) return 0;
            auto e = peek();
            if (!e) return 3;
            if (e->time > max_time) return 1;
            step();
        }
    } catch (RefPanic& p) {
        panicked = true;
        panic_msg = p.what();
        panic_time = clock;
        return 2;
    }
}

/* dslab step_until_time: process events with time <= t, then set the clock to t. */
void Sim::step_until_time(double t) {
    try {
        for (;;) {
            auto e = peek();
            if (!e || e->time > t) break;
            step();
        }
        clock = t;
    } catch (RefPanic& p) {
        panicked = true;
        panic_msg = p.what();
        panic_time = clock;
    }
}

void Sim::dispatch(Ev& e) {
    int k = e.kind;
    if (k <= K10S_EV_M_GAUGE_TICK) on_metrics(e);
    else if (k <= K10S_EV_AS_CREATE_GROUP_REQ) on_as(e);
    else if (k <= K10S_EV_PS_POD_REMOVED) on_ps(e);
    else if (k <= K10S_EV_S_REMOVE_POD) on_sched(e);
    else if (k <= K10S_EV_N_REMOVE_POD) on_node(e);
    else if (k <= K10S_EV_CA_RESP) on_ca(e);
    else on_hpa(e);
}

/* ---------------------------------------------------------------------------------------- */
/* MetricsCollector (collector.rs:263-337, 410-431)                                           */
/* ---------------------------------------------------------------------------------------- */
void Sim::collect_pod_metrics(double t) {
    pod_utilization.clear();
    std::map<std::string, size_t> counts;
    for (auto& kv : created_nodes)
        for (auto& rp : comps[kv.second].running_pods)
            if (rp.second.has_group) counts[rp.second.group] += 1;
    for (auto& kv : created_nodes) {
        for (auto& rp : comps[kv.second].running_pods) {
            RunningPodInfo& info = rp.second;
            if (!info.has_group) continue;
            size_t total = counts.at(info.group);
            double cu = info.has_cpu_model ? info.cpu_model.current_usage(t, true, total) : 0.0;
            double ru = info.has_ram_model ? info.ram_model.current_usage(t, true, total) : 0.0;
            auto& u = pod_utilization[info.group];
            u.first.add(cu);
            u.second.add(ru);
        }
    }
}

void Sim::on_metrics(Ev& e) {
    if (e.kind == K10S_EV_M_POD_METRICS_TICK) {
        collect_pod_metrics(e.time);
        emit(K10S_EV_M_POD_METRICS_TICK, 60.0);
    } else {
        /* record_gauge_metrics (collector.rs:352-407): a CSV row, no simulation state changes.
           collect_utilizations sums over api_server.all_created_nodes() — HashMap order in the
           reference (not bit-stable); here name order (= the engine's order, defined). */
        if (gauge_rows.size() < gauge_cap) {
            double navg_c = 0.0, navg_r = 0.0;
            uint64_t rq_c = 0, rq_r = 0, cap_c = 0, cap_r = 0;
            for (auto& cn : created_nodes) {
                const Node& n = comps[cn.second].node;
                uint64_t cr = (uint64_t)n.cap_cpu - (uint64_t)n.alloc_cpu;
                uint64_t rr = (uint64_t)n.cap_ram - (uint64_t)n.alloc_ram;
                navg_c += (double)cr / (double)n.cap_cpu;
                navg_r += (double)rr / (double)n.cap_ram;
                rq_c += cr;
                rq_r += rr;
                cap_c += (uint64_t)n.cap_cpu;
                cap_r += (uint64_t)n.cap_ram;
            }
            navg_c /= (double)created_nodes.size();
            navg_r /= (double)created_nodes.size();
            gauge_rows.push_back({e.time, (double)gauge.current_nodes, (double)gauge.current_pods,
                                  (double)gauge.pods_in_scheduling_queues, navg_c, navg_r,
                                  (double)rq_c / (double)cap_c, (double)rq_r / (double)cap_r});
        }
        emit(K10S_EV_M_GAUGE_TICK, 5.0);
    }
}

/* ---------------------------------------------------------------------------------------- */
/* KubeApiServer::on (api_server.rs:127-457)                                                  */
/* ---------------------------------------------------------------------------------------- */
void Sim::on_as(Ev& e) {
    switch (e.kind) {
    case K10S_EV_AS_CREATE_NODE_REQ: {            /* 132-146 */
        gauge.current_nodes += 1;
        Node n = *e.node_obj;
        n.alloc_cpu = n.cap_cpu;
        n.alloc_ram = n.cap_ram;
        pending_node_creation[n.name] = n;
        auto f = emit(K10S_EV_PS_CREATE_NODE_REQ, cfg.as_to_ps);
        f->node_obj = std::make_shared<Node>(n);
        f->node = n.name;
        break;
    }
    case K10S_EV_AS_CREATE_NODE_RESP: {           /* 147-150 -> handle_create_node 96-115 */
        auto it = pending_node_creation.find(e.node);
        if (it == pending_node_creation.end()) panic("pending_node_creation_requests.remove().unwrap()");
        Node n = it->second;
        pending_node_creation.erase(it);
        if (pool.empty()) panic("No nodes to allocate in pool");   /* node_component_pool.rs:56-59 */
        int slot = pool.front();
        pool.pop_front();
        comps[slot].has_runtime = true;
        comps[slot].node = n;
        if (created_nodes.count(n.name)) panic("Trying to add node to api server which already exists");
        created_nodes[n.name] = slot;
        auto f = emit(K10S_EV_PS_NODE_ADDED, cfg.as_to_ps);
        f->node = n.name;
        f->t = e.time;
        break;
    }
    case K10S_EV_AS_CREATE_POD_REQ: {             /* 151-162 */
        gauge.current_pods += 1;
        auto f = emit(K10S_EV_PS_CREATE_POD_REQ, cfg.as_to_ps);
        f->pod_obj = e.pod_obj;
        f->pod = e.pod;
        break;
    }
    case K10S_EV_AS_ASSIGN_REQ: {                 /* 163-193 */
        if (pending_node_removal.count(e.node) || !created_nodes.count(e.node)) return;
        if (pending_pod_removal.count(e.pod)) return;
        auto f = emit(K10S_EV_PS_ASSIGN_REQ, cfg.as_to_ps);
        f->pod = e.pod;
        f->node = e.node;
        f->t = e.t;
        break;
    }
    case K10S_EV_AS_ASSIGN_RESP: {                /* 194-218 */
        auto it = created_nodes.find(e.node);
        if (it == created_nodes.end()) panic("created_nodes.get(node).unwrap() on assign response");
        auto f = emit(K10S_EV_N_BIND, cfg.as_to_node);
        f->slot = it->second;
        f->pod = e.pod;
        f->node = e.node;
        f->pod_obj = e.pod_obj;
        break;
    }
    case K10S_EV_AS_POD_NOT_SCHEDULED: {          /* 219-232 */
        auto f = emit(K10S_EV_PS_POD_NOT_SCHEDULED, cfg.as_to_ps);
        f->pod = e.pod;
        f->t = e.t;
        break;
    }
    case K10S_EV_AS_POD_STARTED: {                /* 233-246 */
        auto f = emit(K10S_EV_PS_POD_STARTED, cfg.as_to_ps);
        f->pod = e.pod;
        f->t = e.t;
        break;
    }
    case K10S_EV_AS_POD_FINISHED: {               /* 247-277 */
        c.terminated_pods++;
        c.pods_succeeded++;
        gauge.current_pods -= 1;
        auto f = emit(K10S_EV_PS_POD_FINISHED, cfg.as_to_ps);
        f->pod = e.pod;
        f->node = e.node;
        f->t = e.t;
        break;
    }
    case K10S_EV_AS_REMOVE_NODE_REQ: {            /* 278-286 */
        pending_node_removal.insert(e.node);
        auto f = emit(K10S_EV_PS_REMOVE_NODE_REQ, cfg.as_to_ps);
        f->node = e.node;
        break;
    }
    case K10S_EV_AS_REMOVE_NODE_RESP: {           /* 287-296 */
        auto it = created_nodes.find(e.node);
        if (it == created_nodes.end()) panic("created_nodes.get(node).unwrap() on remove response");
        auto f = emit(K10S_EV_N_REMOVE_NODE, cfg.as_to_node);
        f->slot = it->second;
        f->node = e.node;
        break;
    }
    case K10S_EV_AS_NODE_REMOVED: {               /* 297-319 */
        auto it = created_nodes.find(e.node);
        if (it == created_nodes.end()) panic("created_nodes.remove(node).unwrap()");
        gauge.current_nodes -= 1;
        int slot = it->second;
        created_nodes.erase(it);
        NodeComponent& nc = comps[slot];             /* reclaim_component, node_component_pool.rs:68-77 */
        nc.has_runtime = false;
        nc.removed = false;
        nc.removal_time = 0.0;
        nc.canceled_pods.clear();
        nc.running_pods.clear();
        pool.push_back(slot);
        pending_node_removal.erase(e.node);
        auto f = emit(K10S_EV_PS_NODE_REMOVED, cfg.as_to_ps);
        f->node = e.node;
        f->t = e.t;
        break;
    }
    case K10S_EV_AS_CA_REQ: {                     /* 320-327 */
        emit(K10S_EV_PS_CA_REQ, cfg.as_to_ps);
        break;
    }
    case K10S_EV_AS_CA_RESP: {                    /* 328-341 */
        auto f = emit(K10S_EV_CA_RESP, cfg.as_to_ca);
        f->up = e.up;
        f->down = e.down;
        break;
    }
    case K10S_EV_AS_REMOVE_POD_REQ: {             /* 342-350: quirk — inserts into NODE removal set */
        pending_node_removal.insert(e.pod);
        auto f = emit(K10S_EV_PS_REMOVE_POD_REQ, cfg.as_to_ps);
        f->pod = e.pod;
        break;
    }
    case K10S_EV_AS_REMOVE_POD_RESP: {            /* 351-369 */
        if (e.flag) {
            auto it = created_nodes.find(e.node);
            if (it == created_nodes.end()) panic("created_nodes.get(assigned_node).unwrap()");
            auto f = emit(K10S_EV_N_REMOVE_POD, cfg.as_to_node);
            f->slot = it->second;
            f->pod = e.pod;
        } else {
            pending_pod_removal.erase(e.pod);
        }
        break;
    }
    case K10S_EV_AS_POD_REMOVED: {                /* 370-404 */
        pending_pod_removal.erase(e.pod);
        if (e.flag) {
            c.terminated_pods++;
            c.pods_removed++;
            gauge.current_pods -= 1;
        }
        auto f = emit(K10S_EV_PS_POD_REMOVED, cfg.as_to_ps);
        f->pod = e.pod;
        f->flag = e.flag;
        f->t = e.t;
        break;
    }
    case K10S_EV_AS_CREATE_GROUP_REQ: {           /* 405-455 */
        auto g = e.group;
        if (g->tmpl.has_dur) panic("Pod groups with specified duration are not supported.");
        auto info = std::make_shared<PodGroupInfo>();
        info->creation_time = e.time;
        info->group = g;
        gauge.current_pods += g->initial;
        for (uint64_t idx = 0; idx < g->initial; idx++) {
            Pod p = g->tmpl;
            p.name = g->name + "_" + std::to_string(idx);
            p.labels["pod_group"] = g->name;
            p.has_group_ct = true;
            p.group_ct = e.time;
            p.has_usage = true;
            p.usage = g->usage;
            auto f = emit(K10S_EV_PS_CREATE_POD_REQ, cfg.as_to_ps);
            f->pod_obj = std::make_shared<Pod>(p);
            f->pod = p.name;
            info->created_pods.insert(p.name);
            info->total_created++;
        }
        if (cfg.hpa_enabled) {
            auto f = emit(K10S_EV_HPA_REGISTER_GROUP, cfg.as_to_hpa);
            f->group_info = info;
        }
        break;
    }
    default:
        panic("unhandled AS event");
    }
}

/* ---------------------------------------------------------------------------------------- */
/* PersistentStorage::on (persistent_storage.rs:185-490)                                      */
/* ---------------------------------------------------------------------------------------- */
void Sim::ps_clean_up(const Pod& pod) {        /* 173-182 */
    auto it = ps_nodes.find(pod.assigned_node);
    if (it != ps_nodes.end()) {
        it->second.alloc_cpu += pod.cpu;
        it->second.alloc_ram += pod.ram;
    }
    auto a = ps_assignments.find(pod.assigned_node);
    if (a != ps_assignments.end()) a->second.erase(pod.name);
}


void Sim::on_ps(Ev& e) {
    switch (e.kind) {
    case K10S_EV_PS_CREATE_NODE_REQ: {            /* 188-196 */
        const Node& n = *e.node_obj;
        if (ps_nodes.count(n.name)) panic("Trying to add node to persistent storage which already exists");
        ps_nodes[n.name] = n;
        ps_assignments[n.name] = {};
        auto f = emit(K10S_EV_AS_CREATE_NODE_RESP, cfg.as_to_ps);
        f->node = n.name;
        break;
    }
    case K10S_EV_PS_NODE_ADDED: {                 /* 197-224 */
        auto it = ps_nodes.find(e.node);
        if (it == ps_nodes.end()) panic("storage_data.nodes.get_mut(node).unwrap() on NodeAddedToCluster");
        auto f = emit(K10S_EV_S_ADD_NODE, cfg.ps_to_sched);
        f->node = e.node;
        f->node_obj = std::make_shared<Node>(it->second);
        c.processed_nodes++;
        break;
    }
    case K10S_EV_PS_CREATE_POD_REQ: {             /* 225-249 */
        Pod p = *e.pod_obj;
        p.t_created = e.time;
        if (!p.has_usage) {              /* default_resource_usage_config, helpers.rs:26-31 */
            p.has_usage = true;
            p.usage.has_cpu = true;
            p.usage.cpu.kind = 1;
            p.usage.cpu.usage = (double)p.cpu;
            p.usage.has_ram = true;
            p.usage.ram.kind = 1;
            p.usage.ram.usage = (double)p.ram;
        }
        if (ps_pods.count(p.name)) panic("Trying to add pod to persistent storage which already exists");
        ps_pods[p.name] = p;
        auto f = emit(K10S_EV_S_POD_SCHEDULE_REQ, cfg.ps_to_sched);
        f->pod_obj = std::make_shared<Pod>(p);
        f->pod = p.name;
        break;
    }
    case K10S_EV_PS_ASSIGN_REQ: {                 /* 250-295 */
        auto pit = ps_pods.find(e.pod);
        if (pit == ps_pods.end()) panic("storage_data.pods.get_mut(pod).unwrap() on assign");
        Pod& p = pit->second;
        p.t_scheduled = e.t;
        p.sched_status = 1;
        p.assigned_node = e.node;
        unscheduled_cache.erase(e.pod);
        auto nit = ps_nodes.find(e.node);
        if (nit == ps_nodes.end()) panic("storage_data.nodes.get_mut(node).unwrap() on assign");
        nit->second.alloc_cpu -= p.cpu;
        nit->second.alloc_ram -= p.ram;
        auto ait = ps_assignments.find(e.node);
        if (ait == ps_assignments.end()) panic("assignments.get_mut(node).unwrap() on assign");
        ait->second.insert(e.pod);
        auto f = emit(K10S_EV_AS_ASSIGN_RESP, cfg.as_to_ps);
        f->pod = e.pod;
        f->node = e.node;
        f->pod_obj = std::make_shared<Pod>(p);
        break;
    }
    case K10S_EV_PS_POD_NOT_SCHEDULED: {          /* 296-308 */
        auto pit = ps_pods.find(e.pod);
        if (pit == ps_pods.end()) panic("storage_data.pods.get_mut(pod).unwrap() on PodNotScheduled");
        pit->second.sched_status = 0;
        unscheduled_cache.insert(e.pod);
        break;
    }
    case K10S_EV_PS_POD_STARTED: {                /* 309-315 */
        auto pit = ps_pods.find(e.pod);
        if (pit == ps_pods.end()) panic("storage_data.pods.get_mut(pod).unwrap() on PodStartedRunning");
        pit->second.t_running = e.t;
        break;
    }
    case K10S_EV_PS_POD_FINISHED: {               /* 316-351 */
        auto pit = ps_pods.find(e.pod);
        if (pit != ps_pods.end()) {
            Pod p = pit->second;
            ps_pods.erase(pit);
            p.t_finished = e.t;
            ps_clean_up(p);
            if (!p.has_dur) panic("pod.spec.running_duration.unwrap() on finish");
            pod_duration.add(p.dur);
            succeeded_pods[p.name] = p;
        }
        auto f = emit(K10S_EV_S_POD_FINISHED, cfg.ps_to_sched);
        f->pod = e.pod;
        f->node = e.node;
        f->t = e.t;
        break;
    }
    case K10S_EV_PS_REMOVE_NODE_REQ: {            /* 352-361 */
        if (!ps_nodes.erase(e.node)) panic("storage_data.nodes.remove(node).unwrap()");
        if (!ps_assignments.erase(e.node)) panic("assignments.remove(node).unwrap()");
        auto f = emit(K10S_EV_AS_REMOVE_NODE_RESP, cfg.as_to_ps);
        f->node = e.node;
        break;
    }
    case K10S_EV_PS_NODE_REMOVED: {               /* 362-380 */
        auto f = emit(K10S_EV_S_REMOVE_NODE, cfg.ps_to_sched);
        f->node = e.node;
        break;
    }
    case K10S_EV_PS_CA_REQ: {                     /* 381-412 (AutoscaleInfoRequestType::Auto) */
        auto f = emit(K10S_EV_AS_CA_RESP, cfg.as_to_ps);
        if (unscheduled_cache.empty()) {
            auto d = std::make_shared<ScaleDownInfo>();   /* scale_down_info 147-168 */
            for (auto& kv : ps_nodes) d->nodes.push_back(kv.second);
            for (auto& n : d->nodes) {
                auto o = n.labels.find("origin");
                if (o == n.labels.end() || o->second != "cluster autoscaler") continue;
                for (auto& pn : ps_assignments.at(n.name)) {
                    auto pit = ps_pods.find(pn);
                    if (pit == ps_pods.end()) panic("storage_data.pods.get_key_value(pod).unwrap()");
                    d->pods_on_autoscaled_nodes[pn] = pit->second;
                }
            }
            for (auto& kv : ps_assignments) d->assignments[kv.first] = kv.second;
            f->down = d;
        } else {
            auto u = std::make_shared<ScaleUpInfo>();     /* scale_up_info 137-145 */
            for (auto& pn : unscheduled_cache) {
                auto pit = ps_pods.find(pn);
                if (pit == ps_pods.end()) panic("storage_data.pods.get(pod).unwrap() in scale_up_info");
                u->unscheduled_pods.push_back(pit->second);
            }
            f->up = u;
        }
        break;
    }
    case K10S_EV_PS_REMOVE_POD_REQ: {             /* 413-459 */
        auto pit = ps_pods.find(e.pod);
        if (pit == ps_pods.end()) {
            auto f = emit(K10S_EV_AS_REMOVE_POD_RESP, cfg.as_to_ps);
            f->pod = e.pod;
            f->flag = false;
            return;
        }
        Pod p = pit->second;
        ps_pods.erase(pit);
        p.t_removed = e.time;
        bool has_assigned = !p.assigned_node.empty();
        if (has_assigned) {
            ps_clean_up(p);
        } else {
            auto g = emit(K10S_EV_S_REMOVE_POD, cfg.ps_to_sched);
            g->pod = e.pod;
        }
        auto f = emit(K10S_EV_AS_REMOVE_POD_RESP, cfg.as_to_ps);
        f->pod = e.pod;
        f->flag = has_assigned;
        f->node = p.assigned_node;
        removed_pods[p.name] = p;
        break;
    }
    case K10S_EV_PS_POD_REMOVED: {                /* 460-488 */
        if (!e.flag) return;
        auto f = emit(K10S_EV_S_REMOVE_POD, cfg.ps_to_sched);
        f->pod = e.pod;
        break;
    }
    default:
        panic("unhandled PS event");
    }
}

/* ---------------------------------------------------------------------------------------- */
/* Scheduler (scheduler.rs)                                                                   */
/* ---------------------------------------------------------------------------------------- */
void Sim::s_move_pods_to_active(const std::vector<UnschedKey>& keys) {   /* 174-185 */
    for (auto& k : keys) {
        if (!s_pods.count(k.pod_name)) continue;  /* stale entry stays in the map */
        auto it = unschedulable.find(k);
        QueuedPodInfo q = it->second;
        unschedulable.erase(it);
        q.attempts += 1;
        action_queue.push(q);
        c.requeued++;
    }
}
void Sim::s_move_all() {                                                  /* 235-244 */
    std::vector<UnschedKey> keys;
    for (auto& kv : unschedulable) keys.push_back(kv.first);
    s_move_pods_to_active(keys);
}
void Sim::s_move_if(std::function<bool(uint32_t, uint64_t)> check) {      /* 210-233 */
    std::vector<UnschedKey> keys;
    for (auto& kv : unschedulable) {
        auto pit = s_pods.find(kv.second.pod_name);
        if (pit == s_pods.end()) panic("objects_cache.pods.get(pod).unwrap() in move_to_active_queue_if");
        if (check(pit->second.cpu, pit->second.ram)) keys.push_back(kv.first);
    }
    s_move_pods_to_active(keys);
}
void Sim::s_move_freed(uint32_t cpu, uint64_t ram) {                      /* 366-379 */
    uint32_t fc = cpu;
    uint64_t fr = ram;
    s_move_if([&](uint32_t rc, uint64_t rr) {
        if (rc <= fc && rr <= fr) {
            fc -= rc;
            fr -= rr;
            return true;
        }
        return false;
    });
}
void Sim::s_release(const Pod& pod) {                                     /* 153-162 */
    auto it = s_nodes.find(pod.assigned_node);
    if (it == s_nodes.end()) panic("objects_cache.nodes.get_mut(assigned_node).unwrap() in release");
    it->second.alloc_cpu += pod.cpu;
    it->second.alloc_ram += pod.ram;
}

void Sim::run_scheduling_cycle(double t) {                                /* 246-334 */
    gauge.pods_in_scheduling_queues = (uint64_t)action_queue.data.size() + (uint64_t)unschedulable.size();  /* 256-259 */
    double cycle_dur = 0.0;
    QueuedPodInfo next;
    while (action_queue.pop(next)) {
        auto pit = s_pods.find(next.pod_name);
        if (pit == s_pods.end()) continue;
        double queue_t = t - next.initial_attempt_timestamp + cycle_dur;
        const Pod& pod = pit->second;
        double sched_time = 0.000001 * (double)s_nodes.size();   /* model.rs:24-26 */
        cycle_dur += sched_time;
        std::string assigned;
        ScoreProfile prof;
        prof.plugins = cfg.score_plugins;
        prof.w_la = cfg.score_weight;
        prof.w_ma = cfg.most_allocated_weight;
        int r = schedule_one(pod, s_nodes, prof, assigned);
        if (!(pod.cpu == 0 && pod.ram == 0) && !s_nodes.empty()) c.attempts++;
        if (r != SE_OK) {
            next.timestamp = t + cycle_dur;
            UnschedKey key{next.pod_name, next.timestamp};
            unschedulable[key] = next;
            auto f = emit(K10S_EV_AS_POD_NOT_SCHEDULED, cfg.sched_to_as);
            f->pod = next.pod_name;
            f->t = t + cycle_dur;
            continue;
        }
        /* reserve_node_resources 118-123 */
        Node& node = s_nodes.at(assigned);
        node.alloc_cpu -= pod.cpu;
        node.alloc_ram -= pod.ram;
        /* assign_node_to_pod 125-151 */
        s_assignments[assigned].insert(next.pod_name);
        pit->second.assigned_node = assigned;
        auto f = emit(K10S_EV_AS_ASSIGN_REQ, cycle_dur + cfg.sched_to_as);
        f->pod = next.pod_name;
        f->node = assigned;
        f->t = t + cycle_dur;
        c.placements++;
        placements.push_back({next.pod_name, assigned, t + cycle_dur});
        sched_latency.add(sched_time);
        queue_time.add(queue_t);
    }
    emit(K10S_EV_S_RUN_CYCLE, std::fmax(cycle_dur, cfg.scheduling_cycle_interval));
}

void Sim::on_sched(Ev& e) {
    switch (e.kind) {
    case K10S_EV_S_RUN_CYCLE:
        run_scheduling_cycle(e.time);
        break;
    case K10S_EV_S_FLUSH: {                       /* 188-203 */
        std::vector<UnschedKey> keys;
        for (auto& kv : unschedulable)
            if (e.time - kv.second.timestamp > 5.0 * 60.0) keys.push_back(kv.first);
        const uint64_t before = c.requeued;
        s_move_pods_to_active(keys);
        c.flushed += c.requeued - before;
        emit(K10S_EV_S_FLUSH, 30.0);
        break;
    }
    case K10S_EV_S_ADD_NODE: {                    /* 391-410 */
        Node n = *e.node_obj;
        uint32_t ac = n.alloc_cpu;
        uint64_t ar = n.alloc_ram;
        s_nodes[n.name] = n;
        if (cfg.cond_move) {
            /* inverted check (A.5): moves pods that do NOT fit the remaining allocatable */
            s_move_if([&](uint32_t rc, uint64_t rr) {
                if (rc <= ac && rr <= ar) {
                    ac -= rc;
                    ar -= rr;
                    return false;
                }
                return true;
            });
        } else {
            s_move_all();
        }
        break;
    }
    case K10S_EV_S_POD_SCHEDULE_REQ: {            /* 411-421 */
        Pod p = *e.pod_obj;
        s_pods[p.name] = p;
        QueuedPodInfo q;
        q.timestamp = e.time;
        q.attempts = 1;
        q.initial_attempt_timestamp = e.time;
        q.pod_name = p.name;
        action_queue.push(q);
        break;
    }
    case K10S_EV_S_POD_FINISHED: {                /* 422-440 */
        auto pit = s_pods.find(e.pod);
        if (pit == s_pods.end()) panic("objects_cache.pods.remove(pod).unwrap() on finish");
        Pod p = pit->second;
        s_pods.erase(pit);
        auto ait = s_assignments.find(e.node);
        if (ait == s_assignments.end()) panic("assignments.get_mut(node).unwrap() on finish");
        ait->second.erase(e.pod);
        s_release(p);
        if (cfg.cond_move) s_move_freed(p.cpu, p.ram);
        else s_move_all();
        break;
    }
    case K10S_EV_S_REMOVE_NODE: {                 /* 441-444, reschedule 336-364 */
        if (!s_nodes.erase(e.node)) panic("objects_cache.nodes.remove(node).unwrap()");
        auto ait = s_assignments.find(e.node);
        if (ait != s_assignments.end()) {
            std::set<std::string> names = ait->second;
            s_assignments.erase(ait);
            for (auto& pn : names) {
                auto pit = s_pods.find(pn);
                if (pit == s_pods.end()) panic("objects_cache.pods.get_mut(pod).unwrap() in reschedule");
                pit->second.assigned_node.clear();
                QueuedPodInfo q;
                q.timestamp = e.time;
                q.attempts = 1;
                q.initial_attempt_timestamp = e.time;
                q.pod_name = pn;
                action_queue.push(q);
            }
        }
        break;
    }
    case K10S_EV_S_REMOVE_POD: {                  /* 445-474 */
        auto pit = s_pods.find(e.pod);
        if (pit == s_pods.end()) return;
        Pod p = pit->second;
        s_pods.erase(pit);
        if (!p.assigned_node.empty()) {
            s_release(p);
            auto ait = s_assignments.find(p.assigned_node);
            if (ait == s_assignments.end()) panic("assignments.get_mut(node).unwrap() on remove pod");
            ait->second.erase(e.pod);
            if (cfg.cond_move) s_move_freed(p.cpu, p.ram);
            else s_move_all();
        }
        break;
    }
    default:
        panic("unhandled scheduler event");
    }
}

/* ---------------------------------------------------------------------------------------- */
/* NodeComponent::on (node_component.rs:178-335)                                              */
/* ---------------------------------------------------------------------------------------- */
void Sim::on_node(Ev& e) {
    NodeComponent& nc = comps[e.slot];
    switch (e.kind) {
    case K10S_EV_N_BIND: {                        /* 181-226 */
        if (nc.removed) panic("Pod is assigned on node which is being removed, looks like a bug.");
        if (!nc.has_runtime) panic("runtime.unwrap() on bind to reclaimed component");
        if (e.node != nc.node.name) panic("Pod is assigned to node with different node name");
        const Pod& p = *e.pod_obj;
        RunningPodInfo info;
        if (p.has_dur) {                          /* simulate_pod_runtime 114-175 */
            auto f = emit(K10S_EV_N_POD_FINISHED, p.dur + cfg.as_to_node);
            f->slot = e.slot;
            f->pod = p.name;
            f->node = nc.node.name;
            f->t = e.time + p.dur;
            info.has_event = true;
            info.event_id = f->id;
        }
        auto g = p.labels.find("pod_group");
        info.has_group = g != p.labels.end();
        if (info.has_group) info.group = g->second;
        bool has_ct = p.has_group_ct;
        double ct = p.group_ct;
        if (p.has_usage && p.usage.has_cpu) {
            info.has_cpu_model = true;
            info.cpu_model = model_from_config(p.usage.cpu, has_ct, ct);
        }
        if (p.has_usage && p.usage.has_ram) {
            info.has_ram_model = true;
            info.ram_model = model_from_config(p.usage.ram, has_ct, ct);
        }
        info.cpu = p.cpu;
        info.ram = p.ram;
        nc.node.alloc_cpu -= p.cpu;               /* allocate_pod_requests (83-86, called at 164) */
        nc.node.alloc_ram -= p.ram;
        nc.running_pods[p.name] = info;
        auto f = emit(K10S_EV_AS_POD_STARTED, cfg.as_to_node);
        f->pod = p.name;
        f->t = e.time;
        break;
    }
    case K10S_EV_N_POD_FINISHED: {                /* 227-246 */
        auto it = nc.running_pods.find(e.pod);
        if (it == nc.running_pods.end()) panic("running_pods.remove(pod).unwrap() on finish");
        nc.node.alloc_cpu += it->second.cpu;      /* free_pod_requests (88-91, called at 235) */
        nc.node.alloc_ram += it->second.ram;
        nc.running_pods.erase(it);
        auto f = emit(K10S_EV_AS_POD_FINISHED, 0.0);
        f->pod = e.pod;
        f->node = e.node;
        f->t = e.t;
        break;
    }
    case K10S_EV_N_REMOVE_NODE: {                 /* 247-274 */
        if (!nc.has_runtime || e.node != nc.node.name) panic("Trying to remove other node than self");
        for (auto& rp : nc.running_pods) {        /* cancel_all_running_pods 95-112 */
            nc.node.alloc_cpu += rp.second.cpu;   /* free_pod_requests at 108 */
            nc.node.alloc_ram += rp.second.ram;
            nc.canceled_pods.insert(rp.first);
            if (rp.second.has_event) cancel(rp.second.event_id);
        }
        nc.running_pods.clear();
        auto f = emit(K10S_EV_AS_NODE_REMOVED, cfg.as_to_node);
        f->node = e.node;
        f->t = e.time;
        nc.removed = true;
        nc.removal_time = e.time;
        break;
    }
    case K10S_EV_N_REMOVE_POD: {                  /* 275-333 */
        if (!nc.has_runtime) panic("runtime.unwrap() on remove pod at reclaimed component");
        auto it = nc.running_pods.find(e.pod);
        auto f = std::shared_ptr<Ev>();
        if (it != nc.running_pods.end()) {
            bool he = it->second.has_event;
            uint64_t id = it->second.event_id;
            nc.node.alloc_cpu += it->second.cpu;  /* free_pod_requests at 279 */
            nc.node.alloc_ram += it->second.ram;
            nc.running_pods.erase(it);
            if (he) cancel(id);
            f = emit(K10S_EV_AS_POD_REMOVED, cfg.as_to_node);
            f->flag = true;
            f->t = e.time;
        } else if (nc.canceled_pods.count(e.pod)) {
            f = emit(K10S_EV_AS_POD_REMOVED, cfg.as_to_node);
            f->flag = true;
            f->t = nc.removal_time;
        } else {
            f = emit(K10S_EV_AS_POD_REMOVED, cfg.as_to_node);
            f->flag = false;
            f->t = 0.0;
        }
        f->pod = e.pod;
        break;
    }
    default:
        panic("unhandled node event");
    }
}

/* ---------------------------------------------------------------------------------------- */
/* Cluster autoscaler (cluster_autoscaler.rs:230-334, kube_cluster_autoscaler.rs:62-326)      */
/* ---------------------------------------------------------------------------------------- */
static bool node_fits_pod(const Pod& p, const Node& n) { return p.cpu <= n.alloc_cpu && p.ram <= n.alloc_ram; }

std::vector<CAAction> Sim::ca_autoscale(std::shared_ptr<ScaleUpInfo> up, std::shared_ptr<ScaleDownInfo> down) {
    std::vector<CAAction> actions;
    uint64_t max_node_count = cfg.ca_max_node_count;
    if (up) {                                                        /* scale_up 191-245 */
        std::vector<Node> allocated;
        uint64_t cur = 0;
        for (auto& kv : ca_groups) cur += kv.second.current_count;
        /* node_count_over_quota 62-80 */
        bool over = true;
        if (cur < max_node_count) {
            for (auto& kv : ca_groups) {
                const CAGroup& g = kv.second;
                if (!g.has_max || g.current_count < g.max_count) { over = false; break; }
            }
        }
        if (over) return actions;
        for (auto& pod : up->unscheduled_pods) {
            bool fit = false;
            for (auto& n : allocated) {                             /* try_fit_in_allocated_nodes */
                if (node_fits_pod(pod, n)) {
                    n.alloc_cpu -= pod.cpu;
                    n.alloc_ram -= pod.ram;
                    fit = true;
                    break;
                }
            }
            if (fit) continue;
            if (cur >= max_node_count) continue;
            bool found = false;                                        /* try_find_fitting_template */
            for (auto& kv : ca_groups) {
                CAGroup& g = kv.second;
                if (g.has_max && g.current_count >= g.max_count) continue;
                if (node_fits_pod(pod, g.tmpl)) {
                    g.current_count++;
                    g.total_allocated++;
                    Node n = g.tmpl;
                    n.name = n.name + "_" + std::to_string(g.total_allocated);
                    n.alloc_cpu = n.cap_cpu;
                    n.alloc_ram = n.cap_ram;
                    allocated.push_back(n);
                    found = true;
                    break;
                }
            }
            if (found) cur++;
        }
        for (auto& n : allocated) {
            Node m = n;
            m.alloc_cpu = m.cap_cpu;
            m.alloc_ram = m.cap_ram;
            actions.push_back({true, m, m.name});
        }
        return actions;
    }
    if (down) {                                                      /* scale_down 247-306 */
        std::vector<size_t> to_remove;
        auto& nodes = down->nodes;
        for (size_t idx = 0; idx < nodes.size(); idx++) {
            auto o = nodes[idx].labels.find("origin");
            if (o == nodes[idx].labels.end() || o->second != "cluster autoscaler") continue;
            /* is_under_threshold_utilization 128-142 */
            const Node& n = nodes[idx];
            double cu = (double)(uint32_t)(n.cap_cpu - n.alloc_cpu) / (double)n.cap_cpu;
            double ru = (double)(uint64_t)(n.cap_ram - n.alloc_ram) / (double)n.cap_ram;
            double util = cu > ru ? cu : ru;
            if (!(util < cfg.ca_threshold)) continue;
            auto ait = down->assignments.find(n.name);
            if (ait != down->assignments.end()) {
                std::vector<const Pod*> pods;
                for (auto& pn : ait->second) {
                    auto pit = down->pods_on_autoscaled_nodes.find(pn);
                    if (pit == down->pods_on_autoscaled_nodes.end()) panic("pods_on_autoscaled_nodes.get(pod).unwrap()");
                    pods.push_back(&pit->second);
                }
                if (!pods.empty()) {                                  /* all_pods_can_be_moved 148-181 */
                    std::vector<Node> original = nodes;
                    bool ok = true;
                    for (const Pod* p : pods) {
                        bool placed = false;
                        for (size_t j = 0; j < nodes.size(); j++) {
                            if (j == idx) continue;
                            if (node_fits_pod(*p, nodes[j])) {
                                nodes[j].alloc_cpu -= p->cpu;
                                nodes[j].alloc_ram -= p->ram;
                                placed = true;
                                break;
                            }
                        }
                        if (!placed) { nodes = original; ok = false; break; }
                    }
                    if (!ok) continue;
                }
            }
            to_remove.push_back(idx);
        }
        for (size_t idx : to_remove) {
            const Node& n = nodes[idx];
            auto gl = n.labels.find("node_group");
            if (gl == n.labels.end()) panic("labels.get(node_group).unwrap()");
            auto git = ca_groups.find(gl->second);
            if (git == ca_groups.end()) panic("node_groups.get_mut(group).unwrap()");
            git->second.current_count -= 1;
            actions.push_back({false, Node(), n.name});
        }
    }
    return actions;
}

void Sim::on_ca(Ev& e) {
    if (e.kind == K10S_EV_CA_TICK) {                                 /* 230-241 */
        ca_last_cycle_time = e.time;
        emit(K10S_EV_AS_CA_REQ, cfg.as_to_ca);
        return;
    }
    std::vector<CAAction> actions = ca_autoscale(e.up, e.down);      /* 309-331 */
    for (auto& a : actions) {
        if (a.up) {
            auto f = emit(K10S_EV_AS_CREATE_NODE_REQ, cfg.as_to_ca);
            f->node_obj = std::make_shared<Node>(a.node);
            f->node = a.node.name;
            c.total_scaled_up_nodes++;
        } else {
            auto f = emit(K10S_EV_AS_REMOVE_NODE_REQ, cfg.as_to_ca);
            f->node = a.name;
            c.total_scaled_down_nodes++;
        }
    }
    double delay = cfg.ca_scan_interval;
    if (e.time - ca_last_cycle_time > cfg.ca_scan_interval) delay = 0.0;
    emit(K10S_EV_CA_TICK, delay);
}

/* ---------------------------------------------------------------------------------------- */
/* Horizontal pod autoscaler (horizontal_pod_autoscaler.rs:146-257,                           */
/* kube_horizontal_pod_autoscaler.rs:54-216).  Groups are visited in name order (the          */
/* reference iterates a HashMap: nondeterministic for more than one group, A.5).              */
/* ---------------------------------------------------------------------------------------- */
static uint64_t desired_by_metric(uint64_t cur, double value, double target, double tol) {
    double ratio = value / target;
    if (std::fabs(ratio - 1.0) <= tol) return cur;
    return f64_as_u64(std::ceil((double)cur * ratio));
}

void Sim::on_hpa(Ev& e) {
    if (e.kind == K10S_EV_HPA_REGISTER_GROUP) {
        hpa_groups[e.group_info->group->name] = *e.group_info;
        return;
    }
    struct Act { bool up; Pod pod; std::string name; };
    std::vector<Act> actions;
    for (auto& kv : pod_utilization) {
        auto git = hpa_groups.find(kv.first);
        if (git == hpa_groups.end()) panic("pod_groups.get_mut(group).unwrap()");
        PodGroupInfo& info = git->second;
        double cpu = kv.second.first.mean(), ram = kv.second.second.mean();
        const PodGroup& g = *info.group;
        uint64_t cur = info.created_pods.size();
        bool hc = g.has_tcpu, hr = g.has_tram;
        uint64_t dc = hc ? desired_by_metric(cur, cpu, g.tcpu, cfg.hpa_tolerance) : 0;
        uint64_t dr = hr ? desired_by_metric(cur, ram, g.tram, cfg.hpa_tolerance) : 0;
        uint64_t desired;
        if (hc && hr) desired = std::min<uint64_t>(g.max_count, std::max(dc, dr));
        else if (hc) desired = std::min<uint64_t>(g.max_count, dc);
        else if (hr) desired = std::min<uint64_t>(g.max_count, dr);
        else desired = cur;
        if (cur < desired) {
            for (uint64_t i = 0; i < desired - cur; i++) {
                Pod p = g.tmpl;
                p.name = g.name + "_" + std::to_string(info.total_created);
                p.labels["pod_group"] = g.name;
                p.has_group_ct = true;
                p.group_ct = info.creation_time;
                p.has_usage = true;
                p.usage = g.usage;
                actions.push_back({true, p, p.name});
                info.created_pods.insert(p.name);
                info.total_created++;
            }
        } else if (cur > desired) {
            for (uint64_t i = 0; i < cur - desired; i++) {
                std::string n = *info.created_pods.begin();
                info.created_pods.erase(info.created_pods.begin());
                actions.push_back({false, Pod(), n});
            }
        }
    }
    for (auto& a : actions) {
        if (a.up) {
            auto f = emit(K10S_EV_AS_CREATE_POD_REQ, cfg.as_to_ca);   /* quirk: as_to_ca delay */
            f->pod_obj = std::make_shared<Pod>(a.pod);
            f->pod = a.name;
            c.total_scaled_up_pods++;
        } else {
            auto f = emit(K10S_EV_AS_REMOVE_POD_REQ, cfg.as_to_ca);
            f->pod = a.name;
            c.total_scaled_down_pods++;
        }
    }
    emit(K10S_EV_HPA_TICK, cfg.hpa_scan_interval);
}

}  // namespace orc

/* ========================================================================================== */
/* Scenario text parser (format documented in DESIGN.md §Scenario format) and C API.          */
/* ========================================================================================== */
namespace orc {

static std::vector<std::string> split_ws(const std::string& line) {
    std::vector<std::string> out;
    std::istringstream is(line);
    std::string t;
    while (is >> t) out.push_back(t);
    return out;
}
static double pf(const std::string& s) {
    char* end = nullptr;
    double v = std::strtod(s.c_str(), &end);
    if (end == s.c_str() || *end) throw std::runtime_error("bad float: " + s);
    return v;
}
static uint64_t pu64(const std::string& s) {
    char* end = nullptr;
    if (!s.empty() && s[0] == '-') throw std::runtime_error("negative integer: " + s);
    unsigned long long v = std::strtoull(s.c_str(), &end, 10);
    if (end == s.c_str() || *end) throw std::runtime_error("bad integer: " + s);
    return (uint64_t)v;
}
static uint32_t pu32(const std::string& s) {
    uint64_t v = pu64(s);
    if (v > 0xffffffffull) throw std::runtime_error("u32 out of range: " + s);
    return (uint32_t)v;
}
static void parse_labels(const std::vector<std::string>& tk, size_t from, std::map<std::string, std::string>& labels) {
    for (size_t i = from; i < tk.size(); i++) {
        size_t eq = tk[i].find('=');
        if (eq == std::string::npos) throw std::runtime_error("bad label: " + tk[i]);
        labels[tk[i].substr(0, eq)] = tk[i].substr(eq + 1);
    }
}
static bool parse_model(const std::string& s, UsageModelConfig& m) {
    if (s == "none") return false;
    if (s.rfind("constant:", 0) == 0) {
        m.kind = 1;
        m.usage = pf(s.substr(9));
        return true;
    }
    if (s.rfind("pod_group:", 0) == 0) {
        m.kind = 2;
        std::string body = s.substr(10);
        size_t pos = 0;
        while (pos < body.size()) {
            size_t comma = body.find(',', pos);
            std::string unit = body.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
            size_t sl = unit.find('/');
            if (sl == std::string::npos) throw std::runtime_error("bad usage unit: " + unit);
            m.seq.push_back({pf(unit.substr(0, sl)), pf(unit.substr(sl + 1))});
            if (comma == std::string::npos) break;
            pos = comma + 1;
        }
        return true;
    }
    throw std::runtime_error("bad usage model: " + s);
}

static void parse_scenario(Sim& sim, const std::string& text) {
    std::istringstream is(text);
    std::string line;
    bool header = false;
    while (std::getline(is, line)) {
        size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        auto tk = split_ws(line);
        if (tk.empty()) continue;
        const std::string& h = tk[0];
        if (h == "k10s_scenario") { header = true; continue; }
        if (!header) throw std::runtime_error("missing k10s_scenario header");
        if (h == "end") break;
        Config& c = sim.cfg;
        if (h == "config") {
            if (tk.size() != 3) throw std::runtime_error("config needs key value");
            const std::string& k = tk[1];
            if (k == "scheduling_cycle_interval") c.scheduling_cycle_interval = pf(tk[2]);
            else if (k == "enable_unscheduled_pods_conditional_move") c.cond_move = pu64(tk[2]) != 0;
            else if (k == "as_to_ps_network_delay") c.as_to_ps = pf(tk[2]);
            else if (k == "ps_to_sched_network_delay") c.ps_to_sched = pf(tk[2]);
            else if (k == "sched_to_as_network_delay") c.sched_to_as = pf(tk[2]);
            else if (k == "as_to_node_network_delay") c.as_to_node = pf(tk[2]);
            else if (k == "as_to_ca_network_delay") c.as_to_ca = pf(tk[2]);
            else if (k == "as_to_hpa_network_delay") c.as_to_hpa = pf(tk[2]);
            else if (k == "score_weight") c.score_weight = pf(tk[2]);
            else if (k == "most_allocated_weight") c.most_allocated_weight = pf(tk[2]);
            else if (k == "score_plugins") {
                c.score_plugins = (uint32_t)pu64(tk[2]);
                if (c.score_plugins == 0 || c.score_plugins > 3) throw std::runtime_error("score_plugins must be 1, 2 or 3");
            }
            else if (k == "seed" || k == "sim_name") {}
            else throw std::runtime_error("unknown config key " + k);
        } else if (h == "ca_config" || h == "hpa_config") {
            for (size_t i = 1; i + 1 < tk.size(); i += 2) {
                const std::string& k = tk[i];
                const std::string& v = tk[i + 1];
                if (h == "ca_config") {
                    if (k == "enabled") c.ca_enabled = pu64(v) != 0;
                    else if (k == "scan_interval") c.ca_scan_interval = pf(v);
                    else if (k == "max_node_count") c.ca_max_node_count = pu64(v);
                    else if (k == "scale_down_utilization_threshold") c.ca_threshold = pf(v);
                    else throw std::runtime_error("unknown ca_config key " + k);
                } else {
                    if (k == "enabled") c.hpa_enabled = pu64(v) != 0;
                    else if (k == "scan_interval") c.hpa_scan_interval = pf(v);
                    else if (k == "target_threshold_tolerance") c.hpa_tolerance = pf(v);
                    else throw std::runtime_error("unknown hpa_config key " + k);
                }
            }
        } else if (h == "ca_group") {
            if (tk.size() < 5) throw std::runtime_error("ca_group needs name max cpu ram");
            CAGroup g;
            g.has_max = tk[2] != "-";
            if (g.has_max) g.max_count = pu64(tk[2]);
            g.tmpl.name = tk[1];
            g.tmpl.cap_cpu = pu32(tk[3]);
            g.tmpl.cap_ram = pu64(tk[4]);
            parse_labels(tk, 5, g.tmpl.labels);
            c.ca_groups.push_back({tk[1], g});
        } else if (h == "default_group") {
            if (tk.size() < 5) throw std::runtime_error("default_group needs count name cpu ram");
            DefaultGroup g;
            g.has_count = tk[1] != "-";
            if (g.has_count) g.count = pu64(tk[1]);
            g.tmpl.name = tk[2] == "-" ? "" : tk[2];
            g.tmpl.cap_cpu = pu32(tk[3]);
            g.tmpl.cap_ram = pu64(tk[4]);
            parse_labels(tk, 5, g.tmpl.labels);
            sim.default_cluster.push_back(g);
        } else if (h == "cluster" || h == "workload") {
            if (tk.size() < 4) throw std::runtime_error("trace event too short");
            TraceEvent te;
            te.ts = pf(tk[1]);
            const std::string& op = tk[2];
            if (op == "create_node" && h == "cluster") {
                if (tk.size() < 6) throw std::runtime_error("create_node needs name cpu ram");
                te.kind = K10S_EV_AS_CREATE_NODE_REQ;
                te.node.name = tk[3];
                te.node.cap_cpu = pu32(tk[4]);
                te.node.cap_ram = pu64(tk[5]);
                parse_labels(tk, 6, te.node.labels);
            } else if (op == "remove_node" && h == "cluster") {
                te.kind = K10S_EV_AS_REMOVE_NODE_REQ;
                te.name = tk[3];
            } else if (op == "create_pod" && h == "workload") {
                if (tk.size() < 7) throw std::runtime_error("create_pod needs name cpu ram duration");
                te.kind = K10S_EV_AS_CREATE_POD_REQ;
                te.pod.name = tk[3];
                te.pod.cpu = pu32(tk[4]);
                te.pod.ram = pu64(tk[5]);
                te.pod.has_dur = tk[6] != "none";
                if (te.pod.has_dur) te.pod.dur = pf(tk[6]);
                parse_labels(tk, 7, te.pod.labels);
            } else if (op == "remove_pod" && h == "workload") {
                te.kind = K10S_EV_AS_REMOVE_POD_REQ;
                te.name = tk[3];
            } else if (op == "create_pod_group" && h == "workload") {
                if (tk.size() != 13) throw std::runtime_error("create_pod_group needs 10 fields");
                te.kind = K10S_EV_AS_CREATE_GROUP_REQ;
                auto g = std::make_shared<PodGroup>();
                g->name = tk[3];
                g->initial = pu64(tk[4]);
                g->max_count = pu64(tk[5]);
                g->tmpl.name = tk[3];
                g->tmpl.cpu = pu32(tk[6]);
                g->tmpl.ram = pu64(tk[7]);
                g->tmpl.has_dur = tk[8] != "none";
                if (g->tmpl.has_dur) g->tmpl.dur = pf(tk[8]);
                g->has_tcpu = tk[9] != "-";
                if (g->has_tcpu) g->tcpu = pf(tk[9]);
                g->has_tram = tk[10] != "-";
                if (g->has_tram) g->tram = pf(tk[10]);
                g->usage.has_cpu = parse_model(tk[11], g->usage.cpu);
                g->usage.has_ram = parse_model(tk[12], g->usage.ram);
                te.group = g;
            } else {
                throw std::runtime_error("unknown trace op " + op);
            }
            (h == "cluster" ? sim.cluster_trace : sim.workload_trace).push_back(te);
        } else {
            throw std::runtime_error("unknown directive " + h);
        }
    }
}

/* ---- JSON dump ---------------------------------------------------------------------------- */
static void jnum(std::string& o, double x) {
    char buf[64];
    if (std::isnan(x)) o += "NaN";
    else if (std::isinf(x)) o += x > 0 ? "Infinity" : "-Infinity";
    else { std::snprintf(buf, sizeof buf, "%.17g", x); o += buf; }
}
static void jstr(std::string& o, const std::string& s) {
    o += '"';
    for (char ch : s) {
        if (ch == '"' || ch == '\\') { o += '\\'; o += ch; }
        else if ((unsigned char)ch < 0x20) { char b[8]; std::snprintf(b, sizeof b, "\\u%04x", ch); o += b; }
        else o += ch;
    }
    o += '"';
}
static void jest(std::string& o, const char* name, const Estimator& e) {
    o += '"'; o += name; o += "\":[";
    o += std::to_string(e.n); o += ',';
    jnum(o, e.mn); o += ','; jnum(o, e.mx); o += ','; jnum(o, e.mean()); o += ','; jnum(o, e.population_variance());
    o += ",[";
    for (int i = 0; i < 32; i++) { if (i) o += ','; o += std::to_string(e.hist[i]); }
    o += "]]";
}

static std::string dump_json(Sim& s, int status, int flags) {
    std::string o = "{";
    o += "\"status\":" + std::to_string(status);
    o += ",\"panicked\":"; o += s.panicked ? "true" : "false";
    o += ",\"panic\":"; jstr(o, s.panic_msg);
    o += ",\"time\":"; jnum(o, s.clock);
    o += ",\"next_id\":" + std::to_string(s.next_id);
    o += ",\"gauges\":[";
    for (size_t i = 0; i < s.gauge_rows.size(); i++) {
        if (i) o += ',';
        o += '[';
        for (int j = 0; j < 8; j++) { if (j) o += ','; jnum(o, s.gauge_rows[i][j]); }
        o += ']';
    }
    o += ']';
    const Counters& c = s.c;
    o += ",\"counters\":{";
    o += "\"total_nodes_in_trace\":" + std::to_string(c.total_nodes_in_trace);
    o += ",\"total_pods_in_trace\":" + std::to_string(c.total_pods_in_trace);
    o += ",\"pods_succeeded\":" + std::to_string(c.pods_succeeded);
    o += ",\"pods_unschedulable\":" + std::to_string(c.pods_unschedulable);
    o += ",\"pods_failed\":" + std::to_string(c.pods_failed);
    o += ",\"pods_removed\":" + std::to_string(c.pods_removed);
    o += ",\"total_scaled_up_nodes\":" + std::to_string(c.total_scaled_up_nodes);
    o += ",\"total_scaled_down_nodes\":" + std::to_string(c.total_scaled_down_nodes);
    o += ",\"total_scaled_up_pods\":" + std::to_string(c.total_scaled_up_pods);
    o += ",\"total_scaled_down_pods\":" + std::to_string(c.total_scaled_down_pods);
    o += ",\"processed_nodes\":" + std::to_string(c.processed_nodes);
    o += ",\"terminated_pods\":" + std::to_string(c.terminated_pods);
    o += ",\"placements\":" + std::to_string(c.placements);
    o += ",\"attempts\":" + std::to_string(c.attempts);
    o += ",\"events\":" + std::to_string(c.events);
    o += ",\"requeued\":" + std::to_string(c.requeued);
    o += ",\"flushed\":" + std::to_string(c.flushed);
    o += "},\"estimators\":{";
    jest(o, "pod_duration", s.pod_duration); o += ',';
    jest(o, "pod_schedule_time", s.sched_latency); o += ',';
    jest(o, "pod_queue_time", s.queue_time);
    o += "}";
    o += ",\"unschedulable_len\":" + std::to_string(s.unschedulable.size());
    o += ",\"active_len\":" + std::to_string(s.action_queue.size());
    o += ",\"node_counts\":[" + std::to_string(s.created_nodes.size()) + "," + std::to_string(s.ps_nodes.size()) +
         "," + std::to_string(s.s_nodes.size()) + "]";
    if (flags & 1) {
        auto names = [&](const std::map<std::string, Node>& m) {
            o += '[';
            bool f = true;
            for (auto& kv : m) {
                if (!f) o += ',';
                f = false;
                o += '['; jstr(o, kv.first);
                o += ',' + std::to_string(kv.second.cap_cpu) + ',' + std::to_string(kv.second.cap_ram) + ',' +
                     std::to_string(kv.second.alloc_cpu) + ',' + std::to_string(kv.second.alloc_ram) + ']';
            }
            o += ']';
        };
        std::map<std::string, Node> as_nodes;
        for (auto& kv : s.created_nodes) as_nodes[kv.first] = s.comps[kv.second].node;
        o += ",\"nodes\":{\"as\":"; names(as_nodes);
        o += ",\"ps\":"; names(s.ps_nodes);
        o += ",\"s\":"; names(s.s_nodes);
        o += "}";
    }
    o += ",\"hpa_groups\":{";
    bool first = true;
    for (auto& kv : s.hpa_groups) {
        if (!first) o += ',';
        first = false;
        jstr(o, kv.first);
        o += ":[" + std::to_string(kv.second.created_pods.size()) + "," + std::to_string(kv.second.total_created) + "]";
    }
    o += "}";
    if (flags & 1) {
        o += ",\"placements\":[";
        for (size_t i = 0; i < s.placements.size(); i++) {
            if (i) o += ',';
            o += '['; jstr(o, s.placements[i].pod); o += ','; jstr(o, s.placements[i].node); o += ',';
            jnum(o, s.placements[i].assign_time); o += ']';
        }
        o += "]";
        o += ",\"pods\":{";
        bool f2 = true;
        auto add_pod = [&](const Pod& p, int state) {
            if (!f2) o += ',';
            f2 = false;
            jstr(o, p.name);
            o += ":[";
            jnum(o, p.t_created); o += ','; jnum(o, p.t_scheduled); o += ','; jnum(o, p.t_running); o += ',';
            jnum(o, p.t_finished); o += ','; jnum(o, p.t_removed); o += ',' + std::to_string(state) + ']';
        };
        for (auto& kv : s.ps_pods) add_pod(kv.second, 0);
        for (auto& kv : s.succeeded_pods) add_pod(kv.second, 1);
        for (auto& kv : s.removed_pods) add_pod(kv.second, 2);
        o += "}";
    }
    if (flags & 2) {
        o += ",\"log\":[";
        for (size_t i = 0; i < s.log.size(); i++) {
            const LogEntry& l = s.log[i];
            if (i) o += ',';
            o += '[' + std::to_string(l.id) + ',';
            jnum(o, l.time);
            o += ',' + std::to_string(l.kind) + ',';
            jstr(o, l.pod); o += ','; jstr(o, l.node);
            o += ',' + std::to_string(l.slot) + ']';
        }
        o += "]";
    }
    o += "}";
    return o;
}

struct Handle {
    Sim sim;
    int status = -1;
    std::string out;
};

}  // namespace orc

using namespace orc;

extern "C" {

void* orc_new(const char* text, char* err, int errlen) {
    auto* h = new Handle();
    try {
        parse_scenario(h->sim, std::string(text));
        h->sim.initialize();
    } catch (std::exception& ex) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", ex.what());
        delete h;
        return nullptr;
    }
    return h;
}
void orc_free(void* p) { delete (Handle*)p; }
void orc_set_log(void* p, int on) { ((Handle*)p)->sim.log_events = on != 0; }
void orc_set_gauges(void* p, uint32_t cap) { ((Handle*)p)->sim.gauge_cap = cap; }
int orc_run(void* p, double max_time) {
    auto* h = (Handle*)p;
    h->status = h->sim.run_until_all_finished(max_time);
    return h->status;
}
int orc_step_until(void* p, double t) {
    auto* h = (Handle*)p;
    h->sim.step_until_time(t);
    h->status = h->sim.panicked ? 2 : 4;
    return h->status;
}
double orc_time(void* p) { return ((Handle*)p)->sim.clock; }
/* Returns a pointer to a JSON document owned by the handle (valid until the next call). */
const char* orc_result(void* p, int flags) {
    auto* h = (Handle*)p;
    h->out = dump_json(h->sim, h->status, flags);
    return h->out.c_str();
}

/* ---- unit-test surfaces mirroring the reference's inline unit tests ------------------------ */

/* KubeScheduler::schedule_one over nodes given in any order (kept in a BTreeMap by name).
   Returns SchedErr; on OK writes the chosen node's name. */
int orc_schedule_one(int n, const char** names, const uint32_t* cpu, const uint64_t* ram, uint32_t pcpu,
                     uint64_t pram, double weight, char* out, int outlen) {
    std::map<std::string, Node> nodes;
    for (int i = 0; i < n; i++) {
        Node nd;
        nd.name = names[i];
        nd.cap_cpu = nd.alloc_cpu = cpu[i];
        nd.cap_ram = nd.alloc_ram = ram[i];
        nodes[nd.name] = nd;
    }
    Pod pod;
    pod.name = "pod";
    pod.cpu = pcpu;
    pod.ram = pram;
    std::string res;
    ScoreProfile prof;
    prof.w_la = weight;
    int r = schedule_one(pod, nodes, prof, res);
    if (r == SE_OK && out && outlen > 0) std::snprintf(out, (size_t)outlen, "%s", res.c_str());
    return r;
}

/* LeastAllocatedResources::score (plugin.rs:52-63) */
double orc_least_allocated(uint32_t acpu, uint64_t aram, uint32_t pcpu, uint64_t pram) {
    Node nd;
    nd.alloc_cpu = acpu;
    nd.alloc_ram = aram;
    Pod p;
    p.cpu = pcpu;
    p.ram = pram;
    return least_allocated_score(p, nd);
}

/* Push timestamps into the Rust-BinaryHeap replica in order; write pop order (indices). */
int orc_heap_order(int n, const double* ts, int* out) {
    RustBinaryHeap h;
    for (int i = 0; i < n; i++) {
        QueuedPodInfo q;
        q.timestamp = ts[i];
        q.pod_name = std::to_string(i);
        h.push(q);
    }
    QueuedPodInfo q;
    int k = 0;
    while (h.pop(q)) out[k++] = std::atoi(q.pod_name.c_str());
    return k;
}

/* Order of UnschedulablePodKey entries in the BTreeMap (queue.rs:55-61). */
int orc_unsched_order(int n, const char** names, const double* ts, int* out) {
    std::map<UnschedKey, int> m;
    for (int i = 0; i < n; i++) m[UnschedKey{names[i], ts[i]}] = i;
    int k = 0;
    for (auto& kv : m) out[k++] = kv.second;
    return k;
}

/* PodGroupResourceUsageModel::current_usage over a series of polls; returns 1 if it panics. */
int orc_pod_group_usage(const char* model, double creation, int n, const double* times,
                        const uint64_t* counts, double* out) {
    try {
        UsageModelConfig cfgm;
        if (!parse_model(std::string(model), cfgm)) return 2;
        UsageModel m = model_from_config(cfgm, true, creation);
        for (int i = 0; i < n; i++) out[i] = m.current_usage(times[i], true, counts[i]);
        return 0;
    } catch (RefPanic&) {
        return 1;
    } catch (std::exception&) {
        return 3;
    }
}

/* max_nodes_in_trace (simulator.rs:51-65): kinds 1 = create, 2 = remove, 0 = other. */
uint64_t orc_max_nodes_in_trace(int n, const int* kinds) {
    int64_t count = 0, mx = 0;
    for (int i = 0; i < n; i++) {
        if (kinds[i] == 1) count++;
        else if (kinds[i] == 2) count--;
        mx = std::max(count, mx);
    }
    return (uint64_t)mx;
}

}  // extern "C"
