// k10s_builder.cpp — scenario text -> integer tables (see k10s_builder.h).
#include "k10s_builder.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <set>
#include <sstream>
#include <stdexcept>

namespace k10s {
namespace {

struct BNode {
    std::string name;
    uint32_t cpu = 0;
    uint64_t ram = 0;
    std::map<std::string, std::string> labels;
};
struct BModel {
    uint8_t kind = MODEL_NONE;
    double usage = 0.0;
    std::vector<std::pair<double, double>> units;
};
struct BGroup {
    std::string name;
    uint64_t initial = 0, max = 0;
    uint32_t cpu = 0;
    uint64_t ram = 0;
    bool has_dur = false;
    bool has_tcpu = false, has_tram = false;
    double tcpu = 0, tram = 0;
    BModel cpu_m, ram_m;
};
struct BTrace {
    double ts;
    int kind;          // K10S_EV_AS_*
    BNode node;        // create_node
    std::string name;  // remove_node / remove_pod / create_pod name
    uint32_t cpu = 0;
    uint64_t ram = 0;
    bool has_dur = false;
    double dur = 0;
    int group = -1;    // index into parsed groups (file order)
    uint32_t pos = 0;  // position in its own trace (file order)
};
struct BCAGroup {
    std::string name;
    bool has_max = false;
    uint64_t max = 0;
    uint32_t cpu = 0;
    uint64_t ram = 0;
    std::map<std::string, std::string> labels;
};
struct BDefault {
    bool has_count = false;
    uint64_t count = 1;
    BNode tmpl;
};

std::vector<std::string> toks(const std::string& line) {
    std::vector<std::string> out;
    std::istringstream is(line);
    std::string t;
    while (is >> t) out.push_back(t);
    return out;
}
double f64(const std::string& s) {
    char* end = nullptr;
    double v = std::strtod(s.c_str(), &end);
    if (end == s.c_str() || *end || !std::isfinite(v)) throw std::runtime_error("bad float '" + s + "'");
    return v;
}
uint64_t u64(const std::string& s) {
    if (s.empty() || s[0] == '-' || s[0] == '+') throw std::runtime_error("bad integer '" + s + "'");
    char* end = nullptr;
    errno = 0;
    unsigned long long v = std::strtoull(s.c_str(), &end, 10);
    if (end == s.c_str() || *end || errno) throw std::runtime_error("bad integer '" + s + "'");
    return (uint64_t)v;
}
uint32_t u32(const std::string& s) {
    uint64_t v = u64(s);
    if (v > 0xFFFFFFFFull) throw std::runtime_error("u32 out of range '" + s + "'");
    return (uint32_t)v;
}
void labels(const std::vector<std::string>& tk, size_t from, std::map<std::string, std::string>& out) {
    for (size_t i = from; i < tk.size(); i++) {
        size_t eq = tk[i].find('=');
        if (eq == std::string::npos || eq == 0) throw std::runtime_error("bad label '" + tk[i] + "'");
        out[tk[i].substr(0, eq)] = tk[i].substr(eq + 1);
    }
}
BModel model(const std::string& s) {
    BModel m;
    if (s == "none") return m;
    if (s.rfind("constant:", 0) == 0) {
        m.kind = MODEL_CONSTANT;
        m.usage = f64(s.substr(9));
        return m;
    }
    if (s.rfind("pod_group:", 0) == 0) {
        m.kind = MODEL_POD_GROUP;
        std::string body = s.substr(10);
        size_t pos = 0;
        double total = 0;
        while (pos <= body.size()) {
            size_t comma = body.find(',', pos);
            std::string u = body.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
            size_t sl = u.find('/');
            if (sl == std::string::npos) throw std::runtime_error("bad usage unit '" + u + "'");
            double d = f64(u.substr(0, sl)), l = f64(u.substr(sl + 1));
            if (!(d >= 0)) throw std::runtime_error("negative usage unit duration");
            total += d;
            m.units.push_back({d, l});
            if (comma == std::string::npos) break;
            pos = comma + 1;
        }
        if (m.units.empty() || !(total > 0)) throw std::runtime_error("pod_group usage sequence must have positive total duration");
        return m;
    }
    throw std::runtime_error("bad usage model '" + s + "'");
}

}  // namespace

// Binary trace blocks (k10s_engine_create_bulk).  The blob is a sequence of self-delimiting
// little-endian SoA blocks; nothing may follow the last one.
//   "K10SPOD1" | u64 n | f64 ts[n] | u32 cpu[n] | u32 pad if n odd | u64 ram[n] | f64 dur[n] (NaN: none)
//              | u32 name_off[n + 1] | name bytes[name_off[n]]                -> workload create_pod
//   "K10SNOD1" | u64 n | f64 ts[n] | u32 cpu[n] | u32 pad if n odd | u64 ram[n] | u32 op[n] (0 create,
//              1 remove) | u32 pad if n odd | u32 name_off[n + 1] | name bytes  -> cluster create/remove_node
// Each entry becomes the same BTrace a "workload <ts> create_pod ..." / "cluster <ts> create_node ..."
// / "cluster <ts> remove_node ..." line would (appended after the text's lines of that trace, in
// block order), so the compiled scenario is identical to the all-text one.
// Bytes a name in a binary block may not contain (scenario-text separators; trace_soa.BLOB_NAME_FORBIDDEN).
#define K10S_BLOB_NAME_FORBIDDEN " \t\n\v\f\r#="
static uint64_t parse_bulk_block(const uint8_t* b, uint64_t len, std::vector<BTrace>& cluster,
                                 std::vector<BTrace>& workload) {
    auto need = [&](uint64_t bytes) {
        if (bytes > len) throw std::runtime_error("bulk blob truncated");
    };
    need(16);
    const bool pods = std::memcmp(b, "K10SPOD1", 8) == 0, nodes = std::memcmp(b, "K10SNOD1", 8) == 0;
    if (!pods && !nodes) throw std::runtime_error("bulk blob: bad magic");
    uint64_t n;
    std::memcpy(&n, b + 8, 8);
    if (n > (1ull << 32)) throw std::runtime_error("bulk blob: too many entries");
    const uint64_t pad = 4 * (n & 1);
    const uint64_t o_ts = 16, o_cpu = o_ts + 8 * n, o_ram = o_cpu + 4 * n + pad, o_x = o_ram + 8 * n;
    const uint64_t o_off = pods ? o_x + 8 * n : o_x + 4 * n + pad, o_chr = o_off + 4 * (n + 1);
    need(o_chr);
    std::vector<uint32_t> off(n + 1);
    std::memcpy(off.data(), b + o_off, 4 * (n + 1));
    // the same rules as trace_soa.read_*_blob: offsets start at 0 and never decrease
    if (off[0] != 0) throw std::runtime_error("bulk blob: bad name offsets");
    need(o_chr + off[n]);
    for (uint64_t i = 0; i < n; i++) {
        if (off[i] > off[i + 1] || off[i + 1] > off[n]) throw std::runtime_error("bulk blob: bad name offsets");
        BTrace t;
        std::memcpy(&t.ts, b + o_ts + 8 * i, 8);
        uint32_t cpu;
        uint64_t ram;
        std::memcpy(&cpu, b + o_cpu + 4 * i, 4);
        std::memcpy(&ram, b + o_ram + 8 * i, 8);
        std::string name(reinterpret_cast<const char*>(b + o_chr + off[i]), off[i + 1] - off[i]);
        if (name.empty() || name.find_first_of(K10S_BLOB_NAME_FORBIDDEN) != std::string::npos)
            throw std::runtime_error("bulk blob: invalid name");
        if (pods) {
            double d;
            std::memcpy(&d, b + o_x + 8 * i, 8);
            t.has_dur = d == d;
            if (t.has_dur) t.dur = d;
            t.kind = K10S_EV_AS_CREATE_POD_REQ;
            t.name = name;
            t.cpu = cpu;
            t.ram = ram;
            t.pos = (uint32_t)workload.size();
            workload.push_back(t);
        } else {
            uint32_t op;
            std::memcpy(&op, b + o_x + 4 * i, 4);
            if (op == 0) {
                t.kind = K10S_EV_AS_CREATE_NODE_REQ;
                t.node.name = name;
                t.node.cpu = cpu;
                t.node.ram = ram;
            } else if (op == 1) {
                t.kind = K10S_EV_AS_REMOVE_NODE_REQ;
                t.name = name;
            } else {
                throw std::runtime_error("bulk blob: bad cluster op");
            }
            t.pos = (uint32_t)cluster.size();
            cluster.push_back(t);
        }
    }
    return o_chr + off[n];
}
static void parse_bulk(const uint8_t* b, uint64_t len, std::vector<BTrace>& cluster, std::vector<BTrace>& workload) {
    uint64_t at = 0;
    while (at < len) at += parse_bulk_block(b + at, len - at, cluster, workload);
}

bool build_scenario(const std::string& text, uint32_t group_bound_in, uint32_t ca_bound_in, HostScenario& hs,
                    std::string& err, const uint8_t* bulk, uint64_t bulk_len) {
    try {
        Params& d = hs.defaults;
        std::memset(&d, 0, sizeof d);
        d.scheduling_cycle_interval = 10.0;
        d.as_to_ps_network_delay = 0.050;
        d.ps_to_sched_network_delay = 0.089;
        d.sched_to_as_network_delay = 0.023;
        d.as_to_node_network_delay = 0.152;
        d.as_to_ca_network_delay = 0.67;
        d.as_to_hpa_network_delay = 0.50;
        d.ca_scan_interval = 10.0;
        d.ca_scale_down_utilization_threshold = 0.5;
        d.hpa_scan_interval = 60.0;
        d.hpa_target_threshold_tolerance = 0.1;
        d.score_weight = 1.0;
        d.most_allocated_weight = 1.0;
        d.score_plugins = K10S_SCORE_LEAST_ALLOCATED;
        d.seed = 123;
        std::vector<BCAGroup> cagroups;
        std::vector<BDefault> defaults;
        std::vector<BGroup> groups;
        std::vector<BTrace> cluster, workload;

        std::istringstream is(text);
        std::string line;
        bool header = false;
        while (std::getline(is, line)) {
            size_t hash = line.find('#');
            if (hash != std::string::npos) line.resize(hash);
            auto tk = toks(line);
            if (tk.empty()) continue;
            const std::string& h = tk[0];
            if (h == "k10s_scenario") {
                if (tk.size() != 2 || tk[1] != "1") throw std::runtime_error("unsupported scenario version");
                header = true;
                continue;
            }
            if (!header) throw std::runtime_error("missing 'k10s_scenario 1' header");
            if (h == "end") break;
            if (h == "config") {
                if (tk.size() != 3) throw std::runtime_error("config needs <key> <value>");
                const std::string& k = tk[1];
                const std::string& v = tk[2];
                if (k == "scheduling_cycle_interval") d.scheduling_cycle_interval = f64(v);
                else if (k == "enable_unscheduled_pods_conditional_move") d.enable_unscheduled_pods_conditional_move = u64(v) != 0;
                else if (k == "as_to_ps_network_delay") d.as_to_ps_network_delay = f64(v);
                else if (k == "ps_to_sched_network_delay") d.ps_to_sched_network_delay = f64(v);
                else if (k == "sched_to_as_network_delay") d.sched_to_as_network_delay = f64(v);
                else if (k == "as_to_node_network_delay") d.as_to_node_network_delay = f64(v);
                else if (k == "as_to_ca_network_delay") d.as_to_ca_network_delay = f64(v);
                else if (k == "as_to_hpa_network_delay") d.as_to_hpa_network_delay = f64(v);
                else if (k == "score_weight") d.score_weight = f64(v);
                else if (k == "most_allocated_weight") d.most_allocated_weight = f64(v);
                else if (k == "score_plugins") {
                    d.score_plugins = (uint32_t)u64(v);
                    if (d.score_plugins == 0 || d.score_plugins > 3)
                        throw std::runtime_error("score_plugins must be 1 (LeastAllocated), 2 (MostAllocated) or 3 (both)");
                }
                else if (k == "seed") d.seed = u64(v);
                else if (k == "sim_name") {}
                else throw std::runtime_error("unknown config key '" + k + "'");
            } else if (h == "ca_config" || h == "hpa_config") {
                if (tk.size() % 2 != 1) throw std::runtime_error(h + " needs key/value pairs");
                for (size_t i = 1; i + 1 < tk.size(); i += 2) {
                    const std::string& k = tk[i];
                    const std::string& v = tk[i + 1];
                    if (h == "ca_config") {
                        if (k == "enabled") hs.ca_enabled = u64(v) != 0;
                        else if (k == "scan_interval") d.ca_scan_interval = f64(v);
                        else if (k == "max_node_count") d.ca_max_node_count = u64(v);
                        else if (k == "scale_down_utilization_threshold") d.ca_scale_down_utilization_threshold = f64(v);
                        else throw std::runtime_error("unknown ca_config key '" + k + "'");
                    } else {
                        if (k == "enabled") hs.hpa_enabled = u64(v) != 0;
                        else if (k == "scan_interval") d.hpa_scan_interval = f64(v);
                        else if (k == "target_threshold_tolerance") d.hpa_target_threshold_tolerance = f64(v);
                        else throw std::runtime_error("unknown hpa_config key '" + k + "'");
                    }
                }
            } else if (h == "ca_group") {
                if (tk.size() < 5) throw std::runtime_error("ca_group needs <name> <max|-> <cpu> <ram>");
                BCAGroup g;
                g.name = tk[1];
                g.has_max = tk[2] != "-";
                if (g.has_max) g.max = u64(tk[2]);
                g.cpu = u32(tk[3]);
                g.ram = u64(tk[4]);
                labels(tk, 5, g.labels);
                cagroups.push_back(g);
            } else if (h == "default_group") {
                if (tk.size() < 5) throw std::runtime_error("default_group needs <count|-> <name|-> <cpu> <ram>");
                BDefault g;
                g.has_count = tk[1] != "-";
                if (g.has_count) g.count = u64(tk[1]);
                g.tmpl.name = tk[2] == "-" ? "" : tk[2];
                g.tmpl.cpu = u32(tk[3]);
                g.tmpl.ram = u64(tk[4]);
                labels(tk, 5, g.tmpl.labels);
                defaults.push_back(g);
            } else if (h == "cluster" || h == "workload") {
                if (tk.size() < 4) throw std::runtime_error("trace line too short");
                BTrace t;
                t.ts = f64(tk[1]);
                const std::string& op = tk[2];
                if (h == "cluster" && op == "create_node") {
                    if (tk.size() < 6) throw std::runtime_error("create_node needs <name> <cpu> <ram>");
                    t.kind = K10S_EV_AS_CREATE_NODE_REQ;
                    t.node.name = tk[3];
                    t.node.cpu = u32(tk[4]);
                    t.node.ram = u64(tk[5]);
                    labels(tk, 6, t.node.labels);
                } else if (h == "cluster" && op == "remove_node") {
                    t.kind = K10S_EV_AS_REMOVE_NODE_REQ;
                    t.name = tk[3];
                } else if (h == "workload" && op == "create_pod") {
                    if (tk.size() < 7) throw std::runtime_error("create_pod needs <name> <cpu> <ram> <duration|none>");
                    t.kind = K10S_EV_AS_CREATE_POD_REQ;
                    t.name = tk[3];
                    t.cpu = u32(tk[4]);
                    t.ram = u64(tk[5]);
                    t.has_dur = tk[6] != "none";
                    if (t.has_dur) t.dur = f64(tk[6]);
                    std::map<std::string, std::string> lab;
                    labels(tk, 7, lab);
                    for (auto& kv : lab) {
                        if (kv.first == "scheduler_name" && kv.second != "default_scheduler")
                            throw std::runtime_error("pod " + t.name + ": unknown scheduler profile (reference panics)");
                        if (kv.first == "pod_group" || kv.first == "pod_group_creation_time")
                            throw std::runtime_error("pod " + t.name + ": pod_group labels on trace pods are not supported");
                    }
                } else if (h == "workload" && op == "remove_pod") {
                    t.kind = K10S_EV_AS_REMOVE_POD_REQ;
                    t.name = tk[3];
                } else if (h == "workload" && op == "create_pod_group") {
                    if (tk.size() != 13) throw std::runtime_error("create_pod_group needs 10 fields");
                    t.kind = K10S_EV_AS_CREATE_GROUP_REQ;
                    BGroup g;
                    g.name = tk[3];
                    g.initial = u64(tk[4]);
                    g.max = u64(tk[5]);
                    g.cpu = u32(tk[6]);
                    g.ram = u64(tk[7]);
                    g.has_dur = tk[8] != "none";
                    g.has_tcpu = tk[9] != "-";
                    if (g.has_tcpu) g.tcpu = f64(tk[9]);
                    g.has_tram = tk[10] != "-";
                    if (g.has_tram) g.tram = f64(tk[10]);
                    g.cpu_m = model(tk[11]);
                    g.ram_m = model(tk[12]);
                    t.group = (int)groups.size();
                    groups.push_back(g);
                } else {
                    throw std::runtime_error("unknown trace op '" + h + " " + op + "'");
                }
                auto& tr = h == "cluster" ? cluster : workload;
                t.pos = (uint32_t)tr.size();
                tr.push_back(t);
            } else {
                throw std::runtime_error("unknown directive '" + h + "'");
            }
        }
        if (!header) throw std::runtime_error("empty scenario");
        if (bulk) parse_bulk(bulk, bulk_len, cluster, workload);
        if (hs.ca_enabled && cagroups.empty()) throw std::runtime_error("node groups cannot be empty for CA");

        auto by_ts = [](const BTrace& a, const BTrace& b) { return a.ts < b.ts; };
        std::stable_sort(cluster.begin(), cluster.end(), by_ts);
        std::stable_sort(workload.begin(), workload.end(), by_ts);

        // ---- pod groups and CA groups in name order
        std::vector<int> gorder(groups.size());
        for (size_t i = 0; i < groups.size(); i++) gorder[i] = (int)i;
        std::sort(gorder.begin(), gorder.end(), [&](int a, int b) { return groups[a].name < groups[b].name; });
        for (size_t i = 1; i < gorder.size(); i++)
            if (groups[gorder[i]].name == groups[gorder[i - 1]].name)
                throw std::runtime_error("pod group '" + groups[gorder[i]].name + "' created twice (not supported)");
        std::vector<int> grank(groups.size());
        for (size_t r = 0; r < gorder.size(); r++) grank[gorder[r]] = (int)r;
        std::sort(cagroups.begin(), cagroups.end(), [](const BCAGroup& a, const BCAGroup& b) { return a.name < b.name; });
        for (size_t i = 0; i < cagroups.size(); i++) {
            if (cagroups[i].name.empty()) throw std::runtime_error("CA node group template needs a name");
            if (i && cagroups[i].name == cagroups[i - 1].name) throw std::runtime_error("unique node group name should be used");
        }

        uint32_t gb = group_bound_in;
        if (gb == 0) {
            uint64_t m = 0;
            for (auto& g : groups) m = std::max<uint64_t>(m, std::max(g.initial, g.max));
            gb = (uint32_t)std::min<uint64_t>(m * 8 + 64, 1u << 20);
        }
        uint32_t cb = ca_bound_in;
        if (cb == 0) cb = hs.ca_enabled ? (uint32_t)std::min<uint64_t>(d.ca_max_node_count * 8 + 16, 1u << 20) : 0;
        if (!groups.empty() && gb == 0) gb = 1;
        hs.group_bound = groups.empty() ? 0 : gb;
        hs.ca_bound = cb;

        // ---- default cluster names (simulator.rs:303-344)
        std::vector<BNode> default_nodes;
        uint64_t total_default = 0;
        for (auto& g : defaults) {
            uint64_t cnt = g.has_count ? g.count : 1;
            if (cnt == 1 && !g.tmpl.name.empty()) {
                default_nodes.push_back(g.tmpl);
                continue;
            }
            std::string prefix = g.tmpl.name.empty() ? std::string("default_node") : g.tmpl.name;
            for (uint64_t k = 0; k < cnt; k++) {
                BNode n = g.tmpl;
                n.name = prefix + "_" + std::to_string(total_default++);
                default_nodes.push_back(n);
            }
        }

        // ---- name universes
        std::set<std::string> node_set, pod_set;
        for (auto& n : default_nodes) {
            if (!node_set.insert(n.name).second) throw std::runtime_error("duplicate default-cluster node " + n.name);
        }
        for (auto& t : cluster) {
            if (t.kind == K10S_EV_AS_CREATE_NODE_REQ) node_set.insert(t.node.name);
            else node_set.insert(t.name);
        }
        for (auto& g : cagroups)
            for (uint32_t k = 1; k <= cb; k++) node_set.insert(g.name + "_" + std::to_string(k));
        std::set<std::string> trace_pods;
        for (auto& t : workload) {
            if (t.kind == K10S_EV_AS_CREATE_POD_REQ) {
                if (!trace_pods.insert(t.name).second)
                    throw std::runtime_error("pod '" + t.name + "' created twice in the workload trace (not supported)");
                pod_set.insert(t.name);
            } else if (t.kind == K10S_EV_AS_REMOVE_POD_REQ) {
                pod_set.insert(t.name);
            }
        }
        for (auto& g : groups)
            for (uint32_t k = 0; k < gb; k++) {
                std::string nm = g.name + "_" + std::to_string(k);
                if (trace_pods.count(nm)) throw std::runtime_error("pod-group pod name collides with trace pod " + nm);
                pod_set.insert(nm);
            }
        hs.node_names.assign(node_set.begin(), node_set.end());
        hs.pod_names.assign(pod_set.begin(), pod_set.end());
        std::set<std::string> uni(node_set);
        uni.insert(pod_set.begin(), pod_set.end());
        std::vector<std::string> uvec(uni.begin(), uni.end());
        auto uid_of = [&](const std::string& s) {
            return (uint32_t)(std::lower_bound(uvec.begin(), uvec.end(), s) - uvec.begin());
        };
        auto node_of = [&](const std::string& s) {
            return (uint32_t)(std::lower_bound(hs.node_names.begin(), hs.node_names.end(), s) - hs.node_names.begin());
        };
        auto pod_of = [&](const std::string& s) {
            return (uint32_t)(std::lower_bound(hs.pod_names.begin(), hs.pod_names.end(), s) - hs.pod_names.begin());
        };
        hs.n_nodes = (uint32_t)hs.node_names.size();
        hs.n_pods = (uint32_t)hs.pod_names.size();
        hs.n_uids = (uint32_t)uvec.size();
        hs.node_uid.resize(hs.n_nodes);
        for (uint32_t n = 0; n < hs.n_nodes; n++) hs.node_uid[n] = uid_of(hs.node_names[n]);
        hs.pod_uid.resize(hs.n_pods);
        for (uint32_t p = 0; p < hs.n_pods; p++) hs.pod_uid[p] = uid_of(hs.pod_names[p]);

        // ---- node instance defs
        auto ca_group_of = [&](const std::map<std::string, std::string>& lab) -> int32_t {
            auto it = lab.find("node_group");
            if (it == lab.end()) return -1;
            for (size_t g = 0; g < cagroups.size(); g++)
                if (cagroups[g].name == it->second) return (int32_t)g;
            return -2;
        };
        auto add_def = [&](const std::string& name, uint32_t cpu, uint64_t ram, const std::map<std::string, std::string>& lab) {
            hs.def_node.push_back(node_of(name));
            hs.def_cpu.push_back(cpu);
            hs.def_ram.push_back(ram);
            auto o = lab.find("origin");
            hs.def_ca_origin.push_back(o != lab.end() && o->second == "cluster autoscaler");
            hs.def_ca_group.push_back(ca_group_of(lab));
            return (uint32_t)(hs.def_node.size() - 1);
        };
        for (auto& n : default_nodes) hs.default_defs.push_back(add_def(n.name, n.cpu, n.ram, n.labels));
        hs.n_default = (uint32_t)default_nodes.size();
        std::vector<uint32_t> cluster_def(cluster.size(), 0);
        for (size_t i = 0; i < cluster.size(); i++)
            if (cluster[i].kind == K10S_EV_AS_CREATE_NODE_REQ)
                cluster_def[i] = add_def(cluster[i].node.name, cluster[i].node.cpu, cluster[i].node.ram, cluster[i].node.labels);
        hs.ca_has_max.resize(cagroups.size());
        hs.ca_max.resize(cagroups.size());
        hs.ca_cpu.resize(cagroups.size());
        hs.ca_ram.resize(cagroups.size());
        hs.ca_def.resize(cagroups.size() * (size_t)cb);
        for (size_t g = 0; g < cagroups.size(); g++) {
            hs.ca_group_names.push_back(cagroups[g].name);
            hs.ca_has_max[g] = cagroups[g].has_max;
            hs.ca_max[g] = cagroups[g].max;
            hs.ca_cpu[g] = cagroups[g].cpu;
            hs.ca_ram[g] = cagroups[g].ram;
            std::map<std::string, std::string> lab = cagroups[g].labels;  // cluster_autoscaler.rs:178-187
            lab["origin"] = "cluster autoscaler";
            lab["node_group"] = cagroups[g].name;
            for (uint32_t k = 1; k <= cb; k++)
                hs.ca_def[g * cb + (k - 1)] = add_def(cagroups[g].name + "_" + std::to_string(k), cagroups[g].cpu,
                                                      cagroups[g].ram, lab);
        }

        // ---- pods
        hs.pod_cpu.assign(hs.n_pods, 0);
        hs.pod_ram.assign(hs.n_pods, 0);
        hs.pod_dur.assign(hs.n_pods, 0.0);
        hs.pod_flags.assign(hs.n_pods, 0);
        hs.pod_group.assign(hs.n_pods, -1);
        hs.pod_key.assign(hs.n_pods, 0);
        for (auto& t : workload) {
            if (t.kind != K10S_EV_AS_CREATE_POD_REQ) continue;
            uint32_t p = pod_of(t.name);
            hs.pod_cpu[p] = t.cpu;
            hs.pod_ram[p] = t.ram;
            hs.pod_dur[p] = t.has_dur ? t.dur : 0.0;
            hs.pod_flags[p] = POD_HAS_DEF | POD_PERTURB | (t.has_dur ? POD_HAS_DUR : 0);
            hs.pod_key[p] = t.pos;
        }

        // ---- pod groups (name order)
        const size_t G = groups.size();
        hs.g_pod.assign(G * (size_t)gb, 0);
        hs.g_pos.assign(G * (size_t)gb, 0);
        hs.g_sorted_k.assign(G * (size_t)gb, 0);
        for (size_t r = 0; r < G; r++) {
            const BGroup& g = groups[gorder[r]];
            hs.group_names.push_back(g.name);
            hs.g_initial.push_back((uint32_t)std::min<uint64_t>(g.initial, 0xFFFFFFFFull));
            hs.g_max.push_back((uint32_t)std::min<uint64_t>(g.max, 0xFFFFFFFFull));
            hs.g_cpu.push_back(g.cpu);
            hs.g_ram.push_back(g.ram);
            hs.g_flags.push_back((g.has_tcpu ? GF_HAS_TCPU : 0) | (g.has_tram ? GF_HAS_TRAM : 0) | (g.has_dur ? GF_TMPL_HAS_DUR : 0));
            hs.g_tcpu.push_back(g.tcpu);
            hs.g_tram.push_back(g.tram);
            auto put_model = [&](const BModel& m, std::vector<uint8_t>& kind, std::vector<double>& usage,
                                 std::vector<uint32_t>& off, std::vector<uint32_t>& cnt) {
                kind.push_back(m.kind);
                usage.push_back(m.usage);
                off.push_back((uint32_t)hs.unit_dur.size());
                cnt.push_back((uint32_t)m.units.size());
                for (auto& u : m.units) {
                    hs.unit_dur.push_back(u.first);
                    hs.unit_load.push_back(u.second);
                }
            };
            put_model(g.cpu_m, hs.g_cpu_kind, hs.g_cpu_usage, hs.g_cpu_uoff, hs.g_cpu_ucnt);
            put_model(g.ram_m, hs.g_ram_kind, hs.g_ram_usage, hs.g_ram_uoff, hs.g_ram_ucnt);
            std::vector<std::pair<uint32_t, uint32_t>> ranked;  // (pod idx, k)
            for (uint32_t k = 0; k < gb; k++) {
                uint32_t p = pod_of(g.name + "_" + std::to_string(k));
                hs.g_pod[r * gb + k] = p;
                hs.pod_cpu[p] = g.cpu;
                hs.pod_ram[p] = g.ram;
                hs.pod_dur[p] = 0.0;
                hs.pod_flags[p] = POD_HAS_DEF;
                hs.pod_group[p] = (int32_t)r;
                ranked.push_back({p, k});
            }
            std::sort(ranked.begin(), ranked.end());
            for (uint32_t j = 0; j < gb; j++) {
                hs.g_sorted_k[r * gb + j] = ranked[j].second;
                hs.g_pos[r * gb + ranked[j].second] = j;
            }
        }

        // ---- trace stream: ids 2.. in emission order (cluster then workload), merged by (time, id)
        uint32_t seq = 2;
        std::vector<TraceEv> ct, wt;
        for (size_t i = 0; i < cluster.size(); i++) {
            const BTrace& t = cluster[i];
            TraceEv e;
            e.time = 0.0 + t.ts;  // dslab: time = clock (0 at initialize) + delay, so -0.0 -> +0.0
            e.seq = seq++;
            e.kind = (uint32_t)t.kind;
            e.wpos = K10S_TRACE_CLUSTER;
            if (t.kind == K10S_EV_AS_CREATE_NODE_REQ) {
                e.arg = cluster_def[i];
                hs.total_nodes_in_trace++;
            } else {
                e.arg = node_of(t.name);
            }
            ct.push_back(e);
        }
        hs.n_cluster_trace = (uint32_t)cluster.size();
        // create_pod events among the first k workload events in file (generation) order: a replica
        // with workload_prefix k keeps exactly those (k10s_replica_params.workload_prefix)
        std::vector<uint32_t> is_pod(workload.size(), 0);
        for (const BTrace& t : workload) is_pod[t.pos] = t.kind == K10S_EV_AS_CREATE_POD_REQ ? 1u : 0u;
        hs.wl_pods_upto.assign(1, 0);
        for (uint32_t x : is_pod) hs.wl_pods_upto.push_back(hs.wl_pods_upto.back() + x);
        for (const BTrace& t : workload) {
            TraceEv e;
            e.time = 0.0 + t.ts;  // (as above)
            e.seq = seq++;
            e.kind = (uint32_t)t.kind;
            e.wpos = t.pos;
            if (t.kind == K10S_EV_AS_CREATE_GROUP_REQ) e.arg = (uint32_t)grank[t.group];
            else e.arg = pod_of(t.name);
            if (t.kind == K10S_EV_AS_CREATE_POD_REQ) hs.total_pods_in_trace++;
            wt.push_back(e);
        }
        // initialize emits every trace event at delay = its timestamp (simulator.rs:234-253): dslab-core
        // refuses a negative (or NaN) delay with a panic, so such a trace never starts a simulation.
        // The scenario is refused as a whole, at compile time, even when the event lies past some
        // replica's workload_prefix (that replica alone would not emit it): one compiled scenario
        // serves every replica of the batch.
        for (const std::vector<TraceEv>* v : {&ct, &wt})
            for (const TraceEv& t : *v)
                if (!(t.time >= 0.0))
                    throw std::runtime_error("trace event at a negative (or NaN) timestamp: the reference panics in "
                                             "initialize (dslab-core refuses an event delay < 0); refused for the "
                                             "whole batch, whatever the replicas' workload_prefix");
        hs.trace.resize(ct.size() + wt.size());
        std::merge(ct.begin(), ct.end(), wt.begin(), wt.end(), hs.trace.begin(), [](const TraceEv& a, const TraceEv& b) {
            int64_t ka = total_key(a.time), kb = total_key(b.time);
            return ka < kb || (ka == kb && a.seq < b.seq);
        });

        // ---- node pool (simulator.rs:51-65, 211-230)
        int64_t cnt = 0, mx = 0;
        for (auto& t : cluster) {
            if (t.kind == K10S_EV_AS_CREATE_NODE_REQ) cnt++;
            else cnt--;
            mx = std::max(cnt, mx);
        }
        uint64_t pool = (uint64_t)mx + (hs.ca_enabled ? d.ca_max_node_count : 0);
        if (pool > (1u << 24)) throw std::runtime_error("node pool too large");
        hs.n_pool = (uint32_t)pool;
        hs.n_slots = hs.n_pool + hs.n_default;
        if (hs.n_slots > 32767) throw std::runtime_error("more than 32767 node components per replica");
        return true;
    } catch (std::exception& ex) {
        err = ex.what();
        return false;
    }
}

// ---- packing -------------------------------------------------------------------------------------
namespace {
struct Packer {
    std::vector<uint8_t> buf;
    template <typename T>
    const T* put(const std::vector<T>& v) {
        size_t off = (buf.size() + 255) & ~(size_t)255;
        buf.resize(off + v.size() * sizeof(T) + 8);
        if (!v.empty()) std::memcpy(buf.data() + off, v.data(), v.size() * sizeof(T));
        return reinterpret_cast<const T*>(off);
    }
};
template <typename T>
const T* rb(const T* off, const uint8_t* base) {
    return reinterpret_cast<const T*>(base + reinterpret_cast<uintptr_t>(off));
}
}  // namespace

std::vector<uint8_t> pack_scenario(const HostScenario& hs, Scenario& s) {
    Packer pk;
    std::memset(&s, 0, sizeof s);
    s.n_nodes = hs.n_nodes;
    s.n_pods = hs.n_pods;
    s.n_uids = hs.n_uids;
    s.n_defs = (uint32_t)hs.def_node.size();
    s.n_slots = hs.n_slots;
    s.n_pool = hs.n_pool;
    s.n_default = hs.n_default;
    s.n_trace = (uint32_t)hs.trace.size();
    s.n_groups = (uint32_t)hs.group_names.size();
    s.n_ca_groups = (uint32_t)hs.ca_group_names.size();
    s.group_bound = hs.group_bound;
    s.ca_bound = hs.ca_bound;
    s.n_units = (uint32_t)hs.unit_dur.size();
    s.ca_enabled = hs.ca_enabled;
    s.hpa_enabled = hs.hpa_enabled;
    s.first_dynamic_seq = 2 + s.n_trace;
    s.n_cluster_trace = hs.n_cluster_trace;
    s.n_workload_trace = s.n_trace - hs.n_cluster_trace;
    s.total_pods_in_trace = hs.total_pods_in_trace;
    s.total_nodes_in_trace = hs.total_nodes_in_trace;
    s.node_uid = pk.put(hs.node_uid);
    s.def_node = pk.put(hs.def_node);
    s.def_cpu = pk.put(hs.def_cpu);
    s.def_ram = pk.put(hs.def_ram);
    s.def_ca_group = pk.put(hs.def_ca_group);
    s.def_ca_origin = pk.put(hs.def_ca_origin);
    s.pod_uid = pk.put(hs.pod_uid);
    s.pod_cpu = pk.put(hs.pod_cpu);
    s.pod_ram = pk.put(hs.pod_ram);
    s.pod_dur = pk.put(hs.pod_dur);
    s.pod_flags = pk.put(hs.pod_flags);
    s.pod_group = pk.put(hs.pod_group);
    s.pod_key = pk.put(hs.pod_key);
    s.default_defs = pk.put(hs.default_defs);
    s.trace = pk.put(hs.trace);
    s.wl_pods_upto = pk.put(hs.wl_pods_upto);
    s.g_initial = pk.put(hs.g_initial);
    s.g_max = pk.put(hs.g_max);
    s.g_cpu = pk.put(hs.g_cpu);
    s.g_ram = pk.put(hs.g_ram);
    s.g_flags = pk.put(hs.g_flags);
    s.g_tcpu = pk.put(hs.g_tcpu);
    s.g_tram = pk.put(hs.g_tram);
    s.g_cpu_kind = pk.put(hs.g_cpu_kind);
    s.g_ram_kind = pk.put(hs.g_ram_kind);
    s.g_cpu_usage = pk.put(hs.g_cpu_usage);
    s.g_ram_usage = pk.put(hs.g_ram_usage);
    s.g_cpu_uoff = pk.put(hs.g_cpu_uoff);
    s.g_cpu_ucnt = pk.put(hs.g_cpu_ucnt);
    s.g_ram_uoff = pk.put(hs.g_ram_uoff);
    s.g_ram_ucnt = pk.put(hs.g_ram_ucnt);
    s.g_pod = pk.put(hs.g_pod);
    s.g_pos = pk.put(hs.g_pos);
    s.g_sorted_k = pk.put(hs.g_sorted_k);
    s.unit_dur = pk.put(hs.unit_dur);
    s.unit_load = pk.put(hs.unit_load);
    s.ca_has_max = pk.put(hs.ca_has_max);
    s.ca_max = pk.put(hs.ca_max);
    s.ca_def = pk.put(hs.ca_def);
    s.ca_cpu = pk.put(hs.ca_cpu);
    s.ca_ram = pk.put(hs.ca_ram);
    return pk.buf;
}

Scenario rebase_scenario(const Scenario& o, const uint8_t* base) {
    Scenario s = o;
#define RB(f) s.f = rb(o.f, base)
    RB(node_uid); RB(def_node); RB(def_cpu); RB(def_ram); RB(def_ca_group); RB(def_ca_origin);
    RB(pod_uid); RB(pod_cpu); RB(pod_ram); RB(pod_dur); RB(pod_flags); RB(pod_group); RB(pod_key);
    RB(default_defs); RB(trace); RB(wl_pods_upto);
    RB(g_initial); RB(g_max); RB(g_cpu); RB(g_ram); RB(g_flags); RB(g_tcpu); RB(g_tram);
    RB(g_cpu_kind); RB(g_ram_kind); RB(g_cpu_usage); RB(g_ram_usage); RB(g_cpu_uoff); RB(g_cpu_ucnt);
    RB(g_ram_uoff); RB(g_ram_ucnt); RB(g_pod); RB(g_pos); RB(g_sorted_k); RB(unit_dur); RB(unit_load);
    RB(ca_has_max); RB(ca_max); RB(ca_def); RB(ca_cpu); RB(ca_ram);
#undef RB
    return s;
}

// ---- per-replica layout ----------------------------------------------------------------------
std::string params_error(const Params& p, const HostScenario& hs) {
    if (p.score_plugins == 0 || p.score_plugins > (K10S_SCORE_LEAST_ALLOCATED | K10S_SCORE_MOST_ALLOCATED))
        return "score_plugins must be 1 (LeastAllocatedResources), 2 (MostAllocatedResources) or 3 (both)";
    if (p.workload_prefix + 1 > hs.wl_pods_upto.size())
        return "workload_prefix exceeds the workload trace (" + std::to_string(hs.wl_pods_upto.size() - 1) + " events)";
    return "";
}

bool nodes_packable(const HostScenario& hs) {
    for (size_t d = 0; d < hs.def_cpu.size(); d++)
        if (hs.def_cpu[d] >= (1u << 24) || hs.def_ram[d] >= (1ull << 40)) return false;
    return true;
}

// A delay dslab-core refuses (`delay >= 0.` false: negative numbers, -inf, NaNs); -0.0 is allowed.
static bool signed_time(double x) { return !(x >= 0.0); }

bool times_nonneg(const HostScenario& hs, const Params* params, uint32_t n_params) {
    for (const TraceEv& t : hs.trace)
        if (signed_time(t.time)) return false;
    for (double d : hs.pod_dur)
        if (signed_time(d)) return false;
    for (double d : hs.unit_dur)
        if (signed_time(d)) return false;
    for (uint32_t r = 0; r < n_params; r++) {
        const Params& p = params[r];
        for (double d : {p.scheduling_cycle_interval, p.as_to_ps_network_delay, p.ps_to_sched_network_delay,
                         p.sched_to_as_network_delay, p.as_to_node_network_delay, p.as_to_ca_network_delay,
                         p.as_to_hpa_network_delay, p.ca_scan_interval, p.hpa_scan_interval})
            if (signed_time(d)) return false;
    }
    return true;
}

Layout make_layout(const HostScenario& hs, const k10s_capacities& caps, bool allow_packed, bool tnonneg) {
    Layout L;
    std::memset(&L, 0, sizeof L);
    L.tnonneg = tnonneg ? 1u : 0u;
    L.packed = (allow_packed && caps.node_cache == K10S_NODE_CACHE_AUTO && !caps.pruned_scan && nodes_packable(hs)) ? 1u : 0u;
    const uint64_t N = hs.n_nodes, P = hs.n_pods, S = hs.n_slots, G = hs.group_names.size(),
                   CG = hs.ca_group_names.size();
    L.words_nodes = (uint32_t)((N + 63) / 64);
    L.words_uids = (uint32_t)((hs.n_uids + 63) / 64);
    L.words_group = (uint32_t)((hs.group_bound + 63) / 64);
    L.words_pods = (uint32_t)((P + 63) / 64);
    L.cap_heap = caps.event_heap ? caps.event_heap : (uint32_t)std::min<uint64_t>(3 * P + 4 * N + 4 * S + 64, 0x7FFFFFFF);
    L.cap_aq = caps.active_queue ? caps.active_queue : (uint32_t)(P + 16);
    L.cap_uq = caps.unschedulable ? caps.unschedulable : (uint32_t)(P + 16);
    L.cap_act = hs.ca_enabled ? (uint32_t)std::max<uint64_t>(hs.defaults.ca_max_node_count + 16, N + 16) : 0;
    L.cap_undo = hs.ca_enabled ? (uint32_t)(P + 16) : 0;
    L.cap_log = caps.event_log;
    L.cap_place = caps.placement_log;
    L.cap_gauge = caps.gauge_log;
    L.rec_on = caps.pod_records ? 1 : 0;
    if (caps.delay_fifo == K10S_FIFO_OFF) {
        L.cap_fq = 0;
    } else {
        // default: room for a burst of one event per node (the cluster trace creates every node at
        // once: 4,096 PS create requests in one ring at C3, which a 512-entry ring spilled to the
        // heap), at least 512, at most 8,192 entries per class (2 MiB per replica)
        uint32_t want = caps.delay_fifo ? caps.delay_fifo : (uint32_t)std::min<uint64_t>(std::max<uint64_t>(512, N), 8192);
        if (want > (1u << 20)) want = 1u << 20;
        L.cap_fq = 1;
        while (L.cap_fq < want) L.cap_fq <<= 1;
    }
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        uint64_t o = off;
        off = (off + bytes + 255) & ~(uint64_t)255;
        return o;
    };
    L.hdr = take(sizeof(RepHdr));
    // hot scheduler-cache SoA first (the scan target), then per-entity records
    const uint64_t wide = L.packed ? 0 : 1;
    L.s_node = take(L.packed ? 8 * N : 0);
    // per-block fronts of the packed cache (k10s_engine.h front_scan): up to 64 blocks of 64 nodes
    L.front = (L.packed && N > 512 && N <= 4096) ? 1u : 0u;
    const uint64_t nbf = L.front ? (N + 63) / 64 : 0;
    L.fr_val = take(8 * K10S_FR_K * nbf);
    L.fr_idx = take(K10S_FR_K * nbf);
    L.s_cpu = take(wide * 4 * N);
    L.s_ram = take(wide * 8 * N);
    L.s_present = take(8 * (uint64_t)L.words_nodes);
    L.s_ccpu = take(wide * 4 * N);   // capacities: MostAllocated only (wide layout)
    L.s_cram = take(wide * 8 * N);
    L.pruned = caps.pruned_scan ? 1u : 0u;
    L.stall = caps.stall_guard ? 1u : 0u;
    L.bshift = 6;
    while (((N + (1ull << L.bshift) - 1) >> L.bshift) > 64) L.bshift++;
    L.nblocks = (uint32_t)((N + (1ull << L.bshift) - 1) >> L.bshift);
    L.s_bcpu = take(4 * (uint64_t)L.nblocks);
    L.s_bram = take(8 * (uint64_t)L.nblocks);
    L.node = take(sizeof(NodeState) * N);
    L.pend_rm = take(8 * (uint64_t)L.words_uids);
    L.pod = take(sizeof(PodState) * P);
    L.prec = take(L.rec_on ? sizeof(k10s_pod_record) * P : 0);
    L.slot = take(sizeof(SlotState) * S);
    L.pool_ring = take(4 * S);
    L.grp = take(sizeof(GroupState) * G);
    L.grp_bits = take(8 * G * (uint64_t)L.words_group);
    L.cag = take(8 * CG);
    L.ca_act = take(sizeof(CAAct) * (uint64_t)L.cap_act);
    uint64_t ca_n = hs.ca_enabled ? std::max<uint64_t>(N, L.cap_act) : 0;
    L.ca_cpu = take(4 * ca_n);
    L.ca_ram = take(8 * ca_n);
    L.ca_undo = take(8 * (uint64_t)L.cap_undo);
    const uint64_t ca_on = hs.ca_enabled ? 1 : 0;
    L.ca_ubits = take(ca_on * 8 * (uint64_t)L.words_pods);
    L.ca_live = take(ca_on * 8 * (uint64_t)L.words_nodes);
    L.ps_head = take(ca_on * 4 * N);
    L.ps_link = take(ca_on * 8 * P);
    L.ca_list = take(ca_on * 8 * P);
    L.heap = take(sizeof(HeapEv) * (uint64_t)L.cap_heap);
    L.aq = take(sizeof(QInfo) * (uint64_t)L.cap_aq);
    L.uq = take(sizeof(QInfo) * (uint64_t)L.cap_uq);
    L.log = take(sizeof(k10s_log_entry) * (uint64_t)L.cap_log);
    L.place = take(sizeof(k10s_placement) * (uint64_t)L.cap_place);
    L.fq = take(sizeof(HeapEv) * (uint64_t)L.cap_fq * K10S_NFQ);
    L.gauge = take(sizeof(k10s_gauge_row) * (uint64_t)L.cap_gauge);
    L.g_cpu = take(L.cap_gauge ? 4 * S : 0);
    L.g_ram = take(L.cap_gauge ? 8 * S : 0);
    L.stride = (off + 4095) & ~(uint64_t)4095;
    return L;
}

}  // namespace k10s
