// tests/hostcheck/hostcheck.cpp — TEST-ONLY host build of the engine's per-replica code.
//
// Compiles kubernetriks_amd/csrc/k10s_engine.h with g++ (K10S_LANES == 1) so the kernels' logic
// can be diffed against the CPU oracle on machines without a GPU.  It is not part of the product:
// the product C ABI (include/k10s.h, libk10s.so) only runs on the GPU and fails loudly without one.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../kubernetriks_amd/csrc/k10s_builder.h"
#include "../../kubernetriks_amd/csrc/k10s_engine.h"
#include "../../kubernetriks_amd/csrc/k10s_front_check.h"
#include "../../kubernetriks_amd/csrc/k10s_results.h"

using namespace k10s;

struct HC {
    HostScenario hs;
    std::vector<uint8_t> scen_bytes;
    Scenario sc;
    Layout L;
    std::vector<Params> params;
    std::vector<uint8_t> state;
    uint32_t R = 0;
    // what the batch was compiled from and every run call since, for the name-bound regrow (the
    // product's k10s_host.cpp regrow, restated for this build)
    std::string text;
    std::vector<uint8_t> blob;
    k10s_capacities caps;
    struct Call {
        int mode;
        double until, max_time;
        uint64_t budget;
    };
    std::vector<Call> history;
    uint32_t regrows = 0;
};

// The engine's working header is a separate copy during a run, like the LDS staging of the device
// kernels, so code that bypassed it would diverge here too.
static Ctx make_ctx(HC* h, uint32_t r, RepHdr* work) {
    Ctx c;
    c.sc = &h->sc;
    c.pr = &h->params[r];
    c.h = work;
    c.v = make_rep(h->state.data(), h->L, r);
    c.Lp = &h->L;
    return c;
}

extern "C" {

void* hc_create_bulk(const char* text, const void* blob, uint64_t blob_len, const k10s_replica_params* params,
                     uint32_t R, const k10s_capacities* caps, char* err, int errlen);
void* hc_create(const char* text, const k10s_replica_params* params, uint32_t R, const k10s_capacities* caps,
                char* err, int errlen) {
    return hc_create_bulk(text, nullptr, 0, params, R, caps, err, errlen);
}
static HC* hc_compile(const char* text, const void* blob, uint64_t blob_len, const k10s_replica_params* params,
                      uint32_t R, const k10s_capacities& c, std::string& e) {
    HC* h = new HC();
    if (!build_scenario(text, c.group_name_bound, c.ca_name_bound, h->hs, e, static_cast<const uint8_t*>(blob),
                        blob_len)) {
        delete h;
        return nullptr;
    }
    Scenario offs;
    h->scen_bytes = pack_scenario(h->hs, offs);
    h->sc = rebase_scenario(offs, h->scen_bytes.data());
    h->R = R;
    h->params.resize(R);
    for (uint32_t r = 0; r < R; r++) {
        if (params) {
            h->params[r] = params[r];
        } else {
            h->params[r] = h->hs.defaults;
            h->params[r].seed = h->hs.defaults.seed + r;
        }
        h->params[r].ca_max_node_count = h->hs.defaults.ca_max_node_count;
        const std::string perr = params_error(h->params[r], h->hs);
        if (!perr.empty()) {
            e = "params[" + std::to_string(r) + "]: " + perr;
            delete h;
            return nullptr;
        }
    }
    bool plugins = false;
    for (uint32_t r = 0; r < R; r++) plugins |= h->params[r].score_plugins != K10S_SCORE_LEAST_ALLOCATED;
    const bool tnn = times_nonneg(h->hs, h->params.data(), R);
    h->L = make_layout(h->hs, c, !plugins && tnn, tnn);
    h->state.assign((size_t)h->L.stride * R, 0);
    for (uint32_t r = 0; r < R; r++) {
        RepHdr work;
        std::memset(&work, 0xA5, sizeof work);
        Ctx c = make_ctx(h, r, &work);
        init_replica(c);
        *c.v.h() = work;
    }
    h->text = text;
    if (blob && blob_len) h->blob.assign((const uint8_t*)blob, (const uint8_t*)blob + blob_len);
    h->caps = c;
    return h;
}
void* hc_create_bulk(const char* text, const void* blob, uint64_t blob_len, const k10s_replica_params* params,
                     uint32_t R, const k10s_capacities* caps, char* err, int errlen) {
    std::string e;
    k10s_capacities c;
    std::memset(&c, 0, sizeof c);
    if (caps) c = *caps;
    HC* h = hc_compile(text, blob, blob_len, params, R, c, e);
    if (!h && err) std::snprintf(err, (size_t)errlen, "%s", e.c_str());
    return h;
}
void hc_free(void* p) { delete (HC*)p; }
int hc_default_params(void* p, k10s_replica_params* out) {
    *out = ((HC*)p)->hs.defaults;
    return 0;
}
static void hc_call(HC* h, const HC::Call& k) {
    for (uint32_t r = 0; r < h->R; r++) {
        RepHdr work;
        Ctx c = make_ctx(h, r, &work);
        int more = 1;
        while (more) {  // one iteration = one device launch: stage, run, write back
            work = *c.v.h();
            more = run_replica(c, k.mode, k.until, k.max_time, k.budget);
            *c.v.h() = work;
        }
    }
}
int hc_run(void* p, int mode, double until, double max_time, uint64_t budget) {
    HC* h = (HC*)p;
    const HC::Call k{mode, until, max_time, budget};
    h->history.push_back(k);
    hc_call(h, k);
    // capacity regrow (k10s_host.cpp regrow): recompile with every exhausted capacity doubled (a
    // generated-name universe, the event heap, the scheduler queues) and replay every call, until no
    // replica stops at K10S_ERR_NAME_BOUND / HEAP_FULL / QUEUE_FULL below its maximum
    for (;;) {
        bool grow_ca = false, grow_group = false, grow_heap = false, grow_queue = false;
        for (uint32_t r = 0; r < h->R; r++) {
            const RepHdr& H = *make_rep(h->state.data(), h->L, r).h();
            if (H.error_code == K10S_ERR_NAME_BOUND) {
                if (H.error_kind == K10S_EV_PS_CA_REQ) grow_ca = true;
                else grow_group = true;
            } else if (H.error_code == K10S_ERR_HEAP_FULL) {
                grow_heap = true;
            } else if (H.error_code == K10S_ERR_QUEUE_FULL) {
                grow_queue = true;
            }
        }
        k10s_capacities c = h->caps;
        c.group_name_bound = h->hs.group_bound;
        c.ca_name_bound = h->hs.ca_bound;
        c.event_heap = h->L.cap_heap;
        c.active_queue = h->L.cap_aq;
        c.unschedulable = h->L.cap_uq;
        const uint32_t MAXB = 1u << 20, MAXQ = 1u << 30;
        auto grow2 = [](uint32_t cur, uint32_t fl, uint32_t mx) { return std::min<uint32_t>(2 * std::max<uint32_t>(cur, fl), mx); };
        bool grown = false;
        if (grow_group && c.group_name_bound < MAXB) {
            c.group_name_bound = grow2(c.group_name_bound, 32, MAXB);
            grown = true;
        }
        if (grow_ca && c.ca_name_bound < MAXB) {
            c.ca_name_bound = grow2(c.ca_name_bound, 32, MAXB);
            grown = true;
        }
        if (grow_heap && c.event_heap < MAXQ) {
            c.event_heap = grow2(c.event_heap, 64, MAXQ);
            grown = true;
        }
        if (grow_queue && (c.active_queue < MAXQ || c.unschedulable < MAXQ)) {
            c.active_queue = grow2(c.active_queue, 16, MAXQ);
            c.unschedulable = grow2(c.unschedulable, 16, MAXQ);
            grown = true;
        }
        if (!grown) return 0;
        std::string e;
        HC* n = hc_compile(h->text.c_str(), h->blob.empty() ? nullptr : h->blob.data(), h->blob.size(),
                           h->params.data(), h->R, c, e);
        if (!n) return -1;
        n->history = h->history;
        n->regrows = h->regrows + 1;
        for (const HC::Call& x : n->history) hc_call(n, x);
        std::swap(*h, *n);
        delete n;
    }
}
int hc_capacities(void* p, k10s_capacities* out, uint32_t* regrows) {
    HC* h = (HC*)p;
    *out = h->caps;
    out->event_heap = h->L.cap_heap;
    out->active_queue = h->L.cap_aq;
    out->unschedulable = h->L.cap_uq;
    out->group_name_bound = h->hs.group_bound;
    out->ca_name_bound = h->hs.ca_bound;
    out->delay_fifo = h->L.cap_fq ? h->L.cap_fq : K10S_FIFO_OFF;
    if (regrows) *regrows = h->regrows;
    return 0;
}
int hc_name_bounds(void* p, uint32_t* group_bound, uint32_t* ca_bound) {
    HC* h = (HC*)p;
    *group_bound = h->hs.group_bound;
    *ca_bound = h->hs.ca_bound;
    return 0;
}
int hc_results(void* p, k10s_replica_result* out) {
    HC* h = (HC*)p;
    for (uint32_t r = 0; r < h->R; r++) {
        Rep v = make_rep(h->state.data(), h->L, r);
        hdr_to_result(*v.h(), out[r]);
    }
    return 0;
}
int hc_event_log(void* p, uint32_t r, k10s_log_entry* out, uint32_t cap, uint32_t* n) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    uint32_t k = v.h()->log_n < cap ? v.h()->log_n : cap;
    if (v.log()) std::memcpy(out, v.log(), sizeof(k10s_log_entry) * k);
    *n = v.log() ? k : 0;
    return 0;
}
int hc_gauges(void* p, uint32_t r, k10s_gauge_row* out, uint32_t cap, uint32_t* n) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    uint32_t k = h->L.cap_gauge ? (v.h()->gauge_n < cap ? v.h()->gauge_n : cap) : 0;
    if (k) std::memcpy(out, v.gauge(), sizeof(k10s_gauge_row) * k);
    *n = k;
    return 0;
}
int hc_placements(void* p, uint32_t r, k10s_placement* out, uint32_t cap, uint32_t* n) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    uint32_t k = v.h()->place_n < cap ? v.h()->place_n : cap;
    if (v.place()) std::memcpy(out, v.place(), sizeof(k10s_placement) * k);
    *n = v.place() ? k : 0;
    return 0;
}
int hc_pod_records(void* p, uint32_t r, k10s_pod_record* out, uint32_t cap, uint32_t* n) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    uint32_t k = h->hs.n_pods < cap ? h->hs.n_pods : cap;
    if (v.prec()) std::memcpy(out, v.prec(), sizeof(k10s_pod_record) * k);
    *n = v.prec() ? k : 0;
    return 0;
}
int hc_group_sizes(void* p, uint32_t r, uint32_t* created, uint32_t* total, uint32_t cap, uint32_t* n) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    uint32_t G = (uint32_t)h->hs.group_names.size();
    uint32_t k = G < cap ? G : cap;
    for (uint32_t g = 0; g < k; g++) {
        created[g] = v.grp()[g].registered ? v.grp()[g].created_count : 0;
        total[g] = v.grp()[g].total_created;
    }
    *n = k;
    return 0;
}
uint32_t hc_num_nodes(void* p) { return ((HC*)p)->hs.n_nodes; }
uint32_t hc_num_pods(void* p) { return ((HC*)p)->hs.n_pods; }
uint32_t hc_num_groups(void* p) { return (uint32_t)((HC*)p)->hs.group_names.size(); }
const char* hc_node_name(void* p, uint32_t i) { return ((HC*)p)->hs.node_names[i].c_str(); }
const char* hc_pod_name(void* p, uint32_t i) { return ((HC*)p)->hs.pod_names[i].c_str(); }
const char* hc_group_name(void* p, uint32_t i) { return ((HC*)p)->hs.group_names[i].c_str(); }
uint64_t hc_replica_bytes(void* p) { return ((HC*)p)->L.stride; }
uint32_t hc_node_entry_bytes(void* p) { return ((HC*)p)->L.packed ? 8u : 12u; }

}  // extern "C"

extern "C" int hc_debug_queues(void* p, uint32_t r, double* aq, uint32_t* aq_pod, uint32_t* naq, double* uq,
                               uint32_t* uq_pod, uint32_t* nuq, uint32_t cap) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    *naq = v.h()->aq_size;
    *nuq = v.h()->uq_size;
    Ctx c = make_ctx(h, r, v.h());   // the replica's header in place (aq_get reads its LDS part)
    for (uint32_t i = 0; i < v.h()->aq_size && i < cap; i++) {
        const QInfo q = aq_get(c, i);
        aq[i] = q.timestamp;
        aq_pod[i] = q.pod;
    }
    for (uint32_t i = 0; i < v.h()->uq_size && i < cap; i++) {
        uq[i] = v.uq()[i].timestamp;
        uq_pod[i] = v.uq()[i].pod;
    }
    return 0;
}

// The action queue's mode (k10s_engine.h aq_push: 1 = sorted) and length, for tests/test_action_queue.py.
extern "C" int hc_aq_mode(void* p, uint32_t r, uint32_t* sorted, uint32_t* n) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    *sorted = v.h()->aq_sorted;
    *n = v.h()->aq_size;
    return 0;
}

// The fronts' invariant (k10s_front_check.h), the test-only mirror of k10s_engine_check_fronts.
extern "C" int hc_check_fronts(void* p, uint32_t r, int32_t* result) {
    HC* h = (HC*)p;
    Rep v = make_rep(h->state.data(), h->L, r);
    *result = h->L.front ? k10s_front_check(v.s_node(), v.fr_val(), v.fr_idx(), h->sc.n_nodes, v.h()->fr_dirty,
                                            v.h()->fr_over, K10S_FR_K)
                         : 0;
    return 0;
}

// The host score (bit-identical to the device's), for tests/test_scan_adversarial.py.
extern "C" double hc_la_score(uint32_t ac, uint64_t ar, uint32_t rc, uint64_t rr) { return la_score(ac, ar, rc, rr); }
// The event loop's screened scan test (k10s_engine.h scan_screen, operands formed as
// scan_lanes_screen forms them), for tests/test_scan_screen.py.
extern "C" int hc_scan_screen(uint32_t ac, uint64_t ar, uint32_t rc, uint64_t rr, float thr) {
    const float fa = (float)rc;
    const float fr = __builtin_fmaf((float)(uint32_t)(rr >> 32), 4294967296.0f, (float)(uint32_t)rr);
    return scan_screen(ac, ar, fa, fr, thr + K10S_SCREEN_EPS) ? 1 : 0;
}
extern "C" float hc_screen_u(double s) { return screen_u(s); }
