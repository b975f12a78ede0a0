// k10s_results.h — conversion of per-replica device state into the C ABI result structs.
#pragma once

#include <cstring>

#include "k10s_state.h"

namespace k10s {

inline void hdr_to_result(const RepHdr& h, k10s_replica_result& r) {
    std::memset(&r, 0, sizeof r);
    r.status = h.status;
    r.error_code = h.error_code;
    r.error_kind = h.error_kind;
    r.error_seq = h.error_seq;
    r.error_time = h.error_time;
    r.clock = h.clock;
    for (int i = 0; i < K10S_NUM_COUNTERS; i++) r.counters[i] = h.counters[i];
    for (int i = 0; i < 3; i++) {
        r.est[i].n = h.est[i].n;
        r.est[i].min = h.est[i].mn;
        r.est[i].max = h.est[i].mx;
        r.est[i].mean = h.est[i].n ? h.est[i].avg : __builtin_nan("");
        r.est[i].sum2 = h.est[i].sum2;
        for (int b = 0; b < K10S_HIST_BINS; b++) r.est[i].hist[b] = h.est[i].hist[b];
    }
    r.unschedulable_len = h.uq_size;
    r.active_len = h.aq_size;
    r.node_count_as = h.as_node_count;
    r.node_count_ps = h.ps_node_count;
    r.node_count_s = h.s_node_count;
    r.log_len = h.log_n;
    r.placements_len = h.place_n;
    r.flags = h.flags;
}

}  // namespace k10s
