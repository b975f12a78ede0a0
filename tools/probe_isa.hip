// tools/probe_isa.hip — static instruction mix of the event-loop pieces (tooling, not product).
//
// Each probe kernel runs ONE piece of k10s_engine.h with the event kind fixed at compile time, so
// the handler's switch folds to a single case; tools/probe_isa.py compiles this file for gfx950
// (with -DK10S_SPLIT=0: everything inlined into the probe) and counts VALU / SALU / LDS / VMEM
// instructions per kernel as a proxy for the dynamic cost of that piece.
#include <hip/hip_runtime.h>

#define K10S_KERNEL_TU 1
#include "../kubernetriks_amd/csrc/k10s_engine.h"

using namespace k10s;

template <int K>
__global__ __launch_bounds__(64) void probe_dispatch(uint32_t a, uint32_t b, double x, int16_t slot) {
    Ctx c;
    HeapEv e;
    e.time = c.H().clock;
    e.seq = c.H().next_seq;
    e.kind = (uint16_t)K;
    e.slot = slot;
    e.a = a;
    e.b = b;
    e.x = x;
    uniform_event(e);
    c.H().cur_ev = e;
    dispatch(c, K10S_EVREF(&c.H().cur_ev), (uint32_t)K);
}

__global__ __launch_bounds__(64) void probe_sl_update(uint32_t q, int64_t key, uint32_t seq) {
    Ctx c;
    sl_update(c, uniform_u32(q), true, (int64_t)uniform_u64((uint64_t)key), uniform_u32(seq));
}

__global__ __launch_bounds__(64) void probe_consume_fifo(int src, uint32_t ntr) {
    Ctx c;
    consume_source(c, uniform_u32((uint32_t)src) & 7, ntr);
}

__global__ __launch_bounds__(64) void probe_consume_heap(uint32_t ntr) {
    Ctx c;
    consume_source(c, SRC_HEAP, ntr);
}

__global__ __launch_bounds__(64) void probe_emit_fifo(uint32_t a, uint32_t b) {
    Ctx c;
    emit(c, K10S_EV_PS_CREATE_POD_REQ, c.P().as_to_ps_network_delay, -1, a, b, 0.0, FQ_AS_TO_PS);
}

__global__ __launch_bounds__(64) void probe_emit_heap(uint32_t a, uint32_t b, double d) {
    Ctx c;
    emit(c, K10S_EV_N_POD_FINISHED, d, 3, a, b, 0.0);
}

#define P(K) template __global__ void probe_dispatch<K>(uint32_t, uint32_t, double, int16_t);
P(K10S_EV_AS_CREATE_POD_REQ)
P(K10S_EV_PS_CREATE_POD_REQ)
P(K10S_EV_S_POD_SCHEDULE_REQ)
P(K10S_EV_AS_ASSIGN_REQ)
P(K10S_EV_PS_ASSIGN_REQ)
P(K10S_EV_AS_ASSIGN_RESP)
P(K10S_EV_N_BIND)
P(K10S_EV_AS_POD_STARTED)
P(K10S_EV_PS_POD_STARTED)
P(K10S_EV_N_POD_FINISHED)
P(K10S_EV_AS_POD_FINISHED)
P(K10S_EV_PS_POD_FINISHED)
P(K10S_EV_S_POD_FINISHED)
P(K10S_EV_S_RUN_CYCLE)
P(K10S_EV_M_GAUGE_TICK)

__global__ __launch_bounds__(64) void probe_scan(uint32_t rc, uint64_t rr, double w) {
    Ctx c;
    int32_t chosen = -1;
    int st = schedule_scan(c.V().s_cpu(), c.V().s_ram(), c.V().s_present(), c.S().n_nodes, rc, rr, w, &chosen);
    c.H().flags = (uint32_t)st + (uint32_t)chosen;
}

__global__ __launch_bounds__(64) void probe_cycle(double t) {
    Ctx c;
    run_scheduling_cycle(c, t);
}

__global__ __launch_bounds__(64) void probe_sl_apply_dirty(uint32_t ntr) {
    Ctx c;
    sl_apply_dirty(c, ntr);
}

__global__ __launch_bounds__(64) void probe_heap_pop() {
    Ctx c;
    heap_pop(c);
}
